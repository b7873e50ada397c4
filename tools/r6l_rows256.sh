# rows256 check: parity tests, isolated probe against gemm256, C4 A/B (OV3D_ROWS256=0), C4 trace
set -e
O=gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm256_gpu.py -q -k rows256 --timeout 120 --timeout-method thread > $O/r6m_t.log 2>&1
timeout -k 10 120 python tools/rows256_probe.py > $O/r6m_p.json 2>&1
BENCH_ARGS="--workload scannet" timeout -k 10 700 bash tools/ab_envs.sh "OV3D_ROWS256=0" > $O/r6m_ab.log 2>&1
TAG=r6m bash tools/gpu_session.sh c4_trace > $O/r6m_sess.log 2>&1
echo ok
