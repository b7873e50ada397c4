# BN + ReLU + pool fusion check: parity tests, the C4 model tests, C4 A/B (OV3D_BN_POOL=0), trace
set -e
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pool_bn_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r6n_t.log 2>&1
BENCH_ARGS="--workload scannet" timeout -k 10 700 bash tools/ab_envs.sh "OV3D_BN_POOL=0" > $O/r6n_ab.log 2>&1
TAG=r6n bash tools/gpu_session.sh c4_trace > $O/r6n_sess.log 2>&1
echo ok
