# BN + ReLU inside the next rows256 product: parity tests, model tests, C4 A/B (OV3D_BN_GEMM=0)
set -e
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pool_bn_gpu.py tests/test_sa_fused_gpu.py tests/test_model_gpu.py tests/test_gemm256_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r6s_t.log 2>&1
BENCH_ARGS="--workload scannet" timeout -k 10 700 bash tools/ab_envs.sh "OV3D_BN_GEMM=0" > $O/r6s_ab.log 2>&1
echo ok
