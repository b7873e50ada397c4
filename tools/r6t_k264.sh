# rows256 K = 264 (interim SA layer 1): parity tests, C4 bench + trace
set -e
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm256_gpu.py tests/test_pool_bn_gpu.py tests/test_model_gpu.py tests/test_sa_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/${TAG:-r6t}_t.log 2>&1
TAG=${TAG:-r6t} bash tools/gpu_session.sh c4 c4_trace > $O/${TAG:-r6t}_sess.log 2>&1
timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/${TAG:-r6t}_c4b.json 2> $O/${TAG:-r6t}_c4b.err
echo ok
