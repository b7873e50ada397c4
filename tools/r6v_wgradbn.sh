# weight gradient with the BN + ReLU on load (no Z rows): parity tests, C4 A/B against the Z rows
set -e
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pool_bn_gpu.py tests/test_wgrad_gpu.py tests/test_wgrad_defer_gpu.py tests/test_model_gpu.py tests/test_sa_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r6v_t.log 2>&1
TAG=r6v bash tools/gpu_session.sh c4 c4_trace > $O/r6v_sess.log 2>&1
timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/r6v_c4b.json 2> $O/r6v_c4b.err
echo ok
