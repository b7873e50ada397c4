# grouped weight-gradient launches of 48 problems: tests, SUN A/B against the 28-problem split, trace
set -e
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wgrad_defer_gpu.py tests/test_wgrad_gpu.py -x -q --timeout 200 --timeout-method thread > $O/r6o_t.log 2>&1
timeout -k 10 700 bash tools/ab_envs.sh "OV3D_WGRAD_SK_MAX=28" > $O/r6o_ab.log 2>&1
TAG=r6o bash tools/gpu_session.sh sun_trace > $O/r6o_sess.log 2>&1
echo ok
