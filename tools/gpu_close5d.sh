# round-5 closing session (fourth): smoke, the full GPU suite, the default bench line, a SUN kernel trace
# (steady per-step figures), C4 / C5 bench lines with traces, PMC of the shipped attention / SA /
# wgrad kernels.  Every GPU step under its own time limit; the first failure ends the script.
set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
step() { echo "== $1"; }
step smoke; timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step tests; timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
step bench; timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('SUN', d['value'], d['ms_per_step_median'], d['roofline']['frac'], d['cpu_baseline']['value'])"
step sun_trace; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sun_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/sun_prof.json 2> $O/sun_prof.err || { tail -5 $O/sun_prof.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/sun_prof -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy9_kernel > $O/sun_trace_steady.json
step c4; timeout -k 10 400 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_bench.json 2> $O/c4_bench.err || { tail -5 $O/c4_bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4_prof -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_prof.json 2> $O/c4_prof.err || { tail -5 $O/c4_prof.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/c4_prof -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy9_kernel > $O/c4_trace_steady.json
step c5; SKIP_TESTS=1 bash tools/c5_quick.sh || exit 1
step pmc; PMC_RE="sa_dy9_kernel|sa_layer_kernel|sa_dy2_fused_kernel|lngemm_bwd_kernel" bash tools/gpu_pmc.sh || exit 1
echo "== done"
