# steady-state kernel trace of the SUN bench step: rocprofv3 --kernel-trace of bench.py, then
# per-kernel per-step figures over the last 8 steps (tools/trace_kernel_avg.py)
set -u
cd ${GRAFT_REPO_ROOT:-.}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/sun_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $O/sun_prof.json 2> $O/sun_prof.err || { tail -5 $O/sun_prof.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/sun_prof -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy8_kernel > $O/sun_trace_steady.json
