set -u
cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r6e_np_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-prefetch > $O/r6e_np.json 2> $O/r6e_np.err || { tail -5 $O/r6e_np.err; exit 1; }
python tools/trace_kernel_avg.py $(find $O/r6e_np_prof -name '*kernel_trace.csv' | head -1) "" --steps 8 --marker sa_dy9_kernel > $O/r6e_np_steady.json
python -c "import json; d=json.load(open('$O/r6e_np.json')); print('noprefetch', d['value'], d['ms_per_step_median'])"
