set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
cat $OUT/c4_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c4prof -o run --output-format csv -- python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4_prof.json 2> $OUT/c4_prof.err || { tail $OUT/c4_prof.err; exit 1; }
echo done
