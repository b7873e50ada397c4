set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python tools/fps_time.py
timeout -k 10 300 python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c4_bench.json 2> $OUT/c4_bench.err || { tail $OUT/c4_bench.err; exit 1; }
cat $OUT/c4_bench.json
timeout -k 10 300 python bench.py --workload scannet --steps 10 --warmup 3 --no-cpu-baseline --no-prefetch > $OUT/c4_bench_nopf.json 2> $OUT/c4_bench_nopf.err || { tail $OUT/c4_bench_nopf.err; exit 1; }
cat $OUT/c4_bench_nopf.json
