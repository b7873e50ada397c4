set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${SEL:-heads or bn}" > $OUT/pq.log 2>&1
rc=$?; tail -3 $OUT/pq.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/pq_bench.json 2> $OUT/pq_bench.err || exit 1
python -c "import json; d=json.load(open('$OUT/pq_bench.json')); print('bench', d['value'], d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/pq -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> $OUT/pq_prof.err || { tail -3 $OUT/pq_prof.err; exit 1; }
echo done
