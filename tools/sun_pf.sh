set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for pf in "" "--no-prefetch" "" "--no-prefetch"; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $pf > $OUT/pf.json 2> $OUT/pf.err || { tail $OUT/pf.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/pf.json')); print('$pf', d['value'], d['ms_per_step'])"
done
timeout -k 10 100 python tools/fps_time.py
