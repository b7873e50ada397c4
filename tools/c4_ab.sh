set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for pf in "" "--no-prefetch"; do
timeout -k 10 300 python bench.py --workload scannet --steps 20 --warmup 5 --no-cpu-baseline $pf > $OUT/c4ab.json 2> $OUT/c4ab.err || { tail $OUT/c4ab.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c4ab.json')); print('$pf', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/sunab.json 2> $OUT/sunab.err || { tail $OUT/sunab.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/sunab.json')); print('sun', d['value'], d['ms_per_step'])"
