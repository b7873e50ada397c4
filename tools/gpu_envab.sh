cd ${GRAFT_REPO_ROOT}; O=gpurun_out; mkdir -p $O
for v in "X=0" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/envab.json 2> $O/envab.err || { echo "$v failed"; tail -3 $O/envab.err; continue; }
  python -c "import json; d=json.load(open('$O/envab.json')); print('$v', d['value'], d['ms_per_step_median'])"
done
