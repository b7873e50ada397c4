#!/bin/bash
# PMC passes (one counter set per rocprofv3 run, each under its own time limit) over an eager
# bench step: the encoder attention kernels, the fused SA backward and the grouped wgrad
# (PMC_RE / PMC_CMD: another kernel regex / program).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/list.txt 2>&1 || { echo "list failed"; tail -5 $OUT/list.txt; exit 1; }
RE="${PMC_RE:-attn_fwd_kernel|attn_bwd_dq_kernel|attn_bwd_dkdv_kernel|sa_dy8_kernel|wgrad_group_kernel|heads_out}"
# the profiled program (PMC_CMD overrides: a python script path and its arguments)
read -r -a CMD <<< "${PMC_CMD:-bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline}"
PASSES=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i+1))
  ok=1
  for c in $P; do grep -qw "$c" $OUT/list.txt || { echo "skip pass $i: $c not listed"; ok=0; }; done
  [ $ok = 1 ] || continue
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- \
      python "${CMD[@]}" > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 $OUT/p$i.log; exit 1; fi
  echo "pass $i ok"
done
python tools/pmc_summary.py $OUT/summary.json $(find $OUT -name "*counter_collection.csv") > $OUT/summary.txt
find $OUT -name "*counter_collection.csv" -delete
cat $OUT/summary.txt | cut -c1-600
