#!/bin/bash
# Counter passes (one rocprofv3 run per pass, kernel trace only) over a short
# bench run; per-kernel medians are read from gpurun_out/pmcc_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --eager"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmcc_$i -o run --output-format csv \
    -- python bench.py $ARGS > $OUT/pmcc_$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<PASSES
${PMC_PASSES:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES
TCC_HIT_sum TCC_MISS_sum
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS}
PASSES
exit 0
