#!/bin/bash
# SQ (wave / LDS / issue) PMC passes over a short bench run, one rocprofv3
# run per pass (kernel trace only), <= 8 SQ counters per pass.  Summaries:
# gpurun_out/sq_<n>/run_counter_collection.csv; python scripts/sq_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
i=0
P3="${SQ_EXTRA:-}"  # optional third pass, e.g. "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for grp in "$P1" "$P2" ${P3:+"$P3"}; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/sq_$i -o run --output-format csv \
    -- python bench.py $ARGS > $OUT/sq_$i.log 2>&1
  rc=$?
  echo "sq pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
