#!/bin/bash
# SQ / TCC counter passes over scripts/corr_variants.py (one rocprofv3 run
# per pass, kernel trace only); summary: python scripts/pmc_kernels.py
# 'gpurun_out/cv_*/run_counter_collection.csv' full
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ARGS="--reps 30 ${CV_ARGS:-}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
P3="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE"
P4="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA TCC_HIT_sum TCC_MISS_sum"
i=0
for grp in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/cv_$i -o run --output-format csv \
    -- python scripts/corr_variants.py $ARGS > $OUT/cv_$i.log 2>&1
  rc=$?
  echo "cv pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
python scripts/pmc_kernels.py "$OUT/cv_*/run_counter_collection.csv" full > $OUT/cv_summary.txt
