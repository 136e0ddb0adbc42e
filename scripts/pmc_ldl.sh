#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/ldlpmc
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"
P3="SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"
i=0
for grp in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- ./scripts/micro/ldl_bench 11 1 300 ldl > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
exit 0
