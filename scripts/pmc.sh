#!/bin/bash
# PMC passes (one counter per rocprofv3 run, kernel trace only) over a
# short bench run; summaries land in gpurun_out/pmc_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ARGS="--steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for grp in ${PMC_GROUPS:-FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum}; do
  i=$((i + 1))
  timeout -k 10 150 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmc_$i -o run --output-format csv \
    -- python bench.py $ARGS > $OUT/pmc_$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
