#!/bin/bash
# Full GPU suite, window-BA phase timings, and a kernel-trace profile of the
# default bench.  A fault / abort / timeout in a step ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > $O/t_full.log 2>&1
rc=$?
tail -3 $O/t_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python scripts/ba_window_phases.py cfg2 2 > $O/phases.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_prof.log 2>&1 || exit $?
tail -1 $O/bench_prof.log
cd $R
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1
rc2=$?
tail -1 $O/bench_default.log
exit $(( rc ? rc : rc2 ))
