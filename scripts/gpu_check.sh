#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Stops at the first crash / timeout (exit 124/134/137/139); plain test
# failures (exit 1) still let the later steps run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139|-6|-11) return 0;; *) return 1;; esac; }
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    ba) timeout -k 10 240 python -m pytest tests/test_ba_gpu.py -q -rf > $OUT/ba_gpu.log 2>&1; rc=$?;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?;;
    large) timeout -k 10 400 python -u -m pytest tests/test_ba_large_gpu.py tests/test_global_ba_gpu.py tests/test_sharded_hip_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/large.log 2>&1; rc=$?;;
    cfg4) timeout -k 10 300 python bench.py --sharded --steps 5 --warmup 2 > $OUT/cfg4.log 2>&1; rc=$?;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?;;
    cfg4prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof4 -o run --output-format csv -- python bench.py --sharded --steps 3 --warmup 1 > $OUT/cfg4prof.log 2>&1; rc=$?;;
    *) echo "unknown step $s"; rc=0;;
  esac
  echo "step $s rc=$rc"
  tail -3 $OUT/*$s*.log 2>/dev/null | tail -3 || true
  if fatal $rc; then echo "fatal rc=$rc at $s; stopping"; exit $rc; fi
done
exit 0
