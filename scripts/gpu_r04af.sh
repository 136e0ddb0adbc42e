#!/bin/bash
# barrier-free block map: window tests, phases, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${T:-r04af}
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -3 $O/${T}_$name.txt; }
run pytest_window python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_ba_gpu.py tests/test_update_harness_gpu.py
run phases_cfg2 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo10_1 python -u scripts/ba_window_phases.py 10 1
run bench python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline
# full suite, smoke, default bench (with the CPU baseline), kernel stats of the bench
bash scripts/gpu_suite.sh ${T}_suite || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
echo done
