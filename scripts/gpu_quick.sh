#!/bin/bash
# quick check: window tests, BA phases (cfg2, dpvo25, dpvo10), bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${T:-quick}
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -3 $O/${T}_$name.txt; }
run pytest_window python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_ba_gpu.py tests/test_update_harness_gpu.py
run phases_cfg2 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo10_1 python -u scripts/ba_window_phases.py 10 1
