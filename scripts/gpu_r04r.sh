#!/bin/bash
# staged E entries for the apply loops: window tests + phases
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04x
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -5 $O/${T}_$name.txt; }
run pytest_window python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_update_harness_gpu.py
run phases_dpvo25_1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo25_2 python -u scripts/ba_window_phases.py 25 2
run phases_cfg2 python -u scripts/ba_window_phases.py cfg2 2
