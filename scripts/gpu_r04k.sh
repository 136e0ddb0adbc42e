#!/bin/bash
# dense kernel after unconditional J reads: phases + parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04k
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -4 $O/${T}_$name.txt; }
run phases_cfg2_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo10_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 10 1
run pytest_dense env DPVO_BA_DENSE=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_ba_gpu.py
