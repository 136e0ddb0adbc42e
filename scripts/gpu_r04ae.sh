#!/bin/bash
# plan-driven split with a diagonal work weight (DPVO_BA_DIAGW, quarters): tests, phases, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${T:-r04ae}
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -3 $O/${T}_$name.txt; }
run pytest_window python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_ba_gpu.py
DPVO_BA_DIAGW=6 run pytest_window_dw6 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ba_window_gpu.py
run phases_cfg2 python -u scripts/ba_window_phases.py cfg2 2
for w in 0 4 6 8 12; do
  DPVO_BA_DIAGW=$w run phases_dpvo25_w$w python -u scripts/ba_window_phases.py 25 1
  DPVO_BA_DIAGW=$w run phases_dpvo10_w$w python -u scripts/ba_window_phases.py 10 1
done
run bench python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline
