#!/bin/bash
# dense kernel with per-block edge masks: phases A/B and parity of the BA window tests through it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04h
run() { name=$1; shift; timeout -k 10 200 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; cat $O/${T}_$name.txt; }
run phases_cfg2_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo10_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 10 1
run phases_dpvo10_block env DPVO_BA_DENSE=0 python -u scripts/ba_window_phases.py 10 1
run pytest_dense env DPVO_BA_DENSE=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_update_harness_gpu.py tests/test_ba_gpu.py
run pytest_m20 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_update_harness_gpu.py -k m20
run launch python -u scripts/reproject_launch_bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_launchprof -o run --output-format csv -- python scripts/reproject_launch_bench.py > $O/${T}_launchprof.log 2>&1 || { tail -5 $O/${T}_launchprof.log; exit 1; }
f=$(find $O/${T}_launchprof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 12
