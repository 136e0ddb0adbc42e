#!/bin/bash
# dense-kernel stage-A sub-marks, plan round trimming (launch A/B), default bench + profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04j
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -4 $O/${T}_$name.txt; }
run phases_cfg2_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 25 1
run launch python -u scripts/reproject_launch_bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_launchprof -o run --output-format csv -- python scripts/reproject_launch_bench.py > $O/${T}_launchprof.log 2>&1 || { tail -5 $O/${T}_launchprof.log; exit 1; }
f=$(find $O/${T}_launchprof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 8
run pytest_plan python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ba_window_gpu.py -k "plan or fused"
run bench python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 6
