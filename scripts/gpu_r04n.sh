#!/bin/bash
# plan phase stamps; dpvo25 BA phases after the batched E^T dX apply; full GPU suite + bench; cfg2 launch profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04q
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -6 $O/${T}_$name.txt; }
run plan_phases python -u scripts/plan_phases.py
run phases_dpvo25_block python -u scripts/ba_window_phases.py 25 1
run phases_cfg2_block python -u scripts/ba_window_phases.py cfg2 2
bash scripts/gpu_suite.sh $T || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_launchprof -o run --output-format csv -- python scripts/reproject_launch_bench.py cfg2 > $O/${T}_launchprof.log 2>&1 || { tail -5 $O/${T}_launchprof.log; exit 1; }
f=$(find $O/${T}_launchprof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 6
