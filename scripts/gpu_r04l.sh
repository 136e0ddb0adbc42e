#!/bin/bash
# full GPU suite + smoke + bench, then the cfg2-only launch profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04l
bash scripts/gpu_suite.sh $T || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_launchprof -o run --output-format csv -- python scripts/reproject_launch_bench.py cfg2 > $O/${T}_launchprof.log 2>&1 || { tail -5 $O/${T}_launchprof.log; exit 1; }
f=$(find $O/${T}_launchprof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 6
