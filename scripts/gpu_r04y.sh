#!/bin/bash
# full suite + smoke + bench, bench kernel profile, cfg4 sharded line, launch profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04y
bash scripts/gpu_suite.sh $T || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 6
timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline > $O/${T}_bench300.json 2>&1 || exit 1
tail -c 400 $O/${T}_bench300.json
