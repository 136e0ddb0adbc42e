#!/bin/bash
# granule exchange: phases, GPU suite + bench, launch breakdown, drop-in corr, bench profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python -u scripts/ba_window_phases.py cfg2 2 > $O/r04e_phases_cfg2.txt 2>&1 || { cat $O/r04e_phases_cfg2.txt; exit 1; }
cat $O/r04e_phases_cfg2.txt
timeout -k 10 200 python -u scripts/ba_window_phases.py 25 1 > $O/r04e_phases_dpvo25.txt 2>&1 || exit 1
cat $O/r04e_phases_dpvo25.txt
bash scripts/gpu_suite.sh r04e || exit 1
timeout -k 10 200 python -u scripts/reproject_launch_bench.py > $O/r04e_launch.jsonl 2>&1 || { cat $O/r04e_launch.jsonl; exit 1; }
cat $O/r04e_launch.jsonl
timeout -k 10 300 python -u scripts/corr_dropin_bench.py > $O/r04e_corr_dropin.jsonl 2>&1 || { cat $O/r04e_corr_dropin.jsonl; exit 1; }
cat $O/r04e_corr_dropin.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04e_prof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/r04e_prof.log 2>&1 || { tail -5 $O/r04e_prof.log; exit 1; }
tail -c 300 $O/r04e_prof.log
f=$(find $O/r04e_prof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 8
