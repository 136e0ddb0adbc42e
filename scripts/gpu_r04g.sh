#!/bin/bash
# plan fast path + dense (patch-partitioned) BA kernel: phases A/B, suite, launches, corr drop-in, profile, harness study
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04g
run() { name=$1; shift; timeout -k 10 200 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; cat $O/${T}_$name.txt; }
run phases_cfg2_block env DPVO_BA_DENSE=0 python -u scripts/ba_window_phases.py cfg2 2
run phases_cfg2_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo25_block env DPVO_BA_DENSE=0 python -u scripts/ba_window_phases.py 25 1
bash scripts/gpu_suite.sh $T || exit 1
run launch python -u scripts/reproject_launch_bench.py
run corr_dropin python -u scripts/corr_dropin_bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
tail -c 300 $O/${T}_prof.log
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 8
timeout -k 10 400 python -u scripts/harness_error_study.py 80 > $O/${T}_harness_study.jsonl 2>&1 || { tail -5 $O/${T}_harness_study.jsonl; exit 1; }
cat $O/${T}_harness_study.jsonl
