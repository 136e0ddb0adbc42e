#!/bin/bash
# channel-split corr kernel + sharded plan + dense BA kernel (edge masks): parity, A/B, profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04i
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -3 $O/${T}_$name.txt; }
run bgj0 ./scripts/micro/bgj_bench
run pytest_corr python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_corr_gpu.py tests/test_golden_gpu.py
run pytest_plan python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ba_window_gpu.py -k "plan or fused"
run bench_split python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline
run bench_nosplit env DPVO_CORR_SPLIT=0 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 8
run launch python -u scripts/reproject_launch_bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_launchprof -o run --output-format csv -- python scripts/reproject_launch_bench.py > $O/${T}_launchprof.log 2>&1 || { tail -5 $O/${T}_launchprof.log; exit 1; }
f=$(find $O/${T}_launchprof -name "*kernel_stats.csv" | head -1); python scripts/kstats.py $f 12
run phases_cfg2_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo25_block env DPVO_BA_DENSE=0 python -u scripts/ba_window_phases.py 25 1
run phases_dpvo10_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 10 1
run phases_dpvo10_block env DPVO_BA_DENSE=0 python -u scripts/ba_window_phases.py 10 1
run pytest_dense env DPVO_BA_DENSE=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ba_window_gpu.py tests/test_update_harness_gpu.py tests/test_ba_gpu.py
run pytest_m20 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_update_harness_gpu.py -k m20
