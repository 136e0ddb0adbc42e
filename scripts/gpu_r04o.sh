#!/bin/bash
# block GJ with per-thread pivot solves (A/B vs the wave-0 pivot), then r04n (phases + suite)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=r04o
run() { name=$1; shift; timeout -k 10 300 "$@" > $O/${T}_$name.txt 2>&1 || { cat $O/${T}_$name.txt; exit 1; }; tail -6 $O/${T}_$name.txt; }
run bgj_thread ./scripts/micro/bgj_bench
run bgj_wave ./scripts/micro/bgj_bench_wave
run pytest_large python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ba_large_gpu.py tests/test_global_ba_gpu.py
bash scripts/gpu_r04n.sh || exit 1
timeout -k 10 300 python -u bench.py --sharded --steps 5 --warmup 1 --no-cpu-baseline > $O/${T}_cfg4.json 2>&1 || { tail -5 $O/${T}_cfg4.json; exit 1; }
tail -c 600 $O/${T}_cfg4.json
run phases_cfg2_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py cfg2 2
run phases_dpvo25_dense env DPVO_BA_DENSE=1 python -u scripts/ba_window_phases.py 25 1
