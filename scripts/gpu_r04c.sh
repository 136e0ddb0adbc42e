#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/gj_bench 1 > gpurun_out/r04c_gj_bench.txt 2>&1 || { cat gpurun_out/r04c_gj_bench.txt; exit 1; }
cat gpurun_out/r04c_gj_bench.txt
timeout -k 10 200 python -u scripts/ba_window_phases.py cfg2 2 > gpurun_out/r04c_phases_cfg2.txt 2>&1 || { cat gpurun_out/r04c_phases_cfg2.txt; exit 1; }
cat gpurun_out/r04c_phases_cfg2.txt
timeout -k 10 200 python -u scripts/ba_window_phases.py 25 1 > gpurun_out/r04c_phases_dpvo25.txt 2>&1 || exit 1
cat gpurun_out/r04c_phases_dpvo25.txt
bash scripts/gpu_suite.sh r04c
