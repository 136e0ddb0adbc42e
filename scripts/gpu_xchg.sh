set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ba_window_gpu.py tests/test_golden_gpu.py tests/test_ba_gpu.py tests/test_update_harness_gpu.py > gpurun_out/xchg_tests.log 2>&1
timeout -k 10 200 python scripts/ba_window_phases.py cfg2 2 > gpurun_out/xchg_phases.txt 2>&1
timeout -k 10 300 python scripts/ba_repeat_check.py > gpurun_out/xchg_repeat.txt 2>&1
timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/xchg_bench.json 2>/dev/null
