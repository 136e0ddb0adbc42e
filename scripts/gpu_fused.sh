set -e
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ba_window_gpu.py -k "fused or insert" > gpurun_out/fused_test.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --separate-insert > gpurun_out/bench_sep.json 2> gpurun_out/bench_sep.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_fused.log 2>&1
bash scripts/ba_shares.sh
