#!/bin/bash
# round 4, first GPU call: full GPU suite, BA relative-parity probe, default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04a_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 124|134|137|139) tail -30 gpurun_out/r04a_pytest.txt; exit $rc;; esac
tail -3 gpurun_out/r04a_pytest.txt
timeout -k 10 400 python -u scripts/ba_parity_probe.py --cfg4 > gpurun_out/r04a_probe.jsonl 2>&1 || exit 1
cat gpurun_out/r04a_probe.jsonl
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 > gpurun_out/r04a_bench.json 2>&1 || exit 1
tail -c 600 gpurun_out/r04a_bench.json
