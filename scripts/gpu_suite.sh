#!/bin/bash
# GPU suite + smoke + default bench (tag = $1)
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/${tag}_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2>&1 || exit 1
tail -c 300 gpurun_out/${tag}_bench.json
