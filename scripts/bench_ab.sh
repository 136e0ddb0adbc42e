#!/bin/bash
# A/B of whole source trees on the bench (interleaved): scratch_ab/<v> holds a
# tree with its own in-tree build (VARIANTS="A B"); each runs bench.py (300
# steps) and a rocprofv3 kernel table of a 100-step bench.
#   output: gpurun_out/${T}_bench_ab.txt, gpurun_out/${T}_ab_<v>_<r>/ (rocprof)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${T:-ab}_bench_ab.txt
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in ${VARIANTS:-A B}; do
    cd $R/scratch_ab/$v || exit 2
    echo "== $v round $r" >> $out
    timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline 2>&1 | grep '"metric"' >> $out || exit $?
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T:-ab}_ab_${v}_$r -o run --output-format csv \
      -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > /dev/null 2>&1 || exit $?
    python $R/scripts/kstats.py "$(find $R/gpurun_out/${T:-ab}_ab_${v}_$r -name '*kernel_stats.csv' | head -1)" 4 >> $out
  done
done
cd $R && python - "$out" << 'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(round(d["value"], 1), "it/s")
    else:
        print(l.rstrip()[:110])
PY
