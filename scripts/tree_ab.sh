#!/bin/bash
# A/B of whole source trees (scratch_ab/<v>, each with its own in-tree
# build), interleaved: the fork's live BA call at E = 9850
# (scripts/dpvo_window_call.py) and bench.py (300 steps).
#   output: gpurun_out/${T}_tree_ab.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${T:-ab}_tree_ab.txt
mkdir -p $R/gpurun_out
for r in 1 2; do
  for v in ${VARIANTS:-A B}; do
    cd $R/scratch_ab/$v || exit 2
    c=$(timeout -k 10 120 python -u scripts/dpvo_window_call.py 2>&1 | grep '"graph"') || exit 3
    b=$(timeout -k 10 200 python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline 2>&1 | grep '"metric"') || exit 4
    echo "$v $r $c" >> $out
    echo "$v $r $(echo "$b" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "it/s")')" >> $out
  done
done
cat $out
