#!/bin/bash
# A/B of builds of the A-CORR kernels in one GPU call (interleaved runs):
#   scratch_ab/<v> = copies of dpvo_amd/_native built from different trees
#   (VARIANTS="old new" by default); output gpurun_out/${T}_corr_ab.txt
set -o pipefail
out=gpurun_out/${T:-ab}_corr_ab.txt
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${VARIANTS:-old new}; do
    timeout -k 10 120 python -u scripts/corr_variants.py --features ${FEATS:-f32,f16} --native scratch_ab/$v >> $out 2>&1 || exit $?
  done
done
grep features $out
