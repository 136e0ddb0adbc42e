#!/bin/bash
# Build the A-CORR micro-bench variants used by `scripts/gpu.sh corrmicro`
# (run from the repo root, on the CPU side): base, exact (every tile on the
# exact f32 MFMAs), nomma (no matrix ops), noload (no tile loads), noconv
# (fp32 tiles taken as ready split-f16 halves: no per-tile conversion).
set -e
cd "$(dirname "$0")/../.."
for v in base: exact:-DCORR_DIAG_EXACT_F32 nomma:-DCORR_DIAG_NO_MMA noload:-DCORR_DIAG_NO_LOAD noconv:-DCORR_DIAG_NO_CONV; do
  n=${v%%:*}; f=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -I include -I dpvo_amd/csrc $f \
    scripts/micro/corr_bench.hip -o scripts/micro/corr_bench_$n &
done
wait
