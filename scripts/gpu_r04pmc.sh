#!/bin/bash
# round-4 corr traffic counters (FETCH_SIZE / WRITE_SIZE passes) -> gpurun_out/r04_corr_traffic.json
set -o pipefail
export TMPDIR=/tmp
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" bash scripts/pmc.sh || exit 1
python scripts/traffic_summary.py r04 || exit 1
cp profiles/r04_corr_traffic.json gpurun_out/r04_corr_traffic.json
cat gpurun_out/r04_corr_traffic.json
