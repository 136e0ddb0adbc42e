set -e
cd "${GRAFT_REPO_ROOT:-.}"
SQ_EXTRA="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" bash scripts/pmc_sq.sh
PMC_GROUPS="FETCH_SIZE WRITE_SIZE" bash scripts/pmc.sh
python scripts/sq_summary.py gpurun_out > gpurun_out/sq_summary_r03.json
