"""Per-kernel mean of the SQ counters collected by scripts/pmc_sq.sh
(rocprofv3 counter_collection.csv of each pass), for the hot-path kernels.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md)."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/sq_*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        short = next((k for k in ("ba_window_kernel", "ba_plan_kernel", "corr_nhwc_lvl_kernel", "corr_nhwc_kernel", "reproject_plan_insert_kernel",
                                  "pyramid_insert_kernel", "reproject_kernel") if k in name), None)
        if short is None:
            continue
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
for k, d in out.items():
    if "SQ_WAVE_CYCLES" in d:
        w = d["SQ_WAVE_CYCLES"]
        d["frac_wait_any"] = d.get("SQ_WAIT_ANY", 0) / w
        d["frac_wait_inst_any"] = d.get("SQ_WAIT_INST_ANY", 0) / w
        d["frac_active_inst_any"] = d.get("SQ_ACTIVE_INST_ANY", 0) / w
    if "SQ_LDS_IDX_ACTIVE" in d and d["SQ_LDS_IDX_ACTIVE"]:
        d["lds_bank_conflict_frac"] = d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"]
print(json.dumps(out, indent=1))
