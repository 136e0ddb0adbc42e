"""Per-launch HBM traffic of the dominant kernel from the PMC passes of
scripts/pmc.sh (PMC_GROUPS="FETCH_SIZE WRITE_SIZE").

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE tallies wide coalesced
reads at half their bytes, so it is doubled; WRITE_SIZE is taken as is.
Writes profiles/<round>_corr_traffic.json, which bench.py reports as
roofline.traffic.

usage: python scripts/traffic_summary.py [round-tag]
"""
import csv
import glob
import json
import statistics
import sys

KERNEL = "corr_nhwc_lvl_kernel"  # the fp32 A-CORR kernel of the bench (round 6)


def per_launch(counter):
    vals = []
    for f in glob.glob("gpurun_out/pmc_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} samples for {KERNEL}")
    return statistics.median(vals), len(vals)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    fetch_kib, nf = per_launch("FETCH_SIZE")
    write_kib, nw = per_launch("WRITE_SIZE")
    out = {
        "kernel": KERNEL,
        "workload": "cfg2 (bench.py default)",
        "fetch_size_kib_median": fetch_kib,
        "write_size_kib_median": write_kib,
        "launches": [nf, nw],
        "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count)",
        "traffic_bytes_per_launch": 2 * fetch_kib * 1024 + write_kib * 1024,
    }
    path = f"profiles/{tag}_corr_traffic.json"
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
