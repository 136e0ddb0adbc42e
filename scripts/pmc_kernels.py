"""Per-kernel medians of rocprofv3 --pmc counters (one value per dispatch:
the rows of a dispatch are summed).

    python scripts/pmc_kernels.py 'gpurun_out/pmc_*/run_counter_collection.csv'
"""
import collections
import csv
import glob
import sys

SHORT = [("corr_nhwc", "corr"), ("ba_window_kernel", "ba_window"),
         ("reproject_plan_insert", "fused_launch"), ("ba_plan_kernel", "plan"),
         ("corr_nchw", "corr_nchw")]


FULL = False  # argv[2] == "full": group by the whole kernel name (template variants apart)


def short(name):
    if FULL:
        return name.split("(")[0][-70:] if any(k in name for k, _ in SHORT) else None
    for k, v in SHORT:
        if k in name:
            return v
    return None


def main():
    global FULL
    FULL = len(sys.argv) > 2 and sys.argv[2] == "full"
    for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else
                              "gpurun_out/pmc_*/run_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                per[(k, r["Counter_Name"], r.get("Dispatch_Id", r.get("Correlation_Id")))] += \
                    float(r["Counter_Value"])
        agg = collections.defaultdict(list)
        for (k, c, _), v in per.items():
            agg[(k, c)].append(v)
        for (k, c), v in sorted(agg.items()):
            v.sort()
            print(f"{f.split('/')[1]:12s} {k:13s} {c:28s} n={len(v):4d} median {v[len(v) // 2]:.0f}")


if __name__ == "__main__":
    main()
