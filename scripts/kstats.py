"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:n]:
    print(f"{x['Name'][:60]:60s} calls={x['Calls']:>6} avg_us={float(x['AverageNs'])/1e3:9.1f} "
          f"tot_ms={float(x['TotalDurationNs'])/1e6:8.2f}")
