"""Per-kernel summary of a rocprofv3 --kernel-trace --stats directory: calls, mean and total time
per kernel (short names), from the *_kernel_stats.csv files below the given directory."""
import csv
import glob
import sys

rows = []
for path in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(path)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows:
    name = r["Name"].split("(")[0].replace("void ", "")
    print(f"{name[:60]:60s} calls {int(r['Calls']):6d}  mean {float(r['AverageNs']) / 1e3:9.2f} us  "
          f"total {float(r['TotalDurationNs']) / 1e6:9.3f} ms")
