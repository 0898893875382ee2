"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total GPU kernel time %.2f ms, %d launches" % (tot / 1e6, sum(int(r["Calls"]) for r in rows)))
for r in rows[:n]:
    print("%6.2f%% %7d %9.1fus  %s" % (float(r["Percentage"]), int(r["Calls"]), float(r["AverageNs"]) / 1e3,
                                         r["Name"][:100]))
