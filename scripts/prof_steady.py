"""Steady-state kernel summary from a rocprofv3 kernel_trace.csv: drops everything up to the
last MIOpen/CK tuning launch (find-mode benchmarking in the warmup steps) and reports the
top kernels of the remaining trace."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tune = [i for i, r in enumerate(rows) if "naive_conv" in r["Kernel_Name"] or "batched_gemm_xdlops_bwd" in r["Kernel_Name"]]
rows = rows[(tune[-1] + 1 if tune else 0):]
agg = collections.defaultdict(lambda: [0, 0])
for r in rows:
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = sum(v[1] for v in agg.values())
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print("steady state: %d launches, kernel time %.2f ms over a %.2f ms span (%.0f%% busy)"
      % (len(rows), tot / 1e6, span / 1e6, 100.0 * tot / span))
for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:n]:
    print("%6.2f%% %7d %9.1fus  %s" % (100.0 * t / tot, c, t / c / 1e3, name[:100]))
