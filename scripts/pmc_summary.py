"""Per-kernel sums of rocprofv3 --pmc counters (counter_collection.csv), top kernels by
SQ_WAVE_CYCLES (or the first counter) summed over dispatches; usage: pmc_summary.py <counter_collection.csv> [top]."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:90]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    calls[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
names = sorted({c for v in agg.values() for c in v})
print("%-90s %7s " % ("kernel", "calls") + " ".join("%22s" % c for c in names))
key = "SQ_WAVE_CYCLES" if "SQ_WAVE_CYCLES" in names else names[0]
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get(key, 0) * len(calls[kv[0]]))[:top]:
    n = max(len(calls[k]), 1)
    print("%-90s %7d " % (k, n) + " ".join("%22.4g" % (v[c] / n) for c in names))
print("(values are per-dispatch means)")
