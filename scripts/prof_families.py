"""Aggregate a rocprofv3 kernel_stats.csv by kernel family (template arguments dropped)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
tot = sum(float(r["TotalDurationNs"]) for r in rows)
fam = collections.defaultdict(lambda: [0.0, 0])
for r in rows:
    m = re.search(r"katib_hip::(?:\w+::)*?(\w+_kernel)", r["Name"])
    k = m.group(1) if m else r["Name"][:48]
    fam[k][0] += float(r["TotalDurationNs"])
    fam[k][1] += int(r["Calls"])
print("total GPU kernel time %.2f ms" % (tot / 1e6))
for k, (v, c) in sorted(fam.items(), key=lambda x: -x[1][0])[:n]:
    print("%6.2f%% %9.2f ms %6d calls  %s" % (100 * v / tot, v / 1e6, c, k))
