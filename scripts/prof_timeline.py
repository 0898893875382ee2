"""Timeline view of a rocprofv3 --kernel-trace CSV: for the last N occurrences of a marker kernel
(one per training step), the step span, the summed kernel time, the idle gaps between kernels
and the per-kernel-family time / launch count / median workgroups inside the steps.

    python scripts/prof_timeline.py <kernel_trace.csv> <marker substring> [steps=5]
"""
import collections
import csv
import statistics
import sys


def main():
    path, marker = sys.argv[1], sys.argv[2]
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        gy = int(r.get("Grid_Size_Y", 1) or 1)
        wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        wy = int(r.get("Workgroup_Size_Y", 1) or 1)
        wgs = max(1, (gx // max(wx, 1))) * max(1, (gy // max(wy, 1)))
        ks.append((st, en, name, wgs))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if marker in k[2]]
    if len(marks) < 2:
        print("marker %r found %d times" % (marker, len(marks)))
        return
    marks = marks[-(nsteps + 1):]
    spans, busy, gaps, launches = [], [], [], []
    fam = collections.defaultdict(lambda: [0.0, 0, []])
    for a, b in zip(marks, marks[1:]):
        seg = ks[a:b]
        spans.append((ks[b][0] - seg[0][0]) / 1e3)
        busy.append(sum(e - s for s, e, _, _ in seg) / 1e3)
        g = 0
        for (s0, e0, _, _), (s1, _, _, _) in zip(seg, seg[1:]):
            g += max(0, s1 - e0)
        gaps.append(g / 1e3)
        launches.append(len(seg))
        for s, e, n, w in seg:
            short = n.split("(")[0].replace("void ", "")[:70]
            f = fam[short]
            f[0] += (e - s) / 1e3
            f[1] += 1
            f[2].append(w)
    n = len(spans)
    print("steps %d: span %.1f us, kernel busy %.1f us, gaps %.1f us, launches %d (per step, median)"
          % (n, statistics.median(spans), statistics.median(busy), statistics.median(gaps),
             statistics.median(launches)))
    print("%-72s %9s %7s %8s %7s" % ("kernel", "us/step", "calls", "us/call", "WGs"))
    for k, (t, c, w) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:40]:
        print("%-72s %9.1f %7.1f %8.2f %7d" % (k, t / n, c / n, t / c, int(statistics.median(w))))


if __name__ == "__main__":
    main()
