"""Ordered kernel sequence of one training step from a rocprofv3 --kernel-trace CSV: the kernels
between the last two occurrences of a marker kernel, one line each (start offset, duration,
workgroups, short name), so framework (at::) launches can be located next to the HIP kernels
around them.

    python scripts/prof_sequence.py <kernel_trace.csv> <marker substring> [filter substring]
"""
import csv
import sys


def main():
    path, marker = sys.argv[1], sys.argv[2]
    filt = sys.argv[3] if len(sys.argv) > 3 else None
    ks = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        gy = int(r.get("Grid_Size_Y", 1) or 1)
        wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, max(1, gx // max(wx, 1)) * gy))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if marker in k[2]]
    if len(marks) < 2:
        print("marker %r found %d times" % (marker, len(marks)))
        return
    a, b = marks[-2], marks[-1]
    t0 = ks[a][0]
    for i in range(a, b):
        st, en, name, wgs = ks[i]
        short = name.split("(")[0][:90]
        if filt and filt not in name:
            continue
        print("%4d %9.1f %7.2f %6d  %s" % (i - a, (st - t0) / 1e3, (en - st) / 1e3, wgs, short))


if __name__ == "__main__":
    main()
