"""Achieved memory bandwidth per kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
KB per dispatch) joined with each pass's kernel trace (durations). FETCH_SIZE is doubled: on
gfx950 it reports half of a wide streaming read (MI355X_MICROARCH.md, HBM).
usage: pmc_bw.py <fetch_dir> <write_dir>"""
import collections
import csv
import glob
import os
import sys


def load(d, counter):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(cc)):
        if r["Counter_Name"].startswith(counter):
            vals[r["Kernel_Name"][:80]].append(float(r["Counter_Value"]))
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dur = collections.defaultdict(list)
    if kt:
        for r in csv.DictReader(open(kt[0])):
            dur[r["Kernel_Name"][:80]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, dur


fv, fd = load(sys.argv[1], "FETCH_SIZE")
wv, wd = load(sys.argv[2], "WRITE_SIZE")
rows = []
for k in fv:
    n = len(fv[k])
    fkb = 2 * sum(fv[k]) / n
    wkb = sum(wv.get(k, [0])) / max(len(wv.get(k, [1])), 1)
    d = fd.get(k) or wd.get(k) or [0]
    us = sorted(d)[len(d) // 2] / 1e3
    rows.append((us * n, k, n, us, fkb, wkb, (fkb + wkb) * 1e3 / (us * 1e3) / 1e3 if us else 0))
print("%-80s %6s %9s %10s %10s %8s" % ("kernel", "calls", "med_us", "read_KB", "write_KB", "TB/s"))
for tot, k, n, us, f, w, bw in sorted(rows, reverse=True)[:30]:
    print("%-80s %6d %9.1f %10.0f %10.0f %8.2f" % (k, n, us, f, w, bw))
