#!/usr/bin/env python3
"""The last window of a rocprofv3 --kernel-trace CSV in launch order: every dispatch from the
last one whose name contains START to the end of the trace (or the next START), with its
duration and the idle gap before it — one multi-source sweep or one SSSP run read kernel by
kernel — then the window's totals per kernel.

usage: ktimeline.py DIR START [skip]   (skip: drop that many trailing windows first)"""
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1).replace("tgo::", "")
    return name.split("(")[0][:60]


def main():
    d, start = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if start in r[2]]
    if len(marks) <= skip:
        sys.exit(f"no window starting at {start!r}")
    lo = marks[-1 - skip]
    hi = marks[-skip] if skip else len(rows)
    t0 = rows[lo][0]
    prev = None
    busy = 0.0
    for s, e, name in rows[lo:hi]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        busy += (e - s) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {name}")
        prev = e
    print(f"window {(rows[hi - 1][1] - t0) / 1e3:.1f} us, kernels busy {busy:.1f} us, {hi - lo} dispatches")
    per = {}
    prev = None
    for s, e, name in rows[lo:hi]:
        c = per.setdefault(name, [0, 0.0, 0.0])
        c[0] += 1
        c[1] += (e - s) / 1e3
        c[2] += max(0.0, (s - prev) / 1e3) if prev is not None else 0.0
        prev = e
    for name, (c, t, g) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"  {name:60s} n={c:5d} busy {t:9.1f} us  gaps before {g:8.1f} us")


if __name__ == "__main__":
    main()
