#!/usr/bin/env python3
"""Per-kernel breakdown of a rocprofv3 --kernel-trace CSV (any run), plus the largest dispatches.

usage: ktrace.py DIR [KEEP substrings, comma-separated] [top]
Prints, per kernel (name cut at its argument list): dispatches, total / mean / max µs, and for
the kernels matched by KEEP the `top` longest dispatches in launch order, with the idle gap
before each dispatch summed per kernel (the launch-bound share of a many-step loop)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    return name.split("(")[0]


def main():
    d = sys.argv[1]
    keep = sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] else []
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    tot, cnt, mx, gap = defaultdict(float), defaultdict(int), defaultdict(float), defaultdict(float)
    prev_end = None
    for s, e, k in rows:
        us = (e - s) / 1e3
        tot[k] += us
        cnt[k] += 1
        mx[k] = max(mx[k], us)
        if prev_end is not None and s > prev_end:
            gap[k] += (s - prev_end) / 1e3
        prev_end = max(prev_end or 0, e)
    span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0.0
    print(f"{len(rows)} dispatches over {span:.1f} us; busy {sum(tot.values()):.1f} us; gaps {sum(gap.values()):.1f} us")
    for k in sorted(tot, key=lambda x: -tot[x]):
        print(f"  {k[:48]:48s} n={cnt[k]:6d} total={tot[k]:10.1f} mean={tot[k] / cnt[k]:8.2f} max={mx[k]:8.1f} "
              f"gap_before={gap[k]:8.1f}")
    for k in keep:
        sel = [(e - s, i, s) for i, (s, e, kk) in enumerate(rows) if k in kk]
        sel.sort(reverse=True)
        print(f"top {top} {k}: " + ", ".join(f"#{i}:{dur / 1e3:.1f}us" for dur, i, _ in sorted(sel[:top], key=lambda x: x[1])))


if __name__ == "__main__":
    main()
