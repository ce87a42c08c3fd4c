#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv), any counters.

usage: pmc_kernels.py OUT.json DIR [DIR ...]
For every kernel (name cut at its argument list) and counter: the mean value per dispatch
and the dispatch count; kernels matched by substring KEEP (env PMC_KEEP, comma-separated;
default: the PageRank and multi-source BFS kernels and the gather probe)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEEP = os.environ.get("PMC_KEEP", "gather_hot_fx,cold_fx,finalize_long_fx,gather_hot_pf,cold_gather,cold_fold,gather_chunks,lds_window,ms_pull,gather<").split(",")


def short(name):
    for k in KEEP:
        if k in name:
            return k
    return None


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))
            names = {}
            for row in csv.DictReader(open(f)):
                did = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
                k = short(row["Kernel_Name"])
                if k is None:
                    continue
                names[did] = k
                per[did][row["Counter_Name"]] += float(row["Counter_Value"])
            for did, cs in sorted(per.items()):
                for c, v in cs.items():
                    acc[names[did]][c].append(v)
    res = {k: {c: {"mean": sum(v) / len(v), "dispatches": len(v)} for c, v in cs.items()} for k, cs in acc.items()}
    if os.environ.get("PMC_PER_DISPATCH"):      # every dispatch in order (probes that vary per launch)
        for k, cs in acc.items():
            for c, v in cs.items():
                res[k][c]["values"] = v
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, cs in sorted(res.items()):
        print(k, {c: round(x["mean"], 1) for c, x in sorted(cs.items())})


if __name__ == "__main__":
    main()
