#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes into per-launch HBM traffic for bench.py's roofline.

usage: pmc_traffic.py OUT.json FETCH_DIR WRITE_DIR [HIT_DIR [EA_DIR [REQ_DIR]]]

Each *_DIR holds one rocprofv3 `--pmc` pass (`--output-format csv`) of the same bench
command: FETCH_SIZE, WRITE_SIZE and (optionally) TCC_HIT_sum + TCC_MISS_sum.  Kernels are
grouped the way bench.py prices them:

  pagerank_update : gather_short + gather_chunks + finalize_long (one group = one rank update)
  msbfs_sweep     : ms_seed + ms_pull + ms_push + ms_settle (one group = one 64-source sweep)
  sssp_source     : the delta-stepping device loop's kernels (one group = one source)

Corrections (MI355X_MICROARCH.md §HBM, calibrated for these access shapes by
scripts/pmc_calib.hip, profiles/r02f_pmc_calibration.txt): FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE = TCC_EA0_RDREQ x 64 B while every request moves a 128-byte line — for 16-B
and 4-B-per-lane streams AND for random 8-byte gathers alike — so `traffic` doubles it.
WRITE_SIZE is exact for 8-byte-per-lane stores.  Infinity-Cache hits are counted like HBM
reads (a warmed 128 MiB table gave the same requests per gather as a 2 GiB one), so
`traffic` is L2->fabric line traffic, an upper bound on HBM bytes; TCC_EA0_RDREQ is kept
beside it as the request count that bounds the gather (~55 G requests/s measured).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GROUPS = {
    # one rank update of the cache-blocked gather (spmv.hip): cold pass, fold, hot pass, long rows
    # (gather_hot_pf: the prefetching hot pass; gather_short_packed: its TGO_PR_PF=0 form)
    # (round 5 default: cold_fx + cold_fold + gather_hot_fx + finalize_long_fx, fixed-point tile sums)
    "pagerank_update": ("cold_gather<", "cold_fold(", "gather_hot_pf<", "gather_hot_pf(", "gather_short_packed<",
                        "gather_chunks<tgo::(anonymous namespace)::PackedOp",
                        "finalize_long<tgo::(anonymous namespace)::PackedOp",
                        "cold_fx<", "gather_hot_fx<", "finalize_long_fx("),
    # ms_pull is templated on its round-trip width (ms_pull<8>)
    "msbfs_sweep": ("ms_seed(", "ms_pull(", "ms_pull<", "ms_push(", "ms_settle(", "ms_queue(", "ms_fbitmap("),
    # one delta-stepping source of the device-driven loop (delta_loop.hip): every step's kernels
    "sssp_source": ("ds_loop_seed(", "ds_decide(", "ds_decide_bins(", "ds_extract_dev(", "ds_extract_bins(",
                    "ds_commit_dev<", "ds_relax_dev<", "ds_pull_heavy(", "ds_publish(", "ds_pull_flip("),
}
# one dispatch per unit: the fixed-point hot pass counts only its emitting launch (kPass 0, or
# kPass 2 = the last of a source split) — counting every gather_hot_fx dispatch halved the
# round-5 per-update figures (two launches an update with TGO_PR_FX_SPLIT=2)
UNIT_KERNEL = {"pagerank_update": ("gather_hot_pf<", "gather_hot_pf(", "gather_short_packed<", "gather_hot_fx<4096, 0, 0,",
                                   "gather_hot_fx<4096, 0, 2,", "gather_hot_fx<8192, 0, 0,"),
               "msbfs_sweep": ("ms_seed(",), "sssp_source": ("ds_loop_seed(",)}


def load(d):
    """{(dispatch_id): (kernel_name, {counter: value})} of one pass."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            did = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            name = row["Kernel_Name"]
            ent = out.setdefault(did, (name, defaultdict(float)))
            ent[1][row["Counter_Name"]] += float(row["Counter_Value"])
    return out


def group_of(name):
    for g, keys in GROUPS.items():
        if any(k in name for k in keys):
            return g
    return None


def per_unit(passes, counter):
    tot, units = defaultdict(float), defaultdict(int)
    for p in passes:
        for _, (name, cs) in p.items():
            g = group_of(name)
            if g is None or counter not in cs:
                continue
            tot[g] += cs[counter]
            if any(k in name for k in UNIT_KERNEL[g]):
                units[g] += 1
    return {g: tot[g] / units[g] for g in tot if units[g]}


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    passes = [load(d) for d in dirs]
    fetch = per_unit(passes, "FETCH_SIZE")
    write = per_unit(passes, "WRITE_SIZE")
    rdreq = per_unit(passes, "TCC_EA0_RDREQ_sum")
    hit = per_unit(passes, "TCC_HIT_sum")
    miss = per_unit(passes, "TCC_MISS_sum")
    # request-rate set: L2 requests, and busy cycles over all 128 L2 channels /
    # 256 TAs against the XCD cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
    req = per_unit(passes, "TCC_REQ_sum")
    l1req = per_unit(passes, "TCP_TCC_READ_REQ_sum")
    busy = per_unit(passes, "TCC_BUSY_sum")
    ta = per_unit(passes, "TA_TA_BUSY_sum")
    gui = per_unit(passes, "GRBM_GUI_ACTIVE")
    res = {}
    for g in GROUPS:
        if g not in fetch or g not in write:
            continue
        f_b, w_b = fetch[g] * 1024.0, write[g] * 1024.0
        ent = {"fetch_bytes_raw": f_b, "write_bytes": w_b, "traffic_bytes": 2.0 * f_b + w_b,
               "correction": "FETCH_SIZE x2 (one 128-B line per TCC_EA0_RDREQ, tallied as 64 B; calibrated for streams "
                             "and 8-B gathers, profiles/r02f_pmc_calibration.txt), WRITE_SIZE x1; KiB->B; Infinity-Cache "
                             "hits included"}
        if g in rdreq:
            ent["ea_read_requests"] = rdreq[g]
        if g in hit and g in miss and hit[g] + miss[g] > 0:
            ent["l2_hit_rate"] = hit[g] / (hit[g] + miss[g])
        if g in req:
            ent["l2_requests"] = req[g]
        if g in l1req:
            ent["l1_to_l2_read_requests"] = l1req[g]
        if g in gui and gui[g] > 0:
            cyc = gui[g] / 8.0
            if g in busy:
                ent["l2_channel_busy"] = busy[g] / (128.0 * cyc)
            if g in ta:
                ent["ta_busy"] = ta[g] / (256.0 * cyc)
        res[g] = ent
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
