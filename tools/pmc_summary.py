"""Summarise a tools/profile.sh run: per-kernel average duration from the
kernel-trace stats, and per-dispatch PMC counters of the leaf kernel
(k_reduce<true, true, 2>), with the gfx950 FETCH_SIZE x2 correction
(MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a wide
coalesced stream; FETCH_SIZE/WRITE_SIZE are in KiB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

LEAF = os.environ.get("KERNEL", "k_leaf_lock_sc")


def counters(d):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            out[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main(d):
    import socket

    res = {"dir": d, "box": f"GPU box {socket.gethostname()}", "kernel": LEAF}
    stats = glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        res["kernel_stats"] = [
            {"name": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
             "pct": float(r["Percentage"])} for r in csv.DictReader(open(stats[0]))]
    agg = {}
    for sub in ("fetch", "write", "sq", "lds"):
        for k, cs in counters(os.path.join(d, sub)).items():
            if LEAF in k:
                for c, vals in cs.items():
                    # one value per dispatch (summed over XCD/SE instances by rocprofv3)
                    agg[c] = sum(vals) / len(vals)
                    agg[c + "_dispatches"] = len(vals)
    res["leaf_counters_per_dispatch"] = agg
    if os.environ.get("ALL"):  # every kernel's counters, averaged per dispatch
        allk = defaultdict(dict)
        for sub in ("fetch", "write", "sq", "lds"):
            for k, cs in counters(os.path.join(d, sub)).items():
                for c, vals in cs.items():
                    allk[k[:60]][c] = sum(vals) / len(vals)
        res["per_kernel"] = allk
    if "FETCH_SIZE" in agg:
        fetch = agg["FETCH_SIZE"] * 1024 * 2  # KiB -> B, x2 gfx950 correction
        write = agg.get("WRITE_SIZE", 0.0) * 1024
        res["hbm_bytes_per_leaf_launch"] = fetch + write
        res["hbm_fetch_bytes_corrected"] = fetch
        res["hbm_write_bytes"] = write
    if "SQ_INSTS_VALU" in agg and "SQ_WAVES" in agg:
        res["valu_insts_per_wave"] = agg["SQ_INSTS_VALU"] / agg["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in agg and res.get("kernel_stats"):
        leaf = [k for k in res["kernel_stats"] if LEAF in k["name"]]
        if leaf:
            res["effective_clock_GHz"] = agg["GRBM_GUI_ACTIVE"] / 8 / leaf[0]["avg_ns"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
