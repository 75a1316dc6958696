#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (one counter set per pass) into per-kernel averages and HBM
bytes per launch, corrected as MI355X_MICROARCH.md §HBM prescribes:
  FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports 1/2 of a wide (16 B/lane) coalesced
  read stream -> doubled; WRITE_SIZE is exact for 16 B/lane stores (other widths uncalibrated).
Usage: pmc_summary.py PMC_DIR KERNEL_TRACE_STATS_CSV OUT_JSON ROUND_TAG
"""
import collections
import csv
import glob
import json
import re
import sys


def short(name: str) -> str:
    """rpt::kernel plus its template arguments (the probe and build instantiations of one kernel
    differ there), e.g. partition_kernel<0,true,false>."""
    m = re.search(r"rpt::(\w+)(<[^>]*>)?", name)
    if not m:
        return name.split("(")[0][:48]
    return m.group(1) + (m.group(2).replace(" ", "") if m.group(2) else "")


def main(pmc_dir, stats_csv, out_json, tag):
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = {}
    for r in csv.DictReader(open(stats_csv)):
        durs[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
    out = {"round": tag, "note": __doc__.strip().splitlines()[0], "kernels": {}}
    for k, cs in ctr.items():
        med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
        entry = {"counters_median_per_launch": med}
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            rd = 2 * med["FETCH_SIZE"] * 1024
            wr = med["WRITE_SIZE"] * 1024
            entry.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes_per_launch=rd + wr)
        if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med and med["TCC_HIT_sum"] + med["TCC_MISS_sum"] > 0:
            entry["l2_hit_rate"] = med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
        if k in durs:
            entry.update(durs[k])
            if "hbm_bytes_per_launch" in entry:
                entry["hbm_GBps"] = entry["hbm_bytes_per_launch"] / (durs[k]["avg_ms"] * 1e-3) / 1e9
        if "GRBM_GUI_ACTIVE" in med and k in durs:
            entry["effective_clock_GHz"] = med["GRBM_GUI_ACTIVE"] / 8 / (durs[k]["avg_ms"] * 1e-3) / 1e9
        out["kernels"][k] = entry
    json.dump(out, open(out_json, "w"), indent=1, sort_keys=True)
    for k, e in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("avg_ms", 0)):
        print(f"{k:24s} avg {e.get('avg_ms', 0):7.3f} ms  HBM {e.get('hbm_bytes_per_launch', 0)/1e9:7.3f} GB "
              f"({e.get('hbm_GBps', 0):7.0f} GB/s)  L2 hit {e.get('l2_hit_rate', 0):.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:5])
