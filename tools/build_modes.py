#!/usr/bin/env python3
"""Build time by slice-merge mode (one GPU): the insert of --rows keys into a filter sized for
--filter-rows, (a) into a fresh filter (pristine: plain stores), (b) after rpt_bf_clear (the deferred
clear: every slice stored whole), (c) into a filter that already holds them (read-modify-write).
Device time per insert, HIP events on the current stream, median of --reps.
  python3 tools/build_modes.py [--rows 1e9] [--filter-rows 8e9]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))
import rpt_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--filter-rows", type=float, default=8e9)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    keys = rpt_amd.synth_build_keys(int(args.rows), device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"fresh": [], "after_clear": [], "rmw": []}
    for _ in range(args.reps):
        bf = rpt_amd.BloomFilter(int(args.filter_rows), device=dev)
        bf.insert(keys[:1 << 20])  # workspace / code-object warm-up
        bf.close()
        bf = rpt_amd.BloomFilter(int(args.filter_rows), device=dev)
        torch.cuda.synchronize()
        for mode in ("fresh", "rmw", "after_clear"):
            if mode == "after_clear":
                bf.clear()
            e0.record()
            bf.insert(keys)
            e1.record()
            torch.cuda.synchronize()
            res[mode].append(e0.elapsed_time(e1))
        bf.close()
        torch.cuda.empty_cache()
    for k, v in res.items():
        v.sort()
        print(f"{k:12s} {v[len(v) // 2]:8.3f} ms (min {v[0]:.3f})", flush=True)


if __name__ == "__main__":
    main()
