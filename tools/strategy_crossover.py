#!/usr/bin/env python3
"""Time every applicable probe strategy for batch sizes 2^12..2^28 against filters of several sizes
(device-resident keys, HIP events). Used to set the AUTO thresholds (rpt_gpu.hip resolve_strategy)."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))
import rpt_amd  # noqa: E402

STRATS = {"gather": 1, "lds": 2, "partitioned": 3, "bucketed": 4}


def time_probe(bf, keys, n, reps=5):
    ws = torch.empty(bf.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    sel = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    bf.probe_async(keys, n=n, out_sel=sel, out_count=cnt, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        bf.probe_async(keys, n=n, out_sel=sel, out_count=cnt, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def time_insert(bf, keys, n, strategy, reps=3):
    bf.insert(keys[:n], strategy=strategy)  # warm-up (workspace, code objects)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        bf.insert(keys[:n], strategy=strategy)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def insert_sweep():
    lib = rpt_amd.load()
    keys = rpt_amd.synth_build_keys(1 << 27)
    for L in (12, 14, 16, 18, 21, 24, 27):
        bf = rpt_amd.BloomFilter(log_num_blocks=L)
        for lg in (16, 20, 21, 22, 24, 26):
            n = 1 << lg
            lib.rpt_bf_set_insert_strategy(bf._h, 0)  # time_insert pins a strategy: AUTO's choice first
            row = {"op": "insert", "log_blocks": L, "n": n, "auto": bf.insert_strategy_for(n)}
            for name, st in (("atomic", 1), ("partitioned", 2), ("bucketed", 3)):
                if (st == 2 and not lib.rpt_probe_strategy_supported(3, L)) or (st == 3 and not lib.rpt_probe_strategy_supported(4, L)):
                    continue
                row[name] = round(time_insert(bf, keys, n, st), 4)
            print(json.dumps(row), flush=True)
        del bf
        torch.cuda.empty_cache()


def mid_sweep():
    """128 KiB .. 8 MiB filters (1 .. 64 slices), where the LDS, gather and partitioned probes cross."""
    lib = rpt_amd.load()
    n_max = 1 << 28
    for build in (10**5, 2 * 10**5, 4 * 10**5, 8 * 10**5, 16 * 10**5, 32 * 10**5, 64 * 10**5):
        bf = rpt_amd.BloomFilter(build)
        bf.insert(rpt_amd.synth_build_keys(build))
        L = bf.log_num_blocks
        keys = rpt_amd.synth_probe_keys(n_max, build, 100)
        for lg in range(16, 29, 2):
            n = 1 << lg
            row = {"op": "probe_mid", "build": build, "log_blocks": L, "n": n, "auto": bf.probe_strategy_for(n)}
            for name, st in STRATS.items():
                if st == 4 or not lib.rpt_probe_strategy_supported(st, L):
                    continue
                bf.probe_strategy = st
                row[name] = round(time_probe(bf, keys, n), 4)
            bf.probe_strategy = 0
            print(json.dumps(row), flush=True)
        del bf, keys
        torch.cuda.empty_cache()


def main():
    if "--insert" in sys.argv:
        return insert_sweep()
    if "--mid" in sys.argv:
        return mid_sweep()
    lib = rpt_amd.load()
    n_max = 1 << 28
    for build in (10**5, 10**7, 3 * 10**7, 10**8, 10**9):
        bf = rpt_amd.BloomFilter(build)
        bf.insert(rpt_amd.synth_build_keys(min(build, 10**8)))
        L = bf.log_num_blocks
        keys = rpt_amd.synth_probe_keys(n_max, min(build, 10**8), 100)
        for lg in range(12, 29, 2):
            n = 1 << lg
            row = {"build": build, "log_blocks": L, "n": n, "auto": bf.probe_strategy_for(n)}
            for name, st in STRATS.items():
                if not lib.rpt_probe_strategy_supported(st, L):
                    continue
                bf.probe_strategy = st
                row[name] = round(time_probe(bf, keys, n), 4)
            bf.probe_strategy = 0
            print(json.dumps(row), flush=True)
        del bf, keys
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
