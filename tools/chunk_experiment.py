#!/usr/bin/env python3
"""Experiment: does the partitioned probe get faster when it runs over row chunks whose intermediates
(records, row map, pass bits: ~6.4 B/row) stay resident in the 256 MiB Infinity Cache?

Probes the C2 workload (1e9 int64 keys vs the 1e7-key / 16 MiB filter) as ONE rpt_bf_probe call and
as a loop of rpt_bf_probe calls over chunks of 2^k rows that reuse one workspace, and prints device
time per 1e9 keys (HIP events around the whole loop). Each chunk's sel lands at its own offset (the
concatenation is not compacted: this measures the kernels, not the API).
  python3 tools/chunk_experiment.py [--log-chunks 22 23 24 25 26]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))
import rpt_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-chunks", type=int, nargs="*", default=[21, 22, 23, 24, 25, 26, 27])
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--build", type=float, default=1e7)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n, nb = int(args.n), int(args.build)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bf = rpt_amd.BloomFilter(nb, device=dev)
    bf.insert(rpt_amd.synth_build_keys(nb, device=dev))
    keys = rpt_amd.synth_probe_keys(n, nb, 100, device=dev)
    sel = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.zeros(1024, dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for lg in [None] + args.log_chunks:
        chunk = n if lg is None else 1 << lg
        ws = torch.empty(bf.workspace_bytes(min(chunk, n)), dtype=torch.uint8, device=dev)
        times = []
        for rep in range(args.reps + 1):
            e0.record()
            for i, lo in enumerate(range(0, n, chunk)):
                hi = min(n, lo + chunk)
                bf.probe_async(keys[lo:hi], n=hi - lo, out_sel=sel[lo:hi], out_count=counts[i % 1024:i % 1024 + 1],
                               workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                times.append(e0.elapsed_time(e1))
        times.sort()
        print(f"chunk {'all' if lg is None else '2^%d' % lg:>5s} ({(n + chunk - 1) // chunk:5d} calls, ws "
              f"{ws.numel() / 2**20:8.1f} MiB): {times[len(times) // 2] * 1e9 / n:7.3f} ms per 1e9 keys "
              f"(min {times[0] * 1e9 / n:.3f})", flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
