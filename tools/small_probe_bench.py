"""Fused small-probe latency: one workgroup vs several (probe_small_kernel vs probe_small_mw_kernel).

The several-workgroup kernel was measured in commit 8980ddc and rejected (DESIGN §5 rejected list);
at later commits both modes run the one-workgroup kernel.

Keys in device memory and in pinned host memory (device-mapped, what the DuckDB host mirror passes).
Per n: the synchronized per-call latency (probe + count read back, what a USE_BF vector waits for)
for AUTO with the filter's workspace (several workgroups from RPT_SMALL_MW_MIN_ROWS rows) and with an
8-byte workspace (one workgroup). Run under rocprofv3 --kernel-trace --stats for the kernel durations.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "duckdb-robust-predicate-transfer_amd"))
import rpt_amd as rpt  # noqa: E402
from rpt_amd import bloom as rb  # noqa: E402


def probe(bf, keys, n, sel, cnt, ws):
    """rpt_bf_probe straight through the C-ABI: keys may be pinned host memory (device-mapped)."""
    col = rb.KeyColumn(rb.key_type_of(keys, None), keys.data_ptr(), None, None)
    rb.check(bf._lib.rpt_bf_probe(bf._h, rb.ctypes.byref(col), None, n, sel.data_ptr(), cnt.data_ptr(),
                                  ws.data_ptr(), ws.numel() * ws.element_size(), rb._stream(bf.device, None)))


def main():
    sizes = [int(x) for x in (sys.argv[1:] or ["2048", "4096", "8192", "16384"])]
    rng = np.random.default_rng(7)
    build = rng.integers(-2**40, 2**40, size=1 << 20, dtype=np.int64)
    bf = rpt.BloomFilter(build.size)
    bf.insert(torch.from_numpy(build).cuda())
    tiny = torch.empty(1, dtype=torch.int64, device="cuda")
    big = torch.empty(1 << 16, dtype=torch.int64, device="cuda")
    sel = torch.empty(16384, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    calls = 2000
    for n in sizes:
        pkeys = np.concatenate([build[:n // 10], rng.integers(-2**40, 2**40, size=n - n // 10, dtype=np.int64)])
        for where in ("device", "pinned"):
            keys = torch.from_numpy(pkeys).cuda() if where == "device" else torch.from_numpy(pkeys).pin_memory()
            out = {}
            for mode, ws in (("multi", big), ("one", tiny)):
                probe(bf, keys, n, sel, cnt, ws)
                ref = int(cnt.item())
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(calls):
                    probe(bf, keys, n, sel, cnt, ws)
                    c = int(cnt.item())
                dt = (time.perf_counter() - t0) / calls * 1e6
                assert c == ref
                out[mode] = round(dt, 1)
                out[mode + "_count"] = c
            # the same calls queued back to back (no host round trip between them): kernel durations
            # under the tracer without the GPU idling between calls
            for mode, ws in (("multi", big), ("one", tiny)):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(calls):
                    probe(bf, keys, n, sel, cnt, ws)
                torch.cuda.synchronize()
                out[mode + "_queued"] = round((time.perf_counter() - t0) / calls * 1e6, 1)
            assert out["multi_count"] == out["one_count"]
            print(json.dumps({"op": "small_probe", "n": n, "keys": where, "us_per_call_multi": out["multi"],
                              "us_per_call_one": out["one"],
                              "us_per_call_queued_multi": out["multi_queued"], "us_per_call_queued_one": out["one_queued"],
                              "survivors": out["one_count"]}), flush=True)


if __name__ == "__main__":
    main()
