#!/usr/bin/env python3
"""Quick cross-strategy check on the GPU: probe the same keys with every supported strategy, compare
with the oracle and print per-kernel device times (developer tool)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"), os.path.join(REPO, "oracle")]
import rpt_amd  # noqa: E402
import rpt_oracle as orc  # noqa: E402
from rpt_amd import _lib  # noqa: E402

n_build = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10**6
n_probe = int(float(sys.argv[2])) if len(sys.argv) > 2 else 4 * 10**6
log_nb = int(sys.argv[3]) if len(sys.argv) > 3 else None
torch.cuda.set_device(0)
bkeys = rpt_amd.synth_build_keys(n_build)
pkeys = rpt_amd.synth_probe_keys(n_probe, n_build, 100)
bf = rpt_amd.BloomFilter(n_build) if log_nb is None else rpt_amd.BloomFilter(log_num_blocks=log_nb)
bf.insert(bkeys)
L = bf.log_num_blocks
w = bf.export_words()
ref = orc.probe_keys(w, L, pkeys.cpu().numpy())
print(f"filter 2^{L} blocks, {n_probe} probes, oracle survivors {ref.size}")
for st, name in [(1, "gather"), (2, "lds"), (3, "partitioned")]:
    if not _lib.load().rpt_probe_strategy_supported(st, L):
        print(f"{name:12s} n/a")
        continue
    bf.probe_strategy = st
    _lib.profiling_reset()
    _lib.profiling(True)
    sel = bf.lookup_sel(pkeys)
    torch.cuda.synchronize()
    _lib.profiling(False)
    kt = {k: round(v[1] / v[0], 3) for k, v in _lib.kernel_times().items()}
    got = sel.cpu().numpy().view(np.uint32)
    ok = np.array_equal(got, ref)
    print(f"{name:12s} {'OK ' if ok else 'MISMATCH'} survivors {got.size} kernels_ms {kt}")
    if not ok:
        gs, rs = set(got.tolist()), set(ref.tolist())
        missing = sorted(rs - gs)
        extra = sorted(gs - rs)
        print(f"   missing {len(missing)} (first {missing[:8]}), extra {len(extra)} (first {extra[:8]})")
        if missing:
            m = np.array(missing)
            print("   missing rows by 16Ki tile:", np.bincount(m // 16384)[:20].tolist())
