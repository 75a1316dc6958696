"""Probe cost when the probe keys are skewed: a fraction f of the rows carry ONE hot key (a member of the filter,
or not), the rest are C2's synthetic probe stream; per filter size and probe strategy (ms per 2^27 keys).

A partitioned probe routes every row of a key to one 128 KiB slice, so a hot key loads one slice's workgroups.
Run on a GPU box:
    python tools/probe_skew.py > gpurun_out/probe_skew.jsonl
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))
import rpt_amd  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from strategy_crossover import STRATS, time_probe  # noqa: E402


def main():
    lib = rpt_amd.load()
    n = 1 << 27
    for n_build in (10**7, 10**8):
        build = rpt_amd.synth_build_keys(n_build)
        bf = rpt_amd.BloomFilter(n_build)
        bf.insert(build)
        torch.cuda.synchronize()
        base = rpt_amd.synth_probe_keys(n, n_build)
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        u = torch.rand(n, device="cuda", generator=g)
        for hot in ("member", "absent"):
            hot_key = build[12345] if hot == "member" else torch.tensor(-77, dtype=torch.int64, device="cuda")
            for f in (0.0, 0.1, 0.5, 0.9, 1.0):
                keys = torch.where(u < f, hot_key, base)
                row = {"op": "probe_skew", "filter_log_blocks": bf.log_num_blocks, "n": n, "hot_key": hot, "hot_fraction": f}
                for name in ("gather", "partitioned"):
                    if not lib.rpt_probe_strategy_supported(STRATS[name], bf.log_num_blocks):
                        continue
                    bf.probe_strategy = STRATS[name]
                    row[name + "_ms"] = round(time_probe(bf, keys, n), 4)
                bf.probe_strategy = 0
                print(json.dumps(row), flush=True)
        del bf, build, base, u
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
