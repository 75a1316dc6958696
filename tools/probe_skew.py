"""Probe cost when the probe keys are skewed: a fraction f of the rows carry ONE hot key (a member of the filter,
or not), the rest are C2's synthetic probe stream; per filter size and probe strategy (ms per 2^27 keys).

A partitioned probe routes every row of a key to one 128 KiB slice, so a hot key loads one slice's workgroups.
Every timed run's survivors are checked: the strategies must return the same selection vector, and `run(check=...)`
hands each run's keys and survivors to a checker; tests/test_gpu_probe_skew_tool.py runs this tool with the oracle
as that checker (tools may not load the oracle themselves: it is test infrastructure).
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
from strategy_crossover import STRATS  # noqa: E402


def time_probe_sel(bf, keys, n, reps=5):
    """ms per probe (mean of reps after a warm-up) and the survivors (int64 row ids on the host)."""
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
    return e0.elapsed_time(e1) / reps, sel[: int(cnt.item())].cpu().numpy().astype("int64")


def run(check=None, builds=(10**7, 10**8), fractions=(0.0, 0.1, 0.5, 0.9, 1.0), hot_keys=("member", "absent"),
        out=sys.stdout):
    """Time every (filter, hot key, fraction, strategy); assert all strategies return the same survivors and, with
    check(keys, n_build, survivors), what the checker says."""
    lib = rpt_amd.load()
    n = 1 << 27
    for n_build in builds:
        build = rpt_amd.synth_build_keys(n_build)
        bf = rpt_amd.BloomFilter(n_build)
        bf.insert(build)
        torch.cuda.synchronize()
        base = rpt_amd.synth_probe_keys(n, n_build)
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        u = torch.rand(n, device="cuda", generator=g)
        for hot in hot_keys:
            hot_key = build[12345] if hot == "member" else torch.tensor(-77, dtype=torch.int64, device="cuda")
            for f in fractions:
                keys = torch.where(u < f, hot_key, base)
                row = {"op": "probe_skew", "filter_log_blocks": bf.log_num_blocks, "n": n, "hot_key": hot, "hot_fraction": f}
                sels = {}
                for name in ("gather", "partitioned"):
                    if not lib.rpt_probe_strategy_supported(STRATS[name], bf.log_num_blocks):
                        continue
                    bf.probe_strategy = STRATS[name]
                    ms, sels[name] = time_probe_sel(bf, keys, n)
                    row[name + "_ms"] = round(ms, 4)
                bf.probe_strategy = 0
                first = next(iter(sels.values()))
                assert all((s.size == first.size and (s == first).all()) for s in sels.values()), \
                    f"strategies disagree: {row}"
                if check is not None:
                    check(keys, n_build, first)
                    row["checked"] = "oracle"
                row["survivors"] = int(first.size)
                print(json.dumps(row), file=out, flush=True)
        del bf, build, base, u
        torch.cuda.empty_cache()


if __name__ == "__main__":
    run()
