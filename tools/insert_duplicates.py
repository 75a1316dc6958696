"""Insert cost when keys repeat: random keys vs CONSTANT chunks (2048 equal keys), one key for the whole
batch, and 1000 distinct keys in random order, per filter size and insert strategy (ms per call).

Memory-side atomics on one word serialize; the partitioned insert ORs in LDS first. Run on a GPU box:
    python tools/insert_duplicates.py > gpurun_out/insert_duplicates.jsonl
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))
import rpt_amd  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from strategy_crossover import time_insert  # noqa: E402


def main():
    lib = rpt_amd.load()
    n_max = 1 << 22
    rnd = rpt_amd.synth_build_keys(n_max)
    shapes = {
        "random": rnd,
        "constant_chunks": rnd[: n_max // 2048].repeat_interleave(2048),
        "one_key": rnd[:1].repeat(n_max),
        "1000_distinct": rnd[:1000][torch.randint(0, 1000, (n_max,), device=rnd.device)],
    }
    for L in (7, 10, 14, 24):
        bf = rpt_amd.BloomFilter(log_num_blocks=L)
        for n in (2048, 1 << 20, n_max):
            for name, keys in shapes.items():
                k = keys[:n].contiguous()
                row = {"op": "insert_duplicates", "log_blocks": L, "n": n, "keys": name}
                for sname, st in (("atomic", 1), ("partitioned", 2)):
                    if st == 2 and not lib.rpt_probe_strategy_supported(3, L):
                        continue
                    row[sname + "_ms"] = round(time_insert(bf, k, n, st), 4)
                print(json.dumps(row), flush=True)
        del bf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
