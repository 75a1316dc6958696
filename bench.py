#!/usr/bin/env python3
"""Headline benchmark: USE_BF Bloom-filter probe throughput on MI355X (BASELINE.json metric
"bloom probe keys/sec (whole node)", config C2).

One step = one probe pass of the hot path (PTBloomFilter::LookupSel, reference
src/bloom_filter.cpp:60-68, as PhysicalUseBF::ExecuteInternal drives it) over this rank's batch of
1e9 device-resident int64 keys against the filter CREATE_BF built from 1e7 keys: hash, gather,
ascending uint32 selection vector + survivor count. Multi-GPU (torch.distributed.run, one process
per GPU): the build rows are split by row range, partial filters are OR-merged over RCCL, and
every rank probes its own 1e9-row slice of the global probe column (weak scaling, no data-path
collective in the probe).

Prints ONE JSON line on rank 0. `roofline` prices the dominant kernel (probe phase 1) from HIP
events recorded on the launch stream; `cpu_baseline` times the C++ restatement (oracle/) on a
bounded sample on rank 0's host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))

HBM_PEAK_BPS = 8.0e12  # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
KEY_BYTES = 8           # int64 key read per probed row (algorithmic)
SEL_BYTES = 4           # uint32 sel entry written per survivor (algorithmic)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--probe-rows", type=float, default=1e9, help="probe rows per GPU")
    ap.add_argument("--build-rows", type=float, default=1e7, help="global build rows")
    ap.add_argument("--filter-rows", type=float, default=None,
                    help="size the filter for this many rows (default: --build-rows). C5 on one GPU = one "
                         "rank's share: --filter-rows 8e9 --build-rows 1e9")
    ap.add_argument("--p", type=float, default=0.10, help="fraction of probe rows drawn from the build keys")
    ap.add_argument("--cpu-sample", type=float, default=None,
                    help="probe rows in the CPU-baseline sample (default: the whole per-GPU probe workload)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("RPT_CPU_THREADS", "16")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--key-type", default="i64", choices=["i64", "i32"],
                    help="key column type (i32: the synthetic keys truncated to int32, as JOB's INTEGER keys)")
    ap.add_argument("--strategy", default="auto", choices=["auto", "gather", "lds", "partitioned", "bucketed"],
                    help="probe strategy (auto picks by filter size)")
    return ap.parse_args()


def algorithmic_bytes(kernel: str, n: int, survivors: int, key_bytes: int = KEY_BYTES) -> int:
    """SURVEY §8(d) per-unit bytes for the kernel's part of the probe: every kernel that streams the
    key column is charged 8 B/key (the key read; its own intermediates are implementation traffic,
    counted in `traffic`); the kernels that write the selection vector (the compaction, or the fused
    unpermute) are charged the 4 B/survivor they write."""
    if kernel.startswith(("compact", "unpermute_sel")):
        return SEL_BYTES * survivors
    if kernel.startswith(("slice_probe", "unpermute", "group_", "bucket_unpermute", "bucket_scan", "runs_transpose",
                          "tile_count")):
        return 0
    return key_bytes * n


def pmc_traffic(kernel: str, key_k: int = 0):
    """HBM bytes per launch of `kernel` from the PMC summary tools/pmc_summary.py wrote for this build
    (FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE, separate rocprofv3 --pmc passes)."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    # the kernel's instantiations (name or name<template args>); the probe's is the longest-running
    # (key-typed instantiations: the first template argument is the key type, 0 = int64, 1 = int32)
    cands = [v for name, v in d.get("kernels", {}).items()
             if (name == kernel or name.startswith(kernel + "<")) and "hbm_bytes_per_launch" in v
             and not (name.startswith(kernel + "<") and name[len(kernel) + 1:].split(",")[0] in ("0", "1")
                      and name[len(kernel) + 1:].split(",")[0] != str(key_k))]
    if not cands:
        return None
    k = max(cands, key=lambda v: v.get("avg_ms", 0.0))
    return {"bytes_per_launch": k["hbm_bytes_per_launch"], "source": f"profiles/pmc_latest.json ({d.get('round')})"}


def cpu_baseline(n_build: int, p_permille: int, sample: int, threads: int, key_type: str = "i64") -> dict:
    """The C++ restatement of the reference CPU path, morsel-parallel in 2048-row vectors. int32 keys run
    zero-extended to int64: DuckDB hashes an INTEGER through uint32 -> uint64, so hashes and survivors
    are the same (the port then reads 8 B per key instead of 4)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import rpt_oracle as orc

    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    lnb = orc.log_num_blocks(n_build)
    words = orc.new_words(lnb)
    as_i32 = (lambda k: k.astype(np.int32).view(np.uint32).astype(np.int64)) if key_type == "i32" else (lambda k: k)
    build_keys = as_i32(orc.synth_build_keys(n_build))
    build_s = orc.build_mt(words, lnb, build_keys, threads)
    del build_keys
    keys = as_i32(orc.synth_probe_keys(sample, n_build, p_permille))
    orc.probe_mt(words, lnb, keys, threads)  # warm-up
    runs = [orc.probe_mt(words, lnb, keys, threads) for _ in range(5)]
    med = statistics.median(r[0] for r in runs)
    return {
        "value": sample / med,
        "unit": "keys/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"probe of the first {sample:.0e} rows (the GPU's whole per-step workload when equal to its "
                   f"probe rows) of the same synthetic probe stream against the same "
                   f"{n_build:.0e}-key filter (2^{lnb} blocks), {threads} std::threads, 2048-row vectors, "
                   f"{'int32 keys zero-extended (same hashes), ' if key_type == 'i32' else ''}"
                   f"hash included; median of 5 after 1 warm-up; build of the filter {n_build / build_s:.3e} keys/s"),
        "cpu_model": _cpu_model(),
        "survivors": runs[0][1],
    }


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RPT_BENCH_BACKEND=gloo is a rehearsal mode for boxes with fewer GPUs than ranks: ranks share
    # devices and the OR-merge collectives run over gloo through host memory. Default: RCCL.
    backend = os.environ.get("RPT_BENCH_BACKEND", "nccl")
    dev_index = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    import rpt_amd
    from rpt_amd import _lib as rpt_lib
    from rpt_amd.distributed import allreduce_or_filter, shard_range

    n_probe = int(args.probe_rows)
    n_build = int(args.build_rows)
    n_filter = int(args.filter_rows) if args.filter_rows else n_build
    p_permille = int(round(args.p * 1000))
    cfg = {(10**7, 10**7): "C2", (10**8, 10**8): "C3", (10**9, 8 * 10**9): "C5 (one rank's share)",
           (8 * 10**9, 8 * 10**9): "C5"}.get((n_build, n_filter), "custom")

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev_index]) if backend == "nccl" else dist.barrier()

    # ---- CREATE_BF: sharded build + OR merge (reported, not the headline) -------------------------
    lo, hi = shard_range(n_build, rank, world)
    build_keys = rpt_amd.synth_build_keys(hi - lo, start=lo, device=device)
    if args.key_type == "i32":
        build_keys = build_keys.to(torch.int32)
    bf = rpt_amd.BloomFilter(n_filter, device=device)
    bf.insert(build_keys)  # warm-up: workspace allocation, code-object load
    build_reps = 5
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(build_reps):  # clear + insert: the filter ends up holding exactly this rank's keys
        bf.clear()
        bf.insert(build_keys)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    allreduce_or_filter(bf) if world > 1 else None
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    bf.finalized = True
    merge_check = None
    if world > 1:
        # untimed: the OR-merged filter must be bit-identical to a single-GPU build of all rows
        ref = rpt_amd.BloomFilter(n_filter, device=device)
        all_keys = rpt_amd.synth_build_keys(n_build, device=device)
        ref.insert(all_keys.to(torch.int32) if args.key_type == "i32" else all_keys)
        a = torch.empty(bf.num_blocks, dtype=torch.int64, device=device)
        b = torch.empty_like(a)
        bf.copy_words_to(a)
        ref.copy_words_to(b)
        ok = torch.tensor([1 if torch.equal(a, b) else 0], dtype=torch.int64,
                          device=device if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        merge_check = "bit-identical to a single-GPU build on every rank" if ok.item() else "MISMATCH"
        del ref, a, b
        if not ok.item():
            raise SystemExit("OR-merged filter differs from the single-GPU build")
    bf.probe_strategy = {"auto": 0, "gather": 1, "lds": 2, "partitioned": 3, "bucketed": 4}[args.strategy]
    strategy_name = {1: "gather", 2: "lds", 3: "partitioned", 4: "bucketed"}[bf.probe_strategy_for(n_probe)]
    del build_keys

    # ---- USE_BF probe workload: this rank's slice of the global probe column --------------------
    keys = rpt_amd.synth_probe_keys(n_probe, n_build, p_permille, start=rank * n_probe, device=device)
    key_bytes = KEY_BYTES
    if args.key_type == "i32":
        keys = keys.to(torch.int32)
        key_bytes = 4
        torch.cuda.empty_cache()
    out_sel = torch.empty(n_probe, dtype=torch.int32, device=device)
    out_count = torch.zeros(1, dtype=torch.int64, device=device)
    ws = torch.empty(bf.workspace_bytes(n_probe), dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream(device)

    def step(ev=None):
        # one LookupSel over the whole per-GPU column (rpt_bf_probe: hash, probe, ascending sel)
        if ev is not None:
            ev[0].record(stream)
        bf.probe_async(keys, n=n_probe, out_sel=out_sel, out_count=out_count, workspace=ws)
        if ev is not None:
            ev[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    # per-kernel HIP events on the launch stream (rpt_profiling_*) over the timed region
    rpt_lib.profiling_reset()
    rpt_lib.profiling(True)
    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - ts
    rpt_lib.profiling(False)
    ktimes = rpt_lib.kernel_times()

    survivors = int(out_count.item())
    probe_ms = statistics.mean(e[0].elapsed_time(e[1]) for e in events)

    t = torch.tensor([elapsed, (t1 - t0) / build_reps, t2 - t1], dtype=torch.float64,
                     device=device if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, insert_s, merge_s = t.tolist()

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = world * n_probe * args.steps / elapsed
        probe_bytes = key_bytes * n_probe + SEL_BYTES * survivors
        # dominant kernel of the step (largest total device time)
        dom_name, (dom_calls, dom_total) = max(ktimes.items(), key=lambda kv: kv[1][1])
        dom_ms = dom_total / dom_calls
        dom_bytes = algorithmic_bytes(dom_name, n_probe, survivors, key_bytes)
        achieved = dom_bytes / (dom_ms * 1e-3)
        key_k = 1 if args.key_type == "i32" else 0
        traffic = pmc_traffic(dom_name, key_k)
        # whole-step HBM traffic: every kernel of the step at its PMC bytes per launch
        step_traffic, unprofiled = 0.0, []
        for name, (calls, _total) in ktimes.items():
            t = pmc_traffic(name, key_k)
            if t is None:
                unprofiled.append(name)
            else:
                step_traffic += t["bytes_per_launch"] * calls / args.steps
        line = {
            "metric": "bloom probe keys/sec (whole node)",
            "value": value,
            "unit": "keys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32" if args.key_type == "i32" else "int64",
            "data": "synthetic: seeded splitmix64 int64 key columns generated on device (SURVEY §8d)",
            "config": {
                "workload": (f"{cfg}: USE_BF probe of {n_probe:.0e} {'int32' if args.key_type == 'i32' else 'int64'} keys per GPU against a blocked Bloom "
                             f"filter built from {n_build:.0e} keys (sized for {n_filter:.0e}: "
                             f"2^{bf.log_num_blocks} blocks = {bf.num_blocks * 8 / 2**20:.0f} MiB), p={args.p}"),
                "probe_rows_per_gpu": n_probe,
                "build_rows": n_build,
                "filter_bytes": bf.num_blocks * 8,
                "pass_fraction": survivors / n_probe,
                "parallelism": f"row-range shards over {world} GPU(s), filter replicated "
                               f"({'RCCL' if backend == 'nccl' else backend + ' rehearsal'} OR-merge)",
                "probe_strategy": strategy_name,
                "job_geomean": "not measured: needs DuckDB v1.4.4 + job.duckdb (SURVEY §8f row 1)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom_name,
                "achieved": achieved / 1e9,
                "peak": HBM_PEAK_BPS / 1e9,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_BPS,
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "traffic_source": traffic["source"] if traffic else None,
                "avg_launch_ms": dom_ms,
                "algorithmic_bytes_per_launch": dom_bytes,
            },
            "kernels_ms": {k: v[1] / v[0] for k, v in sorted(ktimes.items(), key=lambda kv: -kv[1][1])},
            "probe_total": {
                "avg_ms": probe_ms,
                "algorithmic_bytes": probe_bytes,
                "achieved_GBps": probe_bytes / (probe_ms * 1e-3) / 1e9,
                "frac": probe_bytes / (probe_ms * 1e-3) / HBM_PEAK_BPS,
                # HBM bytes the whole step moves (PMC, every kernel) and their rate over the step
                "traffic": step_traffic if not unprofiled else None,
                "traffic_GBps": step_traffic / (probe_ms * 1e-3) / 1e9 if not unprofiled else None,
                "traffic_unprofiled_kernels": unprofiled,
            },
            "build": {
                "rows": n_build,
                "insert_ms": insert_s * 1e3,
                "insert_keys_per_s": (n_build / world) / insert_s if insert_s > 0 else None,
                "or_merge_ms": merge_s * 1e3,
                "merge_check": merge_check,
            },
        }
        if not args.no_cpu_baseline and world == 1:
            sample = int(args.cpu_sample) if args.cpu_sample else n_probe
            cb = cpu_baseline(n_build, p_permille, sample, args.cpu_threads, args.key_type)
            if sample == n_probe:  # same rows, same filter: a full-size cross-check of the survivor count
                cb["survivors_match_gpu"] = cb["survivors"] == survivors
            line["cpu_baseline"] = cb
        print(json.dumps(line), flush=True)

    if world > 1:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
