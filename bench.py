#!/usr/bin/env python3
"""Headline benchmark: USE_BF Bloom-filter probe throughput on MI355X (BASELINE.json metric
"bloom probe keys/sec (whole node)"; default config C2).

One step = one probe pass of the hot path (PTBloomFilter::LookupSel, reference
src/bloom_filter.cpp:60-68, as PhysicalUseBF::ExecuteInternal drives it) over this rank's batch of
1e9 device-resident int64 keys against the filter CREATE_BF built: hash, filter test, ascending
uint32 selection vector + survivor count.

Configs (--config; BASELINE.json configs[1], [2], [4]):
  C2  1e7-key build (16 MiB filter), 1e9-key probe per GPU                     (default)
  C3  1e8-key build (128 MiB filter), 1e9-key probe per GPU
  C5  filter sized for 8e9 rows (8 GiB); every rank inserts its 1e9-row shard of the build column
      (8e9 rows at 8 GPUs, weak-scaled below), partial filters OR-merged over RCCL, 1e9-key probe per GPU

Multi-GPU: one process per GPU. `--gpus N` without a launcher starts N ranks itself
(torch.distributed.run, 127.0.0.1) before any GPU call; under a launcher WORLD_SIZE must equal N.
The build rows are split by row range, each rank's partial filter (sized for the GLOBAL row count)
is OR-merged through the C-ABI's rpt_bf_allreduce_or over an RCCL communicator the library creates
(the product path a C++ caller gets), checked bit-identical to a single-GPU build of all rows, and
every rank probes its own 1e9-row slice of the global probe column (weak scaling, no data-path
collective in the probe). A communicator that cannot be built ends the run with a non-zero exit on
every rank. RPT_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices; every merge,
the C5 section's included, then runs the torch.distributed composition over host memory, reported as
torch_merge_ms, never as or_merge_ms).

At N > 1 (and with --c5-merge at N = 1) the line also carries `c5_merge`: the north_star's C5 pipeline at
this node's N, after the headline is timed: every rank inserts its 1e9-row shard into an 8 GiB filter sized
for 8e9 rows, rpt_bf_allreduce_or_ws OR-merges the partials over RCCL (xGMI), the merged filter is checked
bit-identical to a single build of all N * 1e9 rows, and every rank probes its 1e9-row slice against it. The
record carries each rank's peak device memory over the section (hipMemGetInfo) and the section's wall time.

Prints ONE JSON line on rank 0. `roofline` prices the dominant kernel from HIP events the library
records on the launch stream (rpt_profiling_*) and its PMC traffic from profiles/pmc/<config>.json
(the exact template instantiation, or null); `cpu_baseline` times the C++ restatement (oracle/) on
rank 0's host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "duckdb-robust-predicate-transfer_amd"))

HBM_PEAK_BPS = 8.0e12  # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
KEY_BYTES = 8           # int64 key read per probed row (algorithmic)
SEL_BYTES = 4           # uint32 sel entry written per survivor (algorithmic)

C5_FILTER_ROWS = 8 * 10**9  # BASELINE config 4: the filter of 8e9 rows (2^30 blocks = 8 GiB)
C5_ROWS_PER_RANK = 10**9

CONFIGS = {  # name -> (global build rows at N GPUs, filter sized for)
    "C2": (lambda n: 10**7, lambda n: 10**7),
    "C3": (lambda n: 10**8, lambda n: 10**8),
    "C5": (lambda n: n * 10**9, lambda n: 8 * 10**9),
    # supplementary (not a BASELINE config): a JOB-sized dimension filter, 1e5 keys -> 128 KiB, the whole filter
    # in LDS
    "JOBDIM": (lambda n: 10**5, lambda n: 10**5),
    # supplementary: a 2e5-key dimension filter (256 KiB: JOB's keyword / company_name tables), the hybrid LDS probe
    "JOBDIM256": (lambda n: 2 * 10**5, lambda n: 2 * 10**5),
    "JOBDIM512": (lambda n: 4 * 10**5, lambda n: 4 * 10**5),  # 512 KiB, the hybrid probe's upper size
}
STREAM_CAL_BYTES = 8 << 30  # stream calibration buffer (>= 8 GB: well past the 256 MiB Infinity Cache)


def cpu_share() -> int:
    """Host threads this process may use: the affinity mask, capped by the cgroup CPU quota (the GPU
    box grants each job a share of a larger machine: `nproc` shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="BASELINE config (sets --build-rows / --filter-rows); default C2")
    ap.add_argument("--probe-rows", type=float, default=1e9, help="probe rows per GPU")
    ap.add_argument("--build-rows", type=float, default=None, help="global build rows (default: the config's)")
    ap.add_argument("--filter-rows", type=float, default=None,
                    help="size the filter for this many rows (default: the config's, else --build-rows)")
    ap.add_argument("--p", type=float, default=0.10, help="fraction of probe rows drawn from the build keys")
    ap.add_argument("--cpu-sample", type=float, default=None,
                    help="probe rows in the CPU-baseline sample (default: the whole per-GPU probe workload)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("RPT_CPU_THREADS", "0")) or None,
                    help="CPU-baseline threads (default: this process's CPU share, see cpu_share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-lag", type=int, default=0,
                    help="CPU baseline: rows between a row's hash + prefetch and its filter test (0: the default, 24; "
                         "2048: the whole vector hashed first, the pre-r05 loop)")
    ap.add_argument("--cpu-lag-sweep", default=None,
                    help="with --cpu-baseline-only: comma-separated prefetch lags timed interleaved (A B C A B C ...) "
                         "in one process against one filter and sample, with the cgroup's CPU throttling and the "
                         "host's load average around each measurement (VERDICT r05 item 6)")
    ap.add_argument("--cpu-sweep-rounds", type=int, default=3)
    ap.add_argument("--cpu-pin-sweep", default="0",
                    help="with --cpu-lag-sweep: comma-separated thread placements (0 the OS's, 1 compact: thread t on "
                         "the t-th CPU of the affinity mask, 2 spread over the mask), crossed with the lags")
    ap.add_argument("--cpu-baseline-only", action="store_true",
                    help="print only the cpu_baseline object for this config (no GPU; e.g. to put the CPU "
                         "restatement at T threads beside the host-resident GPU path of tools/host_bench)")
    ap.add_argument("--cpu-chain", type=int, default=0,
                    help="with --cpu-baseline-only: USE_BF's loop over this many filters instead (column 0 BIGINT "
                         "10%% hits, column 1 INTEGER 50%%, column 2 BIGINT 50%%, ...: the shape of tools/host_bench "
                         "--chain)")
    ap.add_argument("--merge", default="native", choices=["native", "torch"],
                    help="N > 1: the product merge rpt_bf_allreduce_or_ws over RCCL (default; a failing "
                         "communicator exits non-zero), or the torch.distributed composition (reported as "
                         "torch_merge_ms, not or_merge_ms)")
    ap.add_argument("--no-merge-check", action="store_true",
                    help="skip the (untimed) bit-identity check of the OR-merged filter (N > 1)")
    ap.add_argument("--key-type", default="i64", choices=["i64", "i32"],
                    help="key column type (i32: the synthetic keys truncated to int32, as JOB's INTEGER keys)")
    ap.add_argument("--strategy", default="auto", choices=["auto", "gather", "lds", "partitioned", "bucketed"],
                    help="probe strategy (auto picks by filter and batch size)")
    ap.add_argument("--c5-merge", action="store_true",
                    help="run the C5 build + RCCL merge + probe section at N = 1 too (a one-rank communicator; "
                         "at N > 1 it runs by default)")
    ap.add_argument("--no-c5-merge", action="store_true", help="N > 1: skip the C5 build + merge + probe section")
    ap.add_argument("--c5-rows-per-rank", type=float, default=C5_ROWS_PER_RANK,
                    help="C5 section: build and probe rows per rank (the filter stays sized for 8e9 rows)")
    ap.add_argument("--c5-merge-reps", type=int, default=3, help="C5 section: timed merges (after one warm-up)")
    ap.add_argument("--collective-timeout-ms", type=int, default=None,
                    help="bound of every OR all-reduce's waits (rpt_collective_set_timeout_ms; default the library's)")
    ap.add_argument("--no-stream-calibration", action="store_true",
                    help="skip the (untimed) read / copy stream calibration the roofline fractions are set beside")
    ap.add_argument("--kernel-events-in-timed-region", action="store_true",
                    help="record the per-kernel HIP events inside the timed steps (r01-r05 arrangement; they cost "
                         "~25 us per step) instead of in an identical second pass of K steps after them")
    return ap.parse_args()


def stream_calibration(device, nbytes: int = STREAM_CAL_BYTES, reps: int = 5) -> dict:
    """What this box's HBM streams, measured in this process before the timed steps (so the kernels' fractions
    of the 8 TB/s spec can be read against the box they ran on): a plain 16-B-load read stream over `nbytes`
    (rpt_stream_read) and a read + write copy of nbytes / 2 into the other half (rpt_stream_copy), each the
    best of `reps` after one warm-up, timed with HIP events on the launch stream."""
    import torch

    import rpt_amd
    from rpt_amd._lib import check

    lib = rpt_amd.load()
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    buf.fill_(0x5A)
    sink = torch.empty(int(lib.rpt_stream_sink_words(device.index or 0)), dtype=torch.int64, device=device)
    stream = torch.cuda.current_stream(device)
    sh = stream.cuda_stream
    half = nbytes // 2

    def timed(fn):
        fn()
        best = float("inf")
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            b.synchronize()
            best = min(best, a.elapsed_time(b) * 1e-3)
        return best

    t_read = timed(lambda: check(lib.rpt_stream_read(buf.data_ptr(), nbytes, sink.data_ptr(), sh)))
    t_copy = timed(lambda: check(lib.rpt_stream_copy(buf.data_ptr() + half, buf.data_ptr(), half, sh)))
    del buf, sink
    torch.cuda.empty_cache()
    return {
        "read_GBps": nbytes / t_read / 1e9,
        "copy_GBps": 2 * half / t_copy / 1e9,  # bytes read + bytes written
        "bytes": nbytes,
        "how": ("rpt_stream_read: 16-B non-temporal loads over 8 GiB, 8 in flight per lane, 16 x 256-thread "
                "workgroups per CU; rpt_stream_copy: 4 GiB -> 4 GiB, one 16-B unit per lane, read + write bytes; "
                "best of 5 after a warm-up, HIP events (the fastest variants of tools/ubench/ubench_stream.hip)"),
    }


def config_tag(cfg: str, key_type: str) -> str:
    return cfg + ("-i32" if key_type == "i32" else "")


def algorithmic_bytes(kernel: str, n: int, survivors: int, key_bytes: int = KEY_BYTES) -> int:
    """SURVEY §8(d) per-unit bytes for the kernel's part of the probe: kernels that stream the key
    column are charged 8 B/key (4 B for int32; their own intermediates are implementation traffic,
    counted in `traffic`); the kernels that write the selection vector (the compaction, or the fused
    unpermute) are charged the 4 B/survivor they write; everything else (routing intermediates, scans,
    the bucketed level-2 pass over the split-hash array) is charged 0."""
    if kernel.startswith(("compact", "unpermute_sel")):
        return SEL_BYTES * survivors
    if kernel.startswith(("probe_bits", "probe_small", "bucket_count", "bucket_scatter")):
        return key_bytes * n
    if kernel.startswith("partition_kernel<") and kernel[len("partition_kernel<"):].split(",")[0] in ("0", "1", "2"):
        return key_bytes * n
    return 0


def c5_merge_record(world: int, filter_bytes: int, rows_per_rank: int, insert_ms: float, merge_ms: list,
                    probe_ms: float, survivors: int, merge_check: str, timeout_ms, native: bool = True,
                    merge_path: str = "", mem: dict = None, wall_s: float = None) -> dict:
    """The `c5_merge` object of the bench line (times are the max over ranks). The merge moves 2 (W-1)/W of
    the filter per GPU, 2 S / W over each of its W-1 point-to-point xGMI links. Only the product
    merge (rpt_bf_allreduce_or_ws over RCCL, native=True) reports or_merge_*; the torch.distributed
    composition (the gloo rehearsal, --merge torch) reports torch_merge_ms instead."""
    t = statistics.median(merge_ms) if merge_ms else None
    rec = {
        "what": ("BASELINE config 4 (C5) at this node's N: every rank inserts its shard of the N x rows_per_rank "
                 "build column into a filter sized for 8e9 rows, the partials are OR-merged, every rank probes "
                 "its rows_per_rank-row slice against the merged filter"),
        "n_gpus": world,
        "filter_bytes": filter_bytes,
        "rows_per_rank": rows_per_rank,
        "build_rows": world * rows_per_rank,
        "insert_ms": insert_ms,
        "merge_path": merge_path,
        "or_merge_ms": t * 1e3 if t and native else None,
        "or_merge_ms_reps": [m * 1e3 for m in merge_ms] if native else None,
        "or_merge_GBps_per_gpu": 2 * (world - 1) / world * filter_bytes / t / 1e9 if t and world > 1 and native else None,
        "or_merge_GBps_per_link": 2 / world * filter_bytes / t / 1e9 if t and world > 1 and native else None,
        "torch_merge_ms": t * 1e3 if t and not native else None,
        "torch_merge_ms_reps": [m * 1e3 for m in merge_ms] if not native else None,
        "probe_ms": probe_ms,
        "probe_keys_per_s_node": world * rows_per_rank / (probe_ms * 1e-3) if probe_ms else None,
        "survivors_rank0": survivors,
        "merge_check": merge_check,
        "collective_timeout_ms": timeout_ms,
    }
    if mem is not None:
        rec["device_memory"] = mem
    if wall_s is not None:
        rec["wall_s"] = wall_s
    return rec


class DeviceMemTracker:
    """Peak device memory in use (hipMemGetInfo through torch.cuda.mem_get_info: total - free, so it counts the
    library's own hipMalloc'd filters as well as torch's cached blocks) sampled at the phase boundaries of the
    C5 section. On a device shared by several ranks (the gloo rehearsal) the figure is the device's, not the
    rank's."""

    def __init__(self, device, progress: bool = False):
        import torch

        self._torch = torch
        self.progress = progress  # rank 0: one stderr line per phase (a long rehearsal shows it is alive)
        self.t0 = time.perf_counter()
        self.device = device
        free, self.total = torch.cuda.mem_get_info(device)
        self.base = self.total - free
        self.peak = self.base
        self.phases = {}
        # this process's own share, which stays meaningful when ranks share a device: torch's caching allocator
        # (reserved) plus the filters the library allocated itself (note_filters), sampled at the same points
        torch.cuda.reset_peak_memory_stats(device)
        self.filters = 0
        self.own_peak = 0
        self.own_phases = {}

    def note_filters(self, nbytes: int) -> None:
        """Bytes of library-allocated filters (hipMalloc in rpt_bf_create) this rank holds from now on."""
        self.filters = nbytes

    def sample(self, phase: str) -> None:
        self._torch.cuda.synchronize(self.device)
        free, _ = self._torch.cuda.mem_get_info(self.device)
        used = self.total - free
        self.phases[phase] = used
        self.peak = max(self.peak, used)
        own = self._torch.cuda.max_memory_reserved(self.device) + self.filters
        self._torch.cuda.reset_peak_memory_stats(self.device)
        self.own_phases[phase] = own
        self.own_peak = max(self.own_peak, own)
        if self.progress:
            print(f"[bench c5] {phase} done at {time.perf_counter() - self.t0:.1f} s, device memory in use "
                  f"{used / 2**30:.1f} GiB", file=sys.stderr, flush=True)


def run_c5_merge(args, rank: int, world: int, device, comm, barrier, reduce_max, all_ok, gather_ints,
                 merge_path: str, shared_device_ranks: int = 1) -> dict:
    """C5 build + merge + probe (see the module docstring). Collective: every rank runs it. `comm` is the
    RcclComm of the product merge (rpt_bf_allreduce_or_ws), or None for the torch.distributed composition
    (the gloo rehearsal / --merge torch; reported as torch_merge_ms)."""
    import torch

    import rpt_amd
    from rpt_amd.distributed import allreduce_or_filter, allreduce_or_native, allreduce_workspace

    t_section = time.perf_counter()
    mem = DeviceMemTracker(device, progress=rank == 0)
    native = comm is not None
    rows = int(args.c5_rows_per_rank)
    bf = rpt_amd.BloomFilter(C5_FILTER_ROWS, device=device)
    mem.note_filters(bf.num_blocks * 8)
    keys = rpt_amd.synth_build_keys(rows, start=rank * rows, device=device)
    bf.insert(keys)  # warm-up (workspace, code objects)
    torch.cuda.synchronize()
    bf.clear()
    barrier()
    t0 = time.perf_counter()
    bf.insert(keys)
    torch.cuda.synchronize()
    insert_s = time.perf_counter() - t0
    mem.sample("insert")
    if native:
        ws = allreduce_workspace(bf, comm)

        def merge():
            allreduce_or_native(bf, comm, workspace=ws)
    else:
        ws = None
        # the host-staged gloo composition of an 8 GiB filter takes many seconds per merge: rank 0 reports its
        # rounds, so a long rehearsal keeps showing progress
        t_m = [time.perf_counter()]

        def progress(done, total):
            if rank == 0 and (done == total or time.perf_counter() - t_m[0] > 10):
                t_m[0] = time.perf_counter()
                print(f"[bench c5] torch merge: {done}/{total} rounds at {t_m[0] - mem.t0:.1f} s", file=sys.stderr,
                      flush=True)

        def merge():
            allreduce_or_filter(bf, progress=progress)
    merge()  # warm-up merge: OR is idempotent, the words do not change
    mem.sample("merge")
    merge_s = []
    for _ in range(args.c5_merge_reps):
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        merge()
        torch.cuda.synchronize()
        merge_s.append(time.perf_counter() - t0)
    del ws
    mem.sample("merge_timed")
    torch.cuda.empty_cache()  # the merge's staging (RCCL rounds, or the torch composition's word copy)
    # untimed: the merged filter against a single build of all world * rows rows (inserted piece by piece),
    # compared on the device (rpt_bf_is_same_as: no word copies, so a rank holds its filter + the reference)
    ref = rpt_amd.BloomFilter(C5_FILTER_ROWS, device=device)
    mem.note_filters(2 * bf.num_blocks * 8)
    for r in range(world):
        rpt_amd.synth_build_keys(rows, start=r * rows, device=device, out=keys)
        ref.insert(keys)
    del keys
    same = bf.is_same_as(ref) and bf.minmax() == ref.minmax() and not bf.is_empty()
    mem.sample("merge_check")
    del ref
    mem.note_filters(bf.num_blocks * 8)
    torch.cuda.empty_cache()
    ok = all_ok(same)
    check = ("bit-identical (words + key min/max) to a single-GPU build of all rows on every rank" if ok
             else "MISMATCH")
    # the node-wide probe: every rank its slice of the global probe column against the merged filter
    n_probe = rows
    pkeys = rpt_amd.synth_probe_keys(n_probe, world * rows, int(round(args.p * 1000)), start=rank * n_probe,
                                     device=device)
    out_sel = torch.empty(n_probe, dtype=torch.int32, device=device)
    out_count = torch.zeros(1, dtype=torch.int64, device=device)
    pws = torch.empty(bf.workspace_bytes(n_probe), dtype=torch.uint8, device=device)
    bf.probe_async(pkeys, n=n_probe, out_sel=out_sel, out_count=out_count, workspace=pws)  # warm-up
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        bf.probe_async(pkeys, n=n_probe, out_sel=out_sel, out_count=out_count, workspace=pws)
    torch.cuda.synchronize()
    probe_s = (time.perf_counter() - t0) / reps
    mem.sample("probe")
    survivors = int(out_count.item())
    nbytes = bf.num_blocks * 8
    del pkeys, out_sel, pws, bf
    torch.cuda.empty_cache()
    insert_s, probe_s, *merge_s = reduce_max([insert_s, probe_s] + merge_s)
    peaks = gather_ints([mem.peak - mem.base, mem.peak, mem.own_peak])
    wall_s = reduce_max([time.perf_counter() - t_section])[0]
    mem_rec = {
        "source": "hipMemGetInfo (torch.cuda.mem_get_info): total - free, sampled after each phase",
        "device_total_bytes": mem.total,
        "rank0_phase_used_bytes": mem.phases,
        "section_peak_bytes_per_rank": [p[0] for p in peaks],
        "device_peak_used_bytes_per_rank": [p[1] for p in peaks],
        # each rank's own footprint (torch's reserved peak + the library's filters), per phase on rank 0: what one
        # rank of the driver's N-GPU run holds, whether or not ranks share a device here
        "rank_own_peak_bytes_per_rank": [p[2] for p in peaks],
        "rank0_own_phase_bytes": mem.own_phases,
        "ranks_per_device": shared_device_ranks,
    }
    rec = c5_merge_record(world, nbytes, rows, insert_s * 1e3, merge_s, probe_s * 1e3, survivors, check,
                          (args.collective_timeout_ms or rpt_amd.load().rpt_collective_timeout_ms()) if native else None,
                          native=native, merge_path=merge_path, mem=mem_rec, wall_s=wall_s)
    if not ok:
        raise SystemExit("C5: OR-merged filter differs from the single-GPU build")
    return rec


def pmc_traffic(kernel: str, tag: str):
    """HBM bytes per launch of exactly this kernel instantiation in this config, from the PMC summary
    tools/profile_round.sh wrote (profiles/pmc/<tag>.json: FETCH_SIZE doubled per the gfx950 correction +
    WRITE_SIZE, separate rocprofv3 --pmc passes of the same bench command). None if not profiled."""
    path = os.path.join(REPO, "profiles", "pmc", f"{tag}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    k = d.get("kernels", {}).get(kernel)
    if not k or "hbm_bytes_per_launch" not in k:
        return None
    return {"bytes_per_launch": k["hbm_bytes_per_launch"], "source": f"profiles/pmc/{tag}.json ({d.get('round')})"}


def cpu_baseline(n_build: int, n_filter: int, p_permille: int, sample: int, threads: int, threads_src: str,
                 key_type: str = "i64", lag: int = 0) -> dict:
    """The C++ restatement of the reference CPU path, morsel-parallel in 2048-row vectors, against the
    SAME filter geometry the GPU probes (sized for n_filter rows, n_build keys inserted). int32 keys run
    zero-extended to int64: DuckDB hashes an INTEGER through uint32 -> uint64, so hashes and survivors
    are the same (the port then reads 8 B per key instead of 4)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import rpt_oracle as orc

    lnb = orc.log_num_blocks(n_filter)
    words = orc.new_words(lnb)
    as_i32 = (lambda k: k.astype(np.int32).view(np.uint32).astype(np.int64)) if key_type == "i32" else (lambda k: k)
    build_keys = as_i32(orc.synth_build_keys(n_build))
    build_s = orc.build_mt(words, lnb, build_keys, threads)
    del build_keys
    keys = as_i32(orc.synth_probe_keys(sample, n_build, p_permille))
    # the loop's prefetch distance: which of 24 rows and the whole vector (2048) is faster depends on the box's
    # thread placement and neighbours, not on the filter (CPU baseline), so both run and the faster is
    # the baseline (--cpu-lag pins one)
    by_lag = {}
    for lg in ([lag] if lag else [24, 2048]):
        orc.set_probe_lag(lg)
        orc.probe_mt(words, lnb, keys, threads)  # warm-up
        runs = [orc.probe_mt(words, lnb, keys, threads) for _ in range(5)]
        by_lag[lg] = (statistics.median(r[0] for r in runs), runs)
    best = min(by_lag, key=lambda g: by_lag[g][0])
    med, runs = by_lag[best]
    orc.set_probe_lag(best)
    return {
        "value": sample / med,
        "unit": "keys/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"probe of the first {sample:.0e} rows (the GPU's whole per-step workload when equal to its "
                   f"probe rows) of the same synthetic probe stream against the same filter "
                   f"({n_build:.0e} keys inserted, sized for {n_filter:.0e} rows: 2^{lnb} blocks), {threads} "
                   f"std::threads ({threads_src}), 2048-row vectors, "
                   f"{'int32 keys zero-extended (same hashes), ' if key_type == 'i32' else ''}"
                   f"hash included; median of 5 after 1 warm-up, the faster of the prefetch distances "
                   f"{sorted(by_lag)}; build of the filter {n_build / build_s:.3e} keys/s"),
        "cpu_model": _cpu_model(),
        "survivors": runs[0][1],
        "prefetch_lag_rows": int(orc.lib().rpt_oracle_probe_lag()),
        "keys_per_s_by_lag": {str(g): sample / v[0] for g, v in by_lag.items()},
    }


def _cgroup_cpu_stat() -> dict:
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if line.strip())}
    except (OSError, ValueError):
        return {}


def cpu_lag_sweep(n_build: int, n_filter: int, p_permille: int, sample: int, threads: int, lags: list,
                  rounds: int, pins: list = (0,)) -> dict:
    """The CPU baseline's probe loop at several prefetch lags, interleaved round by round in one process (same filter,
    same sample), so a neighbour's load on the shared host or the cgroup's CPU quota shows up in every lag alike
    instead of as a difference between them; each measurement is the median of 5 runs after a warm-up."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import rpt_oracle as orc

    lnb = orc.log_num_blocks(n_filter)
    words = orc.new_words(lnb)
    orc.build_mt(words, lnb, orc.synth_build_keys(n_build), threads)
    keys = orc.synth_probe_keys(sample, n_build, p_permille)
    out = []
    for r in range(rounds):
        for pin, lag in ((p, g) for p in pins for g in lags):
            orc.set_pin_mode(pin)
            orc.set_probe_lag(lag)
            orc.probe_mt(words, lnb, keys, threads)  # warm-up
            st0, la0, t0 = _cgroup_cpu_stat(), os.getloadavg(), time.perf_counter()
            runs = [orc.probe_mt(words, lnb, keys, threads) for _ in range(5)]
            st1, wall = _cgroup_cpu_stat(), time.perf_counter() - t0
            d = {k: st1[k] - st0.get(k, 0) for k in st1}
            out.append({"round": r, "lag": lag, "pin": pin, "keys_per_s": sample / statistics.median(x[0] for x in runs),
                        "runs_s": [x[0] for x in runs], "wall_s": wall, "loadavg_1m_before": la0[0],
                        "cpu_usage_s": d.get("usage_usec", 0) / 1e6,
                        "throttled_s": d.get("throttled_usec", 0) / 1e6, "nr_throttled": d.get("nr_throttled", 0),
                        "survivors": runs[0][1]})
    orc.set_probe_lag(0)
    orc.set_pin_mode(0)
    return {"threads": threads, "sample": sample, "filter_log_blocks": lnb, "cpu_model": _cpu_model(),
            "host_cpus": os.cpu_count(), "cpu_share": cpu_share(), "measurements": out}


def cpu_chain_baseline(k: int, n_build: int, n_filter: int, sample: int, threads: int) -> dict:
    """USE_BF's filter loop (physical_use_bf.cpp:137-183) as the C++ restatement runs it: k filters, each sized for
    n_filter rows with n_build keys (separate copies, so each has its own cache footprint), probe column f hitting
    with 10 % (f = 0) or 50 % (f > 0), INTEGER for odd f (zero-extended: same hashes); per 2048-row vector, filter f
    over the survivors of filters 0..f-1."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import rpt_oracle as orc

    lnb = orc.log_num_blocks(n_filter)
    as_i32 = lambda x: x.astype(np.int32).view(np.uint32).astype(np.int64)  # noqa: E731
    bases = []
    for i32 in (False, True):  # the INTEGER columns' filter holds the build keys as INTEGERs
        w = orc.new_words(lnb)
        bk = orc.synth_build_keys(n_build)
        orc.build_mt(w, lnb, as_i32(bk) if i32 else bk, threads)
        bases.append(w)
    words = [bases[f % 2].copy() for f in range(k)]
    keys = []
    for f in range(k):
        kf = orc.synth_probe_keys(sample, n_build, 100 if f == 0 else 500, start=f << 40)
        keys.append(as_i32(kf) if f % 2 else kf)
    orc.probe_chain_mt(words, [lnb] * k, keys, threads)  # warm-up
    runs = [orc.probe_chain_mt(words, [lnb] * k, keys, threads) for _ in range(5)]
    med = statistics.median(r[0] for r in runs)
    return {"value": sample / med, "unit": "rows/s", "cores": threads, "kind": "port", "filters": k,
            "pass_fraction": runs[0][1] / sample,
            "sample": (f"{sample:.0e} rows, {k} filters of 2^{lnb} blocks ({n_build:.0e} keys each), {threads} "
                       "std::threads, 2048-row vectors, filter f over filter f-1's survivors, hash included; "
                       "median of 5 after 1 warm-up"),
            "cpu_model": _cpu_model()}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start n ranks of this script under torch.distributed.run (before this process touches a GPU) and
    return their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.cpu_baseline_only:
        cfg = args.config or "C2"
        n_build = int(args.build_rows) if args.build_rows else CONFIGS[cfg][0](1)
        n_filter = int(args.filter_rows) if args.filter_rows else (CONFIGS[cfg][1](1) if not args.build_rows else n_build)
        sample = int(args.cpu_sample) if args.cpu_sample else int(args.probe_rows)
        threads = args.cpu_threads or cpu_share()
        if args.cpu_lag_sweep:
            lags = [int(x) for x in args.cpu_lag_sweep.split(",")]
            sw = cpu_lag_sweep(n_build, n_filter, int(round(args.p * 1000)), sample, threads, lags,
                               args.cpu_sweep_rounds, [int(x) for x in args.cpu_pin_sweep.split(",")])
            print(json.dumps({"cpu_lag_sweep": sw, "config": cfg}), flush=True)
            return
        if args.cpu_chain:
            cb = cpu_chain_baseline(args.cpu_chain, n_build, n_filter, sample, threads)
            print(json.dumps({"cpu_baseline": cb, "config": cfg}), flush=True)
            return
        cb = cpu_baseline(n_build, n_filter, int(round(args.p * 1000)), sample, threads,
                          "--cpu-threads" if args.cpu_threads else "this process's CPU share", args.key_type,
                          args.cpu_lag)
        print(json.dumps({"cpu_baseline": cb, "config": cfg, "key_type": args.key_type}), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
        world = 1
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with --nproc-per-node {args.gpus}")

    # stdout carries exactly ONE line, the JSON record: native libraries print banners there (RCCL prints its
    # version block at communicator init), so this rank's fd 1 goes to stderr and the record is written to a
    # duplicate of the original stdout
    record_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RPT_BENCH_BACKEND=gloo is a rehearsal mode for boxes with fewer GPUs than ranks: ranks share
    # devices and the OR merge runs the torch.distributed composition over host memory. Default: RCCL.
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
    from rpt_amd._lib import RptError
    from rpt_amd.distributed import RcclComm, allreduce_or_filter, allreduce_or_native, allreduce_workspace, shard_range

    if args.collective_timeout_ms:
        rpt_lib.check(rpt_amd.load().rpt_collective_set_timeout_ms(args.collective_timeout_ms))

    cfg = args.config or ("C2" if args.build_rows is None and args.filter_rows is None else None)
    n_probe = int(args.probe_rows)
    if cfg is not None:
        n_build = int(args.build_rows) if args.build_rows else CONFIGS[cfg][0](world)
        n_filter = int(args.filter_rows) if args.filter_rows else CONFIGS[cfg][1](world)
    else:
        n_build = int(args.build_rows)
        n_filter = int(args.filter_rows) if args.filter_rows else n_build
    if cfg is not None and (n_build, n_filter) != (CONFIGS[cfg][0](world), CONFIGS[cfg][1](world)):
        cfg = None
    if cfg is None:
        cfg = "custom"
    tag = config_tag(cfg, args.key_type)
    p_permille = int(round(args.p * 1000))

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev_index]) if backend == "nccl" else dist.barrier()

    def keys_of(t):
        return t.to(torch.int32) if args.key_type == "i32" else t

    # ---- what this box streams (untimed, before anything else is resident) ------------------------
    shared_device = backend == "gloo" and world > max(1, torch.cuda.device_count())
    stream_cal = None
    if not args.no_stream_calibration and not shared_device:
        stream_cal = stream_calibration(device)

    # ---- CREATE_BF: sharded build + OR merge (reported, not the headline) -------------------------
    lo, hi = shard_range(n_build, rank, world)
    build_keys = keys_of(rpt_amd.synth_build_keys(hi - lo, start=lo, device=device))
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
    del build_keys
    # The product merge is rpt_bf_allreduce_or_ws over a library-made RCCL communicator. A failing
    # communicator ends the run (non-zero exit on every rank): a merge time is only ever reported for
    # the product path. `--merge torch` (or the gloo rehearsal) times the torch.distributed composition
    # instead, reported as torch_merge_ms, never as or_merge_ms.
    comm, merge_ws = None, None
    native = world > 1 and backend == "nccl" and args.merge == "native"
    merge_path = ("none (one GPU)" if world == 1 else
                  "rpt_bf_allreduce_or_ws (C-ABI: RCCL grouped send/recv reduce-scatter in 32 MiB rounds, OR kernel "
                  "on a helper stream, all-gather)" if native else
                  f"torch.distributed all_to_all + all_gather ({'--merge torch' if backend == 'nccl' else 'gloo rehearsal'})")
    if native:
        try:
            comm = RcclComm(device)  # every rank checks RCCL first and all agree: they fail together
        except RptError as e:
            print(f"[rank {rank}] native RCCL communicator failed: {e}", file=sys.stderr, flush=True)
            dist.destroy_process_group()
            sys.exit(3)
        merge_ws = allreduce_workspace(bf, comm)  # bounded staging, allocated outside the timed merge
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter() if world > 1 else t1
    if comm is not None:
        allreduce_or_native(bf, comm, workspace=merge_ws)  # rpt_bf_allreduce_or_ws (C-ABI), the product merge
    elif world > 1:
        allreduce_or_filter(bf)  # torch.distributed composition
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    merge_ws = None
    bf.finalized = True
    merge_check = None
    if world > 1 and not args.no_merge_check:
        # untimed: the OR-merged filter must be bit-identical to a single-GPU build of all rows (built
        # here in 1e9-row pieces: inserts into one filter compose)
        ref = rpt_amd.BloomFilter(n_filter, device=device)
        piece = 10**9
        for s0 in range(0, n_build, piece):
            ref.insert(keys_of(rpt_amd.synth_build_keys(min(piece, n_build - s0), start=s0, device=device)))
        same = bf.is_same_as(ref) and bf.minmax() == ref.minmax()  # rpt_bf_is_same_as: compared on the device
        ok = torch.tensor([1 if same else 0], dtype=torch.int64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        merge_check = ("bit-identical (words + key min/max) to a single-GPU build of all rows on every rank"
                       if ok.item() else "MISMATCH")
        del ref
        torch.cuda.empty_cache()
        if not ok.item():
            raise SystemExit("OR-merged filter differs from the single-GPU build")
    bf.probe_strategy = {"auto": 0, "gather": 1, "lds": 2, "partitioned": 3, "bucketed": 4}[args.strategy]
    strategy_name = {1: "gather", 2: "lds", 3: "partitioned", 4: "bucketed"}[bf.probe_strategy_for(n_probe)]

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
    # Per-kernel durations (roofline, kernels_ms) come from HIP events bracketing each kernel on its launch stream
    # (rpt_profiling_*). Between dependent kernels those events cost ~25 us per step (JOBDIM 1.774-1.778 ms with them,
    # 1.745-1.753 without: profiles/r06/kernel_events_overhead.txt), so by default the timed steps run without them
    # and an identical second pass of K steps records them; the kernels' durations are the same in either pass.
    rpt_lib.profiling_reset()
    rpt_lib.profiling(args.kernel_events_in_timed_region)
    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - ts
    rpt_lib.profiling(False)
    kernel_events = "inside the timed steps"
    if not args.kernel_events_in_timed_region:
        kernel_events = "an identical second pass of K steps right after the timed ones (the timed steps run without them)"
        rpt_lib.profiling(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        rpt_lib.profiling(False)
    ktimes = rpt_lib.kernel_times()

    survivors = int(out_count.item())
    probe_ms = statistics.mean(e[0].elapsed_time(e[1]) for e in events)

    t = torch.tensor([elapsed, (t1 - t0) / build_reps, t2 - t1], dtype=torch.float64,
                     device=device if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, insert_s, merge_s = t.tolist()

    # ---- C5 build + product merge + probe (after the headline; N > 1 by default, --c5-merge at N = 1) ----
    # At N > 1 it runs whatever the merge path: the product merge over RCCL, or the torch.distributed
    # composition (the gloo rehearsal on a box with fewer GPUs than ranks, --merge torch), so bench's sharding,
    # merge check, reductions and record assembly run before the driver's multi-GPU run does them.
    c5 = None
    if (world > 1 and not args.no_c5_merge) or (world == 1 and args.c5_merge):
        del keys, out_sel, ws
        torch.cuda.empty_cache()
        c5_comm = comm if comm is not None else (RcclComm.single(device) if world == 1 else None)
        coll_dev = device if backend == "nccl" else "cpu"

        def reduce_max(vals):
            v = torch.tensor(vals, dtype=torch.float64, device=coll_dev)
            if world > 1:
                dist.all_reduce(v, op=dist.ReduceOp.MAX)
            return v.tolist()

        def all_ok(flag):
            v = torch.tensor([1 if flag else 0], dtype=torch.int64, device=coll_dev)
            if world > 1:
                dist.all_reduce(v, op=dist.ReduceOp.MIN)
            return bool(v.item())

        def gather_ints(vals):
            v = torch.tensor(vals, dtype=torch.int64, device=coll_dev)
            if world == 1:
                return [v.tolist()]
            out = [torch.empty_like(v) for _ in range(world)]
            dist.all_gather(out, v)
            return [o.tolist() for o in out]

        shared = -(-world // max(1, torch.cuda.device_count())) if backend == "gloo" else 1
        c5_path = ("rpt_bf_allreduce_or_ws (C-ABI: RCCL grouped send/recv reduce-scatter in 32 MiB rounds, OR kernel "
                   "on a helper stream, all-gather)" if c5_comm is not None else
                   "torch.distributed all_to_all + all_gather in 256 MiB rounds ("
                   + ("gloo rehearsal, host-staged, ranks sharing GPUs" if backend == "gloo" else "--merge torch") + ")")
        c5 = run_c5_merge(args, rank, world, device, c5_comm, barrier, reduce_max, all_ok, gather_ints, c5_path,
                          shared_device_ranks=max(1, shared))
        if c5_comm is not None and c5_comm is not comm:
            c5_comm.close()

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = world * n_probe * args.steps / elapsed
        probe_bytes = key_bytes * n_probe + SEL_BYTES * survivors
        # dominant kernel of the step (largest total device time)
        dom_name, (dom_calls, dom_total) = max(ktimes.items(), key=lambda kv: kv[1][1])
        dom_ms = dom_total / dom_calls
        dom_calls_per_step = dom_calls / args.steps
        dom_bytes = algorithmic_bytes(dom_name, n_probe, survivors, key_bytes) / dom_calls_per_step
        achieved = dom_bytes / (dom_ms * 1e-3)
        traffic = pmc_traffic(dom_name, tag)
        # whole-step HBM traffic: every kernel of the step at its PMC bytes per launch
        step_traffic, unprofiled = 0.0, []
        for name, (calls, _total) in ktimes.items():
            tr = pmc_traffic(name, tag)
            if tr is None:
                unprofiled.append(name)
            else:
                step_traffic += tr["bytes_per_launch"] * calls / args.steps
        filter_bytes = bf.num_blocks * 8
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
                "workload": (f"{cfg}: USE_BF probe of {n_probe:.0e} {'int32' if args.key_type == 'i32' else 'int64'} keys "
                             f"per GPU against a blocked Bloom filter built from {n_build:.0e} keys (sized for "
                             f"{n_filter:.0e}: 2^{bf.log_num_blocks} blocks = {filter_bytes / 2**20:.0f} MiB), p={args.p}"),
                "config": cfg,
                "supplementary": {"JOBDIM": "not a BASELINE config: a JOB-sized dimension filter (1e5 keys, 128 KiB, whole "
                                            "filter in LDS), where the 60 % whole-probe target is plausible",
                                  "JOBDIM256": "not a BASELINE config: a 2e5-key dimension filter (256 KiB), the first "
                                               "128 KiB in LDS and the rest gathered from L2",
                                  "JOBDIM512": "not a BASELINE config: a 4e5-key dimension filter (512 KiB), the first "
                                               "128 KiB in LDS and the rest gathered from L2"}.get(cfg),
                "probe_rows_per_gpu": n_probe,
                "build_rows": n_build,
                "filter_bytes": filter_bytes,
                "pass_fraction": survivors / n_probe,
                "parallelism": f"row-range shards over {world} GPU(s), filter replicated "
                               f"({'RCCL rpt_bf_allreduce_or' if comm is not None else (backend + ' rehearsal' if world > 1 else 'no')} OR-merge)",
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
                "kernel_events": kernel_events,
                "launches_per_step": dom_calls_per_step,
                "algorithmic_bytes_per_launch": dom_bytes,
                # the same kernel against what this box streams (measured in this process, untimed): separates the
                # box from the code
                "stream_GBps": stream_cal["read_GBps"] if stream_cal else None,
                "copy_GBps": stream_cal["copy_GBps"] if stream_cal else None,
                "frac_of_stream": achieved / 1e9 / stream_cal["read_GBps"] if stream_cal else None,
                # the kernel's real HBM traffic rate (PMC bytes / its duration) against the box's read + write copy
                "traffic_frac_of_copy": (traffic["bytes_per_launch"] / (dom_ms * 1e-3) / 1e9 / stream_cal["copy_GBps"]
                                         if stream_cal and traffic else None),
            },
            "stream_calibration": stream_cal if stream_cal else (
                "skipped: ranks share one GPU (gloo rehearsal)" if shared_device else "skipped (--no-stream-calibration)"),
            "kernels_ms": {k: v[1] / v[0] for k, v in sorted(ktimes.items(), key=lambda kv: -kv[1][1])},
            "kernels_launches_per_step": {k: v[0] / args.steps for k, v in ktimes.items()},
            "probe_total": {
                "avg_ms": probe_ms,
                "algorithmic_bytes": probe_bytes,
                "achieved_GBps": probe_bytes / (probe_ms * 1e-3) / 1e9,
                "frac": probe_bytes / (probe_ms * 1e-3) / HBM_PEAK_BPS,
                "frac_of_stream": probe_bytes / (probe_ms * 1e-3) / 1e9 / stream_cal["read_GBps"] if stream_cal else None,
                # HBM bytes the whole step moves (PMC, every kernel) and their rate over the step
                "traffic": step_traffic if not unprofiled else None,
                "traffic_GBps": step_traffic / (probe_ms * 1e-3) / 1e9 if not unprofiled else None,
                "traffic_frac_of_copy": (step_traffic / (probe_ms * 1e-3) / 1e9 / stream_cal["copy_GBps"]
                                         if stream_cal and not unprofiled else None),
                "traffic_unprofiled_kernels": unprofiled,
            },
            "build": {
                "rows": n_build,
                "insert_ms": insert_s * 1e3,
                "insert_keys_per_s": (n_build / world) / insert_s if insert_s > 0 else None,
                # the product merge only (rpt_bf_allreduce_or_ws; workspace allocated before the timer)
                "or_merge_ms": merge_s * 1e3 if comm is not None else None,
                "torch_merge_ms": merge_s * 1e3 if world > 1 and comm is None else None,
                # per-GPU xGMI bytes of the OR all-reduce: 2 (W-1)/W of the filter
                "or_merge_GBps_per_gpu": (2 * (world - 1) / world * filter_bytes / merge_s / 1e9
                                          if comm is not None and merge_s > 0 else None),
                # the merge is direct point-to-point (every rank sends its 1/W slices to every peer, twice):
                # each of a GPU's W-1 xGMI links carries 2 S / W of it (GB/s per link)
                "or_merge_GBps_per_link": (2 / world * filter_bytes / merge_s / 1e9
                                           if comm is not None and merge_s > 0 else None),
                "merge_check": merge_check,
                "merge_path": merge_path,
            },
        }
        if c5 is not None:
            line["c5_merge"] = c5
        if not args.no_cpu_baseline and world == 1:
            sample = int(args.cpu_sample) if args.cpu_sample else n_probe
            threads = args.cpu_threads or cpu_share()
            src = "--cpu-threads" if args.cpu_threads else "this process's CPU share: affinity mask capped by the cgroup quota"
            cb = cpu_baseline(n_build, n_filter, p_permille, sample, threads, src, args.key_type, args.cpu_lag)
            if sample == n_probe:  # same rows, same filter: a full-size cross-check of the survivor count
                cb["survivors_match_gpu"] = cb["survivors"] == survivors
            line["cpu_baseline"] = cb
        print(json.dumps(line), file=record_out, flush=True)

    if comm is not None:
        comm.close()
    if world > 1:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
