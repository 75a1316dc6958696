"""Multi-GPU build: per-rank partial filters OR-merged over RCCL (xGMI), one process per GPU.

The reference has no distributed path (DuckDB morsel threads only); this is the
MI355X-native scale-out of PhysicalCreateBF's parallel sink (physical_create_bf.hpp:43-45):

  * build rows are split by contiguous row range across ranks; every rank sizes its partial filter
    by the GLOBAL row count, so all partials share log_num_blocks;
  * OR is commutative and idempotent, so OR-ing the partials gives exactly the single-GPU filter;
  * RCCL has no bitwise-OR reduction (rccl.h ncclRedOp_t = sum/prod/max/min/avg), so the OR
    all-reduce is composed as a reduce-scatter by OR + all-gather:
        1. all_to_all_single: rank j receives slice j of every peer's filter (all xGMI links busy),
        2. local HIP kernel ORs the W received slices (rpt_words_or_slices),
        3. all_gather_into_tensor replicates the merged slices.
    Per-GPU traffic is 2(W-1)/W * S bytes, spread over the point-to-point links.
  * the probe is sharded by row range with a replicated filter: each rank's ascending local sel plus
    its row offset, concatenated in rank order, is the global ascending sel — no exchange.

Two implementations of the OR all-reduce:
  * `RcclComm` + `allreduce_or_native`: the product path. librpt_gpu.so's `rpt_bf_allreduce_or_ws`
    (grouped ncclSend/ncclRecv reduce-scatter by OR in bounded rounds overlapped with the OR kernel,
    then an all-gather, in place on the filter words) over a communicator the library creates
    (`rpt_rccl_comm_init_rank`, unique id broadcast over the torch.distributed group). This is what a
    C++ / DuckDB caller gets; bench.py uses it on GPUs.
  * `allreduce_or_filter`: the same choreography in torch.distributed collectives, used to rehearse
    the multi-rank path on CPU (gloo); `or_slices` is injectable so it runs without a GPU in tests.
"""
from __future__ import annotations

import ctypes
import functools
from typing import Callable, Optional

import torch
import torch.distributed as dist

OrSlices = Callable[[torch.Tensor, torch.Tensor, int, int], None]
INT64_MAX, INT64_MIN = (1 << 63) - 1, -(1 << 63)


def cpu_or_slices(dst: torch.Tensor, srcs: torch.Tensor, k: int, n_words: int) -> None:
    """Reference OR of k slices (torch, any device) — used by the gloo tests."""
    v = srcs[: k * n_words].view(k, n_words)
    dst[:n_words] = functools.reduce(torch.bitwise_or, [v[i] for i in range(k)])


def gpu_or_slices(dst: torch.Tensor, srcs: torch.Tensor, k: int, n_words: int) -> None:
    from .bloom import words_or_slices

    words_or_slices(dst, srcs, k, n_words)


def padded_words(num_words: int, world: int) -> int:
    """Smallest multiple of `world` >= num_words (filters are 2^k words; world may be any size)."""
    return ((num_words + world - 1) // world) * world


def or_allreduce_words(full: torch.Tensor, group=None, or_slices: Optional[OrSlices] = None) -> None:
    """In-place bitwise-OR all-reduce of an int64 word tensor whose length is a multiple of world size."""
    world = dist.get_world_size(group)
    if world == 1:
        return
    if full.numel() % world:
        raise ValueError("word count must be a multiple of the world size (use padded_words)")
    if or_slices is None:
        or_slices = gpu_or_slices if full.is_cuda else cpu_or_slices
    slice_words = full.numel() // world
    recv = torch.empty_like(full)
    dist.all_to_all_single(recv, full, group=group)  # recv[j] = peer j's slice <my rank>
    mine = torch.empty(slice_words, dtype=full.dtype, device=full.device)
    or_slices(mine, recv, world, slice_words)
    del recv
    dist.all_gather_into_tensor(full, mine, group=group)


class RcclComm:
    """An RCCL communicator created by librpt_gpu.so for the ranks of a torch.distributed group (one GPU
    per rank): rank 0 draws the unique id (rpt_rccl_get_unique_id), the group broadcasts it, every rank
    joins with rpt_rccl_comm_init_rank. Pass `.handle` to rpt_bf_allreduce_or (allreduce_or_native).
    nonblocking=True joins with rpt_rccl_comm_init_rank_nonblocking instead: every RCCL call on the
    communicator returns at once and the merge polls it against the collective timeout, so even RCCL's
    host-side connection setup with a dead peer cannot block a rank past that bound."""

    ID_BYTES = 128  # RPT_RCCL_UNIQUE_ID_BYTES

    def __init__(self, device: torch.device, group=None, *, nonblocking: bool = False):
        from ._lib import RPT_ERR_COLLECTIVE, RptError, load

        self._lib = load()
        self.handle = None
        self.aborted = False
        self.device = torch.device(device)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        on_device = dist.get_backend(group) != "gloo"
        # 1. every rank checks that librccl loads and its GPU is usable, and the group agrees before
        #    anyone enters the collective init (a rank failing there would leave the others blocked in
        #    ncclCommInitRank)
        st = self._lib.rpt_rccl_available(dev)
        err = "" if st == 0 else self._lib.rpt_last_error().decode(errors="replace")
        ok = torch.tensor([1 if st == 0 else 0], dtype=torch.int64, device=self.device if on_device else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if not int(ok.item()):
            where = "this rank: " + err if st != 0 else "another rank"
            raise RptError(RPT_ERR_COLLECTIVE, f"RCCL unavailable on {where}")
        # 2. rank 0 draws the id; a status byte rides along, so a failure there reaches every rank
        uid = torch.zeros(self.ID_BYTES + 1, dtype=torch.uint8)
        err = ""
        if self.rank == 0:
            st = self._lib.rpt_rccl_get_unique_id(uid.data_ptr())
            if st != 0:
                err = self._lib.rpt_last_error().decode(errors="replace")
                uid[self.ID_BYTES] = 1
        t = uid.to(self.device) if on_device else uid
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = t.cpu().contiguous()
        if int(uid[self.ID_BYTES]) != 0:
            raise RptError(RPT_ERR_COLLECTIVE, f"rpt_rccl_get_unique_id failed on rank 0{': ' + err if err else ''}")
        # 3. the collective init
        h = ctypes.c_void_p()
        init = self._lib.rpt_rccl_comm_init_rank_nonblocking if nonblocking else self._lib.rpt_rccl_comm_init_rank
        st = init(dev, self.world, uid.data_ptr(), self.rank, ctypes.byref(h))
        if st != 0:
            raise RptError(st, self._lib.rpt_last_error().decode(errors="replace"))
        self.handle = h

    @classmethod
    def single(cls, device: torch.device, *, nonblocking: bool = False) -> "RcclComm":
        """A one-rank communicator without a torch.distributed group (bench.py --c5-merge at N = 1: the
        merge's min/max all-reduce and bounded wait run through real RCCL; no peer words move)."""
        from ._lib import RptError, load

        self = cls.__new__(cls)
        self._lib = load()
        self.handle = None
        self.aborted = False
        self.device = torch.device(device)
        self.world, self.rank = 1, 0
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        uid = (ctypes.c_uint8 * cls.ID_BYTES)()
        h = ctypes.c_void_p()
        init = self._lib.rpt_rccl_comm_init_rank_nonblocking if nonblocking else self._lib.rpt_rccl_comm_init_rank
        for call in (lambda: self._lib.rpt_rccl_available(dev), lambda: self._lib.rpt_rccl_get_unique_id(uid),
                     lambda: init(dev, 1, uid, 0, ctypes.byref(h))):
            st = call()
            if st != 0:
                raise RptError(st, self._lib.rpt_last_error().decode(errors="replace"))
        self.handle = h
        return self

    def close(self) -> None:
        if self.handle is not None and self.handle.value:
            self._lib.rpt_rccl_comm_destroy(self.handle)
        self.handle = None

    def mark_aborted(self) -> None:
        """A failed merge aborted this communicator (ncclCommAbort freed it): release the library's record of it
        (rpt_rccl_comm_destroy does nothing else for an aborted one) and drop the handle."""
        self.aborted = True
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def allreduce_workspace(bf, comm: RcclComm) -> torch.Tensor:
    """Staging for rpt_bf_allreduce_or_ws: <= 2 (W-1) x 32 MiB + 256 B whatever the filter size; allocate
    it once, before a timed merge."""
    n = int(bf._lib.rpt_allreduce_workspace_bytes(comm.world, bf.log_num_blocks))
    return torch.empty(n, dtype=torch.uint8, device=bf.device)


# Workspaces of merges whose aborted streams did not drain: RCCL / OR kernels may still write them, so they
# are never returned to the caching allocator (the C wrapper rpt_bf_allreduce_or leaks its own the same way).
_STUCK_WORKSPACES: list = []


def allreduce_or_native(bf, comm: RcclComm, stream=None, workspace: Optional[torch.Tensor] = None) -> None:
    """CREATE_BF Combine across GPUs through the C-ABI (rpt_bf_allreduce_or_ws): words OR-merged in place,
    key min/max and has_data reduced; returns once has_data is known (one stream sync).

    A merge that fails after its first collective call aborts the communicator (RPT_ERR_COMM_ABORTED): the
    RcclComm is then marked dead (its handle dropped, the library's record of it released), so a later merge
    on it raises at once instead of handing RCCL a freed communicator."""
    from ._lib import RPT_ERR_COLLECTIVE, RPT_ERR_COMM_ABORTED, RptError, check
    from .bloom import _stream

    if comm.handle is None or not comm.handle.value:
        raise RptError(RPT_ERR_COLLECTIVE, "RcclComm is closed or was aborted by an earlier failed merge: make a "
                                           "new communicator")
    ws = workspace if workspace is not None else allreduce_workspace(bf, comm)
    try:
        check(bf._lib.rpt_bf_allreduce_or_ws(bf.handle, comm.handle, ws.data_ptr(), ws.numel(),
                                             _stream(bf.device, stream)), bf._lib)
    except RptError as e:
        if "did not drain" in str(e) or "still blocked" in str(e):
            _STUCK_WORKSPACES.append(ws)
        if e.status == RPT_ERR_COMM_ABORTED:
            comm.mark_aborted()
        raise


TORCH_MERGE_ROUND_WORDS = 32 << 20  # 256 MiB of words per round of the torch composition


def or_allreduce_words_rounds(full: torch.Tensor, group=None, round_words: int = TORCH_MERGE_ROUND_WORDS,
                              progress: Optional[Callable[[int, int], None]] = None) -> None:
    """or_allreduce_words over `full` in rounds of at most round_words words (rounded down to a multiple of the
    world size, at least one word per rank). A CUDA tensor under a gloo group is staged through host memory one
    round at a time; a CPU tensor is reduced in place. progress(done, total) is called after every round."""
    world = dist.get_world_size(group)
    total = full.numel()
    if total % world:
        raise ValueError("word count must be a multiple of the world size (use padded_words)")
    stage = full.is_cuda and dist.get_backend(group) == "gloo"
    step = max(world, (int(round_words) // world) * world)
    rounds = (total + step - 1) // step
    for i, lo in enumerate(range(0, total, step)):
        view = full[lo: min(total, lo + step)]  # a multiple of world words: total and step both are
        if stage:
            host = view.cpu()
            or_allreduce_words(host, group, or_slices=cpu_or_slices)
            view.copy_(host)
        else:
            or_allreduce_words(view, group)
        if progress is not None:
            progress(i + 1, rounds)


def allreduce_or_filter(bf, group=None, round_words: int = TORCH_MERGE_ROUND_WORDS,
                        progress: Optional[Callable[[int, int], None]] = None) -> None:
    """OR-merge a BloomFilter across all ranks (all ranks must hold the same log_num_blocks), and
    reduce its has_data flag and key min/max (CreateBF Combine, physical_create_bf.cpp:244-275).

    The words go through the all-reduce in rounds of at most `round_words` (rounded down to a multiple of
    the world size; every rank derives the same rounds from the same block count), so the receive buffers
    and, for gloo, the host staging stay bounded whatever the filter size (C5's 8 GiB filter included).
    With RCCL the words stay on the device. A gloo group (CPU collectives; used to rehearse the
    multi-rank path on a box with fewer GPUs than ranks) stages each round through host memory."""
    world = dist.get_world_size(group)
    buf = torch.zeros(padded_words(bf.num_blocks, world), dtype=torch.int64, device=bf.device)
    bf.copy_words_to(buf)
    on_device = dist.get_backend(group) != "gloo"
    or_allreduce_words_rounds(buf, group, round_words, progress)
    bf.copy_words_from(buf)
    del buf
    mm, has = allreduce_minmax_flag(bf.minmax(), not bf.is_empty(), group,
                                    device=bf.device if on_device else torch.device("cpu"))
    bf.set_minmax(mm)
    bf.set_has_data(has)


def allreduce_minmax_flag(mm: Optional[tuple], has_data: bool, group=None, device=None):
    """Combine per-rank (min, max) (or None) and has_data flags across ranks in ONE MIN all-reduce:
    the max and the flag are sent bit-complemented (~x = -x-1 reverses order without overflow).
    Returns (global (min, max) or None, global has_data)."""
    mn, mx = mm if mm is not None else (INT64_MAX, INT64_MIN)
    v = torch.tensor([mn, ~mx, ~int(bool(has_data))], dtype=torch.int64, device=device or "cpu")
    dist.all_reduce(v, op=dist.ReduceOp.MIN, group=group)
    g_mn, g_mx, g_has = int(v[0]), ~int(v[1]), ~int(v[2])
    return ((g_mn, g_mx) if g_mn <= g_mx else None), bool(g_has)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row range [lo, hi) of rank `rank` (remainder spread over the first ranks)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def build_sharded(local_keys: torch.Tensor, n_global: int, group=None, **insert_kw):
    """Per-rank partial filter sized by the global row count, then OR all-reduce."""
    from .bloom import BloomFilter

    bf = BloomFilter(n_global, device=local_keys.device)
    if local_keys.numel():
        bf.insert(local_keys, **insert_kw)
    allreduce_or_filter(bf, group)
    return bf
