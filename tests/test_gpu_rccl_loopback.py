"""The product multi-GPU merge, rpt_bf_allreduce_or_ws (CREATE_BF Combine across GPUs; the reference's
single-node analogue is PhysicalCreateBF::Combine, physical_create_bf.cpp:244-275), run with W = 2..8
ranks on ONE GPU.

RCCL refuses two ranks on one device, so the ranks here are host threads of this process talking
through the loopback RCCL of tests/loopback/rccl_loopback.cpp (grouped send/recv matched at
ncclGroupEnd by device-to-device copies, stream-event ordered; MIN all-reduce through the host). The
merge code is the product's: the test build of csrc/rpt_gpu.hip (tests/loopback/build/
librpt_gpu_testing.so, compiled with RPT_TESTING_HOOKS, which only adds the entry point that swaps
the RCCL table). Every rank's merged words must equal the oracle's filter of all ranks' keys, and the
key min/max and has_data must be reduced:

* W in {2, 3, 5, 8}: uneven slices (W does not divide the block count), several reduce-scatter rounds
  (slices over RPT_ALLREDUCE_ROUND_WORDS words), an empty rank, all ranks empty, a filter smaller than
  one 32-word slice granule;
* C5's geometry: the 8 GiB / 2^30-block filter sized for 8e9 rows, W = 4;
* an error injected inside a group: every rank fails with RPT_ERR_COMM_ABORTED (the communicator was
  aborted), every group is closed, and the filters stay usable;
* non-blocking communicators (rpt_rccl_comm_init_rank_nonblocking): every grouped call and the all-reduce
  return ncclInProgress and the merge polls them to completion; results as with blocking ones;
* a silent peer (a rank that dies mid-merge without posting its side): the surviving ranks' grouped calls
  "succeed" and their streams block, as with RCCL, so only the merge's bounded wait ends them: every
  surviving rank aborts its communicator and returns RPT_ERR_COMM_ABORTED within the collective timeout (at
  once when RCCL reports the peer's death asynchronously), and no thread hangs;
* the owner-aborts mode (rpt_collective_set_abort_on_error(0)) for a caller that owns its communicator: the
  same failures return RPT_ERR_COLLECTIVE with every communicator untouched, and the owner's abort releases
  the blocked streams;
* the Python binding: an RcclComm whose merge aborted it is marked dead, and a second merge on it raises at
  once (no freed communicator reaches RCCL);
* rpt_rccl_comm_destroy of a non-blocking communicator finalizes it (ncclCommFinalize polled to completion).
"""
import ctypes
import os
import threading
import time

import numpy as np
import pytest
import torch

import rpt_oracle as orc
from conftest import REPO

pytestmark = pytest.mark.gpu

LOOP_DIR = os.path.join(REPO, "tests", "loopback", "build")
API_FIELDS = ["get_unique_id", "comm_init_rank", "comm_destroy", "group_start", "group_end", "send", "recv",
              "all_reduce", "comm_count", "comm_user_rank", "error_string", "comm_abort", "get_async_error",
              "comm_init_rank_config", "comm_finalize"]
LOOP_SYMBOLS = ["ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclGroupStart", "ncclGroupEnd",
                "ncclSend", "ncclRecv", "ncclAllReduce", "ncclCommCount", "ncclCommUserRank", "ncclGetErrorString",
                "ncclCommAbort", "ncclCommGetAsyncError", "ncclCommInitRankConfig", "ncclCommFinalize"]
ROUND_WORDS = 4 << 20  # RPT_ALLREDUCE_ROUND_WORDS
RPT_ERR_COLLECTIVE = 6
RPT_ERR_COMM_ABORTED = 7  # a merge that failed after its first collective call aborted the communicator


class ApiTable(ctypes.Structure):  # rpt_rccl_api_table (csrc/rpt_gpu_testing.h)
    _fields_ = [(f, ctypes.c_void_p) for f in API_FIELDS]


@pytest.fixture(scope="module")
def env():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    torch.cuda.set_device(0)
    from rpt_amd import _lib

    _lib.load()
    tlib = _lib.load_variant(os.path.join(LOOP_DIR, "librpt_gpu_testing.so"))
    tlib.rpt_testing_set_rccl_api.restype = ctypes.c_int
    tlib.rpt_testing_set_rccl_api.argtypes = [ctypes.c_void_p]
    loop = ctypes.CDLL(os.path.join(LOOP_DIR, "librccl_loopback.so"))
    loop.rpt_loopback_fail_op.argtypes = [ctypes.c_int, ctypes.c_int]
    loop.rpt_loopback_silent_peer.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    loop.rpt_loopback_stuck.argtypes = [ctypes.c_int]
    loop.rpt_loopback_group_depth.restype = ctypes.c_int
    loop.rpt_loopback_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    loop.rpt_loopback_finalize_count.restype = ctypes.c_int
    loop.ncclCommAbort.argtypes = [ctypes.c_void_p]
    table = ApiTable(*[ctypes.cast(getattr(loop, s), ctypes.c_void_p) for s in LOOP_SYMBOLS])
    assert tlib.rpt_testing_set_rccl_api(ctypes.byref(table)) == 0, tlib.rpt_last_error()
    yield tlib, loop
    assert tlib.rpt_testing_set_rccl_api(None) == 0


def in_threads(world, fn, join_timeout=600):
    """Run fn(rank) on `world` threads (ctypes releases the GIL inside the library calls)."""
    errs = []

    def wrap(r):
        try:
            fn(r)
        except Exception as e:  # surfaced below
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=wrap, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    deadline = time.monotonic() + join_timeout
    for t in ts:
        t.join(timeout=max(0.0, deadline - time.monotonic()))
    assert not any(t.is_alive() for t in ts), "a rank thread hung"
    assert not errs, errs


def make_comms(tlib, world, nonblocking=False):
    uid = (ctypes.c_uint8 * 128)()
    assert tlib.rpt_rccl_get_unique_id(uid) == 0, tlib.rpt_last_error()
    comms = [ctypes.c_void_p() for _ in range(world)]
    st = [None] * world
    init_fn = tlib.rpt_rccl_comm_init_rank_nonblocking if nonblocking else tlib.rpt_rccl_comm_init_rank

    def init(r):
        st[r] = init_fn(0, world, uid, r, ctypes.byref(comms[r]))

    in_threads(world, init)
    assert st == [0] * world
    return comms


def destroy_comms(tlib, comms):
    for c in comms:
        assert tlib.rpt_rccl_comm_destroy(c) == 0


def slices(nw, world):
    """Rank j's word range (MergeGeom in csrc/rpt_gpu.hip): starts rounded down to 32 words."""
    lo = [((nw * j) // world) & ~31 for j in range(world)] + [nw]
    return [(lo[j], lo[j + 1]) for j in range(world)]


def expected_rounds(nw, world):
    mx = max(b - a for a, b in slices(nw, world))
    r = max(2, min(ROUND_WORDS, (mx + 1) & ~1))
    return -(-mx // r)


def shard(n, rank, world):
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def build_partials(tlib, world, log_nb, n_build, empty):
    import rpt_amd

    bfs, keys_used = [], []
    all_keys = orc.synth_build_keys(n_build) if n_build else np.zeros(0, dtype=np.uint64)
    for r in range(world):
        bf = rpt_amd.BloomFilter(log_num_blocks=log_nb, lib=tlib)
        lo, hi = shard(n_build, r, world)
        if r not in empty and hi > lo:
            bf.insert(rpt_amd.synth_build_keys(hi - lo, start=lo, device="cuda:0"))
            keys_used.append(all_keys[lo:hi])
        bfs.append(bf)
    torch.cuda.synchronize()
    keys = np.concatenate(keys_used) if keys_used else np.zeros(0, dtype=np.uint64)
    return bfs, keys


def allreduce_all(tlib, bfs, comms):
    world = len(bfs)
    L = bfs[0].log_num_blocks
    need = tlib.rpt_allreduce_workspace_bytes(world, L)
    wss = [torch.empty(need, dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    streams = [torch.cuda.Stream(device="cuda:0") for _ in range(world)]
    st = [None] * world

    def run(r):
        st[r] = tlib.rpt_bf_allreduce_or_ws(bfs[r].handle, comms[r], wss[r].data_ptr(), need, streams[r].cuda_stream)

    in_threads(world, run)
    torch.cuda.synchronize()
    return st, need


@pytest.mark.parametrize("world,log_nb,n_build,empty", [
    (2, 14, 20_000, ()),
    (3, 20, 300_000, ()),            # 2^20 words over 3 ranks: uneven slices
    (5, 25, 3_000_000, (2,)),        # 2^25 / 5 words per slice: 2 rounds, an empty rank
    (8, 20, 1_000_000, (0, 7)),      # empty first and last rank
    (8, 3, 40, (1,)),                # 8 words < one 32-word granule: the last rank owns them all
    (2, 24, 0, (0, 1)),              # every rank empty
    (3, 26, 4_000_000, ()),          # 2^26 / 3 words per slice: 6 rounds
])
def test_loopback_allreduce_matches_single_build(env, world, log_nb, n_build, empty):
    tlib, loop = env
    comms = make_comms(tlib, world)
    bfs, keys = build_partials(tlib, world, log_nb, n_build, set(empty))
    g0, b0 = ctypes.c_uint64(), ctypes.c_uint64()
    assert loop.rpt_loopback_stats(comms[0], ctypes.byref(g0), ctypes.byref(b0)) == 0
    st, need = allreduce_all(tlib, bfs, comms)
    assert st == [0] * world, tlib.rpt_last_error()
    nw = 1 << log_nb
    # bounded staging: 256 B + 2 (W-1) round pieces of <= 32 MiB
    assert need <= 256 + 2 * (world - 1) * ROUND_WORDS * 8
    g1, b1 = ctypes.c_uint64(), ctypes.c_uint64()
    assert loop.rpt_loopback_stats(comms[0], ctypes.byref(g1), ctypes.byref(b1)) == 0
    assert g1.value - g0.value == expected_rounds(nw, world) + 1  # reduce-scatter rounds + the all-gather
    # every word crosses W-1 links twice: reduce-scatter pieces in, merged slices out
    assert b1.value - b0.value == 2 * (world - 1) * nw * 8
    ref = orc.new_words(log_nb)
    if keys.size:
        orc.insert_keys(ref, log_nb, keys)
    want_mm = orc.minmax(keys) if keys.size else None
    for r, bf in enumerate(bfs):
        assert np.array_equal(bf.export_words(), ref), f"rank {r} words"
        assert bf.minmax() == want_mm, f"rank {r} min/max"
        assert bf.is_empty() == (keys.size == 0), f"rank {r} has_data"
    destroy_comms(tlib, comms)
    for bf in bfs:
        bf.close()


def test_loopback_allreduce_c5_geometry(env):
    """C5: a filter sized for 8e9 rows (2^30 blocks = 8 GiB) on every rank, W = 4 (4 x 8 GiB on one GPU),
    1.2e7 build keys over the ranks; every rank's 8 GiB of words against rank 0's on the device, and rank
    0's against the oracle's."""
    tlib, _loop = env
    world, log_nb, n_build = 4, 30, 12_000_000
    assert tlib.rpt_bf_log_num_blocks_for_rows(8 * 10**9) == log_nb
    comms = make_comms(tlib, world)
    bfs, keys = build_partials(tlib, world, log_nb, n_build, set())
    st, need = allreduce_all(tlib, bfs, comms)
    assert st == [0] * world, tlib.rpt_last_error()
    assert need <= 1 << 30  # staging <= 1 GiB (here 2 * 3 * 32 MiB)
    nw = 1 << log_nb
    w0 = torch.empty(nw, dtype=torch.int64, device="cuda:0")
    bfs[0].copy_words_to(w0)
    wr = torch.empty_like(w0)
    for r in range(1, world):
        bfs[r].copy_words_to(wr)
        assert torch.equal(w0, wr), f"rank {r} differs from rank 0"
    del wr
    ref = orc.new_words(log_nb)
    orc.insert_keys(ref, log_nb, keys)
    assert np.array_equal(w0.cpu().numpy().view(np.uint64), ref)
    for bf in bfs:
        assert bf.minmax() == orc.minmax(keys)
    destroy_comms(tlib, comms)
    del w0
    for bf in bfs:
        bf.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("fail_rank,fail_op", [(1, 1), (0, 0), (2, 9)])
def test_loopback_error_inside_group(env, fail_rank, fail_op):
    """An RCCL call failing inside a group: the failing rank closes its group before returning, every
    rank's all-reduce returns RPT_ERR_COMM_ABORTED (none hangs), no group stays open on any thread, and
    each filter is still usable afterwards (its write order was released)."""
    tlib, loop = env
    world, log_nb = 3, 25  # 2^25 / 3 words per slice: 3 rounds, so op 9 lands in a later round
    comms = make_comms(tlib, world)
    bfs, _keys = build_partials(tlib, world, log_nb, 300_000, set())
    need = tlib.rpt_allreduce_workspace_bytes(world, log_nb)
    wss = [torch.empty(need, dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    streams = [torch.cuda.Stream(device="cuda:0") for _ in range(world)]
    st, depth = [None] * world, [None] * world

    def run(r):
        st[r] = tlib.rpt_bf_allreduce_or_ws(bfs[r].handle, comms[r], wss[r].data_ptr(), need, streams[r].cuda_stream)
        depth[r] = loop.rpt_loopback_group_depth()

    loop.rpt_loopback_fail_op(fail_rank, fail_op)
    try:
        in_threads(world, run)
    finally:
        loop.rpt_loopback_fail_op(-1, -1)
    torch.cuda.synchronize()
    assert st == [RPT_ERR_COMM_ABORTED] * world
    assert depth == [0] * world
    for bf in bfs:  # still usable: a write after the failed merge and an export both complete
        bf.insert(torch.arange(1000, dtype=torch.int64, device="cuda:0"))
        assert bf.export_words().any()
    destroy_comms(tlib, comms)
    for bf in bfs:
        bf.close()


def test_loopback_workspace_is_checked(env):
    tlib, _loop = env
    comms = make_comms(tlib, 2)
    bfs, _ = build_partials(tlib, 2, 20, 1000, set())
    ws = torch.empty(64, dtype=torch.uint8, device="cuda:0")
    st = [None, None]

    def run(r):
        st[r] = tlib.rpt_bf_allreduce_or_ws(bfs[r].handle, comms[r], ws.data_ptr(), 64, None)

    in_threads(2, run)
    assert st == [4, 4]  # RPT_ERR_WORKSPACE, before any collective call
    destroy_comms(tlib, comms)


@pytest.mark.parametrize("silent_rank,silent_op,report", [(1, 1, 0), (0, 0, 1), (2, 9, 0), (1, 4, 1)])
def test_loopback_silent_peer_is_bounded(env, silent_rank, silent_op, report):
    """A rank fails inside a group and goes silent (rpt_loopback_silent_peer): it never posts the rest of
    its sends and tells nobody. The surviving ranks' ncclGroupEnd / ncclAllReduce return success and their
    streams block, as RCCL's kernels would wait for the dead peer. rpt_bf_allreduce_or_ws must not wait
    blindly: every rank returns RPT_ERR_COMM_ABORTED, the survivors within the collective timeout (promptly
    when ncclCommGetAsyncError reports the death), each communicator aborted (rpt_rccl_comm_destroy then
    does nothing), no thread left hanging, and the filters usable afterwards."""
    tlib, loop = env
    world, log_nb, bound_ms = 3, 25, 3000  # 3 reduce-scatter rounds: op 9 lands in round 2
    prev = tlib.rpt_collective_timeout_ms()
    assert tlib.rpt_collective_set_timeout_ms(0) == 1  # RPT_ERR_INVALID_ARGUMENT
    assert tlib.rpt_collective_set_timeout_ms(bound_ms) == 0
    comms = make_comms(tlib, world)
    bfs, _keys = build_partials(tlib, world, log_nb, 300_000, set())
    need = tlib.rpt_allreduce_workspace_bytes(world, log_nb)
    wss = [torch.empty(need, dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    streams = [torch.cuda.Stream(device="cuda:0") for _ in range(world)]
    st, took, err, depth = [None] * world, [None] * world, [None] * world, [None] * world

    def run(r):
        t0 = time.monotonic()
        st[r] = tlib.rpt_bf_allreduce_or_ws(bfs[r].handle, comms[r], wss[r].data_ptr(), need, streams[r].cuda_stream)
        took[r] = time.monotonic() - t0
        err[r] = tlib.rpt_last_error().decode(errors="replace")
        depth[r] = loop.rpt_loopback_group_depth()

    loop.rpt_loopback_silent_peer(silent_rank, silent_op, report)
    try:
        in_threads(world, run, join_timeout=bound_ms / 1000 * 4 + 30)
    finally:
        loop.rpt_loopback_silent_peer(-1, -1, 0)
        assert tlib.rpt_collective_set_timeout_ms(prev) == 0
    torch.cuda.synchronize()  # every stream drained: the aborts released the blocked ones
    assert st == [RPT_ERR_COMM_ABORTED] * world, err
    assert depth == [0] * world
    for r in range(world):
        assert "communicator aborted" in err[r], err[r]
        assert "did not drain" not in err[r], err[r]
        if r == silent_rank:
            continue
        assert took[r] < bound_ms / 1000 + 10, (r, took[r])
        if report:
            assert "asynchronous error" in err[r] and took[r] < bound_ms / 1000, (r, took[r], err[r])
        else:
            assert "no progress within" in err[r] and took[r] >= bound_ms / 1000 * 0.9, (r, took[r], err[r])
    for bf in bfs:  # still usable: its write order was released
        bf.insert(torch.arange(1000, dtype=torch.int64, device="cuda:0"))
        assert bf.export_words().any()
    destroy_comms(tlib, comms)  # aborted communicators: accepted, nothing called
    for bf in bfs:
        bf.close()


@pytest.mark.parametrize("world,log_nb,n_build", [(3, 25, 3_000_000), (2, 14, 20_000)])
def test_loopback_nonblocking_comms(env, world, log_nb, n_build):
    """Non-blocking communicators: init, every ncclGroupEnd and the all-reduce return ncclInProgress and
    report it twice more through ncclCommGetAsyncError (the loopback's emulation), so the merge's polling of
    in-progress calls runs for every group; the merged filters equal the oracle's as with blocking ones."""
    tlib, loop = env
    comms = make_comms(tlib, world, nonblocking=True)
    bfs, keys = build_partials(tlib, world, log_nb, n_build, set())
    st, _need = allreduce_all(tlib, bfs, comms)
    assert st == [0] * world, tlib.rpt_last_error()
    ref = orc.new_words(log_nb)
    orc.insert_keys(ref, log_nb, keys)
    for r, bf in enumerate(bfs):
        assert np.array_equal(bf.export_words(), ref), f"rank {r} words"
        assert bf.minmax() == orc.minmax(keys)
    f0 = loop.rpt_loopback_finalize_count()
    destroy_comms(tlib, comms)  # non-blocking: finalized (polled through ncclInProgress) before destroyed
    assert loop.rpt_loopback_finalize_count() - f0 == world
    for bf in bfs:
        bf.close()


def test_loopback_inprogress_forever_is_bounded(env):
    """A non-blocking communicator whose grouped call never leaves ncclInProgress (one rank, so nothing else
    waits): the merge polls it until the collective timeout, aborts the communicator and returns
    RPT_ERR_COMM_ABORTED; the filter stays usable and rpt_rccl_comm_destroy accepts the aborted handle."""
    tlib, loop = env
    bound_ms = 1500
    prev = tlib.rpt_collective_timeout_ms()
    comms = make_comms(tlib, 1, nonblocking=True)
    bfs, _keys = build_partials(tlib, 1, 20, 100_000, set())
    need = tlib.rpt_allreduce_workspace_bytes(1, 20)
    ws = torch.empty(need, dtype=torch.uint8, device="cuda:0")
    assert tlib.rpt_collective_set_timeout_ms(bound_ms) == 0
    loop.rpt_loopback_stuck(1)
    try:
        t0 = time.monotonic()
        st = tlib.rpt_bf_allreduce_or_ws(bfs[0].handle, comms[0], ws.data_ptr(), need, None)
        took = time.monotonic() - t0
        err = tlib.rpt_last_error().decode(errors="replace")
    finally:
        loop.rpt_loopback_stuck(0)
        assert tlib.rpt_collective_set_timeout_ms(prev) == 0
    assert st == RPT_ERR_COMM_ABORTED and "communicator aborted" in err, err
    assert bound_ms / 1000 * 0.9 <= took < bound_ms / 1000 + 10, took
    torch.cuda.synchronize()
    bfs[0].insert(torch.arange(1000, dtype=torch.int64, device="cuda:0"))
    assert bfs[0].export_words().any()
    destroy_comms(tlib, comms)
    bfs[0].close()


@pytest.mark.parametrize("silent_op,report", [(1, 0), (4, 1)])
def test_loopback_owner_aborts_mode(env, silent_op, report):
    """rpt_collective_set_abort_on_error(0), for a caller that owns its communicator: a silent peer
    still ends every rank's merge within the bound, but with RPT_ERR_COLLECTIVE and the communicator NOT
    aborted; the survivors' streams stay blocked in RCCL until the owner calls ncclCommAbort, which releases
    them; the filters are usable afterwards."""
    tlib, loop = env
    world, log_nb, bound_ms, silent_rank = 3, 25, 2000, 1
    prev = tlib.rpt_collective_timeout_ms()
    assert tlib.rpt_collective_abort_on_error() == 1  # the default
    assert tlib.rpt_collective_set_timeout_ms(bound_ms) == 0
    assert tlib.rpt_collective_set_abort_on_error(0) == 0 and tlib.rpt_collective_abort_on_error() == 0
    comms = make_comms(tlib, world)
    bfs, _keys = build_partials(tlib, world, log_nb, 300_000, set())
    need = tlib.rpt_allreduce_workspace_bytes(world, log_nb)
    wss = [torch.empty(need, dtype=torch.uint8, device="cuda:0") for _ in range(world)]
    streams = [torch.cuda.Stream(device="cuda:0") for _ in range(world)]
    st, took, err = [None] * world, [None] * world, [None] * world

    def run(r):
        t0 = time.monotonic()
        st[r] = tlib.rpt_bf_allreduce_or_ws(bfs[r].handle, comms[r], wss[r].data_ptr(), need, streams[r].cuda_stream)
        took[r] = time.monotonic() - t0
        err[r] = tlib.rpt_last_error().decode(errors="replace")

    loop.rpt_loopback_silent_peer(silent_rank, silent_op, report)
    try:
        in_threads(world, run, join_timeout=bound_ms / 1000 * 4 + 30)
    finally:
        loop.rpt_loopback_silent_peer(-1, -1, 0)
        assert tlib.rpt_collective_set_abort_on_error(1) == 0
        assert tlib.rpt_collective_set_timeout_ms(prev) == 0
    assert st == [RPT_ERR_COLLECTIVE] * world, err
    for r in range(world):
        assert "NOT aborted" in err[r] and "communicator aborted" not in err[r], err[r]
        if r != silent_rank:
            assert took[r] < bound_ms / 1000 + 10, (r, took[r])
            assert "still blocked" in err[r], err[r]  # RCCL's kernels hold the survivor's stream
            assert streams[r].query() is False
    for c in comms:  # the owner aborts its communicators: the blocked streams resume
        assert loop.ncclCommAbort(c) == 0
    torch.cuda.synchronize()
    for bf in bfs:
        bf.insert(torch.arange(1000, dtype=torch.int64, device="cuda:0"))
        assert bf.export_words().any()
        bf.close()
    # (the owner aborted them: not handed to rpt_rccl_comm_destroy)


def test_python_comm_marked_dead_after_abort(env):
    """rpt_amd.distributed.allreduce_or_native on a communicator a failed merge aborted: the error
    carries RPT_ERR_COMM_ABORTED, the RcclComm drops its handle, and a second merge on it raises at once with a
    clear message instead of passing a freed communicator to RCCL; close() is then a no-op."""
    from rpt_amd._lib import RptError
    from rpt_amd.distributed import RcclComm, allreduce_or_native

    tlib, loop = env
    world, log_nb = 2, 20
    comms = make_comms(tlib, world)
    bfs, _keys = build_partials(tlib, world, log_nb, 100_000, set())
    pcs = []
    for r in range(world):
        c = RcclComm.__new__(RcclComm)  # an RcclComm around a loopback communicator of the test library
        c._lib, c.handle, c.aborted, c.device, c.world, c.rank = tlib, comms[r], False, torch.device("cuda", 0), world, r
        pcs.append(c)
    errs = [None] * world

    def run(r):
        try:
            allreduce_or_native(bfs[r], pcs[r], stream=torch.cuda.Stream(device="cuda:0"))
        except RptError as e:
            errs[r] = e

    loop.rpt_loopback_fail_op(1, 1)
    try:
        in_threads(world, run)
    finally:
        loop.rpt_loopback_fail_op(-1, -1)
    torch.cuda.synchronize()
    for r in range(world):
        assert errs[r] is not None and errs[r].status == RPT_ERR_COMM_ABORTED, errs[r]
        assert pcs[r].aborted and pcs[r].handle is None
        with pytest.raises(RptError) as e2:
            allreduce_or_native(bfs[r], pcs[r])
        assert e2.value.status == RPT_ERR_COLLECTIVE and "aborted by an earlier failed merge" in str(e2.value)
        pcs[r].close()
    for bf in bfs:
        bf.close()
