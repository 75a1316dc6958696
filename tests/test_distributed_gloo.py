"""Multi-process (gloo, CPU) tests of the multi-GPU choreography in rpt_amd.distributed:
row-range sharding, the OR all-reduce composed from all_to_all + local OR + all_gather, and the
"OR of partials == single build" invariant, with the oracle doing the per-rank filter work."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_build, q):
    import sys

    for p in (PKG, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rpt_oracle as orc
        from rpt_amd.distributed import cpu_or_slices, or_allreduce_words, padded_words, shard_range

        lnb = orc.log_num_blocks(n_build)  # every rank sizes by the GLOBAL row count
        lo, hi = shard_range(n_build, rank, world)
        words = orc.new_words(lnb)
        orc.insert_keys(words, lnb, orc.synth_build_keys(hi - lo, start=lo))
        buf = torch.zeros(padded_words(words.size, world), dtype=torch.int64)
        buf[: words.size] = torch.from_numpy(words.view(np.int64))
        or_allreduce_words(buf, or_slices=cpu_or_slices)
        merged = buf[: words.size].numpy().view(np.uint64)
        # probe sharded by row range with the replicated filter: local sel + offset
        n_probe = 40000
        plo, phi = shard_range(n_probe, rank, world)
        keys = orc.synth_probe_keys(phi - plo, n_build, 250, start=plo)
        sel = orc.probe_keys(merged, lnb, keys).astype(np.int64) + plo
        gathered = [None] * world
        dist.all_gather_object(gathered, sel.tolist())
        if rank == 0:
            q.put((merged.copy(), np.concatenate([np.array(g, dtype=np.int64) for g in gathered])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])  # 8: the driver's largest scaling run
def test_sharded_build_or_merge_and_probe(world):
    n_build = 30011
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_build, q)) for r in range(world)]
    for p in procs:
        p.start()
    merged, sel = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    import rpt_oracle as orc

    lnb = orc.log_num_blocks(n_build)
    single = orc.new_words(lnb)
    orc.insert_keys(single, lnb, orc.synth_build_keys(n_build))
    assert np.array_equal(merged, single)  # bit-identical to the 1-GPU build
    ref = orc.probe_keys(single, lnb, orc.synth_probe_keys(40000, n_build, 250)).astype(np.int64)
    assert np.array_equal(sel, ref)  # concatenated per-rank sel == global ascending sel


def test_shard_range_partitions_rows():
    from rpt_amd.distributed import padded_words, shard_range

    for n in [0, 1, 7, 1000, 10**7 + 3]:
        for w in [1, 2, 3, 8]:
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    assert padded_words(1 << 21, 8) == 1 << 21 and padded_words(16, 3) == 18


def _rounds_worker(rank, world, port, q):
    import sys

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rpt_amd.distributed import or_allreduce_words_rounds, padded_words

        out = []
        for nw, round_words in [(1000, 7), (1000, 1), (4096, 10**9), (96, 64)]:
            g = torch.Generator().manual_seed(1000 * rank + nw)
            words = torch.randint(-(1 << 62), 1 << 62, (padded_words(nw, world),), generator=g, dtype=torch.int64)
            words[nw:] = 0
            mine = words.clone()
            or_allreduce_words_rounds(mine, round_words=round_words)
            out.append((words.numpy(), mine.numpy()))
        with pytest.raises(ValueError):
            or_allreduce_words_rounds(torch.zeros(world + 1, dtype=torch.int64))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_or_allreduce_in_bounded_rounds(world):
    """The torch composition of the OR all-reduce in rounds (what bench's gloo rehearsal and --merge torch run on
    C5's 8 GiB filter: 256 MiB rounds): every round size, including one word per rank and one round over
    everything, gives every rank the OR of all ranks' words."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rounds_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for case in range(4):
        want = np.bitwise_or.reduce([res[r][case][0] for r in range(world)])
        for r in range(world):
            assert np.array_equal(res[r][case][1], want), (case, r)


def _minmax_worker(rank, world, port, q):
    import sys

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rpt_amd.distributed import allreduce_minmax_flag

        i64 = np.iinfo(np.int64)
        cases = [
            # per-rank (min, max) or None, has_data
            [((-5, 9), True), ((3, 12), True), (None, True), ((int(i64.min), -1), True)],
            [(None, False), (None, True), (None, False), (None, False)],
            [(None, False), (None, False), (None, False), (None, False)],
            [((int(i64.max), int(i64.max)), True), (None, False), (None, False), (None, False)],
        ]
        out = []
        for c in cases:
            mm, has = c[rank]
            out.append(allreduce_minmax_flag(mm, has))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_minmax_and_flag_allreduce(world):
    """The one-collective (min, max, has_data) reduce of the multi-GPU build (CreateBF Combine)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_minmax_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    i64 = np.iinfo(np.int64)
    if world == 2:
        expect = [((-5, 12), True), (None, True), (None, False), ((int(i64.max), int(i64.max)), True)]
    else:
        expect = [((int(i64.min), 12), True), (None, True), (None, False), ((int(i64.max), int(i64.max)), True)]
    assert out == expect


def _rccl_id_worker(rank, world, port, mode, q):
    import sys

    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rpt_amd import _lib
        from rpt_amd.distributed import RcclComm

        lib = _lib.load()
        fail_avail = mode == "avail_rank1" and rank == 1
        fail_id = mode == "id_rank0" and rank == 0

        class Patched:  # RCCL / the GPU unusable on one rank, or rank 0 unable to draw an id
            def __getattr__(self, name):
                return getattr(lib, name)

            @staticmethod
            def rpt_rccl_available(_dev):
                return _lib.RPT_ERR_COLLECTIVE if fail_avail else _lib.RPT_OK

            @staticmethod
            def rpt_rccl_get_unique_id(ptr):
                return _lib.RPT_ERR_COLLECTIVE if fail_id else lib.rpt_rccl_get_unique_id(ptr)

        if mode != "none":
            _lib.load = lambda path=None: Patched()
        try:
            RcclComm(torch.device("cuda", 0))
            q.put((rank, "ok"))
        except _lib.RptError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["avail_rank1", "id_rank0", "none"])
def test_rccl_comm_failure_reaches_every_rank(mode):
    """RcclComm never leaves a rank waiting in the collective init: every rank first checks that RCCL
    loads and its GPU is usable and the group agrees (one rank failing -> every rank raises); rank 0's
    id draw carries its status to every rank; without a GPU (this container) every rank fails the
    check. bench.py then exits non-zero on every rank (no silent fallback)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rccl_id_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(got) == [0, 1]
    for r, msg in got.items():
        assert msg != "ok"
        if mode == "id_rank0":
            assert "failed on rank 0" in msg
        if mode == "avail_rank1":
            assert ("this rank" if r == 1 else "another rank") in msg
