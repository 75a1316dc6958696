"""rpt_bf_allreduce_or (the native RCCL OR all-reduce: the product merge, used by bench.py and by C++
callers) over a communicator from rpt_rccl_comm_init_rank.

* one rank: librccl loads, the collective runs, and the filter words, key min/max and has_data come
  back unchanged (with a blocking and a non-blocking communicator the library made, and with one the caller
  created itself through librccl), and through the Python binding's RcclComm.single (blocking and
  non-blocking) with a caller-allocated merge workspace;
* two ranks, one GPU each (skipped on a one-GPU box: RCCL refuses two ranks on one device): every
  rank inserts its row-range shard, the merged filter equals the oracle's filter of all rows, and the
  key min/max / has_data are reduced (an empty rank included). The torch.distributed composition used
  for gloo rehearsals is covered at world sizes 2-4 in tests/test_distributed_gloo.py;
* bench.py's C5 section (the `c5_merge` object of an N > 1 run) end to end at N = 1 through a one-rank
  communicator (`--c5-merge`, fewer rows per rank; the filter stays the 8 GiB one sized for 8e9 rows)."""
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

import rpt_oracle as orc

pytestmark = pytest.mark.gpu


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # rccl.h NCCL_UNIQUE_ID_BYTES


@pytest.fixture(scope="module", params=["library", "library-nonblocking", "caller"])
def comm(request):
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    torch.cuda.set_device(0)
    from rpt_amd import _lib

    lib = _lib.load()
    c = ctypes.c_void_p()
    if request.param.startswith("library"):  # rpt_rccl_get_unique_id + rpt_rccl_comm_init_rank[_nonblocking]
        uid = (ctypes.c_uint8 * 128)()
        assert lib.rpt_rccl_get_unique_id(uid) == 0, lib.rpt_last_error()
        init = lib.rpt_rccl_comm_init_rank_nonblocking if request.param.endswith("nonblocking") else lib.rpt_rccl_comm_init_rank
        assert init(0, 1, uid, 0, ctypes.byref(c)) == 0, lib.rpt_last_error()
        yield c
        assert lib.rpt_rccl_comm_destroy(c) == 0
    else:  # a communicator the caller made itself (a DuckDB shim that owns one)
        rccl = ctypes.CDLL("librccl.so.1")
        uid = _UniqueId()
        assert rccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
        assert rccl.ncclCommInitRank(ctypes.byref(c), 1, uid, 0) == 0
        yield c
        rccl.ncclCommDestroy(c)


@pytest.fixture(scope="module")
def rpt():
    import rpt_amd

    rpt_amd.load()
    return rpt_amd


@pytest.mark.parametrize("n_keys", [0, 100000])
def test_single_rank_allreduce_is_identity(rpt, comm, n_keys):
    from rpt_amd import _lib

    lib = _lib.load()
    keys = orc.synth_build_keys(max(n_keys, 1))[:n_keys]
    bf = rpt.BloomFilter(200000)
    if n_keys:
        bf.insert(torch.from_numpy(keys.view(np.int64)).to("cuda:0"))
    before_words, before_mm, before_has = bf.export_words(), bf.minmax(), not bf.is_empty()
    st = lib.rpt_bf_allreduce_or(bf.handle, comm, None)
    assert st == 0, lib.rpt_last_error()
    torch.cuda.synchronize()
    assert np.array_equal(bf.export_words(), before_words)
    assert bf.minmax() == before_mm
    assert (not bf.is_empty()) == before_has
    if n_keys:
        assert before_mm == (int(keys.view(np.int64).min()), int(keys.view(np.int64).max()))


@pytest.mark.parametrize("nonblocking", [False, True])
def test_rccl_comm_single_through_python(rpt, nonblocking):
    """rpt_amd.distributed.RcclComm.single (bench.py --c5-merge at N = 1), blocking and non-blocking, with
    allreduce_or_native and a caller-allocated workspace: the merged filter is the rank's own."""
    from rpt_amd.distributed import RcclComm, allreduce_or_native, allreduce_workspace

    comm = RcclComm.single(torch.device("cuda", 0), nonblocking=nonblocking)
    try:
        keys = orc.synth_build_keys(250000)
        bf = rpt.BloomFilter(keys.size)
        bf.insert(torch.from_numpy(keys.view(np.int64)).to("cuda:0"))
        ws = allreduce_workspace(bf, comm)
        for _ in range(2):  # OR is idempotent: a second merge changes nothing
            allreduce_or_native(bf, comm, workspace=ws)
        lnb = bf.log_num_blocks
        ref = orc.new_words(lnb)
        orc.insert_keys(ref, lnb, keys)
        assert np.array_equal(bf.export_words(), ref)
        assert bf.minmax() == orc.minmax(keys) and not bf.is_empty()
    finally:
        comm.close()


def _two_rank_worker(rank, world, store_path, n_build, empty_rank, q):
    import torch.distributed as dist

    try:
        torch.cuda.set_device(rank)
        dist.init_process_group("gloo", init_method=f"file://{store_path}", rank=rank, world_size=world)
        import rpt_amd
        from rpt_amd.distributed import RcclComm, allreduce_or_native, shard_range

        comm = RcclComm(torch.device("cuda", rank))
        lo, hi = shard_range(n_build, rank, world)
        bf = rpt_amd.BloomFilter(n_build, device=f"cuda:{rank}")
        if rank != empty_rank:
            bf.insert(rpt_amd.synth_build_keys(hi - lo, start=lo, device=f"cuda:{rank}"))
        allreduce_or_native(bf, comm)
        lnb = bf.log_num_blocks
        ref = orc.new_words(lnb)
        keys = orc.synth_build_keys(n_build)
        if empty_rank >= 0:
            elo, ehi = shard_range(n_build, empty_rank, world)
            keys = np.concatenate([keys[:elo], keys[ehi:]])
        orc.insert_keys(ref, lnb, keys)
        ok = np.array_equal(bf.export_words(), ref) and bf.minmax() == orc.minmax(keys) and not bf.is_empty()
        comm.close()
        dist.destroy_process_group()
        q.put((rank, bool(ok), ""))
    except Exception as e:  # reported to the parent
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("n_build,empty_rank", [(3_000_000, -1), (100_001, 1)])
def test_two_rank_allreduce_matches_single_build(n_build, empty_rank):
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs (RCCL allows one rank per device)")
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        store = os.path.join(d, "store")
        procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, store, n_build, empty_rank, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=180) for _ in procs]
        for p in procs:
            p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_bench_c5_merge_section_one_rank():
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--steps", "2", "--warmup", "1", "--probe-rows", "1e7",
           "--no-cpu-baseline", "--c5-merge", "--c5-rows-per-rank", "2e7", "--collective-timeout-ms", "60000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    c5 = line["c5_merge"]
    assert c5["merge_check"].startswith("bit-identical"), c5
    assert c5["filter_bytes"] == 8 << 30 and c5["rows_per_rank"] == 2 * 10**7 and c5["n_gpus"] == 1
    assert len(c5["or_merge_ms_reps"]) == 3 and c5["or_merge_ms"] > 0 and c5["collective_timeout_ms"] == 60000
    assert 0.09 < c5["survivors_rank0"] / c5["rows_per_rank"] < 0.2  # p = 0.1 plus the filter's false positives
