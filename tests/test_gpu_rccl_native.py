"""rpt_bf_allreduce_or (the native RCCL OR all-reduce for C++ callers) on a single-rank RCCL
communicator: librccl loads, the collective runs, and the filter words, key min/max and has_data come
back unchanged. World sizes > 1 need one GPU per rank (RCCL refuses two ranks on one device); the
Python/torch.distributed merge that bench.py uses is covered at world sizes 2-4 with gloo."""
import ctypes

import numpy as np
import pytest
import torch

import rpt_oracle as orc

pytestmark = pytest.mark.gpu


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # rccl.h NCCL_UNIQUE_ID_BYTES


@pytest.fixture(scope="module")
def comm():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    torch.cuda.set_device(0)
    rccl = ctypes.CDLL("librccl.so.1")
    uid = _UniqueId()
    assert rccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
    c = ctypes.c_void_p()
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
