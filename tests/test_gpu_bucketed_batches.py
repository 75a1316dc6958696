"""Bucketed inserts of more rows than one level-1 pass takes (rpt_bf_insert_ws runs them in batches:
level-1 list positions are 32-bit, so the product batches above 2^31 rows). The test build of the
library (tests/loopback/build/librpt_gpu_testing.so, RPT_TESTING_HOOKS) batches above 2^20 rows, so the
batch loop -- key pointer, validity words and dictionary selection advanced per batch -- runs here at a
few million rows. Filter words and key min/max against the oracle."""
import ctypes
import os

import numpy as np
import pytest
import torch

import golden_util as gu
import rpt_oracle as orc
from conftest import REPO

pytestmark = pytest.mark.gpu

INS_BUCKETED = 3
TEST_LIB = os.path.join(REPO, "tests", "loopback", "build", "librpt_gpu_testing.so")


@pytest.fixture(scope="module")
def tlib():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    torch.cuda.set_device(0)
    from rpt_amd import _lib

    _lib.load()
    t = _lib.load_variant(TEST_LIB)
    t.rpt_testing_bucketed_insert_batch.restype = ctypes.c_uint64
    assert t.rpt_testing_bucketed_insert_batch() == 1 << 20
    return t


def dev(a: np.ndarray) -> torch.Tensor:
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


@pytest.mark.parametrize("dtype,n,nulls,dictionary", [
    (np.int64, 2_500_000, False, False),       # 3 batches, the last ragged
    (np.int64, 3 * (1 << 20), True, False),    # whole batches, validity words advanced per batch
    (np.int32, 2_200_000, True, False),
    (np.int64, 2_100_003, True, True),          # dictionary: the selection advances, keys / validity stay
])
def test_bucketed_insert_in_batches_vs_oracle(tlib, dtype, n, nulls, dictionary):
    import rpt_amd

    log_nb = 25  # 256 MiB, 8 buckets
    rng = np.random.default_rng(n)
    info = np.iinfo(dtype)
    if dictionary:
        dict_keys = rng.integers(info.min, info.max, size=300_000, dtype=dtype, endpoint=True)
        key_sel = rng.integers(0, dict_keys.size, n).astype(np.uint32)
        valid = rng.random(dict_keys.size) > 0.1
        keys, kw = dict_keys, {"key_sel": key_sel}
    else:
        keys = rng.integers(info.min, info.max, size=n, dtype=dtype, endpoint=True)
        valid = rng.random(n) > 0.05 if nulls else None
        kw = {}
    vw = gu.validity_words(valid) if valid is not None else None
    bf = rpt_amd.BloomFilter(log_num_blocks=log_nb, lib=tlib)
    bf.insert(dev(keys), strategy=INS_BUCKETED, validity=dev(vw) if vw is not None else None,
              key_sel=dev(kw["key_sel"]) if dictionary else None, n=n if dictionary else None)
    torch.cuda.synchronize()
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, keys, validity=vw, **kw)
    assert np.array_equal(bf.export_words(), w)
    assert bf.minmax() == orc.minmax(keys, validity=vw, **kw)
    bf.close()


def test_level1_error_path_is_conservative(tlib):
    """A level-1 chunk bound hit (never expected: the bounds cover one list holding a whole group) must not
    turn into false negatives. Forced through the test build's hook: a bucketed probe then passes every row
    and a bucketed insert sets every filter bit; clearing the hook restores exact results."""
    import rpt_amd

    tlib.rpt_testing_force_l1_error.argtypes = [ctypes.c_int]
    tlib.rpt_testing_force_l1_error.restype = None
    log_nb = 23  # 64 MiB, 2 buckets
    rng = np.random.default_rng(5)
    keys = rng.integers(-2**62, 2**62, size=300_000, dtype=np.int64)
    probe = np.where(rng.random(200_003) < 0.2, keys[rng.integers(0, keys.size, 200_003)],
                     rng.integers(-2**62, 2**62, size=200_003, dtype=np.int64))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, keys)
    bf = rpt_amd.BloomFilter(log_num_blocks=log_nb, lib=tlib)
    bf.probe_strategy = 4  # BUCKETED
    bf.insert(dev(keys), strategy=1)  # atomic: exact words
    assert np.array_equal(bf.export_words(), w)
    try:
        tlib.rpt_testing_force_l1_error(1)
        sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
        assert np.array_equal(sel, np.arange(probe.size, dtype=np.uint32))  # every row passes
        full = rpt_amd.BloomFilter(log_num_blocks=log_nb, lib=tlib)
        full.insert(dev(keys), strategy=INS_BUCKETED)
        torch.cuda.synchronize()
        assert (full.export_words() == np.uint64(2**64 - 1)).all()  # every bit set
        assert full.minmax() == orc.minmax(keys)
        full.close()
    finally:
        tlib.rpt_testing_force_l1_error(0)
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe))
    again = rpt_amd.BloomFilter(log_num_blocks=log_nb, lib=tlib)
    again.insert(dev(keys), strategy=INS_BUCKETED)
    assert np.array_equal(again.export_words(), w)
    again.close()
    bf.close()
