"""Min/max dynamic filter and composite keys (§8f row 4) on the HIP path vs the
oracle. Bit-exact / value-exact."""
import numpy as np
import pytest
import torch

import golden_util as gu
import rpt_oracle as orc

pytestmark = pytest.mark.gpu

INT64_MIN, INT64_MAX = np.iinfo(np.int64).min, np.iinfo(np.int64).max


@pytest.fixture(scope="module")
def rpt():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    import rpt_amd

    rpt_amd.load()
    torch.cuda.set_device(0)
    return rpt_amd


def dev(a: np.ndarray) -> torch.Tensor:
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def keys_of(dtype, n, seed):
    rng = np.random.default_rng(seed)
    info = np.iinfo(dtype)
    return rng.integers(info.min, info.max, size=n, dtype=dtype, endpoint=True)


@pytest.mark.parametrize("strategy", ["atomic", "partitioned"])
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [1, 777, 65536, 1_500_000])
def test_minmax_matches_oracle(rpt, strategy, dtype, n):
    keys = keys_of(dtype, n, n)
    bf = rpt.BloomFilter(max(n, 1 << 17))  # 2^14+ blocks: partitioned insert applies
    st = rpt.RPT_INSERT_ATOMIC if strategy == "atomic" else rpt.RPT_INSERT_PARTITIONED
    if strategy == "partitioned" and not rpt.load().rpt_insert_workspace_bytes(n, bf.log_num_blocks):
        pytest.skip("partitioned insert does not apply")
    bf.insert(dev(keys), strategy=st)
    assert bf.minmax() == orc.minmax(keys)
    # the filter bits are unchanged by the fused reduction
    w = orc.new_words(bf.log_num_blocks)
    orc.insert_keys(w, bf.log_num_blocks, keys)
    assert np.array_equal(bf.export_words(), w)


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
def test_minmax_skips_nulls_and_follows_dictionary(rpt, dtype):
    n = 20_000
    keys = keys_of(dtype, n, 7)
    valid = np.random.default_rng(8).random(n) > 0.3
    vw = gu.validity_words(valid)
    bf = rpt.BloomFilter(n)
    bf.insert(dev(keys), validity=dev(vw))
    assert bf.minmax() == orc.minmax(keys, validity=vw)
    # dictionary vector: rows reference a subset of the dictionary; validity is by dictionary index
    sel = np.random.default_rng(9).integers(0, n, size=5000).astype(np.uint32)
    bf2 = rpt.BloomFilter(n)
    bf2.insert(dev(keys), key_sel=dev(sel), validity=dev(vw))
    assert bf2.minmax() == orc.minmax(keys, key_sel=sel, validity=vw)


def test_minmax_extremes_all_null_hash_and_lifecycle(rpt):
    ext = np.array([INT64_MIN, 0, INT64_MAX], dtype=np.int64)
    bf = rpt.BloomFilter(1000)
    assert bf.minmax() is None
    bf.insert(dev(ext))
    assert bf.minmax() == (int(INT64_MIN), int(INT64_MAX))
    bf.clear()
    assert bf.minmax() is None
    # all rows NULL -> no value (TypedUpdateMinMax returns before touching mm)
    bf.insert(dev(np.array([1, 2, 3], dtype=np.int64)), validity=dev(np.zeros(1, dtype=np.uint64)))
    assert bf.minmax() is None and not bf.is_empty()
    # raw hashes carry no key values
    bf.insert(dev(np.array([5, 6], dtype=np.uint64)), key_type=rpt.RPT_KEY_HASH)
    assert bf.minmax() is None
    # int32 values are reported sign-extended
    bf.insert(dev(np.array([-5, 9], dtype=np.int32)))
    assert bf.minmax() == (-5, 9)
    # resize + rehash re-derives the same values
    bf.reinitialize(5000)
    assert bf.minmax() is None
    bf.insert(dev(np.array([-5, 9], dtype=np.int32)))
    assert bf.minmax() == (-5, 9)
    bf.set_minmax((-1, 1))
    assert bf.minmax() == (-1, 1)
    bf.set_minmax(None)
    assert bf.minmax() is None


def test_minmax_merge_of_partials(rpt):
    a = keys_of(np.int64, 10_000, 1)
    b = keys_of(np.int64, 10_000, 2)
    p0, p1 = rpt.BloomFilter(20_000), rpt.BloomFilter(20_000)
    p0.insert(dev(a))
    p1.insert(dev(b))
    p0.merge_or(p1)
    assert p0.minmax() == orc.minmax(np.concatenate([a, b]))
    empty = rpt.BloomFilter(20_000)
    p0.merge_or(empty)  # merging a filter without values keeps them
    assert p0.minmax() == orc.minmax(np.concatenate([a, b]))


@pytest.mark.parametrize("ncols", [2, 3])
def test_hash_columns_matches_oracle(rpt, ncols):
    n = 50_000
    rng = np.random.default_rng(ncols)
    cols_np, cols_dev = [], []
    for j in range(ncols):
        dtype = np.int64 if j % 2 == 0 else np.int32
        keys = keys_of(dtype, n, 100 + j)
        c_np, c_dev = {"keys": keys}, {"keys": dev(keys)}
        if j == 1:  # a column with NULLs
            vw = gu.validity_words(rng.random(n) > 0.1)
            c_np["validity"], c_dev["validity"] = vw, dev(vw)
        cols_np.append(c_np)
        cols_dev.append(c_dev)
    h_gpu = rpt.hash_columns(cols_dev).cpu().numpy().view(np.uint64)
    assert np.array_equal(h_gpu, orc.hash_columns(cols_np))


def test_composite_key_filter_vs_oracle(rpt):
    n_build, n_probe = 30_000, 200_000
    a = keys_of(np.int64, n_build, 11)
    b = keys_of(np.int32, n_build, 12)
    # probe rows: half are build rows, half are random pairs
    rng = np.random.default_rng(13)
    pick = rng.integers(0, n_build, size=n_probe)
    hit = rng.random(n_probe) < 0.5
    pa = np.where(hit, a[pick], keys_of(np.int64, n_probe, 14))
    pb = np.where(hit, b[pick], keys_of(np.int32, n_probe, 15)).astype(np.int32)
    bf = rpt.BloomFilter(n_build)
    bf.insert(rpt.hash_columns([dev(a), dev(b)]), key_type=rpt.RPT_KEY_HASH)
    w = orc.new_words(bf.log_num_blocks)
    orc.insert_hashes(w, bf.log_num_blocks, orc.hash_columns([a, b]))
    assert np.array_equal(bf.export_words(), w)
    sel = bf.lookup_sel(rpt.hash_columns([dev(pa), dev(pb)]), key_type=rpt.RPT_KEY_HASH).cpu().numpy()
    ref = orc.lookup_sel_hashes(w, bf.log_num_blocks, orc.hash_columns([pa, pb]))
    assert np.array_equal(sel.astype(np.uint32), ref.astype(np.uint32))
    assert np.all(np.isin(np.flatnonzero(hit), sel))  # no false negatives
