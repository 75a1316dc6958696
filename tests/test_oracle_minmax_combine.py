"""CPU checks of the oracle's min/max (TypedUpdateMinMax, physical_create_bf.cpp:86-119) and
composite-key CombineHash (bloom_filter.cpp:15-17) restatements against plain numpy / Python."""
import numpy as np
import pytest

import golden_util as gu
import rpt_oracle as orc

M64 = (1 << 64) - 1


def py_murmur(x: int) -> int:
    x ^= x >> 32
    x = (x * 0xD6E8FEB86659FD93) & M64
    x ^= x >> 32
    x = (x * 0xD6E8FEB86659FD93) & M64
    x ^= x >> 32
    return x


def py_hash(v: int, itemsize: int, valid: bool) -> int:
    if not valid:
        return 0xBF58476D1CE4E5B9
    return py_murmur(v & (0xFFFFFFFF if itemsize == 4 else M64))


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
def test_minmax_vs_numpy(dtype):
    rng = np.random.default_rng(1)
    info = np.iinfo(dtype)
    keys = rng.integers(info.min, info.max, size=10_000, dtype=dtype, endpoint=True)
    valid = rng.random(keys.size) > 0.25
    vw = gu.validity_words(valid)
    assert orc.minmax(keys) == (int(keys.min()), int(keys.max()))
    assert orc.minmax(keys, validity=vw) == (int(keys[valid].min()), int(keys[valid].max()))
    sel = rng.integers(0, keys.size, size=333).astype(np.uint32)
    vs = valid[sel]
    assert orc.minmax(keys, key_sel=sel, validity=vw) == (int(keys[sel][vs].min()), int(keys[sel][vs].max()))
    assert orc.minmax(keys[:0]) is None
    assert orc.minmax(keys[:64], validity=np.zeros(1, dtype=np.uint64)) is None


def test_minmax_extremes():
    k = np.array([np.iinfo(np.int64).max, np.iinfo(np.int64).min], dtype=np.int64)
    assert orc.minmax(k) == (int(k[1]), int(k[0]))
    k32 = np.array([-1, np.iinfo(np.int32).min, 7], dtype=np.int32)
    assert orc.minmax(k32) == (int(np.iinfo(np.int32).min), 7)


def test_hash_columns_vs_python():
    rng = np.random.default_rng(2)
    a = rng.integers(-(1 << 62), 1 << 62, size=200, dtype=np.int64)
    b = rng.integers(-(1 << 30), 1 << 30, size=200, dtype=np.int32)
    vb = rng.random(200) > 0.2
    h = orc.hash_columns([a, {"keys": b, "validity": gu.validity_words(vb)}])
    for i in range(200):
        ha = py_hash(int(a[i]), 8, True)
        hb = py_hash(int(b[i]), 4, bool(vb[i]))
        x = ha ^ (ha >> 32)  # DuckDB v1.1+ CombineHashScalar (restated, unpinned)
        assert int(h[i]) == ((x * 0xD6E8FEB86659FD93) & M64) ^ hb
    # one column: plain hash; order matters for two
    assert np.array_equal(orc.hash_columns([a]), orc.hash_keys(a))
    assert not np.array_equal(orc.hash_columns([a, a]), orc.hash_columns([a, a.astype(np.int32)]))
