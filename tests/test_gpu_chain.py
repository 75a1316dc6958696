"""USE_BF's filter chain in one launch (rpt_bf_probe_chain) vs the oracle: the rows passing every filter of
the chain, each probed on its own key column (physical_use_bf.cpp:127-179 probes them one after another, each
LookupSel over the previous survivors: the AND of the per-filter oracle results). Bit-exact."""
import functools
import os

import numpy as np
import pytest
import torch

import golden_util as gu
import rpt_oracle as orc

pytestmark = pytest.mark.gpu


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
    info = np.iinfo(dtype)
    return np.random.default_rng(seed).integers(info.min, info.max, size=n, dtype=dtype, endpoint=True)


def built(rpt, log_nb, keys):
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, keys)
    assert np.array_equal(bf.export_words(), w)
    return bf, w


def mostly_hits(rng, build, n, dtype, seed, frac=0.8):
    return np.where(rng.random(n) < frac, build[rng.integers(0, build.size, n)], keys_of(dtype, n, seed)).astype(dtype)


def sel_of(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n", [1, 63, 511, 2048, 5000, 16384])
@pytest.mark.parametrize("use_row_sel", [False, True])
def test_chain_mixed_columns_vs_oracle(rpt, n, use_row_sel):
    """Three filters (16 KiB, 256 KiB, 16 MiB) on an int64 FLAT column, an int32 column with NULLs and an
    int64 DICTIONARY column; with and without a row selection; ragged segment counts."""
    rng = np.random.default_rng(n)
    b0, b1, b2 = keys_of(np.int64, 2000, 1), keys_of(np.int32, 30000, 2), keys_of(np.int64, 1_000_000, 3)
    (f0, w0), (f1, w1), (f2, w2) = built(rpt, 11, b0), built(rpt, 15, b1), built(rpt, 21, b2)
    c0 = mostly_hits(rng, b0, n, np.int64, 4)
    c1 = mostly_hits(rng, b1, n, np.int32, 5)
    vw1 = gu.validity_words(rng.random(n) < 0.9)
    dict2 = mostly_hits(rng, b2, n // 2 + 1, np.int64, 6)
    ksel2 = rng.integers(0, dict2.size, n).astype(np.uint32)
    refs = [orc.probe_keys(w0, 11, c0), orc.probe_keys(w1, 15, c1, validity=vw1),
            orc.probe_keys(w2, 21, dict2, key_sel=ksel2)]
    exp = functools.reduce(np.intersect1d, refs).astype(np.uint32)
    cols = [dev(c0), {"keys": dev(c1), "validity": dev(vw1)}, {"keys": dev(dict2), "key_sel": dev(ksel2)}]
    row_sel = None
    if use_row_sel:
        row_sel = np.sort(rng.choice(n, size=max(1, n // 3), replace=False)).astype(np.uint32)
        exp = np.intersect1d(exp, row_sel).astype(np.uint32)
    got = rpt.probe_chain([f0, f1, f2], cols, row_sel=dev(row_sel) if row_sel is not None else None)
    assert np.array_equal(sel_of(got), exp)
    if n >= 2048:
        assert 0 < exp.size < (row_sel.size if row_sel is not None else n)  # every filter removes rows


def test_chain_of_one_equals_lookup_sel(rpt):
    b = keys_of(np.int64, 100_000, 7)
    f, _ = built(rpt, 17, b)
    rng = np.random.default_rng(8)
    for n in (1, 777, 16384):
        p = dev(mostly_hits(rng, b, n, np.int64, 9, frac=0.5))
        assert np.array_equal(sel_of(rpt.probe_chain([f], [p])), sel_of(f.lookup_sel(p)))


def test_chain_of_eight_with_hash_column(rpt):
    """RPT_MAX_CHAIN filters; one column given as precomputed hashes (RPT_KEY_HASH: same bits as the
    int64 keys it was hashed from); the same filter twice (idempotent AND)."""
    rng = np.random.default_rng(10)
    n = 12000
    builds = [keys_of(np.int64, 20000, 20 + i) for i in range(7)]
    fw = [built(rpt, 12 + (i % 4), b) for i, b in enumerate(builds)]
    cols_np = [mostly_hits(rng, b, n, np.int64, 40 + i, frac=0.97) for i, b in enumerate(builds)]
    refs = [orc.probe_keys(w, 12 + (i % 4), c) for i, ((_, w), c) in enumerate(zip(fw, cols_np))]
    exp = functools.reduce(np.intersect1d, refs + [refs[0]]).astype(np.uint32)
    cols = [dev(c) for c in cols_np]
    cols[3] = {"keys": rpt.hash_keys(cols[3]), "key_type": rpt.RPT_KEY_HASH}
    filters = [f for f, _ in fw] + [fw[0][0]]
    got = rpt.probe_chain(filters, cols + [cols[0]])
    assert np.array_equal(sel_of(got), exp)
    assert exp.size > 0


def test_chain_segments_emptied_early(rpt):
    """Segments whose rows all fail the first filter next to segments where most pass it."""
    n = 8192
    b0, b1 = keys_of(np.int64, 5000, 11), keys_of(np.int64, 5000, 12)
    (f0, w0), (f1, w1) = built(rpt, 14, b0), built(rpt, 14, b1)
    rng = np.random.default_rng(13)
    c0 = mostly_hits(rng, b0, n, np.int64, 14, frac=1.0)
    c0[:2048] = keys_of(np.int64, 2048, 15)  # four segments of (almost surely) misses
    c1 = mostly_hits(rng, b1, n, np.int64, 16, frac=0.5)
    exp = np.intersect1d(orc.probe_keys(w0, 14, c0), orc.probe_keys(w1, 14, c1)).astype(np.uint32)
    assert np.array_equal(sel_of(rpt.probe_chain([f0, f1], [dev(c0), dev(c1)])), exp)


def test_chain_empty_and_cleared_filters(rpt):
    b = keys_of(np.int64, 3000, 17)
    f, w = built(rpt, 13, b)
    empty = rpt.BloomFilter(log_num_blocks=13)
    p = dev(b[:1000])
    assert sel_of(rpt.probe_chain([f, empty], [p, p])).size == 0  # an empty filter passes nothing
    f.clear()  # deferred clear: the chain settles it before reading
    assert sel_of(rpt.probe_chain([f], [p])).size == 0
    f.insert(dev(b))
    assert np.array_equal(sel_of(rpt.probe_chain([f], [p])), orc.probe_keys(w, 13, b[:1000]))
    out = torch.empty(1, dtype=torch.int32, device="cuda:0")
    cnt = torch.full((1,), 7, dtype=torch.int64, device="cuda:0")
    rpt.probe_chain([f], [p], n=0, out_sel=out, out_count=cnt)
    assert int(cnt.item()) == 0


def test_chain_argument_errors(rpt):
    b = keys_of(np.int64, 100, 18)
    f, _ = built(rpt, 10, b)
    p = dev(b)
    with pytest.raises(rpt.RptError):
        rpt.probe_chain([], [])
    with pytest.raises(rpt.RptError):
        rpt.probe_chain([f] * 9, [p] * 9)  # more than RPT_MAX_CHAIN
    with pytest.raises(rpt.RptError):
        big = dev(np.zeros(16385, dtype=np.int64))
        rpt.probe_chain([f], [big])  # more than RPT_SMALL_PROBE_ROWS
    with pytest.raises(rpt.RptError):
        rpt.probe_chain([f, f], [p])  # one column per filter


# RPT_FUZZ_SEEDS seeds from RPT_FUZZ_SEED_BASE (tools/gpu_soak.sh sweeps more of them)
@pytest.mark.parametrize("seed", range(int(os.environ.get("RPT_FUZZ_SEED_BASE", "0")),
                                       int(os.environ.get("RPT_FUZZ_SEED_BASE", "0")) + int(os.environ.get("RPT_FUZZ_SEEDS", "16"))))
def test_chain_random(rpt, seed):
    """Seeded sweep: 1..8 filters of random sizes (128 B..64 MiB), each over its own column with a random
    key type (int64 / int32 / precomputed hashes), NULL rate, dictionary; random row counts and row
    selections. The AND of the oracle's per-filter results, bit-exact."""
    rng = np.random.default_rng(1000 + seed)
    k = int(rng.integers(1, 9))
    n = int(rng.choice([1, 2, 64, 513, 2048, int(rng.integers(1, 16385))]))
    filters, cols, refs = [], [], []
    for f in range(k):
        log_nb = int(rng.choice([4, 10, 14, 17, 21, 23]))
        dtype = np.int64 if rng.random() < 0.6 else np.int32
        build = keys_of(dtype, int(rng.integers(1, 50_000)), seed * 16 + f)
        bf, w = built(rpt, log_nb, build)
        filters.append(bf)
        m = int(rng.integers(1, 2 * n + 1)) if rng.random() < 0.4 else n  # dictionary size (if used)
        vals = mostly_hits(rng, build, m, dtype, 500 + seed * 16 + f, frac=float(rng.choice([0.5, 0.9, 1.0])))
        ksel = rng.integers(0, m, n).astype(np.uint32) if m != n else None
        valid = gu.validity_words(rng.random(m) >= 0.1) if rng.random() < 0.4 else None
        if rng.random() < 0.2 and dtype == np.int64:  # the column as precomputed hashes (NULLs not applied)
            h = rpt.hash_keys(dev(vals))
            col = {"keys": h, "key_type": rpt.RPT_KEY_HASH}
            ref = orc.probe_keys(w, log_nb, vals, key_sel=ksel)
        else:
            col = {"keys": dev(vals), "validity": dev(valid) if valid is not None else None}
            ref = orc.probe_keys(w, log_nb, vals, key_sel=ksel, validity=valid)
        if ksel is not None:
            col["key_sel"] = dev(ksel)
        cols.append(col)
        refs.append(ref)
    exp = functools.reduce(np.intersect1d, refs).astype(np.uint32)
    row_sel = None
    if rng.random() < 0.3:
        row_sel = np.sort(rng.choice(n, size=int(rng.integers(1, n + 1)), replace=False)).astype(np.uint32)
        exp = np.intersect1d(exp, row_sel).astype(np.uint32)
    got = rpt.probe_chain(filters, cols, row_sel=dev(row_sel) if row_sel is not None else None,
                          n=row_sel.size if row_sel is not None else n)
    assert np.array_equal(sel_of(got), exp)
