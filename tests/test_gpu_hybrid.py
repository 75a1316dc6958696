"""The hybrid LDS/L2 direct probe (`probe_bits_hybrid_kernel`: 256 KiB .. 1 MiB filters, 2^15 .. 2^17 blocks, the
first 2^14 words staged in each workgroup's LDS and the rest gathered from L2) against the oracle, bit-exact: dense
int64 / int32 columns with ragged tails (the pipelined loop and the general loop), NULLs, and a dictionary vector
through a row selection; and AUTO's choice of it."""
import numpy as np
import pytest
import torch

import golden_util as gu
import rpt_oracle as orc

pytestmark = pytest.mark.gpu

GATHER, LDS, PARTITIONED = 1, 2, 3
LOG_NBS = [15, 16, 17]  # 256 KiB, 512 KiB, 1 MiB


@pytest.fixture(scope="module")
def rpt():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    import rpt_amd

    rpt_amd.load()
    torch.cuda.set_device(0)
    return rpt_amd


def dev(a: np.ndarray) -> torch.Tensor:
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def built(rpt, dtype, n_build, seed, LOG_NB):
    info = np.iinfo(dtype)
    rng = np.random.default_rng(seed)
    build = rng.integers(info.min, info.max, size=n_build, dtype=dtype, endpoint=True)
    w = orc.new_words(LOG_NB)
    orc.insert_keys(w, LOG_NB, build)
    bf = rpt.BloomFilter(log_num_blocks=LOG_NB)
    bf.insert(dev(build))
    assert np.array_equal(bf.export_words(), w)
    # keys land in both halves of the filter: the LDS-staged one and the L2-gathered one
    assert w[: 1 << 14].any() and w[1 << 14:].any()
    return bf, build, w, rng


def test_auto_picks_hybrid(rpt):
    # from 4 Mi rows (below, its LDS staging costs more than it saves: the gather); 1 MiB only up to 32 Mi rows
    for log_nb, expect in ((14, LDS), (15, LDS), (16, LDS), (17, LDS), (18, GATHER)):
        bf = rpt.BloomFilter(log_num_blocks=log_nb)
        assert bf.probe_strategy_for(1 << 24) == expect, log_nb
        assert bf.probe_strategy_for(1 << 22) == expect, log_nb
        assert bf.probe_strategy_for((1 << 22) - 1) == (LDS if log_nb == 14 else GATHER), log_nb
        bf.close()
    for log_nb in (15, 16):
        assert rpt.BloomFilter(log_num_blocks=log_nb).probe_strategy_for(1 << 28) == LDS
    assert rpt.BloomFilter(log_num_blocks=17).probe_strategy_for((1 << 25) - 1) == LDS
    assert rpt.BloomFilter(log_num_blocks=17).probe_strategy_for(1 << 25) == PARTITIONED


@pytest.mark.parametrize("LOG_NB", LOG_NBS)
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [16385, 100_003, 1 << 20, 3_000_001, (1 << 22) + 77])
def test_hybrid_dense_vs_oracle(rpt, dtype, n, LOG_NB):
    bf, build, w, rng = built(rpt, dtype, 150_000 << (LOG_NB - 15), n, LOG_NB)
    info = np.iinfo(dtype)
    probe = np.where(rng.random(n) < 0.3, build[rng.integers(0, build.size, n)],
                     rng.integers(info.min, info.max, size=n, dtype=dtype, endpoint=True)).astype(dtype)
    bf.probe_strategy = LDS  # AUTO takes it from 4 Mi rows; smaller batches exercise the same kernel here
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, LOG_NB, probe))
    bf.close()


@pytest.mark.parametrize("LOG_NB", LOG_NBS)
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
def test_hybrid_nulls_vs_oracle(rpt, dtype, LOG_NB):
    n = 200_001
    bf, build, w, rng = built(rpt, dtype, 150_000 << (LOG_NB - 15), 77, LOG_NB)
    probe = build[rng.integers(0, build.size, n)]
    valid = rng.random(n) > 0.1
    vw = gu.validity_words(valid)
    bf.probe_strategy = LDS
    sel = bf.lookup_sel(dev(probe), validity=dev(vw)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, LOG_NB, probe, validity=vw))
    bf.close()


@pytest.mark.parametrize("LOG_NB", LOG_NBS)
def test_hybrid_dictionary_rowsel_vs_oracle(rpt, LOG_NB):
    rng = np.random.default_rng(15)
    dict_vals = rng.integers(-10**12, 10**12, size=60_000, dtype=np.int64)
    n = 90_000
    key_sel = rng.integers(0, dict_vals.size, size=n).astype(np.uint32)
    valid = rng.random(dict_vals.size) > 0.05
    vw = gu.validity_words(valid)
    w = orc.new_words(LOG_NB)
    orc.insert_keys(w, LOG_NB, dict_vals, key_sel=key_sel[:40_000], validity=vw)
    bf = rpt.BloomFilter(log_num_blocks=LOG_NB)
    bf.insert(dev(dict_vals), key_sel=dev(key_sel[:40_000]), validity=dev(vw))
    assert np.array_equal(bf.export_words(), w)
    bf.probe_strategy = LDS
    row_sel = np.sort(rng.choice(n, size=50_000, replace=False)).astype(np.uint32)
    ref_rows = set(orc.probe_keys(w, LOG_NB, dict_vals, key_sel=key_sel, validity=vw).tolist())
    exp = np.array([r for r in row_sel if r in ref_rows], dtype=np.uint32)
    got = bf.lookup_sel(dev(dict_vals), key_sel=dev(key_sel), validity=dev(vw), row_sel=dev(row_sel))
    assert np.array_equal(got.cpu().numpy().view(np.uint32), exp)
    bf.close()
