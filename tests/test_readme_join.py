"""BASELINE config C1, the reference README's example (README.md:60-75), through the HIP path:

    CREATE TEMP TABLE t1 AS SELECT i AS id FROM range(100000) tbl(i);
    CREATE TEMP TABLE t2 AS SELECT i AS id FROM range(50000) tbl(i);
    SELECT count(*) FROM t1 JOIN t2 ON t1.id = t2.id;   -- returns 50000

`range` yields BIGINT ids. Predicate transfer builds a filter on one side's join key (CREATE_BF) and
probes the other side with it (USE_BF) before the join; the query result must not change. Here both
transfer directions run on cuda:0 in DuckDB-sized 2048-row vectors; the surviving rows must equal
the oracle's, must keep every row that has a join partner, and the hash join of the survivors must
return the README's 50000. (DuckDB itself is absent from the image: the join is numpy's.)
"""
import numpy as np
import pytest
import torch

import rpt_oracle as orc

VECTOR = 2048  # STANDARD_VECTOR_SIZE


@pytest.fixture(scope="module")
def rpt():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    import rpt_amd

    rpt_amd.load()
    torch.cuda.set_device(0)
    return rpt_amd


def transfer(rpt, build_ids: np.ndarray, probe_ids: np.ndarray) -> np.ndarray:
    """CREATE_BF over build_ids, then USE_BF over probe_ids vector by vector: surviving probe row ids."""
    bf = rpt.BloomFilter(len(build_ids), device="cuda:0")
    for lo in range(0, len(build_ids), VECTOR):  # PhysicalCreateBF::Sink, one vector at a time
        bf.insert(torch.from_numpy(build_ids[lo:lo + VECTOR]).cuda())
    bf.finalized = True
    lnb = orc.log_num_blocks(len(build_ids))
    words = orc.new_words(lnb)
    orc.insert_keys(words, lnb, build_ids)
    assert np.array_equal(bf.export_words(), words)
    keep = []
    for lo in range(0, len(probe_ids), VECTOR):  # PhysicalUseBF::ExecuteInternal per vector
        chunk = probe_ids[lo:lo + VECTOR]
        sel = bf.lookup_sel(torch.from_numpy(chunk).cuda()).cpu().numpy().view(np.uint32)
        assert np.array_equal(sel, orc.probe_keys(words, lnb, chunk)), f"vector at row {lo}"
        keep.append(sel.astype(np.int64) + lo)
    bf.close()
    return np.concatenate(keep)


def oracle_transfer(build_ids: np.ndarray, probe_ids: np.ndarray) -> np.ndarray:
    lnb = orc.log_num_blocks(len(build_ids))
    words = orc.new_words(lnb)
    orc.insert_keys(words, lnb, build_ids)
    return orc.probe_keys(words, lnb, probe_ids).astype(np.int64)


def test_readme_join_oracle():
    """The same transfer through the CPU restatement alone (no GPU)."""
    t1 = np.arange(100000, dtype=np.int64)
    t2 = np.arange(50000, dtype=np.int64)
    s1, s2 = oracle_transfer(t2, t1), oracle_transfer(t1, t2)
    assert np.isin(np.arange(50000), s1).all() and np.array_equal(s2, np.arange(50000))
    assert 50000 <= s1.size < 100000  # false positives only among t1's unmatched half
    assert np.intersect1d(t1[s1], t2[s2]).size == 50000


@pytest.mark.gpu
def test_readme_join_both_directions(rpt):
    t1 = np.arange(100000, dtype=np.int64)
    t2 = np.arange(50000, dtype=np.int64)
    # filter from t2 applied to t1: every t1 row with a partner survives, a few false positives too
    s1 = transfer(rpt, t2, t1)
    assert np.isin(np.arange(50000), s1).all()
    # filter from t1 applied to t2: every t2 row has a partner
    s2 = transfer(rpt, t1, t2)
    assert np.array_equal(s2, np.arange(50000))
    # the join over the transferred inputs returns the README's count
    assert np.intersect1d(t1[s1], t2[s2]).size == 50000
