"""rpt_bf_clear defers its zeroing to the next operation on the filter (rpt_bf::clear_pending): a
partitioned / bucketed insert whose slice merge owns every slice stores the slices whole (zeros
included), every other operation zeroes the words first. Each case fills the filter with keys A, clears
it, then runs one operation: the result must equal the oracle's for an EMPTY filter followed by that
operation (no bit of A survives), and the filter must keep composing with later inserts. Bit-exact."""
import numpy as np
import pytest
import torch

import rpt_oracle as orc

pytestmark = pytest.mark.gpu

GATHER, PARTITIONED, BUCKETED = 1, 3, 4
INS_ATOMIC, INS_PARTITIONED, INS_BUCKETED = 1, 2, 3


@pytest.fixture(scope="module")
def rpt():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    import rpt_amd

    rpt_amd.load()
    torch.cuda.set_device(0)
    return rpt_amd


def dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def keys(n, seed):
    return np.random.default_rng(seed).integers(-(2**62), 2**62, size=n, dtype=np.int64)


def filled(rpt, log_nb, seed=1, n=300_000):
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys(n, seed)))
    assert bf.count_bits() > 0
    return bf


# (insert strategy, log_num_blocks): 2^21 = 128 slices (two slice workgroups per slice: zeroed first, then
# atomic merges), 2^24 = 1024 slices and the bucketed filters (one workgroup per slice: whole-slice
# stores), the atomic insert (zeroed first)
CASES = [(INS_PARTITIONED, 21), (INS_PARTITIONED, 24), (INS_BUCKETED, 22), (INS_BUCKETED, 25), (INS_ATOMIC, 22)]


@pytest.mark.parametrize("strategy,log_nb", CASES)
@pytest.mark.parametrize("n_b", [1_000, 2_000_000])
def test_clear_then_insert_vs_oracle(rpt, strategy, log_nb, n_b):
    """1000 keys leave most slices without a record (their slices must still be zeroed), 2e6 fill them."""
    bf = filled(rpt, log_nb)
    bf.clear()
    b, c = keys(n_b, 2), keys(50_000, 3)
    bf.insert(dev(b), strategy=strategy)
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, b)
    assert np.array_equal(bf.export_words(), w)
    assert bf.minmax() == (int(b.min()), int(b.max()))
    bf.insert(dev(c), strategy=strategy)  # no longer pristine: the adaptive / atomic merges
    orc.insert_keys(w, log_nb, c)
    assert np.array_equal(bf.export_words(), w)
    probe = np.concatenate([b[:20_000], keys(20_000, 4), c[:1000]])
    assert np.array_equal(bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32), orc.probe_keys(w, log_nb, probe))


@pytest.mark.parametrize("strategy", [GATHER, PARTITIONED, BUCKETED])
def test_clear_then_probe_finds_nothing(rpt, strategy):
    bf = filled(rpt, 22)
    a = keys(300_000, 1)
    bf.clear()
    bf.probe_strategy = strategy
    assert bf.lookup_sel(dev(a)).numel() == 0
    assert bf.export_words().sum() == 0
    bf2 = filled(rpt, 22)
    bf2.clear()
    assert not bf2.find_bits(dev(a)).any()
    bf3 = filled(rpt, 14)
    bf3.clear()
    assert bf3.lookup_sel(dev(a[:1000])).numel() == 0  # small batch: the fused probe


def test_clear_then_readers_and_merges(rpt):
    log_nb = 22
    other = filled(rpt, log_nb, seed=7)
    ref = other.export_words()
    # copy out, count, fold
    bf = filled(rpt, log_nb)
    bf.clear()
    out = torch.full((1 << log_nb,), -1, dtype=torch.int64, device="cuda:0")
    bf.copy_words_to(out)
    torch.cuda.synchronize()
    assert not out.any()
    bf = filled(rpt, log_nb)
    bf.clear()
    assert bf.count_bits() == 0
    bf = filled(rpt, log_nb)
    bf.clear()
    bf.fold()
    assert bf.export_words().sum() == 0
    # merge into a cleared filter, merge a cleared filter in
    bf = filled(rpt, log_nb)
    bf.clear()
    bf.merge_or(other)
    assert np.array_equal(bf.export_words(), ref)
    src = filled(rpt, log_nb, seed=9)
    src.clear()
    dst = filled(rpt, log_nb, seed=7)
    dst.merge_or(src)
    assert np.array_equal(dst.export_words(), ref)
    # copy in / import overwrite every word: nothing left to zero afterwards
    bf = filled(rpt, log_nb)
    bf.clear()
    bf.copy_words_from(torch.from_numpy(ref.view(np.int64)).to("cuda:0"))
    bf.insert(dev(keys(1000, 11)), strategy=INS_BUCKETED)
    w = ref.copy()
    orc.insert_keys(w, log_nb, keys(1000, 11))
    assert np.array_equal(bf.export_words(), w)
    bf = filled(rpt, log_nb)
    bf.clear()
    bf.import_words(ref)
    assert np.array_equal(bf.export_words(), ref)


def test_clear_twice_and_cross_stream(rpt):
    """Clear on one stream, rebuild on another (the insert waits for the clear's ordered write), clear
    twice in a row, and clear an already-empty filter."""
    log_nb = 25
    bf = filled(rpt, log_nb)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    b = keys(1_000_000, 5)
    db = dev(b)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(50_000_000)  # hold s1 back: the clear's stats reset runs late
    bf.clear(stream=s1)
    bf.clear(stream=s1)
    bf.insert(db, strategy=INS_BUCKETED, stream=s2)
    torch.cuda.synchronize()
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, b)
    assert np.array_equal(bf.export_words(), w)
    # the insert's min/max (folded in by its first kernels) landed after the clear's reset
    assert bf.minmax() == orc.minmax(b)
    e = rpt.BloomFilter(log_num_blocks=log_nb)
    e.clear()
    e.insert(db, strategy=INS_BUCKETED)
    assert np.array_equal(e.export_words(), w)


@pytest.mark.parametrize("strategy", [INS_PARTITIONED, INS_BUCKETED])
def test_minmax_ordered_after_cross_stream_clear(rpt, strategy):
    """after a clear enqueued on a delayed stream, an insert on another stream must fold its
    key min/max in after the clear's stats reset (partitioned and bucketed inserts fold them in their
    first kernels, before the slice merge takes the write order), and a merge's stats update stays
    inside its write order."""
    log_nb = 24
    bf = filled(rpt, log_nb)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    b = keys(2_000_000, 11)
    db = dev(b)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(50_000_000)
    bf.clear(stream=s1)
    bf.insert(db, strategy=strategy, stream=s2)
    torch.cuda.synchronize()
    assert bf.minmax() == orc.minmax(b)
    # merge_or: dst cleared on a delayed stream, then merged from src on another stream
    src = rpt.BloomFilter(log_num_blocks=log_nb)
    src.insert(db, strategy=strategy)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(50_000_000)
    bf.clear(stream=s1)
    bf.merge_or(src, stream=s2)
    torch.cuda.synchronize()
    assert bf.minmax() == orc.minmax(b)
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, b)
    assert np.array_equal(bf.export_words(), w)


def test_clear_settled_by_a_reader_orders_other_streams(rpt):
    """the first reader after a clear zeroes the words on ITS stream without a host sync; a
    reader on another stream that finds the clear settled must wait for that zeroing (an event), not
    read the old words."""
    bf = filled(rpt, 22)
    da = dev(keys(300_000, 1))
    out = torch.full((1 << 22,), -1, dtype=torch.int64, device="cuda:0")
    bf.clear()
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):
        torch.cuda._sleep(50_000_000)  # the zeroing enqueued on s1 runs late
    _sel, cnt = bf.probe_async(da, stream=s1)
    bf.copy_words_to(out, stream=s2)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    assert not out.any()
