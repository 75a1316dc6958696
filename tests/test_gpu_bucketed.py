"""Bucketed (two-level) strategy for filters > 128 MiB, on the HIP path vs the oracle and vs the other
strategies. Bit-exact. Filters of 2^22..2^23 blocks (32/64 MiB) are used where the partitioned
strategy also applies, so both can be compared on the same filter; 2^25 (256 MiB) exercises the AUTO
choice at a size only the bucketed strategy routes."""
import numpy as np
import pytest
import torch

import golden_util as gu
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
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def keys_of(dtype, n, seed):
    rng = np.random.default_rng(seed)
    info = np.iinfo(dtype)
    return rng.integers(info.min, info.max, size=n, dtype=dtype, endpoint=True)


def oracle_filter(log_nb, keys, **kw):
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, keys, **kw)
    return w


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("log_nb,n_build,n_probe", [(22, 300_000, 1), (22, 300_000, 100_003), (23, 2_000_000, 1_000_000)])
def test_bucketed_probe_vs_oracle(rpt, dtype, log_nb, n_build, n_probe):
    build = keys_of(dtype, n_build, log_nb)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(build), strategy=INS_ATOMIC)
    w = oracle_filter(log_nb, build)
    assert np.array_equal(bf.export_words(), w)
    rng = np.random.default_rng(n_probe)
    probe = np.where(rng.random(n_probe) < 0.3, build[rng.integers(0, n_build, n_probe)], keys_of(dtype, n_probe, 5))
    probe = probe.astype(dtype)
    ref = orc.probe_keys(w, log_nb, probe)
    for st in (BUCKETED, PARTITIONED, GATHER):
        bf.probe_strategy = st
        assert bf.probe_strategy_for(n_probe) == st
        sel = bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32)
        assert np.array_equal(sel, ref), f"strategy {st}"


def test_bucketed_probe_nulls_dictionary_rowsel(rpt):
    log_nb, n = 22, 400_000
    build = keys_of(np.int64, 200_000, 1)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(build))
    w = oracle_filter(log_nb, build)
    rng = np.random.default_rng(2)
    dict_keys = np.concatenate([build[:50_000], keys_of(np.int64, 50_000, 3)])
    valid = rng.random(dict_keys.size) > 0.2
    vw = gu.validity_words(valid)
    key_sel = rng.integers(0, dict_keys.size, n).astype(np.uint32)
    row_sel = np.sort(rng.choice(n, size=n // 3, replace=False)).astype(np.uint32)
    # oracle: the dictionary vector sliced by row_sel
    ref_rows = orc.probe_keys(w, log_nb, dict_keys, key_sel=np.ascontiguousarray(key_sel[row_sel]), validity=vw)
    ref = row_sel[ref_rows]
    bf.probe_strategy = BUCKETED
    sel = bf.lookup_sel(dev(dict_keys), key_sel=dev(key_sel), validity=dev(vw), row_sel=dev(row_sel)).cpu().numpy()
    assert np.array_equal(sel.astype(np.uint32), ref)


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [1, 5_000, 1_200_000])
def test_bucketed_insert_vs_oracle(rpt, dtype, n):
    log_nb = 22
    keys = keys_of(dtype, n, n + 7)
    valid = np.random.default_rng(n).random(n) > 0.05
    vw = gu.validity_words(valid)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys), validity=dev(vw), strategy=INS_BUCKETED)
    assert np.array_equal(bf.export_words(), oracle_filter(log_nb, keys, validity=vw))
    assert bf.minmax() == orc.minmax(keys, validity=vw)
    # a second insert into the same filter ORs (thread-safe merge of the slices)
    more = keys_of(dtype, 1000, 99)
    bf.insert(dev(more), strategy=INS_BUCKETED)
    w = oracle_filter(log_nb, keys, validity=vw)
    orc.insert_keys(w, log_nb, more)
    assert np.array_equal(bf.export_words(), w)


def test_auto_routes_large_filters(rpt):
    """2^25 blocks (256 MiB): AUTO picks the bucketed insert from 8 Mi rows and the bucketed probe from
    32 Mi rows, the atomic insert / gather below; the chosen paths give the oracle's bits and survivors."""
    log_nb = 25
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    assert bf.insert_strategy_for(1 << 23) == INS_BUCKETED and bf.insert_strategy_for(1 << 21) == INS_ATOMIC
    assert bf.probe_strategy_for(1 << 25) == BUCKETED and bf.probe_strategy_for(10**7) == GATHER
    tiny = rpt.BloomFilter(log_num_blocks=14)  # 128 KiB: the whole filter in each CU's LDS
    assert tiny.probe_strategy_for(1 << 28) == 2 and tiny.probe_strategy_for(1 << 16) == 2
    small = rpt.BloomFilter(log_num_blocks=15)  # 256 KiB (512 KiB too): the hybrid LDS probe at any size
    assert small.probe_strategy_for(1 << 24) == 2 and small.probe_strategy_for(1 << 28) == 2
    small17 = rpt.BloomFilter(log_num_blocks=17)  # 1 MiB: gathers below 4 Mi rows, the hybrid to 32 Mi, routed above
    assert small17.probe_strategy_for(1 << 21) == GATHER and small17.probe_strategy_for(1 << 24) == 2
    assert small17.probe_strategy_for(1 << 28) == PARTITIONED
    small17.close()
    mid19 = rpt.BloomFilter(log_num_blocks=19)  # 4 MiB: routed from 4 Mi rows
    assert mid19.probe_strategy_for(1 << 22) == PARTITIONED and mid19.probe_strategy_for(1 << 21) == GATHER
    mid = rpt.BloomFilter(log_num_blocks=21)  # 16 MiB (C2): routed from 4 Mi rows
    assert mid.probe_strategy_for(1 << 22) == PARTITIONED and mid.probe_strategy_for(1 << 21) == GATHER
    # partitioned inserts from 2 Mi rows, 4 Mi above 128 slices (profiles/r03/strategy_crossover_insert.jsonl)
    assert mid.insert_strategy_for(1 << 21) == INS_PARTITIONED and mid.insert_strategy_for(1 << 20) == INS_ATOMIC
    assert tiny.insert_strategy_for(1 << 21) == INS_PARTITIONED and tiny.insert_strategy_for((1 << 21) - 1) == INS_ATOMIC
    big = rpt.BloomFilter(log_num_blocks=24)  # 128 MiB, 1024 slices
    assert big.insert_strategy_for(1 << 22) == INS_PARTITIONED and big.insert_strategy_for(1 << 21) == INS_ATOMIC
    big.close()
    n_build = 5_000_000
    build = keys_of(np.int64, n_build, 11)
    bf.insert(dev(build))  # AUTO: atomic at this batch size
    w = oracle_filter(log_nb, build)
    assert np.array_equal(bf.export_words(), w)
    bf.insert(dev(build), strategy=INS_BUCKETED)  # re-inserting changes nothing
    assert np.array_equal(bf.export_words(), w)
    rng = np.random.default_rng(12)
    n_probe = 6_000_000
    probe = np.where(rng.random(n_probe) < 0.1, build[rng.integers(0, n_build, n_probe)], keys_of(np.int64, n_probe, 13))
    ref = orc.probe_keys(w, log_nb, probe)
    for st in (0, BUCKETED):  # AUTO (gather here) and the bucketed path
        bf.probe_strategy = st
        sel = bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32)
        assert np.array_equal(sel, ref)


def test_bucketed_skewed_keys(rpt):
    """Every key in one bucket (and one slice): the level-2 array is a single padded bucket."""
    log_nb = 22
    base = keys_of(np.int64, 20_000, 21)
    h = orc.hash_keys(base)
    same = base[(h >> np.uint64(37)) & np.uint64(1) == 0][:5000]  # all keys of bucket 0
    keys = np.repeat(same, 200)  # 1e6 rows, heavy duplicates
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys), strategy=INS_BUCKETED)
    w = oracle_filter(log_nb, keys)
    assert np.array_equal(bf.export_words(), w)
    bf.probe_strategy = BUCKETED
    probe = np.concatenate([keys, base])
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe))


def keys_in_bucket(log_nb, bucket, count, seed):
    """`count` distinct int64 keys whose hashes fall in level-1 bucket `bucket` (hash bits 38..)."""
    nb = 1 << (log_nb - 22)
    cand = keys_of(np.int64, count * nb * 4, seed)
    h = orc.hash_keys(cand)
    sel = cand[((h >> np.uint64(38)) & np.uint64(nb - 1)) == bucket][:count]
    assert sel.size == count
    return sel


@pytest.mark.parametrize("log_nb,n,frac", [(25, 2_000_000, 1.0), (25, 3_000_017, 0.6), (27, 5_000_000, 0.9)])
def test_bucketed_list_overflow(rpt, log_nb, n, frac):
    """Rows crowding into one bucket (bucketed.hpp): its list outgrows its fixed chunks and grows by pool
    extents -- runs of whole 16 Ki-row tiles spanning several chunks, runs starting inside extents other
    tiles took. Insert (filter words) and probe (sel) vs the oracle."""
    rng = np.random.default_rng(n)
    hot = keys_in_bucket(log_nb, 3, 4000, log_nb)
    keys = np.where(rng.random(n) < frac, hot[rng.integers(0, hot.size, n)], keys_of(np.int64, n, 7))
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys), strategy=INS_BUCKETED)
    w = oracle_filter(log_nb, keys)
    assert np.array_equal(bf.export_words(), w)
    assert bf.minmax() == orc.minmax(keys)
    bf.probe_strategy = BUCKETED
    probe = np.where(rng.random(n) < frac, hot[rng.integers(0, hot.size, n)], keys_of(np.int64, n, 8))
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe))


@pytest.mark.timeout(300)
def test_bucketed_grouped_lists_skewed(rpt):
    """A batch of >= 2^27 rows takes 8 list groups per bucket (one per XCD share); 40 % of its rows in one
    of 16 buckets, so that bucket's 8 lists overflow while the others stay within their fixed chunks.
    Insert and probe vs the oracle, every word and sel entry."""
    log_nb, n = 26, (1 << 27) + 12_345
    rng = np.random.default_rng(26)
    hot = keys_in_bucket(log_nb, 11, 3000, 99)
    keys = orc.synth_build_keys(n, start=10**9)
    m = rng.random(n) < 0.4
    keys[m] = hot[rng.integers(0, hot.size, int(m.sum()))]
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys), strategy=INS_BUCKETED)
    w = oracle_filter(log_nb, keys)
    assert np.array_equal(bf.export_words(), w)
    bf.probe_strategy = BUCKETED
    probe = orc.synth_probe_keys(n, n, 10, start=2 * 10**9)
    probe[m] = keys[m]
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32)
    ref = orc.probe_keys(w, log_nb, probe)
    assert ref.size >= int(m.sum())
    assert np.array_equal(sel, ref)


def test_c5_geometry_8gib_filter_vs_oracle(rpt):
    """BASELINE C5's single-rank geometry: a filter sized for 8e9 rows = 2^30 blocks
    (8 GiB), 256 level-1 buckets of 256 slices. Bucketed insert of 1.2e7 keys and bucketed probes of
    1.2e7 rows (flat, with a NULL pattern, through a row selection), each against the oracle: every word
    of the 8 GiB filter and every sel entry."""
    log_nb = 30
    bf = rpt.BloomFilter(8 * 10**9)
    assert bf.log_num_blocks == log_nb
    n_build, n_probe = 12_000_000, 12_000_000
    build = orc.synth_build_keys(n_build, start=3 * 10**9)
    bf.insert(dev(build), strategy=INS_BUCKETED)
    w = oracle_filter(log_nb, build)
    got = torch.empty(bf.num_blocks, dtype=torch.int64, device="cuda:0")
    bf.copy_words_to(got)
    ref_words = torch.from_numpy(w.view(np.int64)).to("cuda:0")
    assert torch.equal(got, ref_words), "8 GiB filter words differ from the oracle"
    del got, ref_words
    torch.cuda.empty_cache()
    assert bf.minmax() == orc.minmax(build)

    probe = orc.synth_probe_keys(n_probe, n_build, 100, start=5 * 10**8)
    probe[::7] = build[: probe[::7].size]  # more hits than p = 0.1
    bf.probe_strategy = BUCKETED
    assert bf.probe_strategy_for(n_probe) == BUCKETED
    dprobe = dev(probe)
    ref = orc.probe_keys(w, log_nb, probe)
    assert ref.size > n_probe // 7
    assert np.array_equal(bf.lookup_sel(dprobe).cpu().numpy().astype(np.uint32), ref)
    rng = np.random.default_rng(30)
    valid = rng.random(n_probe) > 0.01
    vw = gu.validity_words(valid)
    ref_n = orc.probe_keys(w, log_nb, probe, validity=vw)
    sel_n = bf.lookup_sel(dprobe, validity=dev(vw)).cpu().numpy().astype(np.uint32)
    assert np.array_equal(sel_n, ref_n)
    row_sel = np.sort(rng.choice(n_probe, size=n_probe // 3, replace=False)).astype(np.uint32)
    ref_r = row_sel[orc.probe_keys(w, log_nb, probe, key_sel=row_sel)]
    sel_r = bf.lookup_sel(dprobe, row_sel=dev(row_sel)).cpu().numpy().astype(np.uint32)
    assert np.array_equal(sel_r, ref_r)


@pytest.mark.timeout(300)
def test_max_bucketed_geometry_16gib_vs_oracle(rpt):
    """The largest filter the bucketed strategy takes: 2^31 blocks (16 GiB), 512 level-1 buckets. A
    rebuild (clear, then a bucketed insert that stores every slice whole) of 2e7 keys and a bucketed
    probe of 2e7 rows, against the oracle: every filter word and every sel entry."""
    log_nb = 31
    from rpt_amd import _lib

    assert _lib.load().rpt_probe_strategy_supported(BUCKETED, log_nb) == 1
    assert _lib.load().rpt_probe_strategy_supported(BUCKETED, log_nb + 1) == 0
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    n_build, n_probe = 20_000_000, 20_000_000
    bf.insert(dev(orc.synth_build_keys(1000, start=7 * 10**9)))  # then rebuilt: nothing of it may survive
    bf.clear()
    build = orc.synth_build_keys(n_build, start=9 * 10**9)
    bf.insert(dev(build), strategy=INS_BUCKETED)
    w = oracle_filter(log_nb, build)
    got = torch.empty(bf.num_blocks, dtype=torch.int64, device="cuda:0")
    bf.copy_words_to(got)
    assert torch.equal(got, torch.from_numpy(w.view(np.int64)).to("cuda:0")), "16 GiB filter words differ"
    del got
    torch.cuda.empty_cache()
    probe = orc.synth_probe_keys(n_probe, n_build, 300, start=11 * 10**9)
    probe[::5] = build[: probe[::5].size]
    bf.probe_strategy = BUCKETED
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32)
    ref = orc.probe_keys(w, log_nb, probe)
    assert ref.size > n_probe // 5
    assert np.array_equal(sel, ref)


@pytest.mark.parametrize("strategy", [INS_PARTITIONED, INS_BUCKETED])
def test_slice_merge_modes_vs_oracle(rpt, strategy):
    """The slice insert's merges into a 2^22-block filter (256 slices, one workgroup each): plain stores
    into the pristine filter, read-modify-write of slices receiving >= 8192 records, atomic ORs for a
    small insert, and two large inserts racing on two streams from two host threads (the filter orders
    its word writes): every word equals the oracle's."""
    import threading

    log_nb = 22
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    a, b, c = (keys_of(np.int64, n, seed) for n, seed in ((3_000_000, 41), (3_000_000, 42), (1000, 43)))
    w = orc.new_words(log_nb)
    for keys in (a, b, c):  # pristine -> stores; ~11.7k records per slice -> RMW; 1000 keys -> atomics
        bf.insert(dev(keys), strategy=strategy)
        orc.insert_keys(w, log_nb, keys)
        assert np.array_equal(bf.export_words(), w)
    bf.clear()
    assert bf.export_words().sum() == 0
    da, db = dev(a), dev(b)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    threads = [threading.Thread(target=bf.insert, args=(k,), kwargs=dict(strategy=strategy, stream=st))
               for k, st in zip((da, db), streams)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    torch.cuda.synchronize()
    w2 = orc.new_words(log_nb)
    orc.insert_keys(w2, log_nb, a)
    orc.insert_keys(w2, log_nb, b)
    assert np.array_equal(bf.export_words(), w2)
