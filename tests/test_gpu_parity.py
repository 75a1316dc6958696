"""HIP path (librpt_gpu.so on cuda:0) vs the oracle and the Arrow golden vectors. Bit-exact."""
import os

import numpy as np
import pytest
import torch

import golden_util as gu
import rpt_oracle as orc

pytestmark = pytest.mark.gpu

STRATEGIES = {"gather": 1, "lds": 2, "partitioned": 3}


def supported(strategy: str, log_num_blocks: int) -> bool:
    from rpt_amd import _lib

    return bool(_lib.load().rpt_probe_strategy_supported(STRATEGIES[strategy], log_num_blocks))


def with_strategy(bf, strategy: str):
    if not supported(strategy, bf.log_num_blocks):
        pytest.skip(f"{strategy} does not apply to a 2^{bf.log_num_blocks}-block filter")
    bf.probe_strategy = STRATEGIES[strategy]
    assert bf.probe_strategy == STRATEGIES[strategy]
    return bf


KEY_CASES = ["kat16", "raw_hash_100k", "k64_n1", "k64_n100", "k64_n1000", "k64_n50000", "k64_n300000",
             "k32_n5000", "k64_n3000_nulls7", "k32_n3000_nulls5", "k64_n20000_over"]


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


def bits_of(words: torch.Tensor, n: int) -> np.ndarray:
    w = words.cpu().numpy().view(np.uint64)
    return np.unpackbits(w.view(np.uint8), bitorder="little")[:n].astype(bool)


@pytest.mark.parametrize("strategy", list(STRATEGIES))
@pytest.mark.parametrize("case", KEY_CASES)
def test_golden_hash_path(rpt, golden, case, strategy):
    c = golden.cases[case]
    h, p, _ = golden.inputs(case)
    bf = with_strategy(rpt.BloomFilter(log_num_blocks=c["log_num_blocks"]), strategy)
    bf.insert(dev(h), key_type=rpt.RPT_KEY_HASH)
    torch.cuda.synchronize()
    assert np.array_equal(bf.export_words(), golden.words(case))
    assert bf.count_bits() == c["num_bits_set"]
    ref = golden.find_bits(case, p.size)
    assert np.array_equal(bits_of(bf.find_bits(dev(p), key_type=rpt.RPT_KEY_HASH), p.size), ref)
    sel = bf.lookup_sel(dev(p), key_type=rpt.RPT_KEY_HASH).cpu().numpy()
    assert np.array_equal(sel, np.flatnonzero(ref).astype(np.int32))


@pytest.mark.parametrize("strategy", list(STRATEGIES))
@pytest.mark.parametrize("case", [k for k in KEY_CASES if k.startswith("k") and k != "kat16"])
def test_golden_key_path(rpt, golden, case, strategy):
    c = golden.cases[case]
    _, _, kc = golden.inputs(case)
    bf = with_strategy(rpt.BloomFilter(kc.size_rows), strategy)
    assert bf.log_num_blocks == c["log_num_blocks"]
    v = dev(gu.validity_words(kc.valid)) if kc.valid is not None else None
    bf.insert(dev(kc.keys), validity=v)
    assert np.array_equal(bf.export_words(), golden.words(case))
    pv = dev(gu.validity_words(kc.probe_valid)) if kc.probe_valid is not None else None
    sel = bf.lookup_sel(dev(kc.probe), validity=pv).cpu().numpy()
    assert np.array_equal(sel, np.flatnonzero(golden.find_bits(case, kc.probe.size)).astype(np.int32))
    assert np.array_equal(rpt.hash_keys(dev(kc.probe), validity=pv).cpu().numpy().view(np.uint64),
                          kc.hashes(kc.probe, kc.probe_valid))


@pytest.mark.parametrize("case", ["fold_200k_dup1000", "fold_100k_3keys", "fold_dense_noop"])
def test_golden_fold(rpt, golden, case):
    c = golden.cases[case]
    h, p, _ = golden.inputs(case)
    bf = rpt.BloomFilter(golden.size_rows(case))
    bf.insert(dev(h), key_type=rpt.RPT_KEY_HASH)
    assert bf.fold() == c["log_num_blocks"]
    assert np.array_equal(bf.export_words(), golden.words(case))
    if p is not None:
        assert np.array_equal(bits_of(bf.find_bits(dev(p), key_type=rpt.RPT_KEY_HASH), p.size),
                              golden.find_bits(case, p.size))


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [0, 1, 7, 511, 512, 513, 2048, 100003])
def test_ragged_sizes_vs_oracle(rpt, dtype, n):
    rng = np.random.default_rng(n + (dtype == np.int32))
    build = rng.integers(-2**31, 2**31, size=max(n // 3, 1), dtype=np.int64).astype(dtype)
    probe = np.concatenate([build[: n // 2], rng.integers(-2**31, 2**31, size=n - n // 2).astype(dtype)])
    rng.shuffle(probe)
    lnb = orc.log_num_blocks(build.size)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, build)
    bf = rpt.BloomFilter(build.size)
    bf.insert(dev(build))
    assert np.array_equal(bf.export_words(), w)
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32) if n else np.zeros(0, np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, lnb, probe))


@pytest.mark.parametrize("strategy", list(STRATEGIES))
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [1, 16383, 16384, 16385, 3 * 16384 + 5, 200001])
def test_partition_tile_edges_vs_oracle(rpt, strategy, dtype, n):
    """Filters large enough for the partitioned path (2^17 blocks), ragged tile boundaries."""
    rng = np.random.default_rng(n)
    build = rng.integers(-2**40, 2**40, size=100000, dtype=np.int64).astype(dtype)
    probe = np.concatenate([build[rng.integers(0, build.size, size=n // 3)],
                            rng.integers(-2**40, 2**40, size=n - n // 3).astype(dtype)])
    lnb = orc.log_num_blocks(build.size)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, build)
    bf = with_strategy(rpt.BloomFilter(build.size), strategy)
    bf.insert(dev(build))
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, lnb, probe))


@pytest.mark.parametrize("strategy", ["gather", "partitioned"])
@pytest.mark.parametrize("log_nb", [21, 22, 24])
def test_large_filters_vs_oracle(rpt, strategy, log_nb):
    """16 MiB .. 128 MiB filters (256 .. 1024 LDS slices; BASELINE C3 uses 2^24 blocks)."""
    build = orc.synth_build_keys(300000)
    probe = orc.synth_probe_keys(1_000_003, 300000, 300)
    bf = with_strategy(rpt.BloomFilter(log_num_blocks=log_nb), strategy)
    bf.insert(dev(build))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, build)
    assert np.array_equal(bf.export_words(), w)
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe))


@pytest.mark.parametrize("log_nb", [18, 21, 24])
@pytest.mark.parametrize("hot", [0.0, 0.02, 0.3, 1.0])
def test_skewed_probe_keys_vs_oracle(rpt, log_nb, hot):
    """Probe keys skewed onto a few slices (a fraction `hot` of the rows on one key, a tenth of that on a second,
    in and out of the filter): the partitioned probe then gives the overloaded slices finer work items
    (rpt::SkewItems); the selection vector must stay the oracle's, over ragged tiles and repeated calls."""
    rng = np.random.default_rng(int(hot * 100) + log_nb)
    build = orc.synth_build_keys(200000)
    n = 6 * 32768 + 777
    probe = orc.synth_probe_keys(n, 200000, 300).copy()
    u = rng.random(n)
    probe[u < hot] = build[4242]
    probe[(u >= hot) & (u < hot * 1.1)] = -99
    bf = with_strategy(rpt.BloomFilter(log_num_blocks=log_nb), "partitioned")
    bf.insert(dev(build))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, build)
    want = orc.probe_keys(w, log_nb, probe)
    for _ in range(2):
        sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
        assert np.array_equal(sel, want)


def _skewed_column(rpt, n, n_build, hot, hot_key, miss_share=0.1, seed=1):
    """n synthetic probe keys (p = 0.1) on the device with a fraction `hot` of the rows replaced by hot_key and
    a further hot * miss_share by a key that is in no filter (-99): the shape of a foreign-key column's hot
    values (physical_use_bf.cpp:163 probes whatever the column holds)."""
    probe = rpt.synth_probe_keys(n, n_build, 100)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    u = torch.rand(n, device="cuda:0", generator=g)
    probe[u < hot] = hot_key
    probe[(u >= hot) & (u < hot * (1 + miss_share))] = -99
    del u
    return probe


@pytest.mark.timeout(300)
@pytest.mark.parametrize("log_nb,n_build", [(21, 10**7), (24, 10**8)])
@pytest.mark.parametrize("hot", [0.1, 1.0])
def test_full_size_skewed_probe_vs_oracle(rpt, log_nb, n_build, hot):
    """one hot key on 10 % / 100 % of 2^27 + 777 probe rows against C2's 16 MiB (2^21 blocks)
    and C3's 128 MiB (2^24) filters, AUTO strategy (partitioned: 2^13 tiles, the hot slice stamped and split into
    the 32x finer skew items), every row against the oracle, twice (the second call's stamps are fresh)."""
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    n = 2**27 + 777
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    build = rpt.synth_build_keys(n_build)
    bf.insert(build)
    hot_key = int(build[4242].item())
    del build
    assert bf.probe_strategy_for(n) == 3  # partitioned
    ow = orc.new_words(log_nb)
    orc.build_mt(ow, log_nb, orc.synth_build_keys(n_build), threads)
    probe = _skewed_column(rpt, n, n_build, hot, hot_key)
    for _ in range(2):
        sel_t, cnt = bf.probe_async(probe)
        count = int(cnt.item())
        sel = sel_t[:count].cpu().numpy().astype(np.int64)
        del sel_t
        assert np.all(sel[1:] > sel[:-1])
        _full_check(ow, log_nb, probe, sel, piece=1 << 24)
        assert count >= int(hot * n * 0.99)
    del probe
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("hot", [0.5, 1.0])
def test_full_size_hot_bucket_vs_oracle(rpt, hot):
    """The bucketed strategy with one level-1 bucket (32 MiB filter region) holding half / all of 2^27 + 777 rows
    (one hot key): its chunk lists grow through the extent pool far past an even split; every row against the
    oracle (a hit on the bound would degrade to every row passing, and fail here)."""
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    log_nb, n_build, n = 26, 10**7, 2**27 + 777
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.probe_strategy = 4  # bucketed
    build = rpt.synth_build_keys(n_build)
    bf.insert(build)
    hot_key = int(build[777].item())
    del build
    ow = orc.new_words(log_nb)
    orc.build_mt(ow, log_nb, orc.synth_build_keys(n_build), threads)
    probe = _skewed_column(rpt, n, n_build, hot, hot_key, seed=2)
    sel_t, cnt = bf.probe_async(probe)
    count = int(cnt.item())
    sel = sel_t[:count].cpu().numpy().astype(np.int64)
    del sel_t
    assert np.all(sel[1:] > sel[:-1])
    _full_check(ow, log_nb, probe, sel, piece=1 << 24)
    assert count < n or hot == 1.0
    del probe
    torch.cuda.empty_cache()


@pytest.mark.parametrize("log_nb,n", [(4, 10), (14, 100_000), (21, 3_000_000), (27, 2_000_000)])
def test_is_same_as_on_device(rpt, log_nb, n):
    """rpt_bf_is_same_as (Arrow BlockedBloomFilter::IsSameAs): equal builds compare equal; one extra key, a cleared
    filter and a different geometry do not; the differing-word count equals the host comparison's."""
    k = orc.synth_build_keys(n)
    a, b = rpt.BloomFilter(log_num_blocks=log_nb), rpt.BloomFilter(log_num_blocks=log_nb)
    a.insert(dev(k))
    b.insert(dev(k[::-1].copy()))
    assert a.is_same_as(b) and b.is_same_as(a) and a.diff_words(b) == 0
    b.insert(dev(np.array([-12345], dtype=np.int64)))
    assert not a.is_same_as(b)
    assert a.diff_words(b) == int((a.export_words() != b.export_words()).sum()) >= 1
    b.clear()  # deferred clear: the comparison settles it first
    assert b.diff_words(rpt.BloomFilter(log_num_blocks=log_nb)) == 0
    assert not rpt.BloomFilter(log_num_blocks=log_nb + 1).is_same_as(a)


def test_stream_calibration_kernels(rpt):
    """bench.py's stream calibration entry points: the copy moves the bytes exactly, the read runs, both report
    rates below the 8 TB/s spec."""
    from rpt_amd._lib import RPT_ERR_INVALID_ARGUMENT

    lib = rpt.load()
    nbytes = 1 << 28
    src = torch.randint(-2**62, 2**62, (nbytes // 8,), dtype=torch.int64, device="cuda:0")
    dst = torch.zeros_like(src)
    sink = torch.empty(int(lib.rpt_stream_sink_words(0)), dtype=torch.int64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    assert lib.rpt_stream_copy(dst.data_ptr(), src.data_ptr(), nbytes, s) == 0
    assert lib.rpt_stream_read(src.data_ptr(), nbytes, sink.data_ptr(), s) == 0
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert lib.rpt_stream_read(src.data_ptr() + 8, 16, sink.data_ptr(), s) == RPT_ERR_INVALID_ARGUMENT
    import bench

    cal = bench.stream_calibration(torch.device("cuda", 0), nbytes=1 << 30, reps=2)
    assert 1000 < cal["read_GBps"] < 8000 and 1000 < cal["copy_GBps"] < 8000, cal


@pytest.mark.parametrize("log_nb", [21, 22, 24])
@pytest.mark.parametrize("nulls", [False, True])
def test_large_filters_int32_vs_oracle(rpt, log_nb, nulls):
    """int32 keys through the partitioned probe at 128, 256 and 1024 slices (16 and 32 Ki-row tiles: the
    partition keeps its records in registers for both), ragged last tile, optionally with NULL keys."""
    rng = np.random.default_rng(log_nb + 100 * nulls)
    build = rng.integers(-2**31, 2**31, size=250000, dtype=np.int64).astype(np.int32)
    probe = np.concatenate([build[rng.integers(0, build.size, size=300000)],
                            rng.integers(-2**31, 2**31, size=5 * 16384 * 2 + 12345, dtype=np.int64).astype(np.int32)])
    rng.shuffle(probe)
    vw = gu.validity_words(rng.random(probe.size) > 0.02) if nulls else None
    bf = with_strategy(rpt.BloomFilter(log_num_blocks=log_nb), "partitioned")
    bf.insert(dev(build))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, build)
    assert np.array_equal(bf.export_words(), w)
    sel = bf.lookup_sel(dev(probe), validity=dev(vw) if nulls else None).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe, validity=vw))


@pytest.mark.parametrize("strategy", list(STRATEGIES))
def test_dictionary_validity_rowsel_vs_oracle(rpt, strategy):
    rng = np.random.default_rng(7)
    dict_vals = rng.integers(-10**12, 10**12, size=3000, dtype=np.int64)
    n = 20000
    key_sel = rng.integers(0, dict_vals.size, size=n).astype(np.uint32)
    valid = rng.random(dict_vals.size) > 0.05
    vw = gu.validity_words(valid)
    lnb = orc.log_num_blocks(n)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, dict_vals, key_sel=key_sel[:5000], validity=vw)
    bf = rpt.BloomFilter(n)
    if strategy == "lds":
        lnb = 13
        bf = rpt.BloomFilter(log_num_blocks=lnb)
        w = orc.new_words(lnb)
        orc.insert_keys(w, lnb, dict_vals, key_sel=key_sel[:5000], validity=vw)
    with_strategy(bf, strategy)
    bf.insert(dev(dict_vals), key_sel=dev(key_sel[:5000]), validity=dev(vw))
    assert np.array_equal(bf.export_words(), w)
    # probe a dictionary vector through a row selection (an already-sliced chunk)
    row_sel = np.sort(rng.choice(n, size=12000, replace=False)).astype(np.uint32)
    ref_rows = set(orc.probe_keys(w, lnb, dict_vals, key_sel=key_sel, validity=vw).tolist())
    exp = np.array([r for r in row_sel if r in ref_rows], dtype=np.uint32)
    got = bf.lookup_sel(dev(dict_vals), key_sel=dev(key_sel), validity=dev(vw), row_sel=dev(row_sel))
    assert np.array_equal(got.cpu().numpy().view(np.uint32), exp)


def test_unaligned_column_takes_general_path(rpt):
    keys = orc.synth_build_keys(5001)
    bf = rpt.BloomFilter(5000)
    t = dev(keys)
    bf.insert(t[1:])  # 8-byte aligned, not 16: GENERAL loads
    lnb = orc.log_num_blocks(5000)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, keys[1:])
    assert np.array_equal(bf.export_words(), w)
    probe = orc.synth_probe_keys(7001, 5001, 300)
    sel = bf.lookup_sel(dev(probe)[1:]).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, lnb, probe[1:]))


def test_multi_filter_chain_is_and(rpt):
    """PhysicalUseBF's loop (physical_use_bf.cpp:137-183): each filter probes the previous slice."""
    rng = np.random.default_rng(3)
    a_keys = rng.integers(0, 10**6, size=30000, dtype=np.int64)
    b_keys = rng.integers(0, 10**6, size=30000, dtype=np.int32)
    fa_keys = rng.integers(0, 10**6, size=20000, dtype=np.int64)
    fb_keys = rng.integers(0, 10**6, size=5000, dtype=np.int32)
    fa, fb = rpt.BloomFilter(fa_keys.size), rpt.BloomFilter(fb_keys.size)
    fa.insert(dev(fa_keys))
    fb.insert(dev(fb_keys))
    s1 = fa.lookup_sel(dev(a_keys))
    s2 = fb.lookup_sel(dev(b_keys), row_sel=s1)
    la, lb = orc.log_num_blocks(fa_keys.size), orc.log_num_blocks(fb_keys.size)
    wa, wb = orc.new_words(la), orc.new_words(lb)
    orc.insert_keys(wa, la, fa_keys)
    orc.insert_keys(wb, lb, fb_keys)
    exp = np.intersect1d(orc.probe_keys(wa, la, a_keys), orc.probe_keys(wb, lb, b_keys))
    assert np.array_equal(s2.cpu().numpy().view(np.uint32), exp)


def test_merge_of_partials_equals_single_build(rpt):
    keys = orc.synth_build_keys(300000)
    whole = rpt.BloomFilter(keys.size)
    whole.insert(dev(keys))
    parts = [rpt.BloomFilter(keys.size) for _ in range(4)]
    for i, p in enumerate(parts):
        lo, hi = i * 75000, (i + 1) * 75000
        p.insert(dev(keys[lo:hi]))
    for p in parts[1:]:
        parts[0].merge_or(p)
    assert np.array_equal(parts[0].export_words(), whole.export_words())
    # slice OR kernel (the local step of the multi-GPU all-reduce)
    nw = whole.num_blocks
    stack = torch.cat([torch.from_numpy(p.export_words().view(np.int64)) for p in parts[1:]]).cuda()
    dst = torch.zeros(nw, dtype=torch.int64, device="cuda")
    rpt.words_or_slices(dst, stack, 3, nw)
    ref = parts[1].export_words() | parts[2].export_words() | parts[3].export_words()
    assert np.array_equal(dst.cpu().numpy().view(np.uint64), ref)


@pytest.mark.parametrize("log_nb", [14, 17, 21, 24])
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
def test_partitioned_insert_vs_oracle(rpt, log_nb, dtype):
    """Partitioned build (slice-local LDS OR + atomic merge) == atomic build == oracle, incl. NULLs,
    ragged tiles and a second batch into the same filter."""
    rng = np.random.default_rng(log_nb)
    keys = rng.integers(-2**40, 2**40, size=3 * 16384 + 77, dtype=np.int64).astype(dtype)
    valid = rng.random(keys.size) > 0.01
    vw = gu.validity_words(valid)
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, keys, validity=vw)
    more = rng.integers(-2**40, 2**40, size=20001, dtype=np.int64).astype(dtype)
    orc.insert_keys(w, log_nb, more)
    for strategy in (rpt.RPT_INSERT_PARTITIONED, rpt.RPT_INSERT_ATOMIC):
        bf = rpt.BloomFilter(log_num_blocks=log_nb)
        bf.insert(dev(keys), validity=dev(vw), strategy=strategy)
        bf.insert(dev(more), strategy=strategy)
        assert np.array_equal(bf.export_words(), w), strategy


@pytest.mark.parametrize("log_nb", [7, 14])
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("shape", ["one_key", "runs", "pairs", "dictionary"])
def test_atomic_insert_repeated_keys_vs_oracle(rpt, log_nb, dtype, shape):
    """The atomic insert drops a row whose hash equals the previous row's (within a lane and across lanes,
    never from lane 0): runs of equal keys of every length, NULLs inside runs, ragged ends and the
    dictionary (key_sel) path give the oracle's words."""
    rng = np.random.default_rng(7 + log_nb)
    n = 5 * 4096 + 131
    if shape == "one_key":
        keys = np.full(n, 123456789, dtype=np.int64)
    elif shape == "runs":  # run lengths 1..300
        vals = rng.integers(-2**40, 2**40, size=n, dtype=np.int64)
        keys = np.repeat(vals, rng.integers(1, 300, size=n))[:n]
    elif shape == "pairs":  # every key twice in a row: duplicates at odd rows, across lane boundaries
        keys = np.repeat(rng.integers(-2**40, 2**40, size=n // 2 + 1, dtype=np.int64), 2)[:n]
    else:
        keys = rng.integers(-2**40, 2**40, size=37, dtype=np.int64)
    keys = keys.astype(dtype)
    valid = rng.random(n) > 0.05
    vw = gu.validity_words(valid)
    w = orc.new_words(log_nb)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    if shape == "dictionary":
        sel = np.repeat(rng.integers(0, keys.size, size=n).astype(np.uint32), 3)[:n]
        orc.insert_keys(w, log_nb, keys, key_sel=sel, validity=vw)
        bf.insert(dev(keys), key_sel=dev(sel), validity=dev(vw), strategy=rpt.RPT_INSERT_ATOMIC)
    else:
        orc.insert_keys(w, log_nb, keys, validity=vw)
        bf.insert(dev(keys), validity=dev(vw), strategy=rpt.RPT_INSERT_ATOMIC)
    assert np.array_equal(bf.export_words(), w)


def test_concurrent_inserts_on_two_streams(rpt):
    keys = orc.synth_build_keys(400000)
    bf = rpt.BloomFilter(keys.size)
    t = dev(keys)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    bf.insert(t[:200000], stream=s1)
    bf.insert(t[200000:], stream=s2)
    torch.cuda.synchronize()
    lnb = orc.log_num_blocks(keys.size)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, keys)
    assert np.array_equal(bf.export_words(), w)


def test_side_stream_probes_regrow_the_filter_workspace(rpt):
    """probe_async on a side stream with the filter's own workspace, growing it between probes (the
    smaller buffer is freed while the earlier probe may still run: the binding records the side stream on
    it), while the current stream allocates; every result equals the oracle's."""
    keys = orc.synth_build_keys(300000)
    bf = rpt.BloomFilter(keys.size)
    bf.insert(dev(keys))
    lnb = orc.log_num_blocks(keys.size)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, keys)
    s = torch.cuda.Stream()
    sizes = (5000, 60000, 700000, 2100000)
    probes = [orc.synth_probe_keys(n, keys.size, 300, start=7 * n) for n in sizes]
    torch.cuda.synchronize()
    outs = []
    for p in probes:
        t = dev(p)
        s.wait_stream(torch.cuda.current_stream())
        sel = torch.empty(p.size, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        bf.probe_async(t, out_sel=sel, out_count=cnt, stream=s)
        for _ in range(4):  # churn the current stream's allocator while the probe runs
            torch.empty(p.size * 3, dtype=torch.int64, device="cuda").fill_(-1)
        outs.append((t, sel, cnt))
    torch.cuda.synchronize()
    for p, (_, sel, cnt) in zip(probes, outs):
        assert np.array_equal(sel[: int(cnt.item())].cpu().numpy().view(np.uint32), orc.probe_keys(w, lnb, p))


def test_empty_filter_and_empty_input(rpt):
    bf = rpt.BloomFilter(1000)
    assert bf.is_empty()
    probe = dev(orc.synth_probe_keys(10000, 1000, 500))
    assert bf.lookup_sel(probe).numel() == 0  # empty filter: no survivors (physical_use_bf.cpp:144-155)
    bf.insert(probe[:0])
    assert bf.is_empty()  # zero-row insert keeps IsEmpty (bloom_filter.cpp:72-74)
    bf.insert(probe[:1])
    assert not bf.is_empty()
    assert bf.lookup_sel(probe[:0]).numel() == 0


def test_reinitialize_and_rehash_resize_rule(rpt):
    """PhysicalCreateBF::Finalize: undersized filter -> ReinitializeAndRehash(actual) (cpp:386-406)."""
    est, actual = 1000, 50000
    keys = orc.synth_build_keys(actual)
    bf = rpt.BloomFilter(est)
    chunks = [dict(keys=dev(keys[i:i + 2048])) for i in range(0, actual, 2048)]
    for ch in chunks:
        bf.insert(**ch)
    assert rpt.needs_resize(bf.sized_for_rows(), actual) and bf.needs_resize(actual)
    bf.reinitialize_and_rehash(actual, chunks)
    assert bf.sized_for_rows() == actual and bf.log_num_blocks == orc.log_num_blocks(actual)
    lnb = orc.log_num_blocks(actual)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, keys)
    assert np.array_equal(bf.export_words(), w)


def test_resize_predicate_on_allocation_matches_oracle(rpt):
    """Finalize's resize rule on the real allocation (rpt_bf_needs_resize_alloc) == the oracle's, at the
    sized_for = 1000 boundary (1024 / 1025 / 2048 actual rows) and over random estimates."""
    bf = rpt.BloomFilter(1000)
    assert bf.log_num_blocks == 7
    assert [bf.needs_resize(a) for a in (0, 1024, 1025, 2048)] == [False, False, True, True]
    rng = np.random.default_rng(5)
    for est in [0, 1, 63, 64, 65, 1000, 4096, 10**5, int(rng.integers(1, 10**6))]:
        f = rpt.BloomFilter(est)
        for a in [0, 1, est, est * 2, (64 << f.log_num_blocks) // 8, (64 << f.log_num_blocks) // 8 + 1,
                  int(rng.integers(0, 10**7))]:
            assert f.needs_resize(a) == orc.needs_resize_alloc(f.log_num_blocks, a), (est, a)


def test_synthetic_generators_match_oracle(rpt):
    b = rpt.synth_build_keys(100000, start=123).cpu().numpy()
    assert np.array_equal(b, orc.synth_build_keys(100000, start=123))
    p = rpt.synth_probe_keys(100000, 10**7, 100, start=10**9 - 100000).cpu().numpy()
    assert np.array_equal(p, orc.synth_probe_keys(100000, 10**7, 100, start=10**9 - 100000))


def _window_check(bf, w, lnb, probe_dev, sel, lo, hi):
    win = probe_dev[lo:hi].cpu().numpy()
    exp = orc.probe_keys(w, lnb, win).astype(np.int64) + lo
    a = np.searchsorted(sel, lo)
    b = np.searchsorted(sel, hi)
    assert np.array_equal(sel[a:b], exp)


def _i32_as_oracle(k):
    """int32 keys as the oracle hashes them: zero-extended through uint32 (DuckDB's Hash<int32_t>)."""
    return k.astype(np.int32).view(np.uint32).astype(np.int64)


def _full_check(w, lnb, probe_dev, sel, piece=10**8):
    """Every row of the probe against the oracle: the column is copied back in `piece`-row slices and
    each slice's expected survivors (oracle LookupSel + slice offset) must equal the sel entries that
    fall inside it. Slices are probed on host threads (ctypes releases the GIL). int32 columns are
    zero-extended for the oracle."""
    from concurrent.futures import ThreadPoolExecutor

    n = probe_dev.numel()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def one(lo_keys):
        lo, keys = lo_keys
        return lo, orc.probe_keys(w, lnb, keys).astype(np.int64) + lo

    conv = _i32_as_oracle if probe_dev.dtype == torch.int32 else (lambda k: k)
    jobs = ((lo, conv(probe_dev[lo:min(lo + piece, n)].cpu().numpy())) for lo in range(0, n, piece))
    checked = 0
    with ThreadPoolExecutor(threads) as ex:
        for lo, exp in ex.map(one, jobs):
            hi = min(lo + piece, n)
            a, b = np.searchsorted(sel, lo), np.searchsorted(sel, hi)
            assert np.array_equal(sel[a:b], exp), f"rows [{lo}, {hi}) differ from the oracle"
            checked += b - a
    assert checked == sel.size


@pytest.mark.parametrize("n_probe,n_build,p,strategy", [(10**8, 10**7, 100, "gather"),
                                                         (10**8, 10**7, 1000, "partitioned"),
                                                         (10**9, 10**7, 100, "partitioned")])
def test_full_size_probe_properties(rpt, n_probe, n_build, p, strategy):
    """BASELINE sizes (C2 at 1e9 rows): EVERY row's result against the oracle (1e8-row slices on host
    threads), sortedness, count == popcount(find bits), no false negatives."""
    build = rpt.synth_build_keys(n_build)
    bf = with_strategy(rpt.BloomFilter(n_build), strategy)
    bf.insert(build)
    lnb = bf.log_num_blocks
    w = bf.export_words()
    # oracle builds the same filter from the same stream
    ow = orc.new_words(lnb)
    orc.insert_keys(ow, lnb, orc.synth_build_keys(n_build))
    assert np.array_equal(w, ow)
    assert bf.lookup_sel(build).numel() == n_build  # no false negatives
    probe = rpt.synth_probe_keys(n_probe, n_build, p)
    sel_t, cnt = bf.probe_async(probe)
    count = int(cnt.item())
    bits = bf.find_bits(probe)
    pop = int(np.bitwise_count(bits.cpu().numpy().view(np.uint64)).sum())
    assert count == pop
    sel = sel_t[:count]  # int32: n_probe < 2^31
    assert bool((sel[1:] > sel[:-1]).all())
    sel_np = sel.cpu().numpy().astype(np.int64)
    _full_check(w, lnb, probe, sel_np)
    rate = count / n_probe
    assert p / 1000 <= rate < p / 1000 + 0.05
    del probe, sel_t, bits, sel
    torch.cuda.empty_cache()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config,n_build,n_filter", [("C3", 10**8, 10**8), ("C5 share", 10**9, 8 * 10**9),
                                                     ("C2-i32", 10**7, 10**7)])
def test_full_size_configs_every_row(rpt, config, n_build, n_filter):
    """BASELINE C3 (1e8-key build, 128 MiB filter: partitioned, 32 Ki-row tiles), one rank's share of
    C5 (1e9 keys into the 8 GiB filter sized for 8e9: bucketed insert and probe) and C2 with int32 keys
    (JOB's INTEGER join keys: the synthetic streams truncated to int32, as bench.py --key-type i32) at
    full size, as bench.py runs them (AUTO strategies): the filter word for word and every one of the 1e9
    probe rows against the oracle (built with host threads from the same synthetic streams)."""
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    n_probe = 10**9
    i32 = config.endswith("-i32")
    build = rpt.synth_build_keys(n_build)
    if i32:
        build = build.to(torch.int32)
    bf = rpt.BloomFilter(n_filter)
    bf.insert(build)
    del build
    lnb = bf.log_num_blocks
    assert bf.probe_strategy_for(n_probe) == (4 if config.startswith("C5") else 3)
    ow = orc.new_words(lnb)
    okeys = orc.synth_build_keys(n_build)
    orc.build_mt(ow, lnb, _i32_as_oracle(okeys) if i32 else okeys, threads)
    del okeys
    got = torch.empty(bf.num_blocks, dtype=torch.int64, device="cuda:0")
    bf.copy_words_to(got)
    assert torch.equal(got, torch.from_numpy(ow.view(np.int64)).to("cuda:0")), "filter words differ from the oracle"
    del got
    torch.cuda.empty_cache()
    probe = rpt.synth_probe_keys(n_probe, n_build, 100)
    if i32:
        probe = probe.to(torch.int32)
        torch.cuda.empty_cache()
    sel_t, cnt = bf.probe_async(probe)
    count = int(cnt.item())
    sel = sel_t[:count].cpu().numpy().astype(np.int64)
    del sel_t
    torch.cuda.empty_cache()
    assert np.all(sel[1:] > sel[:-1])
    _full_check(ow, lnb, probe, sel)
    assert 0.1 <= count / n_probe < 0.15
    del probe
    torch.cuda.empty_cache()


@pytest.mark.parametrize("strategy", ["partitioned", "gather"])
def test_row_ids_beyond_int32(rpt, strategy):
    """n > 2^31 rows (sel_t is uint32): ids past 2^31 stay exact, ascending, and match the oracle."""
    n_build, n_probe = 10**7, (1 << 31) + (1 << 20) + 12345
    build = rpt.synth_build_keys(n_build)
    bf = with_strategy(rpt.BloomFilter(n_build), strategy)
    bf.insert(build)
    w = bf.export_words()
    lnb = bf.log_num_blocks
    probe = rpt.synth_probe_keys(n_probe, n_build, 100)
    sel_t, cnt = bf.probe_async(probe)
    count = int(cnt.item())
    sel = sel_t[:count].cpu().numpy().view(np.uint32).astype(np.int64)
    assert np.all(sel[1:] > sel[:-1]) and sel[-1] < n_probe and sel[-1] >= (1 << 31)
    for lo, hi in [(0, 10**6), ((1 << 31) - 500_000, (1 << 31) + 500_000), (n_probe - 10**6, n_probe)]:
        _window_check(bf, w, lnb, probe, sel, lo, hi)
    assert 0.1 <= count / n_probe < 0.15
    del probe, sel_t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("log_nb", [17, 21, 24])
def test_partitioned_skewed_and_all_null(rpt, log_nb):
    """Adversarial runs for the partitioned probe and insert: every row of a tile in ONE slice (a run
    of 16384 records, the tile's whole capacity), 2 distinct keys, and an all-NULL column (every row
    hashes to NULL_HASH)."""
    rng = np.random.default_rng(log_nb + 100)
    base = rng.integers(-2**40, 2**40, size=4096, dtype=np.int64)
    h = orc.hash_keys(base)
    slice_of = (h >> np.uint64(16 + 14)) & np.uint64((1 << max(log_nb - 14, 0)) - 1)
    one = base[slice_of == slice_of[0]][:3]  # keys of one 128 KiB slice
    n = 3 * 16384 + 501
    cases = {
        "one_slice": one[rng.integers(0, one.size, n)],
        "two_keys": np.where(rng.random(n) < 0.5, base[0], base[1]),
    }
    for name, keys in cases.items():
        w = orc.new_words(log_nb)
        orc.insert_keys(w, log_nb, keys)
        bf = rpt.BloomFilter(log_num_blocks=log_nb)
        bf.insert(dev(keys), strategy=rpt.RPT_INSERT_PARTITIONED)
        assert np.array_equal(bf.export_words(), w), name
        probe = np.concatenate([keys, base])
        bf.probe_strategy = STRATEGIES["partitioned"]
        sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
        assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe)), name
    # all-NULL: inserted NULL rows set the NULL_HASH bits, probed NULL rows test them
    keys = base[:1].repeat(n)
    vw = gu.validity_words(np.zeros(n, dtype=bool))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, keys, validity=vw)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(keys), validity=dev(vw), strategy=rpt.RPT_INSERT_PARTITIONED)
    assert np.array_equal(bf.export_words(), w)
    bf.probe_strategy = STRATEGIES["partitioned"]
    sel = bf.lookup_sel(dev(keys), validity=dev(vw)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, keys, validity=vw))


@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [1, 63, 513, 2048, 5000, 16383, 16384, 16385])
def test_small_batch_fused_probe(rpt, dtype, n):
    """AUTO batches of <= RPT_SMALL_PROBE_ROWS rows take the fused one-workgroup probe (probe +
    compaction in one launch): == the oracle and == the forced four-kernel gather path, for flat,
    unaligned and dictionary vectors with NULLs and a row selection."""
    rng = np.random.default_rng(n * 3 + (dtype == np.int32))
    dict_vals = rng.integers(-2**40, 2**40, size=4000, dtype=np.int64).astype(dtype)
    build_sel = rng.integers(0, dict_vals.size, size=1500).astype(np.uint32)
    valid = rng.random(dict_vals.size) > 0.05
    vw = gu.validity_words(valid)
    bf = rpt.BloomFilter(1500)
    lnb = bf.log_num_blocks
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, dict_vals, key_sel=build_sel, validity=vw)
    bf.insert(dev(dict_vals), key_sel=dev(build_sel), validity=dev(vw))
    assert np.array_equal(bf.export_words(), w)
    key_sel = rng.integers(0, dict_vals.size, size=n).astype(np.uint32)
    flat = dict_vals[key_sel]
    row_sel = np.sort(rng.choice(n, size=max(n // 2, 1), replace=False)).astype(np.uint32)
    ref_dict = orc.probe_keys(w, lnb, dict_vals, key_sel=key_sel, validity=vw)
    exp_rowsel = np.intersect1d(row_sel, ref_dict).astype(np.uint32)
    padded = np.concatenate([flat[:1], flat])  # the same keys one element off 16-B alignment
    cases = {
        "flat": (dict(keys=dev(flat)), orc.probe_keys(w, lnb, flat)),
        "unaligned": (dict(keys=dev(padded)[1:]), orc.probe_keys(w, lnb, flat)),
        "dict_nulls": (dict(keys=dev(dict_vals), key_sel=dev(key_sel), validity=dev(vw)), ref_dict),
        "dict_rowsel": (dict(keys=dev(dict_vals), key_sel=dev(key_sel), validity=dev(vw), row_sel=dev(row_sel)),
                        exp_rowsel),
    }
    for name, (kw, exp) in cases.items():
        keys = kw.pop("keys")
        for strategy in (rpt.RPT_PROBE_AUTO, rpt.RPT_PROBE_GATHER):
            bf.probe_strategy = strategy
            got = bf.lookup_sel(keys, **kw).cpu().numpy().view(np.uint32)
            assert np.array_equal(got, exp), (name, strategy)


@pytest.mark.parametrize("n", [1, 32767, 32768, 32769, 3 * 32768 + 5, 300007])
def test_double_tile_edges_vs_oracle(rpt, n):
    """Filters of more than 512 slices (here 2^24 blocks = 1024 slices) partition 32 Ki-row tiles
    with an unpadded LDS copy (rpt::tile_mult): ragged tile boundaries for the probe and the insert."""
    log_nb = 24
    rng = np.random.default_rng(n + 5)
    build = rng.integers(-2**40, 2**40, size=max(n // 2, 1), dtype=np.int64)
    probe = np.concatenate([build[rng.integers(0, build.size, size=n // 3)],
                            rng.integers(-2**40, 2**40, size=n - n // 3, dtype=np.int64)])
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, build)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(dev(build), strategy=rpt.RPT_INSERT_PARTITIONED)
    assert np.array_equal(bf.export_words(), w)
    bf.probe_strategy = STRATEGIES["partitioned"]
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, log_nb, probe))


@pytest.mark.parametrize("strategy,log_nb,n,dense", [
    ("partitioned", 17, 3 * 32768 + 777, False), ("partitioned", 21, 3 * 32768 + 777, False),
    ("partitioned", 24, 3 * 32768 + 777, False), ("bucketed", 22, 5 * 16384 + 333, False),
    ("bucketed", 24, 9 * 16384 + 4097, False), ("bucketed", 24, 9 * 16384 + 4097, True)])
@pytest.mark.parametrize("use_row_sel", [False, True])
def test_fused_sel_tail_equals_two_phase_path(rpt, strategy, log_nb, n, dense, use_row_sel):
    """rpt_bf_probe's partitioned pipeline ends in the fused tail (tile counts -> offsets -> the unpermute
    writes the sel); rpt_bf_probe_phase1 + phase2 keep the result-bit path (the bucketed strategy takes it
    in both). Both must give the oracle's sel and count, with and without a row selection: 16 Ki- (2^17,
    2^21) and 32 Ki-row (2^24) partition tiles; bucketed with 1 and 4 buckets, several level-1 tiles and a
    partial last tile, and a probe where every row passes (the dense word-by-word sel expansion)."""
    build = orc.synth_build_keys(200000)
    probe = orc.synth_probe_keys(n, 200000, 250)
    if dense:
        probe = build[np.random.default_rng(7).integers(0, build.size, n)]
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.probe_strategy = {"partitioned": rpt.RPT_PROBE_PARTITIONED, "bucketed": rpt.RPT_PROBE_BUCKETED}[strategy]
    bf.insert(dev(build))
    w = orc.new_words(log_nb)
    orc.insert_keys(w, log_nb, build)
    rng = np.random.default_rng(log_nb)
    row_sel = np.sort(rng.choice(n, size=n // 3, replace=False)).astype(np.uint32) if use_row_sel else None
    ref = orc.probe_keys(w, log_nb, probe)
    exp = ref if row_sel is None else np.intersect1d(row_sel, ref).astype(np.uint32)
    rs = dev(row_sel) if row_sel is not None else None
    m = row_sel.size if row_sel is not None else n
    assert not dense or exp.size == m  # every row passes: the dense expansion runs
    keys = dev(probe)
    fused = bf.lookup_sel(keys, row_sel=rs).cpu().numpy().view(np.uint32)
    ws = torch.empty(bf.workspace_bytes(m), dtype=torch.uint8, device="cuda:0")
    out = torch.full((m,), -1, dtype=torch.int32, device="cuda:0")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    bf.probe_phase1(keys, ws, n=m, row_sel=rs)
    bf.probe_phase2(m, out, cnt, ws, row_sel=rs)
    two = out[: int(cnt.item())].cpu().numpy().view(np.uint32)
    assert np.array_equal(fused, exp)
    assert np.array_equal(two, exp)


@pytest.mark.parametrize("strategy", ["partitioned", "gather"])
def test_concurrent_probes_on_two_streams(rpt, strategy):
    """Two LookupSel calls in flight at once on two streams (DuckDB's operator threads each own a
    stream and workspace): each gets the oracle's sel for its own rows."""
    build = orc.synth_build_keys(300000)
    lnb = 21
    bf = with_strategy(rpt.BloomFilter(log_num_blocks=lnb), strategy)
    bf.insert(dev(build))
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, build)
    probes = [orc.synth_probe_keys(700001, 300000, 200), orc.synth_probe_keys(500003, 300000, 50, start=10**6)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    torch.cuda.synchronize()
    for keys, st in zip(probes, streams):
        n = keys.size
        ws = torch.empty(bf.workspace_bytes(n), dtype=torch.uint8, device="cuda:0")
        sel = torch.empty(n, dtype=torch.int32, device="cuda:0")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
        kd = dev(keys)
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            bf.probe_async(kd, n=n, out_sel=sel, out_count=cnt, workspace=ws, stream=st)
        outs.append((sel, cnt, ws, kd))
    torch.cuda.synchronize()
    for (sel, cnt, _ws, _kd), keys in zip(outs, probes):
        got = sel[: int(cnt.item())].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, orc.probe_keys(w, lnb, keys))


@pytest.mark.parametrize("strategy", ["gather", "lds"])
@pytest.mark.parametrize("dtype", [np.int64, np.int32])
@pytest.mark.parametrize("n", [2**22 + 5, 5 * 2**21, 2**24 + 3 * 512 + 1, 20000003])
def test_direct_probe_pipelined_rounds_vs_oracle(rpt, strategy, dtype, n):
    """The direct probes' software-pipelined loop over full 512-row segments: several rounds of the
    whole grid, groups cut off by the last full segment, and the ragged tail taken by the general loop."""
    rng = np.random.default_rng(n + 7 * (dtype == np.int32))
    build = rng.integers(-2**31, 2**31, size=20000, dtype=np.int64).astype(dtype)
    probe = rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(dtype)
    probe[rng.integers(0, n, size=n // 10)] = build[rng.integers(0, build.size, size=n // 10)]
    lnb = orc.log_num_blocks(build.size)
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, build)
    bf = with_strategy(rpt.BloomFilter(build.size), strategy)
    bf.insert(dev(build))
    sel = bf.lookup_sel(dev(probe)).cpu().numpy().view(np.uint32)
    assert np.array_equal(sel, orc.probe_keys(w, lnb, probe))


@pytest.mark.parametrize("strategy", ["gather", "partitioned", "bucketed"])
@pytest.mark.parametrize("p", [400, 800, 1000])
@pytest.mark.parametrize("use_row_sel", [False, True])
def test_dense_selection_vectors_vs_oracle(rpt, strategy, p, use_row_sel):
    """High pass rates take the word-by-word selection-vector expansion (unpermute_sel_kernel from 192
    survivors per 512 rows, compact_kernel from 384): every sel entry against the oracle, ragged n, with
    and without an incoming row selection."""
    n_build, n, lnb = 300_000, 3_000_001, 22
    bf = rpt.BloomFilter(log_num_blocks=lnb)
    bf.probe_strategy = {"gather": 1, "partitioned": 3, "bucketed": 4}[strategy]
    bf.insert(rpt.synth_build_keys(n_build))
    w = orc.new_words(lnb)
    orc.insert_keys(w, lnb, orc.synth_build_keys(n_build))
    probe = rpt.synth_probe_keys(n, n_build, p)
    keys = probe.cpu().numpy()
    if use_row_sel:
        rng = np.random.default_rng(p)
        rows = np.sort(rng.choice(n, size=n // 2, replace=False)).astype(np.uint32)
        got = bf.lookup_sel(probe, row_sel=torch.from_numpy(rows.view(np.int32)).to("cuda:0"))
        exp = rows[orc.probe_keys(w, lnb, keys, key_sel=rows)]
    else:
        got = bf.lookup_sel(probe)
        exp = orc.probe_keys(w, lnb, keys)
    got = got.cpu().numpy().view(np.uint32)
    assert got.size >= (p / 1000) * (n // 2 if use_row_sel else n) * 0.99
    assert np.array_equal(got, exp.astype(np.uint32))
