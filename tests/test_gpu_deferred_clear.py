"""rpt_bf_clear defers its zeroing to the next operation on the filter (rpt_bf::clear_pending): a
partitioned / bucketed insert whose slice merge owns every slice stores the slices whole (zeros
included), every other operation zeroes the words first. Each case fills the filter with keys A, clears
it, then runs one operation: the result must equal the oracle's for an EMPTY filter followed by that
operation (no bit of A survives), and the filter must keep composing with later inserts. Bit-exact."""
import gc
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


@pytest.mark.parametrize("mode", [2, 0])  # hipStreamCaptureModeRelaxed, hipStreamCaptureModeGlobal (torch's default)
@pytest.mark.parametrize("log_nb,n", [(14, 200_000), (21, 5_000_000)])  # LDS probe; partitioned probe
def test_graph_capture_of_a_cleared_filter(rpt, log_nb, n, mode):
    """a probe captured into a HIP graph must not carry the deferred clear's zeroing (each replay
    would wipe the bits inserted since). A capture that would have to settle the clear is refused
    (RPT_ERR_INVALID_ARGUMENT, the capture itself stays valid); after rpt_bf_settle the probe captures, and
    replays after later inserts see those inserts (the oracle's sel each time)."""
    import ctypes

    from rpt_amd._lib import RptError

    hip = ctypes.CDLL("libamdhip64.so")
    for fn in ("hipStreamBeginCapture", "hipStreamEndCapture", "hipGraphInstantiate", "hipGraphLaunch",
               "hipGraphExecDestroy", "hipGraphDestroy"):
        getattr(hip, fn).restype = ctypes.c_int
    bf = filled(rpt, log_nb)
    bf.clear()
    p = keys(n, 7)
    b, c = keys(300_000, 8), keys(300_000, 9)
    m = min(n // 10, b.size)
    p[:m] = b[:m]  # some probe rows are B's keys, more are C's after the second insert
    p[m: 2 * m] = c[:m]
    kp = dev(p)
    out_sel = torch.empty(n, dtype=torch.int32, device="cuda:0")
    out_count = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    ws = torch.empty(bf.workspace_bytes(n), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.Stream(device="cuda:0")
    sh = ctypes.c_void_p(s.cuda_stream)
    graph, exe = ctypes.c_void_p(), ctypes.c_void_p()

    def capture():
        # as torch.cuda.graph prepares a capture: collect garbage first (a filter an earlier test left to the cycle
        # collector is freed by rpt_bf_destroy -> hipFree, which would invalidate a global-mode capture from any
        # thread of the process) and keep the collector off inside the capture window
        gc.collect()
        torch.cuda.synchronize()
        gc.disable()
        assert hip.hipStreamBeginCapture(sh, mode) == 0
        err = None
        try:
            bf.probe_async(kp, n=n, out_sel=out_sel, out_count=out_count, workspace=ws, stream=s)
        except RptError as e:
            err = e
        st = hip.hipStreamEndCapture(sh, ctypes.byref(graph))
        gc.enable()
        assert st == 0  # still a valid capture
        return err

    err = capture()
    assert err is not None and err.status == 1 and "rpt_bf_settle" in str(err)
    assert hip.hipGraphDestroy(graph) == 0
    bf.settle()
    bf.insert(dev(b))
    assert capture() is None
    assert hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, ctypes.c_size_t(0)) == 0
    ref = orc.new_words(log_nb)
    orc.insert_keys(ref, log_nb, b)
    for extra in (None, c):
        if extra is not None:  # an insert between replays: the replay must see it, and nothing wiped
            bf.insert(dev(extra))
            orc.insert_keys(ref, log_nb, extra)
        torch.cuda.synchronize()
        assert hip.hipGraphLaunch(exe, sh) == 0
        s.synchronize()
        cnt = int(out_count.item())
        want = orc.probe_keys(ref, log_nb, p)
        assert np.array_equal(out_sel[:cnt].cpu().numpy().view(np.uint32), want)
    assert np.array_equal(bf.export_words(), ref)
    assert hip.hipGraphExecDestroy(exe) == 0 and hip.hipGraphDestroy(graph) == 0


@pytest.mark.parametrize("mode", [2, 0])  # relaxed; global, where the library's event query must not break the capture
@pytest.mark.parametrize("strategy,log_nb", [(INS_ATOMIC, 22), (INS_PARTITIONED, 21), (INS_PARTITIONED, 24),
                                             (INS_BUCKETED, 25)])
def test_graph_capture_of_inserts(rpt, strategy, log_nb, mode):
    """writes captured into a HIP graph. (1) An insert captured after a clear is refused (its
    settling memset / whole-slice stores would replay with the graph and wipe what was inserted between
    replays), and so is a clear inside a capture; each capture stays valid. (2) After rpt_bf_settle the insert
    captures (every strategy, through rpt_bf_insert_ws with a workspace that outlives the graph); each replay
    ORs its keys into whatever the filter holds by then: inserts made between replays survive, replays are
    idempotent, words == the oracle's filter of every key inserted."""
    import ctypes

    from rpt_amd._lib import check

    hip = ctypes.CDLL("libamdhip64.so")
    for fn in ("hipStreamBeginCapture", "hipStreamEndCapture", "hipGraphInstantiate", "hipGraphLaunch",
               "hipGraphExecDestroy", "hipGraphDestroy"):
        getattr(hip, fn).restype = ctypes.c_int
    bf = filled(rpt, log_nb)
    lib = bf._lib
    n = 3_000_000 if strategy != INS_ATOMIC else 200_000
    b, c, d = keys(n, 11), keys(200_000, 12), keys(200_000, 13)
    kb = dev(b)
    col = rpt.make_column(kb)
    check(lib.rpt_bf_set_insert_strategy(bf.handle, strategy), lib)
    ws_bytes = max(int(lib.rpt_bf_insert_workspace_bytes(bf.handle, n)), 256)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda:0")  # lives as long as the graph
    s = torch.cuda.Stream(device="cuda:0")
    sh = ctypes.c_void_p(s.cuda_stream)
    graph, exe = ctypes.c_void_p(), ctypes.c_void_p()

    def capture(op):
        gc.collect()  # see test_graph_capture_of_a_cleared_filter
        torch.cuda.synchronize()
        gc.disable()
        assert hip.hipStreamBeginCapture(sh, mode) == 0
        st = op()
        end = hip.hipStreamEndCapture(sh, ctypes.byref(graph))
        gc.enable()
        assert end == 0  # still a valid capture
        return st

    def insert_b():
        return lib.rpt_bf_insert_ws(bf.handle, ctypes.byref(col), n, ws.data_ptr(), ws_bytes, sh)

    bf.clear()
    assert capture(insert_b) == 1 and "rpt_bf_settle" in lib.rpt_last_error().decode()
    assert hip.hipGraphDestroy(graph) == 0
    assert capture(lambda: lib.rpt_bf_clear(bf.handle, sh)) == 1
    assert "clear outside the capture" in lib.rpt_last_error().decode()
    assert hip.hipGraphDestroy(graph) == 0
    bf.settle()
    bf.insert(dev(c))
    assert capture(insert_b) == 0, lib.rpt_last_error().decode()
    assert hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, ctypes.c_size_t(0)) == 0
    ref = orc.new_words(log_nb)
    orc.insert_keys(ref, log_nb, c)  # the clear dropped the filled keys; the capture inserted nothing yet
    torch.cuda.synchronize()
    assert np.array_equal(bf.export_words(), ref)
    orc.insert_keys(ref, log_nb, b)
    for extra in (None, d, None):
        if extra is not None:  # an insert between replays: kept by the next replay
            bf.insert(dev(extra))
            orc.insert_keys(ref, log_nb, extra)
        torch.cuda.synchronize()
        assert hip.hipGraphLaunch(exe, sh) == 0
        s.synchronize()
        assert np.array_equal(bf.export_words(), ref)
    probe = np.concatenate([b[:20_000], keys(20_000, 14), d[:1000]])
    assert np.array_equal(bf.lookup_sel(dev(probe)).cpu().numpy().astype(np.uint32), orc.probe_keys(ref, log_nb, probe))
    assert hip.hipGraphExecDestroy(exe) == 0 and hip.hipGraphDestroy(graph) == 0
