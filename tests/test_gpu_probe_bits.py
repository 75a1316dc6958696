"""rpt_bf_probe_bits through the C-ABI (the host mirror's bits-back lookups, DESIGN §5 "Result bits back"): the
result bits of every probe strategy, with and without row_sel, NULL rows included, bit for bit against the oracle's
per-row hits; bits past n are 0; argument errors."""
import ctypes

import numpy as np
import pytest
import torch

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


def _bits_to_rows(words: np.ndarray, n: int) -> np.ndarray:
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    assert not bits[n:].any()  # nothing past n
    return np.flatnonzero(bits[:n])


@pytest.mark.parametrize("strategy,log_nb,n", [(1, 14, 70001), (2, 12, 100003), (3, 18, 2_000_001), (4, 22, 3_000_017)])
@pytest.mark.parametrize("with_sel", [False, True])
def test_probe_bits_vs_oracle(rpt, strategy, log_nb, n, with_sel):
    from rpt_amd import _lib

    rng = np.random.default_rng(strategy * 10 + with_sel)
    n_build = 1 << (log_nb + 2)
    build = rng.integers(-(2**62), 2**62, size=n_build, dtype=np.int64)
    bf = rpt.BloomFilter(log_num_blocks=log_nb)
    bf.insert(torch.from_numpy(build).cuda())
    lib = bf._lib
    if not lib.rpt_probe_strategy_supported(strategy, log_nb):
        pytest.skip("strategy unsupported at this size")
    _lib.check(lib.rpt_bf_set_probe_strategy(bf.handle, strategy), lib)
    total = n + 1000 if with_sel else n
    keys = np.where(rng.random(total) < 0.3, build[rng.integers(0, n_build, total)],
                    rng.integers(-(2**62), 2**62, size=total, dtype=np.int64))
    valid = rng.random(total) > 0.02
    vw = np.packbits(valid, bitorder="little")
    vw = np.concatenate([vw, np.zeros((-len(vw)) % 8 + 8, np.uint8)]).view(np.uint64)
    row_sel = np.sort(rng.choice(total, size=n, replace=False)).astype(np.uint32) if with_sel else None
    d_keys = torch.from_numpy(keys).cuda()
    d_valid = torch.from_numpy(vw.view(np.int64)).cuda()
    col = rpt.make_column(d_keys, validity=d_valid)
    d_sel = torch.from_numpy(row_sel.view(np.int32)).cuda() if with_sel else None
    words = (n + 511) // 512 * 8
    out = torch.full((words,), -1, dtype=torch.int64, device="cuda")
    ws_bytes = max(int(lib.rpt_bf_probe_workspace_bytes(bf.handle, n)), 256)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.rpt_bf_probe_bits(bf.handle, ctypes.byref(col), d_sel.data_ptr() if with_sel else None, n,
                                     out.data_ptr(), ws.data_ptr(), ws_bytes, s), lib)
    torch.cuda.synchronize()
    got = _bits_to_rows(out.cpu().numpy().view(np.uint64), n)
    w = bf.export_words()
    rows = row_sel if with_sel else np.arange(n, dtype=np.uint32)
    vsub = np.packbits(valid[rows], bitorder="little")
    vsub = np.concatenate([vsub, np.zeros((-len(vsub)) % 8 + 8, np.uint8)]).view(np.uint64)
    want = orc.probe_keys(w, log_nb, keys[rows], validity=vsub)
    assert np.array_equal(got, want.astype(np.int64))


def test_probe_bits_arguments(rpt):
    bf = rpt.BloomFilter(log_num_blocks=12)
    lib = bf._lib
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.rpt_bf_probe_bits(None, None, None, 10, None, None, 0, s) == 1
    assert lib.rpt_bf_probe_bits(bf.handle, None, None, 10, None, None, 0, s) == 1
