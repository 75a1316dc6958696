"""rpt_keys_widen through the C-ABI: narrow BIGINT keys (4-B low words + one high word per chunk) back to int64 in
HBM, as the host mirror's pipelines send BIGINT ids over PCIe (DESIGN §5 "Narrow BIGINT keys"). Ragged chunks
(empty, one row, 2048, 3000 rows), high words 0 / 5 / 0xFFFFFFFF (negative keys), against numpy; null arguments
and zero chunks."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a visible GPU")
    from rpt_amd import _lib

    torch.cuda.set_device(0)
    return _lib


def test_widen_matches_numpy(lib):
    L = lib.load()
    rng = np.random.default_rng(5)
    sizes = [0, 1, 2048, 3000, 0, 2047, 7, 2048]
    row0 = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    n = int(row0[-1])
    lo = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    hi = np.array([0, 5, 0xFFFFFFFF, 0, 5, 0xFFFFFFFF, 0x7FFFFFFF, 1], dtype=np.uint32)
    want = np.concatenate([(np.uint64(hi[c]) << np.uint64(32)) | lo[row0[c]:row0[c + 1]].astype(np.uint64)
                           for c in range(len(sizes))])
    d_lo = torch.from_numpy(lo.view(np.int32)).cuda()
    d_hi = torch.from_numpy(hi.view(np.int32)).cuda()
    d_row0 = torch.from_numpy(row0.view(np.int32)).cuda()
    out = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    lib.check(L.rpt_keys_widen(d_lo.data_ptr(), d_hi.data_ptr(), d_row0.data_ptr(), len(sizes), out.data_ptr(), s), L)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    assert (out.cpu().numpy()[row0[2]:row0[3]] < 0).all()  # high word 0xFFFFFFFF: negative keys


def test_widen_arguments(lib):
    L = lib.load()
    s = torch.cuda.current_stream().cuda_stream
    assert L.rpt_keys_widen(None, None, None, 0, None, s) == lib.RPT_OK  # nothing to do
    assert L.rpt_keys_widen(None, None, None, 3, None, s) == lib.RPT_ERR_INVALID_ARGUMENT
