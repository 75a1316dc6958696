"""C++ host mirror (include/rpt_host.hpp) of PTBloomFilter / CREATE_BF / USE_BF, end to end.

The GPU test runs tests/cpp/build/test_host_mirror (4 sink threads, FLAT/CONSTANT/DICTIONARY vectors
with NULLs, sink batches kept in HBM with asynchronous and synchronous flushes, resize + rehash from HBM in
Finalize, the parallel source, a two-filter USE_BF chain, early exits, the pipelined batch paths on worker
threads, 2- to 5-filter pipelined chains, the pinned staging cache) against the oracle.
"""
import os
import subprocess

import pytest

from conftest import REPO

CPP = os.path.join(REPO, "tests", "cpp")
BIN = os.path.join(CPP, "build", "test_host_mirror")


def _build():
    subprocess.run(["make", "-s", "-C", CPP], check=True)


def test_host_mirror_links():
    """The mirror is compiled into librpt_gpu.so and a C++ caller links against it (no GPU needed)."""
    _build()
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    assert "librpt_gpu.so" in out and "not found" not in out
    syms = subprocess.run(["nm", "-DC", os.path.join(REPO, "duckdb-robust-predicate-transfer_amd", "build",
                                                      "librpt_gpu.so")], capture_output=True, text=True).stdout
    for name in ["rpt::PTBloomFilter::Insert", "rpt::PTBloomFilter::LookupSel", "rpt::CreateBF::Finalize",
                 "rpt::UseBF::Execute", "rpt::PTBloomFilter::ReinitializeAndRehash",
                 "rpt::CreateBF::GetData", "rpt::CreateBF::GetGlobalSourceState", "rpt::DeviceKeyColumn::Append",
                 "rpt::PTBloomFilter::InsertDevice", "rpt::UseBF::ExecuteBatch", "rpt::UseBF::ExecuteChainPipelined",
                 "rpt::ReleasePinnedCache", "rpt::SetPinnedCacheLimit", "rpt::PinnedCacheBytes"]:
        assert name in syms, name


@pytest.mark.gpu
def test_host_mirror_end_to_end():
    _build()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
