"""C-ABI library checks that need no GPU: it loads, exports every symbol include/*.h declares,
its host-only rules agree with the oracle, and argument errors are reported (not crashed on)."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

import rpt_oracle as orc
from conftest import REPO
from rpt_amd import _lib


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rpt_\w+)\s*\(", src, flags=re.M))
    return names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    declared = declared_functions()
    assert len(declared) >= 25
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes table binds exactly the declared surface
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_library_is_gfx950_code_object():
    path = _lib.LIB_PATH
    blob = open(path, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_status_strings():
    lib = _lib.load()
    assert lib.rpt_abi_version() == 1
    assert lib.rpt_status_string(0) == b"ok"
    assert lib.rpt_status_string(4) == b"workspace too small"
    assert lib.rpt_status_string(6) == b"collective (RCCL) failed"


def test_allreduce_or_rejects_null_communicator():
    lib = _lib.load()
    # argument checks run before RCCL is loaded or any device is touched
    assert lib.rpt_bf_allreduce_or(None, None, None) == _lib.RPT_ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 100, 129, 1000, 4096, 10**5, 10**6, 10**7, 10**8, 10**9,
                               8 * 10**9, 2**40])
def test_sizing_rule_matches_oracle(n):
    assert _lib.load().rpt_bf_log_num_blocks_for_rows(n) == orc.log_num_blocks(n)


def test_resize_rule_matches_oracle():
    lib = _lib.load()
    rng = np.random.default_rng(1)
    for _ in range(2000):
        s = int(rng.integers(0, 10**8))
        a = int(rng.integers(0, 10**9))
        assert lib.rpt_bf_needs_resize(s, a) == orc.lib().rpt_oracle_needs_resize(s, a)
    for s in [0, 1, 42, 1000, 10**7]:
        for a in [0, 1, 64, 65, s * 8, s * 12, s * 16, s * 16 + 1]:
            assert lib.rpt_bf_needs_resize(s, a) == orc.lib().rpt_oracle_needs_resize(s, a)


def test_resize_rules_monotone_in_rows():
    """rpt::CreateBF skips a sink flush's insert once the rows flushed so far make Finalize resize: sound only
    because both resize rules, once true, stay true as the row count grows (physical_create_bf.cpp:383-398)."""
    lib = _lib.load()
    for s in [0, 1, 42, 1000, 20000, 10**7]:
        rows = sorted({0, 1, 64, 65, 512, 1024, 1025, 2048, 2049, s * 8, s * 8 + 1, s * 12, s * 16, s * 16 + 1, 10**9})
        ref = [lib.rpt_bf_needs_resize(s, a) for a in rows]
        assert ref == sorted(ref), (s, ref)  # 0 ... 0 1 ... 1
        L = orc.log_num_blocks(max(s, 1))
        alloc = [orc.needs_resize_alloc(L, a) for a in rows]
        assert alloc == sorted(alloc), (s, alloc)


def test_workspace_size_grows_with_rows():
    lib = _lib.load()
    prev = 0
    for L in [3, 13, 14, 21, 24]:
        prev = 0
        for n in [1, 512, 513, 10**6, 10**9, 2**32 - 1]:
            b = lib.rpt_probe_workspace_bytes(n, L)
            assert b % 256 == 0 and b >= prev and b >= n // 8
            prev = b
    # the partitioned strategy (128 KiB..128 MiB filters) needs records (4 B) + row map (2 B) + pass bits
    assert lib.rpt_probe_workspace_bytes(10**6, 21) >= 6 * 10**6 > lib.rpt_probe_workspace_bytes(10**6, 32)
    # the partitioned insert needs records + run tables; filters it cannot partition need none
    assert lib.rpt_insert_workspace_bytes(10**6, 21) >= 4 * 10**6
    assert lib.rpt_insert_workspace_bytes(10**6, 10) == 0 and lib.rpt_insert_workspace_bytes(10**6, 32) == 0
    # bucketed (filters > 128 MiB): level-1 hash arrays (8 B/row) + level-2 records (4 B/row)
    assert lib.rpt_insert_workspace_bytes(10**6, 26) >= 12 * 10**6
    assert lib.rpt_probe_workspace_bytes(10**6, 26) >= 16 * 10**6 > lib.rpt_probe_workspace_bytes(10**6, 32)


def test_argument_errors_are_reported():
    lib = _lib.load()
    col = _lib.KeyColumn(0, None, None, None)
    assert lib.rpt_bf_insert(None, ctypes.byref(col), 10, None) == _lib.RPT_ERR_INVALID_ARGUMENT
    assert b"null" in lib.rpt_last_error()
    assert lib.rpt_bf_probe(None, ctypes.byref(col), None, 10, None, None, None, 0, None) == _lib.RPT_ERR_INVALID_ARGUMENT
    out = ctypes.c_void_p()
    assert lib.rpt_bf_create_log_blocks(0, 41, ctypes.byref(out)) == _lib.RPT_ERR_INVALID_ARGUMENT
    assert lib.rpt_bf_destroy(None) == 0
    assert lib.rpt_bf_set_probe_strategy(None, 1) == _lib.RPT_ERR_INVALID_ARGUMENT


def test_strategy_support_rules():
    lib = _lib.load()
    for L in range(0, 30):
        assert lib.rpt_probe_strategy_supported(_lib.RPT_PROBE_GATHER, L) == 1
        assert lib.rpt_probe_strategy_supported(_lib.RPT_PROBE_AUTO, L) == 1
        # whole filter in LDS up to 2^14 blocks (128 KiB); 2^15..2^17 (256 KiB..1 MiB): the hybrid, first 128 KiB in LDS
        assert lib.rpt_probe_strategy_supported(_lib.RPT_PROBE_LDS, L) == (L <= 17)
    # partitioned: at least one full LDS slice, at most 1024 slices (128 KiB .. 128 MiB)
    part = [L for L in range(0, 34) if lib.rpt_probe_strategy_supported(_lib.RPT_PROBE_PARTITIONED, L)]
    assert part == list(range(14, 25))
    # bucketed: 1 .. 512 buckets of 32 MiB (32 MiB .. 16 GiB), overlapping the partitioned range
    buck = [L for L in range(0, 40) if lib.rpt_probe_strategy_supported(_lib.RPT_PROBE_BUCKETED, L)]
    assert buck == list(range(22, 32))
    assert lib.rpt_probe_strategy_supported(99, 10) == 0
    assert lib.rpt_synth_probe_keys(None, 1, 10, 0, 10, None) == _lib.RPT_ERR_INVALID_ARGUMENT


def test_testing_hook_absent_from_product():
    # the RCCL-table seam (csrc/rpt_gpu_testing.h) exists only in the test build (tests/loopback)
    lib = _lib.load()
    assert not hasattr(lib, "rpt_testing_set_rccl_api")
    assert not hasattr(lib, "rpt_testing_bucketed_insert_batch")


@pytest.mark.parametrize("world,L", [(1, 30), (2, 3), (2, 20), (3, 25), (8, 24), (8, 30), (8, 31)])
def test_allreduce_workspace_is_bounded(world, L):
    lib = _lib.load()
    b = lib.rpt_allreduce_workspace_bytes(world, L)
    nw = 1 << L
    if world == 1:
        assert b == 256
    else:
        # 256 B + two staging buffers of (W-1) round pieces: <= 32 MiB per peer, <= 1 GiB at C5 (W = 8, 2^30)
        assert b <= 256 + 2 * (world - 1) * (4 << 20) * 8
        assert b >= 256 + 2 * (world - 1) * 8 * min(4 << 20, nw // world - 32)
    if (world, L) == (8, 30):
        assert b <= 1 << 30
    assert lib.rpt_allreduce_workspace_bytes(0, L) == 0
