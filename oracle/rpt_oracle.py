"""numpy/ctypes front end of the CPU restatement (oracle/rpt_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker / reported baseline, never as the measured or shipped path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_uint8, c_uint32, c_uint64, c_void_p
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "librpt_oracle.so")

_SIG = {
    "rpt_oracle_mask_table": (None, [c_void_p]),
    "rpt_oracle_mask": (c_uint64, [c_uint32]),
    "rpt_oracle_mask_of_hash": (c_uint64, [c_uint64]),
    "rpt_oracle_log_num_blocks": (c_int, [c_uint64]),
    "rpt_oracle_needs_resize": (c_int, [c_uint64, c_uint64]),
    "rpt_oracle_needs_resize_alloc": (c_int, [c_int, c_uint64]),
    "rpt_oracle_murmur64": (c_uint64, [c_uint64]),
    "rpt_oracle_null_hash": (c_uint64, []),
    "rpt_oracle_hash_i64": (None, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_hash_i32": (None, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_hash_combine_i64": (None, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_hash_combine_i32": (None, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_minmax_i64": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_minmax_i32": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_insert_hashes": (None, [c_void_p, c_int, c_void_p, c_uint64]),
    "rpt_oracle_insert_i64": (None, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_uint64]),
    "rpt_oracle_insert_i32": (None, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_uint64]),
    "rpt_oracle_find_hashes": (None, [c_void_p, c_int, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_lookup_sel_hashes": (c_uint64, [c_void_p, c_int, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_probe_i64": (c_uint64, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_probe_i32": (c_uint64, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rpt_oracle_count_bits": (c_uint64, [c_void_p, c_uint64]),
    "rpt_oracle_fold": (c_int, [c_void_p, c_int]),
    "rpt_oracle_sm64": (c_uint64, [c_uint64, c_uint64]),
    "rpt_oracle_synth_build_keys": (None, [c_uint64, c_uint64, c_void_p]),
    "rpt_oracle_synth_probe_keys": (None, [c_uint64, c_uint32, c_uint64, c_uint64, c_void_p]),
    "rpt_oracle_build_mt": (c_double, [c_void_p, c_int, c_void_p, c_uint64, c_int]),
    "rpt_oracle_probe_mt": (c_double, [c_void_p, c_int, c_void_p, c_uint64, c_int, POINTER(c_uint64)]),
    "rpt_oracle_probe_chain_mt": (c_double, [c_void_p, c_void_p, c_void_p, c_int, c_uint64, c_int, POINTER(c_uint64)]),
    "rpt_oracle_set_probe_lag": (None, [c_uint64]),
    "rpt_oracle_set_pin_mode": (None, [c_int]),
    "rpt_oracle_probe_lag": (c_uint64, []),
}

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIG.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def mask_table() -> bytes:
    b = (c_uint8 * 136)()
    lib().rpt_oracle_mask_table(b)
    return bytes(b)


def log_num_blocks(n: int) -> int:
    return lib().rpt_oracle_log_num_blocks(n)


def needs_resize(sized_for: int, actual: int) -> bool:
    return bool(lib().rpt_oracle_needs_resize(sized_for, actual))


def needs_resize_alloc(log_num_blocks: int, actual: int) -> bool:
    """Resize iff the ALLOCATED filter (2^log_num_blocks blocks) gives fewer than 8 bits per actual row."""
    return bool(lib().rpt_oracle_needs_resize_alloc(log_num_blocks, actual))


def hash_keys(keys: np.ndarray, key_sel=None, validity=None) -> np.ndarray:
    keys = np.ascontiguousarray(keys)
    n = key_sel.size if key_sel is not None else keys.size
    out = np.empty(n, dtype=np.uint64)
    fn = lib().rpt_oracle_hash_i64 if keys.dtype.itemsize == 8 else lib().rpt_oracle_hash_i32
    fn(_p(keys), _p(key_sel), _p(validity), n, _p(out))
    return out


def hash_combine(hashes: np.ndarray, keys: np.ndarray, key_sel=None, validity=None) -> np.ndarray:
    """CombineHash(hashes, Hash(col)) for composite keys (bloom_filter.cpp:15-17); returns a new array."""
    keys = np.ascontiguousarray(keys)
    out = np.array(hashes, dtype=np.uint64, copy=True)
    n = key_sel.size if key_sel is not None else keys.size
    if out.size != n:
        raise ValueError("hash / key column length mismatch")
    fn = lib().rpt_oracle_hash_combine_i64 if keys.dtype.itemsize == 8 else lib().rpt_oracle_hash_combine_i32
    fn(_p(keys), _p(key_sel), _p(validity), n, _p(out))
    return out


def hash_columns(columns) -> np.ndarray:
    """HashColumns (bloom_filter.cpp:11-24): columns = [keys | dict(keys=, key_sel=, validity=)]."""
    cols = [c if isinstance(c, dict) else {"keys": c} for c in columns]
    h = hash_keys(cols[0]["keys"], cols[0].get("key_sel"), cols[0].get("validity"))
    for c in cols[1:]:
        h = hash_combine(h, c["keys"], c.get("key_sel"), c.get("validity"))
    return h


def minmax(keys: np.ndarray, key_sel=None, validity=None):
    """(min, max) of the valid keys (TypedUpdateMinMax, physical_create_bf.cpp:86-119) or None."""
    keys = np.ascontiguousarray(keys)
    n = key_sel.size if key_sel is not None else keys.size
    out = np.zeros(2, dtype=np.int64)
    fn = lib().rpt_oracle_minmax_i64 if keys.dtype.itemsize == 8 else lib().rpt_oracle_minmax_i32
    return (int(out[0]), int(out[1])) if fn(_p(keys), _p(key_sel), _p(validity), n, _p(out)) else None


def new_words(log_nb: int) -> np.ndarray:
    return np.zeros(1 << log_nb, dtype=np.uint64)


def insert_hashes(words: np.ndarray, log_nb: int, hashes: np.ndarray) -> None:
    h = np.ascontiguousarray(hashes, dtype=np.uint64)
    lib().rpt_oracle_insert_hashes(_p(words), log_nb, _p(h), h.size)


def insert_keys(words: np.ndarray, log_nb: int, keys: np.ndarray, key_sel=None, validity=None) -> None:
    keys = np.ascontiguousarray(keys)
    n = key_sel.size if key_sel is not None else keys.size
    fn = lib().rpt_oracle_insert_i64 if keys.dtype.itemsize == 8 else lib().rpt_oracle_insert_i32
    fn(_p(words), log_nb, _p(keys), _p(key_sel), _p(validity), n)


def find_hashes(words: np.ndarray, log_nb: int, hashes: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(hashes, dtype=np.uint64)
    bv = np.zeros((h.size + 7) // 8, dtype=np.uint8)
    lib().rpt_oracle_find_hashes(_p(words), log_nb, _p(h), h.size, _p(bv))
    return bv


def lookup_sel_hashes(words: np.ndarray, log_nb: int, hashes: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(hashes, dtype=np.uint64)
    sel = np.empty(max(h.size, 1), dtype=np.uint32)
    c = lib().rpt_oracle_lookup_sel_hashes(_p(words), log_nb, _p(h), h.size, _p(sel))
    return sel[:c]


def probe_keys(words: np.ndarray, log_nb: int, keys: np.ndarray, key_sel=None, validity=None) -> np.ndarray:
    keys = np.ascontiguousarray(keys)
    n = key_sel.size if key_sel is not None else keys.size
    sel = np.empty(max(n, 1), dtype=np.uint32)
    fn = lib().rpt_oracle_probe_i64 if keys.dtype.itemsize == 8 else lib().rpt_oracle_probe_i32
    c = fn(_p(words), log_nb, _p(keys), _p(key_sel), _p(validity), n, _p(sel))
    return sel[:c]


def count_bits(words: np.ndarray) -> int:
    return int(lib().rpt_oracle_count_bits(_p(words), words.size))


def fold(words: np.ndarray, log_nb: int) -> int:
    return lib().rpt_oracle_fold(_p(words), log_nb)


def sm64(seed: int, i: int) -> int:
    return int(lib().rpt_oracle_sm64(seed, i))


def synth_build_keys(n: int, start: int = 0) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.int64)
    lib().rpt_oracle_synth_build_keys(start, n, _p(out))
    return out[:n]


def synth_probe_keys(n: int, n_build: int, p_permille: int = 100, start: int = 0) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.int64)
    lib().rpt_oracle_synth_probe_keys(n_build, p_permille, start, n, _p(out))
    return out[:n]


def build_mt(words: np.ndarray, log_nb: int, keys: np.ndarray, threads: int) -> float:
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    return float(lib().rpt_oracle_build_mt(_p(words), log_nb, _p(keys), keys.size, threads))


def probe_mt(words: np.ndarray, log_nb: int, keys: np.ndarray, threads: int) -> tuple[float, int]:
    keys = np.ascontiguousarray(keys, dtype=np.int64)
    cnt = c_uint64()
    s = lib().rpt_oracle_probe_mt(_p(words), log_nb, _p(keys), keys.size, threads, ctypes.byref(cnt))
    return float(s), int(cnt.value)


def set_probe_lag(lag: int) -> None:
    """Rows between a row's hash + prefetch and its test in the CPU-baseline probe loop (0: the default, 24)."""
    lib().rpt_oracle_set_probe_lag(int(lag))


def set_pin_mode(mode: int) -> None:
    """CPU-baseline thread placement: 0 the OS's, 1 compact (mask order), 2 spread over the affinity mask."""
    lib().rpt_oracle_set_pin_mode(int(mode))


def probe_chain_mt(words: list, log_nbs: list, keys: list, threads: int) -> tuple[float, int]:
    """USE_BF's filter loop per 2048-row vector (rpt_oracle_probe_chain_mt): filter f over column f of the rows
    that passed filters 0..f-1. Returns (seconds, survivors)."""
    k = len(words)
    keys = [np.ascontiguousarray(x, dtype=np.int64) for x in keys]
    n = keys[0].size
    assert len(log_nbs) == k == len(keys) and all(x.size == n for x in keys)
    wp = (ctypes.c_void_p * k)(*[w.ctypes.data for w in words])
    kp = (ctypes.c_void_p * k)(*[x.ctypes.data for x in keys])
    lp = (ctypes.c_int * k)(*log_nbs)
    cnt = c_uint64()
    s = lib().rpt_oracle_probe_chain_mt(wp, lp, kp, k, n, threads, ctypes.byref(cnt))
    return float(s), int(cnt.value)
