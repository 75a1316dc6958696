"""Python mirror of the PTBloomFilter seam over librpt_gpu.so, on torch device tensors.

Mirrors the reference interface (src/include/bloom_filter.hpp:22-57):
    Initialize(est_num_rows)            -> BloomFilter(est_num_rows, device=...)
    Insert(chunk, cols)                 -> BloomFilter.insert(keys, key_sel=, validity=)
    LookupSel(chunk, sel, cols, _)      -> BloomFilter.lookup_sel(keys, ...) -> ascending sel
    ReinitializeAndRehash(rows, data)   -> BloomFilter.reinitialize_and_rehash(rows, chunks)
    SizedForRows() / IsEmpty() / finalized_
Errors surface as RptError (the reference raises DuckDB exceptions).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

from ._lib import (
    RPT_KEY_HASH,
    RPT_KEY_I32,
    RPT_KEY_I64,
    BfInfo,
    KeyColumn,
    RptError,
    check,
    load,
)

SEG_ROWS = 512


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(device: torch.device, stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def key_type_of(keys: torch.Tensor, key_type: Optional[int]) -> int:
    if key_type is not None:
        return key_type
    if keys.dtype == torch.int64:
        return RPT_KEY_I64
    if keys.dtype == torch.int32:
        return RPT_KEY_I32
    raise RptError(1, f"unsupported key dtype {keys.dtype}; pass key_type=RPT_KEY_HASH for hashes")


def probe_chain(filters, columns, *, row_sel: Optional[torch.Tensor] = None, n: Optional[int] = None,
                out_sel: Optional[torch.Tensor] = None, out_count: Optional[torch.Tensor] = None,
                stream=None) -> torch.Tensor:
    """USE_BF's filter chain in one launch (rpt_bf_probe_chain): ascending ids (int32) of the rows passing
    every filters[i] on its own key column. columns[i]: a device key tensor, or a dict of make_column's
    arguments (keys, key_type, key_sel, validity). n <= RPT_SMALL_PROBE_ROWS, 1..RPT_MAX_CHAIN filters."""
    if not filters or len(filters) != len(columns):
        raise RptError(1, "one key column per filter, at least one filter")
    cols = [make_column(**c) if isinstance(c, dict) else make_column(c) for c in columns]
    if n is None:
        c0 = columns[0] if isinstance(columns[0], dict) else {"keys": columns[0]}
        n = (row_sel.numel() if row_sel is not None else
             (c0["key_sel"].numel() if c0.get("key_sel") is not None else c0["keys"].numel()))
    if row_sel is not None and (row_sel.element_size() != 4 or not row_sel.is_cuda):
        raise RptError(1, "row_sel must be a 32-bit device tensor")
    device = filters[0].device
    if out_sel is None:
        out_sel = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    if out_count is None:
        out_count = torch.zeros(1, dtype=torch.int64, device=device)
    handles = (ctypes.c_void_p * len(filters))(*[f._h for f in filters])
    arr = (KeyColumn * len(cols))(*cols)
    check(filters[0]._lib.rpt_bf_probe_chain(handles, arr, len(filters), _ptr(row_sel), n, out_sel.data_ptr(),
                                              out_count.data_ptr(), _stream(device, stream)))
    return out_sel[: int(out_count.item())]


def make_column(keys: torch.Tensor, key_type: Optional[int] = None, key_sel: Optional[torch.Tensor] = None,
                validity: Optional[torch.Tensor] = None) -> KeyColumn:
    """rpt_key_column for a FLAT (key_sel None) or DICTIONARY (key_sel uint32/int32) key vector."""
    if not keys.is_cuda:
        raise RptError(1, "keys must be a device tensor")
    if not keys.is_contiguous():
        raise RptError(1, "keys must be contiguous")
    for name, t in (("key_sel", key_sel), ("validity", validity)):
        if t is not None and (not t.is_cuda or not t.is_contiguous() or t.device != keys.device):
            raise RptError(1, f"{name} must be a contiguous tensor on {keys.device}")
    if key_sel is not None and key_sel.element_size() != 4:
        raise RptError(1, "key_sel must be 32-bit")
    if validity is not None and validity.element_size() != 8:
        raise RptError(1, "validity must be 64-bit words")
    return KeyColumn(key_type_of(keys, key_type), keys.data_ptr(), _ptr(key_sel), _ptr(validity))


def validity_from_mask(valid: torch.Tensor) -> torch.Tensor:
    """Pack a bool row mask into DuckDB ValidityMask words (bit i%64 of word i/64 = row i valid)."""
    n = valid.numel()
    nw = (n + 63) // 64
    v = torch.zeros(nw * 64, dtype=torch.int64, device=valid.device)
    v[:n] = valid.to(torch.int64)
    v = v.view(nw, 64)
    shifts = torch.arange(64, device=valid.device, dtype=torch.int64)
    # bit 63 wraps to the sign bit of int64 (two's complement), which is what the device reads.
    return (v << shifts).sum(dim=1, dtype=torch.int64)


class ProbeWorkspace:
    """Device workspace reused across probes (grown on demand)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.buf: Optional[torch.Tensor] = None

    def get_bytes(self, need: int) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < need:
            self.buf = None  # release before growing
            self.buf = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self.buf

    def get(self, n: int, log_num_blocks: int) -> torch.Tensor:
        """Enough for any strategy on a 2^log_num_blocks-block filter."""
        return self.get_bytes(int(load().rpt_probe_workspace_bytes(n, log_num_blocks)))


class BloomFilter:
    """A device-resident blocked Bloom filter (PTBloomFilter)."""

    def __init__(self, est_num_rows: Optional[int] = None, *, log_num_blocks: Optional[int] = None,
                 device=None, lib=None):
        lib = lib if lib is not None else load()  # lib: a build bound by _lib.load_variant (tests)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if self.device.type != "cuda":
            raise RptError(1, "BloomFilter lives on a GPU device")
        h = ctypes.c_void_p()
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if log_num_blocks is not None:
            check(lib.rpt_bf_create_log_blocks(dev, int(log_num_blocks), ctypes.byref(h)))
        else:
            check(lib.rpt_bf_create(dev, int(est_num_rows or 0), ctypes.byref(h)))
        self._h = h
        self._lib = lib
        self._ws = ProbeWorkspace(self.device)
        self._count = torch.zeros(1, dtype=torch.int64, device=self.device)

    # ---- lifecycle -------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.rpt_bf_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def info(self) -> BfInfo:
        i = BfInfo()
        check(self._lib.rpt_bf_get_info(self._h, ctypes.byref(i)))
        return i

    @property
    def log_num_blocks(self) -> int:
        return self.info().log_num_blocks

    @property
    def num_blocks(self) -> int:
        return self.info().num_blocks

    def sized_for_rows(self) -> int:
        return self.info().sized_for_rows

    def is_empty(self) -> bool:
        return not self.info().has_data

    @property
    def finalized(self) -> bool:
        return bool(self.info().finalized)

    @finalized.setter
    def finalized(self, v: bool) -> None:
        check(self._lib.rpt_bf_set_finalized(self._h, int(bool(v))))

    @property
    def probe_strategy(self) -> int:
        """The strategy a probe runs now (RPT_PROBE_*; AUTO resolved by filter size)."""
        v = self._lib.rpt_bf_probe_strategy(self._h)
        if v < 0:
            check(-v)
        return v

    @probe_strategy.setter
    def probe_strategy(self, strategy: int) -> None:
        check(self._lib.rpt_bf_set_probe_strategy(self._h, int(strategy)))

    def workspace_bytes(self, n: int) -> int:
        """Probe workspace for n rows with the strategy this filter would run (AUTO resolved with n)."""
        return int(self._lib.rpt_bf_probe_workspace_bytes(self._h, n))

    def probe_strategy_for(self, n: int) -> int:
        v = self._lib.rpt_bf_probe_strategy_for(self._h, n)
        if v < 0:
            check(-v)
        return v

    def insert_strategy_for(self, n: int) -> int:
        v = self._lib.rpt_bf_insert_strategy_for(self._h, n)
        if v < 0:
            check(-v)
        return v

    def needs_resize(self, actual_rows: int) -> bool:
        """CREATE_BF Finalize's resize predicate on this filter's real allocation: fewer than 8 allocated
        bits per actual row (physical_create_bf.cpp:383; rpt_bf_needs_resize_alloc)."""
        v = self._lib.rpt_bf_needs_resize_alloc(self._h, int(actual_rows))
        if v < 0:
            check(-v)
        return bool(v)

    def set_has_data(self, v: bool) -> None:
        check(self._lib.rpt_bf_set_has_data(self._h, int(bool(v))))

    # ---- build -----------------------------------------------------------------------------
    def insert(self, keys: torch.Tensor, *, key_type: Optional[int] = None, key_sel=None, validity=None,
               n: Optional[int] = None, stream=None, strategy: Optional[int] = None) -> None:
        """PTBloomFilter::Insert. Large batches use the partitioned / bucketed insert (workspace
        allocated here) unless strategy=RPT_INSERT_ATOMIC; results are identical."""
        n = keys.numel() if (n is None and key_sel is None) else (key_sel.numel() if n is None else n)
        col = make_column(keys, key_type, key_sel, validity)
        if strategy is not None:
            check(self._lib.rpt_bf_set_insert_strategy(self._h, int(strategy)))
        ws_bytes = int(self._lib.rpt_bf_insert_workspace_bytes(self._h, n))  # 0: atomic insert
        if ws_bytes:
            ws = torch.empty(ws_bytes, dtype=torch.uint8, device=self.device)
            if isinstance(stream, torch.cuda.Stream):
                ws.record_stream(stream)  # freed below while the insert may still run on `stream`
            check(self._lib.rpt_bf_insert_ws(self._h, ctypes.byref(col), n, ws.data_ptr(), ws_bytes,
                                             _stream(self.device, stream)))
        else:
            check(self._lib.rpt_bf_insert(self._h, ctypes.byref(col), n, _stream(self.device, stream)))

    def reinitialize(self, actual_rows: int) -> None:
        check(self._lib.rpt_bf_reinitialize(self._h, int(actual_rows)))

    def reinitialize_and_rehash(self, actual_rows: int, chunks: Iterable[dict]) -> None:
        """PTBloomFilter::ReinitializeAndRehash (bloom_filter.cpp:34-58): reallocate for
        actual_rows, then re-insert every materialized chunk (dicts of insert() kwargs)."""
        self.reinitialize(actual_rows)
        for ch in chunks:
            ch = dict(ch)
            self.insert(ch.pop("keys"), **ch)

    def clear(self, stream=None) -> None:
        check(self._lib.rpt_bf_clear(self._h, _stream(self.device, stream)))

    def settle(self, stream=None) -> None:
        """Settle a deferred clear now (rpt_bf_settle; before a stream capture reads the filter)."""
        check(self._lib.rpt_bf_settle(self._h, _stream(self.device, stream)))

    def minmax(self, stream=None) -> Optional[tuple[int, int]]:
        """(min, max) of the valid I32/I64 keys inserted so far, or None (the CREATE_BF min/max
        dynamic filter, physical_create_bf.cpp:82-176, computed inside the insert kernels)."""
        mn, mx, has = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
        check(self._lib.rpt_bf_get_minmax(self._h, ctypes.byref(mn), ctypes.byref(mx), ctypes.byref(has),
                                          _stream(self.device, stream)))
        return (mn.value, mx.value) if has.value else None

    def set_minmax(self, value: Optional[tuple[int, int]], stream=None) -> None:
        mn, mx = value if value is not None else (0, 0)
        check(self._lib.rpt_bf_set_minmax(self._h, int(mn), int(mx), int(value is not None),
                                          _stream(self.device, stream)))

    # ---- probe -----------------------------------------------------------------------------
    def probe_async(self, keys: torch.Tensor, *, key_type: Optional[int] = None, key_sel=None, validity=None,
                    row_sel: Optional[torch.Tensor] = None, n: Optional[int] = None,
                    out_sel: Optional[torch.Tensor] = None, out_count: Optional[torch.Tensor] = None,
                    workspace: Optional[torch.Tensor] = None, stream=None):
        """Enqueue a probe; returns (out_sel, out_count) device tensors (count not synchronized)."""
        if n is None:
            n = row_sel.numel() if row_sel is not None else (key_sel.numel() if key_sel is not None else keys.numel())
        col = make_column(keys, key_type, key_sel, validity)
        if row_sel is not None and (row_sel.element_size() != 4 or not row_sel.is_cuda):
            raise RptError(1, "row_sel must be a 32-bit device tensor")
        if out_sel is None:
            out_sel = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        if out_count is None:
            out_count = self._count
        ws = workspace if workspace is not None else self._ws.get_bytes(self.workspace_bytes(n))
        if workspace is None and isinstance(stream, torch.cuda.Stream):
            ws.record_stream(stream)  # the filter's workspace may be regrown (freed) while this probe runs
        check(self._lib.rpt_bf_probe(self._h, ctypes.byref(col), _ptr(row_sel), n, out_sel.data_ptr(),
                                     out_count.data_ptr(), ws.data_ptr(), ws.numel() * ws.element_size(),
                                     _stream(self.device, stream)))
        return out_sel, out_count

    def probe_phase1(self, keys: torch.Tensor, workspace: torch.Tensor, *, n: Optional[int] = None,
                     key_type: Optional[int] = None, key_sel=None, validity=None, row_sel=None, stream=None) -> None:
        """Hash + gather + result bits (rpt_bf_probe_phase1)."""
        if n is None:
            n = row_sel.numel() if row_sel is not None else (key_sel.numel() if key_sel is not None else keys.numel())
        col = make_column(keys, key_type, key_sel, validity)
        check(self._lib.rpt_bf_probe_phase1(self._h, ctypes.byref(col), _ptr(row_sel), n, workspace.data_ptr(),
                                            workspace.numel() * workspace.element_size(),
                                            _stream(self.device, stream)))

    def probe_phase2(self, n: int, out_sel: torch.Tensor, out_count: torch.Tensor, workspace: torch.Tensor, *,
                     row_sel=None, stream=None) -> None:
        """Selection-vector expansion (rpt_bf_probe_phase2)."""
        check(self._lib.rpt_bf_probe_phase2(self._h, _ptr(row_sel), n, out_sel.data_ptr(), out_count.data_ptr(),
                                            workspace.data_ptr(), workspace.numel() * workspace.element_size(),
                                            _stream(self.device, stream)))

    def lookup_sel(self, keys: torch.Tensor, **kw) -> torch.Tensor:
        """LookupSel: ascending ids (int32 tensor) of the rows that may match."""
        sel, cnt = self.probe_async(keys, **kw)
        c = int(cnt.item())
        return sel[:c]

    def find_bits(self, keys: torch.Tensor, *, key_type: Optional[int] = None, key_sel=None, validity=None,
                  n: Optional[int] = None, stream=None) -> torch.Tensor:
        """Arrow Find(...) bit vector as int64 words (bit i of the LSB-first stream = row i)."""
        if n is None:
            n = key_sel.numel() if key_sel is not None else keys.numel()
        nw = ((n + SEG_ROWS - 1) // SEG_ROWS) * (SEG_ROWS // 64)
        out = torch.zeros(max(nw, 1), dtype=torch.int64, device=self.device)
        col = make_column(keys, key_type, key_sel, validity)
        check(self._lib.rpt_bf_find_bits(self._h, ctypes.byref(col), n, out.data_ptr(),
                                         _stream(self.device, stream)))
        return out

    # ---- merge / fold / export -------------------------------------------------------------
    def merge_or(self, other: "BloomFilter", stream=None) -> None:
        check(self._lib.rpt_bf_merge_or(self._h, other._h, _stream(self.device, stream)))

    def count_bits(self) -> int:
        v = ctypes.c_uint64()
        check(self._lib.rpt_bf_count_bits(self._h, ctypes.byref(v)))
        return v.value

    def is_same_as(self, other: "BloomFilter") -> bool:
        """BlockedBloomFilter::IsSameAs on the device (rpt_bf_is_same_as): same geometry, every word equal."""
        same, diff = ctypes.c_int(), ctypes.c_uint64()
        check(self._lib.rpt_bf_is_same_as(self._h, other._h, ctypes.byref(same), ctypes.byref(diff)))
        return bool(same.value)

    def diff_words(self, other: "BloomFilter") -> int:
        """Number of words that differ from `other` (rpt_bf_is_same_as; 2^64 - 1 for different geometry)."""
        same, diff = ctypes.c_int(), ctypes.c_uint64()
        check(self._lib.rpt_bf_is_same_as(self._h, other._h, ctypes.byref(same), ctypes.byref(diff)))
        return diff.value

    def fold(self) -> int:
        v = ctypes.c_int()
        check(self._lib.rpt_bf_fold(self._h, ctypes.byref(v)))
        return v.value

    def export_words(self) -> np.ndarray:
        nw = self.num_blocks
        out = np.zeros(nw, dtype=np.uint64)
        check(self._lib.rpt_bf_export_words(self._h, out.ctypes.data, nw))
        return out

    def import_words(self, words: np.ndarray) -> None:
        w = np.ascontiguousarray(words, dtype=np.uint64)
        check(self._lib.rpt_bf_import_words(self._h, w.ctypes.data, w.size))

    def copy_words_to(self, dst: torch.Tensor, stream=None) -> None:
        check(self._lib.rpt_bf_copy_words_to(self._h, dst.data_ptr(), self.num_blocks, _stream(self.device, stream)))

    def copy_words_from(self, src: torch.Tensor, stream=None) -> None:
        check(self._lib.rpt_bf_copy_words_from(self._h, src.data_ptr(), self.num_blocks,
                                               _stream(self.device, stream)))


def hash_keys(keys: torch.Tensor, *, key_type: Optional[int] = None, key_sel=None, validity=None,
              stream=None) -> torch.Tensor:
    n = key_sel.numel() if key_sel is not None else keys.numel()
    out = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
    col = make_column(keys, key_type, key_sel, validity)
    check(load().rpt_hash_keys(ctypes.byref(col), n, out.data_ptr(), _stream(keys.device, stream)))
    return out[:n]


def hash_columns(columns: Sequence, stream=None) -> torch.Tensor:
    """HashColumns (reference src/bloom_filter.cpp:11-24) for one or more key columns: Hash(col_0),
    then CombineHash with col_1, col_2, ... on the device. Each column is a tensor or a dict of
    make_column kwargs (keys=, key_type=, key_sel=, validity=). Insert / probe the result with
    key_type=RPT_KEY_HASH."""
    cols = [c if isinstance(c, dict) else {"keys": c} for c in columns]
    if not cols:
        raise RptError(1, "hash_columns needs at least one column")
    first = cols[0]
    out = hash_keys(first["keys"], key_type=first.get("key_type"), key_sel=first.get("key_sel"),
                    validity=first.get("validity"), stream=stream)
    n = out.numel()
    for c in cols[1:]:
        cn = c["key_sel"].numel() if c.get("key_sel") is not None else c["keys"].numel()
        if cn != n:
            raise RptError(1, f"composite key columns differ in length ({cn} vs {n})")
        col = make_column(c["keys"], c.get("key_type"), c.get("key_sel"), c.get("validity"))
        check(load().rpt_hash_combine(ctypes.byref(col), n, out.data_ptr(), _stream(out.device, stream)))
    return out


def words_or_slices(dst: torch.Tensor, srcs: torch.Tensor, k: int, n_words: int, stream=None) -> None:
    """dst[:n_words] = OR of k consecutive n_words slices of srcs (device tensors, 64-bit)."""
    check(load().rpt_words_or_slices(dst.data_ptr(), srcs.data_ptr(), int(k), int(n_words),
                                     _stream(dst.device, stream)))


def synth_build_keys(n: int, start: int = 0, device=None, out: Optional[torch.Tensor] = None,
                     stream=None) -> torch.Tensor:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev) if out is None else out
    check(load().rpt_synth_build_keys(out.data_ptr(), start, n, _stream(dev, stream)))
    return out[:n]


def synth_probe_keys(n: int, n_build: int, p_permille: int = 100, start: int = 0, device=None,
                     out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev) if out is None else out
    check(load().rpt_synth_probe_keys(out.data_ptr(), n_build, p_permille, start, n, _stream(dev, stream)))
    return out[:n]


def log_num_blocks_for_rows(n: int) -> int:
    return int(load().rpt_bf_log_num_blocks_for_rows(n))


def needs_resize(sized_for_rows: int, actual_rows: int) -> bool:
    return bool(load().rpt_bf_needs_resize(sized_for_rows, actual_rows))


__all__: Sequence[str] = [
    "BloomFilter",
    "ProbeWorkspace",
    "make_column",
    "validity_from_mask",
    "hash_keys",
    "hash_columns",
    "words_or_slices",
    "synth_build_keys",
    "synth_probe_keys",
    "log_num_blocks_for_rows",
    "needs_resize",
]
