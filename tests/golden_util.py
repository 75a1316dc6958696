"""Loader for tests/golden/ (Arrow BlockedBloomFilter golden vectors, see tests/golden/README.md)
and numpy re-generation of each case's seeded inputs."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLDEN64 = np.uint64(0x9E3779B97F4A7C15)


def mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def sm64(seed: int, i) -> np.ndarray:
    i = np.asarray(i, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(np.uint64(seed) + (i + np.uint64(1)) * GOLDEN64)


def murmur64(x) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    c = np.uint64(0xD6E8FEB86659FD93)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(32))
        x = x * c
        x = x ^ (x >> np.uint64(32))
        x = x * c
        x = x ^ (x >> np.uint64(32))
    return x


NULL_HASH = np.uint64(0xBF58476D1CE4E5B9)


def validity_words(valid: np.ndarray) -> np.ndarray:
    """DuckDB ValidityMask words from a bool row mask."""
    n = valid.size
    nw = (n + 63) // 64
    bits = np.zeros(nw * 64, dtype=np.uint64)
    bits[:n] = valid.astype(np.uint64)
    return (bits.reshape(nw, 64) << np.arange(64, dtype=np.uint64)).sum(axis=1, dtype=np.uint64)


class KeyCase:
    """Inputs of a `kind: keys` golden case (streams documented in gen_arrow_golden.cc)."""

    def __init__(self, inp: dict):
        seed, n, m = inp["seed"], inp["n"], inp["m"]
        self.width, self.nulls = inp["width"], inp["nulls"]
        raw = sm64(seed, np.arange(n))
        r = np.arange(m)
        pick = (sm64(seed + 1000, r) % np.uint64(2)) == 0
        probe_raw = np.where(pick & (n > 0), sm64(seed, sm64(seed + 2000, r) % np.uint64(max(n, 1))),
                             sm64(seed + 3000, r))
        if self.width == 32:  # low 32 bits, as the generator's static_cast<uint32_t>
            self.keys = (raw & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
            self.probe = (probe_raw & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
        else:
            self.keys = raw.view(np.int64)
            self.probe = probe_raw.view(np.int64)
        if self.nulls:
            k = self.nulls
            self.valid = (np.arange(n) % k) != (k - 1)
            self.probe_valid = (np.arange(m) % k) != (k - 1)
        else:
            self.valid = self.probe_valid = None
        self.size_rows = inp["size_rows"]

    def hashes(self, keys, valid) -> np.ndarray:
        u = keys.view(np.uint32).astype(np.uint64) if self.width == 32 else keys.view(np.uint64)
        h = murmur64(u)
        if valid is not None:
            h = np.where(valid, h, NULL_HASH)
        return h


class Golden:
    def __init__(self, d: str = GOLDEN_DIR):
        self.dir = d
        with open(os.path.join(d, "golden_manifest.json")) as f:
            self.manifest = json.load(f)
        self.cases = self.manifest["cases"]

    def bin(self, name: str, dtype) -> np.ndarray:
        return np.fromfile(os.path.join(self.dir, name), dtype=dtype)

    def words(self, case: str) -> np.ndarray:
        return self.bin(self.cases[case]["words"], np.uint64)

    def find_bits(self, case: str, m: int) -> np.ndarray:
        bv = self.bin(self.cases[case]["find"]["file"], np.uint8)
        return np.unpackbits(bv, bitorder="little")[:m].astype(bool)

    def inputs(self, case: str):
        """(build hashes, probe hashes, key-case or None) for any case kind."""
        c = self.cases[case]
        inp = c["inputs"]
        kind = inp["kind"]
        if kind == "hashes":
            h = np.array([int(x, 0) for x in inp["hashes"]], dtype=np.uint64)
            p = np.array([int(x, 0) for x in inp["probe"]], dtype=np.uint64)
            return h, p, None
        if kind == "raw":
            n, m = inp["n"], inp["m"]
            h = sm64(0xABC, np.arange(n))
            r = np.arange(m)
            p = np.where(r % 3 == 0, h[sm64(0xABD, r) % np.uint64(n)], sm64(0xABE, r))
            return h, p, None
        if kind == "keys":
            kc = KeyCase(inp)
            return kc.hashes(kc.keys, kc.valid), kc.hashes(kc.probe, kc.probe_valid), kc
        if kind == "fold":
            if case == "fold_200k_dup1000":
                i = np.arange(200000)
                h = murmur64(sm64(21, i % 1000))
                r = np.arange(20000)
                p = murmur64(np.where(r % 2 == 1, sm64(21, sm64(22, r) % np.uint64(1000)), sm64(23, r)))
                return h, p, None
            if case == "fold_100k_3keys":
                return murmur64(np.array([1, 2, 3], dtype=np.uint64)), murmur64(np.arange(4096, dtype=np.uint64)), None
            if case == "fold_dense_noop":
                return sm64(0xABC, np.arange(100000)), None, None
        raise KeyError(case)

    def size_rows(self, case: str) -> int:
        inp = self.cases[case]["inputs"]
        if "size_rows" in inp:
            return inp["size_rows"]
        return inp["n"]
