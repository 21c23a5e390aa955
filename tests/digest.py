"""Order-independent digests of an edge multiset / superReadID vector (numpy).

Third, independent implementation of the formulas in oracle/mg_digest.h (the
reference harness's `digest` mode) and of the device's mg_rows_digest /
mg_super_digest (include/mg_overlap.h).  All arithmetic is mod 2^64.
"""
from __future__ import annotations

import numpy as np

M1 = np.uint64(0x7FB5D329728EA185)
M2 = np.uint64(0x81DADEF4BC2DD44D)
GOLD = np.uint64(0x9E3779B97F4A7C15)
SALT = np.uint64(0xD6E8FEB86659FD93)


def mix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(31)
        x *= M1
        x ^= x >> np.uint64(27)
        x *= M2
        x ^= x >> np.uint64(33)
    return x


def _fold(h: np.ndarray) -> dict:
    with np.errstate(over="ignore"):
        s = int(np.sum(h, dtype=np.uint64)) if h.size else 0
        s2 = int(np.sum(mix64(h ^ SALT), dtype=np.uint64)) if h.size else 0
    x = int(np.bitwise_xor.reduce(h)) if h.size else 0
    return {"n": int(h.size), "sum": s, "xor": x, "sum2": s2}


def row_hashes(u, v, orient, offset) -> np.ndarray:
    u = np.asarray(u, dtype=np.uint64)
    v = np.asarray(v, dtype=np.uint64)
    k2 = (np.asarray(orient, dtype=np.uint64) << np.uint64(16)) | np.asarray(offset, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(((u << np.uint64(32)) | v) ^ mix64(k2 + GOLD))


def rows_digest(u, v, orient, offset, chunk: int = 1 << 24) -> dict:
    """Digest of directed rows given as four parallel arrays."""
    n = len(u)
    acc = {"n": 0, "sum": 0, "xor": 0, "sum2": 0}
    for a in range(0, max(n, 1), chunk):
        b = min(n, a + chunk)
        if b <= a:
            break
        d = _fold(row_hashes(u[a:b], v[a:b], orient[a:b], offset[a:b]))
        acc = {"n": acc["n"] + d["n"], "sum": (acc["sum"] + d["sum"]) & (2**64 - 1),
               "xor": acc["xor"] ^ d["xor"], "sum2": (acc["sum2"] + d["sum2"]) & (2**64 - 1)}
    return acc


def super_digest(super_ids) -> dict:
    """super_ids[i] = superReadID of read ID i (index 0 unused)."""
    s = np.asarray(super_ids, dtype=np.uint64)
    ids = np.nonzero(s)[0].astype(np.uint64)
    ids = ids[ids > 0]
    return _fold(mix64((ids << np.uint64(32)) | s[ids]))
