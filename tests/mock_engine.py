"""TEST INFRASTRUCTURE: a CPU stand-in for the exchange-mode engine interface
(``OverlapEngine.key_records / pack / insert_keys / scan_runs / probe_runs /
begin_contained / finalize_contained``) so that the multi-rank orchestration
(metagenomics_amd/sharded.py) and its all-to-all plumbing can be exercised with
the gloo backend on CPU.  It does NOT compute overlaps: it replays a known row
multiset (a golden fixture) under the library's routing rules
(include/mg_overlap.h "exchange mode"), so that a test can check that every
record reaches the rank that owns it and that the union is unchanged.
"""
from __future__ import annotations

import ctypes

import numpy as np

from metagenomics_amd.overlap import EDGE_DTYPE, MG_KEYS, MG_ROWS, MG_RUNS

NB_LOG2 = 20


def mix(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(31)
        x *= np.uint64(0x7FB5D329728EA185)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x81DADEF4BC2DD44D)
        x ^= x >> np.uint64(33)
    return x


def bucket_owner(v: np.ndarray, world: int) -> np.ndarray:
    b = v & np.uint64((1 << NB_LOG2) - 1)
    return ((b * np.uint64(world)) >> np.uint64(NB_LOG2)).astype(np.int64)


def src_owner(src: np.ndarray, n_reads: int, world: int) -> np.ndarray:
    return (src.astype(np.int64) * world - 1) // n_reads


def _read(ptr: int, nbytes: int) -> bytes:
    return ctypes.string_at(ptr, nbytes) if nbytes else b""


class MockEngine:
    def __init__(self, rank: int, world: int, rows: np.ndarray, n_reads: int, lengths_differ: bool = True):
        self.rank, self.world = rank, world
        self.rows = rows  # the full directed multiset (EDGE_DTYPE)
        self.n_reads = n_reads
        self.lengths_differ = lengths_differ
        self.lo, self.hi = n_reads * rank // world, n_reads * (rank + 1) // world
        self._out = None
        self.received_keys = None
        self.sk_ptr = 0
        self.super_keys = None

    def _group(self, recs: np.ndarray, owner: np.ndarray) -> np.ndarray:
        order = np.argsort(owner, kind="stable")
        self._out = recs[order]
        return np.bincount(owner, minlength=self.world).astype(np.uint64)

    # HashTable::insertDataset: 4 key records per source read
    def key_records(self, min_overlap, seed_k, world):
        idx = np.repeat(np.arange(self.lo, self.hi, dtype=np.uint64), 4)
        o = np.tile(np.arange(4, dtype=np.uint64), self.hi - self.lo)
        v = mix(idx * np.uint64(4) + o)
        recs = np.stack([v, (o << np.uint64(32)) | idx], axis=1) if len(idx) else np.zeros((0, 2), np.uint64)
        return self._group(recs, bucket_owner(recs[:, 0], world) if len(idx) else np.zeros(0, np.int64))

    def pack(self, what, ptr, cap):
        data = np.ascontiguousarray(self._out).tobytes()
        assert len(data) <= max(1, cap) * (12 if what == MG_ROWS else 16)
        if data:
            ctypes.memmove(ptr, data, len(data))

    def insert_keys(self, ptr, n):
        recs = np.frombuffer(_read(ptr, n * 16), dtype=np.uint64).reshape(-1, 2)
        assert np.all(bucket_owner(recs[:, 0], self.world) == self.rank), "key record at the wrong rank"
        self.received_keys = recs.copy()

    def begin_contained(self, ptr):
        self.sk_ptr = ptr or 0
        if ptr:
            ctypes.memset(ptr, 0, self.n_reads * 8)
        return self.lengths_differ

    def scan_runs(self, contain, world):
        a = np.arange(self.lo, self.hi, dtype=np.uint64)
        v = mix(a + np.uint64(7919 if contain else 104729))
        recs = np.stack([v, a], axis=1) if len(a) else np.zeros((0, 2), np.uint64)
        return self._group(recs, bucket_owner(v, world))

    def probe_runs(self, contain, ptr, n, world):
        recs = np.frombuffer(_read(ptr, n * 16), dtype=np.uint64).reshape(-1, 2)
        assert np.all(bucket_owner(recs[:, 0], self.world) == self.rank), "run record at the wrong rank"
        a = recs[:, 1].astype(np.int64)
        if contain:  # partial maxima the all-reduce must combine
            sk = np.frombuffer(_read(self.sk_ptr, self.n_reads * 8), dtype=np.int64).copy()
            tgt = (a * 7) % self.n_reads
            np.maximum.at(sk, tgt, a + 1)
            ctypes.memmove(self.sk_ptr, sk.tobytes(), sk.nbytes)
            return np.zeros(world, np.uint64)
        # every row is "discovered" by the rank that probed min(src, dst)'s run
        mine = np.isin(np.minimum(self.rows["src"], self.rows["dst"]).astype(np.int64) - 1, a)
        out = self.rows[mine]
        return self._group(out, src_owner(out["src"], self.n_reads, world))

    def finalize_contained(self, copy=False):
        if self.sk_ptr:
            self.super_keys = np.frombuffer(_read(self.sk_ptr, self.n_reads * 8), dtype=np.int64).copy()
        self.sk_ptr = 0
        return None


def expected_super_keys(n_reads: int) -> np.ndarray:
    sk = np.zeros(n_reads, np.int64)
    a = np.arange(n_reads, dtype=np.int64)
    np.maximum.at(sk, (a * 7) % n_reads, a + 1)
    return sk


def rows_from_buffer(buf, n) -> np.ndarray:
    return buf[: n * 12].numpy().view(EDGE_DTYPE).copy() if n else np.zeros(0, EDGE_DTYPE)
