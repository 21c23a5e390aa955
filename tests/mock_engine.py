"""TEST INFRASTRUCTURE: a CPU stand-in for the exchange-mode engine interface
(``OverlapEngine.xchg_caps / xchg_begin / xchg_pack / xchg_insert_keys /
xchg_probe / begin_contained / finalize_contained``) so that the multi-rank
orchestration (metagenomics_amd/sharded.py) and its all-to-all plumbing can be
exercised with the gloo backend on CPU.  It does NOT compute overlaps: it
replays a known row multiset (a golden fixture) under the library's routing
rules and its SLOT LAYOUT (include/mg_overlap.h "exchange mode"), so that a test
can check that every record reaches the rank that owns it, that cut streams
are detected and the step rerun, and that the union is unchanged.
"""
from __future__ import annotations

import ctypes

import numpy as np

from metagenomics_amd.overlap import EDGE_DTYPE, MG_KEYS, MG_ROWS, MG_RUNS

NB_LOG2 = 20
REC_DTYPE = np.dtype([("x", "<u8"), ("y", "<u8")])  # 16-B key / run records


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


def write_slots(ptr: int, recs: np.ndarray, owner: np.ndarray, world: int, slot: int, rounds: int,
                counts_ptr: int, self_ptr: int = 0, me: int = -1):
    """The library's slot layout: record i of peer d's stream at ((i // slot) * P + d) * slot + i % slot,
    streams cut at rounds * slot, full lengths into the device (here: host) counts; the stream to
    this rank itself goes to self_ptr (the receive buffer) when given."""
    rb = recs.dtype.itemsize
    cnt = np.zeros(world, np.int64)
    for d in range(world):
        stream = np.ascontiguousarray(recs[owner == d])
        cnt[d] = len(stream)
        for t in range(rounds):
            part = stream[t * slot:(t + 1) * slot]
            if len(part):
                base = self_ptr if (self_ptr and d == me) else ptr
                ctypes.memmove(base + (t * world + d) * slot * rb, part.tobytes(), part.nbytes)
    ctypes.memmove(counts_ptr, cnt.tobytes(), cnt.nbytes)


def read_slots(ptr: int, dtype, world: int, slot: int, rounds: int, counts_ptr: int) -> np.ndarray:
    cnt = np.frombuffer(ctypes.string_at(counts_ptr, 8 * world), dtype=np.int64)
    rb = np.dtype(dtype).itemsize
    parts = []
    for s in range(world):
        for t in range(rounds):
            k = min(max(0, int(cnt[s]) - t * slot), slot)
            if k:
                parts.append(np.frombuffer(ctypes.string_at(ptr + (t * world + s) * slot * rb, k * rb), dtype=dtype))
    return np.concatenate(parts) if parts else np.zeros(0, dtype)


class MockEngine:
    def __init__(self, rank: int, world: int, rows: np.ndarray, n_reads: int, lengths_differ: bool = True,
                 caps=(64, 64, 64)):
        self.rank, self.world = rank, world
        self.all_rows = rows  # the full directed multiset (EDGE_DTYPE)
        self.n_reads = n_reads
        self.lengths_differ = lengths_differ
        self.max_len = 150  # (reads <= 1024 bp: the exchange path, not the long-read fallback)
        self.lo, self.hi = n_reads * rank // world, n_reads * (rank + 1) // world
        self.caps = caps  # small first capacities: the steps exercise the overflow rerun
        self.received_keys = None
        self.sk_ptr = 0
        self.super_keys = None
        self.begins = 0
        self.marks_ptr = 0
        self.marks_seen = False

    @staticmethod
    def record_bytes(what):
        return REC_DTYPE.itemsize if what in (MG_KEYS, MG_RUNS) else EDGE_DTYPE.itemsize

    def set_option(self, name, value):
        self.options = getattr(self, "options", {})
        self.options[name] = value

    def num_rows(self):
        return 0 if self.out_rows is None else len(self.out_rows)

    def rows(self, n=None):
        return self.out_rows[: (len(self.out_rows) if n is None else n)].copy()

    def xchg_caps(self, min_overlap, seed_k=0):
        return np.array(self.caps, dtype=np.uint64)

    # one scan of the rank's sources: 4 key records per read + one run per read
    def xchg_begin(self, min_overlap, seed_k=0):
        self.begins += 1
        idx = np.repeat(np.arange(self.lo, self.hi, dtype=np.uint64), 4)
        o = np.tile(np.arange(4, dtype=np.uint64), self.hi - self.lo)
        self.keys = np.zeros(len(idx), REC_DTYPE)
        self.keys["x"] = mix(idx * np.uint64(4) + o)
        self.keys["y"] = (o << np.uint64(32)) | idx
        a = np.arange(self.lo, self.hi, dtype=np.uint64)
        self.runs = np.zeros(len(a), REC_DTYPE)
        self.runs["x"] = mix(a + np.uint64(104729))
        self.runs["y"] = a
        self.out_rows = None

    def xchg_pack(self, what, ptr, slot, rounds, counts_ptr, self_ptr=0):
        if what == MG_KEYS:
            recs, owner = self.keys, bucket_owner(self.keys["x"], self.world)
        elif what == MG_RUNS:
            recs, owner = self.runs, bucket_owner(self.runs["x"], self.world)
        else:
            assert self.out_rows is not None, "rows before the discovery probe"
            recs, owner = self.out_rows, src_owner(self.out_rows["src"], self.n_reads, self.world)
        write_slots(ptr, recs, owner, self.world, slot, rounds, counts_ptr, self_ptr, self.rank)

    def xchg_insert_keys(self, ptr, slot, rounds, counts_ptr):
        recs = read_slots(ptr, REC_DTYPE, self.world, slot, rounds, counts_ptr)
        assert np.all(bucket_owner(recs["x"], self.world) == self.rank), "key record at the wrong rank"
        self.received_keys = recs.copy()

    def xchg_prefix_marks(self, ptr):
        """marks of this rank's own "offset-0 containments": read (3 a + 1) mod n for
        every source a; xchg_probe(contain) checks that the caller all-reduced them"""
        self.marks_ptr = ptr or 0
        if ptr:
            m = np.zeros(self.n_reads, np.uint8)  # (the library writes every read's mark)
            a = np.arange(self.lo, self.hi, dtype=np.int64)
            m[(3 * a + 1) % self.n_reads] = 1
            ctypes.memmove(ptr, m.tobytes(), m.nbytes)

    def begin_contained(self, ptr):
        self.marks_ptr = 0
        self.sk_ptr = ptr or 0
        if ptr:
            ctypes.memset(ptr, 0, self.n_reads * 8)
        return self.lengths_differ

    def xchg_probe(self, contain, ptr, slot, rounds, counts_ptr):
        recs = read_slots(ptr, REC_DTYPE, self.world, slot, rounds, counts_ptr)
        assert np.all(bucket_owner(recs["x"], self.world) == self.rank), "run record at the wrong rank"
        a = recs["y"].astype(np.int64)
        if contain and self.marks_ptr:  # every rank's marks, MAX-all-reduced by the caller
            m = np.frombuffer(ctypes.string_at(self.marks_ptr, self.n_reads), dtype=np.uint8)
            want = np.zeros(self.n_reads, np.uint8)
            want[(3 * np.arange(self.n_reads, dtype=np.int64) + 1) % self.n_reads] = 1
            assert np.array_equal(m, want), "prefix marks not all-reduced over the ranks"
            self.marks_seen = True
        if contain:  # partial maxima the all-reduce must combine
            sk = np.frombuffer(ctypes.string_at(self.sk_ptr, self.n_reads * 8), dtype=np.int64).copy()
            np.maximum.at(sk, (a * 7) % self.n_reads, a + 1)
            ctypes.memmove(self.sk_ptr, sk.tobytes(), sk.nbytes)
            return
        # every row is "discovered" by the rank that probed min(src, dst)'s run
        mine = np.isin(np.minimum(self.all_rows["src"], self.all_rows["dst"]).astype(np.int64) - 1, a)
        self.out_rows = self.all_rows[mine]

    def xchg_probe_own(self, ptr, slot, rounds, counts_ptr):
        """the split discovery probe's first part: this rank's own stream is already in its
        receive buffer (the pack wrote it there); the mock checks that and probes nothing yet"""
        cnt = np.frombuffer(ctypes.string_at(counts_ptr, 8 * self.world), dtype=np.int64)
        own = self.runs[bucket_owner(self.runs["x"], self.world) == self.rank]
        assert int(cnt[self.rank]) == len(own)
        rb = REC_DTYPE.itemsize
        got = b"".join(ctypes.string_at(ptr + (t * self.world + self.rank) * slot * rb,
                                        min(slot, max(0, len(own) - t * slot)) * rb) for t in range(rounds))
        # (a stream longer than rounds * slot is cut: the step reruns with grown capacities)
        assert got == own[: rounds * slot].tobytes(), "own run stream not in the receive buffer before the exchange"
        self.own_probes = getattr(self, "own_probes", 0) + 1

    def finalize_contained(self, copy=False):
        if self.sk_ptr:
            self.super_keys = np.frombuffer(ctypes.string_at(self.sk_ptr, self.n_reads * 8), dtype=np.int64).copy()
        self.sk_ptr = 0
        return None


def expected_super_keys(n_reads: int) -> np.ndarray:
    sk = np.zeros(n_reads, np.int64)
    a = np.arange(n_reads, dtype=np.int64)
    np.maximum.at(sk, (a * 7) % n_reads, a + 1)
    return sk
