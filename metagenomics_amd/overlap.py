"""Python binding of the in-tree native library ``metagenomics_amd/lib/libmgovl.so``.

Thin ctypes layer over the C-ABI in ``include/mg_overlap.h`` (device hot path)
and ``include/mg_host.h`` (host Dataset mirror).  There is no Python or CPU
implementation of the hot path here: without the library, or without a HIP
device, every call raises.  Used by tests/ and bench.py.
"""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import Iterable, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MG_LIB") or os.path.join(_HERE, "lib", "libmgovl.so")  # MG_LIB: A/B builds (tools/)

# exchange-mode record kinds (include/mg_overlap.h); their sizes on the wire
# come from the library (mg_record_bytes: keys and runs 8 B, rows 12 B)
MG_KEYS, MG_RUNS, MG_ROWS = 0, 1, 2

EDGE_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("offset", "<u2"), ("orient", "u1"), ("flags", "u1")])


class MgError(RuntimeError):
    pass


class _Timings(C.Structure):
    _fields_ = [("pack_ms", C.c_float), ("index_ms", C.c_float), ("contained_ms", C.c_float),
                ("overlap_ms", C.c_float), ("total_ms", C.c_float), ("scan_ms", C.c_float),
                ("probe_ms", C.c_float), ("verify_ms", C.c_float), ("upload_ms", C.c_float),
                ("ingest_ms", C.c_float), ("sort_ms", C.c_float), ("layout_ms", C.c_float)]


class _Counters(C.Structure):
    _fields_ = [("sources", C.c_uint64), ("runs", C.c_uint64), ("entries", C.c_uint64),
                ("verified", C.c_uint64), ("rows", C.c_uint64), ("live_cells", C.c_uint64),
                ("c_runs", C.c_uint64), ("c_entries", C.c_uint64), ("c_verified", C.c_uint64),
                ("c_contained", C.c_uint64), ("scan_runs", C.c_uint64)]


_lib = None


def lib() -> C.CDLL:
    """Load the native library (raises MgError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MgError(f"native library missing: {LIB_PATH} (run __graft_entry__.build())")
    # One HIP runtime per process: torch bundles its own libamdhip64 (same
    # SONAME, libamdhip64.so.7).  Loading torch first makes the library bind to
    # that instance, so device buffers are shared with torch (the multi-GPU
    # exchange buffers, sharded.py) instead of two runtimes fighting over the GPU.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    u64, u32, i32, i64 = C.c_uint64, C.c_uint32, C.c_int, C.c_int64
    vp, P = C.c_void_p, C.POINTER
    sig = {
        "mg_create": (i32, [P(vp), i32]),
        "mg_destroy": (None, [vp]),
        "mg_last_error": (C.c_char_p, [vp]),
        "mg_device_count": (i32, []),
        "mg_upload_reads_packed": (i32, [vp, vp, vp, u64, u32]),
        "mg_upload_reads_ascii": (i32, [vp, C.c_char_p, vp, u64]),
        "mg_num_reads": (u64, [vp]),
        "mg_num_rows": (u64, [vp]),
        "mg_download_reads_packed": (i32, [vp, vp, vp, P(u32)]),
        "mg_read_slots": (i32, [vp, vp]),
        "mg_build_index": (i32, [vp, u32, u32]),
        "mg_lookup_key": (i32, [vp, C.c_char_p, u32, vp, u64, P(u64)]),
        "mg_mark_contained": (i32, [vp, vp]),
        "mg_find_overlaps": (i32, [vp, P(u64)]),
        "mg_copy_rows": (i32, [vp, vp, u64, P(u64)]),
        "mg_set_shard": (i32, [vp, u32, u32, u64, u64]),
        "mg_get_timings": (i32, [vp, P(_Timings)]),
        "mg_get_counters": (i32, [vp, P(_Counters)]),
        "mg_set_option": (i32, [vp, C.c_char_p, i64]),
        "mg_stream": (vp, [vp]),
        "mg_record_bytes": (u32, [i32]),
        "mg_ingest_ascii": (i32, [vp, C.c_char_p, vp, u64, u32, P(u64)]),
        "mg_ingest_codes": (i32, [vp, vp, u64, u64, vp, u32, P(u64)]),
        "mg_dataset_counts": (i32, [vp, P(u64), P(u64)]),
        "mg_download_frequency": (i32, [vp, vp]),
        "mg_xchg_caps": (i32, [vp, u32, u32, vp]),
        "mg_xchg_begin": (i32, [vp, u32, u32]),
        "mg_xchg_pack": (i32, [vp, i32, vp, u64, u32, vp, vp]),
        "mg_xchg_insert_keys": (i32, [vp, vp, u64, u32, vp]),
        "mg_xchg_probe": (i32, [vp, i32, vp, u64, u32, vp]),
        "mg_xchg_probe_own": (i32, [vp, vp, u64, u32, vp]),
        "mg_xchg_keys_first": (i32, [vp]),
        "mg_slots_digest": (i32, [vp, vp, u64, u32, vp, vp]),
        "mg_begin_contained": (i32, [vp, vp, P(i32)]),
        "mg_xchg_prefix_marks": (i32, [vp, vp]),
        "mg_finalize_contained": (i32, [vp, vp]),
        "mg_rows_digest": (i32, [vp, vp, u64, vp]),
        "mg_super_digest": (i32, [vp, vp]),
        "mgh_dataset_from_files": (i32, [P(C.c_char_p), i32, u64, P(vp)]),
        "mgh_dataset_from_codes": (i32, [vp, u64, u64, vp, u64, i32, P(vp)]),
        "mgh_dataset_free": (None, [vp]),
        "mgh_num_reads": (u64, [vp]),
        "mgh_num_unique": (u64, [vp]),
        "mgh_shortest": (u64, [vp]),
        "mgh_longest": (u64, [vp]),
        "mgh_packed": (i32, [vp, P(vp), P(vp), P(u32)]),
        "mgh_read_string": (i64, [vp, u64, C.c_char_p, u64]),
        "mgh_frequency": (u32, [vp, u64]),
        "mgh_find_read": (u64, [vp, C.c_char_p, u64]),
        "mgh_graph_replay": (i32, [vp, u64, vp, u64, u32, P(vp)]),
        "mgh_graph_free": (None, [vp]),
        "mgh_graph_nodes": (u64, [vp]),
        "mgh_graph_edges": (u64, [vp]),
        "mgh_graph_rows": (u64, [vp, vp, u64]),
        "mgh_parse_file": (i32, [C.c_char_p, i32, P(vp), P(vp), P(u64), P(C.c_double)]),
        "mgh_parse_files": (i32, [P(C.c_char_p), i32, i32, P(vp), P(vp), P(u64), P(C.c_double)]),
        "mgh_parse_buffer": (i32, [vp, u64, i32, P(vp), P(vp), P(u64), P(C.c_double)]),
        "mgh_parse_free": (None, [vp]),
        "mgh_parse_set_min_chunk": (None, [u64]),
        "mgh_graph_contract": (i32, [vp, i32, P(u64), P(u64), P(u64)]),
        "mgh_graph_read_unitig": (i32, [C.c_char_p, vp, u64, P(vp)]),
        "mgh_graph_sort_edges": (i32, [vp]),
        "mgh_graph_save_unitig": (i32, [vp, C.c_char_p]),
        "mgh_graph_save_lists": (i32, [vp, C.c_char_p]),
        "mgh_graph_unitig_edges": (u64, [vp, vp, u64, vp, vp, vp, vp, u64, P(u64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name, None)
        if fn is None and os.environ.get("MG_LIB"):  # (an older variant library in an A/B: what it lacks stays unbound)
            continue
        if fn is None:
            raise AttributeError(f"{LIB_PATH}: {name} not exported")
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def device_count() -> int:
    return int(lib().mg_device_count())


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


class Dataset:
    """Host Dataset mirror (Dataset.cpp:39-65 semantics), packed reads in ID order."""

    def __init__(self, handle: C.c_void_p, keepalive=None):
        self._h = handle
        self._keep = keepalive

    @classmethod
    def from_files(cls, files: Sequence[str], min_overlap: int) -> "Dataset":
        arr = (C.c_char_p * len(files))(*[f.encode() for f in files])
        h = C.c_void_p()
        rc = lib().mgh_dataset_from_files(arr, len(files), min_overlap, C.byref(h))
        if rc:
            raise MgError(f"Dataset from {list(files)} failed ({'unreadable' if rc == -1 else 'unknown format'})")
        return cls(h)

    @classmethod
    def from_codes(cls, codes: np.ndarray, lens: np.ndarray, min_overlap: int, nthreads: int = 0) -> "Dataset":
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        n = codes.shape[0]
        stride = codes.shape[1] if codes.ndim == 2 else 0
        h = C.c_void_p()
        rc = lib().mgh_dataset_from_codes(_ptr(codes), n, stride, _ptr(lens), min_overlap, nthreads, C.byref(h))
        if rc:
            raise MgError("Dataset.from_codes failed")
        return cls(h)

    @classmethod
    def from_strings(cls, seqs: Iterable[str], min_overlap: int) -> "Dataset":
        seqs = list(seqs)
        maxlen = max((len(s) for s in seqs), default=1)
        table = np.full(256, 4, dtype=np.uint8)
        for ch, v in zip(b"ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3]):
            table[ch] = v
        codes = np.full((len(seqs), max(maxlen, 1)), 4, dtype=np.uint8)
        lens = np.zeros(len(seqs), dtype=np.uint16)
        for i, s in enumerate(seqs):
            b = np.frombuffer(s.encode(), dtype=np.uint8)
            codes[i, : len(b)] = table[b]
            lens[i] = len(b)
        return cls.from_codes(codes, lens, min_overlap)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.mgh_dataset_free(self._h)
            self._h = None

    @property
    def num_unique(self) -> int:
        return int(lib().mgh_num_unique(self._h))

    @property
    def num_reads(self) -> int:
        return int(lib().mgh_num_reads(self._h))

    @property
    def shortest(self) -> int:
        return int(lib().mgh_shortest(self._h))

    @property
    def longest(self) -> int:
        return int(lib().mgh_longest(self._h))

    def packed(self):
        """(words [N, wpr] uint64, lens [N] uint16) views, ID order."""
        w, l, wpr = C.c_void_p(), C.c_void_p(), C.c_uint32()
        lib().mgh_packed(self._h, C.byref(w), C.byref(l), C.byref(wpr))
        n = self.num_unique
        if n == 0:
            return np.zeros((0, wpr.value), np.uint64), np.zeros(0, np.uint16)
        words = np.ctypeslib.as_array(C.cast(w, C.POINTER(C.c_uint64)), shape=(n * wpr.value,))
        lens = np.ctypeslib.as_array(C.cast(l, C.POINTER(C.c_uint16)), shape=(n,))
        return words.reshape(n, wpr.value), lens

    def read(self, rid: int) -> str:
        n = lib().mgh_read_string(self._h, rid, None, 0)
        if n < 0:
            raise MgError(f"ID {rid} out of bound.")
        buf = C.create_string_buffer(n + 1)
        lib().mgh_read_string(self._h, rid, buf, n + 1)
        return buf.value.decode()

    def frequency(self, rid: int) -> int:
        return int(lib().mgh_frequency(self._h, rid))

    def find(self, s: str) -> int:
        b = s.encode()
        return int(lib().mgh_find_read(self._h, b, len(b)))


class OverlapEngine:
    """One device context (include/mg_overlap.h)."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        rc = L.mg_create(C.byref(h), device)
        if rc == -3:
            raise MgError("no HIP device available: the overlap path has no CPU fallback")
        if rc:
            raise MgError(f"mg_create({device}) failed: {rc}")
        self._h = h
        self.n_reads = 0
        self.lengths_differ = False
        self.max_len = 0  # longest uploaded read (> 1024 bp: long-read kernels, no exchange mode)

    def close(self):
        if getattr(self, "_h", None):
            lib().mg_destroy(self._h)
            self._h = None

    __del__ = close

    def _check(self, rc: int, what: str):
        if rc:
            msg = lib().mg_last_error(self._h)
            raise MgError(f"{what}: {msg.decode() if msg else rc}")

    # --- reads
    def upload(self, ds: Dataset):
        words, lens = ds.packed()
        self.upload_packed(words, lens)

    def upload_packed(self, words: np.ndarray, lens: np.ndarray):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        wpr = words.shape[1] if words.ndim == 2 else 1
        self._check(lib().mg_upload_reads_packed(self._h, _ptr(words), _ptr(lens), lens.shape[0], wpr), "upload")
        self.n_reads = int(lens.shape[0])
        self.lengths_differ = bool(lens.shape[0]) and int(lens.min()) != int(lens.max())
        self.max_len = int(lens.max()) if lens.shape[0] else 0

    def upload_ascii(self, seqs: Sequence[str]):
        data = "".join(seqs).encode()
        off = np.zeros(len(seqs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(s) for s in seqs])
        self._check(lib().mg_upload_reads_ascii(self._h, data, _ptr(off), len(seqs)), "upload_ascii")
        self.n_reads = len(seqs)
        self.lengths_differ = len({len(x) for x in seqs}) > 1
        self.max_len = max((len(x) for x in seqs), default=0)

    def ingest_ascii(self, seqs: Sequence[str] | None = None, min_overlap: int = 0, text: bytes | None = None,
                     offsets: np.ndarray | None = None) -> int:
        """Dataset ingest on the device (mg_ingest_ascii): raw reads -> unique
        canonical reads in ID order, resident for build_index.  Returns the
        number of unique reads."""
        if text is None:
            text = "".join(seqs).encode()
            offsets = np.zeros(len(seqs) + 1, dtype=np.uint64)
            offsets[1:] = np.cumsum([len(s) for s in seqs])
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        nu = C.c_uint64()
        self._check(lib().mg_ingest_ascii(self._h, text, _ptr(offsets), offsets.shape[0] - 1, min_overlap,
                                          C.byref(nu)), "ingest_ascii")
        self._after_ingest()
        return int(nu.value)

    def ingest_files(self, files: Sequence[str], min_overlap: int, nthreads: int = 0) -> dict:
        """Dataset(pe, se, l) on the device from FASTA/FASTQ files: the host
        splits the records (mgh_parse_files: mmap, all threads), the device
        canonicalises, sorts and deduplicates them (mg_ingest_ascii).  The
        record buffers go straight from the splitter to the device.  Returns
        {"n_unique", "n_records", "parse_s", "ingest_s"}."""
        L = lib()
        arr = (C.c_char_p * len(files))(*[os.fsencode(f) for f in files])
        t, o, n, sec = C.c_void_p(), C.c_void_p(), C.c_uint64(), C.c_double()
        rc = L.mgh_parse_files(arr, len(files), nthreads, C.byref(t), C.byref(o), C.byref(n), C.byref(sec))
        if rc:
            raise MgError({-1: f"Unable to open file: {list(files)}", -2: f"Unknown input file format: {list(files)}"}
                          .get(rc, f"parse failed ({rc})"))
        try:
            nu = C.c_uint64()
            t0 = time.perf_counter()
            self._check(L.mg_ingest_ascii(self._h, C.cast(t, C.c_char_p), o, n.value, min_overlap, C.byref(nu)),
                        "ingest_files")
            t1 = time.perf_counter()
        finally:
            L.mgh_parse_free(t)
            L.mgh_parse_free(o)
        self._after_ingest()
        return {"n_unique": int(nu.value), "n_records": int(n.value), "parse_s": sec.value, "ingest_s": t1 - t0}

    def ingest_codes(self, codes: np.ndarray, lens: np.ndarray, min_overlap: int) -> int:
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        stride = codes.shape[1] if codes.ndim == 2 else 0
        nu = C.c_uint64()
        self._check(lib().mg_ingest_codes(self._h, _ptr(codes), lens.shape[0], stride, _ptr(lens), min_overlap,
                                          C.byref(nu)), "ingest_codes")
        self._after_ingest()
        return int(nu.value)

    def _after_ingest(self):
        self.n_reads = int(lib().mg_num_reads(self._h))
        if self.n_reads:
            _, lens = self.download_packed()
            self.lengths_differ = int(lens.min()) != int(lens.max())
            self.max_len = int(lens.max())
        else:
            self.lengths_differ = False
            self.max_len = 0

    def dataset_counts(self):
        g, u = C.c_uint64(), C.c_uint64()
        lib().mg_dataset_counts(self._h, C.byref(g), C.byref(u))
        return int(g.value), int(u.value)

    def frequency(self) -> np.ndarray:
        f = np.zeros(self.n_reads, dtype=np.uint32)
        self._check(lib().mg_download_frequency(self._h, _ptr(f)), "download_frequency")
        return f

    def download_packed(self):
        wpr = C.c_uint32()
        lib().mg_download_reads_packed(self._h, None, None, C.byref(wpr))
        words = np.zeros((self.n_reads, wpr.value), np.uint64)
        lens = np.zeros(self.n_reads, np.uint16)
        self._check(lib().mg_download_reads_packed(self._h, _ptr(words), _ptr(lens), C.byref(wpr)), "download")
        return words, lens

    def slot_of_ids(self) -> np.ndarray:
        """Device slot of each read, indexed by ID - 1 (mg_read_slots)."""
        s = np.zeros(self.n_reads, dtype=np.uint32)
        self._check(lib().mg_read_slots(self._h, _ptr(s)), "read_slots")
        return s.astype(np.int64)

    # --- hot path
    def set_option(self, name: str, value: int):
        self._check(lib().mg_set_option(self._h, name.encode(), int(value)), f"option {name}")

    def set_shard(self, rank: int, nranks: int, read_lo: int = 0, read_hi: int = 0):
        self._check(lib().mg_set_shard(self._h, rank, nranks, read_lo, read_hi), "set_shard")

    def build_index(self, min_overlap: int, seed_k: int = 0):
        self._check(lib().mg_build_index(self._h, min_overlap, seed_k), "build_index")

    def mark_contained(self, copy: bool = True):
        """superReadID per ID (index 0 unused); copy=False keeps it on the device."""
        if not copy:
            self._check(lib().mg_mark_contained(self._h, None), "mark_contained")
            return None
        sup = np.zeros(self.n_reads + 1, dtype=np.uint32)
        self._check(lib().mg_mark_contained(self._h, _ptr(sup)), "mark_contained")
        return sup

    def find_overlaps(self) -> int:
        n = C.c_uint64()
        self._check(lib().mg_find_overlaps(self._h, C.byref(n)), "find_overlaps")
        return int(n.value)

    def rows(self, n_rows: int | None = None) -> np.ndarray:
        if n_rows is None:
            n_rows = self.find_overlaps()
        out = np.zeros(n_rows, dtype=EDGE_DTYPE)
        got = C.c_uint64()
        self._check(lib().mg_copy_rows(self._h, _ptr(out), n_rows, C.byref(got)), "copy_rows")
        return out[: got.value]

    def num_rows(self) -> int:
        """Rows held after the last find_overlaps / xchg_probe(0) (mg_num_rows)."""
        return int(lib().mg_num_rows(self._h))

    def copy_rows_to(self, host_ptr: int, cap: int) -> int:
        """mg_copy_rows into caller-owned host memory (e.g. a pinned buffer of cap * 12 bytes)."""
        got = C.c_uint64()
        self._check(lib().mg_copy_rows(self._h, C.c_void_p(host_ptr), cap, C.byref(got)), "copy_rows")
        return int(got.value)

    def lookup(self, key: str):
        n = C.c_uint64()
        cap = 1024
        while True:
            buf = np.zeros(cap, dtype=np.uint64)
            self._check(lib().mg_lookup_key(self._h, key.encode(), len(key), _ptr(buf), cap, C.byref(n)), "lookup")
            if n.value <= cap:
                return [(int(x & ((1 << 62) - 1)), int(x >> 62)) for x in buf[: n.value]]
            cap = int(n.value)

    # --- exchange mode (one process per GPU; metagenomics_amd/sharded.py drives it).
    # Buffers and counts are device pointers in the slot layout of include/mg_overlap.h.
    def xchg_caps(self, min_overlap: int, seed_k: int = 0) -> np.ndarray:
        c = np.zeros(3, dtype=np.uint64)
        self._check(lib().mg_xchg_caps(self._h, min_overlap, seed_k, _ptr(c)), "xchg_caps")
        return c

    @staticmethod
    def record_bytes(what: int) -> int:
        """Bytes per exchange record of kind what (mg_record_bytes)."""
        return int(lib().mg_record_bytes(what))

    def xchg_begin(self, min_overlap: int, seed_k: int = 0):
        self._check(lib().mg_xchg_begin(self._h, min_overlap, seed_k), "xchg_begin")

    def xchg_pack(self, what: int, dptr: int, slot: int, rounds: int, counts_dptr: int, self_dptr: int = 0):
        """self_dptr: the receive buffer; this rank's own stream is written there directly."""
        self._check(lib().mg_xchg_pack(self._h, what, C.c_void_p(dptr or 0), slot, rounds, C.c_void_p(counts_dptr),
                                       C.c_void_p(self_dptr or 0)), "xchg_pack")

    def xchg_insert_keys(self, dptr: int, slot: int, rounds: int, counts_dptr: int):
        self._check(lib().mg_xchg_insert_keys(self._h, C.c_void_p(dptr), slot, rounds, C.c_void_p(counts_dptr)),
                    "xchg_insert_keys")

    def xchg_probe(self, contain: bool, dptr: int, slot: int, rounds: int, counts_dptr: int):
        self._check(lib().mg_xchg_probe(self._h, int(contain), C.c_void_p(dptr), slot, rounds,
                                        C.c_void_p(counts_dptr)), "xchg_probe")

    def xchg_probe_own(self, dptr: int, slot: int, rounds: int, send_counts_dptr: int):
        """mg_xchg_probe_own: the discovery probe of this rank's own run stream (already in the
        receive buffer after xchg_pack) while the peers' streams travel; xchg_probe(False) then
        probes theirs and appends.  A no-op where the step cannot split (one rank, mixed lengths)."""
        self._check(lib().mg_xchg_probe_own(self._h, C.c_void_p(dptr), slot, rounds, C.c_void_p(send_counts_dptr)),
                    "xchg_probe_own")

    def xchg_prefix_marks(self, marks_dptr: int | None):
        """mg_xchg_prefix_marks: this rank's offset-0 containments now, their marks
        (n_reads bytes) for the caller's MAX all-reduce before xchg_probe(True)."""
        self._check(lib().mg_xchg_prefix_marks(self._h, C.c_void_p(marks_dptr or 0)), "xchg_prefix_marks")

    def begin_contained(self, superkey_dptr: int | None) -> bool:
        need = C.c_int()
        self._check(lib().mg_begin_contained(self._h, C.c_void_p(superkey_dptr or 0), C.byref(need)),
                    "begin_contained")
        return bool(need.value)

    def finalize_contained(self, copy: bool = False):
        if not copy:
            self._check(lib().mg_finalize_contained(self._h, None), "finalize_contained")
            return None
        sup = np.zeros(self.n_reads + 1, dtype=np.uint32)
        self._check(lib().mg_finalize_contained(self._h, _ptr(sup)), "finalize_contained")
        return sup

    # --- parity digests (include/mg_overlap.h; tests/digest.py restates them)
    @staticmethod
    def _digest(a: np.ndarray) -> dict:
        return {"n": int(a[0]), "sum": int(a[1]), "xor": int(a[2]), "sum2": int(a[3])}

    def rows_digest(self, dptr: int | None = None, n: int = 0) -> dict:
        """Digest of the context's rows (dptr None) or of n mg_edge rows at device pointer dptr."""
        out = np.zeros(4, dtype=np.uint64)
        self._check(lib().mg_rows_digest(self._h, C.c_void_p(dptr or 0), n, _ptr(out)), "rows_digest")
        return self._digest(out)

    def slots_digest(self, dptr: int, slot: int, rounds: int, counts_dptr: int) -> dict:
        """Digest of exchange-mode rows received in the slot layout."""
        out = np.zeros(4, dtype=np.uint64)
        self._check(lib().mg_slots_digest(self._h, C.c_void_p(dptr), slot, rounds, C.c_void_p(counts_dptr),
                                          _ptr(out)), "slots_digest")
        return self._digest(out)

    def super_digest(self) -> dict:
        out = np.zeros(4, dtype=np.uint64)
        self._check(lib().mg_super_digest(self._h, _ptr(out)), "super_digest")
        return self._digest(out)

    def timings(self) -> dict:
        t = _Timings()
        lib().mg_get_timings(self._h, C.byref(t))
        return {k: float(getattr(t, k)) for k, _ in _Timings._fields_}

    def counters(self) -> dict:
        c = _Counters()
        lib().mg_get_counters(self._h, C.byref(c))
        return {k: int(getattr(c, k)) for k, _ in _Counters._fields_}

    def stream(self) -> int:
        return int(lib().mg_stream(self._h) or 0)


def replay_graph(rows: np.ndarray, lens: np.ndarray, min_overlap: int):
    """The reference's graph after buildOverlapGraphFromHashTable's exploration
    and transitive reduction (OverlapGraph.cpp:144-204, 574-661), replayed on a
    discovery multiset (mgh_graph_replay, host C++).  Returns (numberOfNodes,
    numberOfEdges, rows of every graph[u] list in list order, u ascending)."""
    rows = np.ascontiguousarray(rows, dtype=EDGE_DTYPE)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    L = lib()
    g = C.c_void_p()
    rc = L.mgh_graph_replay(_ptr(rows), rows.shape[0], _ptr(lens), lens.shape[0], min_overlap - 1, C.byref(g))
    if rc:
        raise MgError(f"graph replay failed ({rc})")
    try:
        n = int(L.mgh_graph_rows(g, None, 0))
        out = np.zeros(n, dtype=EDGE_DTYPE)
        L.mgh_graph_rows(g, _ptr(out), n)
        return int(L.mgh_graph_nodes(g)), int(L.mgh_graph_edges(g)), out
    finally:
        L.mgh_graph_free(g)


def _parse_result(L, rc, t, o, n, what):
    if rc:
        raise MgError({-1: f"Unable to open file: {what}", -2: f"Unknown input file format: {what}"}.get(
            rc, f"parse failed ({rc})"))
    try:
        offs = np.ctypeslib.as_array(C.cast(o, C.POINTER(C.c_uint64)), shape=(n.value + 1,)).copy()
        size = int(offs[-1])
        text = (np.ctypeslib.as_array(C.cast(t, C.POINTER(C.c_uint8)), shape=(size,)).copy() if size
                else np.zeros(0, np.uint8))
    finally:
        L.mgh_parse_free(t)
        L.mgh_parse_free(o)
    return text, offs


def parse_file(path: str, nthreads: int = 0):
    """Dataset::readDataset's record splitting (Dataset.cpp:110-193) on a
    memory-mapped file with all host threads (mgh_parse_file).  Returns
    (text uint8, offsets uint64[n+1], seconds): record i's raw sequence is
    text[offsets[i]:offsets[i+1]], the input of OverlapEngine.ingest_ascii."""
    L = lib()
    t, o, n, sec = C.c_void_p(), C.c_void_p(), C.c_uint64(), C.c_double()
    rc = L.mgh_parse_file(os.fsencode(path), nthreads, C.byref(t), C.byref(o), C.byref(n), C.byref(sec))
    text, offs = _parse_result(L, rc, t, o, n, path)
    return text, offs, sec.value


def parse_buffer(data: bytes, nthreads: int = 0, min_chunk: int = 0):
    """parse_file on bytes in memory; min_chunk > 0 lowers the per-thread chunk
    size (tests: exercises the chunk seams on small inputs)."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    t, o, n, sec = C.c_void_p(), C.c_void_p(), C.c_uint64(), C.c_double()
    L.mgh_parse_set_min_chunk(min_chunk)
    try:
        rc = L.mgh_parse_buffer(_ptr(buf), len(data), nthreads, C.byref(t), C.byref(o), C.byref(n), C.byref(sec))
    finally:
        L.mgh_parse_set_min_chunk(0)
    text, offs = _parse_result(L, rc, t, o, n, "<buffer>")
    return text, offs


UNITIG_EDGE_DTYPE = np.dtype({"names": ["src", "dst", "offset", "n_reads", "orient"],
                              "formats": ["<u4", "<u4", "<u8", "<u4", "u1"],
                              "offsets": [0, 4, 8, 16, 20], "itemsize": 24})


class UnitigGraph:
    """The graph new OverlapGraph(ht) returns (OverlapGraph.cpp:107-218): the
    exploration + transitive reduction replay (mgh_graph_replay), then the
    contraction loop :211-215 (contractCompositePaths + removeDeadEndNodes,
    mgh_graph_contract), on host C++.  main.cpp:48-50's sortEdges +
    saveGraphToFile are sort_edges() / save_unitig()."""

    def __init__(self, rows: np.ndarray, lens: np.ndarray, min_overlap: int, track_locations: bool = True):
        rows = np.ascontiguousarray(rows, dtype=EDGE_DTYPE)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        L = self._L = lib()
        self._g = C.c_void_p()
        t0 = time.perf_counter()
        rc = L.mgh_graph_replay(_ptr(rows), rows.shape[0], _ptr(lens), lens.shape[0], min_overlap - 1,
                                C.byref(self._g))
        if rc:
            raise MgError(f"graph replay failed ({rc})")
        self.replay_nodes, self.replay_edges = int(L.mgh_graph_nodes(self._g)), int(L.mgh_graph_edges(self._g))
        t1 = time.perf_counter()
        it, merged, dead = C.c_uint64(), C.c_uint64(), C.c_uint64()
        rc = L.mgh_graph_contract(self._g, int(track_locations), C.byref(it), C.byref(merged), C.byref(dead))
        if rc:
            self.close()
            raise MgError(f"contraction failed ({rc})")
        self.replay_s, self.contract_s = t1 - t0, time.perf_counter() - t1
        self.iterations, self.merged, self.dead_end_nodes = it.value, merged.value, dead.value

    @classmethod
    def from_unitig_file(cls, path: str, lens: np.ndarray) -> "UnitigGraph":
        """OverlapGraph::readGraphFromFile (OverlapGraph.cpp:1270-1367): the
        .unitig checkpoint of a Dataset with these read lengths back into lists."""
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        self = cls.__new__(cls)
        L = self._L = lib()
        self._g = C.c_void_p()
        rc = L.mgh_graph_read_unitig(os.fsencode(path), _ptr(lens), lens.shape[0], C.byref(self._g))
        if rc:
            raise MgError({-1: f"Unable to open file: {path}"}.get(rc, f"readGraphFromFile failed ({rc})"))
        self.replay_s = self.contract_s = 0.0
        self.replay_nodes = self.replay_edges = None
        self.iterations = self.merged = self.dead_end_nodes = 0
        return self

    @property
    def nodes(self) -> int:
        return int(self._L.mgh_graph_nodes(self._g))

    @property
    def edges(self) -> int:
        return int(self._L.mgh_graph_edges(self._g))

    def sort_edges(self):
        if self._L.mgh_graph_sort_edges(self._g):
            raise MgError("sort_edges failed")

    def save_unitig(self, path: str):
        if self._L.mgh_graph_save_unitig(self._g, os.fsencode(path)):
            raise MgError(f"cannot write {path}")

    def save_lists(self, path: str):
        if self._L.mgh_graph_save_lists(self._g, os.fsencode(path)):
            raise MgError(f"cannot write {path}")

    def unitig_edges(self):
        """(edges[UNITIG_EDGE_DTYPE], read_start, reads, offs, ors) of the current lists in list order."""
        L = self._L
        nr = C.c_uint64()
        n = int(L.mgh_graph_unitig_edges(self._g, None, 0, None, None, None, None, 0, C.byref(nr)))
        e = np.zeros(n, dtype=UNITIG_EDGE_DTYPE)
        st = np.zeros(n, dtype=np.uint64)
        reads = np.zeros(nr.value, dtype=np.uint32)
        offs = np.zeros(nr.value, dtype=np.uint16)
        ors = np.zeros(nr.value, dtype=np.uint8)
        L.mgh_graph_unitig_edges(self._g, _ptr(e), n, _ptr(st), _ptr(reads), _ptr(offs), _ptr(ors), nr.value,
                                 C.byref(nr))
        return e, st, reads, offs, ors

    def close(self):
        if self._g:
            self._L.mgh_graph_free(self._g)
            self._g = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sort_rows(rows: np.ndarray) -> np.ndarray:
    """Canonical order (src, dst, orient, offset) for multiset comparison."""
    order = np.lexsort((rows["offset"], rows["orient"], rows["dst"], rows["src"]))
    return rows[order]


def rows_to_tuples(rows: np.ndarray) -> np.ndarray:
    r = sort_rows(rows)
    return np.stack([r["src"].astype(np.int64), r["dst"].astype(np.int64), r["orient"].astype(np.int64),
                     r["offset"].astype(np.int64)], axis=1)
