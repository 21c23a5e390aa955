"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C restatement (mg_oracle.c).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker.  The product (metagenomics_amd/) never imports this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libmgoracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")

ROW_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("offset", "<u2"), ("orient", "u1"), ("pad", "u1")])

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, u64 = C.c_void_p, C.c_uint64
        L.mgo_dataset_from_files.restype = vp
        L.mgo_dataset_from_files.argtypes = [C.POINTER(C.c_char_p), C.c_int, u64]
        L.mgo_dataset_from_seqs.restype = vp
        L.mgo_dataset_from_seqs.argtypes = [C.c_char_p, vp, u64, u64]
        L.mgo_dataset_from_codes.restype = vp
        L.mgo_dataset_from_codes.argtypes = [vp, u64, vp, u64, u64]
        L.mgo_overlaps_digest.restype = C.c_int
        L.mgo_overlaps_digest.argtypes = [vp, u64, C.c_int, vp, vp, vp, C.POINTER(C.c_double),
                                          C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.mgo_dataset_free.argtypes = [vp]
        L.mgo_num_unique.restype = u64
        L.mgo_num_unique.argtypes = [vp]
        L.mgo_num_reads.restype = u64
        L.mgo_num_reads.argtypes = [vp]
        L.mgo_read.restype = C.c_char_p
        L.mgo_read.argtypes = [vp, u64, C.POINTER(C.c_uint32)]
        L.mgo_frequency.restype = C.c_uint32
        L.mgo_frequency.argtypes = [vp, u64]
        L.mgo_overlaps.restype = C.c_int
        L.mgo_overlaps.argtypes = [vp, u64, vp, C.POINTER(vp), C.POINTER(u64), C.POINTER(C.c_double),
                                   C.POINTER(C.c_double)]
        L.mgo_lookup.restype = u64
        L.mgo_lookup.argtypes = [vp, u64, C.c_char_p, vp, u64]
        L.mgo_free.argtypes = [vp]
        L.mgo_rows_digest.argtypes = [vp, u64, vp]
        L.mgo_super_digest.argtypes = [vp, u64, vp]
        _lib = L
    return _lib


class OracleDataset:
    def __init__(self, h):
        self._h = h

    @classmethod
    def from_files(cls, files, l):
        arr = (C.c_char_p * len(files))(*[f.encode() for f in files])
        h = lib().mgo_dataset_from_files(arr, len(files), l)
        if not h:
            raise IOError(f"oracle cannot read {files}")
        return cls(h)

    @classmethod
    def from_strings(cls, seqs, l):
        data = "".join(seqs).encode()
        off = np.zeros(len(seqs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(s) for s in seqs])
        return cls(lib().mgo_dataset_from_seqs(data, C.c_void_p(off.ctypes.data), len(seqs), l))

    @classmethod
    def from_codes(cls, codes, lens, l):
        """2-bit codes [n, stride] uint8 (A0 C1 G2 T3) + lengths: metagenomics_amd.synth's form."""
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        return cls(lib().mgo_dataset_from_codes(C.c_void_p(codes.ctypes.data), codes.shape[1],
                                                C.c_void_p(lens.ctypes.data), codes.shape[0], l))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.mgo_dataset_free(self._h)
            self._h = None

    @property
    def num_unique(self):
        return int(lib().mgo_num_unique(self._h))

    @property
    def num_reads(self):
        return int(lib().mgo_num_reads(self._h))

    def read(self, rid):
        return lib().mgo_read(self._h, rid, None).decode()

    def frequency(self, rid):
        return int(lib().mgo_frequency(self._h, rid))

    def overlaps(self, l):
        """-> (rows structured array, super[N+1] uint64, t_hash_s, t_disc_s)"""
        n = self.num_unique
        sup = np.zeros(n + 1, dtype=np.uint64)
        rows_p = C.c_void_p()
        nrows = C.c_uint64()
        th, td = C.c_double(), C.c_double()
        rc = lib().mgo_overlaps(self._h, l, C.c_void_p(sup.ctypes.data), C.byref(rows_p), C.byref(nrows),
                                C.byref(th), C.byref(td))
        if rc:
            raise RuntimeError("oracle overlaps failed")
        if nrows.value:
            buf = (C.c_char * (nrows.value * ROW_DTYPE.itemsize)).from_address(rows_p.value)
            rows = np.frombuffer(bytes(buf), dtype=ROW_DTYPE).copy()
        else:
            rows = np.zeros(0, dtype=ROW_DTYPE)
        lib().mgo_free(rows_p)
        return rows, sup, th.value, td.value

    def overlaps_digest(self, l, nthreads, want_super=False):
        """Threaded hot path, digests only (mgo_overlaps_digest): -> (rows digest,
        super digest, super[N+1] or None, {hash_s, contain_s, discovery_s})"""
        rd = np.zeros(4, dtype=np.uint64)
        sd = np.zeros(4, dtype=np.uint64)
        sup = np.zeros(self.num_unique + 1, dtype=np.uint64) if want_super else None
        th, tc, td = C.c_double(), C.c_double(), C.c_double()
        rc = lib().mgo_overlaps_digest(self._h, l, nthreads, C.c_void_p(rd.ctypes.data), C.c_void_p(sd.ctypes.data),
                                       C.c_void_p(sup.ctypes.data) if want_super else None,
                                       C.byref(th), C.byref(tc), C.byref(td))
        if rc:
            raise RuntimeError("oracle overlaps_digest failed")
        d = lambda a: {"n": int(a[0]), "sum": int(a[1]), "xor": int(a[2]), "sum2": int(a[3])}  # noqa: E731
        return d(rd), d(sd), sup, {"hash_s": th.value, "contain_s": tc.value, "discovery_s": td.value}

    def lookup(self, l, key):
        out = np.zeros(1 << 16, dtype=np.uint64)
        n = lib().mgo_lookup(self._h, l, key.encode(), C.c_void_p(out.ctypes.data), out.shape[0])
        return [(int(x & ((1 << 62) - 1)), int(x >> 62)) for x in out[: min(n, out.shape[0])]]


def rows_digest(rows) -> dict:
    """oracle/mg_digest.h over a ROW_DTYPE array (C)."""
    rows = np.ascontiguousarray(rows, dtype=ROW_DTYPE)
    out = np.zeros(4, dtype=np.uint64)
    lib().mgo_rows_digest(C.c_void_p(rows.ctypes.data), rows.shape[0], C.c_void_p(out.ctypes.data))
    return {"n": int(out[0]), "sum": int(out[1]), "xor": int(out[2]), "sum2": int(out[3])}


def super_digest(sup) -> dict:
    sup = np.ascontiguousarray(sup, dtype=np.uint64)
    out = np.zeros(4, dtype=np.uint64)
    lib().mgo_super_digest(C.c_void_p(sup.ctypes.data), max(0, sup.shape[0] - 1), C.c_void_p(out.ctypes.data))
    return {"n": int(out[0]), "sum": int(out[1]), "xor": int(out[2]), "sum2": int(out[3])}


def sorted_tuples(rows) -> np.ndarray:
    order = np.lexsort((rows["offset"], rows["orient"], rows["dst"], rows["src"]))
    r = rows[order]
    return np.stack([r["src"].astype(np.int64), r["dst"].astype(np.int64), r["orient"].astype(np.int64),
                     r["offset"].astype(np.int64)], axis=1)


def readdataset_records(data: bytes) -> list:
    """Dataset::readDataset's record splitting (Dataset.cpp:110-193), restated
    with libstdc++'s getline semantics: getline erases its string only when the
    stream is still good on entry, so after EOF a record keeps the previous
    string (a FASTA file that ends inside a header line yields that header as
    the last record's sequence).  Returns the raw sequence of every record,
    good or bad, in file order (bytes as in the file, before upper-casing).
    Pure Python: small inputs only."""
    if not data or data[:1] not in (b">", b"@"):
        raise ValueError("Unknown input file format.")  # :126-135
    n = len(data)
    st = {"pos": 0, "eof": False, "fail": False}

    def getline(cur: bytes, delim: bytes) -> bytes:
        if st["eof"] or st["fail"]:  # sentry fails: failbit, string untouched
            st["fail"] = True
            return cur
        p = st["pos"]
        q = data.find(delim, p)
        if q < 0:  # runs into EOF
            st["eof"] = True
            if p == n:
                st["fail"] = True
            st["pos"] = n
            return data[p:]
        st["pos"] = q + 1
        return data[p:q]

    recs, text = [], b""
    fasta = data[:1] == b">"
    while not st["eof"]:  # while(!myFile.eof())
        if fasta:
            text = getline(text, b"\n")
            text = getline(text, b">")
            recs.append(text.replace(b"\n", b""))
        else:
            lines = []
            for _ in range(4):
                text = getline(text, b"\n")
                lines.append(text)
            recs.append(lines[1])
    return recs
