"""Diagnostics: does a locality-preserving read layout speed up the probe?
Reads are clustered by their canonical global minimizer (smallest hash of
any m-mer or its reverse complement, then its offset), the packed slots are
permuted into that order and the C3 step is timed on both layouts, with the
bucket sort of the runs on and off.  (Relabelled IDs: timing only.)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from metagenomics_amd import synth  # noqa: E402
from metagenomics_amd.overlap import Dataset, OverlapEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
m = 31
c, L = synth.uniform_read_set(n, 150, n * 150 // 20, seed=31)
ds = Dataset.from_codes(c, L, 50, nthreads=16)
words, lens = ds.packed()
words = np.array(words)
lens = np.array(lens)
N, wpr = words.shape
t0 = time.time()
M1 = np.uint64((1 << 62) - 1)
gm = np.empty(N, np.uint64)
gp = np.empty(N, np.int64)
CH = 400_000
for s in range(0, N, CH):
    w = words[s:s + CH]
    k = w.shape[0]
    codes = np.empty((k, 150), np.uint64)
    for b in range(150):
        codes[:, b] = (w[:, b >> 5] >> np.uint64(62 - 2 * (b & 31))) & np.uint64(3)
    P = 150 - m + 1
    fw = np.zeros((k, P), np.uint64)
    rc = np.zeros((k, P), np.uint64)
    for i in range(m):
        fw = ((fw << np.uint64(2)) | codes[:, i:i + P]) & M1
        rc = rc | ((np.uint64(3) - codes[:, i:i + P]) << np.uint64(2 * i))
    with np.errstate(over="ignore"):
        hf = (fw * np.uint64(0x9E3779B97F4A7C15)) ^ (fw >> np.uint64(29))
        hr = (rc * np.uint64(0x9E3779B97F4A7C15)) ^ (rc >> np.uint64(29))
        hf = hf * np.uint64(0xBF58476D1CE4E5B9)
        hr = hr * np.uint64(0xBF58476D1CE4E5B9)
    h = np.minimum(hf, hr)
    gm[s:s + k] = h.min(axis=1)
    gp[s:s + k] = h.argmin(axis=1)
order = np.lexsort((gp, gm))
print("cluster keys + order", round(time.time() - t0, 1), "s", flush=True)
layouts = {"id": (words, lens), "cluster": (words[order], lens[order])}
res = []
for name, (wv, lv) in layouts.items():
    for sort_runs in (1, 0, 1, 0):
        e = OverlapEngine(0)
        e.set_option("sort_runs", sort_runs)
        e.upload_packed(wv, lv)
        ts = []
        for _ in range(5):
            e.build_index(50, 31)
            e.mark_contained(copy=False)
            rows = e.find_overlaps()
            t = e.timings()
            ts.append((t["total_ms"], t["index_ms"], t["sort_ms"], t["probe_ms"]))
        e.close()
        b = min(ts[1:])
        r = {"layout": name, "sort_runs": sort_runs, "rows": rows, "total_ms": round(b[0], 3),
             "index_ms": round(b[1], 3), "sort_ms": round(b[2], 3), "probe_ms": round(b[3], 3)}
        res.append(r)
        print(json.dumps(r), flush=True)
