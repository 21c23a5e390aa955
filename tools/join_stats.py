"""Diagnostics: work counters (runs probed, index entries examined, partners
verified, rows) of the join and the cell path on C3 (or n reads)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from metagenomics_amd import synth  # noqa: E402
from metagenomics_amd.overlap import Dataset, OverlapEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
c, L = synth.uniform_read_set(n, 150, n * 150 // 20, seed=31)
ds = Dataset.from_codes(c, L, 50, nthreads=16)
for opts in ({}, {"join": 0}):
    e = OverlapEngine(0)
    for k, v in opts.items():
        e.set_option(k, v)
    e.set_option("stats", 1)
    e.upload(ds)
    e.build_index(50, 31)
    e.mark_contained(copy=False)
    rows = e.find_overlaps()
    print(json.dumps({"opts": opts, "rows": rows, "counters": e.counters(), "timings": e.timings()}), flush=True)
    e.close()
