"""Diagnostics: C3 index build time with the whole table vs one bucket range
of P (k_index_build computes every key's minimizer either way; only the
owned keys are filed).  usage: index_cost.py [n_reads]"""
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
for P in (1, 2, 8):
    e = OverlapEngine(0)
    e.set_option("overlap_scan", 0)
    e.set_shard(0, P, 0, 0)
    e.upload(ds)
    ts = []
    for _ in range(4):
        e.build_index(50, 31)
        ts.append(e.timings()["index_ms"])
    e.close()
    print(json.dumps({"P": P, "index_ms": round(min(ts[1:]), 3)}), flush=True)
