"""Diagnostics: C3 (or C5 with MG_SWEEP_CONFIG=c5) step time (device wall, HIP
events) under engine options, all on one GPU in one process so the variants
share the box.
usage: variant_sweep.py [n_reads]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from metagenomics_amd import synth  # noqa: E402
from metagenomics_amd.overlap import Dataset, OverlapEngine  # noqa: E402

if os.environ.get("MG_SWEEP_CONFIG") == "c5":  # bench.py CONFIGS["c5"]
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    c, L = synth.metagenome_read_set(n, 100, 250, 100, n * 175 // 20, 55)
else:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    c, L = synth.uniform_read_set(n, 150, n * 150 // 20, seed=31)
ds = Dataset.from_codes(c, L, 50, nthreads=16)
del c, L
VARIANTS = json.loads(os.environ["MG_VARIANTS"]) if os.environ.get("MG_VARIANTS") else [{}, {}]
res = []
for opts in VARIANTS:
    e = OverlapEngine(0)
    for k, v in opts.items():
        e.set_option(k, v)
    e.upload(ds)
    e.upload(ds)  # the second upload: layout buffers and kernels warm
    lay = e.timings()["layout_ms"]
    ts = []
    rows = 0
    for _ in range(6):
        e.build_index(50, 31)
        e.mark_contained(copy=False)
        rows = e.find_overlaps()
        t = e.timings()
        ts.append((t["total_ms"], t["index_ms"], t["scan_ms"], t["probe_ms"], t["contained_ms"], t["verify_ms"]))
    e.close()
    best = min(ts[1:])
    r = {"opts": opts, "rows": rows, "layout_ms": round(lay, 3), "total_ms": round(best[0], 3), "index_ms": round(best[1], 3),
         "scan_ms": round(best[2], 3), "probe_ms": round(best[3], 3), "contained_ms": round(best[4], 3), "verify_ms": round(best[5], 3)}
    res.append(r)
    print(json.dumps(r), flush=True)
