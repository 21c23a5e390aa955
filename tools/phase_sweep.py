"""Diagnostics: time the discovery kernel stopped after each phase (C3 by default)."""
import os, sys, json, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from metagenomics_amd import synth
from metagenomics_amd.overlap import Dataset, OverlapEngine
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
G = n * 150 // 20
c, L = synth.uniform_read_set(n, 150, G, seed=31)
ds = Dataset.from_codes(c, L, 50, nthreads=16)
eng = OverlapEngine(0)
eng.upload(ds)
eng.build_index(50, 31)
eng.mark_contained(copy=False)
res = {}
extra = [("max_blocks", int(x)) for x in sys.argv[2:]]
for opt in [None] + extra:
    if opt: eng.set_option(*opt)
    for ph in [1, 2, 3, 4, 5, 6, 7]:
        eng.set_option("phase_limit", ph)
        ts = []
        for _ in range(3):
            eng.find_overlaps()
            t = eng.timings()
            ts.append((t["probe_ms"], t.get("scan_ms", 0.0), t.get("probe_ms", 0.0)))
        best = min(ts)
        res[f"{opt}:{ph}"] = best[0]
        print(opt, "phase", ph, "overlap_ms", round(best[0], 3), "scan", round(best[1], 3),
              "probe", round(best[2], 3), flush=True)
eng.set_option("phase_limit", 99)
print(json.dumps(res))
