"""Diagnostic: GPU rows vs golden/oracle on fixtures; prints set differences."""
import sys, os, collections
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from conftest import fixture_input, golden_rows, load_meta
from metagenomics_amd.overlap import Dataset, OverlapEngine, rows_to_tuples

eng = OverlapEngine(0)
for name in sys.argv[1:] or ["tworead", "small", "highdup", "tandem", "mixed"]:
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    eng.upload(ds); eng.build_index(meta["l"]); sup = eng.mark_contained()
    n = eng.find_overlaps(); rows = eng.rows(n)
    t = rows_to_tuples(rows); g = golden_rows(name)
    ct = collections.Counter(map(tuple, t.tolist())); cg = collections.Counter(map(tuple, g.tolist()))
    miss = cg - ct; extra = ct - cg
    print(f"{name}: gpu {len(t)} golden {len(g)} missing {sum(miss.values())} extra {sum(extra.values())} "
          f"super_ok {({str(i): int(s) for i, s in enumerate(sup) if s} == meta['super'])}")
    mo = collections.Counter(k[2] for k in miss.elements()); eo = collections.Counter(k[2] for k in extra.elements())
    print("  missing by orient", dict(mo), "extra by orient", dict(eo))
    print("  missing sample", list(miss.items())[:6]); print("  extra sample", list(extra.items())[:6])
    print("  timings", eng.timings())
