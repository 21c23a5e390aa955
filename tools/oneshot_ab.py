#!/usr/bin/env python3
"""Per-dataset (one-shot) A/B on C3: upload (H2D + slot layout) then steps, per
variant of the layout options; prints the layout's kernel time and the first
two steps' wall and device times after each upload, so the first step's extra
time can be told from the layout's.

usage: oneshot_ab.py [OPT=VAL,OPT=VAL ...]  (one variant per argument; none = default)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from metagenomics_amd.overlap import OverlapEngine  # noqa: E402


def main():
    import torch

    variants = sys.argv[1:] or [""]
    cfg = bench.CONFIGS["c3"]
    l, k = cfg[4], cfg[5]
    ds, _, _, _ = bench.make_dataset(cfg, 16, "c3")
    for var in variants:
        e = OverlapEngine(0)
        for kv in filter(None, var.split(",")):
            name, val = kv.split("=")
            e.set_option(name, int(val))
        out = {"variant": var or "default", "trials": []}
        for trial in range(4):
            e.upload(ds)
            lay = e.timings()["layout_ms"]
            steps = []
            for s in range(3):
                torch.cuda.synchronize(0)
                t0 = time.perf_counter()
                e.build_index(l, k)
                e.mark_contained(copy=False)
                n = e.find_overlaps()
                torch.cuda.synchronize(0)
                t = e.timings()
                steps.append({"wall_ms": round((time.perf_counter() - t0) * 1e3, 3), "rows": n,
                              **{kk: round(t[kk], 3) for kk in ("total_ms", "index_ms", "scan_ms", "probe_ms")}})
            out["trials"].append({"layout_ms": round(lay, 3), "steps": steps})
        e.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
