#!/usr/bin/env python3
"""C3 step time against the minimizer (seed) length k: the configs' k has no
reference counterpart (any k <= l - 1 gives the same discovery set),
so this measures what the seed length alone costs or saves.  Each k: 1 warm-up
step, then 5 timed steps on one context; rows must equal the k = 31 count and
the rows digest must equal tests/golden/c3.json.

usage: seedk_ab.py K [K ...]"""
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

    ks = [int(x) for x in sys.argv[1:]] or [31]
    cfg = bench.CONFIGS["c3"]
    l = cfg[4]
    ds, _, _, _ = bench.make_dataset(cfg, 16, "c3")
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "c3.json")))
    e = OverlapEngine(0)
    e.upload(ds)
    for rep in range(2):
        for k in ks:
            e.set_option("stats", 1)
            e.build_index(l, k)
            e.mark_contained(copy=False)
            rows = e.find_overlaps()
            cnt = e.counters()
            e.set_option("stats", 0)
            dig = e.rows_digest()
            torch.cuda.synchronize(0)
            t0 = time.perf_counter()
            dev = {"index_ms": 0.0, "scan_ms": 0.0, "probe_ms": 0.0, "total_ms": 0.0}
            for _ in range(5):
                e.build_index(l, k)
                e.mark_contained(copy=False)
                e.find_overlaps()
                t = e.timings()
                for kk in dev:
                    dev[kk] += t[kk] / 5
            torch.cuda.synchronize(0)
            ms = (time.perf_counter() - t0) * 1e3 / 5
            print(json.dumps({"k": k, "rep": rep, "ms_per_step": round(ms, 3), "rows": rows,
                              "digest_ok": dig == gold["rows"], **{kk: round(v, 3) for kk, v in dev.items()},
                              "runs": cnt.get("runs"), "entries": cnt.get("entries"),
                              "verified": cnt.get("verified")}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
