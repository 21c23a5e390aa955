#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output per kernel.

usage: pmc_summary.py OUT.json DIR [DIR ...]
Each DIR holds one rocprofv3 pass (*_counter_collection.csv).  Writes per-kernel
mean counter values per dispatch, and for the discovery kernel the HBM traffic
per launch: FETCH_SIZE and WRITE_SIZE are in KiB (rocprofv3 derived metrics);
on gfx950 FETCH_SIZE counts 64 B per TCC_EA0_RDREQ, which reads exactly half the
bytes of 128-B streaming requests (MI355X_MICROARCH.md §HBM), so both the raw
and the x2-corrected read figures are recorded.

Provenance: the summary records the sha256 (first 16 hex digits) of the native
library the counters were captured with (MG_LIB, else the in-tree
metagenomics_amd/lib/libmgovl.so, which is what the profiled bench loaded), so
bench.py can refuse to quote traffic measured on another build.
"""
import hashlib
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0].strip()


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def library_provenance():
    path = os.environ.get("MG_LIB") or os.path.join(ROOT, "metagenomics_amd", "lib", "libmgovl.so")
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        return {"path": os.path.relpath(path, ROOT), "sha256_16": hashlib.sha256(f.read()).hexdigest()[:16]}


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[2:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", row.get("Kernel-Name", "?")))
                    cname = row.get("Counter_Name", row.get("Counter-Name"))
                    val = float(row.get("Counter_Value", row.get("Counter-Value", 0)))
                    disp = row.get("Dispatch_Id", row.get("Dispatch-Id"))
                    acc[k][cname].append((disp, val))
    res = {}
    disp_n = {}
    for k, cs in acc.items():
        res[k] = {}
        for c, vals in cs.items():
            per = defaultdict(float)
            for disp, v in vals:
                per[disp] += v  # sum over dimensions (XCD/SE instances) per dispatch
            res[k][c] = sum(per.values()) / max(1, len(per))
            disp_n[k] = max(disp_n.get(k, 0), len(per))
    summary = {"kernels": res, "library": library_provenance()}
    per_kernel = {}
    for k, cs in res.items():
        fetch, write = cs.get("FETCH_SIZE"), cs.get("WRITE_SIZE")
        if fetch is not None and write is not None:
            per_kernel[k] = {"fetch_bytes_raw": fetch * 1024, "write_bytes": write * 1024,
                             "traffic_bytes_per_launch": (2 * fetch + write) * 1024,
                             "dispatches": disp_n.get(k, 0)}
    summary["traffic"] = per_kernel
    main_k = [k for k in per_kernel if k.startswith("k_probe") and k.endswith("false>")]
    if main_k:
        k = main_k[0]
        summary["kernel"] = k
        summary.update(per_kernel[k])
        summary["note"] = ("traffic = (2 x FETCH_SIZE + WRITE_SIZE) KiB -> bytes per launch of the dominant "
                           "kernel; FETCH_SIZE x2 per the gfx950 correction (MI355X_MICROARCH.md §HBM)")
    with open(out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True)[:4000])


if __name__ == "__main__":
    main()
