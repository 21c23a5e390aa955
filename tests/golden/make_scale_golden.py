#!/usr/bin/env python3
"""Scale golden digests: the REFERENCE itself on the bench's exact workloads.

Writes tests/golden/<name>.json with the order-independent digests
(oracle/mg_digest.h, tests/digest.py) of the directed edge multiset and of the
superReadID vector that the reference's own HashTable::insertDataset +
markContainedReads + insertAllEdgesOfRead loop produces (oracle/_ref/ref_harness
digest, compiled from /root/reference by oracle/Makefile).  Runs in this
container only (the reference does not travel); the -m gpu tests and bench.py
compare the device's digest with these numbers.

  c3  : bench.py CONFIGS["c3"] = 10M x 150 bp, 75 Mb genome, seed 31, l = 50
  c5s : C5-shaped metagenome at the size the reference finishes here:
        5M x 100-250 bp, 100 genomes, 43.75 Mb total (20x), seed 55, l = 50
  c2  : bench.py CONFIGS["c2"] (1M x 150 bp), a quick self-check of the recipe

  c5  : bench.py CONFIGS["c5"] = BASELINE configs[4]: 50M x 100-250 bp, 100
        genomes, 437.5 Mb (20x), seed 55, l = 50.  The reference needs ~10x the
        c5s hours and more memory than this container has, so this one is made
        by the ORACLE (--oracle): oracle/mg_oracle.c's mgo_overlaps_digest, the
        C restatement pinned bit-exact to the reference on every fixture, run
        over source-read ranges in threads (its containment ranges folded in
        source order with the reference's rule, its discovery digests added).
        Before it is trusted, --oracle --check c5s must reproduce the
        reference's own c5s digests.

usage: make_scale_golden.py NAME [NAME ...]            (reference; tens of minutes for c3)
       make_scale_golden.py --oracle [--threads T] NAME  (oracle, threaded)
       make_scale_golden.py --oracle --check NAME       (oracle vs the committed golden)
       make_scale_golden.py --fasta NAME PATH           (only write the workload's FASTA)
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from metagenomics_amd import synth  # noqa: E402

# name: (kind, n, lo, hi, genome_len, n_genomes, seed, l)
SETS = {
    "c2": ("uniform", 1_000_000, 150, 150, 7_500_000, 0, 21, 50),
    "c3": ("uniform", 10_000_000, 150, 150, 75_000_000, 0, 31, 50),
    "c5s": ("meta", 5_000_000, 100, 250, 43_750_000, 100, 55, 50),
    "c5": ("meta", 50_000_000, 100, 250, 437_500_000, 100, 55, 50),
}


def make_codes(name):
    kind, n, lo, hi, G, ng, seed, l = SETS[name]
    if kind == "meta":
        return synth.metagenome_read_set(n, lo, hi, ng, G, seed)
    return synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)


def write_fasta_fast(path, codes, lens):
    """'>r' header line + one sequence line per read (vectorised)."""
    n, hi = codes.shape
    rec = np.zeros((n, hi + 4), dtype=np.uint8)
    rec[:, 0:2] = np.frombuffer(b">r", dtype=np.uint8)
    rec[:, 2] = ord("\n")
    rec[:, 3:3 + hi] = synth.ALPHABET[codes]
    L = lens.astype(np.int64)
    rec[np.arange(n), 3 + L] = ord("\n")
    keep = np.arange(hi + 4)[None, :] < (4 + L)[:, None]
    with open(path, "wb") as f:
        for a in range(0, n, 1 << 20):
            b = min(n, a + (1 << 20))
            f.write(rec[a:b][keep[a:b]].tobytes())


def generator_text(kind):
    return ("synth.metagenome_read_set(n, lo, hi, genomes, genome_len, seed)" if kind == "meta" else
            "synth.uniform_read_set(n, 0, genome_len, seed=seed, lo=lo, hi=hi)")


def oracle_main(names, threads, check):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    for name in names:
        kind, n, lo, hi, G, ng, seed, l = SETS[name]
        t0 = time.time()
        codes, lens = make_codes(name)
        od = oracle.OracleDataset.from_codes(codes, lens, l)
        del codes, lens
        t1 = time.time()
        rd, sd, _, secs = od.overlaps_digest(l, threads)
        res = {
            "name": name,
            "workload": {"kind": kind, "reads": n, "read_len": [lo, hi], "genome_len": G, "genomes": ng,
                         "seed": seed, "min_overlap": l, "generator": generator_text(kind)},
            "recipe": ("oracle/mg_oracle.c mgo_overlaps_digest (the C restatement of insertDataset + "
                       "markContainedReads + ID-order insertAllEdgesOfRead, HashTable.cpp:50-80, "
                       "OverlapGraph.cpp:225-290,529-565; pinned to the reference on every fixture and on "
                       "the reference's own c5s digests), %d threads over source-read ranges" % threads),
            "n_unique": od.num_unique, "n_reads": od.num_reads, "rows": rd, "super": sd,
            "oracle_seconds": dict(secs, dataset_s=round(t1 - t0, 1)), "threads": threads,
            "wall_s": round(time.time() - t0, 1),
        }
        del od
        if check:
            g = json.load(open(os.path.join(HERE, f"{name}.json")))
            ok = all(g[k] == res[k] for k in ("n_unique", "n_reads", "rows", "super"))
            print(json.dumps({"name": name, "check": ok, "oracle": res}), flush=True)
            if not ok:
                sys.exit(1)
            continue
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)


def main():
    if sys.argv[1:2] == ["--fasta"]:
        codes, lens = make_codes(sys.argv[2])
        return write_fasta_fast(sys.argv[3], codes, lens)
    if "--oracle" in sys.argv:
        args = [a for a in sys.argv[1:] if a != "--oracle"]
        check = "--check" in args
        args = [a for a in args if a != "--check"]
        threads = os.cpu_count() or 1
        if "--threads" in args:
            i = args.index("--threads")
            threads = int(args[i + 1])
            del args[i:i + 2]
        return oracle_main(args, threads, check)
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    for name in sys.argv[1:]:
        kind, n, lo, hi, G, ng, seed, l = SETS[name]
        t0 = time.time()
        codes, lens = make_codes(name)
        with tempfile.TemporaryDirectory(dir=os.environ.get("MG_SCRATCH", "/tmp")) as td:
            fa = os.path.join(td, f"{name}.fa")
            write_fasta_fast(fa, codes, lens)
            del codes, lens
            out = os.path.join(td, "d.json")
            subprocess.run([harness, "digest", fa, str(l), out], check=True, stdout=subprocess.DEVNULL)
            d = json.load(open(out))
        res = {
            "name": name,
            "workload": {"kind": kind, "reads": n, "read_len": [lo, hi], "genome_len": G, "genomes": ng,
                         "seed": seed, "min_overlap": l,
                         "generator": ("synth.metagenome_read_set(n, lo, hi, genomes, genome_len, seed)"
                                       if kind == "meta" else
                                       "synth.uniform_read_set(n, 0, genome_len, seed=seed, lo=lo, hi=hi)")},
            "recipe": "oracle/_ref/ref_harness digest (the reference's insertDataset + markContainedReads + "
                      "ID-order insertAllEdgesOfRead, OverlapGraph.cpp:225-290,529-565), digests of oracle/mg_digest.h",
            "n_unique": d["n_unique"], "n_reads": d["n_reads"],
            "rows": {"n": d["directed_rows"], "sum": d["rows_sum"], "xor": d["rows_xor"], "sum2": d["rows_sum2"]},
            "super": {"n": d["contained"], "sum": d["super_sum"], "xor": d["super_xor"], "sum2": d["super_sum2"]},
            "reference_seconds": {k: d[k] for k in ("dataset_s", "hash_s", "contain_s", "discovery_s")},
            "wall_s": round(time.time() - t0, 1),
        }
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
