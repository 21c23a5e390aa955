#!/usr/bin/env python3
"""Benchmark: overlap edges/sec (+ reads/sec) of the MI355X hot path.

A "step" = one pass of the hot path over the resident read set: index build
(HashTable::insertDataset) + containment (skipped for equal lengths, as in the
reference) + overlap discovery producing the full directed edge multiset in
HBM.  Inputs (2-bit packed reads) are resident in HBM before timing starts.

Default workload = BASELINE.json configs[2] (C3): 10M x 150 bp synthetic
reads, 20x coverage of a 75 Mb random genome, 50 % reverse-complemented,
l = 50, seed k = 31.  Multi-GPU (torchrun, one process per GPU): the same 10M
reads on N GPUs (strong scaling), DESIGN.md §6:
  --multi auto (the default): bucket for one read length on <= 4 ranks, else
    exchange -- the choice DESIGN.md §6c's per-rank tables and xGMI model make
    (profiles/r06_xchg_model_c3.md);
  --multi exchange (north_star's bucket-range design, BASELINE configs[3]):
    each rank owns a bucket range of the index and a source-read range; 8-B
    key records and 8-B window runs move to their bucket owners with
    equal-split RCCL all-to-alls over xGMI (torch.distributed "nccl"), ordered
    on the engine's HIP stream; every rank keeps the rows it verifies
    (--route-rows: they move on to their src owners);
  --multi bucket: each rank owns a bucket range of the index and scans EVERY
    read, filing and keeping only its buckets' keys and runs, then probes
    them; no data-path collective (SURVEY §8(e) alternative (i)): the scan
    does not divide by P, but nothing crosses a link;
  --multi replicated: every rank builds the whole index and discovers from
    its source-read range; no data-path collective; SURVEY §8(e) alternative
    (ii), kept as the comparison point (its index build and containment pass
    do not divide by P).
--sim-world P runs all P ranks of the chosen mode inside one process on one
GPU (replicated / bucket: each rank timed alone, step = slowest rank;
exchange: buffers exchanged on the device).

Prints ONE JSON line (rank 0).  See DESIGN.md §5 for the roofline numbers.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from metagenomics_amd import synth  # noqa: E402
from metagenomics_amd.overlap import Dataset, OverlapEngine  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec 8.0 TB/s)

CONFIGS = {
    # name: (n_reads, read_len lo, hi, genome_len, l, k, seed, description)
    "c1": (100_000, 100, 100, 500_000, 40, 21, 7, "C1: 100k x 100 bp, l=40, k=21"),
    "c2": (1_000_000, 150, 150, 7_500_000, 50, 31, 21, "C2: 1M x 150 bp, l=50, k=31"),
    "c3": (10_000_000, 150, 150, 75_000_000, 50, 31, 31, "C3: 10M x 150 bp, l=50, k=31"),
    # C5 (BASELINE configs[4]): metagenome of 100 random genomes, log-normal
    # abundance, 437.5 Mb in total (20x mean coverage), 100-250 bp reads
    "c5": (50_000_000, 100, 250, 437_500_000, 50, 31, 55,
           "C5: 50M x 100-250 bp metagenome (100 genomes), l=50, k=31"),
    # C5-shaped at the size the reference itself finishes in the build
    # container (tests/golden/c5s.json pins it)
    "c5s": (5_000_000, 100, 250, 43_750_000, 50, 31, 55,
            "C5-shaped: 5M x 100-250 bp metagenome (100 genomes), l=50, k=31"),
}
META_GENOMES = {"c5": 100, "c5s": 100}
GOLDEN_DIGEST = os.path.join(ROOT, "tests", "golden", "{}.json")  # reference digests (make_scale_golden.py)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_dataset(cfg, nthreads, name=""):
    n, lo, hi, G, l, k, seed, _ = cfg
    t0 = time.time()
    if name in META_GENOMES:
        c, L = synth.metagenome_read_set(n, lo, hi, META_GENOMES[name], G, seed)
    else:
        c, L = synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)
    t1 = time.time()
    ds = Dataset.from_codes(c, L, l, nthreads=nthreads)
    t2 = time.time()
    log(f"[bench] generated {n} reads in {t1 - t0:.1f}s, Dataset ingest {t2 - t1:.1f}s, unique {ds.num_unique}")
    return ds, c, L, t2 - t1


def device_ingest(ds, codes, lens, l, k, device, host_s, nthreads, rows=None):
    """the same Dataset built on the device (mg_ingest_codes),
    checked against the host mirror's packed reads (IDs, lengths, frequencies).

    The device ingest ends with the clustered slot layout (apply_layout after the
    dedup write), so its packed reads land in HBM already in slot order: the
    per-dataset device cost after them is ONE step, timed here right after a
    fresh ingest (first_step_ms), with the layout's own
    kernel time inside ingest (layout_ms)."""
    import torch

    e = OverlapEngine(device)
    try:
        e.ingest_codes(codes, lens, l)  # warm-up (hipcub temp sizing, code load)
        e.build_index(l, k)             # (the step's buffers, as a steady caller holds them)
        e.mark_contained(copy=False)
        e.find_overlaps()
        t0 = time.perf_counter()
        nu = e.ingest_codes(codes, lens, l)
        wall = time.perf_counter() - t0
        t = e.timings()
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        e.build_index(l, k)
        e.mark_contained(copy=False)
        n = e.find_overlaps()
        torch.cuda.synchronize(device)
        first = (time.perf_counter() - t1) * 1e3
        ts = e.timings()
        w1, l1 = e.download_packed()
        w0, l0 = ds.packed()
        ok = (nu == ds.num_unique and np.array_equal(l0, l1) and np.array_equal(w0, w1[:, : w0.shape[1]])
              and e.dataset_counts()[0] == ds.num_reads and (rows is None or n == rows))
        return {"device_ms": t["ingest_ms"], "h2d_ms": t["upload_ms"], "layout_ms": t["layout_ms"], "wall_s": wall,
                "host_s": host_s, "host_threads": nthreads, "unique_reads": nu, "match_host": bool(ok),
                "first_step_ms": first, "first_step_rows": n,
                "first_step_device_ms": {kk: round(ts[kk], 3) for kk in ("total_ms", "index_ms", "scan_ms", "probe_ms")}}
    finally:
        e.close()


def cpu_baseline(cfg, sample_reads: int, full_build: bool = True):
    """Reference CPU path on a bounded sample of the same workload shape (same
    read length, l, coverage), rank 0 at N=1 only.

    value = the reference's own `ref_harness disc` (oracle/ref_harness.cpp):
    HashTable::insertDataset + markContainedReads + the insertAllEdgesOfRead loop
    (HashTable.cpp:50-80, OverlapGraph.cpp:225-290,529-565), i.e. the same work
    as the GPU step (index + containment + raw edge multiset).  The shipped
    path's full `new OverlapGraph(ht)` (with the interleaved transitive
    reduction and the contraction loop, main.cpp:45-47) is reported beside it as
    full_build_edges_per_sec.  The reference is single-threaded: cores = 1."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the checker / baseline only

    n, lo, hi, G, l, k, seed, _ = cfg
    cov = n * (lo + hi) / 2 / G
    Gs = int(sample_reads * (lo + hi) / 2 / cov)
    c, L = synth.uniform_read_set(sample_reads, 0, Gs, seed=seed + 1000, lo=lo, hi=hi)
    seqs = synth.codes_to_strings(c, L)
    od = oracle.OracleDataset.from_strings(seqs, l)
    rows, _, th, td = od.overlaps(l)
    edges = rows.shape[0] // 2
    sample = f"{sample_reads} reads x {lo}-{hi} bp, {cov:.0f}x coverage of {Gs} bp, l={l}"
    share = os.environ.get("OMP_NUM_THREADS")
    common = {"unit": "edges/s", "cores": 1, "host_cores_total": os.cpu_count(),
              "host_cores_share": int(share) if share and share.isdigit() else None,
              "edges": edges, "port_discovery_edges_per_sec": edges / (th + td)}
    if os.path.exists(oracle.REF_HARNESS):
        with tempfile.TemporaryDirectory() as td_:
            fa = os.path.join(td_, "s.fa")
            synth.write_fasta(fa, seqs)
            out = os.path.join(td_, "d.json")
            subprocess.run([oracle.REF_HARNESS, "disc", fa, str(l), out], check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            r = json.load(open(out))
            full = None
            if full_build:
                subprocess.run([oracle.REF_HARNESS, "time", fa, str(l), out], check=True,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
                full = json.load(open(out))
        if r["directed_rows"] != rows.shape[0]:
            raise RuntimeError(f"reference rows {r['directed_rows']} != oracle rows {rows.shape[0]}")
        secs = r["hash_s"] + r["discovery_s"]
        res = dict(common, value=edges / secs, kind="reference", seconds=secs,
                   sample=sample + "; reference insertDataset + markContainedReads + insertAllEdgesOfRead loop "
                                   "(oracle/_ref/ref_harness disc: the GPU step's work), 1 thread",
                   reads_per_sec=od.num_unique / secs)
        if full is not None:
            fs = full["hash_s"] + full["graph_s"]
            res["full_build_edges_per_sec"] = edges / fs
            res["full_build_seconds"] = fs
        return res
    secs = th + td
    return dict(common, value=edges / secs, kind="port", seconds=secs,
                sample=sample + "; oracle C restatement index + containment + discovery, 1 thread",
                reads_per_sec=od.num_unique / secs)


def one_shot(e, ds, fused_step, device, rows):
    """Per-dataset time: the reference builds its index and
    graph once per dataset (main.cpp:45-47), so the clustered slot layout, built
    once per upload, belongs to a dataset's cost.  layout_ms = the layout's
    device time (kernels only: its buffers are kept between uploads); one_shot_ms
    = layout_ms + the wall of one step right after it.  Beside it the same with
    the slots in ID order (option layout = 0: no layout pass).  The packed reads'
    H2D copy is outside both, as it is outside ms_per_step."""
    import torch

    def cycle(eng):
        eng.upload(ds)
        lay = eng.timings()["layout_ms"]
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        n = fused_step(eng)
        torch.cuda.synchronize(device)
        return lay, (time.perf_counter() - t0) * 1e3, n

    out = {}
    lay, ms, n = cycle(e)
    assert n == rows, (n, rows)
    t = e.timings()
    out.update(layout_ms=lay, step_ms=ms, one_shot_ms=lay + ms,
               step_device_ms={k: round(t[k], 3) for k in ("total_ms", "index_ms", "scan_ms", "probe_ms")})
    e0 = OverlapEngine(device)
    try:
        e0.set_option("layout", 0)
        e0.set_shard(0, 1)
        cycle(e0)  # allocations
        _, ms0, n0 = cycle(e0)
        assert n0 == rows, (n0, rows)
        out.update(id_order_step_ms=ms0, id_order_one_shot_ms=ms0)
    finally:
        e0.close()
    # which one-shot is faster here, beside the library's default slot order
    # (clustered: every later step over the same upload runs ~25 % faster)
    out["faster_one_shot"] = "layout" if out["one_shot_ms"] <= out["id_order_one_shot_ms"] else "id_order"
    out["default"] = "layout"
    return out


def d2h_rows(e, rows):
    """SURVEY §8(d) "H2D/D2H reported separately": the drop-in's caller reads
    graph[u] on the host (OverlapGraph.cpp:390-419), so the rows leave the device
    through mg_copy_rows (region compaction on the device + one D2H copy).
    Timed into a pinned buffer (the rate a caller that pins its buffer sees)
    and into pageable memory; not part of ms_per_step (inputs and outputs
    resident in HBM), reported beside it."""
    import torch

    out = {"rows": rows, "bytes": rows * 12}
    pinned = torch.empty(max(1, rows * 12), dtype=torch.uint8, pin_memory=True)
    e.copy_rows_to(pinned.data_ptr(), rows)  # first call sizes the compaction buffer
    t0 = time.perf_counter()
    got = e.copy_rows_to(pinned.data_ptr(), rows)
    ms = (time.perf_counter() - t0) * 1e3
    assert got == rows, (got, rows)
    out.update(pinned_ms=ms, pinned_gbs=rows * 12 / ms / 1e6)
    del pinned
    page = np.empty(rows * 12, dtype=np.uint8)
    page[:: 4096] = 0  # fault the pages in before timing
    t0 = time.perf_counter()
    e.copy_rows_to(page.ctypes.data, rows)
    ms = (time.perf_counter() - t0) * 1e3
    out.update(pageable_ms=ms, pageable_gbs=rows * 12 / ms / 1e6)
    return out


def full_size_reference(config):
    """The reference's own time for the bench's exact workload, from the
    committed golden (tests/golden/<config>.json, made by make_scale_golden.py
    with oracle/_ref/ref_harness digest: insertDataset + markContainedReads +
    the insertAllEdgesOfRead loop, 1 thread, in the build container's Xeon)."""
    path = GOLDEN_DIGEST.format(config)
    if not os.path.exists(path):
        return None
    g = json.load(open(path))
    rs = g.get("reference_seconds")
    if not rs:
        return None
    secs = rs["hash_s"] + rs["contain_s"] + rs["discovery_s"]
    return {"edges_per_sec": g["rows"]["n"] / 2 / secs, "seconds": secs, "reads": g["n_reads"],
            "source": os.path.relpath(path, ROOT) + " (reference harness, 1 thread, build container)"}


def combine_digests(ds):
    out = {"n": 0, "sum": 0, "xor": 0, "sum2": 0}
    for d in ds:
        out = {"n": out["n"] + d["n"], "sum": (out["sum"] + d["sum"]) % 2**64, "xor": out["xor"] ^ d["xor"],
               "sum2": (out["sum2"] + d["sum2"]) % 2**64}
    return out


def parity_digest(engines, last, mode, dist, config):
    """Digests (include/mg_overlap.h mg_rows_digest / mg_super_digest) of the
    last step's rows and superReadIDs, computed on the device, combined over
    the ranks, and compared with the reference's own digest of the same
    workload (tests/golden/<config>.json, made by oracle/_ref/ref_harness)."""
    import torch

    if mode.startswith("exchange") and last.rows_in_slots:
        rows = [e.slots_digest(buf.data_ptr(), slot, rounds, cnt.data_ptr())
                for e, (buf, cnt, slot, rounds) in zip(engines, last.rows)]
    else:
        rows = [e.rows_digest() for e in engines]
    sup = engines[0].super_digest() if engines else {"n": 0, "sum": 0, "xor": 0, "sum2": 0}
    rd = combine_digests(rows)
    if dist is not None:  # gather every rank's rows digest (xor does not all-reduce)
        mine = torch.tensor([rd[k] - (2**64 if rd[k] >= 2**63 else 0) for k in ("n", "sum", "xor", "sum2")],
                            dtype=torch.int64)
        dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        allv = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(dist.get_world_size())]
        dist.all_gather(allv, mine.to(dev))
        rd = combine_digests([{k: int(v) % 2**64 for k, v in zip(("n", "sum", "xor", "sum2"), t.cpu().tolist())}
                              for t in allv])
    out = {"rows": rd, "super": sup}
    path = GOLDEN_DIGEST.format(config)
    if os.path.exists(path):
        g = json.load(open(path))
        out["golden"] = os.path.relpath(path, ROOT)
        out["digest_ok"] = bool(g["rows"] == rd and g["super"] == sup)
    else:
        out["golden"] = None
        out["digest_ok"] = None
    return out


# rocprofv3 --pmc summaries (tools/pmc_summary.py) of the default step: profiles/*_pmc_<config>.json


def find_pmc(explicit, config, lib_sha):
    """(traffic bytes, source note) from the newest committed PMC summary of this
    config that was captured on the library this run loaded (or the explicit
    --pmc file); none matching -> (None, why)."""
    import glob

    if explicit:
        return load_pmc(explicit, lib_sha)
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{config}.json")), key=os.path.getmtime,
                   reverse=True)
    first_note = None
    for p in cands:
        t, note = load_pmc(p, lib_sha)
        if t is not None:
            return t, note
        first_note = first_note or note
    return None, first_note or "no PMC summary for this config"


def library_sha16():
    """sha256 (16 hex digits) of the native library this process loaded."""
    import hashlib

    from metagenomics_amd import overlap

    try:
        with open(overlap.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def load_pmc(path, lib_sha=None):
    """HBM traffic of one step from a committed rocprofv3 --pmc summary
    (tools/pmc_summary.py): (2 x FETCH_SIZE + WRITE_SIZE) summed over the step's
    kernels, per launch (MI355X_MICROARCH.md §HBM gfx950 correction).
    Returns (bytes or None, note): a summary captured on another build of the
    library (its recorded sha256 differs from lib_sha), or one without that
    record, gives no traffic -- counters of other kernels are not this run's."""
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception:
        return None, f"unreadable PMC summary {path}"
    prov = (d.get("library") or {}).get("sha256_16")
    if prov is None:
        return None, f"{os.path.basename(path)} records no library build: not quoted"
    if lib_sha is not None and prov != lib_sha:
        return None, f"{os.path.basename(path)} was captured on library {prov}, this run loaded {lib_sha}: not quoted"
    tr = d.get("traffic", {})
    step = ("k_index_build", "k_index_live", "k_scan", "k_probe", "k_prefix_contain", "k_live_runs",
            "k_super_finalize")
    if any("dispatches" in v for v in tr.values()):
        # every dispatch of the step's kernels over the number of step passes
        # (one k_scan each); the default step has no run sort since the
        # clustered slot layout (the rocprim passes in the trace are the
        # upload's layout sort, outside the step)
        passes = sum(v.get("dispatches", 0) for k, v in tr.items() if k.startswith("k_scan")) or 1
        tot = sum(v["traffic_bytes_per_launch"] * v.get("dispatches", 1) for k, v in tr.items()
                  if k.startswith(step)) / passes
    else:
        tot = sum(v["traffic_bytes_per_launch"] for k, v in tr.items() if k.startswith(step))
    return (tot or None), f"{os.path.basename(path)} (library {prov})"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--sim-world", type=int, default=0,
                    help="run all SIM-WORLD ranks of the exchange mode in this process on one GPU")
    ap.add_argument("--exchange", action="store_true",
                    help="use the RCCL exchange mode even with one rank (checks the torch.distributed plumbing)")
    ap.add_argument("--multi", choices=["auto", "replicated", "exchange", "bucket"], default="auto",
                    help="N > 1 (and --sim-world): exchange (north_star, BASELINE configs[3]) = "
                         "bucket-range index shards + RCCL all-to-all of 8-B key and run records; bucket = "
                         "bucket-range index shards, every rank scans every read and keeps its buckets' runs, no "
                         "data-path collective (SURVEY 8(e)(i)); replicated = every rank builds the whole index "
                         "and probes its source-read range (SURVEY 8(e)(ii)); auto (default) = bucket for one read length "
                         "on <= 4 ranks, else exchange.  DESIGN.md 6c")
    ap.add_argument("--route-rows", action="store_true",
                    help="exchange mode: route every row to the owner of its src after discovery (graph[u] by "
                         "source range; one more all-to-all); default: each rank keeps the rows it verified")
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--no-cpu-full", action="store_true", help="skip the reference's full-build timing")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ingest", action="store_true", help="skip the device Dataset ingest measurement")
    ap.add_argument("--replay", action="store_true",
                    help="also time the host replay of the exploration + transitive reduction + contraction on the rows")
    ap.add_argument("--pmc", default=None,
                    help="committed rocprofv3 --pmc summary for roofline.traffic (default: the newest profiles/*_pmc_<config>.json "
                         "captured on this build of the library)")
    ap.add_argument("--nb-log2", type=int, default=0)
    ap.add_argument("--no-d2h", action="store_true", help="skip the rows' D2H timing (mg_copy_rows)")
    ap.add_argument("--no-one-shot", action="store_true",
                    help="skip the per-dataset one-shot timing (layout + one step, and ID order + one step)")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option NAME=VALUE (mg_set_option), repeatable; diagnostics / A-B runs")
    args = ap.parse_args()
    # stdout carries exactly one JSON line: native libraries (RCCL prints its
    # version banner at communicator creation) write to fd 1, so fd 1 goes to
    # stderr for the whole run and the JSON line to a duplicate of the original
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = CONFIGS[args.config]
    n, lo, hi, G, l, k, seed, desc = cfg
    multi_auto = args.multi == "auto"
    if args.multi == "auto":
        # DESIGN.md §6c (simulated per-rank tables + the xGMI model): one read length, up to 4
        # ranks: the bucket mode (no data-path collective; the exchange's run streams cost
        # more link time than the scan they save); more ranks or mixed lengths (containment
        # needs every bucket): the exchange mode
        Pm = world if world > 1 else max(1, args.sim_world)
        args.multi = "bucket" if lo == hi and Pm <= 4 else "exchange"
    nthreads = max(2, 16 // max(1, world))
    ds, codes, lens, host_ingest_s = make_dataset(cfg, nthreads, args.config)
    N = ds.num_unique

    import torch

    dist = None
    xchg = None
    if world > 1 or args.exchange:
        import torch.distributed as dist

        from metagenomics_amd.sharded import TorchExchange

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        backend = os.environ.get("MG_BENCH_PG_BACKEND", "nccl")
        if backend == "gloo":
            # rehearsal with several ranks on fewer GPUs (RCCL refuses two ranks on one
            # device): replicated mode has no data-path collective, so gloo carries the
            # barrier and the clocks; the exchange mode stages its all-to-alls through
            # host copies (TorchExchange.staged), so its timing is not a measurement
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank,
                                    world_size=world)  # RCCL over xGMI
        if args.multi == "exchange" or args.exchange:
            xchg = TorchExchange(torch.device("cuda", local))
            mode = "exchange"
        else:  # the process group only times the step (barrier, MAX of the clocks)
            mode = args.multi
    elif args.sim_world > 1:
        if args.multi == "exchange":
            from metagenomics_amd.sharded import LocalExchange

            xchg = LocalExchange(args.sim_world, torch.device("cuda", local))
            mode = "exchange-sim"
        else:
            mode = args.multi + "-sim"
    else:
        mode = "fused"
    P = world if mode in ("exchange", "replicated", "bucket") else max(1, args.sim_world)

    from metagenomics_amd.sharded import sharded_step, source_range

    engines = []
    layout_ms = 0.0
    t0 = time.time()
    for r in ([rank] if mode in ("exchange", "replicated", "bucket") else range(P)):
        e = OverlapEngine(local)
        e.set_option("nb_log2", args.nb_log2)
        for kv in args.opt:
            name, val = kv.split("=", 1)
            e.set_option(name, int(val))
        if mode.startswith("replicated"):
            # the whole index on every rank, this rank's source reads only: the
            # index build (k_index_build) then a scan + probe of [lo, hi)
            s_lo, s_hi = source_range(N, r, P)
            if s_hi == s_lo:  # more ranks than reads (read_hi = 0 would mean "all")
                e.close()
                continue
            e.set_shard(0, 1, s_lo, s_hi)
        else:
            e.set_shard(r, P, 0, 0)
        e.upload(ds)
        layout_ms = max(layout_ms, e.timings()["layout_ms"])
        engines.append(e)
    log(f"[bench] rank {rank}: upload {time.time() - t0:.2f}s ({mode}, P={P})")

    rank_ms = [0.0] * len(engines)  # replicated-sim / bucket-sim: per simulated rank, summed over the timed steps

    def step():
        """one pass of the hot path; returns directed rows held by this process"""
        if mode in ("fused", "replicated", "bucket"):
            return fused_step(engines[0]) if engines else 0
        if mode in ("replicated-sim", "bucket-sim"):
            tot = 0
            for i, e in enumerate(engines):  # the ranks one after the other, each timed alone
                torch.cuda.synchronize(local)
                ta = time.perf_counter()
                e.build_index(l, k)
                e.mark_contained(copy=False)
                tot += e.find_overlaps()
                torch.cuda.synchronize(local)
                rank_ms[i] += (time.perf_counter() - ta) * 1e3
            return tot
        res = sharded_step(engines, xchg, l, k, plan=plan[0], route_rows=args.route_rows)
        plan[0] = plan[0] or res.plan
        last_res[0] = res
        for kk, v in res.ms.items():
            phase_ms[kk] = phase_ms.get(kk, 0.0) + v
        reruns[0] += res.reruns
        return sum(res.n_rows)

    phase_ms = {}
    last_res = [None]
    plan = [None]    # exchange stream capacities, kept from step to step
    reruns = [0]     # exchange steps rerun after a capacity overflow (timed steps only)

    def fused_step(e):
        e.build_index(l, k)
        e.mark_contained(copy=False)
        return e.find_overlaps()

    def sync_barrier():
        torch.cuda.synchronize(local)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(local)

    # one counting pass (untimed) for the roofline's algorithmic bytes
    for e in engines:
        e.set_option("stats", 1)
    rows = step()
    cnt = {}
    for e in engines:
        for kk, v in e.counters().items():
            cnt[kk] = cnt.get(kk, 0) + v
        e.set_option("stats", 0)
    cnt["sources"] = N if mode != "exchange" else cnt.get("sources", 0)
    for _ in range(args.warmup):
        step()

    dev_ms = {"index_ms": 0.0, "contained_ms": 0.0, "overlap_ms": 0.0, "scan_ms": 0.0, "sort_ms": 0.0,
              "probe_ms": 0.0, "verify_ms": 0.0, "total_ms": 0.0}
    phase_ms.clear()
    reruns[0] = 0
    rank_ms[:] = [0.0] * len(engines)
    sync_barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rows = step()
        for e in engines:
            t = e.timings()
            for kk in dev_ms:
                dev_ms[kk] += t[kk]
    torch.cuda.synchronize(local)
    t1 = time.perf_counter()
    sync_barrier()
    ms_step = (t1 - t0) * 1000.0 / args.steps
    dev_ms = {kk: v / args.steps for kk, v in dev_ms.items()}
    sim_rank_ms = None
    if mode in ("replicated-sim", "bucket-sim"):
        # P ranks with no data-path collective: the job's step is its slowest rank
        sim_rank_ms = [v / args.steps for v in rank_ms]
        ms_step = max(sim_rank_ms)
        dev_ms = {kk: v / P for kk, v in dev_ms.items()}
    if dist is not None:
        red_dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        tt = torch.tensor([ms_step], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ms_step = float(tt.item())
        ee = torch.tensor([rows], dtype=torch.int64, device=red_dev)
        dist.all_reduce(ee, op=dist.ReduceOp.SUM)
        rows = int(ee.item())
    edges = rows // 2
    # parity at the bench's own size: device digests of the last step vs the
    # reference's digests of the same workload (outside the timed region)
    parity = parity_digest(engines, last_res[0], mode, dist, args.config)
    if rank != 0:
        dist.barrier()
        dist.destroy_process_group()
        return

    # Roofline: SURVEY §8(d) algorithmic bytes per read,
    #   B = ceil(n/4) + 4*16 + W*16 + D*(ceil(n/4) + 16),  D = directed rows per read,
    # times the reads one step processes, over the step's summed kernel durations
    # (HIP events on the context's stream: index build incl. cell memset, scan, probe).
    nbar = (lo + hi) / 2.0
    W = max(0.0, nbar - (l - 1) - 1)
    D = rows / max(1, N)
    per_read = -(-nbar // 4) + 64 + W * 16 + D * (-(-nbar // 4) + 16)
    alg = N * per_read
    # device wall of the step (the scan overlaps the index build on a second stream)
    kern_ms = dev_ms["total_ms"] if dev_ms.get("total_ms") else (
        dev_ms["index_ms"] + dev_ms["contained_ms"] + dev_ms["overlap_ms"])
    roof = None
    lib_sha = library_sha16()
    if mode == "fused":
        achieved = alg / (kern_ms / 1000.0) / 1e9 if kern_ms > 0 else 0.0
        traffic, traffic_src = find_pmc(args.pmc, args.config, lib_sha)
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "kernel": ("step = k_scan<INDEX> (window scan + fused index build), "
                           + ("bucket sort of the runs (rocprim onesweep), " if dev_ms.get("sort_ms") else
                              "runs in read order on the clustered slot layout, ")
                           + "then k_probe (containment, then discovery); device wall, HIP events"),
                "alg_bytes_per_step": alg, "alg_bytes_per_read": per_read, "kernel_ms_per_step": kern_ms,
                "probe_ms": dev_ms["probe_ms"], "verify_ms": dev_ms["verify_ms"], "scan_ms": dev_ms["scan_ms"]}
    else:
        # per-rank work is 1/P of the reads: roofline of rank 0's kernels on its share
        achieved = alg / P / (kern_ms / 1000.0) / 1e9 if kern_ms > 0 else 0.0
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "kernel": ("rank 0 step kernels (whole index build, scan + probe of its source range)"
                           if mode.startswith("replicated") else
                           "rank 0 step kernels (scan of every read filing and keeping its buckets' keys and runs, "
                           "probe of those runs)" if mode.startswith("bucket") else
                           "rank 0 step device wall (scan + run sort + key exchange + insert, "
                           "containment + discovery probes; ev0 -> discovery end on the engine's stream)"),
                "alg_bytes_per_step": alg / P, "kernel_ms_per_step": kern_ms}
    par = {"fused": "1 GPU, fused path",
           "replicated": f"{P} ranks: whole index on every rank, source-read range shards, no data-path collective",
           "replicated-sim": f"{P} simulated ranks on 1 GPU (whole index each, source-read shards; step = slowest rank)",
           "exchange": f"{P} ranks: bucket-range index + source-range shards, RCCL all-to-all of 8-B key and "
                       f"run records" + (" and of the rows" if args.route_rows else ""),
           "exchange-sim": f"{P} simulated ranks on 1 GPU (device-local exchange)",
           "bucket": f"{P} ranks: bucket-range index shards, every rank scans every read and keeps its buckets' "
                     "runs, no data-path collective",
           "bucket-sim": f"{P} simulated ranks on 1 GPU (bucket-range shards, every read scanned by each; "
                         "step = slowest rank)"}[mode]
    res = {
        "metric": "overlap edges/sec",
        "value": edges / (ms_step / 1000.0),
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": desc, "reads": n, "unique_reads": N, "read_len": [lo, hi], "genome_len": G,
                   "min_overlap": l, "seed_k": k, "seed": seed, "parallelism": par},
        "reads_per_sec": N / (ms_step / 1000.0),
        "undirected_edges": edges,
        "device_ms": dev_ms,
        # the device Dataset's slot layout (reads clustered by canonical global
        # minimizer), built once per upload like the packing: not in
        # ms_per_step.  layout_ms = its kernels on a context that already holds the
        # layout's buffers (one_shot re-upload, below, when it runs); the first
        # upload also allocates them (layout_first_upload_ms)
        "layout_ms": layout_ms,
        "layout_first_upload_ms": layout_ms,
        "phase_wall_ms": {kk: v / args.steps for kk, v in phase_ms.items()} or None,
        # which multi-GPU mode ran and why (N > 1 / --sim-world): --multi auto's choice rests on
        # simulated per-rank tables and the xGMI model, not on an 8-GPU run
        "multi_mode": None if mode == "fused" else {
            "mode": mode, "requested": "--exchange" if args.exchange else ("auto" if multi_auto else args.multi),
            "process_group": dist.get_backend() if dist is not None else None,
            "rule": ("auto: bucket for one read length on <= 4 ranks, else exchange; chosen from simulated "
                     "per-rank kernel tables + the xGMI link model (DESIGN.md §6c, profiles/r06_xchg_model_c3.md), "
                     "not yet confirmed on a multi-GPU node") if multi_auto and not args.exchange else "explicit"},
        "exchange_reruns": reruns[0] if mode.startswith("exchange") else None,
        "exchange_rows": (("routed to their src owners" if args.route_rows and P > 1 else
                           "held by the rank that verified them (union = the multiset)")
                          if mode.startswith("exchange") else None),
        # slot-layout padding: records moved between ranks vs records sent (rank 0's, or all
        # simulated ranks'), from the last step's counts
        "exchange_padding": (last_res[0].padding(P, [rank] if mode == "exchange" else list(range(P)))
                             if mode.startswith("exchange") and last_res[0] is not None and P > 1 else None),
        "counters": cnt,
        "library_sha16": lib_sha,
        "roofline": roof,
        "parity": parity,
    }
    if sim_rank_ms is not None:
        res["sim_rank_ms"] = sim_rank_ms
    if world == 1 and mode == "fused" and not args.no_d2h:
        try:
            d2h = d2h_rows(engines[0], rows)
            res["d2h_rows"] = d2h
            res["d2h_rows_ms"] = d2h["pinned_ms"]
            # PCIe-inclusive rate (never `value`): the step plus the rows' copy to pinned host memory
            res["edges_per_sec_with_d2h"] = edges / ((ms_step + d2h["pinned_ms"]) / 1000.0)
        except Exception as e:  # report, never fake
            res["d2h_rows"] = {"error": str(e)}
    if world == 1 and mode == "fused" and not args.no_one_shot:
        try:
            res["one_shot"] = one_shot(engines[0], ds, fused_step, local, rows)
            res["layout_ms"] = res["one_shot"]["layout_ms"]
            res["one_shot_ms"] = res["one_shot"]["one_shot_ms"]
            res["one_shot_edges_per_sec"] = edges / (res["one_shot"]["one_shot_ms"] / 1000.0)
        except Exception as e:  # report, never fake
            res["one_shot"] = {"error": str(e)}
    if world == 1 and mode == "fused" and args.replay:
        from metagenomics_amd.overlap import UnitigGraph

        t0 = time.perf_counter()
        allrows = engines[0].rows(rows)
        t1 = time.perf_counter()
        ug = UnitigGraph(allrows, ds.packed()[1], l)
        res["graph_replay"] = {"copy_rows_s": t1 - t0, "replay_s": ug.replay_s, "nodes": ug.replay_nodes,
                               "edges_after_reduction": ug.replay_edges, "contract_s": ug.contract_s,
                               "unitig_nodes": ug.nodes, "unitig_edges": ug.edges,
                               "contract_iterations": ug.iterations, "threads": 1}
        ug.close()
        del allrows
    if world == 1 and mode == "fused" and not args.no_ingest:
        try:
            res["dataset_ingest"] = device_ingest(ds, codes, lens, l, k, local, host_ingest_s, nthreads, rows)
            di = res["dataset_ingest"]
            # per dataset once the packed reads are in HBM: the device ingest leaves
            # them in slot order (its layout inside), so one step remains
            res["one_shot_after_device_ingest_ms"] = di["first_step_ms"]
            res["one_shot_after_device_ingest_edges_per_sec"] = edges / (di["first_step_ms"] / 1000.0)
        except Exception as e:  # report, never fake
            res["dataset_ingest"] = {"error": str(e)}
    if world == 1 and mode == "fused" and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample, not args.no_cpu_full)
        except Exception as e:  # report, never fake
            res["cpu_baseline"] = {"value": None, "error": str(e)}
        fsr = full_size_reference(args.config)
        if fsr is not None:
            res["cpu_baseline"]["full_size_reference"] = fsr
    print(json.dumps(res), file=json_out, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
