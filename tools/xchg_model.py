"""Per-phase model of the multi-GPU step wall at P = 2 / 4 / 8, from
measurements on ONE MI355X:

* compute per rank: the simulated ranks' kernel tables (tools/rank_table.py output of
  `tools/gpu_run.sh profsimP`: every simulated rank's kernels timed alone,
  MG_SIM_SERIAL=1), "step compute kernels" = the step's kernels without the simulated
  exchange's device copies;
* bytes per rank: the exchange's own slot-layout counts (bench.py `exchange_padding`:
  records moved between ranks, summed over the ranks, and the bytes per record on the
  wire -- round 6: keys and runs 8 B, rows 12 B and only when routed), plus the MAX
  all-reduce of the n x 8 B containment keys when lengths differ;
* replicated mode and bucket mode (every rank scans every read, keeps its
  buckets' keys and runs): the slowest simulated rank of `bench.py --multi replicated|bucket
  --sim-world P` (no data-path collective).

xGMI (MI355X, one node): every GPU has 7 point-to-point links to its 7 peers.  An
all-to-all moves each peer's share over that peer's own link, all links at once, so its
time is the per-peer share / the per-direction link rate; a ring all-reduce of S bytes
moves 2 (P-1)/P S per rank, spread over the P - 1 links.  Link rates modelled: 64 GB/s
(MI300X-class, conservative), 76.5 GB/s (153 GB/s per link counted in both directions),
153 GB/s per direction (optimistic).  Each collective round adds a fixed latency alpha
(30 us).

Two bounds: "serial" = compute + every transfer after it; "overlap" = what the hosts
(sharded.py, csrc/host/mg_xchg.cpp) schedule: the run streams travel on a second stream
while the received keys are sorted and filed, and -- equal lengths, no containment pass --
while each rank probes its own run stream (mg_xchg_probe_own, ~1/P of the probe); with
containment the runs must all be in before the containment probe, so only the key build
hides them.  Keys first (the default since round 6: keys inserted inside the receiver's
scan) leaves no key build to hide the runs behind, so only the own-stream probe does,
and only up to P = 4 (xchg_split_max).  "+rows" lines add the rows' all-to-all (12-B mg_edge records to their src
owners, bench.py --route-rows), estimated from the measured row count, after the probe.

usage: xchg_model.py OUT.md FUSED_BENCH.json CONFIG DIR
  DIR holds profsim{P}_{CONFIG}_ranks.md, profsim{P}_{CONFIG}_bench.json and
  bench_simrep{P}_{CONFIG}.json / bench_simbkt{P}_{CONFIG}.json (replicated / bucket; without
  the _{CONFIG} suffix for c3) for P in 2 4 8."""
import json
import os
import re
import sys

LINKS = (64.0, 76.5, 153.0)    # GB/s per direction per link
ALPHA_MS = 0.030               # per collective round
OLD_REC_BYTES = {"keys": 16, "runs": 16, "rows": 12}  # (bench lines before round 6 carry no record_bytes)
SPLIT_MAX = 4                  # mg_ctx xchg_split_max: the discovery probe is split up to P = 4
KEY_BUILD = ("k_xkeys_dense", "k_key_class", "k_cells_", "k_over_heads",
             "rocprim::trampoline_kernel<rocprim::wrapped_radix_sort", "rocprim::trampoline_kernel<rocprim::wrapped_scan")


def step_compute_ms(md_path):
    txt = open(md_path).read()
    m = re.search(r"\*\*step compute kernels\*\*.*?\*\*([0-9.]+)\*\*", txt)
    return float(m.group(1))


def kernel_ms(md_path, prefix):
    tot = 0.0
    for line in open(md_path):
        m = re.match(r"\| `([^`]+)`[^|]*\| [0-9.]+ \| ([0-9.]+) \|", line)
        if m and m.group(1).startswith(prefix) and "(not in the step)" not in line:
            tot += float(m.group(2))
    return tot


def main():
    out, fused_path, cfg, d = sys.argv[1:5]
    fused = json.load(open(fused_path))
    t1 = fused["ms_per_step"]
    edges = fused["undirected_edges"]
    n_reads = fused["config"]["unique_reads"]
    mixed = fused["config"]["read_len"][0] != fused["config"]["read_len"][1]
    lines = [f"### {cfg}: modelled multi-GPU step wall (tools/xchg_model.py)\n",
             f"1 GPU (fused path): {t1:.3f} ms/step, {edges / t1 * 1e3:.3e} edges/s.\n",
             "| mode | P | compute / rank (ms) | xGMI MB / rank (keys + runs [+ rows]) | link GB/s | transfer (ms) | "
             "wall serial (ms) | wall overlap (ms) | speedup vs 1 GPU (serial / overlap) |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---|"]
    res = {"config": cfg, "fused_ms": t1, "rows": []}
    for P in (2, 4, 8):
        md = os.path.join(d, f"profsim{P}_{cfg}_ranks.md")
        bj = os.path.join(d, f"profsim{P}_{cfg}_bench.json")
        if os.path.exists(md) and os.path.exists(bj):
            comp = step_compute_ms(md)
            # the sorted key build (k_xkeys_dense + sort + cell fill) runs while the runs travel;
            # keys first (round 6 default) inserts the keys inside the scan, before the runs exist
            keybuild = sum(kernel_ms(md, k) for k in KEY_BUILD) if kernel_ms(md, "k_xkeys_dense") else 0.0
            probe = kernel_ms(md, "k_probe")
            # mg_xchg_probe_own: the rank's own stream, ~1/P of the probe (equal lengths, P <= 4)
            own_probe = 0.0 if mixed or P > SPLIT_MAX else probe / P
            pad = json.load(open(bj))["exchange_padding"]
            per_kind = {k: v["moved_records"] * (v.get("record_bytes") or OLD_REC_BYTES[k]) / P
                        for k, v in pad.items()}  # bytes per rank
            # rows to their src owners (--route-rows): each rank's rows/P, (P-1)/P of them leave
            rows_routed = 2 * edges / P * (P - 1) / P * 12
            ar = (2.0 * (P - 1) / P * n_reads * 8) if mixed else 0.0  # containment keys, ring all-reduce
            for variant in ("exchange", "exchange +rows"):
                kinds = dict(per_kind)
                if variant.endswith("rows") and "rows" not in kinds:
                    kinds["rows"] = rows_routed
                tot_b = sum(kinds.values()) + ar
                for B in LINKS:
                    bw = B * 1e9
                    a2a = {k: v / (P - 1) / bw * 1e3 for k, v in kinds.items()}
                    ar_ms = ar / (P - 1) / bw * 1e3
                    rounds = len(kinds) + (2 if mixed else 0)
                    xfer = sum(a2a.values()) + ar_ms + ALPHA_MS * rounds
                    serial = comp + xfer
                    overlap = serial - min(a2a.get("runs", 0.0), keybuild + own_probe)
                    mb = " + ".join(f"{kinds[k] / 1e6:.0f}" for k in ("keys", "runs", "rows") if k in kinds)
                    lines.append(f"| {variant} | {P} | {comp:.3f} | {tot_b / 1e6:.0f} ({mb}) | {B:.1f} | {xfer:.3f} | "
                                 f"{serial:.3f} | {overlap:.3f} | {t1 / serial:.2f}x / {t1 / overlap:.2f}x |")
                    res["rows"].append({"mode": variant, "P": P, "compute_ms": comp, "bytes_per_rank": tot_b,
                                        "bytes_by_kind": kinds, "allreduce_bytes": ar, "link_gbs": B,
                                        "transfer_ms": xfer, "wall_serial_ms": serial, "wall_overlap_ms": overlap,
                                        "key_build_ms": keybuild, "own_probe_ms": own_probe,
                                        "speedup_overlap": t1 / overlap})
        for mode, stem in (("replicated", "simrep"), ("bucket", "simbkt")):
            rj = os.path.join(d, f"bench_{stem}{P}_{cfg}.json")
            if not os.path.exists(rj) and cfg == "c3":
                rj = os.path.join(d, f"bench_{stem}{P}.json")
            if os.path.exists(rj):
                r = json.load(open(rj))
                w = max(r["sim_rank_ms"])
                lines.append(f"| {mode} | {P} | {w:.3f} | 0 | — | 0 | {w:.3f} | {w:.3f} | "
                             f"{t1 / w:.2f}x / {t1 / w:.2f}x |")
                res["rows"].append({"mode": mode, "P": P, "compute_ms": w, "bytes_per_rank": 0,
                                    "wall_serial_ms": w, "wall_overlap_ms": w, "speedup_overlap": t1 / w,
                                    "digest_ok": r["parity"].get("digest_ok")})
    lines.append("")
    lines.append(f"Link model: all-to-all = per-peer share / link rate (P - 1 links at once); ring all-reduce "
                 f"of the containment keys over P - 1 links; {ALPHA_MS * 1e3:.0f} us per collective round.  Compute = "
                 "simulated ranks' kernels, each rank timed alone on one MI355X; on N GPUs each rank has a whole "
                 "GPU, so per-rank compute is what it is here.  '+rows' adds the rows' transfer only (its routing "
                 "kernel is not in the compute column).")
    open(out, "w").write("\n".join(lines) + "\n")
    json.dump(res, open(os.path.splitext(out)[0] + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
