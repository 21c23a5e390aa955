"""Per-phase model of the multi-GPU step wall at P = 2 / 4 / 8 (VERDICT r4 item 2,
DESIGN.md §6c), from measurements on ONE MI355X:

* compute per rank: the simulated ranks' kernel tables (tools/rank_table.py
  output of `tools/gpu_run.sh profsimP`: every simulated rank's kernels timed
  alone, MG_SIM_SERIAL=1), "step compute kernels" = the step's kernels without
  the simulated exchange's device copies;
* bytes per rank: the exchange's own slot-layout counts (bench.py
  `exchange_padding`: records moved between ranks, summed over the ranks), plus
  the MAX all-reduce of the n x 8 B containment keys when lengths differ;
* replicated mode: the slowest simulated rank of
  `bench.py --multi replicated --sim-world P` (no data-path collective).

xGMI (MI355X, one node): every GPU has 7 point-to-point links to its 7 peers.
An all-to-all moves each peer's share over that peer's own link, all links at
once, so its time is the largest per-peer share / the per-direction link rate;
a ring all-reduce of S bytes moves 2 (P-1)/P S per rank, spread here over the
P - 1 links (the ideal; RCCL's channels approach it).  Link rates modelled:
64 GB/s (MI300X-class, conservative), 76.5 GB/s (153 GB/s per link counted in
both directions), 153 GB/s per direction (optimistic).  Each collective round
adds a fixed latency alpha (30 us).  Two bounds: "serial" = compute + every
transfer after it; "overlap" = the run exchange hidden behind the key build and
the rows' behind nothing (what the C++ host's side stream can reach).

usage: xchg_model.py OUT.md FUSED_BENCH.json CONFIG DIR
  DIR holds profsim{P}_{CONFIG}_ranks.md, profsim{P}_{CONFIG}_bench.json and
  bench_simrep{P}_{CONFIG}.json (replicated; bench_simrep{P}.json for c3) for P in 2 4 8."""
import json
import os
import re
import sys

LINKS = (64.0, 76.5, 153.0)    # GB/s per direction per link
ALPHA_MS = 0.030               # per collective round
REC_BYTES = {"keys": 16, "runs": 16, "rows": 12}


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
             "| mode | P | compute / rank (ms) | xGMI bytes / rank (MB) | link GB/s | transfer (ms) | "
             "wall serial (ms) | wall overlap (ms) | speedup vs 1 GPU (serial / overlap) |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---|"]
    res = {"config": cfg, "fused_ms": t1, "rows": []}
    for P in (2, 4, 8):
        md = os.path.join(d, f"profsim{P}_{cfg}_ranks.md")
        bj = os.path.join(d, f"profsim{P}_{cfg}_bench.json")
        if os.path.exists(md) and os.path.exists(bj):
            comp = step_compute_ms(md)
            keybuild = sum(kernel_ms(md, k) for k in ("k_xkeys_dense", "k_key_class", "k_cells_", "k_over_heads",
                                                     "rocprim::trampoline_kernel<rocprim::wrapped_radix_sort"))
            pad = json.load(open(bj))["exchange_padding"]
            per_kind = {k: pad[k]["moved_records"] * REC_BYTES[k] / P for k in REC_BYTES}  # bytes per rank
            ar = (2.0 * (P - 1) / P * n_reads * 8) if mixed else 0.0  # containment keys, ring all-reduce
            tot_b = sum(per_kind.values()) + ar
            for B in LINKS:
                bw = B * 1e9
                a2a = {k: v / (P - 1) / bw * 1e3 for k, v in per_kind.items()}
                ar_ms = ar / (P - 1) / bw * 1e3
                xfer = sum(a2a.values()) + ar_ms + ALPHA_MS * (3 + (2 if mixed else 0))
                serial = comp + xfer
                overlap = comp + xfer - min(a2a["runs"], keybuild)
                lines.append(f"| exchange | {P} | {comp:.3f} | {tot_b / 1e6:.0f} | {B:.1f} | {xfer:.3f} | "
                             f"{serial:.3f} | {overlap:.3f} | {t1 / serial:.2f}x / {t1 / overlap:.2f}x |")
                res["rows"].append({"mode": "exchange", "P": P, "compute_ms": comp, "bytes_per_rank": tot_b,
                                    "bytes_by_kind": per_kind, "allreduce_bytes": ar, "link_gbs": B,
                                    "transfer_ms": xfer, "wall_serial_ms": serial, "wall_overlap_ms": overlap,
                                    "key_build_ms": keybuild})
        rj = os.path.join(d, f"bench_simrep{P}_{cfg}.json")
        if not os.path.exists(rj) and cfg == "c3":
            rj = os.path.join(d, f"bench_simrep{P}.json")
        if os.path.exists(rj):
            r = json.load(open(rj))
            w = max(r["sim_rank_ms"])
            lines.append(f"| replicated | {P} | {w:.3f} | 0 | — | 0 | {w:.3f} | {w:.3f} | "
                         f"{t1 / w:.2f}x / {t1 / w:.2f}x |")
            res["rows"].append({"mode": "replicated", "P": P, "compute_ms": w, "bytes_per_rank": 0,
                                "wall_serial_ms": w, "wall_overlap_ms": w, "digest_ok": r["parity"].get("digest_ok")})
    lines.append("")
    lines.append(f"Link model: all-to-all = largest per-peer share / link rate (P - 1 links at once); ring all-reduce "
                 f"of the containment keys over P - 1 links; {ALPHA_MS * 1e3:.0f} us per collective round.  Compute = "
                 "simulated ranks' kernels, each rank timed alone on one MI355X; on N GPUs each rank has a whole "
                 "GPU, so per-rank compute is what it is here.")
    open(out, "w").write("\n".join(lines) + "\n")
    json.dump(res, open(os.path.splitext(out)[0] + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
