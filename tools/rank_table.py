"""Per-rank kernel table of a simulated-world run (bench.py --sim-world P):
the P simulated ranks' kernels all land in one rocprofv3 kernel_stats.csv, and
every rank runs the same kernels on its own share, so a kernel's per-rank cost
is its total duration / P, and per step / (P * S) for S step executions in the
run (bench: 1 counting pass + warmup + steps).  Upload-time kernels (packing,
layout) run once per rank and are divided by S all the same: read them as such.
usage: rank_table.py kernel_stats.csv P S [title]"""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", name)
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)", name)
    s = m.group(1) if m else name
    return s[:90]


# kernels that run once per upload or only for the parity check, not in the step
OUTSIDE = ("k_layout_", "k_rows_digest", "k_super_digest", "k_ingest", "k_pack_ascii")
# the layout's radix sort (64-bit keys, 32-bit slot values; the step's own sorts
# have 32-bit keys), told apart by its full template name
LAYOUT_SORT = re.compile(r"radix_sort_onesweep_config<rocprim::\w+::default_config, unsigned long, unsigned int>")


def main():
    path, P, S = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    title = sys.argv[4] if len(sys.argv) > 4 else path
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"### {title}: kernel time per rank per step at P={P} (total / (P x {S}))\n")
    print("| kernel | calls/rank/step | ms/rank/step | share |")
    print("|---|---:|---:|---:|")
    step = copies = 0.0
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        name = short(r["Name"])
        out = name.startswith(OUTSIDE) or bool(LAYOUT_SORT.search(r["Name"]))
        if LAYOUT_SORT.search(r["Name"]):
            name += " (layout sort)"
        if not out:
            step += t
            if name.startswith("__amd_rocclr_copyBuffer"):
                copies += t
        print(f"| `{name}`{' (not in the step)' if out else ''} | {int(r['Calls']) / P / S:.2f} | "
              f"{t / P / S / 1e6:.3f} | {100 * t / tot:.1f}% |")
    print(f"| **all kernels** | | **{tot / P / S / 1e6:.3f}** | |")
    print(f"| **step kernels** (upload / layout / parity kernels excluded) | | "
          f"**{step / P / S / 1e6:.3f}** | |")
    # the simulated exchange moves the slot buffers with device copies; on N GPUs
    # RCCL's transfers over xGMI take their place
    print(f"| **step compute kernels** (the step kernels without the simulated exchange's device copies, "
          f"`__amd_rocclr_copyBuffer`) | | **{(step - copies) / P / S / 1e6:.3f}** | |")


if __name__ == "__main__":
    main()
