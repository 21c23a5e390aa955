"""SURVEY §8(f) row 4 measurement: FASTA/FASTQ -> Dataset throughput.

Writes a C3-shaped read set (BASELINE configs[1]: 10M x 150 bp, genome
n*150/20, seed 31) as FASTQ and as 2-line-wrapped FASTA under $TMPDIR, then
times, min over repeats:
  * the record splitter alone (mgh_parse_file) at several thread counts;
  * Dataset.from_files (splitter + host canonicalise/sort/dedup, all threads);
  * OverlapEngine.ingest_files (splitter -> device ingest), when a GPU is there;
  * the reference's own Dataset constructor (oracle/_ref/ref_harness time,
    single thread: getline + sort + dedup) on a bounded sample of the file.
One JSON line on stdout.  usage: parse_bench.py [n_reads] [--no-ref]"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from metagenomics_amd import synth  # noqa: E402
from metagenomics_amd.overlap import Dataset, parse_file  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 10_000_000
    d = tempfile.mkdtemp(prefix="mgparse_", dir=os.environ.get("TMPDIR", "/tmp"))
    c, L = synth.uniform_read_set(n, 150, n * 150 // 20, seed=31)
    seqs = synth.codes_to_strings(c, L)
    del c
    fq, fa = os.path.join(d, "c3.fq"), os.path.join(d, "c3.fa")
    t0 = time.perf_counter()
    synth.write_fastq(fq, seqs)
    with open(fa, "w") as f:
        for i in range(0, len(seqs), 1 << 20):
            f.write("".join(">r%d\n%s\n%s\n" % (i + k, s[:75], s[75:]) for k, s in enumerate(seqs[i:i + (1 << 20)])))
    print("wrote files in %.1f s" % (time.perf_counter() - t0), file=sys.stderr, flush=True)
    res = {"n_reads": n, "files": {}}
    cpus = os.cpu_count() or 1
    threads = [t for t in (1, 4, 8, 16) if t <= max(16, cpus)]
    for name, path in (("fastq", fq), ("fasta", fa)):
        size = os.path.getsize(path)
        r = {"bytes": size, "split_s": {}}
        for t in threads:
            best = min(parse_file(path, t)[2] for _ in range(3))
            r["split_s"][str(t)] = round(best, 4)
            print(f"{name} split {t} threads: {best:.3f} s ({size / best / 1e9:.2f} GB/s)", file=sys.stderr, flush=True)
        best_t = min(r["split_s"].values())
        r["split_GBps"] = round(size / best_t / 1e9, 3)
        t0 = time.perf_counter()
        ds = Dataset.from_files([path], 50)
        r["host_dataset_s"] = round(time.perf_counter() - t0, 3)
        r["n_unique"] = ds.num_unique
        del ds
        try:
            import torch

            if torch.cuda.is_available():
                from metagenomics_amd.overlap import OverlapEngine

                e = OverlapEngine(0)
                e.set_shard(0, 1)
                t0 = time.perf_counter()
                info = e.ingest_files([path], 50, 16)
                r["device_dataset_s"] = round(time.perf_counter() - t0, 3)
                r["device_ingest"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in info.items()}
                assert info["n_unique"] == r["n_unique"], (info, r["n_unique"])
                e.close()
        except ImportError:
            pass
        res["files"][name] = r
    if "--no-ref" not in sys.argv:
        harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
        if os.path.exists(harness):
            # bounded sample: the first 1M records (about 10 s of the reference's CPU time)
            m = min(n, 1_000_000)
            sample = os.path.join(d, "sample.fq")
            with open(fq) as f, open(sample, "w") as g:
                for _ in range(4 * m):
                    g.write(f.readline())
            out = os.path.join(d, "ref.txt")
            subprocess.run([harness, "dstime", sample, "50", out], check=True, timeout=600,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            with open(out) as f:
                ref_s = float(f.read().split()[1])
            res["reference_dataset"] = {"sample_records": m, "seconds": round(ref_s, 3),
                                        "records_per_s": round(m / ref_s), "threads": 1,
                                        "note": "Dataset(pe, se, l) constructor of the reference (ref_harness dstime)"}
    for f in (fq, fa):
        os.unlink(f)
    for f in os.listdir(d):
        os.unlink(os.path.join(d, f))
    os.rmdir(d)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
