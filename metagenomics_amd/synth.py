"""Deterministic synthetic read sets (SURVEY §8(d) "Synthetic inputs").

Reads are sampled uniformly from a uniform random genome, 50 % of them
reverse-complemented, as the survey's generator does; this generator uses
numpy's PCG64 instead of Python's ``random`` so that 10M-read sets are made in
seconds.  Exact edge counts therefore differ from the survey's numbers and are
regenerated through the oracle (tests/golden/make_golden.py).

Bases are 2-bit codes A0 C1 G2 T3 (lexicographic order).
"""
from __future__ import annotations

import numpy as np

ALPHABET = np.frombuffer(b"ACGT", dtype=np.uint8)


def random_genome(length: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.integers(0, 4, size=length, dtype=np.uint8)


def revcomp_codes(codes: np.ndarray, lengths: np.ndarray) -> np.ndarray:
    """Reverse complement each row of a padded [n, maxlen] code matrix."""
    n, maxlen = codes.shape
    k = np.arange(maxlen, dtype=np.int64)[None, :]
    src = lengths.astype(np.int64)[:, None] - 1 - k
    valid = src >= 0
    src = np.where(valid, src, 0)
    out = 3 - np.take_along_axis(codes, src, axis=1)
    out[~valid] = 0
    return out.astype(np.uint8)


def sample_reads(genome: np.ndarray, n_reads: int, lo: int, hi: int, seed: int,
                 rc_fraction: float = 0.5, chunk: int = 1 << 20):
    """Return (codes[n, hi] uint8, lengths[n] uint16).

    Each read: length ~ U[lo, hi], start ~ U[0, G-len], reverse-complemented
    with probability ``rc_fraction``.  Built in chunks of ``chunk`` reads so
    10M-read sets stay within a few GB of host memory."""
    rng = np.random.default_rng(seed)
    G = genome.shape[0]
    lengths = rng.integers(lo, hi + 1, size=n_reads).astype(np.int64)
    starts = rng.integers(0, G - lengths + 1)
    rc = rng.random(n_reads) < rc_fraction
    codes = np.zeros((n_reads, hi), dtype=np.uint8)
    if lo == hi and G >= hi:
        # fixed length: rows of a sliding-window view, reversed + complemented in
        # place for the rc reads (same values as the general path below)
        win = np.lib.stride_tricks.sliding_window_view(genome, hi)
        for a in range(0, n_reads, chunk):
            b = min(n_reads, a + chunk)
            c = win[starts[a:b]]
            m = rc[a:b]
            c[m] = 3 - c[m][:, ::-1]
            codes[a:b] = c
        return codes, lengths.astype(np.uint16)
    # mixed lengths: windows of hi bases of a zero-padded genome.  A forward read
    # is the window at its start; a reverse-complemented one is the window that
    # ENDS at its last base, reversed and complemented (so its first len codes
    # are rc(genome[start:start+len])); codes past len are zeroed.
    k = np.arange(hi, dtype=np.int64)[None, :]
    gp = np.zeros(G + 2 * hi, dtype=np.uint8)
    gp[hi:hi + G] = genome
    win = np.lib.stride_tricks.sliding_window_view(gp, hi)
    for a in range(0, n_reads, chunk):
        b = min(n_reads, a + chunk)
        s0, ln, m = starts[a:b], lengths[a:b], rc[a:b]
        c = win[s0 + hi]
        if m.any():
            c[m] = 3 - win[s0[m] + ln[m]][:, ::-1]
        c[k >= ln[:, None]] = 0
        codes[a:b] = c
    return codes, lengths.astype(np.uint16)


def uniform_read_set(n_reads: int, read_len: int, genome_len: int, seed: int,
                     lo: int | None = None, hi: int | None = None):
    """Config-style set: genome from ``seed``, reads from ``seed + 1``."""
    g = random_genome(genome_len, seed)
    lo = read_len if lo is None else lo
    hi = read_len if hi is None else hi
    return sample_reads(g, n_reads, lo, hi, seed + 1)


def metagenome_read_set(n_reads: int, lo: int, hi: int, n_genomes: int, total_len: int,
                        seed: int, sigma: float = 1.0):
    """C5-style metagenome: ``n_genomes`` random genomes with log-normal
    abundance; reads drawn per genome proportionally to abundance x length."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(total_len // (2 * n_genomes), 3 * total_len // (2 * n_genomes) + 1,
                         size=n_genomes)
    abund = rng.lognormal(0.0, sigma, size=n_genomes)
    w = abund * sizes
    counts = np.floor(w / w.sum() * n_reads).astype(np.int64)
    counts[0] += n_reads - counts.sum()
    parts_c, parts_l = [], []
    for gi in range(n_genomes):
        if counts[gi] == 0:
            continue
        g = random_genome(int(sizes[gi]), seed * 1000003 + gi)
        c, l = sample_reads(g, int(counts[gi]), lo, hi, seed * 7919 + gi)
        parts_c.append(c)
        parts_l.append(l)
    codes = np.concatenate(parts_c)
    lengths = np.concatenate(parts_l)
    perm = np.random.default_rng(seed + 17).permutation(codes.shape[0])
    return codes[perm], lengths[perm]


def codes_to_strings(codes: np.ndarray, lengths: np.ndarray) -> list[str]:
    asc = ALPHABET[codes]
    return [asc[i, : int(lengths[i])].tobytes().decode() for i in range(codes.shape[0])]


def write_fasta(path: str, seqs, wrap: int = 0) -> None:
    with open(path, "w") as f:
        for i, s in enumerate(seqs):
            f.write(f">r{i}\n")
            if wrap and len(s) > wrap:
                for p in range(0, len(s), wrap):
                    f.write(s[p:p + wrap] + "\n")
            else:
                f.write(s + "\n")


def write_fastq(path: str, seqs) -> None:
    with open(path, "w") as f:
        for i, s in enumerate(seqs):
            f.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")


def revcomp_str(s: str) -> str:
    return s.translate(str.maketrans("ACGTacgt", "TGCAtgca"))[::-1]
