"""record splitting throughput (mgh_parse_file,
metagenomics_amd/csrc/host/mg_parse.cpp) with Dataset::readDataset's exact
semantics (Dataset.cpp:110-193).

Checker: oracle.readdataset_records, the reference's getline loop restated with
libstdc++'s getline/sentry behaviour, pinned to the reference itself on the
quirk it produces (tests/golden/parse_cases.json: the reference's Dataset on
every hand case, via oracle/_ref/ref_harness; make_golden.py --parse).
The parallel splitter is compared record by record at many chunk sizes and
thread counts, so every chunk seam position is exercised."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ids_sha256
from metagenomics_amd.overlap import Dataset, MgError, parse_buffer, parse_file
from oracle import readdataset_records


def records(text, offs):
    b = text.tobytes()
    return [b[int(offs[i]):int(offs[i + 1])] for i in range(offs.shape[0] - 1)]


def nonempty(recs):
    # the reference's loop adds empty records at EOF (always bad reads, never stored)
    return [r for r in recs if r]


def cases():
    with open(os.path.join(GOLDEN, "parse_cases.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_hand_cases_match_reference(case, tmp_path):
    data = case["input"].encode()
    want = nonempty(readdataset_records(data))
    for threads, chunk in ((1, 0), (4, 1), (3, 2), (8, 5), (2, 7)):
        assert nonempty(records(*parse_buffer(data, threads, chunk))) == want, (threads, chunk)
    # the reference's own Dataset on the same file (IDs -> canonical strings)
    p = tmp_path / ("in" + case["ext"])
    p.write_bytes(data)
    ds = Dataset.from_files([str(p)], case["l"])
    assert ds.num_unique == case["n_unique"]
    assert ds.num_reads == case["n_reads"]
    assert ids_sha256(ds.read, ds.num_unique) == case["ids_sha256"]


def random_file(rng, fastq: bool, n: int) -> bytes:
    out = []
    for i in range(n):
        L = int(rng.integers(0, 40))
        s = "".join(rng.choice(list("ACGTacgtN"), size=L))
        if fastq:
            out.append("@r%d%s\n%s\n+\n%s\n" % (i, ">" if i % 7 == 0 else "", s, "I" * L))
        else:
            hdr = ">r%d%s" % (i, " x>y" if i % 5 == 0 else "")
            wrap = int(rng.integers(1, 12))
            body = "\n".join(s[k:k + wrap] for k in range(0, len(s), wrap))
            if i % 9 == 0:
                body = body.replace("\n", "\r\n")
            out.append(hdr + "\n" + body + ("\n" if i % 4 else ""))
    txt = "".join(out)
    if not fastq and rng.random() < 0.5:
        txt += ">tailheader" + "ACGT" * int(rng.integers(0, 5))  # ends inside a header
    if rng.random() < 0.3:
        txt = txt.rstrip("\n")
    return txt.encode()


@pytest.mark.parametrize("fastq", [False, True])
def test_random_files_every_seam(fastq):
    rng = np.random.default_rng(5 + fastq)
    for trial in range(12):
        data = random_file(rng, fastq, int(rng.integers(1, 60)))
        want = nonempty(readdataset_records(data))
        for chunk in (1, 2, 3, 5, 8, 13, 64):
            got = nonempty(records(*parse_buffer(data, 4, chunk)))
            assert got == want, (trial, chunk)


def test_unknown_format_and_missing_file(tmp_path):
    for bad in (b"", b"ACGT\n", b"\n>r\nACGT\n"):
        with pytest.raises(MgError):
            parse_buffer(bad)
    with pytest.raises(MgError):
        parse_file(str(tmp_path / "absent.fa"))


def test_large_file_threads_agree(tmp_path):
    """~24 MB FASTQ and FASTA: 1 thread == 8 threads, offsets/text identical."""
    from metagenomics_amd import synth

    c, L = synth.uniform_read_set(80_000, 150, 400_000, seed=3)
    seqs = synth.codes_to_strings(c, L)
    fq, fa = tmp_path / "x.fq", tmp_path / "x.fa"
    synth.write_fastq(str(fq), seqs)
    fa.write_text("".join(">r%d\n%s\n%s\n" % (i, s[:70], s[70:]) for i, s in enumerate(seqs)))
    for p in (fq, fa):
        t1, o1, _ = parse_file(str(p), 1)
        t8, o8, _ = parse_file(str(p), 8)
        assert np.array_equal(o1, o8) and np.array_equal(t1, t8)
        assert o1.shape[0] - 1 == len(seqs)
        assert t1[: int(o1[1])].tobytes().decode() == seqs[0]
