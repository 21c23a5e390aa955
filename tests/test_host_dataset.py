"""Host Dataset mirror (metagenomics_amd/csrc/host, via include/mg_host.h)
against the reference's ID -> canonical-string map and read counts
(Dataset.cpp:110-202,316-345,398-413), on CPU."""
import numpy as np
import pytest

from conftest import FIXTURES, fixture_input, ids_sha256, load_meta
from metagenomics_amd import synth
from metagenomics_amd.overlap import Dataset
from oracle import OracleDataset


@pytest.mark.parametrize("name", FIXTURES)
def test_dataset_ids_match_reference(name):
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    assert ds.num_unique == meta["n_unique"]
    assert ids_sha256(ds.read, ds.num_unique) == meta["ids_sha256"]


@pytest.mark.parametrize("name", ["dirty", "mixed", "highdup"])
def test_dataset_counts_match_oracle(name):
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    od = OracleDataset.from_files([fixture_input(name)], meta["l"])
    assert ds.num_reads == od.num_reads
    freqs = [ds.frequency(i) for i in range(1, ds.num_unique + 1)]
    assert freqs == [od.frequency(i) for i in range(1, od.num_unique + 1)]
    assert sum(freqs) == ds.num_reads


def test_from_codes_equals_from_files(tmp_path):
    c, L = synth.uniform_read_set(500, 0, 3000, seed=3, lo=60, hi=120)
    seqs = synth.codes_to_strings(c, L)
    p = tmp_path / "r.fa"
    synth.write_fasta(str(p), seqs)
    a = Dataset.from_files([str(p)], 30)
    b = Dataset.from_codes(c, L, 30, nthreads=4)
    wa, la = a.packed()
    wb, lb = b.packed()
    assert np.array_equal(la, lb) and np.array_equal(wa, wb)
    assert a.shortest == b.shortest and a.longest == b.longest


def test_find_read_either_strand():
    c, L = synth.uniform_read_set(200, 80, 2000, seed=4)
    seqs = synth.codes_to_strings(c, L)
    ds = Dataset.from_strings(seqs, 40)
    for s in seqs[:50]:
        rid = ds.find(s)
        assert rid >= 1
        assert ds.read(rid) in (s, synth.revcomp_str(s))
        assert ds.find(synth.revcomp_str(s)) == rid
    assert ds.find("ACGT" * 20 + "N") == 0


def test_dataset_filters():
    # len <= l, non-ACGT, >= 80 % one base are dropped; lower case accepted
    good = "ACGTTGCAAGGCTTACGATC" * 3
    reads = [good, good.lower(), "A" * 50 + "CGT" * 3, good[:30], good[:-1] + "N", synth.revcomp_str(good)]
    ds = Dataset.from_strings(reads, 30)
    od = OracleDataset.from_strings(reads, 30)
    assert ds.num_reads == od.num_reads == 3
    assert ds.num_unique == od.num_unique == 1
    assert ds.frequency(1) == 3
    assert ds.read(1) == min(good, synth.revcomp_str(good))


def test_empty_dataset():
    ds = Dataset.from_strings(["ACGT"], 30)
    assert ds.num_unique == 0 and ds.num_reads == 0
