"""The oracle (C restatement, oracle/mg_oracle.c) against the reference's own
outputs committed in tests/golden/ (made by oracle/_ref/ref_harness, i.e. the
reference's Dataset/HashTable/OverlapGraph compiled in place)."""
import numpy as np
import pytest

from conftest import FIXTURES, fixture_input, golden_rows, ids_sha256, load_meta, rows_sha256
from oracle import OracleDataset, sorted_tuples


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference_fixture(name):
    meta = load_meta(name)
    ds = OracleDataset.from_files([fixture_input(name)], meta["l"])
    assert ds.num_unique == meta["n_unique"]
    assert ids_sha256(ds.read, ds.num_unique) == meta["ids_sha256"]
    rows, sup, _, _ = ds.overlaps(meta["l"])
    t = sorted_tuples(rows)
    g = golden_rows(name)
    assert t.shape == g.shape
    assert np.array_equal(t, g)
    assert rows_sha256(t) == meta["rows_sha256"]
    got_super = {str(i): int(s) for i, s in enumerate(sup) if s}
    assert got_super == meta["super"]


def test_oracle_c1_digest():
    """BASELINE configs[0] (100k x 100 bp, l=40): digest of the reference's rows."""
    from metagenomics_amd import synth

    meta = load_meta("c1")
    r = meta["recipe"]
    c, L = synth.uniform_read_set(r["n_reads"], r["read_len"], r["genome_len"], r["seed"])
    ds = OracleDataset.from_strings(synth.codes_to_strings(c, L), meta["l"])
    assert ds.num_unique == meta["n_unique"]
    rows, _, _, _ = ds.overlaps(meta["l"])
    assert rows.shape[0] == meta["directed_rows"]
    assert rows_sha256(sorted_tuples(rows)) == meta["rows_sha256"]


def test_oracle_lookup_matches_reference_order():
    """getListOfReads order: ID ascending then orientation (HashTable.cpp:58-60,98-101)."""
    meta = load_meta("highdup")
    ds = OracleDataset.from_files([fixture_input("highdup")], meta["l"])
    h = meta["l"] - 1
    s = ds.read(1)
    lst = ds.lookup(meta["l"], s[:h])
    assert lst, "prefix of read 1 must be in the table"
    assert (1, 0) in lst
    assert lst == sorted(lst)


@pytest.mark.parametrize("name", ["highdup", "tandem", "mixed"])
def test_oracle_lookup_golden(name):
    meta = load_meta(name)
    ds = OracleDataset.from_files([fixture_input(name)], meta["l"])
    for key, exp in meta["lookups"].items():
        assert [list(x) for x in ds.lookup(meta["l"], key)] == exp, key


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_oracle_threaded_digest_matches_reference_fixture(name, nthreads):
    """mgo_overlaps_digest (source-range threads, digests only; the recipe of
    the 50M C5 golden) == the reference's rows and superReadIDs on every fixture."""
    import digest

    meta = load_meta(name)
    ds = OracleDataset.from_files([fixture_input(name)], meta["l"])
    rd, sd, sup, _ = ds.overlaps_digest(meta["l"], nthreads, want_super=True)
    g = golden_rows(name)
    assert rd == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]
    s = np.zeros(meta["n_unique"] + 1, dtype=np.uint64)
    for k, v in meta["super"].items():
        s[int(k)] = v
    assert sd == digest.super_digest(s)


def test_oracle_from_codes_equals_from_strings():
    from metagenomics_amd import synth

    c, L = synth.metagenome_read_set(3000, 100, 250, 5, 60_000, 9)
    a = OracleDataset.from_codes(c, L, 50)
    b = OracleDataset.from_strings(synth.codes_to_strings(c, L), 50)
    assert a.num_unique == b.num_unique and a.num_reads == b.num_reads
    assert all(a.read(i) == b.read(i) for i in range(1, a.num_unique + 1, 7))
