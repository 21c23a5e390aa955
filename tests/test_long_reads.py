"""Reads longer than 1,024 bp, up to Read::getReadLength's UINT16 (Read.h:62):
the long-read kernels (k_index_long, k_probe_long, k_ingest_long) behind the
same C-ABI, against the oracle (a plain-C restatement of the reference pinned
to the reference's own outputs, tests/test_oracle.py).  Bit-exact rows and
superReadIDs; getListOfReads order; the device Dataset ingest."""
import numpy as np
import pytest

from metagenomics_amd import synth
from metagenomics_amd.overlap import Dataset, OverlapEngine, rows_to_tuples
from oracle import OracleDataset, sorted_tuples

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = OverlapEngine(0)
    yield e
    e.close()


def run(engine, ds, l, k=0, shard=(0, 1, 0, 0)):
    engine.set_option("nb_log2", 0)
    engine.set_shard(*shard)
    engine.upload(ds)
    engine.build_index(l, k)
    sup = engine.mark_contained()
    rows = engine.rows(engine.find_overlaps())
    return rows, sup


def oracle_of(seqs, l):
    od = OracleDataset.from_strings(seqs, l)
    rows, sup, _, _ = od.overlaps(l)
    return od, sorted_tuples(rows), sup


def long_set(n, lo, hi, G, seed):
    c, L = synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)
    return synth.codes_to_strings(c, L)


# (reads, lo, hi, genome, l, k, seed): 2-20 kb sets with containment (mixed
# lengths), a uniform-length set (no containment pass), the UINT16 ceiling
LONG_CASES = {
    "2k_20k": (240, 2000, 20000, 150_000, 60, 31, 201),
    "uniform_3k": (300, 3000, 3000, 120_000, 50, 31, 202),
    "1025_1500": (500, 1025, 1500, 60_000, 40, 21, 203),
    "max_65535": (12, 60000, 65535, 200_000, 100, 32, 204),
}


@pytest.mark.parametrize("name", sorted(LONG_CASES))
def test_long_reads_vs_oracle(engine, name):
    n, lo, hi, G, l, k, seed = LONG_CASES[name]
    seqs = long_set(n, lo, hi, G, seed)
    ds = Dataset.from_strings(seqs, l)
    od, orows, osup = oracle_of(seqs, l)
    assert ds.num_unique == od.num_unique
    rows, sup = run(engine, ds, l, k)
    assert np.array_equal(sup.astype(np.uint64), osup)
    t = rows_to_tuples(rows)
    assert t.shape[0] > 0
    assert np.array_equal(t, orows)


def test_long_and_short_reads_mixed(engine):
    """150 bp reads next to 1.5-8 kb reads of the same genome: one long-mode
    context (slot width from the longest read), containment of the short reads
    in the long ones, exact prefixes (offset-0 containment) of both strands."""
    rng = np.random.default_rng(205)
    g = synth.codes_to_strings(synth.random_genome(40_000, 205)[None, :], np.array([40_000], np.uint16))[0]
    comp = str.maketrans("ACGT", "TGCA")
    rc = lambda x: x.translate(comp)[::-1]  # noqa: E731
    seqs = []
    for _ in range(400):
        p = int(rng.integers(0, 40_000 - 150))
        s = g[p:p + 150]
        seqs.append(rc(s) if rng.random() < 0.5 else s)
    for _ in range(40):
        L = int(rng.integers(1500, 8000))
        p = int(rng.integers(0, 40_000 - L))
        s = g[p:p + L]
        seqs.append(rc(s) if rng.random() < 0.5 else s)
        seqs.append(s[:150])          # exact prefix: found only through suffix keys
        seqs.append(rc(s[:700]))      # reverse-complement prefix
    ds = Dataset.from_strings(seqs, 50)
    od, orows, osup = oracle_of(seqs, 50)
    rows, sup = run(engine, ds, 50, 31)
    assert int((osup != 0).sum()) > 100
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), orows)


def test_long_tandem_self_overlaps(engine):
    """Tandem repeats longer than 1 kb: self-overlaps (4 rows per forward self
    hit) and multi-edges through the long probe."""
    unit = "ACGTTGCAAGGCTTACGATCGATTACGGATCCAGT"
    seqs = [unit * 40, (unit * 60)[5:], "TTGCA" + unit * 35]
    ds = Dataset.from_strings(seqs, 60)
    od, orows, osup = oracle_of(seqs, 60)
    rows, sup = run(engine, ds, 60, 25)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), orows)


def test_long_reads_source_shards(engine):
    """Replicated-index source-range shards on long reads:
    the union over ranks is the whole multiset."""
    n, lo, hi, G, l, k, seed = LONG_CASES["2k_20k"]
    seqs = long_set(n, lo, hi, G, seed)
    ds = Dataset.from_strings(seqs, l)
    _, orows, _ = oracle_of(seqs, l)
    N, P = ds.num_unique, 3
    parts = []
    for r in range(P):
        rows, _ = run(engine, ds, l, k, shard=(0, 1, r * N // P, (r + 1) * N // P))
        assert rows.shape[0] > 0
        parts.append(rows)
    engine.set_shard(0, 1)
    assert np.array_equal(rows_to_tuples(np.concatenate(parts)), orows)


def test_long_reads_lookup(engine):
    """getListOfReads (HashTable.cpp:202-221) on a long-read index, list order
    included, against the oracle."""
    n, lo, hi, G, l, k, seed = LONG_CASES["1025_1500"]
    seqs = long_set(n, lo, hi, G, seed)
    ds = Dataset.from_strings(seqs, l)
    od = OracleDataset.from_strings(seqs, l)
    engine.set_option("nb_log2", 0)
    engine.set_shard(0, 1)
    engine.upload(ds)
    engine.build_index(l, k)
    h = l - 1
    checked = 0
    for rid in range(1, ds.num_unique + 1, 37):
        s = ds.read(rid)
        for key in (s[:h], s[-h:], synth.revcomp_str(s)[:h], s[500:500 + h]):
            exp = od.lookup(l, key)
            assert engine.lookup(key) == exp, key
            checked += len(exp)
    assert checked > 0


def test_long_reads_device_ingest(engine):
    """k_ingest_long: testRead, canonical strand, std::string order and
    dedup for reads > 1 kb equal the host Dataset mirror; then the rows."""
    n, lo, hi, G, l, k, seed = LONG_CASES["1025_1500"]
    c, L = synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)
    c = np.concatenate([c, c[:50]])              # duplicates
    L = np.concatenate([L, L[:50]])
    c[7, 1100] = 4                               # an invalid base
    c[8, :] = 1                                  # low complexity (80 % rule)
    ds = Dataset.from_codes(c, L, l)
    engine.set_option("nb_log2", 0)
    engine.set_shard(0, 1)
    nu = engine.ingest_codes(c, L, l)
    assert nu == ds.num_unique
    w1, l1 = engine.download_packed()
    w0, l0 = ds.packed()
    assert np.array_equal(l0, l1)
    assert np.array_equal(w0, w1[:, : w0.shape[1]])
    assert engine.dataset_counts() == (ds.num_reads, ds.num_unique)
    assert int(engine.frequency().sum()) == ds.num_reads
    engine.build_index(l, k)
    sup = engine.mark_contained()
    rows = engine.rows(engine.find_overlaps())
    seqs = [ds.read(i) for i in range(1, ds.num_unique + 1)]
    _, orows, osup = oracle_of(seqs, l)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), orows)


def test_long_reads_exchange_refused(engine):
    """The bucket-sharded exchange kernels are for reads <= 1 kb: at the C-ABI a
    clear error (sharded_step falls back to the replicated mode, below)."""
    seqs = long_set(20, 1500, 2000, 20_000, 206)
    ds = Dataset.from_strings(seqs, 50)
    engine.set_shard(0, 1)
    engine.upload(ds)
    with pytest.raises(RuntimeError, match="1024"):
        engine.xchg_begin(50, 31)


@pytest.mark.parametrize("world", [1, 3])
def test_long_reads_exchange_step_falls_back(world):
    """sharded_step (the multi-GPU default, bench --gpus N) on a set with reads
    over 1,024 bp runs the replicated mode (whole index per rank, source-range
    shards) and says so: the union over the simulated ranks is the reference's
    multiset (the reference-generated longreads fixture: 150 bp-9 kb reads) and
    the superReadIDs are the reference's."""
    import torch

    from conftest import fixture_input, golden_rows, load_meta
    from metagenomics_amd.sharded import LocalExchange, sharded_step

    meta = load_meta("longreads")
    l = meta["l"]
    ds = Dataset.from_files([fixture_input("longreads")], l)
    engines = []
    for r in range(world):
        e = OverlapEngine(0)
        e.set_shard(r, world, 0, 0)
        e.upload(ds)
        engines.append(e)
    assert max(e.max_len for e in engines) > 1024
    xchg = LocalExchange(world, torch.device("cuda:0"))
    res = sharded_step(engines, xchg, l, 0, want_super=True)
    assert res.mode == "replicated"
    assert set(res.ms) == {"index", "contained", "overlap"} and res.ms["index"] > 0
    rows = np.concatenate([res.rows_numpy(r) for r in range(world)])
    assert sum(res.n_rows) == rows.shape[0]
    assert np.array_equal(rows_to_tuples(rows), golden_rows("longreads"))
    assert {str(i): int(x) for i, x in enumerate(res.super_read_id) if x} == meta["super"]
    # the same engines then take a short-read set: the fallback gave them their
    # bucket-range shards back, so this step is a real exchange step
    m2 = load_meta("mixed")
    ds2 = Dataset.from_files([fixture_input("mixed")], m2["l"])
    for e in engines:
        e.upload(ds2)
    res2 = sharded_step(engines, xchg, m2["l"], 0, want_super=True)
    assert res2.mode == "exchange"
    rows2 = np.concatenate([res2.rows_numpy(r) for r in range(world)])
    for e in engines:
        e.close()
    assert np.array_equal(rows_to_tuples(rows2), golden_rows("mixed"))
    assert {str(i): int(x) for i, x in enumerate(res2.super_read_id) if x} == m2["super"]
