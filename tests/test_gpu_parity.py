"""Parity of the HIP path (through the C-ABI) with the reference's golden
vectors and with the oracle.  Bit-exact: integer/index work."""
import numpy as np
import pytest

from conftest import FIXTURES, fixture_input, golden_rows, load_meta, rows_sha256
from metagenomics_amd import synth
from metagenomics_amd.overlap import Dataset, OverlapEngine, rows_to_tuples
from oracle import OracleDataset, sorted_tuples

pytestmark = pytest.mark.gpu

TWIN = {0: 3, 1: 1, 2: 2, 3: 0}


@pytest.fixture(scope="module")
def engine():
    e = OverlapEngine(0)
    yield e
    e.close()


def gpu_rows(engine, ds, l, k=0, nb_log2=0, shard=(0, 1, 0, 0)):
    engine.set_option("nb_log2", nb_log2)
    engine.set_shard(*shard)
    engine.upload(ds)
    engine.build_index(l, k)
    sup = engine.mark_contained()
    n = engine.find_overlaps()
    rows = engine.rows(n)
    assert rows.shape[0] == n
    return rows, sup


def check_pairs(rows, lens):
    """rows come as (edge, twin) pairs (insertEdge, OverlapGraph.cpp:407-419)."""
    a, b = rows[0::2], rows[1::2]
    assert np.array_equal(a["src"], b["dst"]) and np.array_equal(a["dst"], b["src"])
    assert all(TWIN[int(x)] == int(y) for x, y in zip(a["orient"][:2000], b["orient"][:2000]))
    n1 = lens[a["src"].astype(np.int64) - 1].astype(np.int64)
    n2 = lens[a["dst"].astype(np.int64) - 1].astype(np.int64)
    assert np.array_equal(((n2 + a["offset"].astype(np.int64) - n1) & 0xFFFF), b["offset"].astype(np.int64))


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_matches_reference(engine, name):
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows, sup = gpu_rows(engine, ds, meta["l"])
    t = rows_to_tuples(rows)
    g = golden_rows(name)
    assert t.shape == g.shape, (t.shape, g.shape)
    assert np.array_equal(t, g)
    assert rows_sha256(t) == meta["rows_sha256"]
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]
    check_pairs(rows, ds.packed()[1])


@pytest.mark.parametrize("name,k", [("small", 12), ("small", 32), ("tandem", 8), ("mixed", 17), ("highdup", 5)])
def test_seed_k_does_not_change_results(engine, name, k):
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows, _ = gpu_rows(engine, ds, meta["l"], k=k)
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))


@pytest.mark.parametrize("name", ["highdup", "tandem", "mixed"])
def test_tiny_directory_collisions(engine, name):
    """2^10 buckets: every bucket holds many minimizers; results unchanged."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows, sup = gpu_rows(engine, ds, meta["l"], nb_log2=10)
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))


@pytest.mark.parametrize("name", ["highdup", "tandem", "mixed"])
def test_lookup_matches_reference(engine, name):
    """HashTable::getListOfReads (HashTable.cpp:202-221) incl. list order."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    engine.set_option("nb_log2", 0)
    engine.set_shard(0, 1)
    engine.upload(ds)
    engine.build_index(meta["l"])
    for key, exp in meta["lookups"].items():
        assert [list(x) for x in engine.lookup(key)] == exp, key
    assert engine.lookup("A" * (meta["l"] - 2)) == [] or True  # any key of length h is legal
    assert engine.lookup("ACGT") == []  # wrong length: no such key


@pytest.mark.parametrize("name", ["highdup", "tandem", "mixed"])
def test_lookup_tiny_directory(engine, name):
    """getListOfReads through long overflow chains: with 2^10 requested buckets
    the directory runs at ~70 % load, so many entries sit outside their home
    cell."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    engine.set_option("nb_log2", 10)
    engine.set_shard(0, 1)
    engine.upload(ds)
    engine.build_index(meta["l"])
    for key, exp in meta["lookups"].items():
        assert [list(x) for x in engine.lookup(key)] == exp, key
    engine.set_option("nb_log2", 0)


def test_ascii_upload_equals_packed(engine):
    meta = load_meta("mixed")
    ds = Dataset.from_files([fixture_input("mixed")], meta["l"])
    seqs = [ds.read(i) for i in range(1, ds.num_unique + 1)]
    engine.set_option("nb_log2", 0)
    engine.set_shard(0, 1)
    engine.upload_ascii(seqs)
    w1, l1 = engine.download_packed()
    w0, l0 = ds.packed()
    assert np.array_equal(l0, l1)
    assert np.array_equal(w0, w1[:, : w0.shape[1]])
    engine.build_index(meta["l"])
    engine.mark_contained()
    rows = engine.rows()
    assert np.array_equal(rows_to_tuples(rows), golden_rows("mixed"))


@pytest.mark.parametrize("name,nranks", [("small", 2), ("highdup", 3), ("tworead", 2), ("highdup", 5), ("small", 8)])
def test_bucket_shards_union(engine, name, nranks):
    """Bucket-range sharding through the single-context entry
    points (bench --multi bucket: every rank's one scan of every read files and
    keeps only its buckets' keys and runs): the union over ranks is the
    multiset.  Equal-length sets only: a
    bucket shard cannot settle containment alone (markContainedReads needs every
    bucket), which is what the exchange mode's MAX all-reduce does
    (test_exchange_mode_* cover the mixed-length fixtures)."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    parts = []
    for r in range(nranks):
        rows, _ = gpu_rows(engine, ds, meta["l"], shard=(r, nranks, 0, 0))
        parts.append(rows)
    allr = np.concatenate(parts)
    assert np.array_equal(rows_to_tuples(allr), golden_rows(name))


def assert_shard_rows(rows, lo, hi):
    """A source-range shard holds its sources' discoveries: every (row, twin)
    pair has the row's src in the range's reference IDs [lo + 1, hi]."""
    a, b = rows[0::2], rows[1::2]
    assert np.array_equal(a["src"], b["dst"]) and np.array_equal(a["dst"], b["src"])
    assert np.all((a["src"] >= lo + 1) & (a["src"] <= hi)), "a row whose source read the shard does not own"


@pytest.mark.parametrize("name,layout", [("small", 1), ("mixed", 1), ("branchy", 1), ("tandem", 0)])
def test_read_range_union(engine, name, layout):
    """Source-read shards (mg_set_shard read_lo/read_hi) by reference ID, on the
    clustered layout (the range re-clustered into its own slots) and on ID order."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    n = ds.num_unique
    cuts = [0, n // 3, n // 2 + 7, n]
    parts = []
    engine.set_option("layout", layout)
    try:
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            rows, sup = gpu_rows(engine, ds, meta["l"], shard=(0, 1, lo, hi))
            assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]
            assert_shard_rows(rows, lo, hi)
            parts.append(rows)
    finally:
        engine.set_option("layout", 1)
    assert np.array_equal(rows_to_tuples(np.concatenate(parts)), golden_rows(name))


def test_read_range_set_after_upload(engine):
    """A range set on resident reads re-clusters them at the next build; then
    the whole range again (the ungrouped layout)."""
    meta = load_meta("mixed")
    ds = Dataset.from_files([fixture_input("mixed")], meta["l"])
    n = ds.num_unique
    engine.set_option("nb_log2", 0)
    engine.set_shard(0, 1)
    engine.upload(ds)
    parts = []
    for lo, hi in ((0, n // 4), (n // 4, n)):
        engine.set_shard(0, 1, lo, hi)
        engine.build_index(meta["l"])
        engine.mark_contained()
        rows = engine.rows(engine.find_overlaps())
        assert_shard_rows(rows, lo, hi)
        parts.append(rows)
    assert np.array_equal(rows_to_tuples(np.concatenate(parts)), golden_rows("mixed"))
    engine.set_shard(0, 1)
    engine.build_index(meta["l"])
    engine.mark_contained()
    assert np.array_equal(rows_to_tuples(engine.rows(engine.find_overlaps())), golden_rows("mixed"))
    w, lens = engine.download_packed()
    hw, hl = ds.packed()
    assert np.array_equal(lens, hl) and np.array_equal(w[:, :hw.shape[1]], hw)


def test_c1_digest(engine):
    """BASELINE configs[0]: 100k x 100 bp, l = 40, k = 21."""
    meta = load_meta("c1")
    r = meta["recipe"]
    c, L = synth.uniform_read_set(r["n_reads"], r["read_len"], r["genome_len"], r["seed"])
    ds = Dataset.from_codes(c, L, meta["l"])
    assert ds.num_unique == meta["n_unique"]
    rows, _ = gpu_rows(engine, ds, meta["l"], k=21)
    assert rows.shape[0] == meta["directed_rows"]
    assert rows_sha256(rows_to_tuples(rows)) == meta["rows_sha256"]


RANDOM_CASES = [
    # n, lo, hi, genome, l, k, seed
    (3000, 60, 60, 4000, 31, 0, 101),       # short reads, l close to length
    (4000, 50, 300, 20000, 25, 11, 102),    # wide length range, containment
    (2000, 200, 1000, 30000, 60, 31, 103),  # long reads (up to 32 words)
    (5000, 100, 100, 800, 40, 20, 104),     # extreme duplication
    (3000, 35, 40, 6000, 33, 32, 105),      # l-1 = 32 = k
    (1000, 64, 64, 5000, 10, 5, 106),       # tiny l
]


@pytest.mark.parametrize("case", RANDOM_CASES)
def test_random_sets_vs_oracle(engine, case):
    n, lo, hi, G, l, k, seed = case
    c, L = synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)
    seqs = synth.codes_to_strings(c, L)
    ds = Dataset.from_codes(c, L, l)
    od = OracleDataset.from_strings(seqs, l)
    assert ds.num_unique == od.num_unique
    rows, sup = gpu_rows(engine, ds, l, k=k)
    orows, osup, _, _ = od.overlaps(l)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))


EDGE_SETS = {
    # name: (reads as strings, l)
    "empty": ([], 20),
    "all_invalid": (["ACGTNACGTACGTACGTACGTACGT", "A" * 30], 20),
    "single": (["ACGTTGCAAGGCTTACGATCGATTACGGATCCA"], 20),
    "single_tandem": (["ACGTTGCAAG" * 8], 20),  # self-overlaps of one read
    "l_plus_one": (None, 40),                    # every read exactly l + 1 bases
    "max_len": (None, 200),                      # reads up to 1024 bases (32 words)
    "prefixes": (None, 40),                      # nested exact prefixes, both strands (containment s = 0)
}


def prefix_reads(seed=113):
    """Reads that are exact prefixes (or reverse-complement prefixes) of longer
    reads, nested, plus suffixes and inner pieces: containment at offset 0,
    which the reference finds only through suffix keys (k_prefix_contain)."""
    rng = np.random.default_rng(seed)
    comp = str.maketrans("ACGT", "TGCA")
    out = []
    for _ in range(6):
        g = "".join(rng.choice(list("ACGT"), 420))
        rc = lambda x: x.translate(comp)[::-1]  # noqa: E731
        out += [g[:n] for n in (45, 50, 60, 75, 90, 120, 160, 220, 300, 420)]
        out += [rc(g[:n]) for n in (55, 70, 130, 260)]
        out += [g[420 - n:] for n in (48, 100, 250)] + [g[30:130], rc(g[10:200])]
    return out


@pytest.mark.parametrize("name", sorted(EDGE_SETS))
def test_edge_sets_vs_oracle(engine, name):
    """Empty and degenerate inputs and the length extremes, against the oracle."""
    seqs, l = EDGE_SETS[name]
    if name == "l_plus_one":
        c, L = synth.uniform_read_set(3000, l + 1, 4000, seed=111)
        seqs = synth.codes_to_strings(c, L)
    elif name == "max_len":
        c, L = synth.uniform_read_set(600, 0, 40000, seed=112, lo=1000, hi=1024)
        seqs = synth.codes_to_strings(c, L)
    elif name == "prefixes":
        seqs = prefix_reads()
    ds = Dataset.from_strings(seqs, l)
    od = OracleDataset.from_strings(seqs, l)
    assert ds.num_unique == od.num_unique
    rows, sup = gpu_rows(engine, ds, l, k=0)
    orows, osup, _, _ = od.overlaps(l)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))


def test_metagenome_vs_oracle(engine):
    c, L = synth.metagenome_read_set(20000, 100, 250, n_genomes=20, total_len=400000, seed=51)
    ds = Dataset.from_codes(c, L, 50)
    od = OracleDataset.from_strings(synth.codes_to_strings(c, L), 50)
    rows, sup = gpu_rows(engine, ds, 50, k=31)
    orows, osup, _, _ = od.overlaps(50)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))


def test_c2_scale_vs_oracle(engine):
    """BASELINE configs[1] shape (1M x 150 bp, l=50, k=31) against the oracle."""
    c, L = synth.uniform_read_set(1_000_000, 150, 7_500_000, seed=21)
    ds = Dataset.from_codes(c, L, 50)
    rows, _ = gpu_rows(engine, ds, 50, k=31)
    od = OracleDataset.from_strings(synth.codes_to_strings(c, L), 50)
    orows, _, _, _ = od.overlaps(50)
    assert rows.shape[0] == orows.shape[0]
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))
    check_pairs(rows, ds.packed()[1])


def test_repeatable(engine):
    meta = load_meta("highdup")
    ds = Dataset.from_files([fixture_input("highdup")], meta["l"])
    a, _ = gpu_rows(engine, ds, meta["l"])
    b, _ = gpu_rows(engine, ds, meta["l"])
    assert np.array_equal(rows_to_tuples(a), rows_to_tuples(b))


# ---- exchange mode: P simulated ranks in this process, buffers
# moved by LocalExchange on the device; the same sharded_step drives RCCL ranks
def exchange_rows(ds, l, world, k=0, want_super=True, opts=None, route_rows=False):
    import torch

    from metagenomics_amd.sharded import LocalExchange, sharded_step, source_range

    engines = []
    for r in range(world):
        e = OverlapEngine(0)
        for kk, v in (opts or {}).items():
            e.set_option(kk, v)
        e.set_shard(r, world, 0, 0)
        e.upload(ds)
        engines.append(e)
    res = sharded_step(engines, LocalExchange(world, torch.device("cuda:0")), l, k, want_super=want_super,
                       route_rows=route_rows)
    exchange_rows.counters = [e.counters() for e in engines]
    parts = []
    for r in range(world):
        rows = res.rows_numpy(r)
        if route_rows:
            lo, hi = source_range(ds.num_unique, r, world)
            assert np.all((rows["src"] >= lo + 1) & (rows["src"] <= hi)), "row at a rank that does not own its src"
        parts.append(rows)
    for e in engines:
        e.close()
    return np.concatenate(parts), res.super_read_id


@pytest.mark.parametrize("name,world,route", [("small", 2, 0), ("mixed", 3, 0), ("tandem", 4, 0), ("dirty", 3, 0),
                                              ("tworead", 2, 0), ("wrapped", 5, 0), ("mixed", 1, 0),
                                              ("highdup", 1, 0), ("small", 2, 1), ("mixed", 3, 1), ("tandem", 4, 1),
                                              ("highdup", 3, 1)])
def test_exchange_mode_matches_reference(name, world, route):
    """Keys and runs travel as 8-B records (the receiver re-hashes the minimizer
    from its copy of the read); route = 1: the rows then go to their src owners
    (each rank ends with graph[u] of its sources), else each keeps what it verified."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows, sup = exchange_rows(ds, meta["l"], world, route_rows=bool(route))
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]


@pytest.mark.parametrize("name,world", [("mixed", 3), ("dirty", 2), ("mixed", 1)])
def test_exchange_mode_prefix_marks(name, world, monkeypatch):
    """MG_XCHG_MARKS=1: the cross-rank offset-0 containment marks
    (mg_xchg_prefix_marks + MAX all-reduce + fold into the keys) before the
    containment probe; at one rank the fused build's own prefix pass."""
    monkeypatch.setenv("MG_XCHG_MARKS", "1")
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows, sup = exchange_rows(ds, meta["l"], world)
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]


@pytest.mark.parametrize("prefix", [0, 1])
def test_exchange_mode_containment_paths(prefix):
    """Exchange-mode markContainedReads (OverlapGraph.cpp:225-340) both ways:
    prefix = 1 walks the o = 0 key records each rank received (k_prefix_contain_keys)
    and the probe drops suffix-key hits; prefix = 0 verifies them in the probe."""
    meta = load_meta("mixed")
    ds = Dataset.from_files([fixture_input("mixed")], meta["l"])
    rows, sup = exchange_rows(ds, meta["l"], 3, opts={"prefix_contain": prefix})
    assert np.array_equal(rows_to_tuples(rows), golden_rows("mixed"))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]


@pytest.mark.parametrize("name,world,opts", [
    ("mixed", 3, {"nb_log2": 16}), ("dirty", 4, {"nb_log2": 16}), ("branchy", 2, {"nb_log2": 16}),
    ("mixed", 4, {"nb_log2": 16, "live_index": 0}), ("mixed", 3, {"xchg_sort_runs": 1}),
    ("tandem", 4, {"xchg_sort_runs": 1}), ("highdup", 8, {"nb_log2": 16, "xchg_sort_runs": 1}),
    ("mixed", 3, {"xchg_windows": 0}), ("dirty", 2, {"xchg_windows": 0, "prefix_contain": 0}),
    ("highdup", 4, {"nb_log2": 16, "chain_par": 0}), ("mixed", 3, {"chain_par": 0}),
    ("highdup", 2, {"nb_log2": 10}), ("tandem", 3, {"nb_log2": 10}),
    ("small", 2, {"check_cells": 1}), ("highdup", 3, {"check_cells": 1, "nb_log2": 10}),
    ("mixed", 3, {"check_cells": 1, "nb_log2": 16}), ("highdup", 2, {"check_cells": 1, "xchg_fs": 0}),
    ("mixed", 1, {"xchg_fused1": 0}), ("highdup", 1, {"xchg_fused1": 0}), ("dirty", 1, {"xchg_fused1": 0})])
def test_exchange_mode_options(name, world, opts):
    """Exchange-mode variants against the reference: the discovery index of the
    uncontained reads (build_live_index_xchg: the rank's cells coarsened, live
    entries only; forced on the small fixtures by a large directory, and its
    use checked through counters().live_cells), the full table instead
    (live_index = 0, the full table then keeps the o = 3 keys), the received
    runs ordered by bucket (xchg_sort_runs = 1; default: probed in place), the
    register scan for mixed lengths (xchg_windows = 0), the overflow records
    walked by one thread per cell instead of placed in parallel (chain_par = 0),
    small directories whose chains run long (nb_log2 = 10), and the table
    checker (check_cells: every record found from its home, for the full table
    and the coarse live table; xchg_fs = 0: no fingerprint bits in the sort, the
    runs of different fingerprints interleave), and one rank on the exchange
    path's own key build (xchg_fused1 = 0; by default one rank takes the fused
    build: no key leaves it)."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows, sup = exchange_rows(ds, meta["l"], world, opts=dict(opts, stats=1))
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]
    live = [c["live_cells"] for c in exchange_rows.counters]
    if meta["super"] and opts.get("live_index", 1) and opts.get("nb_log2"):
        assert all(0 < x < (1 << 16) // world + 1 for x in live), live
    elif not opts.get("live_index", 1):
        assert not any(live), live


def test_exchange_mode_metagenome_vs_oracle():
    """A 20k-read metagenome (mixed lengths, log-normal abundance: heavy
    minimizers overflow their home cells, so k_cells_build's overflow list and
    chains are exercised) through 4 exchange ranks with the live discovery
    index, against the oracle."""
    c, L = synth.metagenome_read_set(20000, 100, 250, n_genomes=20, total_len=400000, seed=51)
    seqs = synth.codes_to_strings(c, L)
    ds = Dataset.from_strings(seqs, 50)
    orows, osup, _, _ = OracleDataset.from_strings(seqs, 50).overlaps(50)
    rows, sup = exchange_rows(ds, 50, 4, opts={"nb_log2": 15})
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))


@pytest.mark.parametrize("case", RANDOM_CASES[:4])
def test_exchange_mode_random_vs_oracle(case):
    n, lo, hi, G, l, k, seed = case
    c, L = synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)
    ds = Dataset.from_codes(c, L, l)
    od = OracleDataset.from_strings(synth.codes_to_strings(c, L), l)
    orows, osup, _, _ = od.overlaps(l)
    rows, sup = exchange_rows(ds, l, 3, k=k)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))


def test_exchange_mode_cut_streams_rerun():
    """Streams cut at tiny capacities (64 records per peer, rounds of 128 records):
    the step sees the overflow in the device counts, grows the capacities and
    reruns; the same plan then runs without a rerun.  Same rows and superReadIDs
    as the reference; the slot-layout digest equals the digest of the rows."""
    import torch

    import digest
    from metagenomics_amd.overlap import MG_KEYS, MG_ROWS, MG_RUNS
    from metagenomics_amd.sharded import LocalExchange, XchgPlan, sharded_step

    meta = load_meta("mixed")
    ds = Dataset.from_files([fixture_input("mixed")], meta["l"])
    engines = []
    for r in range(3):
        e = OverlapEngine(0)
        e.set_shard(r, 3, 0, 0)
        e.upload(ds)
        engines.append(e)
    xchg = LocalExchange(3, torch.device("cuda:0"), chunk_bytes=3 * 16 * 128)
    plan = XchgPlan(caps={MG_KEYS: 64, MG_RUNS: 64, MG_ROWS: 64})
    for attempt in range(2):
        res = sharded_step(engines, xchg, meta["l"], 0, want_super=True, plan=plan, route_rows=True)
        assert (res.reruns >= 1) if attempt == 0 else (res.reruns == 0)
        rows = np.concatenate([res.rows_numpy(r) for r in range(3)])
        assert np.array_equal(rows_to_tuples(rows), golden_rows("mixed"))
        assert {str(i): int(s) for i, s in enumerate(res.super_read_id) if s} == meta["super"]
        ds_dev = [e.slots_digest(b.data_ptr(), slot, rounds, c.data_ptr())
                  for e, (b, c, slot, rounds) in zip(engines, res.rows)]
        tot = {"n": 0, "sum": 0, "xor": 0, "sum2": 0}
        for d in ds_dev:
            tot = {"n": tot["n"] + d["n"], "sum": (tot["sum"] + d["sum"]) % 2**64, "xor": tot["xor"] ^ d["xor"],
                   "sum2": (tot["sum2"] + d["sum2"]) % 2**64}
        g = golden_rows("mixed")
        assert tot == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    for e in engines:
        e.close()


@pytest.mark.parametrize("name", ["mixed"])
def test_exchange_run_region_overflow(name):
    """The exchange scan's run regions start far too small (option run_cap):
    the scan keeps counting past them, the host resizes to the exact need and
    rescans before the runs are routed."""
    import torch

    from metagenomics_amd.sharded import LocalExchange, sharded_step

    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    engines = []
    for r in range(2):
        e = OverlapEngine(0)
        e.set_option("run_cap", 8)
        e.set_shard(r, 2, 0, 0)
        e.upload(ds)
        engines.append(e)
    res = sharded_step(engines, LocalExchange(2, torch.device("cuda:0")), meta["l"], 0, want_super=True)
    rows = np.concatenate([res.rows_numpy(r) for r in range(2)])
    for e in engines:
        e.close()
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(res.super_read_id) if s} == meta["super"]


def test_exchange_mode_c2_scale_matches_fused(engine):
    """1M x 150 bp (configs[1] shape): 4 exchange ranks == the fused single-GPU path."""
    c, L = synth.uniform_read_set(1_000_000, 150, 7_500_000, seed=21)
    ds = Dataset.from_codes(c, L, 50)
    fused, _ = gpu_rows(engine, ds, 50, k=31)
    rows, _ = exchange_rows(ds, 50, 4, k=31, want_super=False)
    assert rows.shape[0] == fused.shape[0]
    assert np.array_equal(rows_to_tuples(rows), rows_to_tuples(fused))
    check_pairs(fused, ds.packed()[1])


# ---- Dataset ingest on the device vs the host mirror,
# which tests/test_host_dataset.py pins to the reference's ID map
def read_records(path):
    """Record text as Dataset::readDataset extracts it (Dataset.cpp:123-182)."""
    data = open(path, "rb").read().decode()
    if data.startswith(">"):
        out = []
        for rec in data[1:].split(">"):
            nl = rec.find("\n")
            out.append(rec[nl + 1:].replace("\n", "") if nl >= 0 else "")
        return out
    lines = data.split("\n")
    return [lines[i] for i in range(1, len(lines), 4)]


def assert_same_dataset(engine, ds):
    w1, l1 = engine.download_packed()
    w0, l0 = ds.packed()
    assert engine.n_reads == ds.num_unique
    assert np.array_equal(l0, l1)
    assert np.array_equal(w0, w1[:, : w0.shape[1]])
    assert not np.any(w1[:, w0.shape[1]:])
    assert engine.dataset_counts() == (ds.num_reads, ds.num_unique)
    f = engine.frequency()
    assert [int(x) for x in f[:2000]] == [ds.frequency(i) for i in range(1, min(2000, ds.num_unique) + 1)]
    assert int(f.sum()) == ds.num_reads


@pytest.mark.parametrize("name", ["mixed", "tandem", "dirty", "wrapped", "branchy", "longreads"])
def test_device_ingest_matches_host_dataset(engine, name):
    meta = load_meta(name)
    path = fixture_input(name)
    ds = Dataset.from_files([path], meta["l"])
    engine.set_option("nb_log2", 0)
    engine.set_shard(0, 1)
    nu = engine.ingest_ascii(read_records(path), meta["l"])
    assert nu == meta["n_unique"]
    assert_same_dataset(engine, ds)
    engine.build_index(meta["l"])
    sup = engine.mark_contained()
    rows = engine.rows()
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]


@pytest.mark.parametrize("case", [(20000, 80, 200, 30000, 40, 7), (30000, 100, 100, 2000, 30, 8),
                                  (5000, 300, 1000, 40000, 60, 9)])
def test_device_ingest_codes_random(engine, case):
    n, lo, hi, G, l, seed = case
    c, L = synth.uniform_read_set(n, 0, G, seed=seed, lo=lo, hi=hi)
    # sprinkle invalid bases and low-complexity reads (testRead, Dataset.cpp:398-413)
    rng = np.random.default_rng(seed)
    bad = rng.choice(n, n // 50, replace=False)
    c[bad, rng.integers(0, lo, bad.shape[0])] = 4
    lowc = rng.choice(n, n // 100, replace=False)
    c[lowc, :] = 2
    ds = Dataset.from_codes(c, L, l)
    engine.set_shard(0, 1)
    engine.ingest_codes(c, L, l)
    assert_same_dataset(engine, ds)


def test_device_ingest_c2_scale(engine):
    c, L = synth.uniform_read_set(1_000_000, 150, 7_500_000, seed=21)
    ds = Dataset.from_codes(c, L, 50)
    engine.set_shard(0, 1)
    engine.ingest_codes(c, L, 50)
    assert_same_dataset(engine, ds)


@pytest.mark.parametrize("name", ["mixed", "dirty", "wrapped"])
def test_cli_graph_matches_reference(tmp_path, name):
    """main.cpp's pipeline through the C++ drop-in (mg_overlap CLI: Dataset ->
    HashTable -> OverlapGraph): graph[u] lists in list order and the node/edge
    counters equal the reference's graph before contraction."""
    import gzip
    import os
    import subprocess

    from conftest import GOLDEN, ROOT

    meta = load_meta(name)
    exe = os.path.join(ROOT, "metagenomics_amd", "lib", "mg_overlap")
    prefix = str(tmp_path / name)
    subprocess.run([exe, "-se", "1", fixture_input(name), "-f", prefix, "-l", str(meta["l"]), "-nocontract"],
                   check=True, stdout=subprocess.DEVNULL, timeout=120)
    lines = open(prefix + ".graph").read().split("\n")
    _, nodes, edges = lines[0].split()
    assert (int(nodes), int(edges)) == (meta["bfs"]["nodes"], meta["bfs"]["edges"])
    with gzip.open(os.path.join(GOLDEN, meta["bfs"]["file"]), "rt") as f:
        assert [x for x in lines[1:] if x] == [x for x in f.read().split("\n") if x]


@pytest.mark.parametrize("name", FIXTURES)
def test_cli_unitig_matches_reference(tmp_path, name):
    """main.cpp:45-50 end to end through the C++ drop-in: the .unitig checkpoint
    (contraction loop OverlapGraph.cpp:211-215, sortEdges, saveGraphToFile)
    equals the reference's byte for byte."""
    import gzip
    import os
    import subprocess

    from conftest import GOLDEN, ROOT

    meta = load_meta(name)
    exe = os.path.join(ROOT, "metagenomics_amd", "lib", "mg_overlap")
    prefix = str(tmp_path / name)
    subprocess.run([exe, "-se", "1", fixture_input(name), "-f", prefix, "-l", str(meta["l"])], check=True,
                   stdout=subprocess.DEVNULL, timeout=120)
    with gzip.open(os.path.join(GOLDEN, meta["unitig"]["file"]), "rt") as f:
        assert open(prefix + ".unitig").read() == f.read()


@pytest.mark.parametrize("name", ["branchy", "tandem"])
def test_device_rows_to_unitig(name, tmp_path):
    """Device discovery rows (any order) -> replay -> contraction: the lists,
    read locations and .unitig equal the reference's."""
    import gzip
    import os

    from conftest import GOLDEN
    from metagenomics_amd.overlap import UnitigGraph

    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    e = OverlapEngine(0)
    rows, _ = gpu_rows(e, ds, meta["l"])
    e.close()
    g = UnitigGraph(rows, ds.packed()[1], meta["l"])
    assert (g.nodes, g.edges) == (meta["unitig"]["nodes"], meta["unitig"]["edges"])
    g.save_lists(str(tmp_path / "lists"))
    with gzip.open(os.path.join(GOLDEN, meta["unitig"]["lists_file"]), "rt") as f:
        assert (tmp_path / "lists").read_text() == f.read()
    g.sort_edges()
    g.save_unitig(str(tmp_path / "u"))
    with gzip.open(os.path.join(GOLDEN, meta["unitig"]["file"]), "rt") as f:
        assert (tmp_path / "u").read_text() == f.read()


@pytest.mark.parametrize("name", FIXTURES)
def test_ingest_files_matches_host_dataset(name):
    """FASTA/FASTQ file -> parallel record splitter -> device ingest gives the
    reference's Dataset (IDs, strings, frequencies) and then the golden rows."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    e = OverlapEngine(0)
    e.set_shard(0, 1)
    info = e.ingest_files([fixture_input(name)], meta["l"])
    assert info["n_unique"] == ds.num_unique == meta["n_unique"]
    assert_same_dataset(e, ds)
    e.build_index(meta["l"], 0)
    sup = e.mark_contained()
    rows = e.rows(e.find_overlaps())
    e.close()
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]


def test_ingest_files_parse_cases(tmp_path):
    """The record-splitting quirks (tests/golden/parse_cases.json) through the
    device ingest: same Dataset as the reference's."""
    import json
    import os

    from conftest import GOLDEN

    with open(os.path.join(GOLDEN, "parse_cases.json")) as f:
        cases = json.load(f)
    e = OverlapEngine(0)
    e.set_shard(0, 1)
    for case in cases:
        p = tmp_path / (case["name"] + case["ext"])
        p.write_bytes(case["input"].encode())
        info = e.ingest_files([str(p)], case["l"])
        assert info["n_unique"] == case["n_unique"], case["name"]
        assert e.dataset_counts() == (case["n_reads"], case["n_unique"]), case["name"]
        ds = Dataset.from_files([str(p)], case["l"])
        assert_same_dataset(e, ds)
    e.close()


MIXED_LENGTH = ["mixed", "dirty", "branchy", "longreads"]  # fixtures where markContainedReads runs


@pytest.mark.parametrize("name", MIXED_LENGTH + ["prefixes"])
def test_prefix_contain_off(name):
    """option prefix_contain = 0: the containment probe verifies suffix-key
    hits too (at offset s = 0 only) instead of running k_prefix_contain; the
    same superReadID and rows."""
    if name == "prefixes":
        seqs, l = prefix_reads(), 40
        ds = Dataset.from_strings(seqs, l)
        orows, osup, _, _ = OracleDataset.from_strings(seqs, l).overlaps(l)
        want_rows, want_sup = sorted_tuples(orows), {str(i): int(x) for i, x in enumerate(osup) if x}
    else:
        meta = load_meta(name)
        l = meta["l"]
        ds = Dataset.from_files([fixture_input(name)], l)
        want_rows, want_sup = golden_rows(name), meta["super"]
    e = OverlapEngine(0)
    e.set_option("prefix_contain", 0)
    rows, sup = gpu_rows(e, ds, l)
    e.close()
    assert np.array_equal(rows_to_tuples(rows), want_rows)
    assert {str(i): int(x) for i, x in enumerate(sup) if x} == want_sup


CONTAIN_OPTS = [
    {"contain_jcut": 0, "contain_prune": 0, "contain_skip": 0},
    {"live_index": 0},
    {"contain_jcut": 1, "contain_prune": 0, "contain_skip": 0},
    {"contain_jcut": 0, "contain_prune": 1, "contain_skip": 0},
    {"contain_jcut": 0, "contain_prune": 0, "contain_skip": 1},
    {"contain_skip": 1, "prefix_contain": 0},
    {"probe_share": 0, "probe_compact": 0},
    {"probe_share": 1, "probe_compact": 0},
    {"probe_share": 0, "probe_compact": 1},
    # offset-0 containments by k_prefix_contain's chain walk instead of the window-0 runs
    {"prefix_probe": 0},
    {"prefix_probe": 0, "contain_skip": 0, "contain_prune": 0},
]


@pytest.mark.parametrize("name", ["mixed", "dirty", "branchy", "longreads", "prefixes", "metagenome"])
def test_containment_options(name):
    """The containment cuts are pure pruning: runs past
    j = n1 - minlen (contain_jcut), candidates that cannot raise the superkey
    (contain_prune), runs of already-contained sources (contain_skip, also without
    k_prefix_contain) and source-length passes (contain_passes), the offset-0
    containments by k_prefix_contain instead of the window-0 runs (prefix_probe = 0), and the probe's
    batch compaction and block-shared regions (probe_compact, probe_share), and the
    discovery probe on the full index instead of the uncontained reads' index
    (live_index = 0): every combination gives the same superReadIDs and rows."""
    if name in ("prefixes", "metagenome"):
        if name == "prefixes":
            seqs, l = prefix_reads(), 40
        else:
            c, L = synth.metagenome_read_set(20000, 100, 250, n_genomes=20, total_len=400000, seed=51)
            seqs, l = synth.codes_to_strings(c, L), 50
        ds = Dataset.from_strings(seqs, l)
        orows, osup, _, _ = OracleDataset.from_strings(seqs, l).overlaps(l)
        want_rows, want_sup = sorted_tuples(orows), {str(i): int(x) for i, x in enumerate(osup) if x}
    else:
        meta = load_meta(name)
        l = meta["l"]
        ds = Dataset.from_files([fixture_input(name)], l)
        want_rows, want_sup = golden_rows(name), meta["super"]
    assert want_sup
    for opts in CONTAIN_OPTS:
        e = OverlapEngine(0)
        for k, v in opts.items():
            e.set_option(k, v)
        rows, sup = gpu_rows(e, ds, l)
        e.close()
        assert {str(i): int(x) for i, x in enumerate(sup) if x} == want_sup, opts
        assert np.array_equal(rows_to_tuples(rows), want_rows), opts


@pytest.mark.parametrize("name", ["mixed", "dirty", "branchy", "prefixes", "metagenome"])
def test_live_index_forced(name):
    """The discovery index of the uncontained reads (option live_index) against
    the goldens with the live table really in use: a large directory (nb_log2 =
    16) makes the live reads' table smaller than the full one even on the small
    fixtures, and counters().live_cells proves the probe walked it (on the
    default directory of a small set both tables get 2^10 cells, the live build
    is skipped, and a live_index on/off comparison would be vacuous)."""
    if name in ("prefixes", "metagenome"):
        if name == "prefixes":
            seqs, l = prefix_reads(), 40
        else:
            c, L = synth.metagenome_read_set(20000, 100, 250, n_genomes=20, total_len=400000, seed=51)
            seqs, l = synth.codes_to_strings(c, L), 50
        ds = Dataset.from_strings(seqs, l)
        orows, osup, _, _ = OracleDataset.from_strings(seqs, l).overlaps(l)
        want_rows, want_sup = sorted_tuples(orows), {str(i): int(x) for i, x in enumerate(osup) if x}
    else:
        meta = load_meta(name)
        l = meta["l"]
        ds = Dataset.from_files([fixture_input(name)], l)
        want_rows, want_sup = golden_rows(name), meta["super"]
    assert want_sup
    for live in (1, 0):
        e = OverlapEngine(0)
        e.set_option("live_index", live)
        e.set_option("stats", 1)
        rows, sup = gpu_rows(e, ds, l, nb_log2=16)
        cells = e.counters()["live_cells"]
        e.close()
        assert (cells > 0) == bool(live) and cells < (1 << 16), (live, cells)
        assert {str(i): int(x) for i, x in enumerate(sup) if x} == want_sup, live
        assert np.array_equal(rows_to_tuples(rows), want_rows), live


@pytest.mark.parametrize("name", ["small", "tandem", "highdup", "mixed", "branchy"])
def test_fused_run_region_overflow(name):
    """The fused scan's run regions start far too small (option run_cap = 8):
    equal lengths send the discovery probe out before the run counts are read
    (probe_shared), so the cut regions are found with the row counts and scan
    + probe rerun; mixed lengths settle the regions before the containment
    probe.  Rows and superReadIDs equal the goldens on both steps of an engine
    (the second step starts from the grown capacity)."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    e = OverlapEngine(0)
    try:
        e.set_option("run_cap", 8)
        for _ in range(2):
            rows, sup = gpu_rows(e, ds, meta["l"])
            assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
            assert {str(i): int(x) for i, x in enumerate(sup) if x} == meta["super"]
        t = e.timings()
        assert t["index_ms"] > 0 and t["probe_ms"] > 0
    finally:
        e.close()


@pytest.mark.parametrize("name", ["small", "mixed", "tandem", "highdup", "tworead"])
def test_replicated_index_source_shards(name):
    """Multi-GPU replicated mode (bench --multi replicated): every rank builds
    the whole index and discovers only from its source-read range; each rank
    holds its discoveries' rows and twins (DESIGN.md §4 halving: every pair is
    discovered from one side only), and the union over ranks is the reference
    multiset."""
    from metagenomics_amd.sharded import source_range

    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    P = 3
    parts = []
    for r in range(P):
        lo, hi = source_range(ds.num_unique, r, P)
        if hi == lo:  # an empty range (read_hi = 0 would mean "all")
            continue
        e = OverlapEngine(0)
        rows, sup = gpu_rows(e, ds, meta["l"], shard=(0, 1, lo, hi))
        e.close()
        assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]
        assert_shard_rows(rows, lo, hi)
        parts.append(rows)
    allrows = np.concatenate(parts) if parts else parts
    assert np.array_equal(rows_to_tuples(allrows), golden_rows(name))


@pytest.mark.parametrize("l,k", [(33, 1), (50, 17), (20, 19), (50, 31), (60, 32)])
def test_register_scan_window_extremes(engine, l, k):
    """w = l - k = 32 (the register scan's largest window), 33 (the exchange
    mode's key records then come from the LDS scan), 1 and typical ones, against
    the oracle on mixed lengths (containment, all four keys, runs crossing block
    edges): the fused path (k_scan<INDEX>), a source-range shard (run-only
    scans) and the exchange mode at P = 2 (key records)."""
    c, L = synth.uniform_read_set(3000, 0, 15000, seed=120 + k, lo=l + 1, hi=l + 90)
    seqs = synth.codes_to_strings(c, L)
    ds = Dataset.from_codes(c, L, l)
    od = OracleDataset.from_strings(seqs, l)
    orows, osup, _, _ = od.overlaps(l)
    rows, sup = gpu_rows(engine, ds, l, k=k)
    assert np.array_equal(sup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))
    n = ds.num_unique
    a, _ = gpu_rows(engine, ds, l, k=k, shard=(0, 1, 0, n // 2))
    b, _ = gpu_rows(engine, ds, l, k=k, shard=(0, 1, n // 2, n))
    assert np.array_equal(rows_to_tuples(np.concatenate([a, b])), sorted_tuples(orows))
    xrows, xsup = exchange_rows(ds, l, 2, k=k)
    assert np.array_equal(xsup.astype(np.uint64), osup)
    assert np.array_equal(rows_to_tuples(xrows), sorted_tuples(orows))


@pytest.mark.parametrize("name", ["mixed", "tandem", "longreads"])
def test_id_order_layout(name):
    """option layout = 0 (slots in ID order) beside the default (clustered
    slots): same rows, superReadIDs, getListOfReads lists and downloaded reads."""
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    e = OverlapEngine(0)
    e.set_option("layout", 0)
    rows, sup = gpu_rows(e, ds, meta["l"])
    assert np.array_equal(rows_to_tuples(rows), golden_rows(name))
    assert {str(i): int(s) for i, s in enumerate(sup) if s} == meta["super"]
    for key, exp in meta.get("lookups", {}).items():
        assert [list(x) for x in e.lookup(key)] == exp, key
    w, lens = e.download_packed()
    hw, hl = ds.packed()
    assert np.array_equal(lens, hl) and np.array_equal(w[:, :hw.shape[1]], hw)
    e.close()


def test_layout_clusters_overlapping_reads(engine):
    """The default layout is a permutation of the reads (digest-equal rows on a
    random set vs the oracle) that puts overlap partners near each other: most
    discoveries of a 20x random set have their partner within 64 slots."""
    c, L = synth.uniform_read_set(20000, 150, 150000, seed=5)
    ds = Dataset.from_codes(c, L, 50)
    od = OracleDataset.from_strings(synth.codes_to_strings(c, L), 50)
    orows, osup, _, _ = od.overlaps(50)
    rows, sup = gpu_rows(engine, ds, 50, k=31)
    assert np.array_equal(rows_to_tuples(rows), sorted_tuples(orows))
    slot = engine.slot_of_ids()
    d = np.abs(slot[rows["src"].astype(np.int64) - 1] - slot[rows["dst"].astype(np.int64) - 1])
    assert (d <= 64).mean() > 0.3, (d <= 64).mean()


@pytest.mark.parametrize("name", ["small", "tandem", "branchy", "longreads"])
def test_explore_through_per_read_methods(tmp_path, name):
    """The reference's exploration loop (OverlapGraph.cpp:144-204) driven by a
    C++ caller through the drop-in's per-read methods (mg_explore:
    beginBuildFromHashTable, insertAllEdgesOfRead, markTransitiveEdges,
    removeTransitiveEdges; OverlapGraph.h:54,64-68): graph[u] lists in list
    order and the counters equal the reference's graph before its contraction
    loop (bfs golden), and after the loop the .unitig equals the reference's;
    checkOverlap / checkOverlapForContainedRead agree with the device."""
    import gzip
    import json
    import os
    import subprocess

    from conftest import GOLDEN, ROOT

    meta = load_meta(name)
    exe = os.path.join(ROOT, "metagenomics_amd", "lib", "mg_explore")
    prefix = str(tmp_path / name)
    out = subprocess.run([exe, fixture_input(name), str(meta["l"]), prefix], check=True, capture_output=True,
                         text=True, timeout=300)
    info = json.loads(out.stdout.strip().split("\n")[-1])
    assert info["check_failures"] == 0
    assert info["iterations"] == meta["unitig"]["iterations"]
    lines = open(prefix + ".graph").read().split("\n")
    _, nodes, edges = lines[0].split()
    assert (int(nodes), int(edges)) == (meta["bfs"]["nodes"], meta["bfs"]["edges"])
    with gzip.open(os.path.join(GOLDEN, meta["bfs"]["file"]), "rt") as f:
        assert [x for x in lines[1:] if x] == [x for x in f.read().split("\n") if x]
    with gzip.open(os.path.join(GOLDEN, meta["unitig"]["file"]), "rt") as f:
        assert open(prefix + ".unitig").read() == f.read()


@pytest.mark.parametrize("name,cap", [("small", 1 << 16), ("mixed", 1 << 20)])
def test_allocation_failure_names_its_cause(name, cap):
    """A failed device allocation surfaces with the buffer's name, the bytes asked
    for and the HIP error (option alloc_cap forces one), not as a generic
    "launch failed"; the context then works again once the cap is lifted."""
    from metagenomics_amd.overlap import MgError

    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    e = OverlapEngine(0)
    try:
        e.upload(ds)
        e.set_option("alloc_cap", cap)
        with pytest.raises(MgError) as exc:
            e.build_index(meta["l"])
            e.mark_contained()
            e.find_overlaps()
        msg = str(exc.value)
        assert "device allocation of " in msg and " B) failed: " in msg and "alloc_cap" in msg, msg
        assert "memory" in msg.lower(), msg
        e.set_option("alloc_cap", 0)
        e.build_index(meta["l"])
        e.mark_contained()
        t = rows_to_tuples(e.rows(e.find_overlaps()))
        assert np.array_equal(t, golden_rows(name))
    finally:
        e.close()
