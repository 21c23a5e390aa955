"""Parity at the bench's full sizes through order-independent digests.

tests/golden/{c2,c3,c5s}.json hold the digests (oracle/mg_digest.h) of the
REFERENCE's own edge multiset and superReadID vector on the bench's exact
workloads (tests/golden/make_scale_golden.py runs oracle/_ref/ref_harness
digest on them in the build container).  tests/golden/c5.json (BASELINE
configs[4], 50M reads: beyond the reference's reach in this container) is the
oracle's (mgo_overlaps_digest over source-read ranges), which
tests/golden/c5s_oracle_check.json shows reproducing the reference's own c5s
digests.  The device computes the same digests
(mg_rows_digest / mg_super_digest) without downloading 10^8 rows.  Three
independent implementations of the digest (C in the harness and the oracle,
numpy in tests/digest.py, HIP in the product) are checked against each other.
"""
import json
import os

import numpy as np
import pytest

import digest
from conftest import FIXTURES, GOLDEN, ROOT, fixture_input, golden_rows, load_meta
from metagenomics_amd import synth
from oracle import OracleDataset, rows_digest as oracle_rows_digest, super_digest as oracle_super_digest

SCALE = {name: os.path.join(GOLDEN, name + ".json") for name in ("c2", "c3", "c5s", "c5")}


def super_array(meta, n):
    s = np.zeros(n + 1, dtype=np.uint64)
    for k, v in meta["super"].items():
        s[int(k)] = v
    return s


# ------------------------------------------------------------------ CPU ----
@pytest.mark.parametrize("name", FIXTURES)
def test_numpy_digest_equals_c_digest(name):
    """tests/digest.py == oracle/mg_digest.h (C) on every golden multiset."""
    g = golden_rows(name)
    rows = np.zeros(g.shape[0], dtype=[("src", "<u4"), ("dst", "<u4"), ("offset", "<u2"), ("orient", "u1"),
                                       ("pad", "u1")])
    rows["src"], rows["dst"], rows["orient"], rows["offset"] = g[:, 0], g[:, 1], g[:, 2], g[:, 3]
    assert digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3]) == oracle_rows_digest(rows)
    meta = load_meta(name)
    sup = super_array(meta, meta["n_unique"])
    assert digest.super_digest(sup) == oracle_super_digest(sup)


def test_digest_is_order_independent_and_multiplicity_sensitive():
    rng = np.random.default_rng(3)
    u, v = rng.integers(1, 10**6, 1000), rng.integers(1, 10**6, 1000)
    o, f = rng.integers(0, 4, 1000), rng.integers(0, 65536, 1000)
    d = digest.rows_digest(u, v, o, f)
    p = rng.permutation(1000)
    assert digest.rows_digest(u[p], v[p], o[p], f[p]) == d
    d2 = digest.rows_digest(np.r_[u, u[:1]], np.r_[v, v[:1]], np.r_[o, o[:1]], np.r_[f, f[:1]])
    assert d2["n"] == 1001 and d2["sum"] != d["sum"]


@pytest.mark.parametrize("name", ["small", "mixed", "tandem"])
def test_oracle_digest_matches_reference_harness_recipe(name):
    """The oracle restatement's multiset digest on a fixture equals the digest
    of the reference's golden rows (the recipe the scale goldens use)."""
    meta = load_meta(name)
    od = OracleDataset.from_files([fixture_input(name)], meta["l"])
    orows, osup, _, _ = od.overlaps(meta["l"])
    g = golden_rows(name)
    assert oracle_rows_digest(orows) == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert oracle_super_digest(osup) == digest.super_digest(super_array(meta, meta["n_unique"]))


@pytest.mark.parametrize("name", sorted(SCALE))
def test_scale_goldens_are_well_formed(name):
    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    m = json.load(open(SCALE[name]))
    assert m["rows"]["n"] % 2 == 0 and m["rows"]["n"] > 0
    assert m["n_unique"] <= m["n_reads"] <= m["workload"]["reads"]
    if m["workload"]["read_len"][0] == m["workload"]["read_len"][1]:
        assert m["super"]["n"] == 0  # markContainedReads skipped (OverlapGraph.cpp:228-233)


# ------------------------------------------------------------------ GPU ----
def _engine_rows(e, ds, l, k=0):
    e.set_shard(0, 1)
    e.upload(ds)
    e.build_index(l, k)
    e.mark_contained(copy=False)
    return e.find_overlaps()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small", "mixed", "tandem", "branchy"])
def test_device_digest_matches_golden(name):
    """mg_rows_digest / mg_super_digest on the device == numpy digest of the golden rows."""
    from metagenomics_amd.overlap import Dataset, OverlapEngine

    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    e = OverlapEngine(0)
    try:
        _engine_rows(e, ds, meta["l"])
        g = golden_rows(name)
        assert e.rows_digest() == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
        assert e.super_digest() == digest.super_digest(super_array(meta, meta["n_unique"]))
        rows = e.rows()
        # the flat-buffer form over a device copy of the same rows
        import torch

        t = torch.from_numpy(rows.view(np.uint8).copy()).to("cuda:0")
        assert e.rows_digest(t.data_ptr(), rows.shape[0]) == e.rows_digest()
    finally:
        e.close()


def scale_dataset(name):
    from metagenomics_amd.overlap import Dataset

    sys_path_golden = os.path.join(GOLDEN)
    import sys

    sys.path.insert(0, sys_path_golden)
    import make_scale_golden

    m = json.load(open(SCALE[name]))
    codes, lens = make_scale_golden.make_codes(name)
    ds = Dataset.from_codes(codes, lens, m["workload"]["min_overlap"], nthreads=16)
    return m, ds


def test_c5_oracle_recipe_pinned_on_c5s():
    """The threaded oracle recipe behind c5.json reproduced the reference's own
    c5s digests (rows and superReadIDs) in the build container."""
    chk = json.load(open(os.path.join(GOLDEN, "c5s_oracle_check.json")))
    ref = json.load(open(SCALE["c5s"]))
    assert chk["check"] is True
    for k in ("n_unique", "n_reads", "rows", "super"):
        assert chk["oracle"][k] == ref[k], k
    c5 = json.load(open(SCALE["c5"]))
    assert c5["recipe"] == chk["oracle"]["recipe"].replace(str(chk["oracle"]["threads"]) + " threads",
                                                          str(c5["threads"]) + " threads")
    assert c5["workload"]["reads"] == 50_000_000 and c5["super"]["n"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["c2", "c3", "c5s", "c5"])
def test_scale_digest_matches_reference(name):
    """The bench's exact workloads (C2, C3 = the headline metric's config, and a
    C5-shaped metagenome with containment): the device's edge multiset and
    superReadID vector have the reference's digests (OverlapGraph.cpp:225-340,
    529-565; HashTable.cpp:50-80)."""
    from metagenomics_amd.overlap import OverlapEngine

    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    m, ds = scale_dataset(name)
    assert (ds.num_unique, ds.num_reads) == (m["n_unique"], m["n_reads"])
    e = OverlapEngine(0)
    try:
        n = _engine_rows(e, ds, m["workload"]["min_overlap"], 31)
        assert n == m["rows"]["n"]
        assert e.rows_digest() == m["rows"]
        assert e.super_digest() == m["super"]
    finally:
        e.close()


def combine(ds):
    out = {"n": 0, "sum": 0, "xor": 0, "sum2": 0}
    for d in ds:
        out = {"n": out["n"] + d["n"], "sum": (out["sum"] + d["sum"]) % 2**64, "xor": out["xor"] ^ d["xor"],
               "sum2": (out["sum2"] + d["sum2"]) % 2**64}
    return out


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,world,route", [("c3", 8, False), ("c5s", 8, True), ("c5", 8, False)])
def test_exchange_scale_digest(name, world, route):
    """The multi-GPU exchange mode (bucket-range index shards,
    key / run / row all-to-alls, MAX all-reduce of the containment keys) with
    `world` simulated ranks on this GPU (LocalExchange moves the slot buffers):
    C4's data path on the C3 workload, containment through the exchange on the
    C5-shaped set, and BASELINE configs[4] itself (50M mixed reads, 8 ranks:
    the 8 contexts share the one 288 GB device, so each frees its layout's
    double buffers); the union of the ranks' rows has the reference's digest
    (c5: the pinned oracle's, tests/golden/c5s_oracle_check.json).  route: the
    rows also move to their src owners (c5s); else each rank keeps the rows it
    verified (the default)."""
    import torch

    from metagenomics_amd.overlap import OverlapEngine
    from metagenomics_amd.sharded import LocalExchange, sharded_step, source_range

    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    m, ds = scale_dataset(name)
    engines = []
    try:
        for r in range(world):
            e = OverlapEngine(0)
            e.set_option("layout_scratch", 0)
            e.set_shard(r, world, 0, 0)
            e.upload(ds)
            engines.append(e)
        del ds  # (the host Dataset: 50M reads at c5)
        res = sharded_step(engines, LocalExchange(world, torch.device("cuda:0")), m["workload"]["min_overlap"], 31,
                           route_rows=route)
        assert res.rows_routed == route
        if route:
            rd = combine([e.slots_digest(b.data_ptr(), slot, rounds, c.data_ptr())
                          for e, (b, c, slot, rounds) in zip(engines, res.rows)])
        else:
            rd = combine([e.rows_digest() for e in engines])
        assert rd == m["rows"]
        assert engines[0].super_digest() == m["super"]
        # each rank holds rows (with route: those of the sources it owns, by reference ID)
        for r in range(world):
            assert res.n_rows[r] > 0
            lo, hi = source_range(m["n_unique"], r, world)
            assert lo < hi
    finally:
        for e in engines:
            e.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,world", [("c3", 8), ("c2", 3)])
def test_bucket_scale_digest(name, world):
    """The bucket mode (bench --multi bucket, SURVEY §8(e) alternative (i)):
    `world` bucket-range shards over every source, each context's one scan of
    every read filing and keeping only its buckets' keys and runs, then its probe;
    no data-path collective.  The union of the ranks' rows has the reference's
    digest."""
    from metagenomics_amd.overlap import OverlapEngine

    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    m, ds = scale_dataset(name)
    engines = []
    try:
        digests = []
        for r in range(world):
            e = OverlapEngine(0)
            e.set_option("layout_scratch", 0)
            e.set_shard(r, world, 0, 0)
            e.upload(ds)
            engines.append(e)
            e.build_index(m["workload"]["min_overlap"], 31)
            e.mark_contained(copy=False)
            assert e.find_overlaps() > 0
            digests.append(e.rows_digest())
        assert combine(digests) == m["rows"]
    finally:
        for e in engines:
            e.close()


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,launcher", [("c3", "direct"), ("c5s", "torchrun")])
def test_cli_exchange_over_rccl(name, launcher, tmp_path):
    """The C++ host's exchange mode (mg_overlap -xchg, metagenomics_amd/csrc/host/
    mg_xchg.cpp: collectives issued by C++ over RCCL on the library's stream) at
    world 1 on the workload's FASTA: the reference's row and superReadID digests.
    c5s goes through torchrun --no-python, the launcher of the N-GPU runs."""
    import subprocess
    import sys

    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    m = json.load(open(SCALE[name]))
    fa = str(tmp_path / f"{name}.fa")
    subprocess.run([sys.executable, os.path.join(GOLDEN, "make_scale_golden.py"), "--fasta", name, fa],
                   check=True, timeout=600)
    cli = os.path.join(ROOT, "metagenomics_amd", "lib", "mg_overlap")
    args = [cli, "-se", "1", fa, "-f", str(tmp_path / "x"), "-l", str(m["workload"]["min_overlap"]), "-k", "31",
            "-xchg", "3"]
    if launcher == "torchrun":
        args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                "--master-addr", "127.0.0.1", "--master-port", "29731", "--no-python"] + args
    out = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert r["world"] == 1 and r["unique_reads"] == m["n_unique"]
    assert r["rows"] == m["rows"]
    assert r["super"] == m["super"]
    assert r["contained"] == (m["super"]["n"] > 0)


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["c2", "c5s"])
def test_exchange_two_processes(name):
    """The exchange mode as the N-GPU bench runs it -- one process per rank under
    torchrun, bench.py's TorchExchange, each rank's own context -- with two ranks
    on this one GPU.  RCCL refuses two ranks on one device, so the process group
    is gloo and the all-to-alls stage the device buffers through host copies;
    everything else (routing kernels, slot layout, counts, capacity reruns, MAX
    all-reduce of the containment keys, rows digest over ranks) is the N-GPU
    path.  The union of the two ranks' rows has the reference's digest."""
    import subprocess
    import sys

    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    env = dict(os.environ, MG_BENCH_PG_BACKEND="gloo")
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", "29733", os.path.join(ROOT, "bench.py"),
            "--gpus", "2", "--config", name, "--multi", "exchange", "--steps", "1", "--warmup", "1",
            "--no-cpu-baseline", "--no-ingest"]
    out = subprocess.run(args, capture_output=True, text=True, timeout=800, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"].startswith("2 ranks")
    assert r["parity"]["golden"] and r["parity"]["digest_ok"] is True, r["parity"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,mode", [("c2", "bucket-range index"), ("c5s", "bucket-range index")])
def test_two_processes_default_mode(name, mode):
    """bench.py --gpus N with no --multi (auto, DESIGN.md §6c: the bucket mode for
    one read length on 2 ranks (c2), the exchange mode for mixed lengths (c5s);
    both bucket-range index shards) as the driver's N-GPU runs launch it: two
    torchrun processes, each rank's own context; gloo stages the all-to-alls
    (two ranks share this one GPU).  The rows and superReadIDs over both ranks
    have the reference's digests."""
    import subprocess
    import sys

    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    env = dict(os.environ, MG_BENCH_PG_BACKEND="gloo")
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", "29735", os.path.join(ROOT, "bench.py"),
            "--gpus", "2", "--config", name, "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-ingest"]
    out = subprocess.run(args, capture_output=True, text=True, timeout=800, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert r["n_gpus"] == 2 and mode in r["config"]["parallelism"]
    assert r["parity"]["golden"] and r["parity"]["digest_ok"] is True, r["parity"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode,desc", [("replicated", "whole index on every rank"),
                                       ("bucket", "every rank scans every read")])
def test_two_processes_no_collective_modes(mode, desc):
    """bench.py --gpus 2 --multi replicated / bucket (SURVEY §8(e) alternatives
    (ii) / (i)): the whole index on every rank with
    source-read shards, or bucket-range shards scanning every read; no data-path
    collective; the union has the reference's C2 digest."""
    import subprocess
    import sys

    if not os.path.exists(SCALE["c2"]):
        pytest.skip("c2.json not generated")
    env = dict(os.environ, MG_BENCH_PG_BACKEND="gloo")
    args = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1", "--master-port", "29737", os.path.join(ROOT, "bench.py"),
            "--gpus", "2", "--config", "c2", "--multi", mode, "--steps", "1", "--warmup", "1",
            "--no-cpu-baseline", "--no-ingest"]
    out = subprocess.run(args, capture_output=True, text=True, timeout=800, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert r["n_gpus"] == 2 and desc in r["config"]["parallelism"]
    assert r["parity"]["golden"] and r["parity"]["digest_ok"] is True, r["parity"]
