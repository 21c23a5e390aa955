"""The C++ exchange host (metagenomics_amd/csrc/host/mg_xchg.cpp, the binary
INTEGRATION.md hands to the N-GPU run: mg_overlap -xchg) at P > 1.

`-xchg-sim P` runs P ranks as threads of one process on one GPU, each with its
own mg_ctx and HIP stream; LocalTransport moves the slot-layout buffers between
the contexts by device copies and does the MAX all-reduce with a device kernel.
Everything else -- XchgStep::run, its slot geometry, the per-peer routing of
keys / runs / rows (mg_xchg_pack with self_dst), the counts all-to-all, the
capacity check and the rerun after a cut stream -- is the code the RCCL ranks
run (RcclExchange implements the same Transport interface).

Parity: the union of the ranks' rows has the digest of the reference's golden
multiset (OverlapGraph.cpp:225-290, 529-565; HashTable.cpp:50-80), and rank 0's
superReadIDs the golden's (tests/golden/*.json; c3/c5s: the reference's own
digests of the bench workloads)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import digest
from conftest import FIXTURES, GOLDEN, ROOT, fixture_input, golden_rows, load_meta

CLI = os.path.join(ROOT, "metagenomics_amd", "lib", "mg_overlap")


def golden_super_digest(meta):
    s = np.zeros(meta["n_unique"] + 1, dtype=np.uint64)
    for k, v in meta["super"].items():
        s[int(k)] = v
    return digest.super_digest(s)


def run_cli(inp, l, world, steps=1, k=None, caps=None, timeout=600, env=None):
    args = [CLI, "-se", "1", inp, "-f", "/tmp/mg_xchg_host_unused", "-l", str(l), "-xchg", str(steps),
            "-xchg-sim", str(world)]
    if k is not None:
        args += ["-k", str(k)]
    if caps is not None:
        args += ["-xchg-caps", str(caps)]
    out = subprocess.run(["timeout", "-k", "10", str(timeout)] + args, capture_output=True, text=True,
                         timeout=timeout + 30, env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


# ------------------------------------------------------------------ CPU ----
def test_cli_sim_without_device_fails_cleanly(tmp_path):
    """No HIP device: every rank thread fails at its context (no CPU fallback),
    the process exits 2 with the reason, and no rank waits at a barrier."""
    if os.environ.get("HIP_VISIBLE_DEVICES") is None:
        from conftest import gpu_available

        if gpu_available():
            pytest.skip("a HIP device is present")
    out = subprocess.run(["timeout", "-k", "5", "60", CLI, "-se", "1", fixture_input("small"), "-f",
                          str(tmp_path / "x"), "-l", "40", "-xchg", "1", "-xchg-sim", "3"],
                         capture_output=True, text=True, timeout=90)
    assert out.returncode == 2, (out.returncode, out.stderr[-2000:])
    assert "rank" in out.stderr


def test_cli_rejects_bad_sim_world(tmp_path):
    for bad in (["-xchg-sim", "17"], ["-xchg-sim", "-1"], ["-xchg-caps", "0"]):
        out = subprocess.run([CLI, "-se", "1", fixture_input("small"), "-f", str(tmp_path / "x"), "-l", "40",
                              "-xchg", "1"] + bad, capture_output=True, text=True, timeout=60)
        assert out.returncode == 1 and "Usage" in out.stderr


# ------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_xchg_host_fixtures_p3(name):
    """Every golden fixture through the C++ host at P = 3 (longreads: reads over
    1,024 bp take the replicated fallback, as sharded.py's does)."""
    meta = load_meta(name)
    r = run_cli(fixture_input(name), meta["l"], 3)
    g = golden_rows(name)
    assert r["world"] == 3 and r["unique_reads"] == meta["n_unique"]
    assert r["mode"] == ("replicated" if name == "longreads" else "xchg")
    assert r["rows"] == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert r["super"] == golden_super_digest(meta)
    assert sum(r["rows_held"]) == g.shape[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("mixed", 2), ("mixed", 8), ("tandem", 5), ("highdup", 8), ("small", 16),
                                        ("tworead", 4)])
def test_xchg_host_worlds(name, world):
    """Other world sizes, up to 16 ranks (tworead: more ranks than source reads)."""
    meta = load_meta(name)
    r = run_cli(fixture_input(name), meta["l"], world, steps=2)
    g = golden_rows(name)
    assert r["world"] == world
    assert r["rows"] == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert r["super"] == golden_super_digest(meta)


@pytest.mark.gpu
@pytest.mark.parametrize("name,world,caps", [("mixed", 3, 0.02), ("highdup", 4, 0.05), ("small", 2, 0.001)])
def test_xchg_host_capacity_rerun(name, world, caps):
    """First capacities scaled far down: the streams are cut, XchgStep sees the
    MAX over ranks of the send counts above its capacities, grows them and
    reruns the step (mg_xchg.cpp run()); the result is unchanged."""
    meta = load_meta(name)
    r = run_cli(fixture_input(name), meta["l"], world, steps=1, caps=caps)
    g = golden_rows(name)
    assert r["reruns"] >= 1
    assert r["rows"] == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert r["super"] == golden_super_digest(meta)


SCALE = {name: os.path.join(GOLDEN, name + ".json") for name in ("c2", "c3", "c5s")}


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,world,caps", [("c3", 8, None), ("c5s", 8, None), ("c5s", 3, 0.5)])
def test_xchg_host_scale_digest(name, world, caps, tmp_path):
    """The bench workloads through the C++ host at P = 8 (C4's data path on the
    C3 workload; containment through the exchange on the C5-shaped set) and one
    cut-stream rerun at scale: the reference's own row and superReadID digests."""
    if not os.path.exists(SCALE[name]):
        pytest.skip(f"{name}.json not generated")
    m = json.load(open(SCALE[name]))
    fa = str(tmp_path / f"{name}.fa")
    subprocess.run([sys.executable, os.path.join(GOLDEN, "make_scale_golden.py"), "--fasta", name, fa],
                   check=True, timeout=600)
    r = run_cli(fa, m["workload"]["min_overlap"], world, steps=1, k=31, caps=caps, timeout=700)
    assert r["world"] == world and r["unique_reads"] == m["n_unique"]
    assert r["rows"] == m["rows"]
    assert r["super"] == m["super"]
    assert all(h > 0 for h in r["rows_held"])
    if caps is not None:
        assert r["reruns"] >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("mixed", 3), ("dirty", 4), ("branchy", 2)])
def test_xchg_host_prefix_marks(name, world):
    """MG_XCHG_MARKS=1: each rank's offset-0 containments run first and their
    marks are MAX-all-reduced (mg_xchg_prefix_marks, RcclExchange /
    LocalTransport allreduce_max_u8) before the containment probe; same rows and
    superReadIDs as the reference."""
    meta = load_meta(name)
    r = run_cli(fixture_input(name), meta["l"], world, env={"MG_XCHG_MARKS": "1"})
    g = golden_rows(name)
    assert r["rows"] == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert r["super"] == golden_super_digest(meta)


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("mixed", 3), ("highdup", 4), ("tandem", 2)])
def test_xchg_host_route_rows(name, world):
    """MG_XCHG_ROUTE_ROWS=1: after the discovery probe the rows travel to the
    owners of their src IDs (mg_xchg_pack(MG_ROWS) + the slot all-to-all), so
    each rank holds graph[u] of its own source reads; same union as the default
    (rows held where they were verified)."""
    meta = load_meta(name)
    r = run_cli(fixture_input(name), meta["l"], world, env={"MG_XCHG_ROUTE_ROWS": "1"})
    g = golden_rows(name)
    assert r["rows_routed"] is True
    assert r["rows"] == digest.rows_digest(g[:, 0], g[:, 1], g[:, 2], g[:, 3])
    assert r["super"] == golden_super_digest(meta)
    assert sum(r["rows_held"]) == g.shape[0]
