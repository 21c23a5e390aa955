"""the host replay of the reference's exploration order and
transitive reduction (mgh_graph_replay, metagenomics_amd/csrc/host/mg_graph.cpp)
reproduces the reference's graph before contraction: every graph[u] list in
LIST ORDER plus numberOfNodes / numberOfEdges (golden: oracle/_ref/ref_harness
bfs, i.e. the reference's own insertAllEdgesOfRead / markTransitiveEdges /
removeTransitiveEdges).  Input: the discovery multiset (the golden rows the GPU
path is pinned to), so this runs on CPU."""
import gzip
import os

import numpy as np
import pytest

from conftest import FIXTURES, GOLDEN, golden_rows, load_meta, fixture_input, rows_sha256
from metagenomics_amd.overlap import EDGE_DTYPE, Dataset, replay_graph
from oracle import OracleDataset


def to_edges(t: np.ndarray) -> np.ndarray:
    r = np.zeros(t.shape[0], dtype=EDGE_DTYPE)
    r["src"], r["dst"], r["orient"], r["offset"] = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    return r


def tuples(rows: np.ndarray) -> np.ndarray:
    return np.stack([rows["src"], rows["dst"], rows["orient"], rows["offset"]], axis=1).astype(np.int64)


def golden_bfs(name):
    meta = load_meta(name)
    with gzip.open(os.path.join(GOLDEN, meta["bfs"]["file"]), "rt") as f:
        txt = f.read().split()
    return np.array(txt, dtype=np.int64).reshape(-1, 4) if txt else np.zeros((0, 4), np.int64)


@pytest.mark.parametrize("name", FIXTURES)
def test_replay_matches_reference_graph(name):
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows = to_edges(golden_rows(name))
    rng = np.random.default_rng(0)
    rows = rows[rng.permutation(rows.shape[0])]  # the device emits rows in any order
    nodes, edges, out = replay_graph(rows, ds.packed()[1], meta["l"])
    assert (nodes, edges) == (meta["bfs"]["nodes"], meta["bfs"]["edges"])
    assert np.array_equal(tuples(out), golden_bfs(name))


def test_replay_c1_digest():
    """BASELINE configs[0] (100k x 100 bp, l=40): oracle multiset -> replay."""
    from metagenomics_amd import synth

    meta = load_meta("c1")
    r = meta["recipe"]
    c, L = synth.uniform_read_set(r["n_reads"], r["read_len"], r["genome_len"], r["seed"])
    od = OracleDataset.from_strings(synth.codes_to_strings(c, L), meta["l"])
    orows, _, _, _ = od.overlaps(meta["l"])
    rows = np.zeros(orows.shape[0], dtype=EDGE_DTYPE)
    for k in ("src", "dst", "orient", "offset"):
        rows[k] = orows[k]
    lens = np.full(od.num_unique, r["read_len"], dtype=np.uint16)
    nodes, edges, out = replay_graph(rows, lens, meta["l"])
    assert (nodes, edges) == (meta["bfs"]["nodes"], meta["bfs"]["edges"])
    assert rows_sha256(tuples(out)) == meta["bfs"]["rows_sha256"]


def test_replay_rejects_inconsistent_rows():
    rows = np.zeros(1, dtype=EDGE_DTYPE)
    rows["src"], rows["dst"], rows["orient"], rows["offset"] = 1, 2, 3, 90  # j = 90 >= n - h
    with pytest.raises(Exception):
        replay_graph(rows, np.array([100, 100], np.uint16), 40)
