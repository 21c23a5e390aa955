"""unitig contraction + the .unitig checkpoint.

new OverlapGraph(ht) ends with the contraction loop (OverlapGraph.cpp:211-215:
contractCompositePaths :669-696 + removeDeadEndNodes :931-988, with mergeEdges,
mergeList, removeEdge and the read-location bookkeeping :1048-1115), and
main.cpp:48-50 then runs sortEdges + saveGraphToFile.  UnitigGraph
(metagenomics_amd/csrc/host/mg_unitig.cpp, C-ABI mgh_graph_contract /
mgh_graph_save_unitig) replays it on the device's discovery multiset.

Golden: oracle/_ref/ref_harness unitig, i.e. the reference's own
contractCompositePaths / removeDeadEndNodes / sortEdges / saveGraphToFile run
on its own graph (tests/golden/make_golden.py --unitig).  Compared: the
numberOfNodes / numberOfEdges counters, the loop's iteration count, every list
in list order with each edge's read / offset / orientation lists, every read's
location lists, and the .unitig file byte for byte.  Input: the golden
discovery multiset the GPU path is pinned to, so this runs on CPU."""
import gzip
import hashlib
import os

import numpy as np
import pytest

from conftest import FIXTURES, GOLDEN, golden_rows, load_meta, fixture_input
from metagenomics_amd.overlap import EDGE_DTYPE, Dataset, MgError, UnitigGraph


def to_edges(t: np.ndarray) -> np.ndarray:
    r = np.zeros(t.shape[0], dtype=EDGE_DTYPE)
    r["src"], r["dst"], r["orient"], r["offset"] = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    return r


def golden_text(name, key):
    meta = load_meta(name)
    with gzip.open(os.path.join(GOLDEN, meta["unitig"][key]), "rt") as f:
        return f.read()


def build(name, track=True, seed=0):
    meta = load_meta(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    rows = to_edges(golden_rows(name))
    rows = rows[np.random.default_rng(seed).permutation(rows.shape[0])]  # device row order is arbitrary
    return meta, UnitigGraph(rows, ds.packed()[1], meta["l"], track_locations=track)


@pytest.mark.parametrize("name", FIXTURES)
def test_contraction_matches_reference(name, tmp_path):
    meta, g = build(name)
    u = meta["unitig"]
    assert (g.replay_nodes, g.replay_edges) == (meta["bfs"]["nodes"], meta["bfs"]["edges"])
    assert (g.nodes, g.edges, g.iterations) == (u["nodes"], u["edges"], u["iterations"])
    g.save_lists(str(tmp_path / "lists"))
    assert (tmp_path / "lists").read_text() == golden_text(name, "lists_file")
    g.sort_edges()
    g.save_unitig(str(tmp_path / "x.unitig"))
    assert (tmp_path / "x.unitig").read_text() == golden_text(name, "file")


def test_branchy_exercises_the_loop():
    """The stress fixture reaches every branch of the loop: several iterations,
    dead-end removal, composite edges longer than deadEndLength, self-loops."""
    meta, g = build("branchy")
    assert g.iterations >= 4 and g.merged > 0 and g.dead_end_nodes > 0
    e, st, reads, offs, ors = g.unitig_edges()
    assert (e["src"] == e["dst"]).any()
    assert (e["n_reads"] > 10).any()


@pytest.mark.parametrize("name", ["branchy", "tandem"])
def test_location_tracking_does_not_change_the_graph(name, tmp_path):
    _, a = build(name, track=True)
    _, b = build(name, track=False, seed=1)
    for g, p in ((a, "a"), (b, "b")):
        g.sort_edges()
        g.save_unitig(str(tmp_path / p))
    assert (tmp_path / "a").read_text() == (tmp_path / "b").read_text()


def test_unitig_edges_export_matches_lists(tmp_path):
    """mgh_graph_unitig_edges returns the same lists as the text dump."""
    meta, g = build("branchy")
    e, st, reads, offs, ors = g.unitig_edges()
    lines = []
    for k in range(e.shape[0]):
        s = int(st[k])
        n = int(e["n_reads"][k])
        parts = ["%d %d %d %d %d" % (e["src"][k], e["dst"][k], e["orient"][k], e["offset"][k], n)]
        parts += ["%d:%d:%d" % (reads[q], offs[q], ors[q]) for q in range(s, s + n)]
        lines.append(" ".join(parts) + "\n")
    want = [ln for ln in golden_text("branchy", "lists_file").splitlines(True) if ln[0].isdigit()]
    assert lines == want


def test_unitig_record_count():
    """saveGraphToFile writes one record per undirected edge (self-loops once)."""
    for name in FIXTURES:
        meta = load_meta(name)
        txt = golden_text(name, "file").split()
        vals = list(map(int, txt))
        k = recs = 0
        while k < len(vals):
            n = vals[k + 4]
            k += 5 + 3 * n
            recs += 1
        assert recs == meta["unitig"]["unitig_records"]


def test_contract_twice_is_rejected():
    _, g = build("small")
    rc = g._L.mgh_graph_contract(g._g, 1, None, None, None)
    assert rc == -1


def test_c1_digest(tmp_path):
    """BASELINE configs[0] (100k x 100 bp, l = 40): oracle multiset -> replay ->
    contraction -> .unitig, against the reference's digests."""
    from metagenomics_amd import synth
    from oracle import OracleDataset

    meta = load_meta("c1")
    r = meta["recipe"]
    c, L = synth.uniform_read_set(r["n_reads"], r["read_len"], r["genome_len"], r["seed"])
    od = OracleDataset.from_strings(synth.codes_to_strings(c, L), meta["l"])
    orows, _, _, _ = od.overlaps(meta["l"])
    rows = np.zeros(orows.shape[0], dtype=EDGE_DTYPE)
    for k in ("src", "dst", "orient", "offset"):
        rows[k] = orows[k]
    g = UnitigGraph(rows, np.full(od.num_unique, r["read_len"], np.uint16), meta["l"])
    u = meta["unitig"]
    assert (g.nodes, g.edges, g.iterations) == (u["nodes"], u["edges"], u["iterations"])
    g.save_lists(str(tmp_path / "lists"))
    assert hashlib.sha256((tmp_path / "lists").read_bytes()).hexdigest() == u["lists_sha256"]
    g.sort_edges()
    g.save_unitig(str(tmp_path / "x.unitig"))
    assert hashlib.sha256((tmp_path / "x.unitig").read_bytes()).hexdigest() == u["unitig_sha256"]


def reread_golden(name):
    meta = load_meta(name)
    with gzip.open(os.path.join(GOLDEN, meta["reread"]["file"]), "rt") as f:
        return meta, f.read()


@pytest.mark.parametrize("name", FIXTURES)
def test_read_graph_from_file_matches_reference(name, tmp_path):
    """readGraphFromFile (OverlapGraph.cpp:1270-1367): the committed .unitig
    golden read back gives the reference's own lists (list order, composite
    edges' read lists with the reverse edges' rebuilt offsets / orientations),
    read locations and counters (tests/golden/make_reread_golden.py runs the
    reference on the same file); sortEdges + saveGraphToFile then write the
    reference's re-saved file."""
    meta, text = reread_golden(name)
    ds = Dataset.from_files([fixture_input(name)], meta["l"])
    path = tmp_path / "in.unitig"
    path.write_text(golden_text(name, "file"))
    g = UnitigGraph.from_unitig_file(str(path), ds.packed()[1])
    assert (g.nodes, g.edges) == (meta["reread"]["nodes"], meta["reread"]["edges"])
    g.save_lists(str(tmp_path / "lists"))
    assert (tmp_path / "lists").read_text() == text.split("\n", 1)[1]
    g.sort_edges()
    g.save_unitig(str(tmp_path / "out.unitig"))
    want = golden_text(name, "file") if meta["reread"]["resave_identical"] else None
    if want is None:
        with gzip.open(os.path.join(GOLDEN, meta["reread"]["resaved_file"]), "rt") as f:
            want = f.read()
    assert (tmp_path / "out.unitig").read_text() == want
    g.close()


@pytest.mark.parametrize("name", ["branchy", "tandem", "small"])
def test_cli_resume_from_unitig(name, tmp_path):
    """main.cpp:36-42 (-s) through the C++ drop-in CLI, no device needed:
    OverlapGraph() -> setDataset -> readGraphFromFile -> sortEdges -> the
    re-saved checkpoint equals the reference's, the lists its lists."""
    import subprocess

    from conftest import ROOT

    meta, text = reread_golden(name)
    prefix = tmp_path / name
    (tmp_path / f"{name}.unitig").write_text(golden_text(name, "file"))
    exe = os.path.join(ROOT, "metagenomics_amd", "lib", "mg_overlap")
    subprocess.run([exe, "-se", "1", fixture_input(name), "-f", str(prefix), "-l", str(meta["l"]), "-s"], check=True,
                   stdout=subprocess.DEVNULL, timeout=120)
    assert (tmp_path / f"{name}.resumed.unitig").read_text() == golden_text(name, "file")
    got = (tmp_path / f"{name}.resumed.graph").read_text().split("\n")
    assert got[0] == "#C %d %d" % (meta["reread"]["nodes"], meta["reread"]["edges"])


def test_read_graph_from_file_errors(tmp_path):
    meta = load_meta("small")
    ds = Dataset.from_files([fixture_input("small")], meta["l"])
    with pytest.raises(Exception, match="Unable to open"):
        UnitigGraph.from_unitig_file(str(tmp_path / "missing.unitig"), ds.packed()[1])
    bad = tmp_path / "bad.unitig"
    bad.write_text("1\n999999\n3\n10\n0\n")  # a read ID past the Dataset (getReadFromID's range check)
    with pytest.raises(Exception):
        UnitigGraph.from_unitig_file(str(bad), ds.packed()[1])
    empty = tmp_path / "empty.unitig"
    empty.write_text("")
    g = UnitigGraph.from_unitig_file(str(empty), ds.packed()[1])
    assert (g.nodes, g.edges) == (0, 0)
