"""Multi-rank exchange orchestration (metagenomics_amd/sharded.py) on CPU with
the gloo backend, world_size 2 and 3: every key/run record reaches its bucket
owner, every row reaches its src owner, the union of the ranks' rows is the
reference multiset, the containment keys (and the prefix marks before the
containment probe) are MAX-reduced across ranks, and
streams cut at their slot capacity are detected and the step rerun with grown
capacities (the mock starts every stream at 64 records).
The engine is tests/mock_engine.py (routing rules of include/mg_overlap.h); the
GPU kernels behind the same calls are covered by tests/test_gpu_parity.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT, golden_rows, load_meta

sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, outdir, chunk, route):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    if chunk:
        os.environ["MG_A2A_CHUNK_BYTES"] = str(chunk)  # force the multi-round exchange
    os.environ["MG_XCHG_MARKS"] = "1"  # the cross-rank prefix marks' all-reduce (off by default)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist

    from conftest import golden_rows as gr, load_meta as lm
    from metagenomics_amd.overlap import EDGE_DTYPE
    from metagenomics_amd.sharded import TorchExchange, sharded_step
    from mock_engine import MockEngine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = gr(name)
    rows = np.zeros(g.shape[0], dtype=EDGE_DTYPE)
    rows["src"], rows["dst"], rows["orient"], rows["offset"] = g[:, 0], g[:, 1], g[:, 2], g[:, 3]
    n = lm(name)["n_unique"]
    eng = MockEngine(rank, world, rows, n, lengths_differ=(name != "small"))
    res = sharded_step([eng], TorchExchange(), lm(name)["l"], 0, route_rows=route)
    mine = res.rows_numpy(0)
    assert res.n_rows == [len(mine)]
    assert res.rows_routed == route
    pad = res.padding(world, [rank])  # bench.py's exchange_padding
    assert set(pad) == ({"keys", "runs", "rows"} if route else {"keys", "runs"})
    assert eng.options["xchg_route_rows"] == int(route)
    for v in pad.values():
        assert 0 <= v["sent_records"] <= v["moved_records"] and 0.0 <= v["padding_frac"] <= 1.0
    np.save(os.path.join(outdir, f"reruns{rank}.npy"), np.array([res.reruns, eng.begins]))
    np.save(os.path.join(outdir, f"rows{rank}.npy"), mine)
    np.save(os.path.join(outdir, f"keys{rank}.npy"), eng.received_keys)
    np.save(os.path.join(outdir, f"sk{rank}.npy"), eng.super_keys)
    np.save(os.path.join(outdir, f"marks{rank}.npy"), np.array([eng.marks_seen, eng.lengths_differ]))
    np.save(os.path.join(outdir, f"own{rank}.npy"), np.array([getattr(eng, "own_probes", 0)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world,chunk,route", [("small", 2, 0, True), ("tandem", 3, 0, True),
                                                    ("mixed", 2, 0, True), ("small", 2, 4096, True),
                                                    ("tandem", 3, 8192, True), ("small", 2, 0, False),
                                                    ("mixed", 3, 4096, False)])
def test_exchange_routes_every_record(tmp_path, name, world, chunk, route):
    """route: rows to their src owners (MG_XCHG_ROUTE_ROWS=1); else each rank keeps the
    rows it verified and only keys and runs travel (the default)."""
    from mock_engine import expected_super_keys, src_owner

    mp.spawn(_worker, args=(world, _free_port(), name, str(tmp_path), chunk, route), nprocs=world, join=True)
    meta = load_meta(name)
    n = meta["n_unique"]
    parts, keys = [], 0
    for r in range(world):
        rows = np.load(tmp_path / f"rows{r}.npy")
        if route:
            assert np.all(src_owner(rows["src"], n, world) == r), "row at a rank that does not own its src"
        parts.append(rows)
        keys += np.load(tmp_path / f"keys{r}.npy").shape[0]
        seen, differ = np.load(tmp_path / f"marks{r}.npy")
        if differ:
            assert np.array_equal(np.load(tmp_path / f"sk{r}.npy"), expected_super_keys(n))
        # equal lengths ("small"): the split discovery probe, own stream first
        assert np.load(tmp_path / f"own{r}.npy")[0] == (0 if differ else np.load(tmp_path / f"reruns{r}.npy")[1])
        assert seen == differ  # the cross-rank prefix marks: made, all-reduced, seen by the containment probe
    assert keys == 4 * n
    rr = [np.load(tmp_path / f"reruns{r}.npy") for r in range(world)]
    assert all(x[0] == rr[0][0] for x in rr), "ranks disagree on the reruns"
    assert all(x[1] == x[0] + 1 for x in rr)  # one begin per attempt
    allr = np.concatenate(parts)
    t = np.stack([allr["src"], allr["dst"], allr["orient"], allr["offset"]], axis=1).astype(np.int64)
    t = t[np.lexsort((t[:, 3], t[:, 2], t[:, 1], t[:, 0]))]
    assert np.array_equal(t, golden_rows(name))


def test_slot_geometry():
    from metagenomics_amd.sharded import BIG_SLOT_ALIGN, SLOT_ALIGN, slot_geometry

    for cap, world, rb, ch in [(1, 1, 16, 256 << 20), (10**8, 1, 16, 256 << 20), (10**8, 8, 12, 256 << 20),
                               (1000, 2, 16, 4096), (64, 3, 12, 100), (5 * 10**6, 64, 16, 256 << 20)]:
        slot, rounds = slot_geometry(cap, world, rb, ch)
        assert slot % SLOT_ALIGN == 0 and slot >= SLOT_ALIGN and rounds >= 1
        if cap >= 64 * BIG_SLOT_ALIGN:  # whole 1024-record probe regions
            assert slot % BIG_SLOT_ALIGN == 0
        assert slot * rounds >= cap
        assert world * slot * rb <= max(ch, world * SLOT_ALIGN * rb)  # a round stays within the chunk
        assert world * slot * rb < 2**31  # every all-to-all call's byte count fits int32
