"""Multi-GPU exchange mode of the overlap path.

One process per GPU. Every rank holds all packed reads. Rank r of P owns two things:
* the index buckets b with floor(b P / 2^nb) == r (bucket-range sharding);
* the source reads (IDs - 1) in [floor(r N / P), floor((r+1) N / P)), i.e. graph[u] of those u.

One step is three all-to-all(v) exchanges of packed record buffers, plus one all-reduce when read lengths
differ:

1. key records of the rank's source reads → bucket owners → local index (``HashTable::insertDataset``,
   HashTable.cpp:50-80);
2. (mixed lengths) containment runs → bucket owners → probe → all-reduce MAX of the per-read
   containment keys (``markContainedReads``, OverlapGraph.cpp:225-290);
3. window runs of the rank's sources → bucket owners → probe + verify (``insertAllEdgesOfRead``,
   OverlapGraph.cpp:529-565) → rows (+ twins, ``insertEdge`` :407-419) → src owners.

The compute is the HIP library (``include/mg_overlap.h``, exchange-mode entry points). This module only
moves the buffers between ranks. ``TorchExchange`` uses ``torch.distributed`` ``all_to_all_single`` over
RCCL/xGMI (backend "nccl"), or gloo for CPU tests. ``LocalExchange`` drives P simulated ranks inside one
process, for single-GPU parity tests. The step logic in :func:`sharded_step` is the same for both.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np

from .overlap import EDGE_DTYPE, MG_KEYS, MG_ROWS, MG_RUNS, RECORD_BYTES


class Exchange:
    """Moves per-destination-grouped byte buffers between the ranks this process drives."""

    world: int
    ranks: list  # the ranks driven by this process

    def empty(self, nbytes: int):
        raise NotImplementedError

    def all_to_all(self, sends: list, counts: list, rec_bytes: int) -> list:
        """sends[i]: buffer of local rank i, grouped by destination, counts[i][d]
        records for d.  Returns [(recv_buffer, n_records)] per local rank."""
        raise NotImplementedError

    def allreduce_max(self, bufs: list) -> None:
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def sync(self) -> None:
        pass


class TorchExchange(Exchange):
    """One rank per process over a torch.distributed group (nccl = RCCL on ROCm, or gloo).

    Every all-to-all(v) call moves at most ``chunk_bytes`` in total per rank:
    the torch-bundled RCCL (2.26.6, ROCm 7.0) corrupts ``all_to_all_single``
    payloads above ~1 GiB per call (measured with one rank, every dtype:
    tools/a2a_probe.py), so larger exchanges run in rounds of
    per-peer slices."""

    def __init__(self, device=None, chunk_bytes: int = 256 << 20):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.ranks = [self.rank]
        self.device = device if device is not None else torch.device("cpu")
        self.chunk_bytes = int(os.environ.get("MG_A2A_CHUNK_BYTES", chunk_bytes))

    def empty(self, nbytes: int):
        return self.torch.empty(max(1, int(nbytes)), dtype=self.torch.uint8, device=self.device)

    def sync(self):
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    def all_to_all(self, sends, counts, rec_bytes):
        torch, dist = self.torch, self.dist
        (send,), (cnt,) = sends, counts
        P, me, rb = self.world, self.rank, rec_bytes
        # the full P x P count matrix: M[s, d] = records s -> d
        sc = torch.tensor([int(c) for c in cnt], dtype=torch.int64, device=self.device)
        mat = torch.empty(P * P, dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(mat, sc)
        M = mat.view(P, P).cpu().numpy()
        scnt, rcnt = M[me, :], M[:, me]
        soff = np.concatenate([[0], np.cumsum(scnt)])
        roff = np.concatenate([[0], np.cumsum(rcnt)])
        n_in = int(rcnt.sum())
        recv = self.empty(n_in * rb)
        per_peer = max(1, self.chunk_bytes // (P * rb))  # records per peer per round
        rounds = max(1, -(-int(M.max()) // per_peer))
        if rounds == 1:
            dist.all_to_all_single(recv[: n_in * rb], send[: int(soff[-1]) * rb],
                                   output_split_sizes=[int(c) * rb for c in rcnt],
                                   input_split_sizes=[int(c) * rb for c in scnt])
        else:
            for t in range(rounds):
                lo = t * per_peer
                s_sz = np.clip(scnt - lo, 0, per_peer)
                r_sz = np.clip(rcnt - lo, 0, per_peer)
                sbuf = torch.cat([send[int(soff[d] + lo) * rb: int(soff[d] + lo + s_sz[d]) * rb] for d in range(P)])
                rbuf = self.empty(int(r_sz.sum()) * rb)
                dist.all_to_all_single(rbuf[: int(r_sz.sum()) * rb], sbuf,
                                       output_split_sizes=[int(c) * rb for c in r_sz],
                                       input_split_sizes=[int(c) * rb for c in s_sz])
                at = 0
                for s_ in range(P):
                    nbytes = int(r_sz[s_]) * rb
                    if nbytes:
                        dst = int(roff[s_] + lo) * rb
                        recv[dst: dst + nbytes].copy_(rbuf[at: at + nbytes])
                    at += nbytes
        self.sync()
        return [(recv, n_in)]

    def allreduce_max(self, bufs):
        (b,) = bufs
        step = max(1, self.chunk_bytes // b.element_size())
        for i in range(0, b.numel(), step):
            self.dist.all_reduce(b[i: i + step], op=self.dist.ReduceOp.MAX)
        self.sync()

    def barrier(self):
        self.sync()
        self.dist.barrier()


class LocalExchange(Exchange):
    """P simulated ranks in one process, all buffers on one device (parity tests)."""

    def __init__(self, world: int, device=None):
        import torch

        self.torch = torch
        self.world = world
        self.ranks = list(range(world))
        self.device = device if device is not None else torch.device("cpu")

    def empty(self, nbytes: int):
        return self.torch.empty(max(1, int(nbytes)), dtype=self.torch.uint8, device=self.device)

    def sync(self):
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    def all_to_all(self, sends, counts, rec_bytes):
        torch = self.torch
        offs = [np.concatenate([[0], np.cumsum(np.asarray(c, dtype=np.int64))]) * rec_bytes for c in counts]
        out = []
        for d in range(self.world):
            parts = [sends[s][int(offs[s][d]): int(offs[s][d + 1])] for s in range(self.world)]
            n = sum(int(counts[s][d]) for s in range(self.world))
            buf = torch.cat(parts) if n else self.empty(0)
            out.append((buf, n))
        self.sync()
        return out

    def allreduce_max(self, bufs):
        m = bufs[0].clone()
        for b in bufs[1:]:
            m = self.torch.maximum(m, b)
        for b in bufs:
            b.copy_(m)
        self.sync()


@dataclass
class ShardResult:
    rows: list            # per local rank: (uint8 buffer of rows, n_rows): the rows whose src it owns
    ms: dict = field(default_factory=dict)
    contained: bool = False
    super_read_id: np.ndarray | None = None  # superReadID per ID (index 0 unused), if requested

    def rows_numpy(self, i: int = 0) -> np.ndarray:
        buf, n = self.rows[i]
        if n == 0:
            return np.zeros(0, dtype=EDGE_DTYPE)
        return buf[: n * 12].cpu().numpy().view(EDGE_DTYPE).copy()


def source_range(n_reads: int, rank: int, world: int):
    """Source reads (0-based) owned by a rank; matches the library's routing rule."""
    return n_reads * rank // world, n_reads * (rank + 1) // world


def sharded_step(engines: list, xchg: Exchange, min_overlap: int, seed_k: int = 0,
                 want_super: bool = False) -> ShardResult:
    """One exchange-mode step over the local ranks' engines (set up with
    ``set_shard(rank, world)`` and the full read set uploaded)."""
    P = xchg.world
    ms = {}
    t0 = time.perf_counter()

    def route(kind, counts):
        rb = RECORD_BYTES[kind]
        sends = []
        for e, c in zip(engines, counts):
            n = int(np.sum(c))
            buf = xchg.empty(n * rb)
            e.pack(kind, buf.data_ptr(), n)
            sends.append(buf)
        return xchg.all_to_all(sends, counts, rb)

    # 1. HashTable::insertDataset: key records -> bucket owners -> local index
    counts = [e.key_records(min_overlap, seed_k, P) for e in engines]
    for e, (buf, n) in zip(engines, route(MG_KEYS, counts)):
        e.insert_keys(buf.data_ptr(), n)
    t1 = time.perf_counter()
    ms["index"] = (t1 - t0) * 1e3

    # 2. markContainedReads (only when lengths differ, OverlapGraph.cpp:228-233)
    # keys (len << 32 | ~index) < 2^48: int64 MAX is the library's unsigned atomicMax
    contained = bool(engines[0].lengths_differ)
    skeys = [xchg.torch.empty(max(1, engines[0].n_reads), dtype=xchg.torch.int64, device=xchg.device)
             if contained else None for _ in engines]
    for e, sk in zip(engines, skeys):
        e.begin_contained(sk.data_ptr() if sk is not None else None)
    if contained:
        counts = [e.scan_runs(True, P) for e in engines]
        for e, (buf, n) in zip(engines, route(MG_RUNS, counts)):
            e.probe_runs(True, buf.data_ptr(), n, P)
        xchg.allreduce_max(skeys)
    sup = None
    for i, e in enumerate(engines):
        s = e.finalize_contained(copy=want_super and i == 0)
        sup = s if s is not None else sup
    del skeys
    t2 = time.perf_counter()
    ms["contained"] = (t2 - t1) * 1e3

    # 3. insertAllEdgesOfRead: window runs -> bucket owners -> rows -> src owners
    counts = [e.scan_runs(False, P) for e in engines]
    counts = [e.probe_runs(False, buf.data_ptr(), n, P) for e, (buf, n) in zip(engines, route(MG_RUNS, counts))]
    rows = route(MG_ROWS, counts)
    ms["overlap"] = (time.perf_counter() - t2) * 1e3
    return ShardResult(rows=rows, ms=ms, contained=contained, super_read_id=sup)
