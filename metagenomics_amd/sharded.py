"""Multi-GPU exchange mode of the overlap path.

One process per GPU. Every rank holds all packed reads. Rank r of P owns two things:
* the index buckets b with floor(b P / 2^nb) == r (bucket-range sharding);
* the source reads (IDs - 1) in [floor(r N / P), floor((r+1) N / P)), i.e. graph[u] of those u.

One step (``sharded_step``):

1. ``xchg_begin``: one window scan of the rank's source reads writes the four index keys of every
   source read (``hashRead``, HashTable.cpp:88-104) and its minimizer runs; the runs are radix-sorted
   by bucket, which also groups them by owning rank;
2. keys -> bucket owners -> local cells (``HashTable::insertDataset``, HashTable.cpp:50-80);
3. runs -> bucket owners (kept for both probes);
4. (mixed lengths) [MG_XCHG_MARKS=1: each rank's offset-0 containments and an all-reduce MAX
   of their marks, so every rank's probe skips sources any rank found contained] the
   containment probe of the received runs, all-reduce MAX of the per-read containment keys
   (``markContainedReads``, OverlapGraph.cpp:225-290);
5. discovery probe + verify of the received runs (``insertAllEdgesOfRead``, OverlapGraph.cpp:529-565)
   -> rows (+ twins, ``insertEdge`` :407-419), held by the rank that verified them (the union over
   ranks is the reference multiset); with ``route_rows`` they then go to their src owners, so each
   rank ends with graph[u] of its own source reads.

Record sizes on the wire (``engine.record_bytes``, mg_record_bytes): a key is its 8-B index entry
and a run its 8-B meta (read slot, minimizer position, window range); the receiver re-hashes the
minimizer m-mer from its own copy of the read (every rank holds all reads), so bucket and
fingerprint never travel.  Rows are 12-B mg_edge records.

Records travel in the library's SLOT LAYOUT (include/mg_overlap.h "exchange mode"): per peer a
fixed-capacity stream of ``rounds * slot`` records, round t of all peers contiguous, so every round
is one group of equal-size sends/receives straight from the packed buffer (no host-side split
sizes, no per-round concatenation), and the per-peer record counts travel as a device tensor in
one equal-split all-to-all. A rank's stream to itself never travels: the pack writes it straight
into the rank's receive buffer (same slot offsets), so one rank moves nothing but its counts. Nothing in the step waits on the host for the exchange: the capacities are
fixed up front (``XchgPlan``) and a stream that would not fit is cut; its full count comes back with
the step's single host read (an all-reduce MAX of the send counts), and the step is rerun with the
capacities grown. With a CUDA device the library calls, the torch copies and the RCCL collectives
are all ordered on the engine's own HIP stream.

``TorchExchange`` uses ``torch.distributed`` (backend "nccl" = RCCL over xGMI, or gloo for CPU
tests). ``LocalExchange`` drives P simulated ranks inside one process (single-GPU parity tests).
"""
from __future__ import annotations

import contextlib
import os
import time
from dataclasses import dataclass, field

import numpy as np

from .overlap import EDGE_DTYPE, MG_KEYS, MG_ROWS, MG_RUNS

SLOT_ALIGN = 64  # slots are whole multiples of this many records (the probe tiles a slot by its divisors)
BIG_SLOT_ALIGN = 1024
# the exchange mode's kernels keep a read in registers and pack window
# positions into 10 bits: reads up to 1,024 bp (longer ones: replicated mode)
EXCHANGE_MAX_BP = 1024
KINDS = (MG_KEYS, MG_RUNS, MG_ROWS)


def slot_geometry(cap: int, world: int, rec_bytes: int, chunk_bytes: int):
    """(slot, rounds) for a per-peer stream of at most ``cap`` records: one round moves
    world * slot records per rank, at most ``chunk_bytes`` (never below one aligned slot).
    Large streams take slots of whole 1024-record regions (the probe's region size over
    the received runs is the largest power of two <= 1024 dividing the slot)."""
    align = BIG_SLOT_ALIGN if cap >= 64 * BIG_SLOT_ALIGN else SLOT_ALIGN
    per_round = max(align, (chunk_bytes // (world * rec_bytes)) // align * align)
    want = max(align, -(-int(cap) // align) * align)
    rounds = -(-want // per_round)
    # the rounds share the stream evenly: a stream just past one round's size
    # moves ~2x its records with full-size rounds, ~cap with even ones
    slot = -(-(-(-want // rounds)) // align) * align
    return slot, rounds


@dataclass
class XchgPlan:
    """Per-peer stream capacities (records) for keys, runs and rows; identical on every rank
    (derived from global quantities only, then grown from all-reduced counts)."""
    caps: dict = field(default_factory=dict)
    reruns: int = 0

    def geometry(self, kind: int, world: int, chunk_bytes: int, rec_bytes: int):
        return slot_geometry(self.caps[kind], world, rec_bytes, chunk_bytes)

    def grow(self, used: dict) -> bool:
        """Fit the capacities to the counts seen (MAX over ranks and peers, identical on every
        rank): streams that overflowed grow (True: rerun the step), the others shrink, so from
        the second step on the slot layout moves ~6 % more than the largest stream instead of
        the first guess (rows: 32 per source read, ~10x C5's).  (15 % until round 6: the
        per-peer counts of a step over the same reads repeat exactly; a batch of other reads
        whose stream outgrows the margin costs one rerun of that step.)"""
        over = False
        for k, c in used.items():
            want = int(c * 1.06) + SLOT_ALIGN
            if c > self.caps[k]:
                over = True
            self.caps[k] = want
        return over


class Exchange:
    """Moves slot-layout buffers between the ranks this process drives."""

    world: int
    ranks: list  # the ranks driven by this process
    device = None

    def empty(self, nbytes: int):
        return self.torch.empty(max(1, int(nbytes)), dtype=self.torch.uint8, device=self.device)

    def counts(self):
        # no fill kernel: the library writes every entry (a fill on another stream could land after it)
        return self.torch.empty(self.world, dtype=self.torch.int64, device=self.device)

    def streams(self, engines):
        """Context in which the step's torch work is ordered with the engines' HIP streams."""
        return contextlib.nullcontext()

    def all_to_all_slots(self, sends: list, recvs: list, counts: list, slot: int, rounds: int,
                         rec_bytes: int) -> list:
        """sends[i] / recvs[i] / counts[i]: slot-layout send and receive buffers and per-peer
        counts of local rank i; its slots for itself are already in recvs[i].  Moves every other
        slot and returns [(recv_buffer, recv_counts)] per local rank."""
        raise NotImplementedError

    def all_to_all_slots_async(self, sends: list, recvs: list, counts: list, slot: int, rounds: int,
                               rec_bytes: int):
        """all_to_all_slots started now; returns finish() -> its result, after which the
        engines' work may read the received slots.  The base class moves them at once."""
        out = self.all_to_all_slots(sends, recvs, counts, slot, rounds, rec_bytes)
        return lambda: out

    def allreduce_max(self, bufs: list) -> None:
        raise NotImplementedError

    def max_counts(self, sent: list) -> np.ndarray:
        """sent[i] = the per-peer send counts (one tensor per kind) of local rank i: the MAX of
        each kind over the local ranks and over all ranks, on the host."""
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def sync(self) -> None:
        pass


class TorchExchange(Exchange):
    """One rank per process over a torch.distributed group (nccl = RCCL on ROCm, or gloo).

    Each round is one equal-split ``all_to_all_single`` of world * slot records, at most
    ``chunk_bytes`` per rank (256 MiB by default): the torch-bundled RCCL corrupted single
    all-to-all payloads above ~1 GiB per call in round 1 (tools/a2a_probe.py), and
    rounds of a few hundred MiB cost nothing measurable on xGMI."""

    def __init__(self, device=None, chunk_bytes: int = 256 << 20):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.ranks = [self.rank]
        self.device = device if device is not None else torch.device("cpu")
        self.chunk_bytes = int(os.environ.get("MG_A2A_CHUNK_BYTES", chunk_bytes))
        # gloo moves host tensors only: device buffers are staged through host copies.  This
        # is the multi-process rehearsal of the real library path on a box with fewer GPUs
        # than ranks (RCCL refuses two ranks on one device); with "nccl" nothing is staged.
        self.staged = self.device.type == "cuda" and dist.get_backend() == "gloo"

    def streams(self, engines):
        if self.device.type != "cuda" or not engines or not hasattr(engines[0], "stream"):
            return contextlib.nullcontext()
        # the collectives and torch copies run on the library's stream: no host round trip
        s = self.torch.cuda.ExternalStream(engines[0].stream(), device=self.device)
        return self.torch.cuda.stream(s)

    def sync(self):
        if self.device.type == "cuda":
            self.torch.cuda.current_stream(self.device).synchronize()

    def all_to_all_slots(self, sends, recvs, counts, slot, rounds, rec_bytes):
        (send,), (recv,), (cnt,) = sends, recvs, counts
        P, me, sb = self.world, self.rank, slot * rec_bytes
        if P == 1:
            return [(recv, cnt)]
        dist = self.dist
        dev_recv = recv
        if self.staged:  # (.cpu() waits for the library's pack on this stream)
            send, recv, cnt = send.cpu(), recv.cpu(), cnt.cpu()
        for t in range(rounds):  # one group of sends/receives per round, none to itself
            ops = []
            for p in range(P):
                if p != me:
                    at = (t * P + p) * sb
                    ops.append(dist.P2POp(dist.isend, send[at: at + sb], p))
                    ops.append(dist.P2POp(dist.irecv, recv[at: at + sb], p))
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        rc = self.torch.empty_like(cnt)
        dist.all_to_all_single(rc, cnt)
        if self.staged:
            dev_recv.copy_(recv)
            return [(dev_recv, rc.to(self.device))]
        return [(recv, rc)]

    def all_to_all_slots_async(self, sends, recvs, counts, slot, rounds, rec_bytes):
        """The transfers go out on a side stream that waits only for the packs so far, so
        the engine stream's next work (the own-stream probe) runs while they are on the
        links; finish() makes the engine stream wait for them."""
        if self.staged or self.world == 1 or self.device.type != "cuda":
            return super().all_to_all_slots_async(sends, recvs, counts, slot, rounds, rec_bytes)
        torch = self.torch
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        packed = torch.cuda.Event()
        packed.record(main)
        with torch.cuda.stream(self._side):
            self._side.wait_event(packed)
            out = self.all_to_all_slots(sends, recvs, counts, slot, rounds, rec_bytes)
            arrived = torch.cuda.Event()
            arrived.record(self._side)

        def finish():
            main.wait_event(arrived)
            return out
        return finish

    def allreduce_max(self, bufs):
        (b,) = bufs
        h = b.cpu() if self.staged else b
        step = max(1, self.chunk_bytes // h.element_size())
        for i in range(0, h.numel(), step):
            self.dist.all_reduce(h[i: i + step], op=self.dist.ReduceOp.MAX)
        if self.staged:
            b.copy_(h)

    def max_counts(self, sent):
        (cnts,) = sent
        v = self.torch.stack([c.max() for c in cnts])
        if self.staged:
            v = v.cpu()
        self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX)
        return v.cpu().numpy()

    def barrier(self):
        self.sync()
        self.dist.barrier()


class LocalExchange(Exchange):
    """P simulated ranks in one process, all buffers on one device (parity tests, --sim-world).
    The engines run on separate HIP streams, so every exchange synchronizes the device."""

    def __init__(self, world: int, device=None, chunk_bytes: int = 256 << 20, serial: bool | None = None):
        import torch

        self.torch = torch
        self.world = world
        # serial: every library call of a simulated rank completes before the next starts, so
        # a kernel trace times each rank's kernels alone (the engines' streams otherwise overlap
        # on the one GPU and every duration includes the other ranks' work; MG_SIM_SERIAL=1)
        self.serial = bool(int(os.environ.get("MG_SIM_SERIAL", "0"))) if serial is None else serial
        self.ranks = list(range(world))
        self.device = device if device is not None else torch.device("cpu")
        self.chunk_bytes = int(os.environ.get("MG_A2A_CHUNK_BYTES", chunk_bytes))

    def sync(self):
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    def all_to_all_slots(self, sends, recvs, counts, slot, rounds, rec_bytes):
        P, sb = self.world, slot * rec_bytes
        self.sync()
        out = []
        for d in range(P):
            recv = recvs[d]
            for t in range(rounds):
                for s in range(P):
                    if s != d:
                        recv[(t * P + s) * sb:(t * P + s + 1) * sb].copy_(
                            sends[s][(t * P + d) * sb:(t * P + d + 1) * sb])
            rc = self.torch.stack([counts[s][d] for s in range(P)])
            out.append((recv, rc))
        self.sync()
        return out

    def allreduce_max(self, bufs):
        self.sync()
        m = bufs[0].clone()
        for b in bufs[1:]:
            m = self.torch.maximum(m, b)
        for b in bufs:
            b.copy_(m)
        self.sync()

    def max_counts(self, sent):
        self.sync()  # the engines wrote the counts on their own streams
        v = self.torch.stack([self.torch.stack([c.max() for c in cnts]) for cnts in sent])
        return v.max(dim=0).values.cpu().numpy()


@dataclass
class ShardResult:
    rows: list            # route_rows: per local rank (uint8 slot buffer, counts tensor, slot, rounds): rows it owns by src
    ms: dict = field(default_factory=dict)
    contained: bool = False
    super_read_id: np.ndarray | None = None  # superReadID per ID (index 0 unused), if requested
    n_rows: list = field(default_factory=list)  # rows held per local rank
    reruns: int = 0       # steps rerun with grown capacities
    plan: XchgPlan | None = None  # the capacities used (pass it to the next step)
    # kind -> (slot, rounds, [per local rank: per-peer send counts]): the slot layout moves
    # rounds * slot records to every peer whatever the count (padding(), outside the timed step)
    streams: dict = field(default_factory=dict)
    # long-read fallback (replicated mode): per local rank the rows it holds, on the host
    host_rows: list | None = None
    # one rank: nothing is routed, the rows stay in the engine (mg_xchg_pack at P = 1)
    engine_rows: list | None = None
    mode: str = "exchange"
    rows_routed: bool = False  # rows moved to their src owners (route_rows) or held where verified
    rec_bytes: dict = field(default_factory=dict)  # kind -> bytes per record on the wire

    @property
    def rows_in_slots(self) -> bool:
        """The rows are in slot-layout receive buffers (self.rows)."""
        return self.host_rows is None and self.engine_rows is None

    def padding(self, world: int, rank_ids: list) -> dict:
        """Per stream kind: records the slot layout moved between ranks vs the records sent
        (own slots excluded; they never travel), summed over the local ranks."""
        out = {}
        for kind, (slot, rounds, cnts) in self.streams.items():
            moved = sent = 0
            for r, c in zip(rank_ids, cnts):
                v = c.cpu().numpy().astype(np.int64)
                for p in range(world):
                    if p != r:
                        moved += slot * rounds
                        sent += int(v[p])
            out[{MG_KEYS: "keys", MG_RUNS: "runs", MG_ROWS: "rows"}[kind]] = {
                "moved_records": moved, "sent_records": sent, "record_bytes": self.rec_bytes.get(kind),
                "padding_frac": (1.0 - sent / moved) if moved else 0.0}
        return out

    def rows_numpy(self, i: int = 0) -> np.ndarray:
        """The rows of local rank i, compacted out of the slot layout (host copy)."""
        if self.host_rows is not None:
            return self.host_rows[i]
        if self.engine_rows is not None:
            return self.engine_rows[i].rows(self.n_rows[i])
        buf, cnt, slot, rounds = self.rows[i]
        c = cnt.cpu().numpy().astype(np.int64)
        P = len(c)
        raw = buf[: rounds * P * slot * 12].cpu().numpy().view(EDGE_DTYPE)
        parts = []
        for s in range(P):
            for t in range(rounds):
                k = min(max(0, int(c[s]) - t * slot), slot)
                if k:
                    at = (t * P + s) * slot
                    parts.append(raw[at: at + k])
        return np.concatenate(parts).copy() if parts else np.zeros(0, dtype=EDGE_DTYPE)


def source_range(n_reads: int, rank: int, world: int):
    """Source reads (0-based) owned by a rank; matches the library's routing rule."""
    return n_reads * rank // world, n_reads * (rank + 1) // world


def initial_plan(engine, world: int, min_overlap: int, seed_k: int) -> XchgPlan:
    caps = engine.xchg_caps(min_overlap, seed_k)
    return XchgPlan(caps={MG_KEYS: int(caps[0]), MG_RUNS: int(caps[1]), MG_ROWS: int(caps[2])})


def route_rows_default() -> bool:
    """MG_XCHG_ROUTE_ROWS=1: route the rows to their src owners (default: held where verified)."""
    return os.environ.get("MG_XCHG_ROUTE_ROWS", "0") == "1"


def sharded_step(engines: list, xchg: Exchange, min_overlap: int, seed_k: int = 0,
                 want_super: bool = False, plan: XchgPlan | None = None,
                 route_rows: bool | None = None) -> ShardResult:
    """One exchange-mode step over the local ranks' engines (set up with
    ``set_shard(rank, world)`` and the full read set uploaded).  ``plan`` carries the
    stream capacities from step to step (grown in place after an overflow).
    ``route_rows``: every row goes to the owner of its src (graph[u] by source range,
    one more all-to-all); else (default) each rank keeps the rows it verified, and the
    union over the ranks is the reference multiset all the same."""
    if route_rows is None:
        route_rows = route_rows_default()
    if any(e.max_len > EXCHANGE_MAX_BP for e in engines):
        return _replicated_step(engines, xchg, min_overlap, seed_k, want_super)
    if plan is None:
        plan = initial_plan(engines[0], xchg.world, min_overlap, seed_k)
    reruns = 0
    while True:
        res, used = _step(engines, xchg, min_overlap, seed_k, want_super, plan, route_rows)
        if not plan.grow(used):
            res.reruns = reruns
            res.plan = plan
            return res
        reruns += 1
        plan.reruns += 1
        if reruns > 3:
            raise RuntimeError(f"exchange capacities still overflow after {reruns} reruns: {used}")


_warned_long = [False]


def _replicated_step(engines, xchg, min_overlap, seed_k, want_super):
    """Reads longer than EXCHANGE_MAX_BP (Read::getReadLength is UINT16, Read.h:62):
    the step runs the replicated mode instead (every rank builds the
    whole index with the long-read kernels and discovers from its source-read
    range; no data-path collective).  Every rank holds the rows + twins of its
    sources' discoveries; their union is the reference multiset.  The engines
    run this step on their source ranges (set_shard(0, 1, lo, hi)) and get their
    bucket-range shards (set_shard(rank, world)) back at its end.  ms splits the
    wall into index / contained / overlap like the exchange step's."""
    if not _warned_long[0]:
        print(f"[sharded] reads longer than {EXCHANGE_MAX_BP} bp: the exchange mode's kernels stop there; "
              "this step runs the replicated mode (whole index per rank, source-read shards, no data-path "
              "collective)", flush=True)
        _warned_long[0] = True
    P = xchg.world
    ranges = [source_range(e.n_reads, r, P) for e, r in zip(engines, xchg.ranks)]
    ms = {}
    sup = None
    try:
        t0 = time.perf_counter()
        for e, (lo, hi) in zip(engines, ranges):
            e.set_shard(0, 1, lo, hi if hi > lo else lo)
            e.build_index(min_overlap, seed_k)
        xchg.sync()
        t1 = time.perf_counter()
        for i, e in enumerate(engines):
            s = e.mark_contained(copy=want_super and i == 0)
            sup = s if s is not None else sup
        xchg.sync()
        t2 = time.perf_counter()
        n_rows = [e.find_overlaps() if hi > lo else 0  # (read_hi == read_lo == 0 would mean "all")
                  for e, (lo, hi) in zip(engines, ranges)]
        xchg.barrier()
        t3 = time.perf_counter()
        host_rows = [e.rows(n) if n else np.zeros(0, dtype=EDGE_DTYPE) for e, n in zip(engines, n_rows)]
    finally:
        # give the engines back the bucket-range shards the caller set up (set_shard(rank, world)),
        # so a later step with short reads runs the exchange mode with the right routing
        for e, r in zip(engines, xchg.ranks):
            e.set_shard(r, P, 0, 0)
    ms = {"index": (t1 - t0) * 1e3, "contained": (t2 - t1) * 1e3, "overlap": (t3 - t2) * 1e3}
    return ShardResult(rows=[], ms=ms, contained=bool(engines[0].lengths_differ), super_read_id=sup,
                       n_rows=n_rows, host_rows=host_rows, mode="replicated")


def _step(engines, xchg, min_overlap, seed_k, want_super, plan, route_rows):
    P = xchg.world
    route_rows = route_rows and P > 1
    kinds = KINDS if route_rows else (MG_KEYS, MG_RUNS)
    for e in engines:  # the discovery probe counts rows per src owner only when they will move
        e.set_option("xchg_route_rows", int(route_rows))
    rec_bytes = {k: int(engines[0].record_bytes(k)) for k in KINDS}
    # cross-rank prefix marks (mg_xchg_prefix_marks): off by default -- at C5,
    # P = 8 the containment probe gained 0.14 ms per rank and the marks cost 0.21 ms plus a
    # 50 MB all-reduce; MG_XCHG_MARKS=1 turns them on
    prefix_marks = os.environ.get("MG_XCHG_MARKS", "0") == "1"
    serial = getattr(xchg, "serial", False)

    def done():  # (serial simulated ranks: one rank's call at a time on the device)
        if serial:
            xchg.sync()
    ch = getattr(xchg, "chunk_bytes", 256 << 20)
    ms = {}
    sent = {}
    geo = {}

    def route(kind, move=True):
        """pack `kind` on every engine; move=False leaves the all-to-all to the caller
        (returns the pack's buffers: (sends, recvs, counts), slot, rounds)"""
        if P == 1:  # one rank: every stream is its own, nothing is packed or sent (the
            # consumers read the context's own key records and run regions; counts = 0)
            cnts = [zero] * len(engines)
            sent[kind] = cnts
            geo[kind] = (0, 0)
            return [(None, c) for c in cnts], 0, 0
        rb = rec_bytes[kind]
        slot, rounds = plan.geometry(kind, P, ch, rb)
        sends, recvs, cnts = [], [], []
        for e in engines:
            recv = xchg.empty(rounds * P * slot * rb)
            send = xchg.empty(rounds * P * slot * rb) if P > 1 else None
            c = xchg.counts()
            e.xchg_pack(kind, send.data_ptr() if send is not None else 0, slot, rounds, c.data_ptr(),
                        recv.data_ptr())
            done()
            sends.append(send)
            recvs.append(recv)
            cnts.append(c)
        sent[kind] = cnts
        geo[kind] = (slot, rounds)
        if not move:
            return (sends, recvs, cnts), slot, rounds
        return xchg.all_to_all_slots(sends, recvs, cnts, slot, rounds, rb), slot, rounds

    zero = xchg.counts().zero_() if P == 1 else None
    t0 = time.perf_counter()
    with xchg.streams(engines):
        # 1. one scan of the rank's sources: index keys + sorted runs
        for e in engines:
            e.xchg_begin(min_overlap, seed_k)
            done()
        # 2. HashTable::insertDataset: key records -> bucket owners -> local cells
        keys, ks, kr = route(MG_KEYS)
        for e, (buf, c) in zip(engines, keys):
            e.xchg_insert_keys(buf.data_ptr() if buf is not None else 0, ks, kr, c.data_ptr())
            done()
        # 3. runs -> bucket owners (both probes read them).  Equal lengths (no containment
        # pass) split the discovery probe: each rank's own stream (written straight into its
        # receive buffer by the pack) is probed while the peers' streams are on the links
        contained = bool(engines[0].lengths_differ)
        split = P > 1 and not contained
        if split:
            (rsend, rrecv, rcnt), rs, rr = route(MG_RUNS, move=False)
            runs_in = xchg.all_to_all_slots_async(rsend, rrecv, rcnt, rs, rr, rec_bytes[MG_RUNS])
        else:
            runs, rs, rr = route(MG_RUNS)
        t1 = time.perf_counter()
        ms["index"] = (t1 - t0) * 1e3

        # 4. markContainedReads (only when lengths differ, OverlapGraph.cpp:228-233)
        # keys (len << 32 | ~index) < 2^48: int64 MAX is the library's unsigned atomicMax
        skeys = [xchg.torch.empty(max(1, engines[0].n_reads), dtype=xchg.torch.int64, device=xchg.device)
                 if contained else None for _ in engines]
        for e, sk in zip(engines, skeys):
            e.begin_contained(sk.data_ptr() if sk is not None else None)
        if contained and P > 1 and prefix_marks:
            # every rank's offset-0 containments before the probe: the all-reduced
            # marks let each rank's probe skip sources another rank found contained
            marks = [xchg.torch.empty(max(1, engines[0].n_reads), dtype=xchg.torch.uint8, device=xchg.device)
                     for _ in engines]
            for e, mk in zip(engines, marks):
                e.xchg_prefix_marks(mk.data_ptr())
                done()
            xchg.allreduce_max(marks)
        else:
            marks = None
        if contained:
            for e, (buf, c) in zip(engines, runs):
                e.xchg_probe(True, buf.data_ptr() if buf is not None else 0, rs, rr, c.data_ptr())
                done()
            xchg.allreduce_max(skeys)
        del marks  # (read by the probes above, on the engines' streams: after the all-reduce's sync)
        sup = None
        for i, e in enumerate(engines):
            s = e.finalize_contained(copy=want_super and i == 0)
            sup = s if s is not None else sup
        del skeys
        t2 = time.perf_counter()
        ms["contained"] = (t2 - t1) * 1e3

        # 5. insertAllEdgesOfRead: probe the received runs -> rows [-> src owners]
        if split:
            for e, buf, c in zip(engines, rrecv, rcnt):  # the own stream, while the peers' travel
                e.xchg_probe_own(buf.data_ptr(), rs, rr, c.data_ptr())
                done()
            runs = runs_in()
        for e, (buf, c) in zip(engines, runs):
            e.xchg_probe(False, buf.data_ptr() if buf is not None else 0, rs, rr, c.data_ptr())
            done()
        if route_rows:
            rows, ws, wr = route(MG_ROWS)
        # the step's one host read: MAX over ranks of every per-peer send count
        # (one rank: nothing was sent, so no collective and no host read of counts)
        mx = (xchg.max_counts([[sent[k][i] for k in kinds] for i in range(len(engines))]) if P > 1
              else np.zeros(len(kinds), dtype=np.int64))
        n_rows = [int(c.sum().item()) for _, c in rows] if route_rows else [e.num_rows() for e in engines]
        # (the key and run buffers stay referenced until here: with LocalExchange the
        # engines' streams may still read them when a del would let torch reuse the memory)
        del keys, runs
    ms["overlap"] = (time.perf_counter() - t2) * 1e3
    used = {k: int(v) for k, v in zip(kinds, mx)}
    res = ShardResult(rows=[(b, c, ws, wr) for b, c in rows] if route_rows else [], ms=ms, contained=contained,
                      super_read_id=sup, n_rows=n_rows, streams={k: geo[k] + (sent[k],) for k in kinds},
                      engine_rows=None if route_rows else list(engines), rows_routed=route_rows,
                      rec_bytes=rec_bytes)
    return res, used
