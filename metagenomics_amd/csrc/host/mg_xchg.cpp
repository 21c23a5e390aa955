// mg_xchg.cpp — see mg_xchg.hpp.  The step mirrors metagenomics_amd/sharded.py
// _step over the C-ABI of include/mg_overlap.h:
//   mg_xchg_begin                          one window scan of this rank's sources
//   mg_xchg_pack(KEYS) -> RCCL -> mg_xchg_insert_keys     HashTable::insertDataset
//   mg_xchg_pack(RUNS) -> RCCL (second stream)     [mg_xchg_probe_own meanwhile]
//   mg_begin_contained; [mg_xchg_prefix_marks; ncclAllReduce MAX (u8);
//                        mg_xchg_probe(1); ncclAllReduce MAX]; mg_finalize_contained
//                                                          markContainedReads
//   mg_xchg_probe(0) [-> mg_xchg_pack(ROWS) -> RCCL]      insertAllEdgesOfRead
// Keys and runs travel as 8-B records (mg_record_bytes); the rows move to
// their src owners only with MG_XCHG_ROUTE_ROWS=1, else each rank keeps the
// rows it verified (the union is the multiset).
// Every library call and every collective is enqueued on the context's HIP
// stream (mg_stream); the step reads the host only for the run and row counts
// inside the library and once at its end (the MAX over ranks of the send
// counts, to detect a stream cut at its capacity).
#include "mg_xchg.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "mg_host.h"

namespace mg {

namespace {
constexpr size_t kChunkBytes = 256ull << 20;
constexpr int kRendezvousMs = 300000;  // every rank of the job connects within 5 minutes
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// rank 0 creates the id and serves it to the other ranks (mgh_rendezvous:
// host names resolve, every wait has a deadline, descriptors never leak)
ncclUniqueId rendezvous(int rank, int world, const std::string& addr, int port) {
  ncclUniqueId id;
  if (rank == 0) nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  if (world == 1) return id;
  const int rc = mgh_rendezvous(rank, world, addr.c_str(), port, &id, sizeof id, kRendezvousMs);
  if (rc)
    throw std::runtime_error("rendezvous with rank 0 at " + addr + ":" + std::to_string(port) + " failed (" +
                             (rc == -2 ? "address does not resolve" : rc == -3 ? "cannot listen" :
                              rc == -4 ? "deadline passed: a rank never connected" : "I/O error") + ")");
  return id;
}
}  // namespace

RcclExchange::RcclExchange(int rank, int world, int device, const std::string& addr, int port)
    : rank_(rank), world_(world) {
  hip_check(hipSetDevice(device), "hipSetDevice");
  const ncclUniqueId id = rendezvous(rank, world, addr, port);
  nccl_check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
}

RcclExchange::~RcclExchange() {
  if (flag_) (void)hipFree(flag_);
  if (comm_) ncclCommDestroy(comm_);
}

void RcclExchange::all_to_all_slots(const uint8_t* send, uint8_t* recv, uint64_t sb, uint32_t rounds,
                                    hipStream_t s) {
  if (world_ == 1) return;
  for (uint32_t t = 0; t < rounds; ++t) {  // one group of point-to-point transfers per round, none to itself
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      const uint64_t at = ((uint64_t)t * world_ + p) * sb;
      nccl_check(ncclSend(send + at, sb, ncclUint8, p, comm_, s), "ncclSend");
      nccl_check(ncclRecv(recv + at, sb, ncclUint8, p, comm_, s), "ncclRecv");
    }
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }
}

void RcclExchange::all_to_all_u64(const uint64_t* send, uint64_t* recv, hipStream_t s) {
  if (world_ == 1) {
    hip_check(hipMemcpyAsync(recv, send, sizeof(uint64_t), hipMemcpyDeviceToDevice, s), "counts copy");
    return;
  }
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  for (int p = 0; p < world_; ++p) {
    nccl_check(ncclSend(send + p, 1, ncclUint64, p, comm_, s), "ncclSend");
    nccl_check(ncclRecv(recv + p, 1, ncclUint64, p, comm_, s), "ncclRecv");
  }
  nccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

void RcclExchange::allreduce_max_u64(uint64_t* buf, size_t n, hipStream_t s) {
  if (world_ == 1) return;
  const size_t step = kChunkBytes / sizeof(uint64_t);  // bounded payload per collective
  for (size_t i = 0; i < n; i += step)
    nccl_check(ncclAllReduce(buf + i, buf + i, std::min(step, n - i), ncclUint64, ncclMax, comm_, s), "ncclAllReduce");
}

void RcclExchange::allreduce_max_u8(uint8_t* buf, size_t n, hipStream_t s) {
  if (world_ == 1) return;
  for (size_t i = 0; i < n; i += kChunkBytes)
    nccl_check(ncclAllReduce(buf + i, buf + i, std::min(kChunkBytes, n - i), ncclUint8, ncclMax, comm_, s),
               "ncclAllReduce");
}

void RcclExchange::allreduce_max_f64(double* buf, size_t n, hipStream_t s) {
  if (world_ > 1) nccl_check(ncclAllReduce(buf, buf, n, ncclFloat64, ncclMax, comm_, s), "ncclAllReduce");
}

void RcclExchange::barrier(hipStream_t s) {
  if (world_ > 1) {
    if (!flag_) hip_check(hipMalloc(&flag_, sizeof(double)), "hipMalloc");
    allreduce_max_f64(flag_, 1, s);
  }
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

void RcclExchange::allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s) {
  if (world_ == 1) {
    hip_check(hipMemcpyAsync(recv, send, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s), "allgather copy");
    return;
  }
  nccl_check(ncclAllGather(send, recv, n, ncclUint64, comm_, s), "ncclAllGather");
}

LocalGroup::LocalGroup(int world, int timeout_ms)
    : world_(world), timeout_ms_(timeout_ms), ptrs_(world, nullptr), dbl_(world, 0.0) {}

void LocalGroup::barrier() {
  std::unique_lock<std::mutex> lk(mu_);
  if (failed_) throw std::runtime_error("a peer rank failed");
  const uint64_t gen = gen_;
  if (++arrived_ == world_) {
    arrived_ = 0;
    ++gen_;
    cv_.notify_all();
    return;
  }
  if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms_), [&] { return gen_ != gen || failed_; })) {
    failed_ = true;
    cv_.notify_all();
    throw std::runtime_error("local barrier: a rank never arrived");
  }
  if (gen_ == gen) throw std::runtime_error("a peer rank failed");
}

void LocalGroup::abort() {
  std::lock_guard<std::mutex> lk(mu_);
  failed_ = true;
  cv_.notify_all();
}

std::vector<const void*> LocalTransport::exchange_ptr(const void* p, hipStream_t s) {
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");  // p's producer (the pack) is done
  g_.slot(rank_) = p;
  g_.barrier();
  std::vector<const void*> v(g_.world());
  for (int r = 0; r < g_.world(); ++r) v[r] = g_.slot(r);
  return v;
}

void LocalTransport::finish(hipStream_t s) {
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  g_.barrier();  // no rank reuses a buffer a peer may still be reading
}

void LocalTransport::all_to_all_slots(const uint8_t* send, uint8_t* recv, uint64_t sb, uint32_t rounds,
                                      hipStream_t s) {
  const int P = g_.world();
  if (P == 1) return;
  const std::vector<const void*> peer = exchange_ptr(send, s);
  for (int p = 0; p < P; ++p) {  // pull peer p's stream to this rank: its round t slot sits at (t P + me) sb
    if (p == rank_) continue;
    const uint8_t* src = static_cast<const uint8_t*>(peer[p]);
    for (uint32_t t = 0; t < rounds; ++t)
      hip_check(hipMemcpyAsync(recv + ((uint64_t)t * P + p) * sb, src + ((uint64_t)t * P + rank_) * sb, sb,
                               hipMemcpyDeviceToDevice, s),
                "slot copy");
  }
  finish(s);
}

void LocalTransport::all_to_all_u64(const uint64_t* send, uint64_t* recv, hipStream_t s) {
  const int P = g_.world();
  const std::vector<const void*> peer = exchange_ptr(send, s);
  for (int p = 0; p < P; ++p)
    hip_check(hipMemcpyAsync(recv + p, static_cast<const uint64_t*>(peer[p]) + rank_, sizeof(uint64_t),
                             hipMemcpyDeviceToDevice, s),
              "count copy");
  finish(s);
}

void LocalTransport::allreduce_max_u64(uint64_t* buf, size_t n, hipStream_t s) {
  const int P = g_.world();
  if (P == 1) return;
  const std::vector<const void*> peer = exchange_ptr(buf, s);
  std::vector<uint64_t*> ptrs(P);
  for (int r = 0; r < P; ++r) ptrs[r] = const_cast<uint64_t*>(static_cast<const uint64_t*>(peer[r]));
  // this rank reduces its slice of every array and writes the maximum to all of them
  local_max_u64(ptrs.data(), P, (uint64_t)n * rank_ / P, (uint64_t)n * (rank_ + 1) / P, s);
  finish(s);
}

void LocalTransport::allreduce_max_u8(uint8_t* buf, size_t n, hipStream_t s) {
  const int P = g_.world();
  if (P == 1) return;
  const std::vector<const void*> peer = exchange_ptr(buf, s);
  std::vector<uint8_t*> ptrs(P);
  for (int r = 0; r < P; ++r) ptrs[r] = const_cast<uint8_t*>(static_cast<const uint8_t*>(peer[r]));
  local_max_u8(ptrs.data(), P, (uint64_t)n * rank_ / P, (uint64_t)n * (rank_ + 1) / P, s);
  finish(s);
}

void LocalTransport::allreduce_max_f64(double* buf, size_t n, hipStream_t s) {
  const int P = g_.world();
  if (P == 1) return;
  std::vector<double> h(n);
  hip_check(hipMemcpyAsync(h.data(), buf, n * sizeof(double), hipMemcpyDeviceToHost, s), "D2H");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  for (size_t i = 0; i < n; ++i) {
    g_.scalars()[rank_] = h[i];
    g_.barrier();
    double m = g_.scalars()[0];
    for (int r = 1; r < P; ++r) m = std::max(m, g_.scalars()[r]);
    g_.barrier();
    h[i] = m;
  }
  hip_check(hipMemcpyAsync(buf, h.data(), n * sizeof(double), hipMemcpyHostToDevice, s), "H2D");
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
}

void LocalTransport::allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s) {
  const int P = g_.world();
  const std::vector<const void*> peer = exchange_ptr(send, s);
  for (int r = 0; r < P; ++r)
    hip_check(hipMemcpyAsync(recv + (size_t)r * n, peer[r], n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s),
              "allgather copy");
  finish(s);
}

void LocalTransport::barrier(hipStream_t s) {
  hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  g_.barrier();
}

void slot_geometry(uint64_t cap, int world, uint32_t rec, uint64_t chunk, uint64_t* slot, uint32_t* rounds) {
  // the probe tiles a slot by its divisors: large streams take whole 1024-record regions
  const uint64_t kAlign = cap >= 64 * 1024 ? 1024 : 64;
  const uint64_t per_round = std::max<uint64_t>(kAlign, (chunk / ((uint64_t)world * rec)) / kAlign * kAlign);
  const uint64_t want = std::max<uint64_t>(kAlign, (cap + kAlign - 1) / kAlign * kAlign);
  // the rounds share the stream evenly (sharded.py slot_geometry)
  *rounds = (uint32_t)((want + per_round - 1) / per_round);
  const uint64_t even = (want + *rounds - 1) / *rounds;
  *slot = (even + kAlign - 1) / kAlign * kAlign;
}

XchgStep::XchgStep(mg_ctx* ctx, Transport& x, uint32_t l, uint32_t k, uint64_t chunk)
    : ctx_(ctx), x_(x), l_(l), k_(k), chunk_(chunk), s_((hipStream_t)mg_stream(ctx)) {
  check(mg_xchg_caps(ctx_, l_, k_, caps_), "mg_xchg_caps");
  const char* mk = std::getenv("MG_XCHG_MARKS");
  use_marks_ = mk && mk[0] == '1';  // (off by default: DESIGN.md §6a, measured)
  const char* rr = std::getenv("MG_XCHG_ROUTE_ROWS");
  route_rows_ = rr && rr[0] == '1' && x.world() > 1;  // (off by default: rows held where verified)
  check(mg_set_option(ctx_, "xchg_route_rows", route_rows_ ? 1 : 0), "mg_set_option");
  hip_check(hipStreamCreateWithFlags(&s2_, hipStreamNonBlocking), "hipStreamCreate");
  hip_check(hipEventCreateWithFlags(&ev_packed_, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&ev_runs_, hipEventDisableTiming), "hipEventCreate");
}

XchgStep::~XchgStep() {
  for (Stream& st : st_)
    for (void* p : {(void*)st.send, (void*)st.recv, (void*)st.counts, (void*)st.rcounts})
      if (p) (void)hipFree(p);
  if (superkey_) (void)hipFree(superkey_);
  if (maxbuf_) (void)hipFree(maxbuf_);
  if (marks_) (void)hipFree(marks_);
  if (ev_packed_) (void)hipEventDestroy(ev_packed_);
  if (ev_runs_) (void)hipEventDestroy(ev_runs_);
  if (s2_) (void)hipStreamDestroy(s2_);
}

void XchgStep::scale_caps(double f) {
  for (uint64_t& c : caps_) c = std::max<uint64_t>(1, (uint64_t)((double)c * f));
}

void XchgStep::check(int rc, const char* what) {
  if (rc) throw std::runtime_error(std::string(what) + ": " + mg_last_error(ctx_));
}

void XchgStep::ensure(Stream& st, int kind) {
  const int P = x_.world();
  slot_geometry(caps_[kind], P, mg_record_bytes(kind), chunk_, &st.slot, &st.rounds);
  const size_t bytes = (size_t)st.rounds * P * st.slot * mg_record_bytes(kind);
  if (bytes > st.bytes) {
    for (uint8_t** p : {&st.send, &st.recv})
      if (*p) hip_check(hipFree(*p), "hipFree");
    st.send = st.recv = nullptr;
    hip_check(hipMalloc(&st.recv, bytes), "hipMalloc");
    if (P > 1) hip_check(hipMalloc(&st.send, bytes), "hipMalloc");
    st.bytes = bytes;
  }
  if (!st.counts) {
    hip_check(hipMalloc(&st.counts, P * sizeof(uint64_t)), "hipMalloc");
    hip_check(hipMalloc(&st.rcounts, P * sizeof(uint64_t)), "hipMalloc");
  }
}

// pack `kind` on the context's stream, then exchange it on stream s (s_ or the
// run exchange's s2_, which waits for the pack first)
void XchgStep::route(int kind, hipStream_t s) {
  Stream& st = st_[kind];
  if (x_.world() == 1) {  // one rank: nothing is packed (mg_xchg_pack at P = 1), the consumers read the context
    if (!st.counts) {
      hip_check(hipMalloc(&st.counts, sizeof(uint64_t)), "hipMalloc");
      hip_check(hipMalloc(&st.rcounts, sizeof(uint64_t)), "hipMalloc");
    }
    check(mg_xchg_pack(ctx_, kind, nullptr, 1, 1, st.counts, nullptr), "mg_xchg_pack");
    x_.all_to_all_u64(st.counts, st.rcounts, s_);
    return;
  }
  ensure(st, kind);
  check(mg_xchg_pack(ctx_, kind, st.send, st.slot, st.rounds, st.counts, st.recv), "mg_xchg_pack");
  if (s != s_) {
    hip_check(hipEventRecord(ev_packed_, s_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(s, ev_packed_, 0), "hipStreamWaitEvent");
  }
  x_.all_to_all_slots(st.send, st.recv, st.slot * mg_record_bytes(kind), st.rounds, s);
  x_.all_to_all_u64(st.counts, st.rcounts, s);
}

int XchgStep::run() {
  const int P = x_.world();
  for (int reruns = 0;; ++reruns) {
    if (reruns > 3) throw std::runtime_error("exchange capacities still overflow after 3 reruns");
    // 1. one scan of this rank's sources: index keys + bucket-sorted runs
    check(mg_xchg_begin(ctx_, l_, k_), "mg_xchg_begin");
    // 2. keys -> bucket owners; 3. runs -> bucket owners (both probes read
    // them) on the second stream, in flight while 4. the received keys are
    // sorted and filed into the local cells (HashTable::insertDataset)
    // (keys first, mg_xchg_keys_first: the runs come out of the window scan
    // inside mg_xchg_insert_keys, so they are packed after it)
    route(MG_KEYS, s_);
    const bool keys_first = mg_xchg_keys_first(ctx_) == 1;
    if (!keys_first) {
      route(MG_RUNS, P > 1 ? s2_ : s_);
      if (P > 1) hip_check(hipEventRecord(ev_runs_, s2_), "hipEventRecord");
    }
    const Stream& ks = st_[MG_KEYS];
    check(mg_xchg_insert_keys(ctx_, ks.recv, ks.slot, ks.rounds, ks.rcounts), "mg_xchg_insert_keys");
    if (keys_first) {
      route(MG_RUNS, P > 1 ? s2_ : s_);
      if (P > 1) hip_check(hipEventRecord(ev_runs_, s2_), "hipEventRecord");
    }
    const Stream& rs = st_[MG_RUNS];
    bool runs_in = P == 1;  // the peers' run streams have arrived (s_ waited for ev_runs_)
    auto wait_runs = [&]() {
      if (!runs_in) hip_check(hipStreamWaitEvent(s_, ev_runs_, 0), "hipStreamWaitEvent");
      runs_in = true;
    };
    // 4. markContainedReads (lengths differ, OverlapGraph.cpp:228-233): MAX of the keys over ranks
    const uint64_t n = mg_num_reads(ctx_);
    if (n > superkey_n_) {
      if (superkey_) hip_check(hipFree(superkey_), "hipFree");
      hip_check(hipMalloc(&superkey_, std::max<uint64_t>(n, 1) * sizeof(unsigned long long)), "hipMalloc");
      superkey_n_ = n;
    }
    int needed = 0;
    check(mg_begin_contained(ctx_, superkey_, &needed), "mg_begin_contained");
    contained_ = needed != 0;
    if (needed) wait_runs();  // (the containment probe reads every stream)
    if (needed && P > 1 && use_marks_) {
      // every rank's offset-0 containments first, their marks MAX-reduced: the
      // probe then skips the sources any rank found contained (contain_skip)
      if (n > marks_n_) {
        if (marks_) hip_check(hipFree(marks_), "hipFree");
        hip_check(hipMalloc(&marks_, std::max<uint64_t>(n, 1)), "hipMalloc");
        marks_n_ = n;
      }
      check(mg_xchg_prefix_marks(ctx_, marks_), "mg_xchg_prefix_marks");
      x_.allreduce_max_u8(marks_, n, s_);
    }
    if (needed) {
      check(mg_xchg_probe(ctx_, 1, rs.recv, rs.slot, rs.rounds, rs.rcounts), "mg_xchg_probe(contain)");
      x_.allreduce_max_u64(reinterpret_cast<uint64_t*>(superkey_), n, s_);
    }
    check(mg_finalize_contained(ctx_, nullptr), "mg_finalize_contained");
    // 5. insertAllEdgesOfRead: probe -> rows [-> src owners].  Equal lengths:
    // this rank's own stream (in rs.recv since the pack) first, while the
    // peers' streams are still on the links (a no-op otherwise)
    if (!runs_in)
      check(mg_xchg_probe_own(ctx_, rs.recv, rs.slot, rs.rounds, rs.counts), "mg_xchg_probe_own");
    wait_runs();
    check(mg_xchg_probe(ctx_, 0, rs.recv, rs.slot, rs.rounds, rs.rcounts), "mg_xchg_probe");
    const int nk = route_rows_ ? 3 : 2;  // the stream kinds that moved
    if (route_rows_) route(MG_ROWS, s_);
    // the step's one host read: the MAX over ranks of every per-peer send count
    std::vector<uint64_t> c(3 * P, 0);
    for (int kind = 0; kind < nk; ++kind)
      hip_check(hipMemcpyAsync(c.data() + kind * P, st_[kind].counts, P * sizeof(uint64_t), hipMemcpyDeviceToHost, s_),
                "counts D2H");
    std::vector<uint64_t> rc(P, 0);
    if (route_rows_)
      hip_check(hipMemcpyAsync(rc.data(), st_[MG_ROWS].rcounts, P * sizeof(uint64_t), hipMemcpyDeviceToHost, s_),
                "counts D2H");
    hip_check(hipStreamSynchronize(s_), "hipStreamSynchronize");
    uint64_t mx[3] = {0, 0, 0};
    for (int kind = 0; kind < 3; ++kind)
      for (int p = 0; p < P; ++p) mx[kind] = std::max(mx[kind], c[kind * P + p]);
    if (!maxbuf_) hip_check(hipMalloc(&maxbuf_, sizeof mx), "hipMalloc");
    uint64_t* dmx = maxbuf_;
    hip_check(hipMemcpyAsync(dmx, mx, sizeof mx, hipMemcpyHostToDevice, s_), "max H2D");
    x_.allreduce_max_u64(dmx, 3, s_);
    hip_check(hipMemcpyAsync(mx, dmx, sizeof mx, hipMemcpyDeviceToHost, s_), "max D2H");
    hip_check(hipStreamSynchronize(s_), "hipStreamSynchronize");
    // fit the capacities to what was sent (grow: rerun; shrink: less padding
    // on the links from the next step on), identically on every rank
    bool over = false;
    for (int kind = 0; kind < nk; ++kind) {
      if (mx[kind] > caps_[kind]) over = true;
      caps_[kind] = mx[kind] + mx[kind] * 6 / 100 + 64;  // (sharded.py XchgPlan.grow's margin)
    }
    rows_held_ = 0;
    for (int p = 0; p < P; ++p) rows_held_ += rc[p];
    if (!route_rows_) rows_held_ = mg_num_rows(ctx_);  // (the rows stay in the context)
    if (!over) return reruns;
  }
}

void XchgStep::rows_digest(uint64_t out[4]) {
  if (!route_rows_) {
    check(mg_rows_digest(ctx_, nullptr, 0, out), "mg_rows_digest");
    return;
  }
  const Stream& ws = st_[MG_ROWS];
  check(mg_slots_digest(ctx_, ws.recv, ws.slot, ws.rounds, ws.rcounts, out), "mg_slots_digest");
}

}  // namespace mg
