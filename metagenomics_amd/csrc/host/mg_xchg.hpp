// mg_xchg.hpp — the exchange mode driven from
// C++ over RCCL: one process per GPU, the same step as
// metagenomics_amd/sharded.py (bucket-range index, key / run / row streams in
// the slot layout of include/mg_overlap.h, MAX all-reduce of the containment
// keys), with the collectives issued by this host code on the context's own
// HIP stream.  Linked into the mg_overlap CLI (-xchg), not into libmgovl.so.
#ifndef MG_XCHG_HPP_
#define MG_XCHG_HPP_
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

#include "mg_overlap.h"

namespace mg {

// One RCCL communicator over the ranks of one node.  The unique id travels
// over TCP: rank 0 listens on addr:port and hands it to the others.
class RcclExchange {
 public:
  RcclExchange(int rank, int world, int device, const std::string& addr, int port);
  ~RcclExchange();
  int rank() const { return rank_; }
  int world() const { return world_; }
  // every peer's slot of every round (slot_bytes each) from send to recv;
  // this rank's own slots are already in recv (mg_xchg_pack's self_dst)
  void all_to_all_slots(const uint8_t* send, uint8_t* recv, uint64_t slot_bytes, uint32_t rounds, hipStream_t s);
  // recv[s] = what rank s sent to this rank (send[r] = what this rank sends to r)
  void all_to_all_u64(const uint64_t* send, uint64_t* recv, hipStream_t s);
  void allreduce_max_u64(uint64_t* buf, size_t n, hipStream_t s);
  void allreduce_max_f64(double* buf, size_t n, hipStream_t s);
  void allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s);
  // every rank's work on s done
  void barrier(hipStream_t s);

 private:
  int rank_, world_;
  ncclComm_t comm_ = nullptr;
  double* flag_ = nullptr;
};

// Slot geometry of one stream kind (sharded.py slot_geometry): slot records
// per peer per round (a multiple of 64) and the number of rounds for `cap`
// records, one round at most chunk_bytes per rank.
void slot_geometry(uint64_t cap, int world, uint32_t rec_bytes, uint64_t chunk_bytes, uint64_t* slot, uint32_t* rounds);

// One rank's exchange-mode step (HashTable::insertDataset + markContainedReads
// + insertAllEdgesOfRead, distributed): buffers and the stream capacities
// (identical on every rank, grown after an overflow) persist from step to step.
class XchgStep {
 public:
  XchgStep(mg_ctx* ctx, RcclExchange& x, uint32_t min_overlap, uint32_t seed_k, uint64_t chunk_bytes = 256ull << 20);
  ~XchgStep();
  // runs the step (rerun with grown capacities after an overflow); rows owned
  // by this rank (by src ID) stay in the rows receive buffer.  Returns the
  // number of reruns; throws std::runtime_error on a library error.
  int run();
  uint64_t rows_held() const { return rows_held_; }
  // digest (mg_rows_digest formula) of this rank's rows
  void rows_digest(uint64_t out[4]);
  bool contained() const { return contained_; }

 private:
  struct Stream {
    uint8_t* send = nullptr;
    uint8_t* recv = nullptr;
    uint64_t* counts = nullptr;   // device: per-peer send counts
    uint64_t* rcounts = nullptr;  // device: per-peer receive counts
    size_t bytes = 0;
    uint64_t slot = 0;
    uint32_t rounds = 0;
  };
  void route(int kind);
  void ensure(Stream& st, int kind);
  void check(int rc, const char* what);
  mg_ctx* ctx_;
  RcclExchange& x_;
  uint32_t l_, k_;
  uint64_t chunk_;
  hipStream_t s_;
  uint64_t caps_[3];
  Stream st_[3];
  unsigned long long* superkey_ = nullptr;
  size_t superkey_n_ = 0;
  uint64_t* maxbuf_ = nullptr;  // the three stream maxima, all-reduced
  uint64_t rows_held_ = 0;
  bool contained_ = false;
};

}  // namespace mg
#endif  // MG_XCHG_HPP_
