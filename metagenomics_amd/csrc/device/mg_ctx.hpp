// mg_ctx.hpp — INTERNAL: the device context behind include/mg_overlap.h,
// shared by the kernel translation units (mg_kernels.hip: index + discovery +
// exchange; mg_dataset.hip: Dataset ingest on the device).
#ifndef MG_CTX_HPP_
#define MG_CTX_HPP_
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "mg_overlap.h"

// Device slot of a read: a power-of-two number of words (W = 5 -> 8 words, one
// aligned 64-B sector), so a partner fetch never straddles two sectors.
__host__ __device__ constexpr int slot_words(int w) {
  return w <= 1 ? 1 : w <= 2 ? 2 : w <= 4 ? 4 : w <= 8 ? 8 : w <= 16 ? 16 : 32;
}

struct mg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // reads
  uint64_t n = 0;
  uint32_t maxw = 0;
  uint32_t stride = 0;  // words per device slot (slot_words(maxw))
  uint32_t minlen = 0, maxlen = 0;
  uint64_t* d_words = nullptr;
  uint16_t* d_len = nullptr;
  size_t words_cap = 0, len_cap = 0;
  // device layout (option "layout"): slots clustered by each
  // read's canonical global minimizer, so overlapping reads sit near each
  // other; d_id[slot] = reference ID - 1, d_phys[ID - 1] = slot (both nullptr:
  // slots in ID order).  Everything on the device works in slots; rows,
  // superReadIDs, lookups and downloads leave in reference IDs.  With a
  // source-read range set (mg_set_shard), the reads of the range take the
  // slots [read_lo, read_hi) (clustered among themselves), so a shard's slot
  // range holds exactly its reference IDs.
  bool layout = true;
  int layout_hash = 0;  // option "layout_hash": the layout's 16-mer hash (0 fmix32, 1 24-bit multiply-adds)
  uint32_t* d_id = nullptr;    // one of id_store[], or nullptr
  uint32_t* d_phys = nullptr;  // one of phys_store[], or nullptr
  uint32_t* id_store[2] = {nullptr, nullptr};  // a re-layout builds the maps in the unused pair
  uint32_t* phys_store[2] = {nullptr, nullptr};
  size_t id_cap[2] = {0, 0}, phys_cap[2] = {0, 0};
  uint64_t layout_lo = 0, layout_hi = 0;  // the source-read range the current layout groups (0, 0: none)
  // layout scratch, kept between uploads so a re-upload allocates nothing:
  // sort keys / values (double buffers), the sort's temporary storage, and the
  // second slot array the gather writes (the two slot arrays swap)
  uint64_t* d_lay_k[2] = {nullptr, nullptr};
  uint32_t* d_lay_v[2] = {nullptr, nullptr};
  size_t lay_k_cap[2] = {0, 0}, lay_v_cap[2] = {0, 0};
  void* d_lay_tmp = nullptr;
  size_t lay_tmp_cap = 0;
  uint64_t* d_words_alt = nullptr;
  size_t words_alt_cap = 0;
  uint16_t* d_len_alt = nullptr;
  size_t len_alt_cap = 0;
  uint32_t* d_tmp32 = nullptr;  // ID-order staging of per-read outputs
  size_t tmp32_cap = 0;
  // index
  uint32_t l = 0, h = 0, m = 0, w = 0;
  uint32_t nb_log2 = 0, nb_log2_opt = 0;
  bool index_ready = false;
  uint64_t* d_cells = nullptr;  // cells of kCell entries (this rank's bucket range)
  size_t cells_cap = 0;
  // option "cells_double" (default off): a second table, cleared on the side
  // stream for the next build (cells_alt_clean entries, done at ev[13]).
  // Measured: the clear beside the scan slowed the scan more than the clear
  // costs (C3 scan 2.22 -> 2.72 ms, step 6.91 -> 7.26; profiles/r06s_ab_cells_double.txt)
  uint64_t* d_cells_alt = nullptr;
  size_t cells_alt_cap = 0;
  size_t cells_alt_clean = 0;
  bool cells_double = false;
  // the index holds the o = 1 keys (suffix keys of the forward strand) only
  // when a probe reads them: discovery never does (an o = 1 hit is the twin of
  // the partner's o = 0 hit) and containment only without the
  // prefix-containment kernel; getListOfReads then takes a lookup table of all
  // four keys, built on the first lookup after a build (d_lkcells)
  bool index_o1 = true;
  // the o = 3 keys likewise (fused mixed lengths with k_prefix_contain and the
  // live discovery index: containment drops o = 1/3 hits, discovery walks the
  // live table, which has them)
  bool index_o3 = true;
  uint64_t* d_lkcells = nullptr;
  size_t lkcells_cap = 0;
  bool lookup_ready = false;
  uint64_t cell_lo = 0, cell_n = 0;  // local bucket range [cell_lo, cell_lo + cell_n)
  // containment
  unsigned long long* d_superkey = nullptr;
  unsigned long long* superkey = nullptr;  // the containment key array in use (d_superkey or caller-owned)
  uint32_t* d_super = nullptr;
  // contained slots as a bitmap (bit a of word a / 32 = d_super[a] != 0,
  // k_super_finalize): the discovery probe drops contained partners before
  // they take a verification (:548), from a 1/32-size array that stays in cache
  uint32_t* d_cbits = nullptr;
  size_t cbits_cap = 0;
  // contained reads counted by k_super_finalize (64 counters, one per 64-B line)
  unsigned int* d_ccnt = nullptr;
  uint64_t n_contained = 0;
  // discovery index (option "live_index", unsharded fused path, mixed lengths):
  // after markContainedReads the discovery probe only needs the keys of
  // uncontained reads (:548 drops contained partners), so it probes a table of
  // those alone, sized for them (C5: a quarter of the entries and chains)
  bool live_index = true;
  bool live_runs = true;          // option live_runs: k_live_runs compacts the runs of contained sources before discovery
  // option live_overlap: k_live_runs (HBM streaming) on a side stream beside the
  // live index build (memory-side atomics), both before the discovery probe
  bool live_overlap = true;
  hipStream_t side = nullptr;
  bool live_ready = false;
  uint64_t* d_lcells = nullptr;
  size_t lcells_cap = 0;
  uint32_t lnb_log2 = 0;
  uint64_t live_cells = 0;  // cells of the discovery index (mg_counters::live_cells)
  unsigned int* d_any = nullptr;
  unsigned long long* d_digest = nullptr;  // mg_rows_digest / mg_super_digest accumulators (4 u64)
  size_t super_cap = 0, superkey_cap = 0;
  bool contained_done = false, super_any = false;
  // rows
  uint32_t* d_rows = nullptr;
  uint64_t rows_cap = 0, rows_cap_opt = 0;
  unsigned long long* d_seg = nullptr;
  uint64_t n_rows = 0;
  std::vector<unsigned long long> seg_host;
  uint64_t seg_cap_regions = 0;
  bool stats = false;
  unsigned long long* d_stats = nullptr;
  mg_counters counters{};
  // shard
  uint32_t rank = 0, nranks = 1;
  uint64_t read_lo = 0, read_hi = 0;  // source-read range: reference IDs - 1 = slots [read_lo, read_hi)
  uint32_t max_blocks = 8192;  // cap on the persistent discovery grid (blocks of 4 wavefronts)
  int phase_limit = 99;        // diagnostics (option "phase_limit")
  int contain_phase_limit = 99;  // diagnostics (option "contain_phase_limit")
  bool halving_low = false;    // option "halving": o=2/3 pair side rule
  int n_cu = 256;              // compute units of the device
  uint64_t nreg = 0;           // row regions of the last discovery launch (one per probe wavefront)
  uint64_t nrun_reg = 0;       // run regions (one per scan wavefront)
  ulonglong2* d_runs = nullptr;  // run records, one region per wavefront
  size_t runs_cap = 0;
  uint64_t run_cap = 0, run_cap_need = 0, run_cap_opt = 0;  // run_cap_opt: option "run_cap" (tests)
  unsigned long long* d_run_cnt = nullptr;
  size_t run_cnt_cap = 0;
  std::vector<unsigned long long> run_cnt_host;
  uint32_t* d_compact = nullptr;
  size_t compact_cap = 0;
  // exchange mode (one process per GPU): mg_xchg_begin's scan
  // leaves key records (d_kb / d_ke) and the run regions of this rank's
  // sources; packable = bit mask of what mg_xchg_pack can route now
  bool xchg = false;                     // the context's current build is an exchange-mode build
  // one rank (P = 1, no source range): mg_xchg_begin runs the fused build and
  // the exchange calls delegate to the fused probes (option "xchg_fused1")
  bool xchg_fused = false;
  bool xchg_fused1 = true;
  bool index_keys = true;  // option "index_keys": LaunchIndex takes k_index_keys (0: k_index_build)
  // mg_xchg_prefix_marks ran this step's offset-0 containments; xmarks = the
  // caller's marks (all-reduced before mg_xchg_probe(1) folds them in)
  uint64_t scan_runs = 0;  // run records of the last window scan (settle_runs)
  bool xmarks_done = false;
  uint8_t* xmarks = nullptr;
  uint64_t xchg_lo = 0, xchg_hi = 0;     // its source reads
  unsigned long long* d_blk = nullptr;   // routing: per-(block, rank) counts / offsets
  size_t blk_cap = 0;
  // exchange mode, equal lengths: the register scan counts its runs per
  // destination rank (one row of nranks per run region), so routing the runs
  // skips k_part's count pass (runs_counted: valid for the last scan)
  unsigned long long* d_rcnt = nullptr;
  size_t rcnt_cap = 0;
  // k_xchg_keys' per-(flat region, rank) counts of the key records (keys first):
  // mg_xchg_pack(MG_KEYS) skips k_part's count pass while keys_counted
  // the keys-first receiver scan's run regions hold 8-B metas, d_rdst their owner ranks
  uint8_t* d_rdst = nullptr;
  size_t rdst_cap = 0;
  bool runs_meta8 = false;
  uint64_t super_zero_n = 0;  // leading d_super entries known to be 0 (skips the equal-length clear)
  unsigned long long* d_kblk = nullptr;
  size_t kblk_cap = 0;
  bool keys_counted = false;
  bool runs_counted = false;
  // mg_build_index leaves its timings (index_ms, shared_scan_ms) to be read once
  // its events have completed (settle_index_times): no host round trip between
  // the build and the probe
  bool index_times_pending = false;
  // exchange-mode discovery probe: rows per (probe wavefront, destination
  // rank), so routing the rows skips k_part's count pass (rows_counted)
  unsigned long long* d_dcnt = nullptr;
  size_t dcnt_cap = 0;
  bool rows_counted = false;
  // option "xchg_route_rows" (default 1): the exchange-mode discovery probe
  // counts its rows per src owner for mg_xchg_pack(MG_ROWS); a host that keeps
  // the rows where they were verified sets 0 and the probe counts nothing
  bool xchg_route_rows = true;
  // option "xchg_scan_lds": the exchange scan of equal lengths takes k_scan<KEYREC>
  // (LDS sliding minimum, all four keys in one pass) instead of k_scan_reg + k_rc_keys
  bool xchg_scan_lds = true;
  uint32_t xchg_region = 512;  // option "xchg_region": records per probe region of the received runs (0: 1,024)
  uint32_t xchg_split_max = 4;  // option "xchg_split_max": mg_xchg_probe_own splits the probe at up to this many ranks
  int packable = 0;                      // 1 << MG_KEYS | 1 << MG_RUNS | 1 << MG_ROWS
  unsigned long long* d_flat_cnt = nullptr;  // per-region counts of the received runs (probe input)
  size_t flat_cnt_cap = 0;
  unsigned long long* d_slot_cnt = nullptr;  // per-region counts of a slot-layout buffer (digest)
  size_t slot_cnt_cap = 0;
  uint32_t* d_kb = nullptr;  // key records: bucket / index entry, key o of read a at o * n + a
  uint64_t* d_ke = nullptr;
  size_t kb_cap = 0, ke_cap = 0;
  // timing
  hipEvent_t ev[16] = {};  // [14], [15]: apply_layout
  // unsharded contexts build the index inside the window scan (k_scan<INDEX>);
  // its runs then serve the containment and the discovery probes
  int scan_state = 0;        // 0 none, 1 launched (not settled), 2 settled
  bool runs_live = false;    // the run regions hold only runs of uncontained sources (k_live_runs)
  bool probe_share = true;     // option "probe_share": a discovery-probe block's 4 wavefronts share its regions
  bool probe_compact = true;   // option "probe_compact": sparse run batches compacted in the probe (C5 probe 30.4 -> 26.8 ms)
  // prefix containments (k_prefix_contain): each read's o = 0 key (bucket,
  // fingerprint, q) written by k_scan<INDEX> for mixed-length sets; when ready
  // the containment probe skips suffix-key hits (containment)
  uint64_t* d_key0 = nullptr;
  size_t key0_cap = 0;
  // offset-0 containments through the containment probe (option prefix_probe,
  // default): the fused scan writes each read's window-0 run (its o = 0 key's
  // minimizer, window range [0, 0]) here, one 16-B record per slot, and the
  // probe takes them first in fixed regions of d_p0cnt records
  bool prefix_probe = true;
  ulonglong2* d_p0runs = nullptr;
  size_t p0runs_cap = 0;
  unsigned long long* d_p0cnt = nullptr;
  size_t p0cnt_cap = 0;
  // exchange mode: the received runs ordered by local bucket (sort_xruns), the
  // input of both probes; xruns_ready until the next mg_xchg_begin
  uint32_t* d_xk[2] = {nullptr, nullptr};
  ulonglong2* d_xv[2] = {nullptr, nullptr};
  size_t xk_cap[2] = {0, 0}, xv_cap[2] = {0, 0};
  void* d_xsort_tmp = nullptr;
  size_t xsort_tmp_cap = 0;
  int xv_sel = 0;
  uint64_t xruns_n = 0;
  bool own_probed = false;
  // exchange mode, keys first (option xchg_keys_first, equal lengths, P > 1):
  // mg_xchg_begin computes the key records only (k_xchg_keys); the window scan
  // runs in mg_xchg_insert_keys and CAS-inserts the received key records
  // (rk_*: slot layout) as it goes (k_scan<RECV>, rk_on during that launch)
  bool xchg_keys_first = true;
  bool keys_first = false;  // the current exchange build is a keys-first one
  bool rk_on = false;
  const uint64_t* rk_keys = nullptr;
  const unsigned long long* rk_cnt = nullptr;
  uint64_t rk_slot = 0, rk_total = 0;
  int xruns_part = 0;       // the probe regions prepared: 0 all, 1 own stream, 2 the peers' (split probe)
  uint64_t xruns_K = 0;     // probe regions per peer slot and round  // mg_xchg_probe_own probed this rank's own stream; mg_xchg_probe(0) appends the peers
  // the received runs expanded to 16-B probe records (k_xruns_expand), slot layout
  ulonglong2* d_xexp = nullptr;
  size_t xexp_cap = 0;
  bool xruns_ready = false;
  ulonglong2* xruns_base = nullptr;  // the probes' run regions: d_xv (sorted), the receive buffer, or (one rank) d_runs
  unsigned long long* xruns_cnt = nullptr;  // their per-region counts
  uint64_t xruns_reg = 0, xruns_nreg = 0;
  // exchange mode: the key records this rank received, dense and sorted by
  // home cell (mg_xchg_insert_keys: key = local home cell, ent = index
  // entry); they build the cells, the o = 0 ones drive the prefix containments
  // (k_prefix_contain_keys, xchg_prefix) and the live ones the discovery index
  uint32_t* d_xkk[2] = {nullptr, nullptr};
  uint64_t* d_xke[2] = {nullptr, nullptr};
  size_t xkk_cap[2] = {0, 0}, xke_cap[2] = {0, 0};
  uint64_t xkeys_n = 0;
  uint32_t xkey_cls = 0;       // 1: key = home cell << 1 | (o == 3) (the full table leaves out o = 3)
  uint32_t xkey_fs = 0;        // low fingerprint bits below the cell / class bits (chain_par)
  bool xkey_par = false;       // the received records' cells are built by the parallel placement
  uint32_t* xkey_k = nullptr;  // the sorted records (one of d_xkk[] / d_kb) and the other buffer pair
  uint64_t* xkey_e = nullptr;
  uint32_t* xkey_k_alt = nullptr;
  uint64_t* xkey_e_alt = nullptr;
  // the live records' in-order compaction (build_live_index_xchg)
  uint8_t* d_xflag = nullptr;
  size_t xflag_cap = 0;
  unsigned long long* d_nlive = nullptr;
  // the exchange mode's discovery index coarsens the rank's cells (cell =
  // local home cell >> live_shift) instead of rebuilding entries
  bool live_coarse = false;
  uint32_t live_shift = 0;
  bool xchg_sort_runs = false;  // option "xchg_sort_runs": received runs ordered by bucket before the probes
  bool xchg_windows = true;    // option "xchg_windows": the exchange scan of mixed lengths in length-ranked windows
  bool layout_scratch = true;  // option "layout_scratch" = 0: free the layout's double buffers after each layout
  // option "chain_par": build_cells places a cell's overflow records in
  // parallel by their index in their fingerprint's run (k_cells_place; else one
  // thread per overflowing cell, k_cells_chain); d_rhead / d_rstart: run heads
  // and their max-scan
  bool chain_par = true;
  bool check_cells = false;  // diagnostics (option "check_cells"): verify each sorted cell build
  int xchg_fs = -1;  // diagnostics (option "xchg_fs"): fingerprint bits in the exchange sort key (-1: fp_sort_bits)
  uint32_t* d_rhead = nullptr;
  uint32_t* d_rstart = nullptr;
  size_t rhead_cap = 0, rstart_cap = 0;
  bool xchg_prefix = false;
  bool key0_ready = false;
  bool prefix_contain = true;  // option "prefix_contain"
  bool contain_jcut = true;    // option "contain_jcut": containment probe drops runs with jlo > n1 - minlen (C5: 60 -> 47 ms)
  bool contain_skip = true;    // option "contain_skip": skip runs of sources already known contained (C5: 42.8 -> 29.7 ms)
  uint32_t probe_split_max = 8;  // option "probe_split_max": virtual run regions per region for the probe's balance (1 = off)
  bool contain_prune = true;   // option "contain_prune": skip candidates that cannot raise the superkey (C5: 388M -> 110M compares)
  float shared_scan_ms = 0.f;  // k_scan<INDEX> kernel time of the last mg_build_index
  mg_timings t{};
  // Dataset ingest on the device (mg_ingest_*): frequency of each unique read
  uint32_t* d_freq = nullptr;
  size_t freq_cap = 0;
  uint64_t n_good = 0;  // reads that passed testRead (Dataset::getNumberOfReads)
  // option "alloc_cap" (tests): a device allocation above this many bytes fails
  // as out of memory (0 = no cap), so the error path is exercised on purpose
  uint64_t alloc_cap = 0;
};

#define MG_TRY(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ctx->err = std::string(#expr) + " failed: " + hipGetErrorString(e_);            \
      return -1;                                                                      \
    }                                                                                 \
  } while (0)

inline int set_err(mg_ctx* ctx, const std::string& s) {
  ctx->err = s;
  return -1;
}

// Every device buffer of a context is allocated here.  A failure -- or, with
// option "alloc_cap" (tests), a request above that many bytes, reported as
// out of memory -- leaves the buffer's name, the bytes asked for and the HIP
// error in ctx->err, so no later message has to guess the cause.
inline hipError_t ctx_malloc(mg_ctx* ctx, void** p, size_t bytes, const char* what) {
  *p = nullptr;
  const hipError_t e =
      (ctx->alloc_cap && bytes > ctx->alloc_cap) ? hipErrorOutOfMemory : hipMalloc(p, std::max<size_t>(bytes, 1));
  if (e != hipSuccess) {
    *p = nullptr;
    ctx->err = std::string("device allocation of ") + what + " (" + std::to_string(bytes) + " B) failed: " +
               hipGetErrorString(e) + (ctx->alloc_cap && bytes > ctx->alloc_cap ? " (option alloc_cap)" : "");
  }
  return e;
}

// grow *p to at least `count` elements (contents not kept)
template <typename T>
inline hipError_t ensure(mg_ctx* ctx, T** p, size_t* cap, size_t count, const char* what) {
  if (*cap >= count && *p) return hipSuccess;
  if (*p) {
    hipError_t e = hipFree(*p);
    if (e != hipSuccess) return e;
    *p = nullptr;
    *cap = 0;
  }
  const size_t c = std::max<size_t>(count, 1);
  hipError_t e = ctx_malloc(ctx, reinterpret_cast<void**>(p), c * sizeof(T), what);
  if (e == hipSuccess) *cap = c;
  return e;
}
// ensure() of a context field; returns -1 from the caller with ctx->err set
#define MG_ENSURE(field, capf, count)                                                            \
  do {                                                                                          \
    if (ensure(ctx, &ctx->field, &ctx->capf, (count), #field) != hipSuccess) return -1;         \
  } while (0)
// a launch wrapper that failed: keep the cause a callee left in ctx->err
inline int launch_fail(mg_ctx* ctx, const std::string& what) {
  ctx->err = ctx->err.empty() ? what : what + ": " + ctx->err;
  return -1;
}

// word counts the kernels are instantiated for (reads up to 1024 bp)
inline uint32_t supported_maxw(uint32_t need) {
  static const uint32_t kW[] = {1, 2, 3, 4, 5, 6, 8, 12, 16, 32};
  for (uint32_t w : kW)
    if (w >= need) return w;
  return 0;
}

// Reads longer than 1024 bp (up to 65,535, Read.h:62) take the long-read
// kernels (mg_kernels.hip: k_index_long, k_probe_long): maxw is then the exact
// word count and a slot holds it plus at least one zero pad word.
inline bool long_mode(const mg_ctx* ctx) { return ctx->maxw > 32; }
inline uint32_t long_stride(uint32_t maxw) { return (maxw + 1 + 7) & ~7u; }
// slot width for reads of `need` words: the instantiated widths up to 32,
// else the long-read width (maxw = need); 0 = longer than 65,535 bp
inline uint32_t slot_maxw(uint32_t need) {
  if (need <= 32) return supported_maxw(need < 1 ? 1 : need);
  return need <= 2048 ? need : 0;
}
inline uint32_t slot_stride(uint32_t maxw) { return maxw > 32 ? long_stride(maxw) : (uint32_t)slot_words((int)maxw); }

// the device layout of freshly uploaded reads (mg_kernels.hip): clusters the
// slots by canonical global minimizer and fills d_id / d_phys (option "layout"
// = 0: ID order); records t.layout_ms
int apply_layout(mg_ctx* ctx);

// new reads invalidate everything derived from them
inline void reset_derived(mg_ctx* ctx) {
  ctx->scan_state = 0;
  ctx->index_ready = false;
  ctx->lookup_ready = false;
  ctx->contained_done = false;
  ctx->super_any = false;
  ctx->live_ready = false;
  ctx->live_coarse = false;
  ctx->n_contained = 0;
  ctx->n_rows = 0;
}

#endif  // MG_CTX_HPP_
