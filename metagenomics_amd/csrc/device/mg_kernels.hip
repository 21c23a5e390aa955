// mg_kernels.hip — CDNA4 (gfx950) kernels for the read-overlap hot path.
//
// Reference path replaced (paths relative to /root/reference/MetaGenomics):
//   Read::setRead / reverseComplement          Read.cpp:75-82,115-127   -> k_pack_ascii, rc_word
//   HashTable::insertDataset/hashRead/insert   HashTable.cpp:50-195     -> k_index_build
//   HashTable::getListOfReads                  HashTable.cpp:202-221    -> cell probe inside k_probe, k_lookup_key
//   OverlapGraph::markContainedReads           OverlapGraph.cpp:225-340 -> k_scan + k_probe<CONTAIN=true> + k_super_finalize
//   OverlapGraph::insertAllEdgesOfRead         OverlapGraph.cpp:529-565 -> k_scan + k_probe<CONTAIN=false>
//   OverlapGraph::checkOverlap / insertEdge    OverlapGraph.cpp:354-419 -> verify + emit inside k_probe
//
// Design:
//  * reads: AoS 2-bit words (A0 C1 G2 T3, MSB-first) in power-of-two slots
//    (150 bp -> one aligned 64-B sector); the reverse strand is never stored,
//    it is derived in registers (rc_word).
//  * index: every key (the h = l-1 prefix/suffix of both strands, 4 per read)
//    is filed under its m-mer minimizer (m = seed k) in a cell table (8 entries
//    per 64-B cell, CAS insert, cell-granular linear probing).  A read's
//    window j matches key K exactly only if both share the minimizer at the
//    same relative offset q, so each exact-key hit of the reference is found
//    once, from the run of windows that share that minimizer; every candidate
//    is then verified over the full overlap, so results are exact.
//  * discovery = k_scan (one lane per source read: rolling m-mers, van Herk
//    sliding minimum, one 16-B record per minimizer run) + k_probe (one run
//    per lane: cell load, fingerprint/offset filter, wavefront prefix-sum
//    compaction into an LDS candidate list, one candidate per lane verified
//    against the partner's slot, ballot-compacted rows into a per-wavefront
//    HBM region).
//  * only half of the symmetric discoveries are verified: o = 1 hits are the
//    twins of the partner's o = 0 hits, an o = 2/3 pair is kept on one side
//    (rc_side_keeps); every verified discovery emits its row and its twin
//    (DESIGN.md §4 proves this reproduces the reference multiset).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "mg_ctx.hpp"
#include "mg_overlap.h"

// two window steps per loop trip in the scan (A/B builds: -DMG_SCAN_UNROLL=2).
// Measured: C3 scan level (2.19-2.21 vs 2.21-2.23 ms), C5 -0.14 ms of 15.8
// (profiles/r06v_ab_scan_unroll2.txt): the step is not bound by its loop control
#ifndef MG_SCAN_UNROLL
#define MG_SCAN_UNROLL 1
#endif

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kSegs = 64;                   // diagnostic counter shards
constexpr uint32_t kFpBits = 9;

// ---------------------------------------------------------------- helpers ---
// Invertible 64-bit mixer: x -> minimizer order and bucket.  Bijective, so
// equal hash <=> equal m-mer.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ULL;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dULL;
  x ^= x >> 33;
  return x;
}

// Minimizer order of an m-mer: a cheap 32-bit hash truncated to 22 bits and
// packed with the m-mer's position (< 1024), so that "smallest key, leftmost
// on ties" is a plain unsigned min.  Index build, discovery and lookup all
// use this same rule, so a key and an identical read window always select
// the same minimizer at the same offset.
// Two rounds of 24-bit multiply-add (v_mad_u32_u24, full rate; a 32-bit
// v_mul_lo_u32 is not) with xor-shifts; the bits a 24-bit product drops come
// back through the added shift.
__device__ __forceinline__ uint32_t order_key(uint64_t mm) {
  const uint32_t lo = (uint32_t)mm, hi = (uint32_t)(mm >> 32);
  uint32_t x = __umul24(lo, 0x9E3779u) + (hi ^ (lo >> 8));
  x ^= x >> 15;
  x = __umul24(x, 0xEBCA77u) + (x >> 8);
  x ^= x >> 13;
  return x & 0xFFFFFC00u;  // 22-bit key in the high bits, position goes in the low 10
}

// Reverse complement of 32 packed bases (Read.cpp:115-127 on 2-bit codes:
// complement = 3 - b = ~b, then reverse the 2-bit groups).
__device__ __forceinline__ uint64_t rc_word(uint64_t x) {
  x = __builtin_bitreverse64(~x);
  return ((x >> 1) & 0x5555555555555555ULL) | ((x & 0x5555555555555555ULL) << 1);
}

__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, int s) {
  return s ? (lo << s) | (hi >> (64 - s)) : lo;
}

// 32 bases starting at `pos` of a packed string stored with word stride S
// (pos >= -31; bases before 0 read as 0).
template <int S>
__device__ __forceinline__ uint64_t ext_fwd(const uint64_t* f, int pos) {
  if (pos < 0) return f[0] >> (-pos * 2);
  const int w = pos >> 5, s = (pos & 31) << 1;
  return funnel(f[w * S], f[(w + 1) * S], s);
}

// 32 bases of a read's slot in HBM starting at base pos (no read past the
// slot's last word)
template <int MAXW>
__device__ __forceinline__ uint64_t ext_slot(const uint64_t* g, int pos) {
  const int wi = pos >> 5;
  return funnel(g[wi], wi + 1 < slot_words(MAXW) ? g[wi + 1] : 0ull, (pos & 31) << 1);
}


// Reference ID - 1 of the read in slot x of the device layout (mg_ctx::d_id:
// reads are stored clustered for locality; nullptr = ID order).
__device__ __forceinline__ uint32_t rid(const uint32_t* id, uint32_t x) { return id ? id[x] : x; }
// Number of set bits of a ballot below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ uint32_t lane_prefix(uint64_t bal) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

// ------------------------------------------------------------ 2-bit pack ---
// One thread per (read, word): ASCII ACGT -> 2-bit codes, MSB-first.
// code = ((c >> 1) ^ (c >> 2)) & 3 maps A,C,G,T (0x41,0x43,0x47,0x54) to 0..3.
__global__ __launch_bounds__(kBlock) void k_pack_ascii(const char* __restrict__ ascii,
                                                      const uint64_t* __restrict__ off, uint64_t n,
                                                      uint32_t maxw, uint32_t stride, uint64_t* __restrict__ words,
                                                      uint16_t* __restrict__ len) {
  const uint64_t idx = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (idx >= n * maxw) return;
  const uint64_t r = idx / maxw;
  const uint32_t k = (uint32_t)(idx - r * maxw);
  const uint64_t s = off[r];
  const int64_t L = (int64_t)(off[r + 1] - s);
  if (k == 0) len[r] = (uint16_t)L;
  uint64_t wd = 0;
  const int64_t p0 = 32 * (int64_t)k;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    const int64_t pos = p0 + i;
    uint32_t code = 0;
    if (pos < L) {
      const uint32_t c = (uint8_t)ascii[s + pos];
      code = ((c >> 1) ^ (c >> 2)) & 3u;
    }
    wd = (wd << 2) | code;
  }
  words[r * stride + k] = wd;
}

// ------------------------------------------------------------ index build ---
// Cell index (replaces HashTable's vector-of-lists, HashTable.h:20): 2^nb_log2
// cells of kCell entries (one 64-B line each) plus a u32 fill count per cell.
// An entry goes to the first cell of its minimizer's home cell chain that has
// room (cell-granular linear probing), so a lookup reads the home cell's count
// and line together and follows the chain only while count > kCell.
// s_waitcnt immediate of gfx9/CDNA: vmcnt(0), expcnt and lgkmcnt not waited for
constexpr int kWaitVm0 = 0x0F70;
constexpr int kCell = 8;
// staged run metas per scan wavefront: a put finds fewer than 64 staged (every
// step flushes at 64), so valid metas stay below 128 and [128, 192) takes the
// stores of the lanes that put nothing (k_scan's put: one unconditional store)
constexpr int kScanBuf = 3 * 64;
// k_scan keeps a +inf sentinel in key slot w of each lane (the window that is
// exactly the current block reads it as its previous-block suffix)
constexpr int kScanKeyPad = 1;
// k_scan<..., G> takes its reads in windows of G groups of 64 consecutive
// slots, one pass of 64 reads of similar length at a time (longest first); the
// runs of group j of a window go to the wavefront's run region j (G regions
// per wave).  G = kWinGroups for the fused index scan of mixed lengths, 1
// (one group, no sort) otherwise.
#ifndef MG_WIN_GROUPS
#define MG_WIN_GROUPS 4  // (A/B and diagnostics builds override)
#endif
constexpr int kWinGroups = MG_WIN_GROUPS;
constexpr int kStageRing = 512;   // register scan: LDS ring of staged run metas per wavefront
constexpr uint64_t kEmpty = ~0ULL;       // free slot (a read index is never 0xFFFFFFFF)
constexpr uint64_t kChain = 1ULL << 63;  // on a cell's last slot: the chain continues in the next cell
constexpr uint32_t kFpMask = (1u << kFpBits) - 1;
constexpr uint64_t kFlatHole = ~0ULL;  // meta of a dead run record (a run meta never has bit 63)

struct IndexParams {
  const uint64_t* words;
  const uint16_t* len;
  uint64_t n;
  int h, m, w;
  uint32_t nb_log2;
  uint32_t rank, nranks;
  uint64_t cell_lo, cell_n;  // this rank's bucket range [cell_lo, cell_lo + cell_n): local cell = bucket - cell_lo
  uint64_t* cells;   // [cell_n * kCell] entries: lo32 = read index, hi32 = chain1 | len10 | fp9 | q10 | o2 (make_entry)
  const uint32_t* id;  // slot -> reference ID - 1 (nullptr: ID order; lookups return IDs)
  uint32_t stride;     // words per slot (the long-read kernels; the templated ones use slot_words(MAXW))
  const uint32_t* cbits;  // k_index_live: the contained slots (bitmap, k_super_finalize)
  int skip_o1;         // leave out the o = 1 keys (index_o1: nothing on this path reads them)
};

__device__ __forceinline__ bool owned(uint64_t bkt, uint32_t nb_log2, uint32_t rank, uint32_t nranks) {
  return nranks <= 1 || (uint32_t)((bkt * nranks) >> nb_log2) == rank;
}

// Minimizer of key o of a read (hashRead, HashTable.cpp:88-104): o=0 F[0,h),
// o=1 F[n-h,n), o=2 R[0,h), o=3 R[n-h,n); the m-mer at key offset i is
// F[s0+i, s0+i+m) for o < 2 and, for o >= 2, R's m-mer = rc(F[t0-i, t0-i+m))
// with t0 = n-m (o=2) or h-m (o=3).  One m-mer is extracted, the other w-1
// are rolled in (one base per step: F[s0+i+m] forward, or the complement of
// F[t0-i-1] appended on the right for the reverse strand), so a key costs w
// hashes and no funnel shifts.  Returns mix64 of the minimizer m-mer (bucket,
// fingerprint) and its offset q.
template <int S>
__device__ __forceinline__ uint64_t key_minimizer(const uint64_t* f, int n, int o, int h, int m, int w,
                                                  int* q) {
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const bool fwd = o < 2;
  const int s0 = fwd ? (o == 0 ? 0 : n - h) : (o == 2 ? n - m : h - m);
  uint64_t mm = fwd ? ext_fwd<S>(f, s0) >> (64 - 2 * m) : rc_word(ext_fwd<S>(f, s0)) & mmask;
  uint32_t bkey = 0xFFFFFFFFu;
  uint64_t bmm = 0;
  for (int i = 0; i < w; ++i) {
    const uint32_t key = order_key(mm) | (uint32_t)i;
    if (key < bkey) {
      bkey = key;
      bmm = mm;
    }
    if (i + 1 < w) {
      const int x = fwd ? s0 + i + m : s0 - i - 1;  // base rolled in next
      const uint64_t b = (f[(x >> 5) * S] >> (62 - 2 * (x & 31))) & 3u;
      mm = ((mm << 2) | (fwd ? b : 3u - b)) & mmask;
    }
  }
  *q = (int)(bkey & 1023u);
  return mix64(bmm);
}

// Next cell of a chain inside the rank's local range (wraps at its end).  The
// step is odd and depends on the entry's fingerprint (double hashing): with a
// step of 1 (linear probing) the overflow of one heavy minimizer (a high-
// abundance genome's m-mer in hundreds of keys) filled the neighbouring home
// cells, and every run of those buckets walked the whole merged cluster (C5:
// 16 entries scanned per containment run at 3.7 % fingerprint hits).  A step
// of 1 + 2 (fp mod 1024) (512 strides with the 9-bit fingerprint) keeps other minimizers' chains out of the cluster;
// an odd step visits every cell of a power-of-two table.  A rank's range of a
// bucket-sharded table (exchange mode) need not be a power of two, and a step
// sharing a factor with it would cycle through a fraction of the cells, so
// those ranges keep the step of 1.  Insertion and every walk (probe, lookup,
// prefix containment) use the same sequence.
__device__ __forceinline__ uint64_t next_cell(uint64_t c, uint64_t n, uint32_t fp) {
  const uint64_t x = c + ((n & (n - 1)) ? 1 : 1 + 2 * (uint64_t)(fp & 1023u));
  return x >= n ? x % n : x;
}
// the fingerprint an entry was filed with (make_entry: hi32 = len10 << 21 | fp9 << 12 | q10 << 2 | o2)
__device__ __forceinline__ uint32_t entry_fp(unsigned long long e) { return (uint32_t)(e >> 44) & kFpMask; }

// Index entry: lo32 = read index, hi32 = len10 << 21 | fp9 << 12 | q10 << 2 |
// o2 (the chain bit, bit 63, is set on a full cell's last slot).  len10 = the
// read's length - 1 (the templated kernels take reads up to 1,024 bp; longer
// reads, whose kernels read the lengths array, store 1,023): the containment
// probe's length conditions (read2 shorter, placed inside read1) are then
// register work instead of one random 2-B load per listed entry (C5: 554 M
// per step).  The fingerprint has 9 bits: an entry of another minimizer in the
// same cell passes it 1 time in 512 and then fails the window-range test or
// the verification, which compares the whole overlap, so results never depend on it.
__device__ __forceinline__ unsigned long long make_entry(uint64_t v, uint32_t nb_log2, int q, int o, uint32_t r,
                                                         int n) {
  const uint32_t fp = (uint32_t)(v >> nb_log2) & kFpMask;
  const uint32_t ln = (uint32_t)(n < 1 ? 0 : n > 1024 ? 1023 : n - 1);
  return ((unsigned long long)((ln << 21) | (fp << 12) | ((uint32_t)q << 2) | (uint32_t)o) << 32) | r;
}
// the length of the read an entry belongs to (reads up to 1,024 bp)
__device__ __forceinline__ int entry_len(uint32_t hi) { return (int)((hi >> 21) & 1023u) + 1; }

// insertIntoTable (HashTable.cpp:163-195) for one entry: one 64-B cell load,
// then CAS into the slots that looked empty (slots only ever go from empty to
// filled, so a stale view just makes a CAS fail); a full cell gets the chain
// flag and the walk moves to the next cell of the local range.
__device__ __forceinline__ void cell_insert(uint64_t* cells, uint64_t c, uint64_t cell_n, unsigned long long entry) {
  for (uint64_t probe = 0; probe < cell_n; ++probe) {  // capacity >= 2x entries: ends in a few steps
    unsigned long long* cell = reinterpret_cast<unsigned long long*>(cells + c * kCell);
    uint64_t e[kCell];
    const ulonglong2* cp = reinterpret_cast<const ulonglong2*>(cell);
#pragma unroll
    for (int s = 0; s < kCell / 2; ++s) {
      const ulonglong2 x = cp[s];
      e[2 * s] = x.x;
      e[2 * s + 1] = x.y;
    }
    bool done = false;
#pragma unroll
    for (int s = 0; s < kCell; ++s)
      if (!done && e[s] == kEmpty) done = atomicCAS(&cell[s], kEmpty, entry) == kEmpty;
    if (done) return;
    // every slot is filled now: flag the chain (slot 7 holds an entry)
    if (e[kCell - 1] == kEmpty || !(e[kCell - 1] & kChain)) atomicOr(&cell[kCell - 1], (unsigned long long)kChain);
    c = next_cell(c, cell_n, entry_fp(entry));
  }
}

// cell s steps along the chain of fingerprint fp from c (next_cell applied s
// times: every step adds the same stride modulo the range)
__device__ __forceinline__ uint64_t chain_cell(uint64_t c, uint64_t n, uint32_t fp, uint64_t s) {
  const uint64_t step = (n & (n - 1)) ? 1 : 1 + 2 * (uint64_t)(fp & 1023u);
  return (c + s * step) % n;
}

// HashTable::insertDataset (HashTable.cpp:50-80): one thread per key (read r,
// key o = hashRead's four strings, HashTable.cpp:88-104) finds the key's
// minimizer and files the entry in its home cell (this rank's buckets only).
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_index_build(IndexParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  uint64_t* f = smem + threadIdx.x;  // word k at f[k * kBlock]
  const uint64_t mask = (1ULL << p.nb_log2) - 1;
  for (uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x; (gid >> 2) < p.n;
       gid += (uint64_t)gridDim.x * kBlock) {
    const uint64_t r = gid >> 2;
    const int o = (int)(gid & 3);
    if (o == 1 && p.skip_o1) continue;
    const uint64_t* g = p.words + r * slot_words(MAXW);
#pragma unroll
    for (int k = 0; k < MAXW; ++k) f[k * kBlock] = g[k];
    f[MAXW * kBlock] = 0;
    const int n = p.len[r];
    int q;
    const uint64_t v = key_minimizer<kBlock>(f, n, o, p.h, p.m, p.w, &q);
    const uint64_t b = v & mask;
    if (owned(b, p.nb_log2, p.rank, p.nranks))
      cell_insert(p.cells, b - p.cell_lo, p.cell_n, make_entry(v, p.nb_log2, q, o, (uint32_t)r, n));
  }
}

// The discovery index of the uncontained reads (build_live_index): the same
// entries as k_index_build for the live slots only, and only the keys the
// discovery lists (o = 0, 2, 3: an o = 1 hit is the twin of the partner's
// o = 0 hit).  A wavefront takes 64 consecutive slots, reads
// their contained bits (p.cbits, two words) and deals the 3 keys of each live
// slot to consecutive lanes, so no lane is spent on a contained read (C5:
// three quarters of them).
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t x, uint32_t k) {  // position of set bit k (0-based)
  uint32_t pos = 0;
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint32_t c = (uint32_t)__popcll(x & ((1ull << s) - 1));
    if (k >= c) {
      k -= c;
      x >>= s;
      pos += (uint32_t)s;
    }
  }
  return pos;
}

template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_index_live(IndexParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  uint64_t* f = smem + threadIdx.x;  // word k at f[k * kBlock]
  const int lane = threadIdx.x & 63;
  const uint64_t mask = (1ULL << p.nb_log2) - 1;
  const uint64_t ngrp = (p.n + kWave - 1) / kWave, nw = (uint64_t)gridDim.x * kWavesPerBlock;
  for (uint64_t g = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); g < ngrp; g += nw) {
    const uint64_t r0 = g * kWave;
    uint64_t live = ~((uint64_t)p.cbits[2 * g] | ((uint64_t)p.cbits[2 * g + 1] << 32));
    if (p.n - r0 < (uint64_t)kWave) live &= (1ull << (p.n - r0)) - 1;
    const uint32_t nk = 3u * (uint32_t)__popcll(live);
    for (uint32_t k0 = 0; k0 < nk; k0 += kWave) {
      const uint32_t k = k0 + (uint32_t)lane;
      if (k >= nk) continue;
      const uint32_t kq = k / 3u, km = k - 3u * kq;
      const uint64_t r = r0 + nth_set_bit(live, kq);
      const int o = km ? (int)km + 1 : 0;  // 0, 2, 3
      const uint64_t* gw = p.words + r * slot_words(MAXW);
#pragma unroll
      for (int kk = 0; kk < MAXW; ++kk) f[kk * kBlock] = gw[kk];
      f[MAXW * kBlock] = 0;
      int q;
      const uint64_t v = key_minimizer<kBlock>(f, p.len[r], o, p.h, p.m, p.w, &q);
      cell_insert(p.cells, v & mask, p.cell_n, make_entry(v, p.nb_log2, q, o, (uint32_t)r, p.len[r]));
    }
  }
}

// markContainedReads at offset s = 0 (OverlapGraph.cpp:225-340): read2 (or
// its reverse strand) is a prefix of read1.  The reference meets these only
// through read2's suffix key (o = 1/3 at window j = n2 - h), because window
// j = 0 is never scanned; every offset s >= 1 is a prefix-key hit (o = 0/2) at
// window j = s.  A prefix of read1 shares read1's own o = 0 key exactly, so one
// thread per read1 walks that key's cell chain: entries with o = 0/2, the same
// fingerprint and offset q, a shorter read2 and F1[0, n2) == F2 (o = 0) or R2
// (o = 2) -> the same atomicMax as the probe.  With this kernel the
// containment probe drops all o = 1/3 hits (ProbeParams::contain_even).
// read1 = slot a with its o = 0 key filed at local cell c (fingerprint fp,
// offset q): walk the chain for shorter reads whose o = 0/2 key is the same
// string at the same offset, compare the whole of read2 (or its reverse
// strand) with F1[0, n2), atomicMax the container key into read2's superkey
template <int MAXW>
__device__ __forceinline__ void prefix_contain_walk(const uint64_t* __restrict__ words,
                                                    const uint16_t* __restrict__ len,
                                                    const uint64_t* __restrict__ cells, uint64_t cell_n, uint64_t c,
                                                    uint32_t a, uint32_t fp, uint32_t q,
                                                    unsigned long long* __restrict__ superkey,
                                                    const uint32_t* __restrict__ id) {
  const int n1 = len[a];
  const uint64_t* f1 = words + (uint64_t)a * slot_words(MAXW);
  for (uint64_t probe = 0; probe < cell_n; ++probe) {
    const ulonglong2* cp = reinterpret_cast<const ulonglong2*>(cells + c * kCell);
    uint64_t e[kCell];
#pragma unroll
    for (int s = 0; s < kCell / 2; ++s) {
      const ulonglong2 x = cp[s];
      e[2 * s] = x.x;
      e[2 * s + 1] = x.y;
    }
    for (int s = 0; s < kCell; ++s) {
      if (e[s] == kEmpty) continue;
      const uint32_t hi = (uint32_t)(e[s] >> 32), r2 = (uint32_t)e[s];
      const int o = (int)(hi & 3u);
      if ((o & 1) || r2 == a || ((hi >> 12) & kFpMask) != fp || ((hi >> 2) & 1023u) != q) continue;
      const int n2 = len[r2];
      if (n2 >= n1) continue;
      const uint64_t* f2 = words + (uint64_t)r2 * slot_words(MAXW);
      uint64_t diff = 0;
      for (int k = 0; 32 * k < n2; ++k) {  // F1 bases [32k, 32k + 32) vs T's
        const uint64_t bv = o == 0 ? f2[k] : rc_word(ext_fwd<1>(f2, n2 - 32 * k - 32));
        const int rem = n2 - 32 * k;
        diff |= (f1[k] ^ bv) & (rem >= 32 ? ~0ULL : ~(~0ULL >> (2 * rem)));
      }
      if (!diff) atomicMax(&superkey[r2], ((unsigned long long)n1 << 32) | (0xFFFFFFFFu - rid(id, a)));
    }
    if (e[kCell - 1] == kEmpty || !(e[kCell - 1] & kChain)) break;
    c = next_cell(c, cell_n, fp);
  }
}

template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_prefix_contain(const uint64_t* __restrict__ words,
                                                           const uint16_t* __restrict__ len,
                                                           const uint64_t* __restrict__ key0,
                                                           const uint64_t* __restrict__ cells, uint64_t cell_n,
                                                           uint32_t nb_log2, uint64_t n,
                                                           unsigned long long* __restrict__ superkey,
                                                           const uint32_t* __restrict__ id) {
  const uint64_t a = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= n) return;
  const uint64_t k0 = key0[a];
  if (k0 == kEmpty) return;
  prefix_contain_walk<MAXW>(words, len, cells, cell_n, k0 & ((1ULL << nb_log2) - 1), (uint32_t)a,
                            (uint32_t)(k0 >> nb_log2) & kFpMask, (uint32_t)(k0 >> 54), superkey, id);
}

// Exchange mode: the same walk from the o = 0 records among the key records
// this rank received (dense and grouped by bin, mg_xchg_insert_keys: key[i] =
// local home cell, ent[i] = index entry), over its own cells; consecutive
// records walk neighbouring cells
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_prefix_contain_keys(const uint64_t* __restrict__ words,
                                                                const uint16_t* __restrict__ len,
                                                                const uint32_t* __restrict__ key,
                                                                const uint64_t* __restrict__ ent, uint64_t n,
                                                                uint32_t cshift,
                                                                const uint64_t* __restrict__ cells, uint64_t cell_n,
                                                                unsigned long long* __restrict__ superkey,
                                                                const uint32_t* __restrict__ id) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint64_t e = ent[i];
    const uint32_t hi = (uint32_t)(e >> 32);
    if (hi & 3u) continue;  // o = 0 keys only
    prefix_contain_walk<MAXW>(words, len, cells, cell_n, key[i] >> cshift, (uint32_t)e, (hi >> 12) & kFpMask,
                              (hi >> 2) & 1023u,
                              superkey, id);
  }
}

template <int W>
struct LaunchPrefixContainKeys {
  static int run(mg_ctx* ctx) {
    const uint64_t n = ctx->xkeys_n;
    if (!n) return 0;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>((n + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 16));
    hipLaunchKernelGGL(k_prefix_contain_keys<W>, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->d_words, ctx->d_len,
                       ctx->xkey_k, ctx->xkey_e, n, ctx->xkey_cls + ctx->xkey_fs, ctx->d_cells, ctx->cell_n,
                       ctx->superkey, ctx->d_id);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

template <int W>
struct LaunchPrefixContain {
  static int run(mg_ctx* ctx) {
    if (!ctx->n) return 0;
    hipLaunchKernelGGL(k_prefix_contain<W>, dim3((uint32_t)((ctx->n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, ctx->d_words, ctx->d_len, ctx->d_key0, ctx->d_cells, ctx->cell_n, ctx->nb_log2,
                       ctx->n, ctx->superkey, ctx->d_id);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

// ---- exchange mode: the received key records filed without CAS inserts
// (HashTable::insertDataset / insertIntoTable, HashTable.cpp:50-80,163-195).
// mg_xchg_insert_keys makes the records dense (k_xkeys_dense: local home cell
// + entry) and radix-sorts them by home cell, so a cell's entries are
// consecutive.  k_cells_fill then files every record with one plain store: its
// slot is its rank among the equal keys before it (a look back over at most 8
// neighbours, cache hits), and the 8th entry of a cell that has more carries
// the chain flag.  A cell's 9th and later entries (heavy minimizers: a
// metagenome's abundant genomes put dozens of keys under one minimizer, 26 %
// of the records at C5) are placed by k_cells_chain once the homes are filled:
// the record of rank 8 walks the chain for its whole group, resuming each
// entry where the previous one with the same fingerprint went, so a group of g
// entries costs ~g/8 cell visits instead of the ~g^2/16 of one walk per entry.
// CAS inserts of received keys (k_insert_slots) ran at ~7 G keys/s of
// memory-side atomics on the step's critical path; the fused path hides the
// same CASes behind its scan.  The same two kernels over the uncontained
// reads' records (compacted in order) with cells coarsened by `shift` build
// the exchange mode's discovery index (build_live_index_xchg).
// mix64 of the minimizer m-mer of index entry e (read slot r, key o, minimizer
// offset q): the m-mer hashRead's key o (HashTable.cpp:88-104) has at offset q,
// re-extracted from the read's slot -- F[q..] (o = 0), F[n-h+q..] (o = 1),
// rc F[n-m-q..] (o = 2), rc F[w-1-q..] (o = 3), as k_scan / k_rc_keys take
// them -- so its bucket and fingerprint are the sender's.  The exchange
// mode's key records travel as the 8-B entry alone, and every rank holds the reads.
template <int MAXW>
__device__ __forceinline__ uint64_t entry_hash(const uint64_t* __restrict__ words, const uint16_t* __restrict__ len,
                                               uint64_t e, int h, int m, int w) {
  const uint32_t r = (uint32_t)e, hi = (uint32_t)(e >> 32);
  const int o = (int)(hi & 3u), q = (int)((hi >> 2) & 1023u), n = len[r];
  const uint64_t* g = words + (uint64_t)r * slot_words(MAXW);
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const int pos = o == 0 ? q : o == 1 ? n - h + q : o == 2 ? n - m - q : w - 1 - q;
  const uint64_t x = ext_slot<MAXW>(g, pos);
  return mix64(o < 2 ? x >> (64 - 2 * m) : rc_word(x) & mmask);
}

// The received records in the slot layout are walked one peer slot of one
// round at a time: blockIdx.y = t P + s (round t, sender s), blockIdx.x tiles
// the slot, so a record's stream index j = t slot + x needs no division (the
// 64-bit divides of a flat index cost more than the records' own work).

// the received key records (8-B entries) -> dense (local home cell, entry)
// pairs for the sort, the home cell recomputed from the read: sender s's
// records go to [sum over s' < s of its received count, ...) in stream order
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_xkeys_dense(const uint64_t* __restrict__ recv, uint64_t slot,
                                                       uint32_t nranks, uint64_t lim,
                                                       const unsigned long long* __restrict__ counts,
                                                       const uint64_t* __restrict__ words,
                                                       const uint16_t* __restrict__ len, int h, int m, int w,
                                                       uint32_t nb_log2, uint64_t cell_lo, uint32_t cls, uint32_t fs,
                                                       uint32_t* __restrict__ key, uint64_t* __restrict__ ent) {
  const uint32_t ts = blockIdx.y, t = ts / nranks, sp = ts - t * nranks;
  const uint64_t cnt = counts[sp] < lim ? counts[sp] : lim;  // (a cut stream: what arrived)
  uint64_t base = 0;
  for (uint32_t q = 0; q < sp; ++q) base += counts[q] < lim ? counts[q] : lim;
  const uint64_t nbmask = (1ULL << nb_log2) - 1;
  const uint64_t* src = recv + (uint64_t)ts * slot;
  for (uint64_t x = (uint64_t)blockIdx.x * kBlock + threadIdx.x; x < slot; x += (uint64_t)gridDim.x * kBlock) {
    const uint64_t j = (uint64_t)t * slot + x;
    if (j >= cnt) break;
    const uint64_t e = src[x];
    const uint32_t cell = (uint32_t)((entry_hash<MAXW>(words, len, e, h, m, w) & nbmask) - cell_lo);
    // the sort key of k_key_class, formed here: ((cell << cls | (o == 3)) << fs) | low fingerprint bits
    const uint32_t c3 = (cls && ((uint32_t)(e >> 32) & 3u) == 3u) ? 1u : 0u;
    key[base + j] = (((cell << cls) | c3) << fs) | (entry_fp(e) & ((1u << fs) - 1u));
    ent[base + j] = e;
  }
}

// the received runs (8-B metas) -> 16-B probe records at the same positions:
// x = mix64 of the minimizer m-mer at p of the run's read (bucket |
// fingerprint, what the sender's scan hashed), y = the meta
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_xruns_expand(const uint64_t* __restrict__ recv, uint64_t slot,
                                                        uint32_t nranks, const unsigned long long* __restrict__ counts,
                                                        const uint64_t* __restrict__ words, int m,
                                                        ulonglong2* __restrict__ out, int part, uint32_t me) {
  const uint32_t ts = blockIdx.y, t = ts / nranks, sp = ts - t * nranks;
  if (part && (part == 1) != (sp == me)) return;  // (a split probe expands the own stream, then the peers')
  const uint64_t cnt = counts[sp];
  const int msh = 64 - 2 * m;
  const uint64_t* src = recv + (uint64_t)ts * slot;
  ulonglong2* dst = out + (uint64_t)ts * slot;
  for (uint64_t x = (uint64_t)blockIdx.x * kBlock + threadIdx.x; x < slot; x += (uint64_t)gridDim.x * kBlock) {
    if ((uint64_t)t * slot + x >= cnt) break;  // (the probe's regions stop at the counts)
    const uint64_t meta = src[x];
    uint64_t v = 0;
    if (meta != kFlatHole) {
      const uint64_t* g = words + (meta & 0xFFFFFFFFull) * slot_words(MAXW);
      v = mix64(ext_slot<MAXW>(g, (int)((meta >> 32) & 1023u)) >> msh);
    }
    dst[x] = make_ulonglong2(v, meta);
  }
}

// grid of the slot-walking kernels: (tiles of a slot, rounds * P slots)
inline dim3 slot_grid(uint64_t slot, uint32_t rounds, uint32_t nranks) {
  // one record per thread: the kernels are a chain of dependent loads per record
  const uint64_t tiles = std::max<uint64_t>(1, (slot + kBlock - 1) / kBlock);
  return dim3((uint32_t)tiles, rounds * nranks);
}

template <int W>
struct LaunchXkeysDense {
  static int run(mg_ctx* ctx, const uint64_t* recv, uint64_t slot, uint32_t rounds, const unsigned long long* counts,
                 uint32_t* key, uint64_t* ent) {
    hipLaunchKernelGGL(k_xkeys_dense<W>, slot_grid(slot, rounds, ctx->nranks), dim3(kBlock), 0, ctx->stream, recv, slot,
                       ctx->nranks, (uint64_t)rounds * slot, counts, ctx->d_words, ctx->d_len, (int)ctx->h,
                       (int)ctx->m, (int)ctx->w, ctx->nb_log2, ctx->cell_lo, ctx->xkey_cls, ctx->xkey_fs, key, ent);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

template <int W>
struct LaunchXrunsExpand {
  static int run(mg_ctx* ctx, const uint64_t* recv, uint64_t slot, uint32_t rounds, const unsigned long long* counts,
                 ulonglong2* out, int part) {
    hipLaunchKernelGGL(k_xruns_expand<W>, slot_grid(slot, rounds, ctx->nranks), dim3(kBlock), 0, ctx->stream, recv,
                       slot, ctx->nranks, counts, ctx->d_words, (int)ctx->m, out, part, ctx->rank);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

// number of records equal to key c (>> shift) directly before record i, capped at kCell
__device__ __forceinline__ int rank_in_cell(const uint32_t* __restrict__ key, uint64_t i, uint32_t shift, uint32_t c) {
  bool eq[kCell + 1];
#pragma unroll
  for (int k = 1; k <= kCell; ++k) eq[k] = i >= (uint64_t)k && (key[i - k] >> shift) == c;
  int r = 0;
#pragma unroll
  for (int k = 1; k <= kCell; ++k) r = (r == k - 1 && eq[k]) ? k : r;
  return r;
}

// n_dev non-null: the record count is on the device (a compaction's output).
// (Appending each group's leader to a list here, for k_cells_chain to visit
// only those, made this kernel 15x slower -- C3 simulated P = 8: 0.42 vs
// 0.028 ms per rank, profiles/r04i_sim8_c3_ranks_leader_list_rejected.md --
// against 0.02 ms saved in the chain kernel.)
// Records group by key >> gshift (equal group = one cell's entries) and file
// into cell key >> cshift; skip_odd: records whose group has bit 0 set (the
// o = 3 class of a classed key, build_cells) are not filed here.  The bits
// below gshift hold low fingerprint bits (build_cells: a group's records of one
// fingerprint adjacent after the sort, for k_cells_place).
__global__ __launch_bounds__(kBlock) void k_cells_fill(const uint32_t* __restrict__ key,
                                                      const uint64_t* __restrict__ ent,
                                                      const unsigned long long* __restrict__ n_dev, uint64_t n_host,
                                                      uint32_t gshift, uint32_t cshift, int skip_odd,
                                                      uint64_t* __restrict__ cells) {
  const uint64_t n = n_dev ? *n_dev : n_host;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t k = key[i];
    const uint32_t g = k >> gshift;
    if (skip_odd && (g & 1u)) continue;
    const int r = rank_in_cell(key, i, gshift, g);
    if (r < kCell) {
      const bool more = r == kCell - 1 && i + 1 < n && (key[i + 1] >> gshift) == g;
      cells[(uint64_t)(k >> cshift) * kCell + r] = more ? (ent[i] | kChain) : ent[i];
    }
  }
}

// the 9th+ entries of each cell, one thread per group (the group's record of rank 8)
__global__ __launch_bounds__(kBlock) void k_cells_chain(const uint32_t* __restrict__ key,
                                                       const uint64_t* __restrict__ ent,
                                                       const unsigned long long* __restrict__ n_dev, uint64_t n_host,
                                                       uint32_t gshift, uint32_t cshift, int skip_odd, uint64_t* cells,
                                                       uint64_t cell_n) {
  const uint64_t n = n_dev ? *n_dev : n_host;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t k = key[i];
    const uint32_t g = k >> gshift, c = k >> cshift;
    if (skip_odd && (g & 1u)) continue;
    if (rank_in_cell(key, i, gshift, g) != kCell || (i >= kCell + 1 && (key[i - kCell - 1] >> gshift) == g)) continue;
    uint32_t last_fp = ~0u;
    uint64_t at = c;
    for (uint64_t j = i; j < n && (key[j] >> gshift) == g; ++j) {
      const unsigned long long e = ent[j];
      const uint32_t fp = entry_fp(e);
      if (fp != last_fp) at = next_cell(c, cell_n, fp);  // the home is full: its chain starts at the next cell
      last_fp = fp;
      // cell_insert from `at`, leaving `at` at the cell that took the entry
      for (uint64_t probe = 0; probe < cell_n; ++probe) {
        unsigned long long* cell = reinterpret_cast<unsigned long long*>(cells + at * kCell);
        uint64_t ev[kCell];
        const ulonglong2* cp = reinterpret_cast<const ulonglong2*>(cell);
#pragma unroll
        for (int s2 = 0; s2 < kCell / 2; ++s2) {
          const ulonglong2 x = cp[s2];
          ev[2 * s2] = x.x;
          ev[2 * s2 + 1] = x.y;
        }
        bool done = false;
#pragma unroll
        for (int s2 = 0; s2 < kCell; ++s2)
          if (!done && ev[s2] == kEmpty) done = atomicCAS(&cell[s2], kEmpty, e) == kEmpty;
        if (done) break;
        if (ev[kCell - 1] == kEmpty || !(ev[kCell - 1] & kChain)) atomicOr(&cell[kCell - 1], (unsigned long long)kChain);
        at = next_cell(at, cell_n, fp);
      }
    }
  }
}

// Chain records placed in parallel (k_over_heads, a max-scan, k_cells_place):
// an overflow record is one past its home's kCell.  A
// RUN is a group's overflow records of one fingerprint, adjacent after the
// sort; the run's record of index x goes straight to slot x % kCell of the
// cell 1 + x / kCell steps along the fingerprint's chain, so a heavy minimizer's
// hundreds of entries take one CAS each instead of one thread walking them all
// (k_cells_chain).  A slot already taken (another group's entries crossing the
// chain, or a run of a second fingerprint on the same chain) sends its record
// walking on from there, as cell_insert walks.  Chain flags: a run's slot-
// (kCell - 1) record carries the flag when the run goes on; if that record
// was displaced, the cell held more than kCell claimants, so one of them
// walked through it full and set the flag.  Every entry stays reachable from
// its home along its fingerprint's chain, which is all a walk needs (the order
// inside a chain is not an output).
__device__ __forceinline__ bool over_rec(const uint32_t* __restrict__ key, uint64_t i, uint32_t gshift, uint32_t g,
                                         bool* first) {
  if (rank_in_cell(key, i, gshift, g) != kCell) return false;
  *first = !(i >= kCell + 1 && (key[i - kCell - 1] >> gshift) == g);
  return true;
}

// head[i] = i at the first record of each run, else 0 (the max-scan then gives
// every overflow record its run's start)
__global__ __launch_bounds__(kBlock) void k_over_heads(const uint32_t* __restrict__ key,
                                                      const uint64_t* __restrict__ ent,
                                                      const unsigned long long* __restrict__ n_dev, uint64_t n_host,
                                                      uint32_t gshift, int skip_odd,
                                                      uint32_t* __restrict__ head) {
  const uint64_t n = n_dev ? *n_dev : n_host;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t g = key[i] >> gshift;
    bool first = false;
    const bool over = !(skip_odd && (g & 1u)) && over_rec(key, i, gshift, g, &first);
    // both fingerprints loaded unconditionally and the head formed by a
    // multiply: the nested-select form of this expression was miscompiled
    // (ROCm 7.2 hipcc, gfx950: every record past index 8 stored 0)
    const uint32_t fp_prev = entry_fp(ent[i ? i - 1 : 0]), fp_cur = entry_fp(ent[i]);
    const uint32_t hd = (over ? 1u : 0u) & ((first ? 1u : 0u) | (fp_prev != fp_cur ? 1u : 0u));
    head[i] = (uint32_t)i * hd;
  }
}

__global__ __launch_bounds__(kBlock) void k_cells_place(const uint32_t* __restrict__ key,
                                                       const uint64_t* __restrict__ ent,
                                                       const uint32_t* __restrict__ start,
                                                       const unsigned long long* __restrict__ n_dev, uint64_t n_host,
                                                       uint32_t gshift, uint32_t cshift, int skip_odd,
                                                       uint64_t* cells, uint64_t cell_n) {
  const uint64_t n = n_dev ? *n_dev : n_host;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t k = key[i];
    const uint32_t g = k >> gshift;
    bool first = false;
    if ((skip_odd && (g & 1u)) || !over_rec(key, i, gshift, g, &first)) continue;
    const unsigned long long e = ent[i];
    const uint32_t fp = entry_fp(e);
    const uint64_t x = i - start[i];  // index in the run
    const int slot = (int)(x % kCell);
    const bool more = slot == kCell - 1 && i + 1 < n && (key[i + 1] >> gshift) == g && entry_fp(ent[i + 1]) == fp;
    uint64_t at = chain_cell(k >> cshift, cell_n, fp, 1 + x / kCell);
    unsigned long long* cell = reinterpret_cast<unsigned long long*>(cells + at * kCell);
    if (atomicCAS(&cell[slot], kEmpty, more ? (e | kChain) : e) == kEmpty) continue;
    // taken: cell_insert from this cell on
    for (uint64_t probe = 0; probe < cell_n; ++probe) {
      cell = reinterpret_cast<unsigned long long*>(cells + at * kCell);
      uint64_t ev[kCell];
      const ulonglong2* cp = reinterpret_cast<const ulonglong2*>(cell);
#pragma unroll
      for (int s2 = 0; s2 < kCell / 2; ++s2) {
        const ulonglong2 y = cp[s2];
        ev[2 * s2] = y.x;
        ev[2 * s2 + 1] = y.y;
      }
      bool done = false;
#pragma unroll
      for (int s2 = 0; s2 < kCell; ++s2)
        if (!done && ev[s2] == kEmpty) done = atomicCAS(&cell[s2], kEmpty, e) == kEmpty;
      if (done) break;
      if (ev[kCell - 1] == kEmpty || !(ev[kCell - 1] & kChain)) atomicOr(&cell[kCell - 1], (unsigned long long)kChain);
      at = next_cell(at, cell_n, fp);
    }
  }
}

// Diagnostics (option check_cells): every filed record must be found by the
// probes' walk (home cell, then the next cell of its fingerprint's chain while
// the current one is full with the chain flag on its last slot); bad[0] counts
// the records that are not, bad[1..] describes the first ones
__global__ __launch_bounds__(kBlock) void k_check_cells(const uint32_t* __restrict__ key,
                                                       const uint64_t* __restrict__ ent,
                                                       const uint32_t* __restrict__ start,
                                                       const unsigned long long* __restrict__ n_dev, uint64_t n_host,
                                                       uint32_t gshift, uint32_t cshift, int skip_odd,
                                                       const uint64_t* __restrict__ cells, uint64_t cell_n,
                                                       unsigned long long* __restrict__ bad) {
  const uint64_t n = n_dev ? *n_dev : n_host;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t k = key[i];
    if (skip_odd && ((k >> gshift) & 1u)) continue;
    const uint64_t e = ent[i];
    const uint32_t fp = entry_fp(e);
    uint64_t at = k >> cshift;
    bool found = false;
    uint64_t steps = 0;
    for (; steps <= cell_n; ++steps) {
      const uint64_t* c = cells + at * kCell;
      for (int s = 0; s < kCell; ++s) found = found || ((c[s] & ~kChain) == e);
      if (found || c[kCell - 1] == kEmpty || !(c[kCell - 1] & kChain)) break;
      at = next_cell(at, cell_n, fp);
    }
    if (!found) {
      const unsigned long long q = atomicAdd(&bad[0], 1ull);
      if (q < 8) {
        bad[1 + q * 4] = i;
        bad[2 + q * 4] = ((uint64_t)(k >> cshift) << 32) | steps;
        bad[3 + q * 4] = start ? (uint64_t)start[i] : ~0ull;
        bad[4 + q * 4] = e;
      }
    }
  }
}

// Sort keys of the exchange mode's received records: ((home cell << cls | c) <<
// fs) | the fingerprint's low fs bits.  A classed build (cls = 1) leaves out the
// o = 3 records from the full table: c = (o == 3), so a cell's o = 0 / 2 records
// group apart from its o = 3 ones (build_cells, index_o3); the fingerprint bits
// put a group's records of one fingerprint next to each other (k_cells_place)
__global__ __launch_bounds__(kBlock) void k_key_class(uint32_t* __restrict__ key, const uint64_t* __restrict__ ent,
                                                     uint64_t n, uint32_t cls, uint32_t fs) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) {
    const uint64_t e = ent[i];
    const uint32_t c = (cls && ((uint32_t)(e >> 32) & 3u) == 3u) ? 1u : 0u;
    key[i] = (((key[i] << cls) | c) << fs) | (entry_fp(e) & ((1u << fs) - 1u));
  }
}

// the uncontained reads' records (cbits clear), flagged for the in-order compaction
__global__ __launch_bounds__(kBlock) void k_live_flags(const uint64_t* __restrict__ ent, uint64_t n,
                                                      const uint32_t* __restrict__ cbits, uint8_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = (uint32_t)ent[i];
  flag[i] = ((cbits[r >> 5] >> (r & 31u)) & 1u) ? 0 : 1;
}

// ------------------------------------------------------------- discovery ---
// Discovery is two kernels:
//   k_scan  : minimizer runs of every source read -> 8-byte run records
//             (read index, minimizer position p, window range [jlo, jhi]) in a
//             per-wavefront HBM region;
//   k_probe : one run per lane -> home cell chain -> exact candidates -> full
//             overlap verification -> rows (insertEdge) or superReadID updates.
struct ScanParams {
  const uint64_t* words;
  const uint16_t* len;
  const uint32_t* super;          // source reads with superReadID != 0 get no windows (:548)
  uint64_t a_lo, a_hi;
  int h, m, w;
  uint32_t nb_log2, rank, nranks;
  ulonglong2* runs;               // one region of run_cap records per wavefront
  unsigned long long* run_cnt;    // [waves] records produced (may exceed run_cap)
  uint64_t run_cap;
  uint64_t* cells;                // k_scan<INDEX>: the (unsharded) cell table the keys go into
  uint64_t cell_n;
  // exchange mode: the four key records of read a go to key_bk / key_ent[o *
  // key_n + a] (bucket, entry) instead of a CAS into the cells; they travel to
  // the bucket owner (k_part) and mg_xchg_insert_keys files them there
  uint32_t* key_bk;
  uint64_t* key_ent;
  uint64_t key_n, key_lo;       // key o of source read a at o * key_n + (a - key_lo)
  // per read: its o = 0 key's hash bits (bucket | fingerprint, 50 bits) | q << 54
  // (k_prefix_contain); nullptr: not written
  uint64_t* key0;
  // per read: its window-0 run (x = mix64 of the o = 0 key's minimizer, window
  // range [0, 0]) for the containment probe's offset-0 pass; nullptr: not written
  ulonglong2* p0runs;
  int skip_o1;                    // INDEX: leave out the o = 1 keys (mg_ctx::index_o1)
  int skip_o3;                    // INDEX (fused): leave out the o = 3 keys (mg_ctx::index_o3)
  int no_insert;                  // diagnostics (phase_limit = 1): the index scan files no keys (timing only)
  // k_scan_reg (exchange mode): runs stored per destination rank, dst_cnt[gw *
  // dst_ranks + d] (nullptr: not counted; k_part's count pass does it)
  unsigned long long* dst_cnt;
  uint32_t dst_ranks;
  // k_scan<RECV> (exchange mode, keys first): the key records this rank
  // received (8-B entries in the slot layout: recv_P peers x recv_slot per
  // round, recv_total positions, recv_cnt = the per-peer counts), CAS-inserted
  // into the rank's cells (local cell = bucket - cell_lo) during the scan
  const uint64_t* recv_keys;
  const unsigned long long* recv_cnt;
  uint64_t recv_slot, recv_total, cell_lo;
  uint32_t recv_P;
  // k_scan<RECV>: what leaves the rank is the run's 8-B meta, so the regions
  // hold 8-B metas (runs viewed as uint64_t, same region positions) and
  // run_dst the owner rank of each (k_part<OWN_META> routes them)
  uint8_t* run_dst;
};

// Exchange-mode key records are o-major in the order o = 0, 2, 3, 1: when the
// index leaves out the o = 1 keys, the valid records are the first three
// segments (one rank: mg_xchg_insert_keys sorts them in place)
__device__ __forceinline__ int key_seg(int o) { return o == 0 ? 0 : (o == 1 ? 3 : o - 1); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Run record (16 B): x = mix64 of the minimizer m-mer (bucket | fingerprint),
// y = read index (32 bits) | p << 32 | jlo << 42 | jhi << 52.
__device__ __forceinline__ uint64_t run_meta(uint64_t a, int p, int jlo, int jhi) {
  return (a & 0xFFFFFFFFull) | ((uint64_t)p << 32) | ((uint64_t)jlo << 42) | ((uint64_t)jhi << 52);
}

// 32 bases of a lane's read starting at base `pos` (per-lane), from its words
// in registers (pos >> 5 selected by a compare chain, not a register index,
// which would go through scratch)

template <int MAXW>
__device__ __forceinline__ uint64_t ext_reg(const uint64_t* rw, int pos) {
  const int wi = pos >> 5;
  uint64_t w0 = rw[0], w1 = rw[1];
#pragma unroll
  for (int k = 1; k <= MAXW; ++k) {
    w0 = wi == k ? rw[k] : w0;
    w1 = wi + 1 == k ? rw[k] : w1;
  }
  if (wi + 1 > MAXW) w1 = 0;
  return funnel(w0, w1, (pos & 31) << 1);
}

// Window minimizers of every source read (the windows of insertAllEdgesOfRead,
// OverlapGraph.cpp:534-537), one read per lane.  Rolling 2-bit m-mer and the
// van Herk / Gil-Werman sliding minimum over blocks of w positions: prefix
// minimum of the current block in a register, suffix minima of the previous
// block in LDS (w u32 per lane, overwritten by the current block's keys exactly
// behind the read front).  Window j = m-mers [j, j+w-1] = the h-mer at j; its
// minimizer is min(suffix_prev[u+1], prefix_cur) under order_key | position,
// the rule the index used for the keys.  Block boundaries depend only on t, so
// control flow is uniform across lanes.  A run ends where the minimizer
// position changes; its record goes straight to HBM (ballot-compacted).
// INDEX: the same pass also builds the index (HashTable::insertDataset,
// HashTable.cpp:50-80).  The four keys of a read (hashRead :88-104) are the
// windows at its two ends on both strands: o = 0 is window j = 0 (its prefix
// minimum at t = w - 1 and the m-mer at t = 0), o = 1 is window j = n - h (one
// extra step, t = n - m, that emits no run), each with the key offset i = t
// shifted by a constant, so the argmin is the scan's; o = 2 / 3 come from a
// w-step pass over the reverse strand's m-mers after the read (uniform trip
// count, no per-step key work in the base loop: C5's mixed lengths kept the
// key branch of the old in-step version open for most steps).  Same keys
// (order_key | i) as key_minimizer, so lookups and the exchange mode's key
// records agree.  The CAS inserts of a read's four keys overlap the ALU-bound
// scan of the other wavefronts.
// 6 waves per SIMD (the LDS limit: 6 blocks of 4 wavefronts per CU): 80 VGPRs
// with a 12-B spill beat 83 VGPRs / 5 waves, index 3.72 vs 3.93 ms at C3
// (profiles/r01s5_ab_scan_waves.log)
// KEYREC (exchange mode with w > 32, INDEX only): key records for the bucket
// owners instead of CAS inserts.  Each instantiation references only the
// parameters it uses, which keeps its scalar registers below the limit.
#ifndef MG_SCAN_WAVES_G
#define MG_SCAN_WAVES_G 6  // waves/SIMD of the length-ranked (G > 1) scan (A/B builds override)
#endif
template <int MAXW, bool INDEX, bool KEYREC = false, int G = 1, bool RECV = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(G > 1 ? MG_SCAN_WAVES_G : 6))) void k_scan(ScanParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = p.h, m = p.m, w = p.w;
  uint32_t* s_keys = reinterpret_cast<uint32_t*>(smem) + (size_t)wv * (w + kScanKeyPad) * kWave + lane;  // slot u at [u*64]
  const int msh = 64 - 2 * m;
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const uint64_t ngroups = (p.a_hi - p.a_lo + kWave - 1) / kWave;
  const int wpb = (int)(blockDim.x >> 6);  // 4, or fewer when w's LDS arrays need it (scan_wpb)
  const uint64_t gw = (uint64_t)blockIdx.x * wpb + wv;
  const uint64_t nw = (uint64_t)gridDim.x * wpb;
  uint64_t* s_buf = reinterpret_cast<uint64_t*>(smem) + (size_t)wpb * (((w + kScanKeyPad) * kWave + 1) / 2) +
                    (size_t)wv * kScanBuf;
  s_keys[w * kWave] = 0xFFFFFFFFu;  // the sentinel (never overwritten)
  // region j of this wavefront (= run region G gw + j) holds the runs
  // of group j of each of its windows: a probe block's share of G
  // consecutive regions then covers consecutive slots, as with one group per
  // region
  ulonglong2* const region = p.runs + gw * G * p.run_cap;
  const uint64_t nbmask = (1ULL << p.nb_log2) - 1;
  uint64_t cur[G] = {};  // records per region (wavefront-uniform)
  // KEYREC with p.dst_cnt: lane j P + d counts the stored runs of region j bound
  // for rank d (k_part's OWN_BUCKET rule), so routing them needs no count pass
  uint32_t dcnt = 0;
  uint32_t nbuf = 0;  // run metas staged in s_buf (wavefront-uniform)

  // close the run of minimizer position pos over windows [jlo, jhi]: stage its
  // meta in LDS (the hashing and the HBM write happen 64 at a time in flush);
  // staged metas carry (owner lane << 8 | slot within the window) where the
  // record will carry the read index
  auto put = [&](bool flag, uint64_t meta) {
    const uint64_t bal = __ballot(flag);
    // every lane stores (no exec-mask branch: the scalar unit is the scan's
    // tightest issue port); lanes without a run write their spare slot
    uint32_t at = nbuf + lane_prefix(bal);
    __asm__ volatile("" : "+v"(at));  // (computed by every lane: a select below, not an exec-mask region)
    s_buf[flag ? at : 2 * kWave + lane] = meta;
    nbuf += (uint32_t)__popcll(bal);
  };
  const uint64_t nwin = (ngroups + G - 1) / G;
  // RECV: this wavefront's share of the received key records (slot-layout
  // positions [r_at, r_end), chunks of 64 -- slots are multiples of 64), a few
  // chunks of CAS inserts after each window, so their latency hides behind the
  // other wavefronts' scan as the fused path's own inserts do
  uint64_t r_at = 0, r_end = 0, r_per = 0;
  if constexpr (RECV) {
    const uint64_t nch = (p.recv_total + 63) / 64;
    const uint64_t ch0 = nch * gw / nw, ch1 = nch * (gw + 1) / nw;
    r_at = ch0 * 64;
    r_end = min(ch1 * 64, p.recv_total);
    const uint64_t wins = gw < nwin ? (nwin - gw + nw - 1) / nw : 0;
    r_per = wins ? ((ch1 - ch0) + wins - 1) / wins : 0;
  }
  auto recv_insert = [&](uint64_t nchunks) {
    for (uint64_t c = 0; c < nchunks && r_at < r_end; ++c, r_at += 64) {
      const uint64_t ts = r_at / p.recv_slot, x = r_at - ts * p.recv_slot + (uint64_t)lane;  // (one divide per chunk)
      const uint64_t t = ts / p.recv_P, sp = ts - t * p.recv_P;
      if (r_at + (uint64_t)lane < r_end && t * p.recv_slot + x < p.recv_cnt[sp]) {
        const uint64_t e = p.recv_keys[r_at + lane];
        const uint64_t v = entry_hash<MAXW>(p.words, p.len, e, h, m, w);
        cell_insert(p.cells, (v & nbmask) - p.cell_lo, p.cell_n, e);
      }
    }
  };
  for (uint64_t win = gw; win < nwin; win += nw) {
   const uint64_t A0 = p.a_lo + win * (G * kWave);  // the window's first slot
   // (length, slot) of the window's reads, ascending: pass q takes ranks
   // [64 q, 64 q + 64), so each pass's base loop runs to about its own
   // longest read instead of every group's (mixed lengths: lanes idle less)
   uint32_t wk[G];
   uint32_t lmin = 0xFFFFFFFFu, lmax = 0;
#pragma unroll
   for (int q = 0; q < G; ++q) {
     const uint32_t idx = (uint32_t)(lane + kWave * q);
     const uint64_t a = A0 + idx;
     uint32_t n = 0;
     if (a < p.a_hi) {
       n = p.len[a];
       if (!INDEX && n && p.super && p.super[a]) n = 0;  // (an index scan covers every source)
     }
     wk[q] = ((0x7FFu - n) << 8) | idx;  // longest first: containers before their contents
     lmin = min(lmin, n);
     lmax = max(lmax, n);
   }
   if constexpr (G > 1) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      lmin = min(lmin, (uint32_t)__shfl_xor((int)lmin, d));
      lmax = max(lmax, (uint32_t)__shfl_xor((int)lmax, d));
    }
   }
   if (G > 1 && __builtin_amdgcn_readfirstlane(lmin) != __builtin_amdgcn_readfirstlane(lmax)) {
     // bitonic sort of the 256 keys, element e = lane + 64 q in wk[q]
#pragma unroll
     for (int k = 2; k <= G * kWave; k <<= 1) {
#pragma unroll
       for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
         for (int q = 0; q < G; ++q) {
           const int e = lane + kWave * q;
           const bool up = (e & k) == 0;
           if (j >= kWave) {  // partner in this lane's own registers
             const int q2 = q ^ (j / kWave);
             if (q < q2) {
               const uint32_t x = wk[q], y = wk[q2];
               const bool sw = up ? x > y : x < y;
               wk[q] = sw ? y : x;
               wk[q2] = sw ? x : y;
             }
           } else {
             const uint32_t o = (uint32_t)__shfl_xor((int)wk[q], j);
             const bool low = (e & j) == 0;
             wk[q] = (low == up) ? min(wk[q], o) : max(wk[q], o);
           }
         }
       }
     }
   }
   for (int q = 0; q < G; ++q) {  // one pass of 64 reads (not unrolled: code size)
    uint32_t key = wk[0];
#pragma unroll
    for (int qq = 1; qq < G; ++qq) key = q == qq ? wk[qq] : key;
    const uint32_t wslot = key & 255u;
    const uint64_t a = A0 + wslot;
    const int n = (int)(0x7FFu - (key >> 8));
    const uint64_t own = G > 1 ? ((uint64_t)lane << 8) | wslot : a;  // a staged run's read (see put)
    const uint64_t* g = p.words + a * slot_words(MAXW);
    const int J = n - h - 1;                 // windows j = 1 .. J (:534)
    const int tend = J >= 1 ? J + w - 1 : 0;  // last m-mer position a window uses
    // INDEX: one more step, t = n - m: its window j = n - h is key o = 1's
    const int tlast = (INDEX && tend) ? tend + 1 : tend;
    int tmax = tlast;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tmax = max(tmax, __shfl_xor(tmax, d));
    tmax = __builtin_amdgcn_readfirstlane(tmax);  // wavefront-uniform loop bound
    // the read's words in registers (no global load inside the base loop); the
    // word holding base t + m is picked by a wavefront-uniform index
    constexpr int kRw = MAXW + 1 <= slot_words(MAXW) ? MAXW + 1 : slot_words(MAXW);
    uint64_t rw[MAXW + 1];
    {
      const uint64_t* gs = a < p.a_hi ? g : p.words;  // a slot every lane may read
#pragma unroll
      for (int k = 0; k <= MAXW; ++k) rw[k] = k < kRw ? gs[k] : 0;
    }
    // the words land before the base loop: otherwise the loop's first use of a
    // word sits behind a vmcnt(0) that the compiler repeats every step (the
    // flushes' run stores and the CAS inserts keep vmcnt open across the back
    // edge), so each step after a flush waited for those stores to retire
    __builtin_amdgcn_s_waitcnt(kWaitVm0);
    auto word_at = [&](int idx) {  // idx wavefront-uniform
      uint64_t v = rw[0];
#pragma unroll
      for (int k = 1; k <= MAXW; ++k) v = idx == k ? rw[k] : v;
      return v;
    };
    // hash the first k (<= 64) staged runs with every lane busy, drop runs whose
    // bucket another rank owns, write full-wavefront 16-B records into the
    // region of each run's group
    auto flush = [&](uint32_t k) {
      wave_sync();
      bool flag = (uint32_t)lane < k;
      uint64_t v = 0, meta = 0;
      if (flag) meta = s_buf[lane];
      // slot within the window; G > 1 stages (lane << 8 | slot) for the read index
      const uint32_t ws = G > 1 ? (uint32_t)meta & 255u : (uint32_t)meta - (uint32_t)A0;
      if (G > 1) meta = (meta & ~0xFFFFFFFFull) | (uint32_t)(A0 + ws);
      if constexpr (MAXW <= 8) {
        // every staged run belongs to a read of this pass (flushed before the
        // next pass): its words come from the owner lane's registers, not HBM
        // (a global load here made every flush wait for the earlier stores)
        const int pos = (int)((meta >> 32) & 1023u), wi = pos >> 5;
        const int src = !flag ? lane : G > 1 ? (int)((uint32_t)s_buf[lane] >> 8 & 63u) : (int)ws;
        uint64_t w0 = 0, w1 = 0;
  #pragma unroll
        for (int kk = 0; kk <= MAXW; ++kk) {
          const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)rw[kk]);
          const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)(rw[kk] >> 32));
          const uint64_t x = ((uint64_t)hi << 32) | lo;
          w0 = wi == kk ? x : w0;
          w1 = wi + 1 == kk ? x : w1;
        }
        if (flag) {
          v = mix64(funnel(w0, w1, (pos & 31) << 1) >> msh);
          // (an index scan keeps every bucket's runs unless it builds a bucket-range shard)
          if (!INDEX || p.nranks > 1) flag = owned(v & nbmask, p.nb_log2, p.rank, p.nranks);
        }
      } else if (flag) {
        const uint64_t* g2 = p.words + (meta & 0xFFFFFFFFull) * slot_words(MAXW);
        const int pos = (int)((meta >> 32) & 1023u);
        v = mix64(funnel(g2[pos >> 5], g2[(pos >> 5) + 1], (pos & 31) << 1) >> msh);
        if (!INDEX || p.nranks > 1) flag = owned(v & nbmask, p.nb_log2, p.rank, p.nranks);
      }
      uint64_t at_rec = 0;  // the record's index in its region
      uint32_t grp_rec = 0;
      if constexpr (G == 1) {
        const uint64_t bal = __ballot(flag);
        const uint64_t at = cur[0] + lane_prefix(bal);
        at_rec = at;
        if constexpr (RECV) {  // the meta and its owner rank (the hash stays here: the owner re-hashes)
          if (flag && at < p.run_cap) {
            reinterpret_cast<uint64_t*>(p.runs)[gw * p.run_cap + at] = meta;
            p.run_dst[gw * p.run_cap + at] = (uint8_t)(((v & nbmask) * p.dst_ranks) >> p.nb_log2);
          }
        } else {
#if defined(MG_DIAG_STORE_NEVER)
        if (flag && at < p.run_cap && v == 0x0123456789ABCDEFull) region[at] = make_ulonglong2(v, meta);
#elif !defined(MG_DIAG_NO_RUNSTORE)
        if (flag && at < p.run_cap) region[at] = make_ulonglong2(v, meta);
#endif
        }
        cur[0] += (uint64_t)__popcll(bal);
      } else {
#ifdef MG_DIAG_ONE_REGION  // (diagnostics build: every run of a window into its first region)
        const uint32_t grp = 0;
#else
        const uint32_t grp = ws >> 6;  // the run's group in the window
#endif
        uint64_t at = 0;
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const uint64_t bal = __ballot(flag && grp == (uint32_t)j);
          if (grp == (uint32_t)j) at = cur[j] + lane_prefix(bal);
          cur[j] += (uint64_t)__popcll(bal);
        }
        at_rec = at;
        grp_rec = grp;
#if defined(MG_DIAG_STORE_NEVER)  // (diagnostics build: runs hashed and placed, but (practically) never stored)
        if (flag && at < p.run_cap && v == 0x0123456789ABCDEFull) region[grp * p.run_cap + at] = make_ulonglong2(v, meta);
#elif !defined(MG_DIAG_NO_RUNSTORE)  // (diagnostics build: the window scan stores no runs)
        if (flag && at < p.run_cap) region[grp * p.run_cap + at] = make_ulonglong2(v, meta);
#endif
      }
      if constexpr (KEYREC || RECV) {
        if (p.dst_cnt) {
          const bool st = flag && at_rec < p.run_cap;  // (k_part routes the stored records of a region)
          const uint32_t d = st ? (uint32_t)(((v & nbmask) * p.dst_ranks) >> p.nb_log2) : 0u;
          for (uint32_t jj = 0; jj < (uint32_t)G; ++jj)
            for (uint32_t dd = 0; dd < p.dst_ranks; ++dd) {
              const uint32_t cc = (uint32_t)__popcll(__ballot(st && grp_rec == jj && d == dd));
              dcnt += (uint32_t)lane == jj * p.dst_ranks + dd ? cc : 0u;
            }
        }
      }
      const uint32_t rest = nbuf - k;  // < 128 left: move them to the front
      const uint64_t m0 = (uint32_t)lane < rest ? s_buf[k + lane] : 0;
      const uint64_t m1 = (uint32_t)lane + kWave < rest ? s_buf[k + kWave + lane] : 0;
      wave_sync();
      if ((uint32_t)lane < rest) s_buf[lane] = m0;
      if ((uint32_t)lane + kWave < rest) s_buf[kWave + lane] = m1;
      nbuf = rest;
      wave_sync();
      // the flush's LDS traffic retired here, on its own (rare) path: otherwise
      // the step after it, reusing those registers, waits on lgkmcnt(0) for every
      // LDS op in flight, the prefetched suffix minimum included, on every step
      __builtin_amdgcn_s_waitcnt(0xC07F);
    };
    uint64_t mm = 0;
    if (tend) mm = funnel(rw[0], rw[1], 2) >> msh;  // m-mer at t = 1
    // INDEX: best (order_key | i) of the keys o = 0 / 1 (hashRead's forward
    // keys = the windows j = 0 and j = n - h of this same scan: key offset i is
    // t shifted by a constant, so the argmin is the scan's); o = 2 / 3 come from
    // a w-step pass over the reverse strand after the read's scan
    uint32_t kb0 = 0xFFFFFFFFu, kb1 = 0xFFFFFFFFu;
    if (INDEX && tend) kb0 = order_key(rw[0] >> msh);  // t = 0 (window j = 0 is no scan window)
    uint32_t pmin = 0xFFFFFFFFu;
    int last_pos = 0, jlo = 1;
    int u = 0;  // offset of t in its block of w positions
    // previous block's suffix minimum at u + 1, read one step ahead so the
    // LDS latency hides behind the step's ALU work
    uint32_t sv_pf = s_keys[kWave];
    // The base steps (cw = the read word holding base t + m), without a per-lane branch (selects only: the CU's one
    // scalar unit is the scan's tightest issue port -- the branchy step issued
    // ~37 scalar instructions per step for its exec masks and flow blocks, 0.90 G
    // SALU vs 1.07 G VALU per C3 launch), in two loops with no per-step test of
    // the phase: the first block t = 1 .. w (window j = 1 at t = w, key o = 0's
    // prefix at t = w - 1), then t > w, where every step is a window j >= 2.  A
    // lane past its read (t > tend) keeps computing; only its run state and keys
    // are held.  The block's prefix minimum restarts at +inf after each block,
    // and the suffix minimum past the block (u = w - 1) is the sentinel slot.
    // sh = 62 - 2 ((t + m) & 31): the shift that brings base t + m of cw down
    // (kept by the loops, wavefront-uniform)
    auto roll_and_advance = [&](uint32_t key, uint64_t cw, int sh) {
      s_keys[u * kWave] = key;
      mm = ((mm << 2) | ((cw >> sh) & 3u)) & mmask;  // roll in the base at t + m
      if (++u == w) {  // block complete: suffix minima in place, 8 reads in flight at a time
        uint32_t run = 0xFFFFFFFFu;
        for (int v0 = w - 1; v0 >= 0; v0 -= 8) {
          uint32_t x8[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) x8[k] = v0 - k >= 0 ? s_keys[(v0 - k) * kWave] : 0xFFFFFFFFu;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            run = x8[k] < run ? x8[k] : run;
            if (v0 - k >= 0) s_keys[(v0 - k) * kWave] = run;
          }
        }
        u = 0;
        pmin = 0xFFFFFFFFu;
      }
      sv_pf = s_keys[(u + 1) * kWave];  // (u + 1 = w: the sentinel)
    };
    // t = 1 .. w: the first block; t = w is window j = 1 (no run closes there)
    auto step_first = [&](int t, uint64_t cw, int sh) {
      const uint32_t key = order_key(mm) | (uint32_t)t;
      pmin = min(pmin, key);
      if (INDEX && t == w - 1) kb0 = min(kb0, pmin);  // o = 0: t in [0, w)
      if (t == w) last_pos = (int)(min(sv_pf, pmin) & 1023u);
      roll_and_advance(key, cw, sh);
    };
    // t > w: window j = t - w + 1 >= 2 (a run closes where its minimizer moves)
    auto step = [&](int t, uint64_t cw, int sh) {
      const uint32_t key = order_key(mm) | (uint32_t)t;
      pmin = min(pmin, key);
      const uint32_t mn = min(sv_pf, pmin);
      const int pos = (int)(mn & 1023u);
      if (INDEX) kb1 = t == tlast ? mn - (uint32_t)(n - h) : kb1;  // o = 1: window j = n - h, i = t - (n - h)
      const bool live = t <= tend;
      const bool emit = live && pos != last_pos;
      const uint64_t e_meta = run_meta(own, last_pos, jlo, t - w);
      jlo = emit ? t - w + 1 : jlo;
      last_pos = live ? pos : last_pos;
      roll_and_advance(key, cw, sh);
      put(emit, e_meta);
      if (nbuf >= (uint32_t)kWave) flush(kWave);  // (< 64 staged before the put: one flush at most)
    };
    if constexpr (MAXW <= 8) {
      // one loop per read word and phase (t + m <= n - 1 < 32 MAXW): the word is
      // a compile-time register, so rw[] never goes to scratch and no vmcnt wait
      // (which would also wait for the flushes' stores) sits in the loop
#pragma unroll
      for (int k = 0; k < MAXW + (INDEX ? 1 : 0); ++k) {  // (INDEX's step t = n - m rolls in base n)
        const int t0 = max(1, 32 * k - m), t1 = min(tmax, 32 * k + 31 - m);
        const int tf = min(t1, w);
        for (int t = t0, sh = 62 - 2 * ((t0 + m) & 31); t <= tf; ++t, sh -= 2) step_first(t, rw[k], sh);
        int t = max(t0, w + 1), sh = 62 - 2 * ((t + m) & 31);
        if (t <= t1) {
#if MG_SCAN_UNROLL == 2
          // two steps per trip: half the loop's scalar counting and branching
          for (; t + 1 <= t1; t += 2, sh -= 4) {
            step(t, rw[k], sh);
            step(t + 1, rw[k], sh - 2);
          }
          if (t <= t1) step(t, rw[k], sh);
#else
          do {  // (bottom-tested: one compare and branch per step)
            step(t, rw[k], sh);
            sh -= 2;
          } while (++t <= t1);
#endif
        }
      }
    } else {
      int cwi = __builtin_amdgcn_readfirstlane((1 + m) >> 5);
      uint64_t cw = word_at(cwi);
      for (int t = 1; t <= tmax; ++t) {
        const int sh = 62 - 2 * ((t + m) & 31);
        if (t <= w) step_first(t, cw, sh); else step(t, cw, sh);
        const int xu = __builtin_amdgcn_readfirstlane(t + m);
        if ((xu & 31) == 31) cw = word_at((xu + 1) >> 5);  // next word (don't-care past a read's end)
      }
    }
    put(tend > 0, run_meta(own, last_pos, jlo, J));  // each read's last run
    while (nbuf) flush(nbuf < (uint32_t)kWave ? nbuf : (uint32_t)kWave);  // the group's runs leave with its registers
    if (INDEX && tend) {
      // o = 3 (R[n-h, n) = rc F[0, h): m-mer i = rc of F's at t = w-1-i) and
      // o = 2 (R[0, h) = rc F[n-h, n): m-mer i = rc of F's at t = n-m-i), both
      // rolled towards smaller t, one base per step, w steps for every lane
      uint32_t kb2 = 0xFFFFFFFFu, kb3 = 0xFFFFFFFFu;
      const bool w32 = w <= 32;  // (wavefront-uniform) every key base within 32 of its start
      if (w32) {
        const uint64_t Aw = ext_reg<MAXW>(rw, n - h);                      // F[n-h, n-h+32)
        uint64_t r3 = rc_word(funnel(rw[0], rw[1], 2 * (w - 1))) & mmask;  // rc(F[w-1, w-1+m))
        uint64_t r2 = rc_word(ext_reg<MAXW>(rw, n - m)) & mmask;          // rc(F[n-m, n))
        for (int i = 0; i < w; ++i) {
          kb3 = min(kb3, order_key(r3) | (uint32_t)i);
          kb2 = min(kb2, order_key(r2) | (uint32_t)i);
          const int t3 = w - 2 - i;  // the base entering: F[t3] (o = 3), F[n-h + t3] (o = 2)
          if (t3 >= 0) {
            r3 = ((r3 << 2) | (3u - ((rw[0] >> (62 - 2 * t3)) & 3u))) & mmask;
            r2 = ((r2 << 2) | (3u - ((Aw >> (62 - 2 * t3)) & 3u))) & mmask;
          }
        }
      } else {  // long keys: each m-mer read from the slot (slow, correct; off the hot path)
        const uint64_t* gk = p.words + a * slot_words(MAXW);
        for (int i = 0; i < w; ++i) {
          kb3 = min(kb3, order_key(rc_word(ext_slot<MAXW>(gk, w - 1 - i)) & mmask) | (uint32_t)i);
          kb2 = min(kb2, order_key(rc_word(ext_slot<MAXW>(gk, n - m - i)) & mmask) | (uint32_t)i);
        }
      }
      // the minimizer m-mers from their offsets: o = 0 / 3 at forward t = i /
      // w - 1 - i, o = 1 / 2 at n - h + i / n - m - i
      const uint64_t nbm = (1ULL << p.nb_log2) - 1;
      const uint32_t kb[4] = {kb0, kb1, kb2, kb3};
      const int i0 = (int)(kb0 & 1023u), i1 = (int)(kb1 & 1023u), i2 = (int)(kb2 & 1023u), i3 = (int)(kb3 & 1023u);
      const uint64_t f0 = w32 ? funnel(rw[0], rw[1], i0 << 1) : ext_reg<MAXW>(rw, i0);
      const uint64_t f3 = w32 ? funnel(rw[0], rw[1], (w - 1 - i3) << 1) : ext_reg<MAXW>(rw, w - 1 - i3);
      const uint64_t mb[4] = {f0 >> msh, ext_reg<MAXW>(rw, n - h + i1) >> msh,
                              rc_word(ext_reg<MAXW>(rw, n - m - i2)) & mmask, rc_word(f3) & mmask};
      uint64_t cb[4];
      unsigned long long ce[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const uint64_t v = mix64(mb[o]);
        const unsigned long long e = make_entry(v, p.nb_log2, (int)(kb[o] & 1023u), o, (uint32_t)a, n);
#ifndef MG_DIAG_NO_KEY0  // (diagnostics build: no o = 0 key records)
        if (o == 0 && p.key0) p.key0[a] = (v & ((1ULL << 50) - 1)) | ((uint64_t)(kb[0] & 1023u) << 54);
        if constexpr (G > 1 || kWinGroups == 1) {  // (mixed lengths only: the length-ranked windows)
          if (o == 0 && p.p0runs) p.p0runs[a] = make_ulonglong2(v, run_meta(a, (int)(kb[0] & 1023u), 0, 0));
        }
#endif
        if constexpr (KEYREC) {  // o-major: each store is one coalesced wavefront line
          p.key_bk[key_seg(o) * p.key_n + a - p.key_lo] = (uint32_t)(v & nbm);
          p.key_ent[key_seg(o) * p.key_n + a - p.key_lo] = (o == 1 && p.skip_o1) ? kEmpty : e;  // (a hole: not routed)
        }
        cb[o] = v & nbm;
        ce[o] = e;
      }
      // (the four inserts with their cell loads and CASes in flight together
      // measured slower: scan 3.06-3.13 vs 2.92-2.94 ms at C3, profiles/r03y_ab_scan.txt)
      if constexpr (!KEYREC) {
#pragma unroll
        for (int o = 0; o < 4; ++o)  // (a bucket-range shard files its own buckets' keys: local cell = bucket - cell_lo)
          if ((o != 1 || !p.skip_o1) && (o != 3 || !p.skip_o3) && !p.no_insert && owned(cb[o], p.nb_log2, p.rank, p.nranks))
            cell_insert(p.cells, cb[o] - p.cell_lo, p.cell_n, ce[o]);
      }
    } else if (INDEX && a < p.a_hi) {  // no keys (n <= l cannot pass setup_index): holes
      if (p.key0) p.key0[a] = kEmpty;
      if constexpr (G > 1 || kWinGroups == 1) {
        if (p.p0runs) p.p0runs[a] = make_ulonglong2(0, kFlatHole);
      }
      if constexpr (KEYREC) {
        for (int o = 0; o < 4; ++o) {
          p.key_bk[key_seg(o) * p.key_n + a - p.key_lo] = 0;
          p.key_ent[key_seg(o) * p.key_n + a - p.key_lo] = kEmpty;
        }
      }
    }
   }
   if constexpr (RECV) recv_insert(r_per);  // this window's share of the received keys
  }
  if constexpr (RECV) recv_insert(~0ull);  // (what is left: a wavefront with fewer windows)
  uint64_t c = cur[0];
#pragma unroll
  for (int j = 1; j < G; ++j) c = lane == j ? cur[j] : c;
  if (lane < G) p.run_cnt[gw * G + lane] = c;
  if constexpr (KEYREC || RECV) {
    if (p.dst_cnt && (uint32_t)lane < (uint32_t)G * p.dst_ranks)  // region gw G + j, rank d at [(gw G + j) P + d]
      p.dst_cnt[(gw * G + lane / p.dst_ranks) * p.dst_ranks + lane % p.dst_ranks] = dcnt;
  }
}

// ---------------------------------------------------------------------------
// Run staging of the register scan: runs are staged in an LDS ring of 64-bit
// metas (ballot + mbcnt), then flushed 64 at a time with every lane busy: the
// minimizer m-mer is re-extracted from the owner lane's registers
// (ds_bpermute), hashed (mix64 -> bucket | fingerprint) and written as one
// coalesced 16-B record per lane into this wavefront's region.
template <int MAXW, int RING = kStageRing, bool FROM_MEM = false>
struct RunStage {
  const ScanParams& p;
  uint64_t* s_buf;
  ulonglong2* region;
  int lane, msh;
  uint64_t nbmask;
  uint64_t cursor = 0;
  uint32_t head = 0, nbuf = 0;  // staged metas: ring [head, head + nbuf) (wavefront-uniform)
  uint32_t dcnt = 0;            // p.dst_cnt: lane d counts the stored runs bound for rank d

  __device__ RunStage(const ScanParams& pp, uint64_t* buf, ulonglong2* reg, int ln)
      : p(pp), s_buf(buf), region(reg), lane(ln), msh(64 - 2 * pp.m), nbmask((1ULL << pp.nb_log2) - 1) {}

  __device__ __forceinline__ void put(bool flag, uint64_t meta) {
    const uint64_t bal = __ballot(flag);
    if (flag) s_buf[(head + nbuf + lane_prefix(bal)) & (RING - 1)] = meta;
    nbuf += (uint32_t)__popcll(bal);
  }

  // hash + write the first k (<= 64) staged runs; rw = this lane's read words,
  // a0 = read index of lane 0 (every staged run belongs to a lane of the group)
  __device__ void flush(uint32_t k, const uint64_t* rw, uint64_t a0) {
    wave_sync();
    bool flag = (uint32_t)lane < k;
    uint64_t v = 0, meta = 0;
    if (flag) meta = s_buf[(head + lane) & (RING - 1)];
    if constexpr (MAXW <= 8 && !FROM_MEM) {
      const int pos = (int)((meta >> 32) & 1023u), wi = pos >> 5;
      const int src = flag ? (int)((uint32_t)meta - (uint32_t)a0) : lane;
      uint64_t w0 = 0, w1 = 0;
#pragma unroll
      for (int kk = 0; kk <= MAXW; ++kk) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)rw[kk]);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)(rw[kk] >> 32));
        const uint64_t x = ((uint64_t)hi << 32) | lo;
        w0 = wi == kk ? x : w0;
        w1 = wi + 1 == kk ? x : w1;
      }
      if (flag) v = mix64(funnel(w0, w1, (pos & 31) << 1) >> msh);
    } else if (flag) {
      const uint64_t* g2 = p.words + (meta & 0xFFFFFFFFull) * slot_words(MAXW);
      const int pos = (int)((meta >> 32) & 1023u), wi = pos >> 5;
      v = mix64(funnel(g2[wi], wi + 1 < slot_words(MAXW) ? g2[wi + 1] : 0ull, (pos & 31) << 1) >> msh);
    }
    if (flag) flag = owned(v & nbmask, p.nb_log2, p.rank, p.nranks);
    const uint64_t bal = __ballot(flag);
    bool stored = false;
    if (flag) {
      const uint64_t at = cursor + lane_prefix(bal);
      stored = at < p.run_cap;
      if (stored) region[at] = make_ulonglong2(v, meta);
    }
    cursor += (uint64_t)__popcll(bal);
    if (p.dst_cnt) {  // k_part's destination rule (OWN_BUCKET), one ballot per rank
      const uint32_t d = (uint32_t)(((v & nbmask) * p.dst_ranks) >> p.nb_log2);
      for (uint32_t dd = 0; dd < p.dst_ranks; ++dd) {
        const uint32_t c = (uint32_t)__popcll(__ballot(stored && d == dd));
        dcnt += (uint32_t)lane == dd ? c : 0u;
      }
    }
    head += k;
    nbuf -= k;
    wave_sync();
  }

  // the region count (and its per-rank split)
  __device__ void finish(uint64_t gw) {
    if (lane == 0) p.run_cnt[gw] = cursor;
    if (p.dst_cnt && (uint32_t)lane < p.dst_ranks) p.dst_cnt[gw * p.dst_ranks + lane] = dcnt;
  }
};

constexpr int kRegW = 32;       // largest w (= h - m + 1) of the register scan
constexpr int kStageEvery = 6;  // register scan: flush check every kStageEvery bases (< 64 + 6 * 64 staged)

// Window minimizers of every source read, one read per lane, with the sliding
// minimum kept in REGISTERS: van Herk / Gil-Werman over blocks of w positions
// (prefix minimum of the current block in a register, suffix minima of the
// previous block in S[0..w), overwritten by the current block's keys exactly
// behind the step that last reads them).  The block loop is unrolled by
// kRegW with a uniform exit at u = w, so every S index is static and no LDS
// or scratch is touched per base (the LDS version, k_scan, stays for w >
// kRegW).  Same windows, keys and runs as k_scan (OverlapGraph.cpp:534-537):
// window j covers m-mers t in [j, j + w - 1]; key = order_key | t; a run ends
// where the minimizer position changes.
// INDEX (HashTable::insertDataset / hashRead, HashTable.cpp:50-104): o = 0 is
// window j = 0 and o = 1 window j = n - h of this same scan (the key's offset i
// is t shifted by a constant, so the argmin is the same); o = 2 / 3 (the
// reverse strand's keys) come from a w-step pass of rolled reverse-complement
// m-mers after the read's scan; then the four CAS inserts (or key records).
template <int MAXW, bool INDEX>
__global__ __launch_bounds__(kBlock) void k_scan_reg(ScanParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = p.h, m = p.m, w = p.w;
  const int msh = 64 - 2 * m;
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const uint64_t ngroups = (p.a_hi - p.a_lo + kWave - 1) / kWave;
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  RunStage<MAXW> st(p, smem + (size_t)wv * kStageRing, p.runs + gw * p.run_cap, lane);
  constexpr int kRwLoad = MAXW + 1 <= slot_words(MAXW) ? MAXW + 1 : slot_words(MAXW);
  uint64_t nx[MAXW + 1];  // the read words of this lane's next group (software pipelined)
  {
    const uint64_t a = p.a_lo + gw * kWave + lane;
    const uint64_t* gs = p.words + (a < p.a_hi && gw < ngroups ? a : 0) * slot_words(MAXW);
#pragma unroll
    for (int k = 0; k <= MAXW; ++k) nx[k] = k < kRwLoad ? gs[k] : 0;
  }

  for (uint64_t grp = gw; grp < ngroups; grp += nw) {
    const uint64_t a = p.a_lo + grp * kWave + lane;
    int n = 0;
    if (a < p.a_hi) {
      n = (int)p.len[a];
      if (n && p.super && p.super[a]) n = 0;
    }
    const int J = n - h - 1;                  // windows j = 1 .. J (:534)
    const int tend = J >= 1 ? J + w - 1 : -1;  // last m-mer position a scanned window uses
    const int tlast = INDEX ? (n ? n - m : -1) : tend;  // INDEX: up to window j = n - h (key o = 1)
    int tmax = tlast;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tmax = max(tmax, __shfl_xor(tmax, d));
    tmax = __builtin_amdgcn_readfirstlane(tmax);
    uint64_t rw[MAXW + 1];
#pragma unroll
    for (int k = 0; k <= MAXW; ++k) rw[k] = nx[k];
    {  // the next group's words load behind this group's scan
      const uint64_t an = a + (uint64_t)nw * kWave;
      const uint64_t* gs = p.words + (an < p.a_hi ? an : 0) * slot_words(MAXW);
#pragma unroll
      for (int k = 0; k <= MAXW; ++k) nx[k] = k < kRwLoad ? gs[k] : 0;
    }
    const uint64_t a0 = p.a_lo + grp * kWave;
    uint32_t S[kRegW + 1];
#pragma unroll
    for (int u = 0; u <= kRegW; ++u) S[u] = 0xFFFFFFFFu;
    uint64_t mm = rw[0] >> msh;  // m-mer at t = 0
    uint64_t cwd = 0;            // read word holding base t + m (refilled at word edges)
    uint32_t pm = 0, kw0 = 0xFFFFFFFFu, kw1 = 0xFFFFFFFFu;  // prefix min; INDEX: windows j = 0 and n - h
    int last = 0, jlo = 1;
    const int t1 = n - m;  // this lane's key-o=1 window position (INDEX)
    for (int t0 = 0; t0 <= tmax; t0 += w) {
#pragma unroll
      for (int u = 0; u < kRegW; ++u) {
        const int t = t0 + u;
        if (u >= w || t > tmax) continue;  // uniform; no break, so the loop unrolls fully
        const int x = t + m;  // base rolled in after this step
        if (t == 0 || (x & 31) == 0) {
          const int xi = x >> 5;
          uint64_t c = rw[0];
#pragma unroll
          for (int k = 1; k <= MAXW; ++k) c = xi == k ? rw[k] : c;
          cwd = c;
        }
        const uint32_t key = order_key(mm) | (uint32_t)t;
        pm = u == 0 ? key : (key < pm ? key : pm);
        const uint32_t win = S[u + 1] < pm ? S[u + 1] : pm;  // S[w] stays all ones
        S[u] = key;
        if (t >= w - 1) {
          const int j = t - w + 1;
          const int pos = (int)(win & 1023u);
          if (INDEX) {
            if (j == 0) kw0 = win;
            if (t == t1) kw1 = win;
          }
          const bool act = j >= 1 && t <= tend;
          const bool emit = act && j > 1 && pos != last;
          st.put(emit, run_meta(a, last, jlo, j - 1));
          if (emit) jlo = j;
          if (act) last = pos;
        }
        mm = ((mm << 2) | ((cwd >> (62 - 2 * (x & 31))) & 3u)) & mmask;
        if (u % kStageEvery == kStageEvery - 1)  // a few flush sites per block (code size)
          while (st.nbuf >= (uint32_t)kWave) st.flush(kWave, rw, a0);
      }
      while (st.nbuf >= (uint32_t)kWave) st.flush(kWave, rw, a0);
      // suffix minima of this block in place: S[u] = min over [u, w)
#pragma unroll
      for (int u = kRegW - 2; u >= 0; --u)
        if (u < w - 1) S[u] = S[u + 1] < S[u] ? S[u + 1] : S[u];
    }
    st.put(tend >= 0, run_meta(a, last, jlo, J));  // each read's last run
    while (st.nbuf) st.flush(st.nbuf < (uint32_t)kWave ? st.nbuf : (uint32_t)kWave, rw, a0);
    if constexpr (INDEX) {  // key records of o = 0 / 1, o-major (k_rc_keys writes o = 2 / 3)
      if (a < p.a_hi) {
        const int p0 = (int)(kw0 & 1023u), p1 = (int)(kw1 & 1023u);
        const uint64_t nbm = (1ULL << p.nb_log2) - 1;
        uint64_t c0 = kEmpty, c1 = kEmpty;  // (no keys: holes, n <= l cannot pass setup_index)
        uint32_t b0 = 0, b1 = 0;
        if (n) {
          const uint64_t v0 = mix64(funnel(rw[0], rw[1], p0 << 1) >> msh);  // p0 < w <= 32
          const uint64_t v1 = mix64(ext_reg<MAXW>(rw, p1) >> msh);
          b0 = (uint32_t)(v0 & nbm);
          b1 = (uint32_t)(v1 & nbm);
          c0 = make_entry(v0, p.nb_log2, p0, 0, (uint32_t)a, n);
          c1 = p.skip_o1 ? kEmpty : make_entry(v1, p.nb_log2, p1 - (n - h), 1, (uint32_t)a, n);
        }
        const uint64_t ka = a - p.key_lo;
        p.key_bk[ka] = b0;
        p.key_ent[ka] = c0;
        p.key_bk[3 * p.key_n + ka] = b1;  // (key_seg(1) = 3)
        p.key_ent[3 * p.key_n + ka] = c1;
      }
    }
  }
  st.finish(gw);
}

// The partner's slot as it lies in memory: words 0 .. MAXW-1 (plus one pad
// word), fetched as 16-B pieces of one aligned line.
template <int MAXW>
__device__ __forceinline__ void load_slot(const uint64_t* words, uint32_t bid, uint64_t* y) {
  const uint64_t* g = words + (uint64_t)bid * slot_words(MAXW);
  if (slot_words(MAXW) < 2) {
    y[0] = g[0];
    y[1] = 0;
  } else {
    const ulonglong2* gp = reinterpret_cast<const ulonglong2*>(g);
#pragma unroll
    for (int k = 0; k < (MAXW + 1) / 2; ++k) {
      const ulonglong2 x = gp[k];
      y[2 * k] = x.x;
      if (2 * k + 1 <= MAXW) y[2 * k + 1] = x.y;
    }
    if (MAXW % 2 == 0) y[MAXW] = 0;
  }
}

// Key records of the reverse strand's keys (hashRead, HashTable.cpp:88-104),
// one thread per read: o = 3 (R[n-h, n) = rc F[0, h): m-mer i = rc of F's at
// t = w-1-i) and o = 2 (R[0, h) = rc F[n-h, n): m-mer i = rc of F's at
// t = n-m-i), both rolled towards smaller t, one base per step; the same
// minimizer rule (order_key | i, smallest wins) as key_minimizer.  Written to
// key_bk / key_ent[key_seg(o) * key_n + a], o = 2, 3 (k_scan_reg<INDEX> writes o = 0, 1).
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_rc_keys(ScanParams p) {
  const uint64_t a = p.a_lo + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (a >= p.a_hi) return;
  const int h = p.h, m = p.m, w = p.w, n = p.len[a];
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  uint64_t rw[MAXW + 1];
  load_slot<MAXW>(p.words, (uint32_t)a, rw);
  uint32_t kb3 = 0xFFFFFFFFu, kb2 = 0xFFFFFFFFu;
  uint64_t mb3 = 0, mb2 = 0;
  const uint64_t Aw = ext_reg<MAXW>(rw, n - h);                      // F[n-h, n-h+32)
  uint64_t r3 = rc_word(funnel(rw[0], rw[1], 2 * (w - 1))) & mmask;  // rc(F[w-1, w-1+m))
  uint64_t r2 = rc_word(ext_reg<MAXW>(rw, n - m)) & mmask;          // rc(F[n-m, n))
  for (int i = 0; i < w; ++i) {
    const uint32_t k3 = order_key(r3) | (uint32_t)i, k2 = order_key(r2) | (uint32_t)i;
    if (k3 < kb3) { kb3 = k3; mb3 = r3; }
    if (k2 < kb2) { kb2 = k2; mb2 = r2; }
    const int t3 = w - 2 - i;  // F base entering at t - 1: F[t3] (o = 3), F[n-h + t3] = F[n-m-1-i] (o = 2)
    if (t3 >= 0) {
      r3 = ((r3 << 2) | (3u - ((rw[0] >> (62 - 2 * t3)) & 3u))) & mmask;
      r2 = ((r2 << 2) | (3u - ((Aw >> (62 - 2 * t3)) & 3u))) & mmask;
    }
  }
  const uint64_t v2 = mix64(mb2), v3 = mix64(mb3);
  const uint64_t nbm = (1ULL << p.nb_log2) - 1;  // (bucket, entry) records, o-major
  const uint64_t ka = a - p.key_lo;
  p.key_bk[p.key_n + ka] = n ? (uint32_t)(v2 & nbm) : 0u;  // (key_seg(2) = 1, key_seg(3) = 2)
  p.key_ent[p.key_n + ka] = n ? make_entry(v2, p.nb_log2, (int)(kb2 & 1023u), 2, (uint32_t)a, n) : kEmpty;
  p.key_bk[2 * p.key_n + ka] = n ? (uint32_t)(v3 & nbm) : 0u;
  p.key_ent[2 * p.key_n + ka] = n ? make_entry(v3, p.nb_log2, (int)(kb3 & 1023u), 3, (uint32_t)a, n) : kEmpty;
}

// checkOverlap's string compare (OverlapGraph.cpp:354-383) on packed words:
// the L partner bases [y0, y0+L) against the source bases [x0, x0+L) of the
// forward strand, or of the reverse strand when rcA.  Partner words are used in
// place (word k holds partner bases [32k, 32k+32)); the source side is
// extracted at the matching shift from the LDS-staged words (stride S), so no
// register array is indexed at run time.  Returns the XOR of the compared
// bases (0 = equal).
template <int MAXW, int S>
__device__ __forceinline__ uint64_t overlap_diff(const uint64_t* f1, int n1, int x0, int y0, int L, bool rcA,
                                                 const uint64_t* y) {
  uint64_t diff = 0;
#pragma unroll
  for (int k = 0; k < MAXW; ++k) {
    const int lo = max(y0 - 32 * k, 0), hi = min(y0 + L - 32 * k, 32);
    if (hi > lo) {
      const int s = x0 - y0 + 32 * k;  // source position of partner base 32k
      const uint64_t av = rcA ? rc_word(ext_fwd<S>(f1, n1 - s - 32)) : ext_fwd<S>(f1, s);
      const uint64_t msk = (lo ? (~0ULL >> (2 * lo)) : ~0ULL) & (hi < 32 ? ~(~0ULL >> (2 * hi)) : ~0ULL);
      diff |= (av ^ y[k]) & msk;
    }
  }
  return diff;
}

struct ProbeParams {
  const uint64_t* words;
  const uint16_t* len;
  int h, m;
  uint32_t nb_log2;
  uint32_t rank, nranks;
  uint64_t cell_lo, cell_n;       // local bucket range of the cell table (IndexParams)
  uint32_t cell_shift;            // cell = (bucket - cell_lo) >> cell_shift (the exchange mode's discovery index)
  const uint64_t* cells;
  const uint32_t* cbits;          // discovery: contained slots as bits (mg_ctx::d_cbits; nullptr: none contained)
  unsigned long long* superkey;   // CONTAIN: max over containers of (len << 32 | ~index)
  const ulonglong2* runs;
  const unsigned long long* run_cnt;
  uint64_t run_cap;
  uint64_t run_regions;           // probe wavefront r consumes run regions r, r + nw, r + 2 nw, ... < run_regions
  // vsplit > 1 (not in the exchange split probe): every run region is walked as
  // vsplit VIRTUAL regions (consecutive parts of its records, whole batch
  // strides each), so the probe's waves get an equal count of them when the
  // scan's region count is not a multiple of the probe's waves
  uint32_t vsplit;
  const uint32_t* src_super;      // runs of sources with superReadID != 0 are dropped (:548; nullptr: none)
  uint64_t src_lo, src_hi;        // only runs of sources in [src_lo, src_hi) (src_hi = 0: all)
  uint32_t* rows;                 // 3 dwords per row (mg_edge); one region per wavefront
  unsigned long long* reg_cnt;    // [waves] rows produced by each wavefront (may exceed reg_cap)
  uint64_t reg_cap;
  int uniform_len;                // every read has this length (0: lengths differ)
  unsigned long long* stats;      // optional [kSegs*4]: runs probed, entries scanned, partners fetched, rows
  int phase_limit;                // diagnostics: 4 no probe, 5 + cell loads, 6 + filter, 7 full
  int halving_low;                // option "halving" = 1: keep o=2/3 pairs at the lower ID (else rc_side_keeps)
  // the halving rule's read numbers: slots (nullptr) when every context that
  // shares the work has the same slot order (one context; the exchange mode's
  // ranks, whose layouts are identical), reference IDs (slot -> ID - 1) for
  // source-range shards, whose layouts group their own range
  const uint32_t* halving_id;
  int contain_even;               // CONTAIN: drop o = 1/3 hits (k_prefix_contain finds the s = 0 containments)
  int contain_minlen;             // CONTAIN (with contain_even): drop runs whose first window jlo > n1 - minlen
  int contain_prune;              // CONTAIN: skip a candidate whose container cannot raise the superkey
  int contain_skip;               // CONTAIN: skip runs of sources already contained (their superkey != 0)
  int compact;                    // park the live items of sparse run batches (filled batches only)
  int share;                      // a block's wavefronts share its regions batch by batch (probe_share)
  int append;                     // rows go after the ones a previous launch left in each region (reg_cnt)
  // a split exchange probe walks one part of the slot-layout regions (K per
  // peer slot and round): part 1 = peer rm_me's, part 2 = every other peer's;
  // logical region L of the part -> physical region (run_cnt / runs index)
  int rm_part;
  uint32_t rm_P, rm_me;
  uint64_t rm_K;
  const uint32_t* id;             // slot -> reference ID - 1 (nullptr: ID order); rows and superkeys carry IDs
  // DCNT (exchange-mode discovery): rows stored per destination rank (the
  // source ID's owner, k_part's OWN_SRC rule) into dst_cnt[gw * dst_ranks + d]
  unsigned long long* dst_cnt;
  uint32_t dst_ranks;
  uint64_t n_ids;
  double inv_n_ids;
};

// Which side of a self-symmetric (o = 2/3) discovery pair {a, b} emits it:
// exactly one of rc_side_keeps(a, b), rc_side_keeps(b, a) holds for a != b,
// and a self pair is kept.  Alternating by the parity of a + b (instead of
// "b >= a") spreads the pairs evenly over the source IDs, so source-range
// shards (bench --multi replicated) carry even verification loads.
__device__ __forceinline__ bool rc_side_keeps(uint32_t a, uint32_t b) {
  return a == b || (((a ^ b) & 1u) ? b > a : b < a);
}

template <int MAXW>
struct ProbeLds {
  static constexpr int CAND = 3 * kWave;  // candidate list (verified 64 at a time)
  static constexpr int PEND = 2 * kWave;  // chained probe items waiting for a batch of their own
  static constexpr size_t o_a = 0;                                      // [MAXW+1][64] u64 source words
  static constexpr size_t o_pk = o_a + (size_t)(MAXW + 1) * kWave * 8;  // [PEND] u64 bucket | fp << 32
  static constexpr size_t o_pm = o_pk + PEND * 8;                       // [PEND] u64 run meta
  static constexpr size_t o_cb = o_pm + PEND * 8;                       // [CAND] u32 partner
  static constexpr size_t o_ci = o_cb + CAND * 4;                       // [CAND] u32 o << 30 | (n2 - 1) << 10 | j
  static constexpr size_t o_ca = o_ci + CAND * 4;                       // [CAND] u32 source read
  static constexpr size_t bytes = o_ca + CAND * 4;
};

// Probe wavefront r consumes its run regions in batches of 64 probe items (one
// per lane).  An item is a run (bucket, fingerprint, read, minimizer position
// p, window range [jlo, jhi]) or the continuation of a chained cell.  The cell
// load of the NEXT batch is issued before the current batch is processed, so
// one random 64-B line per lane is always in flight behind the work.  Entries
// are exact candidates when the fingerprint matches, j = p - q lies in the
// run's window range (the window's minimizer is this very m-mer at offset q)
// and the halving rule keeps them.  Candidates go to an LDS list
// (ballot + mbcnt per slot) and are verified one per lane against the
// partner's slot in HBM; a full cell's chain flag turns the lane's item into a
// pending item (LDS) that a later batch probes at the next cell.
// Waves per SIMD asked of the register allocator: 4 (128 VGPRs) where the
// probe fits them without spilling (reads up to 5 words), else its own choice
// (3 waves at 129-143 VGPRs).  MG_PROBE_WAVES overrides (A/B builds).
#ifndef MG_PROBE_WAVES
#define MG_PROBE_WAVES (MAXW <= 5 ? 4 : 1)
#endif
// the owner rank of 1-based reference ID x1 (k_part's OWN_SRC rule,
// (x1 P - 1) / n), the quotient estimated in double and corrected
__device__ __forceinline__ uint32_t id_owner(uint32_t x1, uint32_t P, uint64_t n, double inv_n) {
  const uint64_t x = (uint64_t)x1 * P - 1;
  uint64_t q = (uint64_t)((double)x * inv_n);
  while (q * n > x) --q;
  while ((q + 1) * n <= x) ++q;
  return (uint32_t)q;
}

// DCNT (exchange mode, P > 1): the rows each wavefront stores are also counted
// per destination rank, so their routing needs no count pass (a separate
// instantiation: the fused path's probe keeps its registers)
// XCHG: the exchange mode's split discovery probe (region remap rm_*, rows
// appended after an earlier launch's); DCNT (exchange only) includes it.  A
// separate instantiation: the remap's divides cost the fused probes registers
// (C5 containment 126 -> 130 VGPRs, one wave per SIMD less, when it was shared)
template <int MAXW, bool CONTAIN, bool DCNT = false, bool XCHG = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(MG_PROBE_WAVES))) void k_probe(ProbeParams p) {
  constexpr bool kXchg = DCNT || XCHG;
  using PL = ProbeLds<MAXW>;
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  __shared__ unsigned int s_dc[DCNT ? kWavesPerBlock * kWave : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if constexpr (DCNT) s_dc[wv * kWave + lane] = p.append && (uint32_t)lane < p.dst_ranks ?
                                                   (unsigned)p.dst_cnt[(blockIdx.x * kWavesPerBlock + wv) * p.dst_ranks + lane]
                                                   : 0u;
  unsigned char* base = reinterpret_cast<unsigned char*>(smem) + (size_t)wv * PL::bytes;
  uint64_t* s_a = reinterpret_cast<uint64_t*>(base + PL::o_a);
  uint64_t* s_pk = reinterpret_cast<uint64_t*>(base + PL::o_pk);
  uint64_t* s_pm = reinterpret_cast<uint64_t*>(base + PL::o_pm);
  uint32_t* s_cb = reinterpret_cast<uint32_t*>(base + PL::o_cb);
  uint32_t* s_ci = reinterpret_cast<uint32_t*>(base + PL::o_ci);
  uint32_t* s_ca = reinterpret_cast<uint32_t*>(base + PL::o_ca);
  const int h = p.h;
  const uint64_t nbmask = (1ULL << p.nb_log2) - 1;
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t nwp = (uint64_t)gridDim.x * kWavesPerBlock;
  const uint32_t seg = (uint32_t)(gw & (kSegs - 1));
  uint32_t* const region = p.rows + gw * p.reg_cap * 3;
  uint64_t cursor = (kXchg && !CONTAIN && p.append) ? p.reg_cnt[gw] : 0;  // (the second part of a split probe)
  uint32_t ncand = 0, npend = 0;
  // diagnostics (p.stats): wavefront sum of a per-lane count into counter i
  // (runs probed, entries scanned, partners fetched, rows); call converged.
  // No per-lane counters stay live across the loop (registers: occupancy)
  auto stat = [&](int i, uint32_t v) {
    if (p.stats) {
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
      if (lane == 0) atomicAdd(&p.stats[seg * 4 + i], (unsigned long long)v);
    }
  };

  // verify the first nc (<= 64) candidates of the list, one per lane
  auto verify = [&](uint32_t nc) {
    const bool have = (uint32_t)lane < nc;
    int nrec = 0;
    uint32_t r0 = 0, r1 = 0, r2 = 0, t0 = 0, t1 = 0, t2 = 0;
    int n1 = 0, n2 = 0, o = 0, j = 0;
    uint32_t bid = 0, sa = 0;
    bool cond = false, rcA = false;
    int x0 = 0, y0 = 0, L = 0;
    uint64_t y[MAXW + 1];
    if (have) {
      bid = s_cb[lane];
      const uint32_t info = s_ci[lane];
      sa = s_ca[lane];
      o = (int)(info >> 30);
      j = (int)(info & 1023u);
      n1 = p.uniform_len ? p.uniform_len : (int)p.len[sa];
      n2 = p.uniform_len ? p.uniform_len : (int)((info >> 10) & 1023u) + 1;
      if (!CONTAIN) {
        if (o == 0) {        // F1[j, n1) == F2[0, L)
          L = n1 - j; cond = L < n2; x0 = j; y0 = 0; rcA = false;
        } else if (o == 2) { // F1[j, n1) == R2[0, L)  <=>  R1[0, L) == F2[n2-L, n2)
          L = n1 - j; cond = L < n2; x0 = 0; y0 = n2 - L; rcA = true;
        } else {             // F1[0, L) == R2[n2-L, n2)  <=>  R1[n1-L, n1) == F2[0, L)
          L = j + h; cond = j <= n2 - h; x0 = n1 - L; y0 = 0; rcA = true;
        }
      } else {
        int s;
        cond = n1 > n2;
        if (o == 0 || o == 2) {
          cond = cond && (j <= n1 - n2);
          s = j;
        } else {
          // o = 1/3 (the partner's suffix key) place the partner at offset
          // s = j - (n2 - h) >= 0, but every s >= 1 is also found by its o = 0/2
          // hit at window j = s (checkOverlapForContainedRead, :302-340, both
          // ranges end at s = n1 - n2), and the atomicMax result depends only on
          // the pair: only s = 0 (a prefix of the container) needs this side
          cond = cond && (j == n2 - h);
          s = 0;
        }
        L = n2;
        y0 = 0;
        rcA = o >= 2;
        x0 = rcA ? n1 - s - n2 : s;
      }
    }
    // partner slot first (the long-latency random load: its words in 16-B
    // pieces of one aligned line) and both reference IDs, then stage the source
    uint32_t ida = sa, idb = bid;
    if (CONTAIN && p.contain_prune && cond) {
      // atomicMax(len << 32 | ~id) would be a no-op when the partner already
      // holds a key >= this container's: skip the slot load and the compare
      // (keys only grow, so a stale view only prunes less)
      const uint32_t ia = p.id ? p.id[sa] : sa;
      const unsigned long long want = ((unsigned long long)n1 << 32) | (0xFFFFFFFFu - ia);
      cond = __hip_atomic_load(&p.superkey[bid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want;
    }
    if (cond) {
      load_slot<MAXW>(p.words, bid, y);
      if (p.id) {
        ida = p.id[sa];
        idb = p.id[bid];
      }
    }
    if (have) {  // the source's words, 16 B per load where the slot allows
      const uint64_t* g = p.words + (uint64_t)sa * slot_words(MAXW);
      if constexpr (slot_words(MAXW) < 2) {
        s_a[lane] = g[0];
      } else {
        const ulonglong2* gp = reinterpret_cast<const ulonglong2*>(g);
#pragma unroll
        for (int k = 0; k < (MAXW + 1) / 2; ++k) {
          const ulonglong2 x = gp[k];
          s_a[2 * k * kWave + lane] = x.x;
          if (2 * k + 1 < MAXW) s_a[(2 * k + 1) * kWave + lane] = x.y;
        }
      }
      s_a[MAXW * kWave + lane] = 0;
    }
    wave_sync();
    uint32_t nhit = 0;
    if (cond) {
      const uint64_t diff = overlap_diff<MAXW, kWave>(s_a + lane, n1, x0, y0, L, rcA, y);
      if (diff == 0) {
        if (CONTAIN) {
          atomicMax(&p.superkey[bid], ((unsigned long long)n1 << 32) | (0xFFFFFFFFu - ida));
          nhit = 1;
        } else {  // (:548 a contained read2 was dropped at listing, p.cbits)
          // orientation/offset switch (:550-557) and the twin (:409-412, :841-855)
          const uint32_t orient = (o == 0) ? 3u : (o == 2 ? 2u : 1u);
          const uint32_t off = (o == 3) ? (uint32_t)(n1 - h - j) : (uint32_t)j;
          const uint32_t torient = (orient == 3u) ? 0u : orient;
          const uint32_t toff = (uint16_t)(n2 + off - n1);
          r0 = ida + 1; r1 = idb + 1; r2 = (orient << 16) | off;
          t0 = idb + 1; t1 = ida + 1; t2 = (torient << 16) | toff;
          nrec = (bid == sa && o == 0) ? 4 : 2;  // self o=0 hit also stands for its o=1 twin
          nhit = (uint32_t)nrec;
        }
      }
    }
    stat(2, cond ? 1u : 0u);
    stat(3, nhit);
    if (!CONTAIN) {
      const uint64_t b2 = __ballot(nrec >= 2), b4 = __ballot(nrec == 4);
      const uint32_t tot = 2u * (uint32_t)(__popcll(b2) + __popcll(b4));
      if (tot) {
        if (cursor + tot <= p.reg_cap) {
          if constexpr (DCNT) {
            if (nrec) {  // nrec / 2 rows to the source's owner, as many twins to the partner's
              atomicAdd(&s_dc[wv * kWave + id_owner(r0, p.dst_ranks, p.n_ids, p.inv_n_ids)], (unsigned)nrec / 2);
              atomicAdd(&s_dc[wv * kWave + id_owner(t0, p.dst_ranks, p.n_ids, p.inv_n_ids)], (unsigned)nrec / 2);
            }
          }
          const uint32_t pr = 2u * (lane_prefix(b2) + lane_prefix(b4));
          uint3* d = reinterpret_cast<uint3*>(region + (cursor + pr) * 3);
          for (int rr = 0; rr < nrec; rr += 2) {
            d[0] = make_uint3(r0, r1, r2);
            d[1] = make_uint3(t0, t1, t2);
            d += 2;
          }
        }
        cursor += tot;  // keeps counting past the capacity: the host resizes and reruns
      }
    }
    wave_sync();
  };

  // ---- run stream: this wavefront's run regions, 64 records per batch
  uint32_t rg = 0;
  uint64_t rpos = 0, rcnt = 0;
  const ulonglong2* rbase = p.runs;
  const uint32_t vsplit = kXchg ? 1u : p.vsplit;
  const uint64_t rlimit = p.run_regions * vsplit;
  // share (option probe_share): the block's 4 wavefronts walk the SAME regions
  // (4 b .. 4 b + 3, then + nwp, ...) and take every 4th batch of each, so a
  // block probes one scan group of 64 neighbouring reads at a time and their
  // shared cells and partner slots stay in its CU's L1 and its XCD's L2;
  // otherwise wavefront gw walks regions gw, gw + nwp, ...
  const bool share = p.share != 0;
  const uint64_t rstep = share ? (uint64_t)kWavesPerBlock * kWave : (uint64_t)kWave;
  auto reg_of = [&](uint32_t r) -> uint64_t {
    return share ? (uint64_t)(r >> 2) * nwp + (uint64_t)blockIdx.x * kWavesPerBlock + (r & 3u)
                 : gw + (uint64_t)r * nwp;
  };
  auto open_region = [&](uint32_t r) {
    uint64_t reg = reg_of(r);
    uint32_t part = 0;
    if (!kXchg && vsplit > 1) {  // virtual region: part `part` of run region reg / vsplit (wavefront-uniform)
      const uint32_t v = (uint32_t)reg;
      reg = v / vsplit;
      part = v - (uint32_t)reg * vsplit;
    }
    if (kXchg && p.rm_part) {  // (wavefront-uniform; once per region)
      const uint64_t blk = reg / p.rm_K, k = reg - blk * p.rm_K;
      uint64_t t = blk, sp = p.rm_me;
      if (p.rm_part == 2) {
        t = blk / (p.rm_P - 1);
        sp = blk - t * (p.rm_P - 1);
        sp += sp >= p.rm_me ? 1 : 0;
      }
      reg = (t * p.rm_P + sp) * p.rm_K + k;
    }
    rbase = p.runs + reg * p.run_cap;
    const uint64_t c = p.run_cnt[reg];
    rcnt = c < p.run_cap ? c : p.run_cap;
    uint64_t lo = 0;
    if (!kXchg && vsplit > 1) {  // records [lo, hi) of the region, lo a whole number of batch strides
      const uint32_t c32 = (uint32_t)rcnt, st = (uint32_t)rstep;
      const uint32_t per = ((c32 + vsplit - 1) / vsplit + st - 1) / st * st;
      lo = min((uint64_t)part * per, rcnt);
      rcnt = min(lo + per, rcnt);
    }
    rpos = lo + (share ? (uint64_t)wv * kWave : 0);
  };
  // skip to the next non-empty batch position; false once the regions are exhausted
  auto hbm_settle = [&]() -> bool {
    while (rpos >= rcnt) {
      if (reg_of(rg + 1) >= rlimit) return false;
      open_region(++rg);
    }
    return true;
  };
  // next batch: pending items first once 64 are waiting, else the run stream
  // (prefetched one batch ahead), else the last pending items
  ulonglong2 rec_pf = make_ulonglong2(0, 0);
  bool pf_ok = false, pf_any = false;
  // (re)load the run batch at the stream position, unconditionally and outside
  // any branch: no branch-merged value ever waits on a load in flight
  auto hbm_fetch = [&]() {
    const uint64_t k = rpos + (uint64_t)lane;
    pf_ok = pf_any && k < rcnt;
    rec_pf = rbase[pf_ok ? k : 0];
  };

  auto take_item = [&](uint64_t& key, uint64_t& meta, bool& valid) -> bool {
   while (true) {
    if (npend >= (uint32_t)kWave) {
      npend -= kWave;
      key = s_pk[npend + lane];
      meta = s_pm[npend + lane];
      valid = true;
      return true;
    }
    if (pf_any) {
      valid = pf_ok && rec_pf.y != kFlatHole;
      meta = rec_pf.y;
      const uint64_t bucket = rec_pf.x & nbmask;
      const uint32_t fpv = (uint32_t)(rec_pf.x >> p.nb_log2) & kFpMask;
      if (valid && (p.src_super || p.src_hi)) {  // contained or foreign sources contribute no windows
        const uint32_t ra = (uint32_t)meta;
        if ((p.src_super && p.src_super[ra]) || (p.src_hi && (ra < p.src_lo || ra >= p.src_hi))) valid = false;
      }
      // containment: read2 sits at s = j <= n1 - n2 <= n1 - minlen, so a run
      // whose first window lies beyond that finds nothing (o = 1/3, the s = 0
      // side, is k_prefix_contain's when contain_even)
      if (CONTAIN && valid && (p.contain_minlen || p.contain_skip)) {
        const uint32_t ra = (uint32_t)meta;
        const int n1 = p.uniform_len ? p.uniform_len : (int)p.len[ra];
        if (p.contain_minlen && (int)((meta >> 42) & 1023u) > n1 - p.contain_minlen) valid = false;
        // a source that is itself contained (in a longer read C) never holds
        // a partner's final superReadID: every read2 it contains is also in
        // C, which is longer, and the longest container is never contained
        if (p.contain_skip && valid &&
            __hip_atomic_load(&p.superkey[ra], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
          valid = false;
      }
      key = (valid ? (bucket - p.cell_lo) >> p.cell_shift : 0) | ((uint64_t)fpv << 32);
      stat(0, valid ? 1u : 0u);
      rpos += rstep;
      pf_any = hbm_settle();
      if (p.compact && npend < (uint32_t)kWave) {
        // a sparse batch (runs of contained sources dropped, containment cuts):
        // park its live items with the pending ones and read on, so batches
        // go out (nearly) full instead of two thirds empty (C5)
        const uint64_t vb = __ballot(valid);
        const uint32_t nv = (uint32_t)__popcll(vb);
        if (nv < (uint32_t)(kWave * 3 / 4)) {
          if (valid) {
            const uint32_t at = npend + lane_prefix(vb);
            s_pk[at] = key;
            s_pm[at] = meta;
          }
          npend += nv;
          wave_sync();
          hbm_fetch();
          continue;
        }
      }
      return true;
    }
    if (npend) {
      valid = (uint32_t)lane < npend;
      key = valid ? s_pk[lane] : 0;
      meta = valid ? s_pm[lane] : 0;
      npend = 0;
      return true;
    }
    valid = false;
    return false;
   }
  };
  // unconditional loads (invalid lanes read cell 0 and discard it): with no
  // branch around them the compiler's vmcnt waits stay exact, so the next
  // batch's line really is in flight behind the current batch
  auto load_cell = [&](uint64_t key, bool valid, uint64_t* e) {
    const ulonglong2* cp = reinterpret_cast<const ulonglong2*>(p.cells + (valid ? (key & 0xFFFFFFFFull) : 0) * kCell);
#pragma unroll
    for (int s = 0; s < kCell / 2; ++s) {
      const ulonglong2 x = cp[s];
      e[2 * s] = valid ? x.x : kEmpty;
      e[2 * s + 1] = valid ? x.y : kEmpty;
    }
  };
  // verify the first 64 candidates and move the rest (< 128) to the front,
  // while at least thr are listed (thr = 64: a full wavefront)
  auto drain = [&](uint32_t thr) {
    while (ncand >= thr) {
      wave_sync();
      if (p.phase_limit > 6) verify(kWave);
      const uint32_t rest = ncand - kWave;  // < 128: move to the front
      uint32_t mb0 = 0, mi0 = 0, ma0 = 0, mb1 = 0, mi1 = 0, ma1 = 0;
      if ((uint32_t)lane < rest) {
        mb0 = s_cb[kWave + lane]; mi0 = s_ci[kWave + lane]; ma0 = s_ca[kWave + lane];
      }
      if ((uint32_t)lane + kWave < rest) {
        mb1 = s_cb[2 * kWave + lane]; mi1 = s_ci[2 * kWave + lane]; ma1 = s_ca[2 * kWave + lane];
      }
      wave_sync();
      if ((uint32_t)lane < rest) {
        s_cb[lane] = mb0; s_ci[lane] = mi0; s_ca[lane] = ma0;
      }
      if ((uint32_t)lane + kWave < rest) {
        s_cb[kWave + lane] = mb1; s_ci[kWave + lane] = mi1; s_ca[kWave + lane] = ma1;
      }
      ncand = rest;
      wave_sync();
    }
  };
  auto process = [&](uint64_t key, uint64_t meta, bool valid, const uint64_t* e) {
    const uint32_t ra = (uint32_t)meta;
    const int rp = (int)((meta >> 32) & 1023u);
    const int rjlo = (int)((meta >> 42) & 1023u), rjhi = (int)((meta >> 52) & 1023u);
    const uint32_t fp = (uint32_t)(key >> 32);
#ifndef MG_DIAG_STAT_FPJ
    if (p.stats) {
      uint32_t ne = 0;
#pragma unroll
      for (int s = 0; s < kCell; ++s) ne += e[s] != kEmpty ? 1u : 0u;
      stat(1, ne);
    }
#endif
    if (p.phase_limit <= 5) return;
    // a full cell's chain flag: probe the next cell in a later batch
    const bool chain = valid && e[kCell - 1] != kEmpty && (e[kCell - 1] & kChain);
    const uint64_t cb = __ballot(chain);
    if (chain) {
      const uint32_t at = npend + lane_prefix(cb);
      s_pk[at] = next_cell(key & 0xFFFFFFFFull, p.cell_n, fp) | (key & 0xFFFFFFFF00000000ull);
      s_pm[at] = meta;
    }
    npend += (uint32_t)__popcll(cb);
    uint32_t keepm = 0;
    const uint32_t ra_h = (!CONTAIN && p.halving_id && valid) ? p.halving_id[ra] : ra;
#pragma unroll
    for (int s = 0; s < kCell; ++s) {
      const uint32_t hi = (uint32_t)(e[s] >> 32);
      const int j = rp - (int)((hi >> 2) & 1023u);
      const int oo = (int)(hi & 3u);
      bool keep = e[s] != kEmpty && ((hi >> 12) & kFpMask) == fp && j >= rjlo && j <= rjhi;
      // halving: o=1 hits are twins of the partner's o=0
      // hits; an o=2/3 pair is kept on one side only (rc_side_keeps)
      bool side = true;
      if (!CONTAIN && oo >= 2 && keep) {
        const uint32_t bh = p.halving_id ? p.halving_id[(uint32_t)e[s]] : (uint32_t)e[s];
        side = p.halving_low ? bh >= ra_h : rc_side_keeps(ra_h, bh);
      }
      keep = keep && (CONTAIN || oo == 0 || (oo >= 2 && side));
      // containment with k_prefix_contain covering offset s = 0: suffix-key
      // hits (o = 1/3) add nothing (see the verify's CONTAIN case)
      keep = keep && !(CONTAIN && p.contain_even && (oo & 1));
      keepm |= (keep ? 1u : 0u) << s;
    }
#ifdef MG_DIAG_STAT_FPJ  // (diagnostics build: counter 1 = entries past the fingerprint / window / o filter)
    stat(1, (uint32_t)__popc(keepm));
#endif
    if (CONTAIN && valid) {
      // the verify's length conditions (checkOverlapForContainedRead, :302-340:
      // read2 strictly shorter, at offset s = j <= n1 - n2, or s = 0 for a
      // suffix-key hit) at listing time, so a candidate that cannot be
      // contained takes no candidate slot and no verification round
      // (read2's length from its entry, make_entry: no load per listed entry)
      const int n1 = p.uniform_len ? p.uniform_len : (int)p.len[ra];
#pragma unroll
      for (int s = 0; s < kCell; ++s) {
        const uint32_t hi = (uint32_t)(e[s] >> 32);
        const int j = rp - (int)((hi >> 2) & 1023u), n2 = entry_len(hi);
        const bool ok = n1 > n2 && ((hi & 1u) ? j == n2 - h : j <= n1 - n2);
        if (!ok) keepm &= ~(1u << s);
      }
    }
    if (!CONTAIN && p.cbits) {
      // :548 a contained read2 is never inserted: drop it before it takes a
      // candidate slot, a partner-slot load and a compare (C5: most
      // candidates), from the bitmap (1/32 of d_super, mostly cache hits);
      // half a cell's lookups in flight together (registers: occupancy)
#pragma unroll
      for (int s0 = 0; s0 < kCell; s0 += kCell / 2) {
        uint32_t cw[kCell / 2];
#pragma unroll
        for (int s = 0; s < kCell / 2; ++s)
          cw[s] = ((keepm >> (s0 + s)) & 1u) ? p.cbits[(uint32_t)e[s0 + s] >> 5] : 0u;
#pragma unroll
        for (int s = 0; s < kCell / 2; ++s) keepm &= ~(((cw[s] >> ((uint32_t)e[s0 + s] & 31u)) & 1u) << (s0 + s));
      }
    }
    while (__ballot(keepm != 0)) {
      // append slot groups while they fit, then verify a full wavefront
#pragma unroll
      for (int s = 0; s < kCell; ++s) {
        const bool k = (keepm >> s) & 1u;
        const uint64_t bal = __ballot(k);
        const uint32_t nb = (uint32_t)__popcll(bal);
        if (nb && ncand + nb <= (uint32_t)PL::CAND) {
          if (k) {
            const uint32_t hi = (uint32_t)(e[s] >> 32);
            const uint32_t at = ncand + lane_prefix(bal);
            s_cb[at] = (uint32_t)e[s];
            // o | partner length - 1 (from its entry) | j: the verify loads no length.  j lies in
            // the run's window range [jlo, jhi] (keep above), so 0 <= j < 1024; the templated
            // probe only runs with reads up to 1,024 bp (LaunchProbe checks maxlen)
            s_ci[at] = ((hi & 3u) << 30) | (((hi >> 21) & 1023u) << 10) |
                       ((uint32_t)(rp - (int)((hi >> 2) & 1023u)) & 1023u);
            s_ca[at] = ra;
            keepm &= ~(1u << s);
          }
          ncand += nb;
        }
      }
      drain(kWave);
    }
  };

  if (p.phase_limit > 4 && reg_of(0) < rlimit) {
    open_region(0);
    pf_any = hbm_settle();
    hbm_fetch();
    uint64_t key_c = 0, meta_c = 0, key_n = 0, meta_n = 0;
    bool val_c = false, val_n = false;
    uint64_t eA[kCell], eB[kCell];
    bool have = take_item(key_c, meta_c, val_c);
    hbm_fetch();
    load_cell(key_c, val_c, eA);
    // two batches per trip with ping-pong cell registers (no copies, so the
    // compiler's vmcnt waits only ever cover the older batch's line)
    while (have) {
      bool have_n = take_item(key_n, meta_n, val_n);
      hbm_fetch();
      load_cell(key_n, val_n, eB);
      process(key_c, meta_c, val_c, eA);
      if (!have_n) {  // the stream ran dry: this batch may have left pending items
        have_n = take_item(key_n, meta_n, val_n);
        if (!have_n) break;
        load_cell(key_n, val_n, eB);
      }
      key_c = key_n; meta_c = meta_n; val_c = val_n;
      have_n = take_item(key_n, meta_n, val_n);
      hbm_fetch();
      load_cell(key_n, val_n, eA);
      process(key_c, meta_c, val_c, eB);
      if (!have_n) {
        have_n = take_item(key_n, meta_n, val_n);
        if (!have_n) break;
        load_cell(key_n, val_n, eA);
      }
      key_c = key_n; meta_c = meta_n; val_c = val_n;
    }
  }
  if (ncand && p.phase_limit > 6) verify(ncand);
  if (!CONTAIN && lane == 0) p.reg_cnt[gw] = cursor;
  if constexpr (DCNT) {
    wave_sync();
    if ((uint32_t)lane < p.dst_ranks) p.dst_cnt[gw * p.dst_ranks + lane] = s_dc[wv * kWave + lane];
  }
}

// Gather per-wavefront row regions into a contiguous array (copy-out path only).
__global__ __launch_bounds__(kBlock) void k_compact_rows(const uint32_t* __restrict__ rows, uint64_t reg_cap,
                                                        const uint64_t* __restrict__ prefix,
                                                        uint32_t* __restrict__ out) {
  const uint64_t r = blockIdx.x;
  const uint64_t c = (prefix[r + 1] - prefix[r]) * 3;
  const uint32_t* src = rows + r * reg_cap * 3;
  uint32_t* dst = out + prefix[r] * 3;
  for (uint64_t i = threadIdx.x; i < c; i += kBlock) dst[i] = src[i];
}

// ------------------------------------------------------- exchange routing ---
// Exchange mode moves records in the SLOT LAYOUT (include/mg_overlap.h): the
// records bound for (or received from) peer d form a stream whose i-th record
// sits at ((i / slot) P + d) slot + i % slot, i < rounds * slot, so round t of
// every peer is one contiguous block and one equal-split all-to-all per round
// moves it; the per-peer counts stay on the device.
//
// Records produced in per-wavefront regions (rows) or o-major key arrays are
// routed as a stable-per-block counting sort by destination: pass 0 counts per
// (block, destination) in LDS, k_part_scan turns the counts into per-
// destination offsets (and the totals into the caller's device counts), pass 1
// re-walks the same records with the same grid and scatters through LDS
// cursors (no global atomics).  Within a wavefront the lanes bound for one
// destination take one LDS cursor step together (ballot + mbcnt); order inside
// a destination is irrelevant (the result is a multiset).
//   OWN_KEY: the four key records (bucket, entry) of every source read, o-major
//            (key_ent[o key_n + a]); owner = bucket range (same rule as owned());
//            what travels is the 8-B entry alone (read slot | o | q | fp |
//            length): the owner recomputes the bucket from the read, which it
//            holds (k_xkeys_dense);
//   OWN_SRC: 12-B rows, owner of src ID = source-read range
//            [floor(r N / P), floor((r+1) N / P)) -> (src P - 1) / N;
//   OWN_BUCKET: 16-B run records of the scan's regions (x = bucket |
//            fingerprint, y = run meta), owner = the bucket's rank; what
//            travels is the 8-B meta alone (read slot | p | jlo | jhi): the owner
//            re-hashes the minimizer m-mer at p of its copy of the read
//            (k_xruns_expand), so a run costs 8 B on xGMI instead of 16.
//   OWN_META: the keys-first receiver scan's regions (k_scan<RECV>): 8-B metas
//            with their owner rank beside them in dst8 (one byte per record).
enum OwnerKind { OWN_KEY = 0, OWN_SRC = 1, OWN_BUCKET = 2, OWN_META = 3 };
constexpr int kMaxRanks = 64;

struct PartParams {
  const void* base;                 // OWN_SRC: region r starts at base + r * cap records
  uint64_t cap;                     // records per region
  const unsigned long long* cnt;    // records per region (nullptr: flat array of flat_n records)
  uint64_t nreg, flat_n;
  uint32_t nranks, nb_log2;
  uint64_t n_reads;
  unsigned long long* blk;          // [gridDim.x * nranks]: pass 0 counts, then offsets
  void* out;                        // slot layout
  void* self_out;                   // non-null: the stream to this rank goes here (same offsets)
  uint32_t self_rank;
  uint64_t slot, rounds;
  const uint32_t* key_bk;           // OWN_KEY: sources [a_lo, a_lo + nsrc), key o of read a at o * key_n + a
  const uint64_t* key_ent;
  uint64_t key_n, a_lo, nsrc;
  const uint8_t* dst8;              // OWN_META: each record's owner rank
};

template <int KIND, int PASS>
__global__ __launch_bounds__(kBlock) void k_part(PartParams p) {
  __shared__ unsigned long long s_cnt[kMaxRanks];
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < kMaxRanks)
    s_cnt[threadIdx.x] = (PASS == 1 && threadIdx.x < p.nranks) ? p.blk[(uint64_t)blockIdx.x * p.nranks + threadIdx.x] : 0;
  __syncthreads();
  const uint64_t lim = p.slot * p.rounds;
  for (uint64_t r = blockIdx.x; r < p.nreg; r += gridDim.x) {
    uint64_t c = p.cnt ? p.cnt[r] : (p.flat_n > r * p.cap ? p.flat_n - r * p.cap : 0);
    c = c < p.cap ? c : p.cap;
    // one record per thread and step, the next step's record loaded before
    // this one is placed (the steps are otherwise one dependent round trip each)
    struct Rec {
      bool valid;
      uint32_t d;
      ulonglong2 x16;
      uint3 x12;
    };
    auto fetch = [&](uint64_t i0) {
      Rec q{false, 0u, make_ulonglong2(0, 0), make_uint3(0, 0, 0)};
      const uint64_t i = i0 + threadIdx.x;
      q.valid = i < c;
      if (q.valid) {
        if (KIND == OWN_KEY) {
          const uint64_t at = r * p.cap + i;  // (the rank's records are contiguous, key_seg order)
          const uint64_t e = p.key_ent[at];
          const uint32_t b = p.key_bk[at];
          q.valid = e != kEmpty;  // a read without keys (never after setup_index's length check)
          q.x16 = make_ulonglong2(b, e);
          q.d = (uint32_t)(((uint64_t)b * p.nranks) >> p.nb_log2);
        } else if (KIND == OWN_BUCKET) {
          q.x16 = reinterpret_cast<const ulonglong2*>(p.base)[r * p.cap + i];
          q.d = (uint32_t)(((q.x16.x & ((1ULL << p.nb_log2) - 1)) * p.nranks) >> p.nb_log2);
        } else if (KIND == OWN_META) {
          q.x16.y = reinterpret_cast<const uint64_t*>(p.base)[r * p.cap + i];
          q.d = p.dst8[r * p.cap + i];
        } else {
          q.x12 = reinterpret_cast<const uint3*>(p.base)[r * p.cap + i];
          q.d = (uint32_t)(((uint64_t)q.x12.x * p.nranks - 1) / p.n_reads);  // src is the 1-based ID
        }
      }
      return q;
    };
    Rec nxt = fetch(0);
    for (uint64_t i0 = 0; i0 < c; i0 += kBlock) {
      const Rec cur = nxt;
      if (i0 + kBlock < c) nxt = fetch(i0 + kBlock);
      const bool valid = cur.valid;
      const uint32_t d = cur.d;
      // wavefront multi-split: one ballot per destination; lane dd then holds
      // destination dd's count and takes its LDS cursor step, all
      // destinations in one LDS atomic (no loop serialised per destination)
      uint64_t mine = 0;
      uint32_t cnt_d = 0;
      for (uint32_t dd = 0; dd < p.nranks; ++dd) {
        const uint64_t m = __ballot(valid && d == dd);
        if (valid && d == dd) mine = m;
        if ((uint32_t)lane == dd) cnt_d = (uint32_t)__popcll(m);
      }
      unsigned long long at = 0;
      if (cnt_d) at = atomicAdd(&s_cnt[lane], (unsigned long long)cnt_d);
      if (PASS == 1) {
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)at, (int)d);
        const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(at >> 32), (int)d);
        const uint64_t k = (((uint64_t)hi << 32) | lo) + lane_prefix(mine);
        if (valid && k < lim) {  // a stream cut at its capacity keeps its full count
          uint64_t q = 0, kk = k;  // (round, position in it): k < rounds * slot, rounds small: no 64-bit divide
          while (kk >= p.slot) {
            kk -= p.slot;
            ++q;
          }
          const uint64_t o = ((q * p.nranks) + d) * p.slot + kk;
          void* dst = (p.self_out && d == p.self_rank) ? p.self_out : p.out;
          if (KIND != OWN_SRC) reinterpret_cast<uint64_t*>(dst)[o] = cur.x16.y;  // entry / run meta (8 B)
          else reinterpret_cast<uint3*>(dst)[o] = cur.x12;
        }
      }
    }
  }
  if (PASS == 0) {
    __syncthreads();
    if (threadIdx.x < p.nranks) p.blk[(uint64_t)blockIdx.x * p.nranks + threadIdx.x] = s_cnt[threadIdx.x];
  }
}

// Per-(block, destination) counts -> offsets within each destination's stream:
// off[b][d] = sum_{b' < b} cnt[b'][d]; totals[d] = the stream's length (the
// caller's device counts).  One block per destination.
__global__ __launch_bounds__(1024) void k_part_scan(unsigned long long* blk, uint32_t nblk, uint32_t nranks,
                                                    unsigned long long* totals) {
  // thread t owns the contiguous blocks [t per, (t + 1) per): their sum, one
  // block-wide scan of the 1,024 sums, then its blocks' offsets -- one
  // synchronised scan per destination instead of one per 1,024 blocks
  __shared__ unsigned long long s_part[16];
  const uint32_t d = blockIdx.x, t = threadIdx.x;
  const uint32_t per = (nblk + 1023) / 1024;
  const uint32_t b0 = t * per, b1 = min(b0 + per, nblk);
  // up to 8 blocks per thread (nblk <= 8,192): the counts stay in registers and
  // their loads are all in flight at once (one round trip, not one per block)
  constexpr uint32_t kRegs = 8;
  unsigned long long v8[kRegs];
  unsigned long long sum = 0;
  if (per <= kRegs) {
#pragma unroll
    for (uint32_t i = 0; i < kRegs; ++i) v8[i] = b0 + i < b1 ? blk[(uint64_t)(b0 + i) * nranks + d] : 0ull;
#pragma unroll
    for (uint32_t i = 0; i < kRegs; ++i) sum += v8[i];
  } else {
    for (uint32_t b = b0; b < b1; ++b) sum += blk[(uint64_t)b * nranks + d];
  }
  // inclusive scan of the 1,024 sums: within each wavefront by shuffles, then
  // the 16 wavefront totals through LDS (two barriers, not twenty)
  const int lane = (int)(t & 63u), wv = (int)(t >> 6);
  unsigned long long inc = sum;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned long long v = (unsigned long long)__shfl_up((long long)inc, o);
    if (lane >= o) inc += v;
  }
  if (lane == kWave - 1) s_part[wv] = inc;
  __syncthreads();
  unsigned long long before = 0, total = 0;
  for (int w2 = 0; w2 < 16; ++w2) {
    const unsigned long long x = s_part[w2];
    before += w2 < wv ? x : 0ull;
    total += x;
  }
  unsigned long long run = before + inc - sum;  // exclusive: the blocks before b0
  if (per <= kRegs) {
#pragma unroll
    for (uint32_t i = 0; i < kRegs; ++i)
      if (b0 + i < b1) {
        blk[(uint64_t)(b0 + i) * nranks + d] = run;
        run += v8[i];
      }
    if (t == 1023) totals[d] = total;
    return;
  }
  for (uint32_t b = b0; b < b1; ++b) {
    const unsigned long long v = blk[(uint64_t)b * nranks + d];
    blk[(uint64_t)b * nranks + d] = run;
    run += v;
  }
  if (t == 1023) totals[d] = total;
}

// Per-region counts of a slot-layout buffer cut into regions of `reg` records
// (reg divides slot; region q covers records [q reg, q reg + reg)).
// part (exchange mode's split discovery probe): 1 = only the regions of peer
// `me` (this rank's own stream), 2 = every other peer's, 0 = all
__global__ __launch_bounds__(kBlock) void k_slot_regions(unsigned long long* __restrict__ out,
                                                         const unsigned long long* __restrict__ counts,
                                                         uint64_t slot, uint64_t reg, uint64_t nreg,
                                                         uint32_t nranks, int part, uint32_t me) {
  const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q >= nreg) return;
  const uint64_t K = slot / reg, blk = q / K, k = q - blk * K, t = blk / nranks, s = blk - t * nranks;
  const uint64_t start = t * slot + k * reg, c = counts[s];
  const bool in = part == 0 || ((part == 1) == (s == me));
  out[q] = (in && c > start) ? (c - start < reg ? c - start : reg) : 0;
}

// Exchange mode: the received runs (slot layout, one stream per peer) ->
// one compact array with a sort key = the top 8 bits of the run's bucket
// within this rank's range.  Record j of peer s goes to position
// sum_{s' < s} counts[s'] + j, so no atomics and the array is dense.
// A stream cut at its capacity (count > rounds * slot, the step reruns)
// contributes the rounds * slot records that arrived.
__global__ __launch_bounds__(kBlock) void k_xruns_keys(const ulonglong2* __restrict__ recv, uint64_t slot,
                                                      uint32_t nranks, uint64_t total,
                                                      const unsigned long long* __restrict__ counts,
                                                      uint64_t nbmask, uint64_t cell_lo, uint32_t shift,
                                                      uint32_t* __restrict__ key, ulonglong2* __restrict__ val) {
  const uint64_t blk = (uint64_t)nranks * slot, lim = total / nranks;  // records per peer stream
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (uint64_t)gridDim.x * kBlock) {
    const uint64_t t = i / blk, rem = i - t * blk, sp = rem / slot, j = t * slot + (rem - sp * slot);
    if (j >= counts[sp]) continue;  // (j < lim always)
    uint64_t at = j;
    for (uint64_t q = 0; q < sp; ++q) at += counts[q] < lim ? counts[q] : lim;
    const ulonglong2 x = recv[i];
    key[at] = (uint32_t)((((x.x & nbmask) - cell_lo) >> shift) & 0xFFu);
    val[at] = x;
  }
}

// run regions of R records over a dense array of n records
__global__ __launch_bounds__(kBlock) void k_fixed_regions(unsigned long long* __restrict__ out, uint64_t n,
                                                          uint64_t R, uint64_t nreg) {
  const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (q < nreg) out[q] = n > q * R ? (n - q * R < R ? n - q * R : R) : 0;
}

// After markContainedReads: sources with superReadID != 0 contribute no
// windows (OverlapGraph.cpp:548), so their runs (about two thirds of them at
// C5) are dropped from every run region before the discovery probe, which
// then streams and batches live runs only.  One wavefront per region, stable
// in-place ballot compaction (a write never passes the batch being read), eight
// batches in flight; run_cnt[r] becomes the live count.
__global__ __launch_bounds__(kBlock) void k_live_runs(ulonglong2* __restrict__ runs,
                                                     unsigned long long* __restrict__ run_cnt, uint64_t run_cap,
                                                     uint64_t nreg, const uint32_t* __restrict__ cbits) {
  const int lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  constexpr int kDepth = 8;
  for (uint64_t r = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); r < nreg; r += nw) {
    ulonglong2* reg = runs + r * run_cap;
    const uint64_t c = run_cnt[r] < run_cap ? run_cnt[r] : run_cap;
    uint64_t out = 0;
    for (uint64_t b = 0; b < c; b += kDepth * kWave) {
      ulonglong2 rec[kDepth];
      bool live[kDepth];
#pragma unroll
      for (int d = 0; d < kDepth; ++d) {
        const uint64_t i = b + (uint64_t)d * kWave + lane;
        rec[d] = i < c ? reg[i] : make_ulonglong2(0, kFlatHole);
      }
#pragma unroll
      for (int d = 0; d < kDepth; ++d) {
        const uint32_t ra = (uint32_t)rec[d].y;  // (the bitmap of contained slots, k_super_finalize)
        live[d] = rec[d].y != kFlatHole && !((cbits[ra >> 5] >> (ra & 31u)) & 1u);
      }
      wave_sync();
#pragma unroll
      for (int d = 0; d < kDepth; ++d) {
        const uint64_t bal = __ballot(live[d]);
        if (live[d]) reg[out + lane_prefix(bal)] = rec[d];
        out += (uint64_t)__popcll(bal);
      }
    }
    if (lane == 0) run_cnt[r] = out;
  }
}

__global__ __launch_bounds__(kBlock) void k_super_finalize(const unsigned long long* __restrict__ key,
                                                          uint64_t n, uint32_t* __restrict__ super,
                                                          unsigned int* __restrict__ any,
                                                          uint32_t* __restrict__ cbits,
                                                          unsigned int* __restrict__ ccnt) {
  // grid-stride over 64-read tiles (i is 64-aligned at lane 0); the wavefront
  // counts its contained reads in a register and adds them once at the end
  // (one add per tile on 64 counters serialised at C5: 0.32 ms per pass)
  const int lane = (int)(threadIdx.x & 63);
  uint32_t cnt = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i - lane < n; i += (uint64_t)gridDim.x * kBlock) {
    uint32_t s = 0;
    if (i < n) {
      const unsigned long long k = key[i];
      s = k ? (0xFFFFFFFFu - (uint32_t)k) + 1u : 0u;  // container index -> ID
      super[i] = s;
    }
    // the tile's 64 contained bits as two bitmap words
    const uint64_t bal = __ballot(s != 0);
    if (lane < 2) cbits[(i - lane) / 32 + lane] = (uint32_t)(bal >> (32 * lane));
    cnt += (uint32_t)__popcll(bal);
  }
  if (cnt && lane == 0) {
    if (ccnt) atomicAdd(&ccnt[(blockIdx.x & 63u) * 16], cnt);
    // the flag is set once: waves that already see it set skip the atomic
    if (__hip_atomic_load(any, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(any, 1u);
  }
}

inline uint32_t super_grid(const mg_ctx* ctx) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((ctx->n + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 8));
}

// Exchange mode, cross-rank prefix marks (mg_xchg_prefix_marks): marks[i] = 1
// for every read whose containment key is set after this rank's offset-0
// containments; after the caller's MAX all-reduce, the marks fold back into
// the key array as key = max(key, mark), so contain_skip (the probe's
// "source already contained" test, superkey != 0) sees every rank's prefix
// containments.  A folded 1 never survives: the rank that set the mark holds
// the read's real key (len << 32 | ~id > 1), and the MAX all-reduce of the keys
// after the probe keeps the larger.
__global__ __launch_bounds__(kBlock) void k_prefix_marks(const unsigned long long* __restrict__ key, uint64_t n,
                                                        uint8_t* __restrict__ marks) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
    marks[i] = key[i] ? 1 : 0;
}
__global__ __launch_bounds__(kBlock) void k_fold_marks(unsigned long long* __restrict__ key, uint64_t n,
                                                      const uint8_t* __restrict__ marks) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
    if (marks[i] && !key[i]) key[i] = 1ull;
}

// Order-independent digests (include/mg_overlap.h, mg_rows_digest): per row
// h = mix64(((src << 32) | dst) ^ mix64(((orient << 16) | offset) + GOLD));
// accumulators {n, sum h, xor h, sum mix64(h ^ SALT)} mod 2^64.  The rows are
// either per-wavefront regions (cnt != nullptr: region r holds cnt[r] rows at
// r * cap) or one flat array of `flat_n` rows; super: g = mix64((id << 32) | sup)
// over contained reads.  One wavefront reduction and 4 atomics per wavefront.
constexpr uint64_t kDigestGold = 0x9E3779B97F4A7C15ULL, kDigestSalt = 0xD6E8FEB86659FD93ULL;

__device__ __forceinline__ void digest_flush(unsigned long long* acc, uint64_t n, uint64_t s, uint64_t x, uint64_t s2) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    n += __shfl_xor(n, d);
    s += __shfl_xor(s, d);
    x ^= __shfl_xor(x, d);
    s2 += __shfl_xor(s2, d);
  }
  if ((threadIdx.x & 63) == 0 && n) {
    atomicAdd(&acc[0], (unsigned long long)n);
    atomicAdd(&acc[1], (unsigned long long)s);
    atomicXor(&acc[2], (unsigned long long)x);
    atomicAdd(&acc[3], (unsigned long long)s2);
  }
}

__global__ __launch_bounds__(kBlock) void k_rows_digest(const uint32_t* __restrict__ rows, uint64_t cap,
                                                        const unsigned long long* __restrict__ cnt, uint64_t nreg,
                                                        uint64_t flat_n, unsigned long long* acc) {
  uint64_t n = 0, s = 0, x = 0, s2 = 0;
  auto add = [&](const uint32_t* r) {
    const uint64_t k2 = (uint64_t)r[2];  // orient << 16 | offset
    const uint64_t hv = mix64((((uint64_t)r[0] << 32) | r[1]) ^ mix64(k2 + kDigestGold));
    n += 1;
    s += hv;
    x ^= hv;
    s2 += mix64(hv ^ kDigestSalt);
  };
  if (cnt) {
    for (uint64_t reg = blockIdx.x; reg < nreg; reg += gridDim.x) {
      const uint64_t c = cnt[reg] < cap ? cnt[reg] : cap;
      for (uint64_t i = threadIdx.x; i < c; i += kBlock) add(rows + (reg * cap + i) * 3);
    }
  } else {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < flat_n; i += (uint64_t)gridDim.x * kBlock)
      add(rows + i * 3);
  }
  digest_flush(acc, n, s, x, s2);
}

__global__ __launch_bounds__(kBlock) void k_super_digest(const uint32_t* __restrict__ super, uint64_t n_reads,
                                                         unsigned long long* acc, const uint32_t* __restrict__ id) {
  uint64_t n = 0, s = 0, x = 0, s2 = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_reads; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t sp = super[i];
    if (sp) {
      const uint64_t g = mix64(((uint64_t)(rid(id, (uint32_t)i) + 1) << 32) | sp);
      n += 1;
      s += g;
      x ^= g;
      s2 += mix64(g ^ kDigestSalt);
    }
  }
  digest_flush(acc, n, s, x, s2);
}

// getListOfReads(key) (HashTable.cpp:202-221): walk the query key's home cell
// chain and keep entries whose key string equals it exactly.
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_lookup_key(IndexParams p, const uint64_t* __restrict__ qkey,
                                                      int qwords, unsigned long long* __restrict__ out,
                                                      uint32_t cap, unsigned int* __restrict__ nout) {
  __shared__ uint64_t q[40];  // h <= 1055 -> at most 33 words + over-read
  __shared__ uint64_t qv;
  __shared__ int qq;
  const int h = p.h;
  if (threadIdx.x < 40) q[threadIdx.x] = threadIdx.x < qwords ? qkey[threadIdx.x] : 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    int qo;
    qv = key_minimizer<1>(q, h, 0, h, p.m, p.w, &qo);  // the key itself is a "read" of length h, o = 0
    qq = qo;
  }
  __syncthreads();
  const uint64_t mask = (1ULL << p.nb_log2) - 1;
  const uint32_t fp = (uint32_t)(qv >> p.nb_log2) & kFpMask;
  uint64_t b = (qv & mask) - p.cell_lo;  // unsharded index only: cell_lo = 0
  for (uint64_t probe = 0; probe < p.cell_n; ++probe) {
    const uint64_t last = p.cells[b * kCell + kCell - 1];
    if (threadIdx.x < (unsigned)kCell) {
      const uint64_t en = p.cells[b * kCell + threadIdx.x];
      const uint32_t hi = (uint32_t)(en >> 32);
      if (en != kEmpty && ((hi >> 12) & kFpMask) == fp && (int)((hi >> 2) & 1023u) == qq) {
        const int o = (int)(hi & 3u);
        const uint32_t r = (uint32_t)en;
        const uint64_t* g = p.words + (uint64_t)r * (MAXW ? (uint64_t)slot_words(MAXW) : (uint64_t)p.stride);
        const int n = p.len[r];
        // key string of (r, o) vs the query, 32 bases at a time
        uint64_t diff = 0;
        for (int cc = 0; cc * 32 < h; ++cc) {
          uint64_t kv;
          if (o < 2) {
            const int pos = (o == 0 ? 0 : n - h) + 32 * cc;
            kv = funnel(g[pos >> 5], g[(pos >> 5) + 1], (pos & 31) << 1);
          } else {
            // R[bb, bb+32) = rc(F[n-bb-32, n-bb)), bb = (o == 2 ? 0 : n-h) + 32cc
            const int bb = (o == 2 ? 0 : n - h) + 32 * cc;
            const int pos = n - bb - 32;
            const uint64_t fw = pos < 0 ? g[0] >> (-pos * 2) : funnel(g[pos >> 5], g[(pos >> 5) + 1], (pos & 31) << 1);
            kv = rc_word(fw);
          }
          const int rem = h - 32 * cc;
          const uint64_t msk = rem >= 32 ? ~0ULL : ~(~0ULL >> (2 * rem));
          diff |= (kv ^ ext_fwd<1>(q, 32 * cc)) & msk;
        }
        if (!diff) {
          const unsigned int slot = atomicAdd(nout, 1u);
          if (slot < cap) out[slot] = ((unsigned long long)(rid(p.id, r) + 1)) | ((unsigned long long)o << 62);
        }
      }
    }
    if (last == kEmpty || !(last & kChain)) break;
    b = next_cell(b, p.cell_n, fp);
  }
}

// ------------------------------------------------------------ long reads ---
// Reads longer than 1,024 bp, up to Read::getReadLength's UINT16 (Read.h:62).
// The templated kernels keep a read's words in registers and pack window
// positions into 10-bit fields; these keep the words in HBM (slots of
// mg_ctx::stride words, at least one zero pad word) and work one WINDOW per
// lane, so positions are plain ints.  Same cell index, same entries, same
// exactness argument as the main path: window F1[j, j+h)
// equals key K only if both select the same minimizer at the same offset q,
// so an entry is a candidate when its fingerprint and q match the window's,
// and every candidate is verified over the full overlap.

// HashTable::insertDataset (HashTable.cpp:50-80) for long reads: one thread
// per key, the key's m-mers read straight from the slot.
__global__ __launch_bounds__(kBlock) void k_index_long(IndexParams p) {
  const uint64_t mask = (1ULL << p.nb_log2) - 1;
  for (uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x; (gid >> 2) < p.n;
       gid += (uint64_t)gridDim.x * kBlock) {
    const uint64_t r = gid >> 2;
    const int o = (int)(gid & 3);
    int q;
    const uint64_t v = key_minimizer<1>(p.words + r * p.stride, p.len[r], o, p.h, p.m, p.w, &q);
    const uint64_t b = v & mask;
    if (owned(b, p.nb_log2, p.rank, p.nranks))
      cell_insert(p.cells, b - p.cell_lo, p.cell_n, make_entry(v, p.nb_log2, q, o, (uint32_t)r, p.len[r]));
  }
}

// Minimizer of the forward window F[s0, s0+h): the same rule as key_minimizer
// (order_key | i, smallest wins), so a window and an identical key agree.
__device__ __forceinline__ uint64_t window_minimizer(const uint64_t* f, int s0, int m, int w, int* q) {
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  uint64_t mm = ext_fwd<1>(f, s0) >> (64 - 2 * m);
  uint32_t bkey = 0xFFFFFFFFu;
  uint64_t bmm = 0;
  for (int i = 0; i < w; ++i) {
    const uint32_t key = order_key(mm) | (uint32_t)i;
    if (key < bkey) {
      bkey = key;
      bmm = mm;
    }
    if (i + 1 < w) {
      const int x = s0 + i + m;
      mm = ((mm << 2) | ((f[x >> 5] >> (62 - 2 * (x & 31))) & 3u)) & mmask;
    }
  }
  *q = (int)(bkey & 1023u);
  return mix64(bmm);
}

// checkOverlap / checkOverlapForContainedRead's compare (OverlapGraph.cpp:
// 302-383) for any length: partner bases [y0, y0+L) of F2 against source bases
// [x0, x0+L) of F1, or of R1 when rcA, 32 bases per step, both from HBM.
__device__ bool overlap_equal_long(const uint64_t* f1, int n1, const uint64_t* f2, int x0, int y0, int L, bool rcA) {
  for (int k = y0 >> 5; 32 * k < y0 + L; ++k) {
    const int lo = max(y0 - 32 * k, 0), hi = min(y0 + L - 32 * k, 32);
    const int s = x0 - y0 + 32 * k;  // source position of partner base 32k
    const uint64_t av = rcA ? rc_word(ext_fwd<1>(f1, n1 - s - 32)) : ext_fwd<1>(f1, s);
    const uint64_t msk = (lo ? (~0ULL >> (2 * lo)) : ~0ULL) & (hi < 32 ? ~(~0ULL >> (2 * hi)) : ~0ULL);
    if ((av ^ f2[k]) & msk) return false;
  }
  return true;
}

struct LongParams {
  const uint64_t* words;
  const uint16_t* len;
  uint32_t stride;
  int h, m, w;
  uint32_t nb_log2;
  uint64_t cell_n;
  const uint64_t* cells;
  uint64_t a_lo, a_hi;            // source reads
  const uint32_t* super;          // superReadID per read (nullptr: none contained)
  unsigned long long* superkey;   // CONTAIN: max over containers of (len << 32 | ~index)
  uint32_t* rows;                 // one region of reg_cap rows per wavefront
  unsigned long long* reg_cnt;
  uint64_t reg_cap;
  int halving_low;
};

// markContainedReads (CONTAIN) or insertAllEdgesOfRead (OverlapGraph.cpp:
// 225-290, 529-565) for long reads: one wavefront per source read (grid-
// stride), one window j in [1, n1-h) per lane, the window's home cell chain,
// then the same filter, halving rule, verification and rows + twins as
// k_probe.  Rows go to the wavefront's region through an LDS
// cursor (the count keeps running past the capacity: the host resizes and
// reruns).
template <bool CONTAIN>
__global__ __launch_bounds__(kBlock) void k_probe_long(LongParams p) {
  __shared__ unsigned long long s_cur[kWavesPerBlock];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
  const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
  if (lane == 0) s_cur[wv] = 0;
  __syncthreads();
  const int h = p.h;
  const uint64_t nbmask = (1ULL << p.nb_log2) - 1;
  uint32_t* const region = p.rows + gw * p.reg_cap * 3;
  for (uint64_t a = p.a_lo + gw; a < p.a_hi; a += nw) {
    if (!CONTAIN && p.super && p.super[a]) continue;  // :548 read1 contained
    const int n1 = p.len[a];
    const uint64_t* f1 = p.words + a * p.stride;
    for (int j = 1 + lane; j < n1 - h; j += kWave) {
      int q;
      const uint64_t v = window_minimizer(f1, j, p.m, p.w, &q);
      const uint32_t fp = (uint32_t)(v >> p.nb_log2) & kFpMask;
      uint64_t c = v & nbmask;
      for (uint64_t probe = 0; probe < p.cell_n; ++probe) {
        const uint64_t* cell = p.cells + c * kCell;
        for (int s = 0; s < kCell; ++s) {
          const uint64_t e = cell[s];
          if (e == kEmpty) continue;
          const uint32_t hi = (uint32_t)(e >> 32), bid = (uint32_t)e;
          if (((hi >> 12) & kFpMask) != fp || (int)((hi >> 2) & 1023u) != q) continue;
          const int o = (int)(hi & 3u);
          const int n2 = p.len[bid];
          const uint64_t* f2 = p.words + (uint64_t)bid * p.stride;
          int L, x0, y0;
          bool cond, rcA;
          if (CONTAIN) {
            // checkOverlapForContainedRead: o = 0/2 place read2 at s = j; o = 1/3
            // only at s = 0 (s >= 1 is the o = 0/2 hit at window j = s, k_probe)
            int sft;
            cond = n1 > n2;
            if (o == 0 || o == 2) {
              cond = cond && j <= n1 - n2;
              sft = j;
            } else {
              cond = cond && j == n2 - h;
              sft = 0;
            }
            L = n2;
            y0 = 0;
            rcA = o >= 2;
            x0 = rcA ? n1 - sft - n2 : sft;
            if (cond && overlap_equal_long(f1, n1, f2, x0, y0, L, rcA))
              atomicMax(&p.superkey[bid], ((unsigned long long)n1 << 32) | (0xFFFFFFFFu - (uint32_t)a));
            continue;
          }
          // halving: o = 1 never, o = 2/3 on one side only
          if (o == 1 || (o >= 2 && !(p.halving_low ? bid >= (uint32_t)a : rc_side_keeps((uint32_t)a, bid)))) continue;
          if (p.super && p.super[bid]) continue;  // :548 read2 contained
          if (o == 0) {        // F1[j, n1) == F2[0, L)
            L = n1 - j; cond = L < n2; x0 = j; y0 = 0; rcA = false;
          } else if (o == 2) { // F1[j, n1) == R2[0, L)  <=>  R1[0, L) == F2[n2-L, n2)
            L = n1 - j; cond = L < n2; x0 = 0; y0 = n2 - L; rcA = true;
          } else {             // F1[0, L) == R2[n2-L, n2)  <=>  R1[n1-L, n1) == F2[0, L)
            L = j + h; cond = j <= n2 - h; x0 = n1 - L; y0 = 0; rcA = true;
          }
          if (!cond || !overlap_equal_long(f1, n1, f2, x0, y0, L, rcA)) continue;
          // orientation/offset switch (:550-557) and the twin (:409-412, :841-855)
          const uint32_t orient = (o == 0) ? 3u : (o == 2 ? 2u : 1u);
          const uint32_t off = (o == 3) ? (uint32_t)(n1 - h - j) : (uint32_t)j;
          const uint32_t torient = (orient == 3u) ? 0u : orient;
          const uint32_t toff = (uint16_t)(n2 + off - n1);
          const int nrec = (bid == (uint32_t)a && o == 0) ? 4 : 2;  // self o=0 hit also stands for its o=1 twin
          const unsigned long long at = atomicAdd(&s_cur[wv], (unsigned long long)nrec);
          if (at + nrec <= p.reg_cap) {
            uint3* d = reinterpret_cast<uint3*>(region + at * 3);
            for (int rr = 0; rr < nrec; rr += 2) {
              d[rr] = make_uint3((uint32_t)a + 1, bid + 1, (orient << 16) | off);
              d[rr + 1] = make_uint3(bid + 1, (uint32_t)a + 1, (torient << 16) | toff);
            }
          }
        }
        const uint64_t last = cell[kCell - 1];
        if (last == kEmpty || !(last & kChain)) break;
        c = next_cell(c, p.cell_n, fp);
      }
    }
  }
  __syncthreads();
  if (!CONTAIN && lane == 0) p.reg_cnt[gw] = s_cur[wv];
}

}  // namespace

namespace {
// ------------------------------------------------------------ layout ---
// Device layout of the reads.  Overlapping reads share
// m-mers, so clustering the slots by each read's canonical global minimizer
// (the smallest hash over its 16-mers and their reverse complements;
// strand-independent) puts a read's overlap partners next to it in memory for
// about half of its discoveries: the probe's partner slots and the shared
// minimizer cells then come from L2 instead of HBM.  The key is
// [group (2, only with a source-read range) | minimizer hash (32) | its offset
// (pb)], so each cluster is ordered along the genome; the radix sort runs over
// those 32 + pb (+ 2) bits only.  A 22-bit hash (order_key) merged too many
// clusters: C3 probe 4.9 vs 4.6 ms.  group = 0 / 1 / 2 for reference IDs
// below / inside / above the range [lo, hi), so the range's reads take exactly
// the slots [lo, hi).  One thread per slot (old_id: the slot's reference
// ID - 1, nullptr = ID order).
// a 32-bit hash from full-rate 24-bit multiply-adds (order_key's rounds,
// keeping all 32 bits)
__device__ __forceinline__ uint32_t lhash24(uint32_t x) {
  uint32_t h = __umul24(x, 0x9E3779u) + (x >> 8);
  h ^= h >> 15;
  h = __umul24(h, 0xEBCA77u) + (h >> 8);
  h ^= h >> 13;
  h = __umul24(h, 0x85EBCAu) + (h >> 16);
  return h;
}
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {  // murmur3 finaliser (bijective)
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_layout_keys(const uint64_t* __restrict__ words,
                                                       const uint16_t* __restrict__ len, uint64_t n,
                                                       const uint32_t* __restrict__ old_id, uint64_t lo, uint64_t hi,
                                                       int grouped, int pb, int hash24, uint64_t* __restrict__ key,
                                                       uint32_t* __restrict__ val) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int L = len[i];
  using mer_t = uint32_t;  // (31-mers hashed by mix64: same probe time, layout 2.3 vs 1.85 ms at C3)
  constexpr int kM = 16;
  const int m = L < kM ? L : kM;
  const mer_t mmask = 2 * m == 8 * (int)sizeof(mer_t) ? ~(mer_t)0 : (((mer_t)1 << (2 * m)) - 1);
  const uint64_t* g = words + i * slot_words(MAXW);
  mer_t fw = 0, rc = 0;
  uint32_t best = 0xFFFFFFFFu, bpos = 0;
  uint64_t cw = 0;
  for (int t = 0; t < L; ++t) {
    if ((t & 31) == 0) cw = g[t >> 5];
    const uint32_t b = (uint32_t)(cw >> (62 - 2 * (t & 31))) & 3u;
    fw = ((fw << 2) | b) & mmask;
    rc = (rc >> 2) | ((mer_t)(3u - b) << (2 * m - 2));
    if (t >= m - 1) {
      const mer_t c = fw < rc ? fw : rc;
      // fmix32 (two 32-bit multiplies, quarter rate) or, option layout_hash = 1,
      // two full-rate 24-bit multiply-adds (ALU: the kernel is issue-bound)
      const uint32_t hv = hash24 ? lhash24(c) : fmix32(c);
      if (hv < best) {  // the hash, leftmost on ties
        best = hv;
        bpos = (uint32_t)(t - m + 1);
      }
    }
  }
  const uint32_t pmax = (1u << pb) - 1u;
  uint64_t k = ((uint64_t)best << pb) | (bpos < pmax ? bpos : pmax);
  if (grouped) {
    const uint64_t id = old_id ? old_id[i] : i;
    const uint64_t grp = id < lo ? 0u : id < hi ? 1u : 2u;
    k |= grp << (32 + pb);
  }
  key[i] = k;
  val[i] = (uint32_t)i;
}

// new slot i <- old slot src[i]: its words (16-B pieces), length and reference
// ID, into the second slot array (committed by swapping)
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_layout_gather(const uint64_t* __restrict__ src_words,
                                                         const uint16_t* __restrict__ src_len,
                                                         const uint32_t* __restrict__ old_id,
                                                         const uint32_t* __restrict__ order, uint64_t n,
                                                         uint64_t* __restrict__ dst_words, uint16_t* __restrict__ dst_len,
                                                         uint32_t* __restrict__ id) {
  constexpr int S = slot_words(MAXW);
  constexpr int P = S >= 2 ? S / 2 : 1;  // 16-B pieces per slot
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= n * P) return;
  const uint64_t i = t / P;
  const int k = (int)(t - i * P);
  const uint32_t r = order[i];
  if (S >= 2) {
    reinterpret_cast<ulonglong2*>(dst_words)[t] = reinterpret_cast<const ulonglong2*>(src_words)[(uint64_t)r * P + k];
  } else {
    dst_words[i] = src_words[r];
  }
  if (k == 0) {
    dst_len[i] = src_len[r];
    id[i] = old_id ? old_id[r] : r;
  }
}

__global__ __launch_bounds__(kBlock) void k_layout_phys(const uint32_t* __restrict__ id, uint64_t n,
                                                       uint32_t* __restrict__ phys) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) phys[id[i]] = (uint32_t)i;
}

// per-slot values -> ID order (superReadIDs leave the device in ID order)
__global__ __launch_bounds__(kBlock) void k_unpermute_u32(const uint32_t* __restrict__ v, const uint32_t* __restrict__ id,
                                                         uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) out[id[i]] = v[i];
}

template <int W>
struct LaunchLayout {
  static int run(mg_ctx* ctx, uint64_t lo, uint64_t hi, int grouped, int pb, uint64_t* key, uint32_t* val) {
    const uint64_t n = ctx->n;
    hipLaunchKernelGGL((k_layout_keys<W>), dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       ctx->d_words, ctx->d_len, n, ctx->d_id, lo, hi, grouped, pb, ctx->layout_hash, key, val);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};
template <int W>
struct LaunchLayoutGather {
  static int run(mg_ctx* ctx, const uint32_t* order, uint64_t* dst_words, uint16_t* dst_len, uint32_t* id) {
    constexpr int S = slot_words(W);
    const uint64_t t = ctx->n * (uint64_t)(S >= 2 ? S / 2 : 1);
    hipLaunchKernelGGL((k_layout_gather<W>), dim3((uint32_t)((t + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       ctx->d_words, ctx->d_len, ctx->d_id, order, ctx->n, dst_words, dst_len, id);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

}  // namespace

// ===================================================================== ABI ===
namespace {


template <template <int> class F, typename... Args>
int dispatch_w(uint32_t maxw, Args&&... args) {
  switch (maxw) {
    case 1: return F<1>::run(args...);
    case 2: return F<2>::run(args...);
    case 3: return F<3>::run(args...);
    case 4: return F<4>::run(args...);
    case 5: return F<5>::run(args...);
    case 6: return F<6>::run(args...);
    case 8: return F<8>::run(args...);
    case 12: return F<12>::run(args...);
    case 16: return F<16>::run(args...);
    case 32: return F<32>::run(args...);
  }
  return -2;
}

// Kernels with more than 64 KiB of dynamic LDS must opt in (gfx950 has 160 KiB per CU).
template <typename K>
void allow_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

IndexParams index_params(mg_ctx* ctx) {
  IndexParams p{};
  p.words = ctx->d_words;
  p.len = ctx->d_len;
  p.n = ctx->n;
  p.h = (int)ctx->h;
  p.m = (int)ctx->m;
  p.w = (int)ctx->w;
  p.nb_log2 = ctx->nb_log2;
  p.rank = ctx->rank;
  p.nranks = ctx->nranks;
  p.cell_lo = ctx->cell_lo;
  p.cell_n = ctx->cell_n;
  p.cells = ctx->d_cells;
  p.id = ctx->d_id;
  p.stride = ctx->stride;
  return p;
}

template <int W>
struct LaunchIndexLive {
  static int run(mg_ctx* ctx, const IndexParams* p) {
    const uint32_t grid = (uint32_t)(((ctx->n + kWave - 1) / kWave + kWavesPerBlock - 1) / kWavesPerBlock);
    const size_t lds = (size_t)(W + 1) * kBlock * sizeof(uint64_t);
    if (grid == 0) return 0;
    allow_lds(k_index_live<W>, lds);
    hipLaunchKernelGGL((k_index_live<W>), dim3(grid), dim3(kBlock), lds, ctx->stream, *p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

// HashTable::insertDataset without a window scan (HashTable.cpp:50-80): the
// index of the replicated mode and of source-range shards, and the all-keys
// lookup table.  One read per lane with its words in registers; the four keys
// (hashRead, :88-104) in two passes of w steps over F[0, h) and F[n-h, n), each
// rolling the forward m-mer and its reverse complement on the same incoming
// base: F[0, h) gives o = 0 (offset t) and o = 3 (R[n-h, n) = rc F[0, h), offset
// w-1-t), F[n-h, n) gives o = 1 and o = 2 (R[0, h) = rc F[n-h, n)).  Same
// (order_key | offset) rule as key_minimizer and k_scan, so the entries equal
// k_index_build's; then one CAS insert per key.  (k_index_build -- a thread per
// key, the read staged in LDS, one LDS read per base -- took 2.0 ms at C3.)
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_index_keys(IndexParams p) {
  const int h = p.h, m = p.m, w = p.w;
  const int msh = 64 - 2 * m;
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const uint64_t nbm = (1ULL << p.nb_log2) - 1;
  for (uint64_t a = (uint64_t)blockIdx.x * kBlock + threadIdx.x; a < p.n; a += (uint64_t)gridDim.x * kBlock) {
    uint64_t rw[MAXW + 1];
    load_slot<MAXW>(p.words, (uint32_t)a, rw);
    const int n = p.len[a];
    uint32_t kf[2], kr[2];  // per pass: best forward (o = 0 / 1) and reverse (o = 3 / 2) key
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int s0 = pass ? n - h : 0;
      uint64_t f = ext_reg<MAXW>(rw, s0) >> msh;       // F[s0, s0 + m)
      uint64_t r = rc_word(f << msh) & mmask;          // its reverse complement
      const uint64_t nx = ext_reg<MAXW>(rw, s0 + m);   // the bases rolled in (w <= 32)
      uint32_t bf = order_key(f), br = order_key(r) | (uint32_t)(w - 1);
      for (int t = 1; t < w; ++t) {
        const uint64_t b = w <= 32 ? (nx >> (62 - 2 * (t - 1))) & 3u
                                   : (ext_reg<MAXW>(rw, s0 + m - 1 + t) >> 62) & 3u;
        f = ((f << 2) | b) & mmask;
        r = (r >> 2) | ((uint64_t)(3u - b) << (2 * m - 2));
        bf = min(bf, order_key(f) | (uint32_t)t);
        br = min(br, order_key(r) | (uint32_t)(w - 1 - t));
      }
      kf[pass] = bf;
      kr[pass] = br;
    }
    const uint32_t kb[4] = {kf[0], kf[1], kr[1], kr[0]};
    const int i0 = (int)(kb[0] & 1023u), i1 = (int)(kb[1] & 1023u), i2 = (int)(kb[2] & 1023u),
              i3 = (int)(kb[3] & 1023u);
    const uint64_t mb[4] = {ext_reg<MAXW>(rw, i0) >> msh, ext_reg<MAXW>(rw, n - h + i1) >> msh,
                            rc_word(ext_reg<MAXW>(rw, n - m - i2)) & mmask,
                            rc_word(ext_reg<MAXW>(rw, w - 1 - i3)) & mmask};
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      if (o == 1 && p.skip_o1) continue;
      const uint64_t v = mix64(mb[o]);
      const uint64_t b = v & nbm;
      if (owned(b, p.nb_log2, p.rank, p.nranks))
        cell_insert(p.cells, b - p.cell_lo, p.cell_n, make_entry(v, p.nb_log2, (int)(kb[o] & 1023u), o, (uint32_t)a, n));
    }
  }
}

// Exchange mode, keys first (option xchg_keys_first, equal lengths): the
// index key records of this rank's source reads [a_lo, a_hi) alone, before
// any window is scanned, so they travel to their bucket owners while nothing
// waits on them and the owners file them with CAS inserts inside their own
// window scan (k_scan<RECV>), where the fused path's inserts hide too.  Same
// keys (hashRead, HashTable.cpp:88-104) and rule as k_index_keys, written as
// the KEYREC scan writes them: key o of source a at key_seg(o) * key_n + a - a_lo
// (bucket, entry); o = 1 a hole when skip_o1.
//   kblk (non-null): the routing pass's per-(region, destination) counts, region
// = kFlatRegion records of the flat key array, so mg_xchg_pack runs no count
// pass: a block's 256 sources put each key segment's records in at most two
// regions, counted in LDS and added to kblk (cleared by the caller) with one
// global atomic per (segment, region, destination)
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_xchg_keys(IndexParams p, uint64_t a_lo, uint64_t a_hi,
                                                     uint32_t* __restrict__ key_bk, uint64_t* __restrict__ key_ent,
                                                     unsigned long long* __restrict__ kblk, uint32_t nranks) {
  constexpr uint64_t kReg = 1024;  // (= kFlatRegion)
  __shared__ unsigned int s_kc[4 * 2 * kMaxRanks];
  const int h = p.h, m = p.m, w = p.w;
  const int msh = 64 - 2 * m;
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const uint64_t nbm = (1ULL << p.nb_log2) - 1, key_n = a_hi - a_lo;
  const uint32_t ncnt = 4 * 2 * nranks;
  for (uint64_t a0 = a_lo + (uint64_t)blockIdx.x * kBlock; a0 < a_hi; a0 += (uint64_t)gridDim.x * kBlock) {
   if (kblk) {  // (block-uniform)
     for (uint32_t i = threadIdx.x; i < ncnt; i += kBlock) s_kc[i] = 0;
     __syncthreads();
   }
   const uint64_t a = a0 + threadIdx.x;
   if (a < a_hi) {
    uint64_t rw[MAXW + 1];
    load_slot<MAXW>(p.words, (uint32_t)a, rw);
    const int n = p.len[a];
    uint32_t kf[2], kr[2];  // per pass: best forward (o = 0 / 1) and reverse (o = 3 / 2) key
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int s0 = pass ? n - h : 0;
      uint64_t f = ext_reg<MAXW>(rw, s0) >> msh;
      uint64_t r = rc_word(f << msh) & mmask;
      const uint64_t nx = ext_reg<MAXW>(rw, s0 + m);
      uint32_t bf = order_key(f), br = order_key(r) | (uint32_t)(w - 1);
      for (int t = 1; t < w; ++t) {
        const uint64_t b = w <= 32 ? (nx >> (62 - 2 * (t - 1))) & 3u : (ext_reg<MAXW>(rw, s0 + m - 1 + t) >> 62) & 3u;
        f = ((f << 2) | b) & mmask;
        r = (r >> 2) | ((uint64_t)(3u - b) << (2 * m - 2));
        bf = min(bf, order_key(f) | (uint32_t)t);
        br = min(br, order_key(r) | (uint32_t)(w - 1 - t));
      }
      kf[pass] = bf;
      kr[pass] = br;
    }
    const uint32_t kb[4] = {kf[0], kf[1], kr[1], kr[0]};
    const int i0 = (int)(kb[0] & 1023u), i1 = (int)(kb[1] & 1023u), i2 = (int)(kb[2] & 1023u),
              i3 = (int)(kb[3] & 1023u);
    const uint64_t mb[4] = {ext_reg<MAXW>(rw, i0) >> msh, ext_reg<MAXW>(rw, n - h + i1) >> msh,
                            rc_word(ext_reg<MAXW>(rw, n - m - i2)) & mmask,
                            rc_word(ext_reg<MAXW>(rw, w - 1 - i3)) & mmask};
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const uint64_t v = mix64(mb[o]);
      const uint64_t at = key_seg(o) * key_n + a - a_lo;
      key_bk[at] = (uint32_t)(v & nbm);
      const bool hole = o == 1 && p.skip_o1;
      key_ent[at] = hole ? kEmpty : make_entry(v, p.nb_log2, (int)(kb[o] & 1023u), o, (uint32_t)a, n);
      if (kblk && !hole) {  // k_part's OWN_KEY rule: owner = bucket range
        const uint32_t d = (uint32_t)(((v & nbm) * nranks) >> p.nb_log2);
        const uint32_t half = (uint32_t)(at / kReg - (key_seg(o) * key_n + a0 - a_lo) / kReg);
        atomicAdd(&s_kc[((uint32_t)key_seg(o) * 2 + half) * nranks + d], 1u);
      }
    }
   }
   if (kblk) {
     __syncthreads();
     for (uint32_t i = threadIdx.x; i < ncnt; i += kBlock) {
       const uint32_t c = s_kc[i];
       if (c) {
         const uint32_t seg = i / (2 * nranks), half = (i / nranks) & 1u, d = i % nranks;
         const uint64_t r = (seg * key_n + a0 - a_lo) / kReg + half;
         atomicAdd(&kblk[r * nranks + d], (unsigned long long)c);
       }
     }
     __syncthreads();  // (the next sources' counters are cleared after every lane read these)
   }
  }
}

template <int W>
struct LaunchIndex {
  static int run(mg_ctx* ctx, uint64_t* cells = nullptr, bool all_keys = false) {
    IndexParams p = index_params(ctx);
    if (cells) p.cells = cells;
    p.skip_o1 = (!all_keys && !ctx->index_o1) ? 1 : 0;
    if (ctx->index_keys) {  // one read per lane (k_index_keys)
      const uint32_t grid = (uint32_t)std::max<uint64_t>(
          1, std::min<uint64_t>((ctx->n + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 16));
      if (!ctx->n) return 0;
      hipLaunchKernelGGL((k_index_keys<W>), dim3(grid), dim3(kBlock), 0, ctx->stream, p);
      return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    uint32_t grid = (uint32_t)((4 * ctx->n + kBlock - 1) / kBlock);  // one thread per key
    const size_t lds = (size_t)(W + 1) * kBlock * sizeof(uint64_t);
    if (grid == 0) return 0;
    allow_lds(k_index_build<W>, lds);
    hipLaunchKernelGGL((k_index_build<W>), dim3(grid), dim3(kBlock), lds, ctx->stream, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

// Persistent grids: exactly the resident blocks (a larger grid would run a
// second, partly idle round of wavefronts).  Scan and probe use the same
// wavefront count: probe wavefront r consumes scan region r.
template <typename K>
uint32_t resident_blocks(mg_ctx* ctx, K kernel, size_t lds, uint64_t want, int block = kBlock) {
  allow_lds(kernel, lds);
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds);
  const uint64_t resident = (uint64_t)std::max(1, per_cu) * (uint64_t)std::max(1, ctx->n_cu);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(std::min<uint64_t>(want, resident), ctx->max_blocks));
}

// LDS of one scan wavefront: the w suffix-minimum keys per lane + the staged
// run metas; blocks carry 4 wavefronts, or 2 / 1 when that does not fit
// (long windows: w = l - k grows with min_overlap).  0 = w too large.
constexpr size_t kLdsPerCu = 160 * 1024;
inline size_t scan_lds_per_wave(uint32_t w) {
  return (((size_t)(w + kScanKeyPad) * kWave + 1) / 2 + kScanBuf) * sizeof(uint64_t);
}
inline uint32_t scan_wpb(uint32_t w) {
  for (uint32_t wpb = kWavesPerBlock; wpb >= 1; wpb >>= 1)
    if (wpb * scan_lds_per_wave(w) <= kLdsPerCu) return wpb;
  return 0;
}
// Which window scan runs.  The index-building scan of the fused path is
// k_scan<INDEX> (LDS sliding minimum, CAS inserts hidden behind its ALU work);
// the exchange mode's scan writes key records instead, from the register
// sliding minimum (k_scan_reg<INDEX> + k_rc_keys) when w fits its unrolled
// window, else from k_scan<INDEX>.  Run-only scans (source-range shards) take
// the register scan when w fits.
// The exchange mode's index scan of mixed lengths takes k_scan's length-ranked
// windows too (option xchg_windows): one read per lane idles the lanes of
// shorter reads, and longest first scans containers before their contents.
inline bool scan_is_reg(const mg_ctx* ctx, bool index) {
  if (ctx->rk_on) return false;  // (the received keys' CAS inserts ride on k_scan<RECV>)
  return ctx->w <= (uint32_t)kRegW &&
         (!index || (ctx->xchg && !ctx->xchg_scan_lds && !(ctx->xchg_windows && ctx->minlen != ctx->maxlen)));
}
// groups per k_scan window (one run region each): the index scan of mixed
// lengths ranks each window's reads by length (kWinGroups); else 1
inline int scan_windows(const mg_ctx* ctx, bool index) {
  return (index && ctx->minlen != ctx->maxlen && !scan_is_reg(ctx, index)) ? kWinGroups : 1;
}
inline uint32_t scan_block_waves(const mg_ctx* ctx, bool index) {
  return scan_is_reg(ctx, index) ? kWavesPerBlock : scan_wpb(ctx->w);
}
inline size_t scan_lds(const mg_ctx* ctx, bool index) {
  return scan_is_reg(ctx, index) ? (size_t)kWavesPerBlock * kStageRing * sizeof(uint64_t)
                                 : (size_t)scan_wpb(ctx->w) * scan_lds_per_wave(ctx->w);
}
template <int W>
uint32_t scan_resident(mg_ctx* ctx, bool index, uint64_t want) {
  const size_t lds = scan_lds(ctx, index);
  const int block = (int)scan_block_waves(ctx, index) * kWave;
  if (scan_is_reg(ctx, index))
    return index ? resident_blocks(ctx, k_scan_reg<W, true>, lds, want, block)
                 : resident_blocks(ctx, k_scan_reg<W, false>, lds, want, block);
  if (index && ctx->xchg)
    return scan_windows(ctx, index) > 1 ? resident_blocks(ctx, k_scan<W, true, true, kWinGroups>, lds, want, block)
                                        : resident_blocks(ctx, k_scan<W, true, true>, lds, want, block);
  if (ctx->rk_on) return resident_blocks(ctx, k_scan<W, false, false, 1, true>, lds, want, block);
  return index ? (scan_windows(ctx, index) > 1 ? resident_blocks(ctx, k_scan<W, true, false, kWinGroups>, lds, want, block)
                                                : resident_blocks(ctx, k_scan<W, true>, lds, want, block))
               : resident_blocks(ctx, k_scan<W, false>, lds, want, block);
}

// Geometry of one discovery pass over source reads [a_lo, a_hi): probe grid =
// its resident blocks; the scan (fewer registers) runs kreg times as many
// wavefronts and probe wavefront r consumes scan regions r + i * (probe waves).
struct DiscGeom {
  uint32_t grid = 0, sgrid = 0, kreg = 1;
  size_t lds_scan = 0, lds_probe = 0;
};

template <int W>
DiscGeom disc_geom(mg_ctx* ctx, bool contain, uint64_t nsrc) {
  DiscGeom g;
  const uint64_t ngroups = (nsrc + kWave - 1) / kWave;
  const uint64_t want = std::max<uint64_t>(1, (ngroups + kWavesPerBlock - 1) / kWavesPerBlock);
  g.lds_scan = scan_lds(ctx, false);
  g.lds_probe = (size_t)kWavesPerBlock * ProbeLds<W>::bytes;
  g.grid = contain ? resident_blocks(ctx, k_probe<W, true>, g.lds_probe, want)
                   : resident_blocks(ctx, k_probe<W, false>, g.lds_probe, want);
  const uint32_t scan_res = scan_resident<W>(ctx, false, ~0ull >> 1);
  g.kreg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(scan_res / g.grid, (want + g.grid - 1) / g.grid));
  g.sgrid = g.grid * g.kreg;
  return g;
}

// Low fingerprint bits appended below hb bits of cell index in a sort key:
// the rest of the sort's last 8-bit digit (a cell's records of one
// fingerprint then mostly sort together, k_cells_place, at no extra pass; a
// whole extra digit cost C3 at P = 8 0.05 ms per rank for nothing, where few
// cells overflow: profiles/r04m_sim8_c3_ranks_fs_extra_digit.md)
uint32_t fp_sort_bits(uint32_t hb) {
  if (hb >= 32) return 0;
  return std::min<uint32_t>((hb + 7) / 8 * 8 - hb, kFpBits);
}

// Window scan over source slots [a_lo, a_hi): one run region per scan
// wavefront in ctx->d_runs.  filter: keep only runs whose bucket this rank owns (a
// bucket-sharded single context); index: the scan also builds the index
// (fused: CAS into the cells; exchange: key records).
template <int W>
struct LaunchScan {
  static int run(mg_ctx* ctx, bool contain, uint64_t a_lo, uint64_t a_hi, uint32_t sgrid, bool filter,
                 hipStream_t stream = nullptr, bool no_super = false, bool index = false) {
    if (!stream) stream = ctx->stream;
    const uint32_t wpb = scan_block_waves(ctx, index);
    const uint64_t nw = (uint64_t)sgrid * wpb;  // scan wavefronts
    const uint64_t ngroups = (a_hi - a_lo + kWave - 1) / kWave;
    // run regions: one per register-scan wavefront, one per window group of k_scan's
    const uint64_t G = scan_is_reg(ctx, index) ? 1 : (uint64_t)scan_windows(ctx, index);
    const uint64_t nreg = nw * G;
    ctx->nrun_reg = nreg;
    // expected runs per read ~ 2 J / (w + 1) + 1 (minimizer density), priced at
    // the middle length with 2x headroom (measured: C3 10.9, C5 13.4 per read);
    // a region that overflows is resized and rescanned (settle_runs).  Priced at
    // the longest read with 3x until round 6, C5's first allocation was 53 GB
    // per context: what failed for 8 replicated C5 contexts on one device
    const uint64_t Jmax = ctx->maxlen > ctx->h + 1 ? ctx->maxlen - ctx->h - 1 : 1;
    const uint64_t mid = ((uint64_t)ctx->minlen + ctx->maxlen) / 2;
    const uint64_t J = mid > ctx->h + 1 ? mid - ctx->h - 1 : 1;
    const uint64_t per_read = std::min<uint64_t>(Jmax, 2 * (2 * J / (ctx->w + 1) + 2));
    const uint64_t groups_per_region = ((ngroups + G - 1) / G + nw - 1) / nw;  // windows per wave
    uint64_t run_cap = std::max<uint64_t>(
        ctx->run_cap_need, ctx->run_cap_opt ? ctx->run_cap_opt : groups_per_region * kWave * per_read);
    if (run_cap * nreg > ctx->runs_cap) {
      if (ctx->d_runs) (void)hipFree(ctx->d_runs);
      ctx->d_runs = nullptr;
      ctx->runs_cap = 0;
      if (ctx_malloc(ctx, (void**)&ctx->d_runs, run_cap * nreg * sizeof(ulonglong2), "d_runs (run regions)")) return -1;
      ctx->runs_cap = run_cap * nreg;
    }
    if (!ctx->run_cap_opt) run_cap = ctx->runs_cap / std::max<uint64_t>(1, nreg);
    ctx->run_cap = run_cap;
    if (ctx->run_cnt_cap < nreg) {
      if (ctx->d_run_cnt) (void)hipFree(ctx->d_run_cnt);
      ctx->d_run_cnt = nullptr;
      ctx->run_cnt_cap = 0;
      if (ctx_malloc(ctx, (void**)&ctx->d_run_cnt, std::max<uint64_t>(1, nreg) * sizeof(unsigned long long), "d_run_cnt"))
        return -1;
      ctx->run_cnt_cap = nreg;
    }
    ctx->runs_live = false;
    ScanParams sp{};
    sp.words = ctx->d_words;
    sp.len = ctx->d_len;
    sp.super = (!no_super && !contain && ctx->contained_done && ctx->super_any) ? ctx->d_super : nullptr;
    sp.a_lo = a_lo;
    sp.a_hi = a_hi;
    sp.h = (int)ctx->h;
    sp.m = (int)ctx->m;
    sp.w = (int)ctx->w;
    sp.nb_log2 = ctx->nb_log2;
    sp.rank = filter ? ctx->rank : 0;
    sp.nranks = filter ? ctx->nranks : 1;
    sp.runs = ctx->d_runs;
    sp.run_cnt = ctx->d_run_cnt;
    sp.run_cap = run_cap;
    const size_t lds = scan_lds(ctx, index);
    sp.cells = ctx->d_cells;
    sp.cell_n = ctx->cell_n;
    sp.cell_lo = ctx->cell_lo;  // (0 unless the cells are a bucket-range shard)
    if (index && ctx->key0_ready) {  // mg_build_index allocated it (mixed lengths)
      if (ctx->prefix_probe)
        sp.p0runs = ctx->d_p0runs;
      else
        sp.key0 = ctx->d_key0;
    }
    sp.skip_o1 = (index && !ctx->index_o1) ? 1 : 0;
    sp.skip_o3 = (index && !ctx->index_o3 && !ctx->xchg) ? 1 : 0;
    sp.no_insert = (index && ctx->phase_limit == 1) ? 1 : 0;
    const bool recv = ctx->rk_on;
    ctx->runs_meta8 = false;  // (set below by the keys-first receiver scan)
    if ((index || recv) && ctx->xchg) ctx->runs_counted = false;
    // the exchange scan counts its runs per destination rank as it stores them
    // (the register scan per region, k_scan<KEYREC> per region and group: G P <= 64)
    if ((index || recv) && ctx->xchg && ctx->nranks > 1 && G * ctx->nranks <= (uint64_t)kWave) {
      MG_ENSURE(d_rcnt, rcnt_cap, nreg * ctx->nranks);
      sp.dst_cnt = ctx->d_rcnt;
      sp.dst_ranks = ctx->nranks;
      ctx->runs_counted = true;
    }
    if (index && ctx->xchg) {  // key records (bucket, entry), o-major: they travel to the bucket owner
      sp.key_bk = ctx->d_kb;
      sp.key_ent = ctx->d_ke;
      sp.key_n = a_hi - a_lo;  // the rank's sources only
      sp.key_lo = a_lo;
    }
    (void)hipEventRecord(ctx->ev[6], stream);
    if (scan_is_reg(ctx, index)) {
      if (index) {
        allow_lds(k_scan_reg<W, true>, lds);
        hipLaunchKernelGGL((k_scan_reg<W, true>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
        if (a_hi > a_lo)  // the reverse strand's keys (o = 2, 3)
          hipLaunchKernelGGL((k_rc_keys<W>), dim3((uint32_t)((a_hi - a_lo + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                             stream, sp);
      } else {
        allow_lds(k_scan_reg<W, false>, lds);
        hipLaunchKernelGGL((k_scan_reg<W, false>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
      }
    } else if (index && ctx->xchg && G > 1) {
      allow_lds(k_scan<W, true, true, kWinGroups>, lds);
      hipLaunchKernelGGL((k_scan<W, true, true, kWinGroups>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
    } else if (index && ctx->xchg) {
      allow_lds(k_scan<W, true, true>, lds);
      hipLaunchKernelGGL((k_scan<W, true, true>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
    } else if (recv) {  // exchange mode, keys first: the runs + the received keys' CAS inserts
      MG_ENSURE(d_rdst, rdst_cap, run_cap * nreg);
      sp.run_dst = ctx->d_rdst;
      ctx->runs_meta8 = true;
      sp.recv_keys = ctx->rk_keys;
      sp.recv_cnt = ctx->rk_cnt;
      sp.recv_slot = ctx->rk_slot;
      sp.recv_total = ctx->rk_total;
      sp.recv_P = ctx->nranks;
      sp.cell_lo = ctx->cell_lo;
      allow_lds(k_scan<W, false, false, 1, true>, lds);
      hipLaunchKernelGGL((k_scan<W, false, false, 1, true>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
    } else if (index && G > 1) {
      allow_lds(k_scan<W, true, false, kWinGroups>, lds);
      hipLaunchKernelGGL((k_scan<W, true, false, kWinGroups>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
    } else if (index) {
      allow_lds(k_scan<W, true>, lds);
      hipLaunchKernelGGL((k_scan<W, true>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
    } else {
      allow_lds(k_scan<W, false>, lds);
      hipLaunchKernelGGL((k_scan<W, false>), dim3(sgrid), dim3(wpb * kWave), lds, stream, sp);
    }
    (void)hipEventRecord(ctx->ev[7], stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

int settle_rows(mg_ctx* ctx, bool* again);
int settle_runs(mg_ctx* ctx, bool* again);

// k_probe over run regions (runs + r * run_cap, run_cnt[r] records), rows into
// ctx->d_rows (one region per probe wavefront) or superkey updates (contain).
// src_lo / src_hi: only runs of source slots in [src_lo, src_hi) (0, 0: all).
template <int W>
struct LaunchProbe {
  static int run(mg_ctx* ctx, bool contain, const ulonglong2* runs, const unsigned long long* run_cnt,
                 uint64_t run_cap, uint64_t run_regions, uint32_t grid, const uint32_t* src_super = nullptr,
                 uint64_t src_lo = 0, uint64_t src_hi = 0, bool append = false) {
    // discovery reads the o = 3 keys: a full table built without them (index_o3
    // = false) is only exact behind the live index that has them
    if (!contain && !ctx->index_o3 && !ctx->live_ready)
      return set_err(ctx, "discovery probe: the full index leaves out the o = 3 keys and no live index was built");
    // the candidate word packs j and the partner's length - 1 into 10 bits each
    // (and entries clamp lengths at 1,024): longer reads take k_probe_long
    if (ctx->maxlen > 1024)
      return set_err(ctx, "templated probe: reads longer than 1,024 bp must take the long-read kernels");
    ctx->nreg = (uint64_t)grid * kWavesPerBlock;  // probe wavefronts = row regions
    ProbeParams pp{};
    pp.words = ctx->d_words;
    pp.len = ctx->d_len;
    pp.h = (int)ctx->h;
    pp.m = (int)ctx->m;
    pp.nb_log2 = ctx->nb_log2;
    pp.rank = ctx->rank;
    pp.nranks = ctx->nranks;
    pp.cell_lo = ctx->cell_lo;
    pp.cell_n = ctx->cell_n;
    pp.cells = ctx->d_cells;
    if (!contain && ctx->live_ready && ctx->live_coarse) {  // exchange mode (build_live_index_xchg)
      pp.cell_shift = ctx->live_shift;
      pp.cell_n = ctx->live_cells;
      pp.cells = ctx->d_lcells;
    } else if (!contain && ctx->live_ready) {  // the discovery index of uncontained reads (build_live_index)
      pp.nb_log2 = ctx->lnb_log2;
      pp.cell_lo = 0;
      pp.cell_n = 1ull << ctx->lnb_log2;
      pp.cells = ctx->d_lcells;
    }
    // contained partners are dropped at listing (:548), except from the live
    // index, which holds the uncontained reads' keys only
    pp.cbits = (!contain && ctx->contained_done && ctx->super_any && !ctx->live_ready) ? ctx->d_cbits : nullptr;
    pp.superkey = ctx->superkey;
    pp.runs = runs;
    pp.run_cnt = run_cnt;
    pp.run_cap = run_cap;
    pp.run_regions = run_regions;
    pp.src_super = src_super;
    pp.src_lo = src_lo;
    pp.src_hi = src_hi;
    pp.rows = ctx->d_rows;
    pp.reg_cnt = ctx->d_seg;
    pp.reg_cap = contain ? 0 : ctx->rows_cap / ctx->nreg;
    pp.uniform_len = ctx->minlen == ctx->maxlen ? (int)ctx->maxlen : 0;
    pp.stats = ctx->stats ? ctx->d_stats : nullptr;
    pp.phase_limit = contain ? ctx->contain_phase_limit : ctx->phase_limit;
    pp.halving_low = ctx->halving_low ? 1 : 0;
    pp.halving_id = (ctx->read_lo || ctx->read_hi) ? ctx->d_id : nullptr;
    pp.contain_even = (contain && (ctx->xchg ? ctx->xchg_prefix : ctx->key0_ready)) ? 1 : 0;
    pp.contain_minlen = (pp.contain_even && ctx->contain_jcut) ? (int)ctx->minlen : 0;
    pp.contain_prune = (contain && ctx->contain_prune) ? 1 : 0;
    pp.contain_skip = (contain && ctx->contain_skip) ? 1 : 0;
    pp.compact = ctx->probe_compact ? 1 : 0;
    // shared regions help the discovery probe (C3 probe 4.56-4.57 vs 4.65-4.78 ms) but cost the
    // containment probe (C5 35.0 vs 29.6 ms: contain_skip finds fewer containers marked in time)
    pp.share = (!contain && ctx->probe_share) ? 1 : 0;
    pp.id = ctx->d_id;
    pp.append = append ? 1 : 0;
    if (runs == ctx->xruns_base && ctx->xruns_part && ctx->nranks > 1) {  // (a split exchange probe)
      pp.rm_part = ctx->xruns_part;
      pp.rm_P = ctx->nranks;
      pp.rm_me = ctx->rank;
      pp.rm_K = ctx->xruns_K;
    }
    // virtual regions: the split (1..probe_split_max) that gives every probe
    // wavefront (or block, with share) the same number of regions -- the fused
    // scan writes one region per scan wavefront, and the scan keeps more
    // wavefronts resident than the probe (C3: 6,144 regions for 4,096 probe
    // wavefronts, so half of them probed two regions and half one)
    // Only regions of many batches are split (a part of a few batches costs its
    // wavefront a region switch per batch: the exchange mode's 1,024-record
    // slot regions probed 2x slower split 8 ways), and only while the regions
    // are too few to even out by themselves (< 4 per probe wavefront)
    pp.vsplit = 1;
    const uint64_t nwp_all = (uint64_t)grid * kWavesPerBlock;
    const uint32_t kmax = (uint32_t)std::min<uint64_t>(ctx->probe_split_max, std::max<uint64_t>(1, run_cap / 4096));
    if (!pp.rm_part && !pp.append && run_regions && run_regions < 4 * nwp_all) {
      const uint64_t nwp = nwp_all;
      double best = 1e300;
      for (uint32_t k = 1; k <= kmax; ++k) {
        const double V = (double)(run_regions * k), rounds = (double)((run_regions * k + nwp - 1) / nwp);
        const double ratio = rounds * (double)nwp / V;  // slowest wavefront's share / the mean, >= 1
        if (ratio < best - 1e-9) {
          best = ratio;
          pp.vsplit = k;
        }
      }
    }
#ifdef MG_PROBE_SPLIT_FORCE  // (A/B builds: a fixed split wherever one is allowed)
    if (pp.vsplit > 1) pp.vsplit = MG_PROBE_SPLIT_FORCE;
#endif
    const size_t lds = (size_t)kWavesPerBlock * ProbeLds<W>::bytes;
    const bool dcnt = !contain && ctx->xchg && ctx->xchg_route_rows && ctx->nranks > 1 &&
                      ctx->nranks <= (uint32_t)kWave && ctx->n;
    if (!contain) ctx->rows_counted = false;
    if (dcnt) {  // the rows' routing takes these counts (mg_xchg_pack, MG_ROWS)
      MG_ENSURE(d_dcnt, dcnt_cap, ctx->nreg * ctx->nranks);
      pp.dst_cnt = ctx->d_dcnt;
      pp.dst_ranks = ctx->nranks;
      pp.n_ids = ctx->n;
      pp.inv_n_ids = 1.0 / (double)ctx->n;
      ctx->rows_counted = true;
      allow_lds(k_probe<W, false, true>, lds);
      hipLaunchKernelGGL((k_probe<W, false, true>), dim3(grid), dim3(kBlock), lds, ctx->stream, pp);
    } else if (contain) {
      if (pp.rm_part || pp.append) return set_err(ctx, "containment probe: no split / append form");
      hipLaunchKernelGGL((k_probe<W, true>), dim3(grid), dim3(kBlock), lds, ctx->stream, pp);
    } else if (pp.rm_part || pp.append) {  // a split exchange probe
      allow_lds(k_probe<W, false, false, true>, lds);
      hipLaunchKernelGGL((k_probe<W, false, false, true>), dim3(grid), dim3(kBlock), lds, ctx->stream, pp);
    } else {
      hipLaunchKernelGGL((k_probe<W, false>), dim3(grid), dim3(kBlock), lds, ctx->stream, pp);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

template <int W>
struct LaunchDiscover {
  // scan + probe over the context's source slots (a source-range shard);
  // `contain` selects markContainedReads semantics (all sources)
  static int run(mg_ctx* ctx, bool contain) {
    const uint64_t a_lo = contain ? 0 : ctx->read_lo;
    const uint64_t a_hi = contain ? ctx->n : (ctx->read_hi ? std::min<uint64_t>(ctx->read_hi, ctx->n) : ctx->n);
    ctx->nreg = 0;
    ctx->nrun_reg = 0;
    if (a_hi <= a_lo) return 0;
    const DiscGeom g = disc_geom<W>(ctx, contain, a_hi - a_lo);
    if (LaunchScan<W>::run(ctx, contain, a_lo, a_hi, g.sgrid, !contain)) return -1;
    return LaunchProbe<W>::run(ctx, contain, ctx->d_runs, ctx->d_run_cnt, ctx->run_cap, ctx->nrun_reg, g.grid);
  }
};

// markContainedReads at offset 0 (s = 0: read2 or its reverse strand a prefix
// of read1, OverlapGraph.cpp:302-340) through the containment probe: each
// read's window-0 run (written by the fused scan) finds, in its o = 0 key's
// cell chain, the o = 0 / 2 entries of shorter reads with the same minimizer
// offset (j = 0 in [0, 0]), and the probe's containment verify at s = 0 is
// k_prefix_contain's compare.  Batched like every other run (the cell line of
// the next batch in flight), where k_prefix_contain walked one chain per
// thread.  Runs before the main containment probe, so its contain_skip sees
// these marks; the window-0 runs never reach the discovery probe (the
// reference scans no window 0).
template <int W>
struct LaunchPrefixProbe {
  static int run(mg_ctx* ctx) {
    if (!ctx->n) return 0;
    constexpr uint64_t kR = 512;  // records per fixed region (consecutive slots)
    const uint64_t nreg = (ctx->n + kR - 1) / kR;
    MG_ENSURE(d_p0cnt, p0cnt_cap, nreg);
    hipLaunchKernelGGL(k_fixed_regions, dim3((uint32_t)((nreg + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       ctx->d_p0cnt, ctx->n, kR, nreg);
    const DiscGeom g = disc_geom<W>(ctx, true, ctx->n);
    return LaunchProbe<W>::run(ctx, true, ctx->d_p0runs, ctx->d_p0cnt, kR, nreg, g.grid);
  }
};

// Exchange mode: the window-0 runs of the o = 0 key records this rank received
// (dense, sorted by local home cell, mg_xchg_insert_keys): x = bucket |
// fingerprint << nb_log2 (what the probe reads of a run's hash), meta = the
// record's read with window range [0, 0] at its key offset q; the other
// records become holes, so the array keeps the cell order
__global__ __launch_bounds__(kBlock) void k_p0_from_keys(const uint32_t* __restrict__ key,
                                                        const uint64_t* __restrict__ ent, uint64_t n, uint32_t cshift,
                                                        uint64_t cell_lo, uint32_t nb_log2,
                                                        ulonglong2* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint64_t e = ent[i];
    const uint32_t hi = (uint32_t)(e >> 32);
    ulonglong2 r = make_ulonglong2(0, kFlatHole);
    if (e != kEmpty && !(hi & 3u))
      r = make_ulonglong2((cell_lo + (key[i] >> cshift)) | ((uint64_t)((hi >> 12) & kFpMask) << nb_log2),
                          run_meta((uint32_t)e, (int)((hi >> 2) & 1023u), 0, 0));
    out[i] = r;
  }
}

template <int W>
struct LaunchPrefixProbeKeys {
  static int run(mg_ctx* ctx) {
    const uint64_t n = ctx->xkeys_n;
    if (!n) return 0;
    MG_ENSURE(d_p0runs, p0runs_cap, n);
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + kBlock - 1) / kBlock,
                                                                           (uint64_t)ctx->n_cu * 16));
    hipLaunchKernelGGL(k_p0_from_keys, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->xkey_k, ctx->xkey_e, n,
                       ctx->xkey_cls + ctx->xkey_fs, ctx->cell_lo, ctx->nb_log2, ctx->d_p0runs);
    constexpr uint64_t kR = 512;
    const uint64_t nreg = (n + kR - 1) / kR;
    MG_ENSURE(d_p0cnt, p0cnt_cap, nreg);
    hipLaunchKernelGGL(k_fixed_regions, dim3((uint32_t)((nreg + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       ctx->d_p0cnt, n, kR, nreg);
    const DiscGeom g = disc_geom<W>(ctx, true, std::max<uint64_t>(1, n / 3));
    return LaunchProbe<W>::run(ctx, true, ctx->d_p0runs, ctx->d_p0cnt, kR, nreg, g.grid);
  }
};

// the exchange mode's offset-0 containments from the received o = 0 key records:
// their window-0 runs through the containment probe (option prefix_probe), else
// k_prefix_contain_keys' chain walk per record
int prefix_contain_keys_pass(mg_ctx* ctx) {
  if (!ctx->xchg_prefix || !ctx->n) return 0;
  if (ctx->prefix_probe ? dispatch_w<LaunchPrefixProbeKeys>(ctx->maxw, ctx)
                        : dispatch_w<LaunchPrefixContainKeys>(ctx->maxw, ctx))
    return launch_fail(ctx, "prefix containment launch failed");
  return 0;
}

// the offset-0 containments of a fused build (key0_ready): the window-0 runs
// through the containment probe (option prefix_probe, default), else k_prefix_contain
int prefix_contain_pass(mg_ctx* ctx) {
  if (!ctx->key0_ready) return 0;
  if (ctx->prefix_probe ? dispatch_w<LaunchPrefixProbe>(ctx->maxw, ctx) : dispatch_w<LaunchPrefixContain>(ctx->maxw, ctx))
    return launch_fail(ctx, "prefix containment launch failed");
  return 0;
}

// getListOfReads reads all four keys: the lookup table when the index left out o = 1
IndexParams lookup_params(mg_ctx* ctx) {
  IndexParams p = index_params(ctx);
  if ((!ctx->index_o1 || !ctx->index_o3) && !long_mode(ctx)) p.cells = ctx->d_lkcells;
  return p;
}

template <int W>
struct LaunchLookup {
  static int run(mg_ctx* ctx, const uint64_t* dq, int qwords, unsigned long long* dout, uint32_t cap,
                 unsigned int* dn) {
    IndexParams p = lookup_params(ctx);
    hipLaunchKernelGGL((k_lookup_key<W>), dim3(1), dim3(kBlock), 0, ctx->stream, p, dq, qwords, dout, cap, dn);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

// ---- long reads (> 1024 bp): the generic kernels behind the same entry points
int launch_index(mg_ctx* ctx) {
  if (!long_mode(ctx)) return dispatch_w<LaunchIndex>(ctx->maxw, ctx);
  if (!ctx->n) return 0;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((4 * ctx->n + kBlock - 1) / kBlock, 65536);
  hipLaunchKernelGGL(k_index_long, dim3(grid), dim3(kBlock), 0, ctx->stream, index_params(ctx));
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lookup(mg_ctx* ctx, const uint64_t* dq, int qwords, unsigned long long* dout, uint32_t cap,
                  unsigned int* dn) {
  if (!long_mode(ctx)) return dispatch_w<LaunchLookup>(ctx->maxw, ctx, dq, qwords, dout, cap, dn);
  hipLaunchKernelGGL((k_lookup_key<0>), dim3(1), dim3(kBlock), 0, ctx->stream, lookup_params(ctx), dq, qwords, dout,
                     cap, dn);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// k_probe_long over sources [a_lo, a_hi): containment (atomicMax into the
// superkeys) or discovery (rows; regions resized and rerun on overflow)
int long_probe(mg_ctx* ctx, bool contain, uint64_t a_lo, uint64_t a_hi) {
  LongParams p{};
  p.words = ctx->d_words;
  p.len = ctx->d_len;
  p.stride = ctx->stride;
  p.h = (int)ctx->h;
  p.m = (int)ctx->m;
  p.w = (int)ctx->w;
  p.nb_log2 = ctx->nb_log2;
  p.cell_n = ctx->cell_n;
  p.cells = ctx->d_cells;
  p.a_lo = a_lo;
  p.a_hi = a_hi;
  p.super = (!contain && ctx->contained_done && ctx->super_any) ? ctx->d_super : nullptr;
  p.superkey = ctx->superkey;
  p.halving_low = ctx->halving_low ? 1 : 0;
  const uint64_t nsrc = a_hi > a_lo ? a_hi - a_lo : 0;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(
      1, std::min<uint64_t>({(nsrc + kWavesPerBlock - 1) / kWavesPerBlock, (uint64_t)ctx->n_cu * 8, ctx->max_blocks}));
  if (contain) {
    hipLaunchKernelGGL(k_probe_long<true>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    return hipGetLastError() == hipSuccess ? 0 : launch_fail(ctx, "long-read containment launch failed");
  }
  ctx->nreg = (uint64_t)grid * kWavesPerBlock;
  for (int attempt = 0; attempt < 3; ++attempt) {
    p.rows = ctx->d_rows;
    p.reg_cnt = ctx->d_seg;
    p.reg_cap = ctx->rows_cap / ctx->nreg;
    MG_TRY(hipEventRecord(ctx->ev[8], ctx->stream));
    hipLaunchKernelGGL(k_probe_long<false>, dim3(grid), dim3(kBlock), 0, ctx->stream, p);
    MG_TRY(hipGetLastError());
    MG_TRY(hipEventRecord(ctx->ev[9], ctx->stream));
    bool again = false;
    if (settle_rows(ctx, &again)) return -1;
    if (!again) return 0;
  }
  return set_err(ctx, "discovery buffers overflow after resize");
}

// d_super in ID order (unpermuted into d_tmp32 when the slots are clustered)
const uint32_t* super_in_id_order(mg_ctx* ctx) {
  if (!ctx->d_id || !ctx->n) return ctx->d_super;
  if (ensure(ctx, &ctx->d_tmp32, &ctx->tmp32_cap, ctx->n, "d_tmp32") != hipSuccess) return ctx->d_super;
  hipLaunchKernelGGL(k_unpermute_u32, dim3((uint32_t)((ctx->n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                     ctx->d_super, ctx->d_id, ctx->n, ctx->d_tmp32);
  return ctx->d_tmp32;
}

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
  return ms;
}

}  // namespace

namespace {
// Read back the scan's per-region run counts; on overflow size the regions
// for the exact need (the scan keeps counting past capacity) and report "again".
int settle_runs(mg_ctx* ctx, bool* again) {
  *again = false;
  if (ctx->run_cnt_host.size() < ctx->nrun_reg) ctx->run_cnt_host.resize(ctx->nrun_reg);
  if (ctx->nrun_reg)
    MG_TRY(hipMemcpyAsync(ctx->run_cnt_host.data(), ctx->d_run_cnt, ctx->nrun_reg * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  uint64_t run_max = 0, total = 0;
  for (uint64_t r = 0; r < ctx->nrun_reg; ++r) {
    run_max = std::max<uint64_t>(run_max, ctx->run_cnt_host[r]);
    total += std::min<uint64_t>(ctx->run_cnt_host[r], ctx->run_cap);
  }
  ctx->scan_runs = total;
  if (run_max > ctx->run_cap) {
    ctx->run_cap_need = run_max + run_max / 8 + 64;
    *again = true;
  }
  return 0;
}

int settle_rows(mg_ctx* ctx, bool* again);

// Fused scan + probe, then check both region kinds for overflow; on overflow
// the exact need is known, so resize and rerun.
int run_discover(mg_ctx* ctx, bool contain) {
  for (int attempt = 0; attempt < 3; ++attempt) {
    const int rc = dispatch_w<LaunchDiscover>(ctx->maxw, ctx, contain);
    if (rc < 0) return launch_fail(ctx, "discovery launch failed");  // (keeps the callee's cause)
    bool again = false;
    if (settle_runs(ctx, &again)) return -1;
    if (!contain && !again && settle_rows(ctx, &again)) return -1;
    if (!again) return 0;
  }
  ctx->err = "discovery buffers overflow after resize";
  return -1;
}
}  // namespace

extern "C" {

int mg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mg_create(mg_ctx** out, int device) {
  if (!out) return -1;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -3;  // no HIP device
  if (device < 0 || device >= ndev) return -4;
  mg_ctx* ctx = new mg_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->n_cu = prop.multiProcessorCount;
  // (the side stream of live_runs_launch is made here: its first creation costs milliseconds)
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess) {
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return -1;
  }
  for (auto& e : ctx->ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      delete ctx;
      return -1;
    }
  }
  *out = ctx;
  return 0;
}

void mg_destroy(mg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  void* bufs[] = {ctx->d_words, ctx->d_len, ctx->d_cells, ctx->d_superkey, ctx->d_super, ctx->d_any, ctx->d_rows,
                  ctx->d_seg, ctx->d_stats, ctx->d_compact, ctx->d_runs, ctx->d_run_cnt, ctx->d_blk, ctx->d_flat_cnt,
                  ctx->d_slot_cnt, ctx->d_freq, ctx->d_kb, ctx->d_ke, ctx->d_key0, ctx->d_xkk[0], ctx->d_xkk[1], ctx->d_xke[0], ctx->d_xke[1], 
                  ctx->d_xflag, ctx->d_nlive,
                  ctx->d_xk[0], ctx->d_xk[1], ctx->d_xv[0], ctx->d_xv[1], ctx->d_xsort_tmp,
                  ctx->d_digest, ctx->id_store[0], ctx->id_store[1], ctx->phys_store[0], ctx->phys_store[1],
                  ctx->d_tmp32, ctx->d_lay_k[0], ctx->d_lay_k[1], ctx->d_lay_v[0], ctx->d_lay_v[1], ctx->d_lay_tmp,
                  ctx->d_words_alt, ctx->d_len_alt, ctx->d_cbits, ctx->d_ccnt, ctx->d_lcells, ctx->d_lkcells,
                  ctx->d_rhead, ctx->d_rstart, ctx->d_rcnt, ctx->d_dcnt, ctx->d_p0runs, ctx->d_p0cnt, ctx->d_xexp,
                  ctx->d_kblk, ctx->d_rdst, ctx->d_cells_alt};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* mg_last_error(const mg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* mg_stream(mg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

uint64_t mg_num_reads(const mg_ctx* ctx) { return ctx ? ctx->n : 0; }

uint64_t mg_num_rows(const mg_ctx* ctx) { return ctx ? ctx->n_rows : 0; }


static int finish_upload(mg_ctx* ctx, const uint16_t* lens_host) {
  // min/max length (Dataset::shortestReadLength / longestReadLength, Dataset.h:35-36)
  uint32_t mn = 0xFFFFFFFFu, mx = 0;
  for (uint64_t i = 0; i < ctx->n; i++) {
    mn = std::min<uint32_t>(mn, lens_host[i]);
    mx = std::max<uint32_t>(mx, lens_host[i]);
  }
  ctx->minlen = ctx->n ? mn : 0;
  ctx->maxlen = mx;
  if (apply_layout(ctx)) return -1;
  reset_derived(ctx);
  return 0;
}

int mg_upload_reads_packed(mg_ctx* ctx, const uint64_t* words, const uint16_t* lens, uint64_t n_reads,
                           uint32_t words_per_read) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (n_reads >= 0xFFFFFFFFull) return set_err(ctx, "too many reads (max 2^32-2)");
  uint32_t mx = 0;
  for (uint64_t i = 0; i < n_reads; i++) mx = std::max<uint32_t>(mx, lens[i]);
  if (mx > 32u * words_per_read) return set_err(ctx, "read longer than words_per_read * 32");
  // the slot width follows the longest read (words past it are zero)
  const uint32_t maxw = slot_maxw(std::max<uint32_t>(1, (mx + 31) / 32));
  if (!maxw) return set_err(ctx, "read longer than 65535 (Read::getReadLength is UINT16)");
  ctx->n = n_reads;
  ctx->maxw = maxw;
  ctx->stride = slot_stride(maxw);
  const size_t nw = (size_t)(n_reads + 2) * ctx->stride + 2;  // zero pad for over-reads
  MG_ENSURE(d_words, words_cap, nw);
  MG_ENSURE(d_len, len_cap, n_reads + 1);
  MG_TRY(hipMemsetAsync(ctx->d_words, 0, nw * sizeof(uint64_t), ctx->stream));
  const uint32_t copy_w = std::min<uint32_t>(words_per_read, ctx->stride);
  if (n_reads && ctx->stride == words_per_read) {
    MG_TRY(hipMemcpyAsync(ctx->d_words, words, n_reads * ctx->stride * sizeof(uint64_t), hipMemcpyHostToDevice,
                          ctx->stream));
  } else if (n_reads) {
    MG_TRY(hipMemcpy2DAsync(ctx->d_words, ctx->stride * sizeof(uint64_t), words, words_per_read * sizeof(uint64_t),
                            copy_w * sizeof(uint64_t), n_reads, hipMemcpyHostToDevice, ctx->stream));
  }
  if (n_reads)
    MG_TRY(hipMemcpyAsync(ctx->d_len, lens, n_reads * sizeof(uint16_t), hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  ctx->n_good = n_reads;
  return finish_upload(ctx, lens);
}

int mg_upload_reads_ascii(mg_ctx* ctx, const char* concat, const uint64_t* offsets, uint64_t n_reads) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (n_reads >= 0xFFFFFFFFull) return set_err(ctx, "too many reads (max 2^32-2)");
  std::vector<uint16_t> lens(n_reads);
  uint64_t mx = 0;
  for (uint64_t i = 0; i < n_reads; i++) {
    const uint64_t L = offsets[i + 1] - offsets[i];
    if (L > 65535) return set_err(ctx, "read longer than 65535 (Read::getReadLength is UINT16)");
    lens[i] = (uint16_t)L;
    mx = std::max(mx, L);
  }
  const uint32_t maxw = slot_maxw((uint32_t)std::max<uint64_t>(1, (mx + 31) / 32));
  ctx->n = n_reads;
  ctx->maxw = maxw;
  ctx->stride = slot_stride(maxw);
  const uint64_t total = n_reads ? offsets[n_reads] : 0;
  // staging buffers freed on every exit path (an error return included)
  struct Staging {
    char* ascii = nullptr;
    uint64_t* off = nullptr;
    ~Staging() {
      if (ascii) (void)hipFree(ascii);
      if (off) (void)hipFree(off);
    }
  } st;
  MG_TRY(hipMalloc(&st.ascii, std::max<uint64_t>(total, 1)));
  MG_TRY(hipMalloc(&st.off, (n_reads + 1) * sizeof(uint64_t)));
  char* const d_ascii = st.ascii;
  uint64_t* const d_off = st.off;
  const size_t nw = (size_t)(n_reads + 2) * ctx->stride + 2;
  MG_ENSURE(d_words, words_cap, nw);
  MG_ENSURE(d_len, len_cap, n_reads + 1);
  MG_TRY(hipMemsetAsync(ctx->d_words, 0, nw * sizeof(uint64_t), ctx->stream));
  if (total) MG_TRY(hipMemcpyAsync(d_ascii, concat, total, hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipMemcpyAsync(d_off, offsets, (n_reads + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  const uint64_t threads = n_reads * maxw;
  if (threads) {
    hipLaunchKernelGGL(k_pack_ascii, dim3((uint32_t)((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, d_ascii, d_off, n_reads, maxw, ctx->stride, ctx->d_words, ctx->d_len);
    MG_TRY(hipGetLastError());
  }
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  ctx->t.pack_ms = elapsed(ctx->ev[0], ctx->ev[1]);
  return finish_upload(ctx, lens.data());
}

int mg_download_reads_packed(mg_ctx* ctx, uint64_t* words, uint16_t* lens, uint32_t* words_per_read) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (words_per_read) *words_per_read = ctx->maxw;
  if (words && ctx->n)
    MG_TRY(hipMemcpy2D(words, ctx->maxw * sizeof(uint64_t), ctx->d_words, ctx->stride * sizeof(uint64_t),
                       ctx->maxw * sizeof(uint64_t), ctx->n, hipMemcpyDeviceToHost));
  if (lens && ctx->n) MG_TRY(hipMemcpy(lens, ctx->d_len, ctx->n * sizeof(uint16_t), hipMemcpyDeviceToHost));
  if (ctx->d_id && ctx->n && (words || lens)) {  // slots -> ID order
    std::vector<uint32_t> id(ctx->n);
    MG_TRY(hipMemcpy(id.data(), ctx->d_id, ctx->n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    const size_t wr = ctx->maxw;
    if (words) {
      std::vector<uint64_t> tmp(words, words + ctx->n * wr);
      for (uint64_t i = 0; i < ctx->n; ++i) std::copy(&tmp[i * wr], &tmp[i * wr] + wr, words + (size_t)id[i] * wr);
    }
    if (lens) {
      std::vector<uint16_t> tmp(lens, lens + ctx->n);
      for (uint64_t i = 0; i < ctx->n; ++i) lens[id[i]] = tmp[i];
    }
  }
  return 0;
}

int mg_read_slots(mg_ctx* ctx, uint32_t* slot_of_id) {
  if (!ctx || !slot_of_id) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (ctx->d_phys && ctx->n)
    MG_TRY(hipMemcpy(slot_of_id, ctx->d_phys, ctx->n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  else
    for (uint64_t i = 0; i < ctx->n; ++i) slot_of_id[i] = (uint32_t)i;
  return 0;
}

int mg_set_option(mg_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return -1;
  auto flag = [&](const char* opt, bool* field) {
    if (strcmp(name, opt)) return false;
    *field = value != 0;
    return true;
  };
  if (!strcmp(name, "nb_log2")) {
    if (value != 0 && (value < 10 || value > 31)) return set_err(ctx, "nb_log2 out of range [10,31]");
    ctx->nb_log2_opt = (uint32_t)value;
    ctx->index_ready = false;
    return 0;
  }
  if (!strcmp(name, "rows_cap")) {
    ctx->rows_cap_opt = (uint64_t)std::max<int64_t>(0, value);
    return 0;
  }
  if (!strcmp(name, "phase_limit")) {  // diagnostics: stop the probe after a phase (1: the scan files no keys)
    ctx->phase_limit = value > 0 ? (int)value : 99;
    return 0;
  }
  if (!strcmp(name, "contain_phase_limit")) {  // diagnostics: stop the containment probe after a phase
    ctx->contain_phase_limit = value > 0 ? (int)value : 99;
    return 0;
  }
  if (!strcmp(name, "index_keys")) {  // index builds without a scan: one read per lane (default 1)
    ctx->index_keys = value != 0;
    return 0;
  }
  if (!strcmp(name, "xchg_fused1")) {  // exchange mode at one rank: the fused build (default 1)
    ctx->xchg_fused1 = value != 0;
    return 0;
  }
  if (!strcmp(name, "check_cells")) {  // diagnostics: verify every sorted cell build (build_cells)
    ctx->check_cells = value != 0;
    return 0;
  }
  if (!strcmp(name, "xchg_fs")) {  // diagnostics: fingerprint bits of the exchange sort key (-1: auto)
    ctx->xchg_fs = (int)std::max<int64_t>(-1, std::min<int64_t>(value, kFpBits));
    return 0;
  }
  if (!strcmp(name, "max_blocks")) {  // diagnostics: cap the persistent probe grid
    ctx->max_blocks = value > 0 ? (uint32_t)value : 8192u;
    return 0;
  }
  if (!strcmp(name, "probe_split_max")) {  // largest virtual split of a run region (1 = off)
    if (value < 1 || value > 64) return set_err(ctx, "probe_split_max out of range [1,64]");
    ctx->probe_split_max = (uint32_t)value;
    return 0;
  }
  if (!strcmp(name, "layout_hash")) {  // slot layout's minimizer hash: 0 fmix32 (default), 1 24-bit multiplies
    ctx->layout_hash = value ? 1 : 0;
    return 0;
  }
  if (!strcmp(name, "xchg_keys_first")) {  // exchange mode, equal lengths: key records first (default 1)
    ctx->xchg_keys_first = value != 0;
    return 0;
  }
  if (!strcmp(name, "xchg_split_max")) {  // exchange mode: mg_xchg_probe_own splits the probe up to this many ranks
    ctx->xchg_split_max = (uint32_t)std::max<int64_t>(0, value);
    return 0;
  }
  if (!strcmp(name, "xchg_region")) {  // exchange mode: records per probe region of the received runs (power of 2)
    if (value < 0 || value > 65536 || (value & (value - 1))) return set_err(ctx, "xchg_region: a power of two <= 65536");
    ctx->xchg_region = (uint32_t)value;
    return 0;
  }
  if (!strcmp(name, "alloc_cap")) {  // tests: device allocations above this many bytes fail (0 = no cap)
    ctx->alloc_cap = (uint64_t)std::max<int64_t>(0, value);
    return 0;
  }
  if (!strcmp(name, "run_cap")) {  // tests: initial run records per scan region (0 = sized from the reads)
    ctx->run_cap_opt = (uint64_t)std::max<int64_t>(0, value);
    ctx->run_cap_need = 0;
    return 0;
  }
  if (flag("stats", &ctx->stats) || flag("halving", &ctx->halving_low) || flag("layout", &ctx->layout) ||
      flag("contain_jcut", &ctx->contain_jcut) || flag("contain_skip", &ctx->contain_skip) ||
      flag("contain_prune", &ctx->contain_prune) || flag("cells_double", &ctx->cells_double) || flag("probe_share", &ctx->probe_share) ||
      flag("probe_compact", &ctx->probe_compact) || flag("live_index", &ctx->live_index) ||
      flag("xchg_sort_runs", &ctx->xchg_sort_runs) || flag("layout_scratch", &ctx->layout_scratch) ||
      flag("xchg_windows", &ctx->xchg_windows) || flag("chain_par", &ctx->chain_par) ||
      flag("live_runs", &ctx->live_runs) || flag("live_overlap", &ctx->live_overlap) ||
      flag("xchg_route_rows", &ctx->xchg_route_rows) || flag("xchg_scan_lds", &ctx->xchg_scan_lds))
    return 0;
  if (flag("prefix_contain", &ctx->prefix_contain) || flag("prefix_probe", &ctx->prefix_probe)) {
    ctx->index_ready = false;
    return 0;
  }
  return set_err(ctx, std::string("unknown option ") + name);
}

int mg_set_shard(mg_ctx* ctx, uint32_t rank, uint32_t nranks, uint64_t read_lo, uint64_t read_hi) {
  if (!ctx) return -1;
  if (nranks == 0 || rank >= nranks) return set_err(ctx, "bad shard rank/nranks");
  if (read_hi && read_hi < read_lo) return set_err(ctx, "bad read range");
  if (rank != ctx->rank || nranks != ctx->nranks || read_lo != ctx->read_lo || read_hi != ctx->read_hi) {
    ctx->index_ready = false;  // the next mg_build_index re-clusters the slots for a new range (ensure_layout_range)
    // a new shard starts a new build: no exchange state of the last one carries over
    ctx->xchg = false;
    ctx->xchg_fused = false;
    ctx->xmarks_done = false;
    ctx->xmarks = nullptr;
    ctx->packable = 0;
  }
  ctx->rank = rank;
  ctx->nranks = nranks;
  ctx->read_lo = read_lo;
  ctx->read_hi = read_hi;
  return 0;
}

}  // extern "C"

namespace {
// Index geometry shared by the fused and the exchange paths: h, m, w, the
// directory size 2^nb (same on every rank: it depends on the global read
// count only) and this rank's bucket range; allocates and clears the local cells.
int setup_cells(mg_ctx* ctx);
int setup_index(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k, bool cells = true) {
  MG_TRY(hipSetDevice(ctx->device));
  if (min_overlap < 2) return set_err(ctx, "min_overlap must be >= 2");
  const uint32_t h = min_overlap - 1;  // HashTable.cpp:54
  uint32_t m = seed_k ? seed_k : std::min<uint32_t>(31, h);
  if (m > 32 || m > h) return set_err(ctx, "seed k must satisfy 1 <= k <= min(32, l-1)");
  const uint32_t w = h - m + 1;
  if (w > 1024) return set_err(ctx, "l-1 - k + 1 must be <= 1024");
  if (!scan_wpb(w)) return set_err(ctx, "l-1 - k + 1 too large for the scan's LDS window (use a larger seed k)");
  if (ctx->minlen && ctx->minlen <= min_overlap)
    return set_err(ctx, "every read must be longer than min_overlap (Dataset.cpp:160)");
  ctx->l = min_overlap;
  ctx->h = h;
  ctx->m = m;
  ctx->w = w;
  // cells: about one per read (4 keys per read, kCell slots per cell -> at most
  // half full); an explicit nb_log2 is raised until slots >= 1.25 x keys,
  // which bounds every probe chain
  uint32_t nbl = ctx->nb_log2_opt ? ctx->nb_log2_opt : 10;
  if (!ctx->nb_log2_opt)
    while (nbl < 31 && (1ull << nbl) < ctx->n) nbl++;
  while (nbl < 31 && (1ull << nbl) * kCell < 5 * std::max<uint64_t>(ctx->n, 1)) nbl++;
  ctx->nb_log2 = nbl;
  // rank r owns buckets b with floor(b P / 2^nb) == r, i.e. [ceil(r 2^nb / P), ceil((r+1) 2^nb / P))
  const uint64_t NB = 1ull << nbl, P = ctx->nranks, r = ctx->rank;
  ctx->cell_lo = (r * NB + P - 1) / P;
  ctx->cell_n = ((r + 1) * NB + P - 1) / P - ctx->cell_lo;
  if (cells && setup_cells(ctx)) return -1;
  ctx->index_ready = false;
  ctx->lookup_ready = false;
  ctx->contained_done = false;
  ctx->super_any = false;
  ctx->live_ready = false;
  ctx->key0_ready = false;  // set by the fused build when it writes the o = 0 keys
  ctx->xchg = false;        // mg_xchg_begin sets it after this
  ctx->xchg_fused = false;  // (a plain build after a one-rank exchange step takes no exchange shortcut)
  ctx->xruns_part = 0;
  ctx->own_probed = false;
  ctx->xmarks_done = false;
  ctx->xmarks = nullptr;
  ctx->packable = 0;
  return 0;
}

// the (cleared) cell table of this rank's bucket range
int setup_cells(mg_ctx* ctx) {
  const size_t need = ctx->cell_n * kCell;
  if (!ctx->cells_double) {
    MG_ENSURE(d_cells, cells_cap, need);
    MG_TRY(hipMemsetAsync(ctx->d_cells, 0xFF, need * sizeof(uint64_t), ctx->stream));  // kEmpty
    return 0;
  }
  // two tables (option cells_double): this build takes the one the previous
  // build cleared on the side stream (its clear ran beside that step's
  // kernels; the stream waits for it), and the table it retires -- the last
  // index, which nothing reads once a new build starts -- is cleared there for
  // the next build.  The first build after a resize clears its own table.
  if (ctx->d_cells_alt && ctx->cells_alt_clean >= need) {
    std::swap(ctx->d_cells, ctx->d_cells_alt);
    std::swap(ctx->cells_cap, ctx->cells_alt_cap);
    MG_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev[13], 0));
  } else {
    MG_ENSURE(d_cells, cells_cap, need);
    MG_TRY(hipMemsetAsync(ctx->d_cells, 0xFF, need * sizeof(uint64_t), ctx->stream));  // kEmpty
  }
  ctx->cells_alt_clean = 0;
  MG_ENSURE(d_cells_alt, cells_alt_cap, need);
  MG_TRY(hipEventRecord(ctx->ev[12], ctx->stream));  // (every reader of the retired table is before this point)
  MG_TRY(hipStreamWaitEvent(ctx->side, ctx->ev[12], 0));
  MG_TRY(hipMemsetAsync(ctx->d_cells_alt, 0xFF, need * sizeof(uint64_t), ctx->side));
  MG_TRY(hipEventRecord(ctx->ev[13], ctx->side));
  ctx->cells_alt_clean = need;
  return 0;
}

// this rank's source reads in exchange mode: [floor(r N / P), floor((r+1) N / P))
void source_range(const mg_ctx* ctx, uint64_t* lo, uint64_t* hi) {
  *lo = ctx->n * ctx->rank / ctx->nranks;
  *hi = ctx->n * (ctx->rank + 1) / ctx->nranks;
}

// Routing of key records or rows (k_part) into a slot-layout buffer; the
// per-peer stream lengths go to the caller's device counts (no host sync).
uint32_t part_grid(uint64_t nreg) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nreg, 8192)); }

// precounted: per-(region, rank) counts the producer wrote (k_scan_reg's
// dst_cnt); then one block per region and no count pass
template <int KIND>
int route_slots(mg_ctx* ctx, PartParams pp, void* out, void* self_out, uint64_t slot, uint32_t rounds,
                unsigned long long* counts, unsigned long long* precounted = nullptr) {
  const uint32_t grid = precounted ? (uint32_t)pp.nreg : part_grid(pp.nreg);
  if (!precounted) MG_ENSURE(d_blk, blk_cap, (size_t)grid * ctx->nranks);
  pp.nranks = ctx->nranks;
  pp.nb_log2 = ctx->nb_log2;
  pp.n_reads = ctx->n;
  pp.blk = precounted ? precounted : ctx->d_blk;
  pp.out = out;
  pp.self_out = self_out;
  pp.self_rank = ctx->rank;
  pp.slot = slot;
  pp.rounds = rounds;
  if (!precounted) {
    hipLaunchKernelGGL((k_part<KIND, 0>), dim3(grid), dim3(kBlock), 0, ctx->stream, pp);
    MG_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_part_scan, dim3(ctx->nranks), dim3(1024), 0, ctx->stream, pp.blk, grid, ctx->nranks,
                     counts);
  MG_TRY(hipGetLastError());
  hipLaunchKernelGGL((k_part<KIND, 1>), dim3(grid), dim3(kBlock), 0, ctx->stream, pp);
  MG_TRY(hipGetLastError());
  return 0;
}

constexpr uint64_t kFlatRegion = 1024;  // records per routing region of a flat array (more blocks in flight)
constexpr uint64_t kXRegion = 1024;     // records per probe region of the ordered received runs

// region counts of a slot-layout buffer into *buf (grown as needed)
int slot_regions(mg_ctx* ctx, unsigned long long** buf, size_t* cap, const unsigned long long* counts,
                 uint64_t slot, uint64_t reg, uint64_t nreg, int part = 0) {
  if (*cap < nreg) {
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    MG_TRY(hipMalloc(buf, nreg * sizeof(unsigned long long)));
    *cap = nreg;
  }
  if (nreg)
    hipLaunchKernelGGL(k_slot_regions, dim3((uint32_t)((nreg + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       *buf, counts, slot, reg, nreg, ctx->nranks, part, ctx->rank);
  MG_TRY(hipGetLastError());
  return 0;
}

// exchange-mode window scan of this rank's sources: key records + flat runs
template <int W>
struct LaunchScanXchg {
  static int run(mg_ctx* ctx, uint64_t lo, uint64_t hi) {
    const uint32_t wpb = scan_block_waves(ctx, true);
    const uint64_t groups = (hi - lo + kWave - 1) / kWave;
    const uint32_t sgrid = scan_resident<W>(ctx, true, (groups + wpb - 1) / wpb);
    return LaunchScan<W>::run(ctx, true, lo, hi, sgrid, false, ctx->stream, true, true);
  }
};

// exchange mode, keys first: the key records of this rank's sources alone
template <int W>
struct LaunchXchgKeys {
  static int run(mg_ctx* ctx, uint64_t lo, uint64_t hi) {
    IndexParams p = index_params(ctx);
    p.skip_o1 = ctx->index_o1 ? 0 : 1;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>((hi - lo + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 16));
    // the routing pass's counts per (flat region, destination): mg_xchg_pack's
    // k_part then runs one block per region with no count pass
    const uint64_t nreg = ((ctx->index_o1 ? 4 : 3) * (hi - lo) + kFlatRegion - 1) / kFlatRegion;
    ctx->keys_counted = false;
    unsigned long long* kblk = nullptr;
    if (ctx->nranks > 1 && nreg && ctx->nranks <= kMaxRanks) {
      MG_ENSURE(d_kblk, kblk_cap, nreg * ctx->nranks);
      MG_TRY(hipMemsetAsync(ctx->d_kblk, 0, nreg * ctx->nranks * sizeof(unsigned long long), ctx->stream));
      kblk = ctx->d_kblk;
    }
    hipLaunchKernelGGL((k_xchg_keys<W>), dim3(grid), dim3(kBlock), 0, ctx->stream, p, lo, hi, ctx->d_kb, ctx->d_ke,
                       kblk, ctx->nranks);
    if (hipGetLastError() != hipSuccess) return -1;
    ctx->keys_counted = kblk != nullptr;
    return 0;
  }
};

// ... and its window scan, which CAS-inserts the received key records (ctx->rk_on)
template <int W>
struct LaunchScanRecv {
  static int run(mg_ctx* ctx, uint64_t lo, uint64_t hi) {
    const uint32_t wpb = scan_block_waves(ctx, false);
    const uint64_t groups = (hi - lo + kWave - 1) / kWave;
    const uint32_t sgrid = scan_resident<W>(ctx, false, (groups + wpb - 1) / wpb);
    return LaunchScan<W>::run(ctx, false, lo, hi, sgrid, false, ctx->stream, true, false);
  }
};

// exchange-mode probe over received runs in the slot layout (regions of `reg`
// records, counts in ctx->d_flat_cnt)
template <int W>
struct LaunchProbeSlots {
  static int run(mg_ctx* ctx, bool contain, const ulonglong2* runs, uint64_t reg, uint64_t nregions,
                 bool append = false) {
    const DiscGeom g = disc_geom<W>(ctx, contain, std::max<uint64_t>(1, ctx->n / ctx->nranks));
    const uint32_t* sup =
        (!contain && ctx->contained_done && ctx->super_any && !ctx->runs_live) ? ctx->d_super : nullptr;
    return LaunchProbe<W>::run(ctx, contain, runs, ctx->xruns_cnt, reg, nregions, g.grid, sup, 0, 0, append);
  }
};

int ensure_rows(mg_ctx* ctx, uint64_t nsrc) {
  const uint64_t max_regions = (uint64_t)ctx->max_blocks * kWavesPerBlock;
  if (ctx->seg_cap_regions < max_regions) {
    if (ctx->d_seg) (void)hipFree(ctx->d_seg);
    ctx->d_seg = nullptr;
    ctx->seg_cap_regions = 0;
    if (ctx_malloc(ctx, (void**)&ctx->d_seg, max_regions * sizeof(unsigned long long), "d_seg")) return -1;
    ctx->seg_cap_regions = max_regions;
  }
  const uint64_t want = ctx->rows_cap_opt ? ctx->rows_cap_opt : std::max<uint64_t>(1u << 20, 48 * nsrc);
  if (want > ctx->rows_cap) {
    if (ctx->d_rows) (void)hipFree(ctx->d_rows);
    ctx->d_rows = nullptr;
    ctx->rows_cap = 0;
    if (ctx_malloc(ctx, (void**)&ctx->d_rows, want * 3 * sizeof(uint32_t), "d_rows (row regions)")) return -1;
    ctx->rows_cap = want;
  }
  if (ctx->stats) {
    if (!ctx->d_stats) MG_TRY(hipMalloc(&ctx->d_stats, (kSegs * 4 + 1) * sizeof(unsigned long long)));
    MG_TRY(hipMemsetAsync(ctx->d_stats, 0, (kSegs * 4 + 1) * sizeof(unsigned long long), ctx->stream));
  }
  return 0;
}

// read back the per-region row counts of the last probe; on overflow grow the
// row buffer and report "again" (the kernels keep counting past capacity)
int settle_rows(mg_ctx* ctx, bool* again) {
  *again = false;
  if (ctx->seg_host.size() < ctx->nreg) ctx->seg_host.resize(ctx->nreg);
  if (ctx->nreg)
    MG_TRY(hipMemcpyAsync(ctx->seg_host.data(), ctx->d_seg, ctx->nreg * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  uint64_t row_max = 0, rows = 0;
  for (uint64_t r = 0; r < ctx->nreg; ++r) {
    row_max = std::max<uint64_t>(row_max, ctx->seg_host[r]);
    rows += ctx->seg_host[r];
  }
  const uint64_t reg_cap = ctx->nreg ? ctx->rows_cap / ctx->nreg : 0;
  if (row_max > reg_cap) {
    const uint64_t want = (row_max + row_max / 4 + 1024) * ctx->nreg;
    if (ctx->d_rows) (void)hipFree(ctx->d_rows);
    ctx->d_rows = nullptr;
    ctx->rows_cap = 0;
    if (ctx_malloc(ctx, (void**)&ctx->d_rows, want * 3 * sizeof(uint32_t), "d_rows (row regions)")) return -1;
    ctx->rows_cap = want;
    *again = true;
    return 0;
  }
  ctx->n_rows = rows;
  return 0;
}

void read_stats(mg_ctx* ctx, uint64_t nsrc) {
  if (!ctx->stats) return;
  std::vector<unsigned long long> st(kSegs * 4 + 1);
  if (hipMemcpy(st.data(), ctx->d_stats, st.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return;
  uint64_t acc[4] = {0, 0, 0, 0};
  for (int s2 = 0; s2 < kSegs; ++s2)
    for (int i = 0; i < 4; ++i) acc[i] += st[s2 * 4 + i];
  ctx->counters.runs = acc[0];
  ctx->counters.entries = acc[1];
  ctx->counters.verified = acc[2];
  ctx->counters.rows = acc[3];
  ctx->counters.sources = nsrc;
  ctx->counters.live_cells = ctx->live_ready ? ctx->live_cells : 0;
}
// The window scan of ALL sources, unfiltered (runs of contained sources are
// dropped by the probe) and fused with the index build (k_scan<INDEX>):
// mg_build_index runs it as THE index build, so one pass over the reads files
// every key and leaves the runs that the containment and the discovery probes
// both consume.
template <int W>
struct LaunchScanAll {
  static int run(mg_ctx* ctx, hipStream_t st) {
    const uint32_t wpb = scan_block_waves(ctx, true);
    const uint64_t groups = (ctx->n + kWave - 1) / kWave;
    const uint32_t sgrid = scan_resident<W>(ctx, true, (groups + wpb - 1) / wpb);
    // (a bucket-range shard of every source: its buckets' keys and runs only)
    return LaunchScan<W>::run(ctx, true, 0, ctx->n, sgrid, ctx->nranks > 1, st, true, true);
  }
};

// the same scan without the index (a rerun after the shared scan's run
// regions overflowed: the cells are already filled)
template <int W>
struct LaunchScanRuns {
  static int run(mg_ctx* ctx) {
    const uint32_t wpb = scan_block_waves(ctx, false);
    const uint64_t groups = (ctx->n + kWave - 1) / kWave;
    const uint32_t sgrid = scan_resident<W>(ctx, false, (groups + wpb - 1) / wpb);
    return LaunchScan<W>::run(ctx, true, 0, ctx->n, sgrid, ctx->nranks > 1, ctx->stream, true, false);
  }
};

// one shared scan per build: an unsharded context over all its sources (a
// source-read range takes the separate index build + a scan of its slots)
// A bucket-range shard over every source (mg_set_shard(ctx, r, P, 0, 0), no
// exchange: every rank scans every read) takes the same one pass, filing and
// keeping only its own buckets' keys and runs (SURVEY §8(e) alternative (i)).
bool shared_scan(const mg_ctx* ctx) {
  return ctx->read_lo == 0 && ctx->read_hi == 0 && (ctx->nranks == 1 || ctx->minlen == ctx->maxlen);
}

// mg_build_index's timings from its events (before a rescan records ev[6] / ev[7] again)
int settle_index_times(mg_ctx* ctx) {
  if (!ctx->index_times_pending) return 0;
  MG_TRY(hipEventSynchronize(ctx->ev[1]));
  ctx->t.index_ms = elapsed(ctx->ev[0], ctx->ev[1]);
  ctx->shared_scan_ms = (!long_mode(ctx) && shared_scan(ctx) && ctx->n) ? elapsed(ctx->ev[6], ctx->ev[7]) : 0.f;
  ctx->index_times_pending = false;
  return 0;
}

// the shared scan's region counts settled (its overflow reruns a plain run scan)
int ensure_scan(mg_ctx* ctx) {
  if (settle_index_times(ctx)) return -1;
  if (ctx->scan_state == 2) return 0;
  if (ctx->scan_state == 1) {
    bool again = false;
    if (settle_runs(ctx, &again)) return -1;
    ctx->scan_state = again ? 0 : 2;
    if (!again) return 0;
  }
  for (int attempt = 0; attempt < 3; ++attempt) {
    if (ctx->n) {
      if (dispatch_w<LaunchScanRuns>(ctx->maxw, ctx)) return launch_fail(ctx, "scan launch failed");
    } else {
      ctx->nrun_reg = 0;
    }
    bool again = false;
    if (settle_runs(ctx, &again)) return -1;
    if (!again) {
      ctx->scan_state = 2;
      return 0;
    }
  }
  return set_err(ctx, "run buffers overflow after resize");
}

template <int W>
struct LaunchProbeShared {
  static int run(mg_ctx* ctx, bool contain) {
    const DiscGeom g = disc_geom<W>(ctx, contain, std::max<uint64_t>(ctx->n, 1));
    // (after k_live_runs every run's source is uncontained: no per-run check)
    const uint32_t* sup =
        (!contain && ctx->contained_done && ctx->super_any && !ctx->runs_live) ? ctx->d_super : nullptr;
    return LaunchProbe<W>::run(ctx, contain, ctx->d_runs, ctx->d_run_cnt, ctx->run_cap, ctx->nrun_reg, g.grid, sup);
  }
};

// probe the shared scan's runs (rows settled for the discovery probe)
// The discovery index (option live_index): the keys of the uncontained reads
// only, in a table sized for them (same minimizer keys and entries as the
// full index, so the runs probe it unchanged; the full table keeps serving
// getListOfReads and containment)
int build_live_index(mg_ctx* ctx) {
  ctx->live_ready = false;
  // (forced when the full table has no o = 3 keys: discovery needs them)
  const bool force = !ctx->index_o3;
  if (!force && (!ctx->live_index || !ctx->super_any || ctx->nranks > 1 || ctx->xchg || long_mode(ctx))) return 0;
  const uint64_t live = ctx->n > ctx->n_contained ? ctx->n - ctx->n_contained : 1;
  uint32_t nbl = 10;  // setup_index's rule for `live` reads
  while (nbl < 31 && (1ull << nbl) < live) nbl++;
  while (nbl < 31 && (1ull << nbl) * kCell < 5 * live) nbl++;
  if (nbl >= ctx->nb_log2 && !force) return 0;  // no smaller than the full table: probe that
  nbl = std::min(nbl, ctx->nb_log2);
  MG_ENSURE(d_lcells, lcells_cap, (1ull << nbl) * kCell);
  MG_TRY(hipMemsetAsync(ctx->d_lcells, 0xFF, (1ull << nbl) * kCell * sizeof(uint64_t), ctx->stream));
  IndexParams p = index_params(ctx);
  p.nb_log2 = nbl;
  p.rank = 0;
  p.nranks = 1;
  p.cell_lo = 0;
  p.cell_n = 1ull << nbl;
  p.cells = ctx->d_lcells;
  p.cbits = ctx->d_cbits;
  if (dispatch_w<LaunchIndexLive>(ctx->maxw, ctx, &p)) return launch_fail(ctx, "live index launch failed");
  ctx->lnb_log2 = nbl;
  ctx->live_cells = 1ull << nbl;
  ctx->live_coarse = false;
  ctx->live_ready = true;
  return 0;
}

// the sort / scan scratch of the exchange build (d_xsort_tmp), grown to tb bytes
hipError_t grow_tmp(mg_ctx* ctx, size_t tb) {
  if (tb > ctx->xsort_tmp_cap) {
    if (ctx->d_xsort_tmp) {
      const hipError_t e = hipFree(ctx->d_xsort_tmp);
      if (e != hipSuccess) return e;
    }
    ctx->d_xsort_tmp = nullptr;
    ctx->xsort_tmp_cap = 0;
    const hipError_t e = ctx_malloc(ctx, &ctx->d_xsort_tmp, tb, "d_xsort_tmp (sort scratch)");
    if (e != hipSuccess) return e;
    ctx->xsort_tmp_cap = tb;
  }
  return hipSuccess;
}

// option check_cells: fail the build when a filed record cannot be walked to
int check_cells(mg_ctx* ctx, const uint32_t* key, const uint64_t* ent, const uint32_t* start,
                const unsigned long long* n_dev, uint64_t n_host, const uint64_t* cells, uint64_t cell_n,
                uint32_t gshift, uint32_t cshift, int skip_odd) {
  if (!ctx->check_cells || !n_host) return 0;
  unsigned long long* d_bad = nullptr;
  MG_TRY(hipMalloc(&d_bad, 33 * sizeof(unsigned long long)));
  MG_TRY(hipMemsetAsync(d_bad, 0, 33 * sizeof(unsigned long long), ctx->stream));
  hipLaunchKernelGGL(k_check_cells, dim3((uint32_t)std::min<uint64_t>((n_host + kBlock - 1) / kBlock, 4096)),
                     dim3(kBlock), 0, ctx->stream, key, ent, start, n_dev, n_host, gshift, cshift, skip_odd, cells,
                     cell_n, d_bad);
  unsigned long long h[33];
  MG_TRY(hipMemcpyAsync(h, d_bad, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  (void)hipFree(d_bad);
  std::string scan_note;
  if (start && n_host <= (1u << 22)) {  // the max-scan against the host's
    std::vector<uint32_t> hh(n_host), hs(n_host);
    MG_TRY(hipMemcpy(hh.data(), ctx->d_rhead, n_host * 4, hipMemcpyDeviceToHost));
    MG_TRY(hipMemcpy(hs.data(), start, n_host * 4, hipMemcpyDeviceToHost));
    uint32_t mx = 0;
    uint64_t heads = 0, bad_scan = 0, first_bad = 0;
    for (uint64_t i = 0; i < n_host; ++i) {
      heads += hh[i] != 0;
      mx = std::max(mx, hh[i]);
      if (hs[i] != mx && !bad_scan++) first_bad = i;
    }
    scan_note = " heads " + std::to_string(heads) + " scan mismatches " + std::to_string(bad_scan) + " first at " +
                std::to_string(first_bad) + " (head " + std::to_string(hh[first_bad]) + " start " +
                std::to_string(hs[first_bad]) + ")";
  }
  if (!h[0]) return 0;
  std::string m = scan_note + " check_cells: " + std::to_string(h[0]) + " of " + std::to_string(n_host) +
                  " records unreachable (gshift " + std::to_string(gshift) + ", cshift " + std::to_string(cshift) +
                  ", cell_n " + std::to_string(cell_n) + "):";
  for (int q = 0; q < 8 && q < (int)h[0]; ++q) {
    char b[160];
    snprintf(b, sizeof(b), " [i %llu home %llu steps %llu start %lld ent %016llx]", h[1 + 4 * q], h[2 + 4 * q] >> 32,
             h[2 + 4 * q] & 0xFFFFFFFFull, (long long)h[3 + 4 * q], h[4 + 4 * q]);
    m += b;
  }
  return set_err(ctx, m);
}

// the cell table `cells` of cell_n cells from sorted records key / ent (count
// n_host, or on the device at n_dev <= n_host): clear, one store per record,
// then the records past their home's kCell: placed in parallel by their index
// in their fingerprint's run (option chain_par, k_cells_place), or walked by
// one thread per overflowing cell (k_cells_chain)
// gshift / cshift / skip_odd: as k_cells_fill (classed keys: the full table
// groups and skips by class, the coarse live table merges the classes)
int build_cells(mg_ctx* ctx, const uint32_t* key, const uint64_t* ent, const unsigned long long* n_dev,
                uint64_t n_host, uint64_t* cells, uint64_t cell_n, uint32_t gshift, uint32_t cshift, int skip_odd,
                bool par) {
  MG_TRY(hipMemsetAsync(cells, 0xFF, cell_n * kCell * sizeof(uint64_t), ctx->stream));  // kEmpty
  if (!n_host) return 0;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(
      1, std::min<uint64_t>((n_host + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 32));
  hipLaunchKernelGGL(k_cells_fill, dim3(grid), dim3(kBlock), 0, ctx->stream, key, ent, n_dev, n_host, gshift, cshift,
                     skip_odd, cells);
  MG_TRY(hipGetLastError());
  if (!par) {
    hipLaunchKernelGGL(k_cells_chain, dim3(grid), dim3(kBlock), 0, ctx->stream, key, ent, n_dev, n_host, gshift,
                       cshift, skip_odd, cells, cell_n);
    MG_TRY(hipGetLastError());
    return check_cells(ctx, key, ent, nullptr, n_dev, n_host, cells, cell_n, gshift, cshift, skip_odd);
  }
  if (n_host > 0xFFFFFFFFull) return set_err(ctx, "cell build: more than 2^32 records");
  MG_ENSURE(d_rhead, rhead_cap, n_host);
  MG_ENSURE(d_rstart, rstart_cap, n_host);
  hipLaunchKernelGGL(k_over_heads, dim3(grid), dim3(kBlock), 0, ctx->stream, key, ent, n_dev, n_host, gshift, skip_odd,
                     ctx->d_rhead);
  MG_TRY(hipGetLastError());
  size_t tb = 0;
  MG_TRY(rocprim::inclusive_scan(nullptr, tb, ctx->d_rhead, ctx->d_rstart, (size_t)n_host,
                                 rocprim::maximum<uint32_t>(), ctx->stream));
  MG_TRY(grow_tmp(ctx, tb));
  tb = ctx->xsort_tmp_cap;
  MG_TRY(rocprim::inclusive_scan(ctx->d_xsort_tmp, tb, ctx->d_rhead, ctx->d_rstart, (size_t)n_host,
                                 rocprim::maximum<uint32_t>(), ctx->stream));
  hipLaunchKernelGGL(k_cells_place, dim3(grid), dim3(kBlock), 0, ctx->stream, key, ent, ctx->d_rstart, n_dev, n_host,
                     gshift, cshift, skip_odd, cells, cell_n);
  MG_TRY(hipGetLastError());
  return check_cells(ctx, key, ent, ctx->d_rstart, n_dev, n_host, cells, cell_n, gshift, cshift, skip_odd);
}

// The exchange mode's discovery index (option live_index): after
// markContainedReads the discovery probe only lists uncontained partners
// (:548), so it walks a table of the uncontained reads' entries only.  The
// rank's cells are coarsened (cell = home cell >> s), which keeps every bucket
// on its owner, and the entries stay as they are (their fingerprints are the
// bits above the full bucket): entries of 2^s buckets share a cell, and a
// fingerprint or offset collision between them is a false candidate that the
// full-overlap verification rejects.  s is the largest shift that keeps one
// cell per live read of the rank (the full table's sizing rule).
int build_live_index_xchg(mg_ctx* ctx) {
  ctx->live_ready = false;
  ctx->live_coarse = false;
  const bool force = !ctx->index_o3;  // (discovery needs the o = 3 keys the full table left out)
  if (!ctx->cell_n || (!force && (!ctx->live_index || !ctx->super_any))) return 0;
  const double frac = (double)ctx->cell_n / (double)(1ull << ctx->nb_log2);
  const uint64_t live_reads = ctx->n > ctx->n_contained ? ctx->n - ctx->n_contained : 1;
  const uint64_t live_local = (uint64_t)((double)live_reads * frac) + 1;
  uint32_t sft = 0;
  while (sft < 24 && (ctx->cell_n >> (sft + 1)) >= live_local && (ctx->cell_n >> (sft + 1)) * kCell >= 5 * live_local)
    ++sft;
  if (!sft && !force) return 0;  // no smaller than the full table: probe that
  const uint64_t live_n = (ctx->cell_n + (1ull << sft) - 1) >> sft;
  MG_ENSURE(d_lcells, lcells_cap, live_n * kCell);
  // the live reads' records, compacted in order into the sort's other buffers
  const uint64_t n = ctx->xkeys_n;
  uint32_t* lk = ctx->xkey_k_alt;
  uint64_t* le = ctx->xkey_e_alt;
  MG_ENSURE(d_xflag, xflag_cap, std::max<uint64_t>(n, 1));
  if (!ctx->d_nlive) MG_TRY(hipMalloc(&ctx->d_nlive, sizeof(unsigned long long)));
  MG_TRY(hipMemsetAsync(ctx->d_nlive, 0, sizeof(unsigned long long), ctx->stream));
  if (n) {
    hipLaunchKernelGGL(k_live_flags, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       ctx->xkey_e, n, ctx->d_cbits, ctx->d_xflag);
    MG_TRY(hipGetLastError());
    for (int pass = 0; pass < 2; ++pass) {
      size_t tb = 0;
      MG_TRY(pass ? hipcub::DeviceSelect::Flagged(nullptr, tb, ctx->xkey_e, ctx->d_xflag, le, ctx->d_nlive, (int)n,
                                                  ctx->stream)
                  : hipcub::DeviceSelect::Flagged(nullptr, tb, ctx->xkey_k, ctx->d_xflag, lk, ctx->d_nlive, (int)n,
                                                  ctx->stream));
      MG_TRY(grow_tmp(ctx, tb));
      tb = ctx->xsort_tmp_cap;
      MG_TRY(pass ? hipcub::DeviceSelect::Flagged(ctx->d_xsort_tmp, tb, ctx->xkey_e, ctx->d_xflag, le, ctx->d_nlive,
                                                  (int)n, ctx->stream)
                  : hipcub::DeviceSelect::Flagged(ctx->d_xsort_tmp, tb, ctx->xkey_k, ctx->d_xflag, lk, ctx->d_nlive,
                                                  (int)n, ctx->stream));
    }
  }
  const uint32_t lsh = sft + ctx->xkey_cls + ctx->xkey_fs;  // (classes merged)
  if (build_cells(ctx, lk, le, ctx->d_nlive, n, ctx->d_lcells, live_n, lsh, lsh, 0, ctx->xkey_par)) return -1;
  ctx->live_shift = sft;
  ctx->live_cells = live_n;
  ctx->live_coarse = true;
  ctx->live_ready = true;
  return 0;
}

// k_live_runs over the run regions: on a side stream (option live_overlap) it
// overlaps the live index build that the caller launches next on the main
// stream (the compaction streams HBM, the build waits on memory-side CAS), and
// live_runs_join() orders the discovery probe after it; else in line
int live_runs_launch(mg_ctx* ctx, ulonglong2* runs, unsigned long long* cnt, uint64_t cap, uint64_t nreg,
                     bool* on_side) {
  *on_side = false;
  uint32_t grid = (uint32_t)std::min<uint64_t>((nreg + kWavesPerBlock - 1) / kWavesPerBlock, (uint64_t)ctx->n_cu * 8);
  hipStream_t st = ctx->stream;
  if (ctx->live_overlap) {
    if (!ctx->side) MG_TRY(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    MG_TRY(hipEventRecord(ctx->ev[10], ctx->stream));
    MG_TRY(hipStreamWaitEvent(ctx->side, ctx->ev[10], 0));
    // 8 wavefronts per CU keep 16 MB of loads in flight, enough for HBM, and
    // leave the CUs' other slots to the live index build
    grid = std::min<uint32_t>(grid, (uint32_t)ctx->n_cu * 2);
    st = ctx->side;
    *on_side = true;
  }
  hipLaunchKernelGGL(k_live_runs, dim3(grid), dim3(kBlock), 0, st, runs, cnt, cap, nreg, ctx->d_cbits);
  MG_TRY(hipGetLastError());
  if (*on_side) MG_TRY(hipEventRecord(ctx->ev[11], ctx->side));
  return 0;
}
int live_runs_join(mg_ctx* ctx, bool on_side) {
  if (on_side) MG_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev[11], 0));
  return 0;
}

// Discovery as the shared scan's first reader (equal lengths: no containment
// pass ran) goes out before the scan's run counts are read: the probe reads at
// most run_cap records of a region, and a region that overflowed is found with
// the row counts, after which scan and probe rerun.  One host round trip per
// step instead of two.
int probe_shared(mg_ctx* ctx, bool contain) {
  if (!(!contain && ctx->scan_state == 1) && ensure_scan(ctx)) return -1;
  for (int attempt = 0; attempt < 4; ++attempt) {
    ctx->nreg = 0;
    MG_TRY(hipEventRecord(ctx->ev[8], ctx->stream));
    bool side = false;
    if (!contain && ctx->contained_done && ctx->super_any && !ctx->runs_live && ctx->nrun_reg && ctx->live_runs) {
      if (live_runs_launch(ctx, ctx->d_runs, ctx->d_run_cnt, ctx->run_cap, ctx->nrun_reg, &side)) return -1;
      ctx->runs_live = true;
    }
    if (!contain && attempt == 0 && ctx->contained_done && build_live_index(ctx)) return -1;
    if (live_runs_join(ctx, side)) return -1;
    if (dispatch_w<LaunchProbeShared>(ctx->maxw, ctx, contain)) return launch_fail(ctx, "probe launch failed");
    MG_TRY(hipEventRecord(ctx->ev[9], ctx->stream));
    if (contain) return 0;
    if (ctx->scan_state == 1) {  // the scan's regions, settled now (the probe above may have cut them)
      bool cut = false;
      if (settle_runs(ctx, &cut)) return -1;
      if (settle_index_times(ctx)) return -1;
      ctx->scan_state = cut ? 0 : 2;
      if (cut) {
        if (ensure_scan(ctx)) return -1;
        continue;
      }
    }
    bool again = false;
    if (settle_rows(ctx, &again)) return -1;
    if (!again) return 0;
  }
  return set_err(ctx, "row buffers overflow after resize");
}
}  // namespace

// Exchange mode: records this rank received (every peer's stream in the slot
// layout; key records or runs, x = bucket [| fingerprint]) -> one dense array
// in the context ordered by the top 8 bits of the bucket within this rank's
// range (one onesweep pass): consecutive consumers then work in a 1/256 slice
// of the cell range, which stays in L2.  One host read: the received total.
static int sort_xrecs(mg_ctx* ctx, const ulonglong2* recv, uint64_t slot, uint32_t rounds,
                      const unsigned long long* counts, uint64_t* n_out) {
  const uint32_t P = ctx->nranks;
  std::vector<unsigned long long> c(P, 0);
  if ((uint64_t)rounds * slot) {
    MG_TRY(hipMemcpyAsync(c.data(), counts, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
  }
  uint64_t n = 0;
  for (uint32_t s = 0; s < P; ++s) n += std::min<uint64_t>(c[s], (uint64_t)rounds * slot);  // cut streams: what arrived
  if (n > 0x7FFFFFFFull) return set_err(ctx, "exchange: more than 2^31 records received on one rank");
  for (int b = 0; b < 2; ++b) {
    MG_ENSURE(d_xk[b], xk_cap[b], std::max<uint64_t>(n, 1));
    MG_ENSURE(d_xv[b], xv_cap[b], std::max<uint64_t>(n, 1));
  }
  int hb = 1;
  while (hb < 40 && (1ULL << hb) < ctx->cell_n) ++hb;  // bits of a local bucket index
  const uint32_t shift = hb > 8 ? (uint32_t)(hb - 8) : 0u;
  ctx->xv_sel = 0;
  if (n) {
    const uint64_t total = (uint64_t)rounds * P * slot;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((total + kBlock - 1) / kBlock, 65536);
    hipLaunchKernelGGL(k_xruns_keys, dim3(grid), dim3(kBlock), 0, ctx->stream, recv, slot, P, total, counts,
                       (1ULL << ctx->nb_log2) - 1, ctx->cell_lo, shift, ctx->d_xk[0], ctx->d_xv[0]);
    MG_TRY(hipGetLastError());
    // one rank: its one stream is its own scan's runs in scan order, which the
    // fused path probes unsorted (the clustered layout's locality); a bucket
    // order only pays for merging the streams of several senders (one RCCL
    // rank at C3: 15.0 -> 13.8 ms per step)
    if (P == 1 || !ctx->xchg_sort_runs) {
      *n_out = n;
      return 0;
    }
    rocprim::double_buffer<uint32_t> keys(ctx->d_xk[0], ctx->d_xk[1]);
    rocprim::double_buffer<ulonglong2> vals(ctx->d_xv[0], ctx->d_xv[1]);
    size_t tb = 0;
    MG_TRY(rocprim::radix_sort_pairs(nullptr, tb, keys, vals, (unsigned int)n, 0u, 8u, ctx->stream));
    if (tb > ctx->xsort_tmp_cap) {
      if (ctx->d_xsort_tmp) MG_TRY(hipFree(ctx->d_xsort_tmp));
      ctx->d_xsort_tmp = nullptr;
      ctx->xsort_tmp_cap = 0;
      if (ctx_malloc(ctx, &ctx->d_xsort_tmp, tb, "d_xsort_tmp (sort scratch)")) return -1;
      ctx->xsort_tmp_cap = tb;
    }
    tb = ctx->xsort_tmp_cap;
    MG_TRY(rocprim::radix_sort_pairs(ctx->d_xsort_tmp, tb, keys, vals, (unsigned int)n, 0u, 8u, ctx->stream));
    ctx->xv_sel = vals.current() == ctx->d_xv[0] ? 0 : 1;
  }
  *n_out = n;
  return 0;
}

// the received runs, ordered, and their probe regions (kXRegion records);
// both probes of the step read them, never the caller's buffer
static int sort_xruns(mg_ctx* ctx, const ulonglong2* recv, uint64_t slot, uint32_t rounds,
                      const unsigned long long* counts) {
  uint64_t n = 0;
  if (sort_xrecs(ctx, recv, slot, rounds, counts, &n)) return -1;
  const uint64_t nreg = (n + kXRegion - 1) / kXRegion;
  MG_ENSURE(d_flat_cnt, flat_cnt_cap, std::max<uint64_t>(nreg, 1));
  if (nreg)
    hipLaunchKernelGGL(k_fixed_regions, dim3((uint32_t)((nreg + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       ctx->d_flat_cnt, n, kXRegion, nreg);
  MG_TRY(hipGetLastError());
  ctx->xruns_n = n;
  ctx->xruns_ready = true;
  return 0;
}

// The received runs as probe regions: by default the receive buffer itself
// (slot layout, compacted in place by k_live_runs before the discovery probe),
// regions of the largest power of two <= kXRegion records dividing the slot,
// with device-side counts (no host read).  Each peer's stream keeps its
// sender's scan order, i.e. the clustered slot order, so consecutive runs
// share cells and partners as in the fused path; ordering them by bucket
// (option xchg_sort_runs) measured slower: C3 simulated P = 8 step 20.5 vs
// 18.4 ms, C5 133.8 vs 123.0 ms (profiles/r04e_ab_xchg_sort_runs.txt).
// part (the split discovery probe, mg_xchg_probe_own): 1 = this rank's own
// stream only (in recv since mg_xchg_pack; counts = the send counts, of which
// only this rank's entry is read), 2 = the peers' streams (after the
// all-to-all), 0 = everything
static int prepare_xruns(mg_ctx* ctx, const void* recv8, uint64_t slot, uint32_t rounds,
                         const unsigned long long* counts, int part = 0) {
  if (ctx->nranks == 1) {  // one rank: the scan's own run regions, as the fused path probes them
    ctx->xruns_base = ctx->d_runs;
    ctx->xruns_cnt = ctx->d_run_cnt;
    ctx->xruns_reg = ctx->run_cap;
    ctx->xruns_nreg = ctx->nrun_reg;
    ctx->xruns_ready = true;
    return 0;
  }
  // the 8-B metas that arrived -> 16-B probe records (x = the minimizer's
  // mix64, re-hashed from this rank's copy of the read) in the context's own
  // buffer, same slot positions, so the slot regions below apply unchanged
  const uint64_t total = (uint64_t)rounds * ctx->nranks * slot;
  MG_ENSURE(d_xexp, xexp_cap, std::max<uint64_t>(total, 1));
  if (total && dispatch_w<LaunchXrunsExpand>(ctx->maxw, ctx, reinterpret_cast<const uint64_t*>(recv8), slot, rounds,
                                             counts, ctx->d_xexp, part))
    return launch_fail(ctx, "run records launch failed");
  const void* recv = ctx->d_xexp;
  if (ctx->xchg_sort_runs) {  // (never split: mg_xchg_probe_own leaves the step whole then)
    if (sort_xruns(ctx, reinterpret_cast<const ulonglong2*>(recv), slot, rounds, counts)) return -1;
    ctx->xruns_cnt = ctx->d_flat_cnt;  // (after sort_xruns: it may have grown the counts)
    ctx->xruns_base = ctx->d_xv[ctx->xv_sel];
    ctx->xruns_reg = kXRegion;
    ctx->xruns_nreg = (ctx->xruns_n + kXRegion - 1) / kXRegion;
    return 0;
  }
  // regions of xchg_region records (default 512): at P = 8 a C3 rank receives
  // 12.7 M runs; regions of 1,024 left the persistent probe grid (4,096
  // wavefronts, a block's 4 sharing each quadruple) a fourth round of 22 blocks
  uint64_t reg = ctx->xchg_region ? ctx->xchg_region : kXRegion;
  while (reg > 1 && slot % reg) reg >>= 1;
  const uint64_t K = slot ? slot / reg : 0;
  const uint64_t nreg = (uint64_t)rounds * ctx->nranks * K;
  // (part 1 reads only this rank's entry of the send counts; part 2 the received counts)
  if (slot_regions(ctx, &ctx->d_flat_cnt, &ctx->flat_cnt_cap, counts, slot, reg, nreg, part)) return -1;
  ctx->xruns_cnt = ctx->d_flat_cnt;
  ctx->xruns_base = reinterpret_cast<ulonglong2*>(const_cast<void*>(recv));
  ctx->xruns_reg = reg;
  // a split probe walks only its part's regions (LaunchProbe maps them, ProbeParams::rm_*)
  ctx->xruns_part = part;
  ctx->xruns_K = K;
  ctx->xruns_nreg = part == 0 ? nreg : (uint64_t)rounds * K * (part == 1 ? 1 : ctx->nranks - 1);
  ctx->xruns_ready = part != 1;  // (after the own part, mg_xchg_probe prepares the peers')
  return 0;
}

// Device layout (mg_ctx.hpp): layout keys -> rocprim radix sort
// of (key, slot) -> gather into the second slot array -> commit.  Every
// buffer is the context's own and kept between uploads, so the timed window
// (ev[14] .. ev[15], t.layout_ms) holds kernels only; nothing the context
// holds changes until the commit, which swaps the slot arrays and the
// ID maps after every launch succeeded.  Composes with the current order
// (d_id), so a new source-read range re-clusters resident reads.
int layout_current(mg_ctx* ctx, bool force) {
  ctx->t.layout_ms = 0.f;
  const uint64_t n = ctx->n;
  if ((!ctx->layout && !force) || n < 2 || long_mode(ctx)) return 0;  // ID order (long reads: always)
  if (n >= 0xFFFFFFFFull) return set_err(ctx, "layout: too many reads");
  uint64_t lo = ctx->read_lo < n ? ctx->read_lo : n;
  uint64_t hi = ctx->read_hi ? std::min<uint64_t>(ctx->read_hi, n) : n;
  if (hi < lo) hi = lo;
  const int grouped = (lo > 0 || hi < n) ? 1 : 0;
  int pb = 1;
  while (pb < 10 && (1u << pb) <= ctx->maxlen) ++pb;  // offsets < maxlen (capped at 10 bits)
  for (int b = 0; b < 2; ++b) {
    MG_ENSURE(d_lay_k[b], lay_k_cap[b], n);
    MG_ENSURE(d_lay_v[b], lay_v_cap[b], n);
  }
  const unsigned kbits = 32u + (unsigned)pb + (grouped ? 2u : 0u);  // the key's significant bits
  size_t tb = 0;
  MG_TRY(rocprim::radix_sort_pairs(nullptr, tb, ctx->d_lay_k[0], ctx->d_lay_k[1], ctx->d_lay_v[0], ctx->d_lay_v[1],
                                   (unsigned int)n, 0u, kbits, ctx->stream));
  if (tb > ctx->lay_tmp_cap) {
    if (ctx->d_lay_tmp) MG_TRY(hipFree(ctx->d_lay_tmp));
    ctx->d_lay_tmp = nullptr;
    ctx->lay_tmp_cap = 0;
    if (ctx_malloc(ctx, &ctx->d_lay_tmp, tb, "d_lay_tmp (layout sort scratch)")) return -1;
    ctx->lay_tmp_cap = tb;
  }
  tb = ctx->lay_tmp_cap;
  MG_ENSURE(d_words_alt, words_alt_cap, ctx->words_cap);
  MG_ENSURE(d_len_alt, len_alt_cap, ctx->len_cap);
  // the new maps go to the pair the current order does not use
  const int sel = (ctx->d_id && ctx->d_id == ctx->id_store[0]) ? 1 : 0;
  MG_ENSURE(id_store[sel], id_cap[sel], n);
  MG_ENSURE(phys_store[sel], phys_cap[sel], n);
  uint32_t* id_new = ctx->id_store[sel];
  uint32_t* ph_new = ctx->phys_store[sel];
  const uint64_t S = slot_words((int)ctx->maxw);
  // --- timed: kernels only
  MG_TRY(hipEventRecord(ctx->ev[14], ctx->stream));
  if (dispatch_w<LaunchLayout>(ctx->maxw, ctx, lo, hi, grouped, pb, ctx->d_lay_k[0], ctx->d_lay_v[0]))
    return launch_fail(ctx, "layout key launch failed");
  MG_TRY(rocprim::radix_sort_pairs(ctx->d_lay_tmp, tb, ctx->d_lay_k[0], ctx->d_lay_k[1], ctx->d_lay_v[0],
                                   ctx->d_lay_v[1], (unsigned int)n, 0u, kbits, ctx->stream));
  if (dispatch_w<LaunchLayoutGather>(ctx->maxw, ctx, ctx->d_lay_v[1], ctx->d_words_alt, ctx->d_len_alt, id_new))
    return launch_fail(ctx, "layout gather launch failed");
  // the zero pad past the last slot (over-reads of the kernels)
  MG_TRY(hipMemsetAsync(ctx->d_words_alt + n * S, 0, (ctx->words_cap - n * S) * sizeof(uint64_t), ctx->stream));
  hipLaunchKernelGGL(k_layout_phys, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream, id_new,
                     n, ph_new);
  MG_TRY(hipGetLastError());
  MG_TRY(hipEventRecord(ctx->ev[15], ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  // --- commit
  std::swap(ctx->d_words, ctx->d_words_alt);
  std::swap(ctx->words_cap, ctx->words_alt_cap);
  std::swap(ctx->d_len, ctx->d_len_alt);
  std::swap(ctx->len_cap, ctx->len_alt_cap);
  ctx->d_id = id_new;
  ctx->d_phys = ph_new;
  ctx->layout_lo = grouped ? lo : 0;
  ctx->layout_hi = grouped ? hi : 0;
  ctx->t.layout_ms = elapsed(ctx->ev[14], ctx->ev[15]);
  if (!ctx->layout_scratch) {  // (option layout_scratch = 0: many contexts on one device, the simulated ranks)
    for (void** b : {(void**)&ctx->d_words_alt, (void**)&ctx->d_len_alt, (void**)&ctx->d_lay_k[0], (void**)&ctx->d_lay_k[1],
                     (void**)&ctx->d_lay_v[0], (void**)&ctx->d_lay_v[1], &ctx->d_lay_tmp,
                     (void**)&ctx->id_store[1 - sel], (void**)&ctx->phys_store[1 - sel]})
      if (*b) {
        MG_TRY(hipFree(*b));
        *b = nullptr;
      }
    ctx->words_alt_cap = ctx->len_alt_cap = ctx->lay_tmp_cap = 0;
    ctx->lay_k_cap[0] = ctx->lay_k_cap[1] = ctx->lay_v_cap[0] = ctx->lay_v_cap[1] = 0;
    ctx->id_cap[1 - sel] = ctx->phys_cap[1 - sel] = 0;
  }
  return 0;
}

// the reads were just written in ID order (upload / ingest)
int apply_layout(mg_ctx* ctx) {
  ctx->d_id = ctx->d_phys = nullptr;
  ctx->layout_lo = ctx->layout_hi = 0;
  return layout_current(ctx, false);
}

// a source-read range set after the upload: re-cluster so that the range's
// reads take the slots [read_lo, read_hi)
int ensure_layout_range(mg_ctx* ctx) {
  if (!ctx->d_id) return 0;  // ID order: slots are IDs
  const uint64_t n = ctx->n;
  const uint64_t lo = ctx->read_lo < n ? ctx->read_lo : n;
  const uint64_t hi = ctx->read_hi ? std::min<uint64_t>(ctx->read_hi, n) : n;
  const bool grouped = lo > 0 || hi < n;
  if (grouped ? (ctx->layout_lo == lo && ctx->layout_hi == hi) : (ctx->layout_lo == 0 && ctx->layout_hi == 0)) return 0;
  if (layout_current(ctx, true)) return -1;  // (option layout = 0 applies from the next upload)
  reset_derived(ctx);
  return 0;
}

extern "C" {

int mg_build_index(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (ensure_layout_range(ctx)) return -1;  // a source-read range set after the upload
  // the cell table exists before the timed window (its clear is inside it)
  if (setup_index(ctx, min_overlap, seed_k, false)) return -1;
  MG_ENSURE(d_cells, cells_cap, ctx->cell_n * kCell);
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  if (setup_cells(ctx)) return -1;
  ctx->scan_state = 0;
  ctx->t.sort_ms = 0.f;
  ctx->shared_scan_ms = 0.f;
  const bool mixed = ctx->minlen != ctx->maxlen;
  ctx->index_o3 = true;
  if (long_mode(ctx)) {  // reads > 1024 bp: k_index_long, one thread per key
    ctx->index_o1 = true;
    if (ctx->nranks > 1) return set_err(ctx, "reads longer than 1024 bp: bucket-sharded index not supported");
    if (launch_index(ctx)) return launch_fail(ctx, "index build launch failed");
  } else if (shared_scan(ctx)) {
    // one pass over the reads: the index inserts ride on the window scan
    // (k_scan<INDEX>), whose runs then serve the containment and discovery
    // probes.  Measured at C3 (same box): 3.58 ms vs index 2.05 + scan 1.83
    // separately; a concurrent scan on a second stream did not overlap (3.95).
    // mixed lengths: each read's o = 0 key for the prefix-containment kernel
    ctx->key0_ready = mixed && ctx->prefix_contain;
    // o = 1 keys: only the containment probe without k_prefix_contain reads them
    ctx->index_o1 = mixed && !ctx->key0_ready;
    // o = 3 keys: with k_prefix_contain the containment probe drops them, and
    // the discovery probe then walks the live reads' table (always built,
    // build_live_index), so this table holds o = 0 / 2 only
    ctx->index_o3 = !(ctx->key0_ready && ctx->live_index);
    if (ctx->key0_ready && ctx->prefix_probe) MG_ENSURE(d_p0runs, p0runs_cap, ctx->n + 1);
    if (ctx->key0_ready && !ctx->prefix_probe) MG_ENSURE(d_key0, key0_cap, ctx->n + 1);
    if (ctx->n && dispatch_w<LaunchScanAll>(ctx->maxw, ctx, ctx->stream))
      return launch_fail(ctx, "index build launch failed");
    if (!ctx->n) ctx->nrun_reg = 0;
    ctx->scan_state = 1;
  } else {  // the whole index for a source-range shard (its containment probe reads suffix-key hits)
    ctx->index_o1 = mixed;
    if (dispatch_w<LaunchIndex>(ctx->maxw, ctx)) return launch_fail(ctx, "index build launch failed");
  }
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  ctx->index_times_pending = true;  // (read by settle_index_times once the events completed)
  ctx->index_ready = true;
  return 0;
}

int mg_mark_contained(mg_ctx* ctx, uint32_t* super_out) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->index_ready) return set_err(ctx, "mg_build_index must run first");
  const uint32_t* super_was = ctx->d_super;
  MG_ENSURE(d_super, super_cap, ctx->n + 1);
  if (ctx->d_super != super_was) ctx->super_zero_n = 0;  // (a new buffer: nothing known about it)
  MG_ENSURE(d_cbits, cbits_cap, (ctx->n + 63) / 64 * 2);
  if (!ctx->d_any) MG_TRY(hipMalloc(&ctx->d_any, sizeof(unsigned int)));
  ctx->t.contained_ms = 0.f;
  if (ctx->minlen != ctx->maxlen) {  // OverlapGraph.cpp:228-233
    MG_ENSURE(d_superkey, superkey_cap, ctx->n + 1);
    ctx->superkey = ctx->d_superkey;
    MG_TRY(hipMemsetAsync(ctx->d_superkey, 0, (ctx->n + 1) * sizeof(unsigned long long), ctx->stream));
    MG_TRY(hipMemsetAsync(ctx->d_any, 0, sizeof(unsigned int), ctx->stream));
    if (!ctx->d_ccnt) MG_TRY(hipMalloc(&ctx->d_ccnt, 64 * 16 * sizeof(unsigned int)));
    MG_TRY(hipMemsetAsync(ctx->d_ccnt, 0, 64 * 16 * sizeof(unsigned int), ctx->stream));
    if (ctx->stats) {  // containment work counters (mg_counters c_*)
      if (!ctx->d_stats) MG_TRY(hipMalloc(&ctx->d_stats, (kSegs * 4 + 1) * sizeof(unsigned long long)));
      MG_TRY(hipMemsetAsync(ctx->d_stats, 0, (kSegs * 4 + 1) * sizeof(unsigned long long), ctx->stream));
    }
    MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
    // sharded contexts still need the full superReadID vector: run over all
    // buckets (the containment pass is small, only for mixed lengths)
    if (ctx->nranks > 1) return set_err(ctx, "containment with a bucket-sharded index: use the exchange mode");
    if (long_mode(ctx)) {
      if (long_probe(ctx, true, 0, ctx->n)) return -1;
    } else {
      if (!shared_scan(ctx)) ctx->key0_ready = false;  // only the shared scan writes the o = 0 keys
      // prefix containments first: what they mark is skipped as a container
      if (prefix_contain_pass(ctx)) return -1;
      if (shared_scan(ctx) ? probe_shared(ctx, true) : run_discover(ctx, true)) return -1;
    }
    if (ctx->n)
      hipLaunchKernelGGL(k_super_finalize, dim3(super_grid(ctx)), dim3(kBlock), 0,
                         ctx->stream, ctx->d_superkey, ctx->n, ctx->d_super, ctx->d_any, ctx->d_cbits, ctx->d_ccnt);
    ctx->super_zero_n = 0;
    MG_TRY(hipGetLastError());
    MG_TRY(hipEventRecord(ctx->ev[3], ctx->stream));
    unsigned int any = 0;
    unsigned int ccnt[64 * 16];
    MG_TRY(hipMemcpyAsync(&any, ctx->d_any, sizeof(any), hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipMemcpyAsync(ccnt, ctx->d_ccnt, sizeof(ccnt), hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
    ctx->t.contained_ms = elapsed(ctx->ev[2], ctx->ev[3]);
    ctx->super_any = any != 0;
    ctx->n_contained = 0;
    for (int c = 0; c < 64; ++c) ctx->n_contained += ccnt[c * 16];
    ctx->live_ready = false;
    if (ctx->stats) {
      std::vector<unsigned long long> st(kSegs * 4 + 1);
      MG_TRY(hipMemcpy(st.data(), ctx->d_stats, st.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      uint64_t acc[4] = {0, 0, 0, 0};
      for (int s2 = 0; s2 < kSegs; ++s2)
        for (int i = 0; i < 4; ++i) acc[i] += st[s2 * 4 + i];
      ctx->counters.c_runs = acc[0];
      ctx->counters.c_entries = acc[1];
      ctx->counters.c_verified = acc[2];
      ctx->counters.c_contained = acc[3];
    }
  } else {
    // every superReadID 0 (one read length: nothing is contained); the memset
    // only when a finalize or a new buffer left other values
    if (ctx->super_zero_n < ctx->n + 1) {
      MG_TRY(hipMemsetAsync(ctx->d_super, 0, (ctx->n + 1) * sizeof(uint32_t), ctx->stream));
      ctx->super_zero_n = ctx->n + 1;
    }
    ctx->super_any = false;
  }
  ctx->contained_done = true;
  if (super_out) {
    super_out[0] = 0;
    if (ctx->n)
      MG_TRY(hipMemcpyAsync(super_out + 1, super_in_id_order(ctx), ctx->n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
  }
  return 0;
}

int mg_find_overlaps(mg_ctx* ctx, uint64_t* n_rows) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->index_ready) return set_err(ctx, "mg_build_index must run first");
  if (!ctx->contained_done && mg_mark_contained(ctx, nullptr)) return -1;
  const uint64_t nsrc = (ctx->read_hi ? std::min(ctx->read_hi, ctx->n) : ctx->n) -
                        std::min(ctx->read_lo, ctx->n);
  if (ensure_rows(ctx, nsrc)) return -1;
  MG_TRY(hipEventRecord(ctx->ev[4], ctx->stream));
  if (long_mode(ctx)) {
    const uint64_t lo = std::min(ctx->read_lo, ctx->n), hi = ctx->read_hi ? std::min(ctx->read_hi, ctx->n) : ctx->n;
    if (long_probe(ctx, false, lo, hi)) return -1;
    MG_TRY(hipEventRecord(ctx->ev[5], ctx->stream));
    MG_TRY(hipEventSynchronize(ctx->ev[5]));
    if (settle_index_times(ctx)) return -1;
    ctx->t.scan_ms = 0.f;
    ctx->t.sort_ms = 0.f;
    ctx->t.verify_ms = 0.f;
    ctx->t.probe_ms = elapsed(ctx->ev[8], ctx->ev[9]);
    ctx->t.overlap_ms = ctx->t.probe_ms;
    ctx->t.total_ms = ctx->t.index_ms + ctx->t.contained_ms + ctx->t.overlap_ms;
    read_stats(ctx, nsrc);
    if (n_rows) *n_rows = ctx->n_rows;
    return 0;
  }
  if (shared_scan(ctx) ? probe_shared(ctx, false) : run_discover(ctx, false)) return -1;
  MG_TRY(hipEventRecord(ctx->ev[5], ctx->stream));
  MG_TRY(hipEventSynchronize(ctx->ev[5]));
  if (settle_index_times(ctx)) return -1;
  // the kernels' own events bracket the last launches (a resize retry included
  // in ev[4]..ev[5] is not kernel time)
  // scan kernel time (shared scan: measured at build time, part of index_ms)
  ctx->t.scan_ms = shared_scan(ctx) ? ctx->shared_scan_ms : elapsed(ctx->ev[6], ctx->ev[7]);
  ctx->t.probe_ms = shared_scan(ctx) ? elapsed(ctx->ev[8], ctx->ev[9]) : elapsed(ctx->ev[7], ctx->ev[5]);
  ctx->t.verify_ms = 0.f;
  ctx->t.sort_ms = 0.f;
  ctx->t.overlap_ms = (shared_scan(ctx) ? 0.f : ctx->t.scan_ms) + ctx->t.probe_ms;
  read_stats(ctx, nsrc);
  // device wall of the step: index build start .. last discovery kernel end
  ctx->t.total_ms = shared_scan(ctx) ? elapsed(ctx->ev[0], ctx->ev[5])
                                     : ctx->t.index_ms + ctx->t.contained_ms + ctx->t.overlap_ms;
  if (n_rows) *n_rows = ctx->n_rows;
  return 0;
}

/* ---------------------------------------------------------- exchange mode --- */
uint32_t mg_record_bytes(int what) { return what == MG_ROWS ? 12u : (what == MG_KEYS || what == MG_RUNS) ? 8u : 0u; }

int mg_xchg_caps(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k, uint64_t* caps) {
  if (!ctx || !caps) return -1;
  if (min_overlap < 2) return set_err(ctx, "min_overlap must be >= 2");
  const uint64_t h = min_overlap - 1, m = seed_k ? seed_k : std::min<uint64_t>(31, h);
  if (m > 32 || m > h) return set_err(ctx, "seed k must satisfy 1 <= k <= min(32, l-1)");
  const uint64_t w = h - m + 1, P = ctx->nranks;
  const uint64_t src = (ctx->n + P - 1) / P;  // the most source reads a rank owns
  const uint64_t J = ctx->maxlen > h + 1 ? ctx->maxlen - h - 1 : 1;
  auto per_peer = [&](uint64_t total) { return P == 1 ? total : total / P + total / (4 * P); };
  caps[0] = per_peer(4 * src) + 1024;                                // 4 keys per read, hashed buckets
  caps[1] = per_peer(src * (2 * J / (w + 1) + 2) * 6 / 5) + 1024;   // the flat scan's run estimate
  caps[2] = per_peer(32 * src) + 4096;                              // rows: grown from the counts seen
  return 0;
}

int mg_xchg_begin(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (ctx->nranks > (uint32_t)kMaxRanks) return set_err(ctx, "at most 64 ranks");
  if (long_mode(ctx)) return set_err(ctx, "reads longer than 1024 bp: exchange mode not supported (use the replicated mode)");
  if (ensure_layout_range(ctx)) return -1;
  ctx->xchg_fused = false;
  if (ctx->nranks == 1 && shared_scan(ctx) && ctx->xchg_fused1) {
    // one rank: no key leaves it, so the step is the fused path's (the CAS
    // inserts ride on the window scan, k_scan<INDEX>, instead of key records
    // sorted and filed by mg_xchg_insert_keys); the mg_xchg_* calls that
    // follow delegate to its containment and discovery
    if (mg_build_index(ctx, min_overlap, seed_k)) return -1;
    ctx->xchg_fused = true;
    ctx->packable = (1 << MG_KEYS) | (1 << MG_RUNS);
    return 0;
  }
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  if (setup_index(ctx, min_overlap, seed_k, false)) return -1;
  // this rank's cells: mg_xchg_insert_keys writes every one of them (no clear)
  MG_ENSURE(d_cells, cells_cap, ctx->cell_n * kCell);
  ctx->xchg = true;
  ctx->xruns_ready = false;
  ctx->own_probed = false;
  ctx->xruns_part = 0;
  ctx->xchg_prefix = ctx->minlen != ctx->maxlen && ctx->prefix_contain;
  ctx->index_o1 = ctx->minlen != ctx->maxlen && !ctx->xchg_prefix;  // (key records of o = 1: holes otherwise)
  // the full table leaves out o = 3 as the fused path does (containment drops
  // them; discovery walks the coarse live table, built from all received records)
  ctx->index_o3 = !(ctx->xchg_prefix && ctx->live_index);
  uint64_t lo, hi;
  source_range(ctx, &lo, &hi);
  ctx->xchg_lo = lo;
  ctx->xchg_hi = hi;
  MG_ENSURE(d_kb, kb_cap, 4 * (hi - lo) + 1);
  MG_ENSURE(d_ke, ke_cap, 4 * (hi - lo) + 1);
  ctx->scan_state = 0;
  ctx->shared_scan_ms = 0.f;
  ctx->t = mg_timings{};
  // keys first (equal lengths, several ranks): only the key records now; the
  // window scan runs in mg_xchg_insert_keys, with the received keys' CAS
  // inserts riding on it (mixed lengths keep the one scan: their containment
  // and live index read the received key records sorted)
  ctx->keys_first = ctx->xchg_keys_first && ctx->nranks > 1 && ctx->minlen == ctx->maxlen;
  ctx->keys_counted = false;  // (set by k_xchg_keys' launch: the scan's key records take k_part's count pass)
  if (ctx->keys_first) {
    ctx->nrun_reg = 0;
    if (hi > lo && dispatch_w<LaunchXchgKeys>(ctx->maxw, ctx, lo, hi)) return launch_fail(ctx, "key records launch failed");
    ctx->packable = 1 << MG_KEYS;
    return 0;
  }
  if (hi > lo) {
    // one scan: the four keys of every source read (o-major records) + its
    // runs in per-wavefront regions, as the fused path writes them
    for (int attempt = 0;; ++attempt) {
      if (attempt == 3) return set_err(ctx, "run buffers overflow after resize");
      if (dispatch_w<LaunchScanXchg>(ctx->maxw, ctx, lo, hi)) return launch_fail(ctx, "scan launch failed");
      bool again = false;
      if (settle_runs(ctx, &again)) return -1;
      if (!again) break;
    }
    ctx->shared_scan_ms = elapsed(ctx->ev[6], ctx->ev[7]);
  } else {
    ctx->nrun_reg = 0;
  }
  ctx->packable = (1 << MG_KEYS) | (1 << MG_RUNS);
  return 0;
}

int mg_xchg_pack(mg_ctx* ctx, int what, void* dst, uint64_t slot, uint32_t rounds, uint64_t* counts,
                 void* self_dst) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (what < MG_KEYS || what > MG_ROWS || !(ctx->packable & (1 << what)))
    return set_err(ctx, "mg_xchg_pack: nothing of that kind to pack now (call order)");
  if (ctx->nranks == 1) {
    // one rank: every stream is its own, so nothing is routed or copied; the
    // consumers (mg_xchg_insert_keys, mg_xchg_probe) read the context's key
    // records and run regions, and the rows stay in the context
    // (mg_num_rows, mg_rows_digest, mg_copy_rows); counts = 0
    if (!counts) return set_err(ctx, "mg_xchg_pack: null counts");
    MG_TRY(hipMemsetAsync(counts, 0, sizeof(uint64_t), ctx->stream));
    return 0;
  }
  if (!slot || !rounds || !counts || (!dst && !(self_dst && ctx->nranks == 1)))
    return set_err(ctx, "mg_xchg_pack: bad slot geometry");
  auto* cnt = reinterpret_cast<unsigned long long*>(counts);
  const uint64_t nsrc = ctx->xchg_hi - ctx->xchg_lo;
  if (what == MG_KEYS) {
    PartParams pp{};
    pp.cap = kFlatRegion;
    pp.flat_n = (ctx->index_o1 ? 4 : 3) * nsrc;  // (no o = 1 keys: the last segment is holes, key_seg)
    pp.nreg = (pp.flat_n + kFlatRegion - 1) / kFlatRegion;
    pp.key_bk = ctx->d_kb;
    pp.key_ent = ctx->d_ke;
    pp.key_n = nsrc;  // (key o of source a - xchg_lo at o * nsrc + a - xchg_lo)
    pp.a_lo = 0;
    pp.nsrc = nsrc;
    if (ctx->keys_counted && pp.nreg)  // k_xchg_keys counted them per (region, rank): no count pass
      return route_slots<OWN_KEY>(ctx, pp, dst, self_dst, slot, rounds, cnt, ctx->d_kblk);
    return route_slots<OWN_KEY>(ctx, pp, dst, self_dst, slot, rounds, cnt);
  }
  if (what == MG_RUNS) {  // the scan's run regions, each run to its bucket's owner
    PartParams pp{};
    pp.base = ctx->d_runs;
    pp.cap = ctx->run_cap;
    pp.cnt = ctx->d_run_cnt;
    pp.nreg = ctx->nrun_reg;
    if (ctx->runs_meta8) {  // (the keys-first receiver scan: 8-B metas + owner bytes, counted per rank)
      pp.dst8 = ctx->d_rdst;
      if (ctx->runs_counted && pp.nreg)
        return route_slots<OWN_META>(ctx, pp, dst, self_dst, slot, rounds, cnt, ctx->d_rcnt);
      return route_slots<OWN_META>(ctx, pp, dst, self_dst, slot, rounds, cnt);
    }
    if (ctx->runs_counted && pp.nreg)  // the scan counted them per rank: one block per region, no count pass
      return route_slots<OWN_BUCKET>(ctx, pp, dst, self_dst, slot, rounds, cnt, ctx->d_rcnt);
    return route_slots<OWN_BUCKET>(ctx, pp, dst, self_dst, slot, rounds, cnt);
  }
  PartParams pp{};
  pp.base = ctx->d_rows;
  pp.cap = ctx->nreg ? ctx->rows_cap / ctx->nreg : 0;
  pp.cnt = ctx->d_seg;
  pp.nreg = ctx->n_rows ? ctx->nreg : 0;
  if (ctx->rows_counted && pp.nreg)  // the probe counted them per rank: no count pass
    return route_slots<OWN_SRC>(ctx, pp, dst, self_dst, slot, rounds, cnt, ctx->d_dcnt);
  return route_slots<OWN_SRC>(ctx, pp, dst, self_dst, slot, rounds, cnt);
}

int mg_xchg_insert_keys(mg_ctx* ctx, const void* recv, uint64_t slot, uint32_t rounds, const uint64_t* counts) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->xchg && !ctx->xchg_fused) return set_err(ctx, "mg_xchg_begin must run first");
  if (ctx->xchg_fused) return 0;  // one rank: the fused build filed the keys already
  const uint32_t P = ctx->nranks;
  if (ctx->keys_first) {
    // the cells cleared, then the window scan of this rank's sources, which
    // CAS-inserts every received key record as it goes (k_scan<RECV>); a rerun
    // after a run-region overflow inserts nothing again
    const uint64_t total = (uint64_t)rounds * P * slot;
    if (total && (!recv || !counts)) return set_err(ctx, "mg_xchg_insert_keys: null buffer");
    if (setup_cells(ctx)) return -1;
    ctx->rk_keys = reinterpret_cast<const uint64_t*>(recv);
    ctx->rk_cnt = reinterpret_cast<const unsigned long long*>(counts);
    ctx->rk_slot = slot;
    ctx->rk_total = total;
    const uint64_t lo = ctx->xchg_lo, hi = ctx->xchg_hi;
    int rc = 0;
    if (hi > lo) {
      for (int attempt = 0;; ++attempt) {
        if (attempt == 3) {
          rc = set_err(ctx, "run buffers overflow after resize");
          break;
        }
        ctx->rk_on = true;
        rc = dispatch_w<LaunchScanRecv>(ctx->maxw, ctx, lo, hi);
        ctx->rk_on = false;
        if (rc) {
          rc = launch_fail(ctx, "scan launch failed");
          break;
        }
        bool again = false;
        if ((rc = settle_runs(ctx, &again))) break;
        if (!again) break;
        ctx->rk_total = 0;  // (the keys are in)
      }
      if (!rc) ctx->shared_scan_ms = elapsed(ctx->ev[6], ctx->ev[7]);
    } else if (total) {  // no sources of its own: the received keys still go in
      ctx->rk_on = true;
      rc = dispatch_w<LaunchScanRecv>(ctx->maxw, ctx, (uint64_t)0, (uint64_t)0);
      ctx->rk_on = false;
      if (rc) rc = launch_fail(ctx, "scan launch failed");
      ctx->nrun_reg = 0;
    }
    ctx->rk_on = false;
    ctx->rk_keys = nullptr;
    ctx->rk_cnt = nullptr;
    if (rc) return -1;
    ctx->xkeys_n = 0;
    ctx->packable = (1 << MG_KEYS) | (1 << MG_RUNS);
    MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
    ctx->index_ready = true;
    return 0;
  }
  uint64_t n = 0;
  uint32_t* k0 = nullptr;
  uint64_t* e0 = nullptr;
  if (P == 1) {
    // one rank: its own key records are the input (mg_xchg_pack packed nothing);
    // without o = 1 keys they are the first three segments (key_seg)
    n = (ctx->index_o1 ? 4 : 3) * (ctx->xchg_hi - ctx->xchg_lo);
    k0 = ctx->d_kb;
    e0 = ctx->d_ke;
    MG_ENSURE(d_xkk[1], xkk_cap[1], std::max<uint64_t>(n, 1));
    MG_ENSURE(d_xke[1], xke_cap[1], std::max<uint64_t>(n, 1));
  } else {
    const uint64_t total = (uint64_t)rounds * P * slot;
    if (total) {
      if (!recv || !counts) return set_err(ctx, "mg_xchg_insert_keys: null buffer");
      std::vector<unsigned long long> c(P, 0);
      MG_TRY(hipMemcpyAsync(c.data(), counts, P * sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
      MG_TRY(hipStreamSynchronize(ctx->stream));
      for (uint32_t q = 0; q < P; ++q) n += std::min<uint64_t>(c[q], (uint64_t)rounds * slot);  // cut streams: what arrived
    }
    for (int b = 0; b < 2; ++b) {
      MG_ENSURE(d_xkk[b], xkk_cap[b], std::max<uint64_t>(n, 1));
      MG_ENSURE(d_xke[b], xke_cap[b], std::max<uint64_t>(n, 1));
    }
    k0 = ctx->d_xkk[0];
    e0 = ctx->d_xke[0];
  }
  if (n > 0x7FFFFFFFull) return set_err(ctx, "exchange: more than 2^31 key records on one rank");
  ctx->xkey_k = k0;
  ctx->xkey_e = e0;
  ctx->xkey_k_alt = ctx->d_xkk[1];
  ctx->xkey_e_alt = ctx->d_xke[1];
  int hb = 0;
  while (hb < 32 && (1ull << hb) < ctx->cell_n) ++hb;  // bits of a local cell index
  ctx->xkey_cls = (!ctx->index_o3 && hb < 31) ? 1 : 0;
  if (!ctx->index_o3 && !ctx->xkey_cls) return set_err(ctx, "exchange: local cell index too wide for the o = 3 class bit");
  hb += (int)ctx->xkey_cls;
  // low fingerprint bits below the cell (chain_par: a group's records of one
  // fingerprint adjacent), filling the sort's last 8-bit digit, or one more
  // digit when that leaves fewer than 4
  uint32_t fs = ctx->chain_par ? fp_sort_bits((uint32_t)hb) : 0u;
  if (ctx->xchg_fs >= 0) fs = std::min<uint32_t>((uint32_t)ctx->xchg_fs, hb < 32 ? 32u - (uint32_t)hb : 0u);
  ctx->xkey_fs = fs;
  // the parallel placement needs a group's fingerprints mostly sorted: with
  // fewer than 3 spare bits in the last digit (one rank at C3: none) runs of
  // different fingerprints interleave, and one walk per group is faster (one
  // RCCL rank, index 4.50 vs 4.68-4.75 ms, profiles/r04x2_ab_chain_par_xchg1.txt)
  ctx->xkey_par = ctx->chain_par && (fs >= 3 || ctx->xchg_fs >= 0);
  if (P > 1 && n) {  // the received records made dense, their sort keys formed on the way
    if (dispatch_w<LaunchXkeysDense>(ctx->maxw, ctx, reinterpret_cast<const uint64_t*>(recv), slot, rounds,
                                     reinterpret_cast<const unsigned long long*>(counts), k0, e0))
      return launch_fail(ctx, "key records launch failed");
  } else if ((ctx->xkey_cls || fs) && n) {
    hipLaunchKernelGGL(k_key_class, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream, k0, e0,
                       n, ctx->xkey_cls, fs);
    MG_TRY(hipGetLastError());
  }
  hb += (int)fs;
  if (hb > 0 && n > 1) {  // a cell's records consecutive
    rocprim::double_buffer<uint32_t> keys(k0, ctx->d_xkk[1]);
    rocprim::double_buffer<uint64_t> vals(e0, ctx->d_xke[1]);
    size_t tb = 0;
    MG_TRY(rocprim::radix_sort_pairs(nullptr, tb, keys, vals, (unsigned int)n, 0u, (unsigned)hb, ctx->stream));
    MG_TRY(grow_tmp(ctx, tb));
    tb = ctx->xsort_tmp_cap;
    MG_TRY(rocprim::radix_sort_pairs(ctx->d_xsort_tmp, tb, keys, vals, (unsigned int)n, 0u, (unsigned)hb, ctx->stream));
    ctx->xkey_k = keys.current();
    ctx->xkey_e = vals.current();
    ctx->xkey_k_alt = keys.alternate();
    ctx->xkey_e_alt = vals.alternate();
  }
  ctx->xkeys_n = n;
  if (build_cells(ctx, ctx->xkey_k, ctx->xkey_e, nullptr, n, ctx->d_cells, ctx->cell_n, fs, fs + ctx->xkey_cls,
                  ctx->xkey_cls, ctx->xkey_par))
    return -1;
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  ctx->index_ready = true;
  return 0;
}

// One rank's exchange step on the fused build (mg_xchg_begin, xchg_fused): the
// probes of mg_mark_contained / mg_find_overlaps over the scan's own run
// regions; the superkey array is mg_begin_contained's, and mg_finalize_contained
// turns it into superReadIDs as in the exchange step
static int xchg_fused_probe(mg_ctx* ctx, bool contain) {
  if (contain) {
    if (!ctx->xmarks_done) MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
    if (!ctx->n) return 0;
    // prefix containments first: what they mark is skipped as a container
    // (one rank: mg_xchg_prefix_marks ran them already, its marks are its own)
    if (!ctx->xmarks_done && prefix_contain_pass(ctx)) return -1;
    ctx->xmarks_done = false;
    ctx->xmarks = nullptr;
    if (probe_shared(ctx, true)) return -1;
    MG_TRY(hipEventRecord(ctx->ev[3], ctx->stream));
    return 0;
  }
  if (ensure_rows(ctx, ctx->n)) return -1;
  MG_TRY(hipEventRecord(ctx->ev[4], ctx->stream));
  if (probe_shared(ctx, false)) return -1;
  MG_TRY(hipEventRecord(ctx->ev[5], ctx->stream));
  MG_TRY(hipEventSynchronize(ctx->ev[5]));
  if (settle_index_times(ctx)) return -1;
  ctx->t.scan_ms = ctx->shared_scan_ms;
  ctx->t.sort_ms = 0.f;
  ctx->t.contained_ms = ctx->minlen != ctx->maxlen ? elapsed(ctx->ev[2], ctx->ev[3]) : 0.f;
  ctx->t.probe_ms = elapsed(ctx->ev[8], ctx->ev[9]);
  ctx->t.verify_ms = 0.f;
  ctx->t.overlap_ms = ctx->t.probe_ms;
  ctx->t.total_ms = elapsed(ctx->ev[0], ctx->ev[5]);
  read_stats(ctx, ctx->n);
  ctx->packable |= 1 << MG_ROWS;
  return 0;
}

int mg_xchg_probe(mg_ctx* ctx, int contain, const void* recv, uint64_t slot, uint32_t rounds, const uint64_t* counts) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if ((!ctx->xchg && !ctx->xchg_fused) || !ctx->index_ready) return set_err(ctx, "mg_xchg_insert_keys must run first");
  if (contain && !ctx->superkey) return set_err(ctx, "mg_begin_contained must run first (lengths differ)");
  if (!contain && !ctx->contained_done) return set_err(ctx, "containment must be settled first (mg_finalize_contained)");
  if (ctx->xchg_fused) return xchg_fused_probe(ctx, contain != 0);
  if (ctx->nranks > 1 && (uint64_t)rounds * slot && (!recv || !counts)) return set_err(ctx, "mg_xchg_probe: null buffer");
  // the first probe of the step sets up the received runs (both probes read
  // them); after mg_xchg_probe_own, the peers' streams only
  const bool split = !contain && ctx->own_probed;
  ctx->own_probed = false;
  if (!ctx->xruns_ready && prepare_xruns(ctx, recv, slot, rounds, reinterpret_cast<const unsigned long long*>(counts),
                                         split ? 2 : 0))
    return -1;
  const uint64_t reg = ctx->xruns_reg;
  uint64_t nregions = ctx->xruns_nreg;
  ulonglong2* runs = ctx->xruns_base;
  ctx->nreg = 0;
  ctx->n_rows = 0;
  if (contain) {
    if (!ctx->xmarks_done) MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
    // prefix containments first (what they mark is skipped as a container);
    // after mg_xchg_prefix_marks they ran already, and the all-reduced marks
    // of every rank fold into the keys here
    if (ctx->xmarks_done) {
      if (ctx->xmarks && ctx->n) {
        const uint32_t grid = (uint32_t)std::min<uint64_t>((ctx->n + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 16);
        hipLaunchKernelGGL(k_fold_marks, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->superkey, ctx->n, ctx->xmarks);
        MG_TRY(hipGetLastError());
      }
    } else if (prefix_contain_keys_pass(ctx)) {
      return -1;
    }
    ctx->xmarks_done = false;
    ctx->xmarks = nullptr;
    if (nregions && dispatch_w<LaunchProbeSlots>(ctx->maxw, ctx, true, runs, reg, nregions))
      return launch_fail(ctx, "probe launch failed");
    MG_TRY(hipEventRecord(ctx->ev[3], ctx->stream));
    return 0;
  }
  if (ensure_rows(ctx, std::max<uint64_t>(1, ctx->n / ctx->nranks))) return -1;
  for (int attempt = 0;; ++attempt) {
    if (attempt == 3) return set_err(ctx, "row buffers overflow after resize");
    if (split && attempt == 1) {  // a rerun probes every stream in one launch
      ctx->xruns_part = 0;
      nregions = (uint64_t)rounds * ctx->nranks * ctx->xruns_K;
      if (slot_regions(ctx, &ctx->d_flat_cnt, &ctx->flat_cnt_cap, reinterpret_cast<const unsigned long long*>(counts),
                       slot, reg, nregions, 0))
        return -1;
    }
    if (!(split && attempt == 0)) MG_TRY(hipEventRecord(ctx->ev[4], ctx->stream));  // (split: at the own part)
    bool side = false;
    if (attempt == 0 && nregions && ctx->contained_done && ctx->super_any) {
      // runs of contained sources contribute nothing (:548): drop them from the
      // run regions in place (the containment probe has read them already), so
      // the probe batches live runs only
      if (live_runs_launch(ctx, runs, ctx->xruns_cnt, reg, nregions, &side)) return -1;
      ctx->runs_live = true;
    }
    if (attempt == 0 && ctx->contained_done && (ctx->super_any || !ctx->index_o3) && build_live_index_xchg(ctx))
      return -1;
    if (live_runs_join(ctx, side)) return -1;
    if (nregions && dispatch_w<LaunchProbeSlots>(ctx->maxw, ctx, false, runs, reg, nregions, split && attempt == 0))
      return launch_fail(ctx, "probe launch failed");
    MG_TRY(hipEventRecord(ctx->ev[5], ctx->stream));
    if (!nregions) break;
    bool again = false;
    if (settle_rows(ctx, &again)) return -1;
    if (!again) break;
  }
  MG_TRY(hipEventSynchronize(ctx->ev[5]));
  // device times of this step (events on the context's stream; the exchanges
  // between them ran on the same stream when the caller used it)
  ctx->t.scan_ms = ctx->shared_scan_ms;
  ctx->t.sort_ms = 0.f;
  ctx->t.index_ms = elapsed(ctx->ev[0], ctx->ev[1]);
  ctx->t.contained_ms = ctx->minlen != ctx->maxlen ? elapsed(ctx->ev[2], ctx->ev[3]) : 0.f;
  ctx->t.probe_ms = elapsed(ctx->ev[4], ctx->ev[5]);
  ctx->t.verify_ms = 0.f;
  ctx->t.overlap_ms = ctx->t.probe_ms;
  ctx->t.total_ms = elapsed(ctx->ev[0], ctx->ev[5]);
  read_stats(ctx, ctx->xchg_hi - ctx->xchg_lo);
  ctx->packable |= 1 << MG_ROWS;
  return 0;
}

int mg_xchg_keys_first(const mg_ctx* ctx) { return ctx && ctx->xchg && ctx->keys_first ? 1 : 0; }

int mg_xchg_probe_own(mg_ctx* ctx, const void* recv, uint64_t slot, uint32_t rounds, const uint64_t* send_counts) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  ctx->own_probed = false;
  if ((!ctx->xchg && !ctx->xchg_fused) || !ctx->index_ready) return set_err(ctx, "mg_xchg_insert_keys must run first");
  if (!ctx->contained_done) return set_err(ctx, "containment must be settled first (mg_finalize_contained)");
  // the split pays where nothing else needs every stream first: equal lengths
  // (no containment pass), several ranks, the runs probed in place
  // and few ranks: the own stream is 1/P of the runs, and a launch over it
  // costs more than it hides once the peers' transfers are short (C3 at P = 8:
  // 0.09 ms for 1.6 M runs, the second part 0.53 vs one probe of 0.55 ms)
  if (ctx->xchg_fused || ctx->nranks == 1 || ctx->nranks > ctx->xchg_split_max || ctx->super_any ||
      ctx->minlen != ctx->maxlen || ctx->xchg_sort_runs || !((uint64_t)rounds * slot))
    return 0;
  if (!recv || !send_counts) return set_err(ctx, "mg_xchg_probe_own: null buffer");
  if (ensure_rows(ctx, std::max<uint64_t>(1, ctx->n / ctx->nranks))) return -1;
  ctx->nreg = 0;
  ctx->n_rows = 0;
  MG_TRY(hipEventRecord(ctx->ev[4], ctx->stream));
  if (prepare_xruns(ctx, recv, slot, rounds, reinterpret_cast<const unsigned long long*>(send_counts), 1)) return -1;
  if (ctx->xruns_nreg &&
      dispatch_w<LaunchProbeSlots>(ctx->maxw, ctx, false, ctx->xruns_base, ctx->xruns_reg, ctx->xruns_nreg, false))
    return launch_fail(ctx, "probe launch failed");
  ctx->own_probed = true;
  return 0;
}

int mg_xchg_prefix_marks(mg_ctx* ctx, void* marks) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if ((!ctx->xchg && !ctx->xchg_fused) || !ctx->index_ready) return set_err(ctx, "mg_xchg_insert_keys must run first");
  if (!ctx->superkey) return set_err(ctx, "mg_begin_contained must run first (lengths differ)");
  MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
  if (ctx->xchg_fused) {  // one rank on the fused build: its own o = 0 keys
    if (ctx->n && prefix_contain_pass(ctx)) return -1;
  } else if (prefix_contain_keys_pass(ctx)) {
    return -1;
  }
  ctx->xmarks = reinterpret_cast<uint8_t*>(marks);
  if (marks && ctx->n) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((ctx->n + kBlock - 1) / kBlock, (uint64_t)ctx->n_cu * 16);
    hipLaunchKernelGGL(k_prefix_marks, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->superkey, ctx->n, ctx->xmarks);
    MG_TRY(hipGetLastError());
  }
  ctx->xmarks_done = true;
  return 0;
}

int mg_begin_contained(mg_ctx* ctx, void* superkey, int* needed) {
  if (!ctx || !needed) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  *needed = ctx->minlen != ctx->maxlen;  // OverlapGraph.cpp:228-233
  ctx->contained_done = false;
  ctx->live_ready = false;
  ctx->n_contained = 0;
  ctx->superkey = nullptr;
  ctx->xmarks_done = false;
  ctx->xmarks = nullptr;
  if (*needed) {
    if (superkey) {
      ctx->superkey = reinterpret_cast<unsigned long long*>(superkey);
    } else {
      MG_ENSURE(d_superkey, superkey_cap, ctx->n + 1);
      ctx->superkey = ctx->d_superkey;
    }
    MG_TRY(hipMemsetAsync(ctx->superkey, 0, ctx->n * sizeof(unsigned long long), ctx->stream));
  }
  return 0;
}

int mg_finalize_contained(mg_ctx* ctx, uint32_t* super_out) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  const uint32_t* super_was = ctx->d_super;
  MG_ENSURE(d_super, super_cap, ctx->n + 1);
  if (ctx->d_super != super_was) ctx->super_zero_n = 0;  // (a new buffer: nothing known about it)
  MG_ENSURE(d_cbits, cbits_cap, (ctx->n + 63) / 64 * 2);
  if (!ctx->d_any) MG_TRY(hipMalloc(&ctx->d_any, sizeof(unsigned int)));
  ctx->super_any = false;
  if (ctx->minlen != ctx->maxlen && ctx->superkey) {
    MG_TRY(hipMemsetAsync(ctx->d_any, 0, sizeof(unsigned int), ctx->stream));
    if (!ctx->d_ccnt) MG_TRY(hipMalloc(&ctx->d_ccnt, 64 * 16 * sizeof(unsigned int)));
    MG_TRY(hipMemsetAsync(ctx->d_ccnt, 0, 64 * 16 * sizeof(unsigned int), ctx->stream));
    if (ctx->n)
      hipLaunchKernelGGL(k_super_finalize, dim3(super_grid(ctx)), dim3(kBlock), 0,
                         ctx->stream, ctx->superkey, ctx->n, ctx->d_super, ctx->d_any, ctx->d_cbits, ctx->d_ccnt);
    ctx->super_zero_n = 0;
    MG_TRY(hipGetLastError());
    unsigned int any = 0;
    unsigned int ccnt[64 * 16];
    MG_TRY(hipMemcpyAsync(&any, ctx->d_any, sizeof(any), hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipMemcpyAsync(ccnt, ctx->d_ccnt, sizeof(ccnt), hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
    ctx->super_any = any != 0;
    ctx->n_contained = 0;
    for (int c = 0; c < 64; ++c) ctx->n_contained += ccnt[c * 16];
  } else {
    // every superReadID 0 (one read length: nothing is contained); the memset
    // only when a finalize or a new buffer left other values
    if (ctx->super_zero_n < ctx->n + 1) {
      MG_TRY(hipMemsetAsync(ctx->d_super, 0, (ctx->n + 1) * sizeof(uint32_t), ctx->stream));
      ctx->super_zero_n = ctx->n + 1;
    }
  }
  ctx->contained_done = true;
  ctx->superkey = nullptr;  // a caller-owned key array is not referenced past this call
  if (super_out) {
    super_out[0] = 0;
    if (ctx->n)
      MG_TRY(hipMemcpyAsync(super_out + 1, super_in_id_order(ctx), ctx->n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
  }
  // (equal lengths and no copy: nothing to wait for; the exchange step keeps
  // its queue full through this call)
  return 0;
}

int mg_copy_rows(mg_ctx* ctx, mg_edge* out, uint64_t cap, uint64_t* n_copied) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (n_copied) *n_copied = 0;
  if (!ctx->nreg || !ctx->n_rows) return 0;
  // gather the per-wavefront regions into one contiguous array, then one copy
  const uint64_t reg_cap = ctx->rows_cap / ctx->nreg;
  std::vector<uint64_t> prefix(ctx->nreg + 1, 0);
  for (uint64_t r = 0; r < ctx->nreg; ++r)
    prefix[r + 1] = prefix[r] + std::min<uint64_t>(ctx->seg_host[r], reg_cap);
  const uint64_t total = prefix[ctx->nreg];
  uint64_t* d_prefix = nullptr;
  MG_TRY(hipMalloc(&d_prefix, prefix.size() * sizeof(uint64_t)));
  MG_TRY(hipMemcpyAsync(d_prefix, prefix.data(), prefix.size() * sizeof(uint64_t), hipMemcpyHostToDevice,
                        ctx->stream));
  MG_ENSURE(d_compact, compact_cap, total * 3);
  hipLaunchKernelGGL(k_compact_rows, dim3((uint32_t)ctx->nreg), dim3(kBlock), 0, ctx->stream, ctx->d_rows, reg_cap,
                     d_prefix, ctx->d_compact);
  MG_TRY(hipGetLastError());
  const uint64_t c = std::min(cap, total);
  if (c) MG_TRY(hipMemcpyAsync(out, ctx->d_compact, c * sizeof(mg_edge), hipMemcpyDeviceToHost, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  (void)hipFree(d_prefix);
  if (n_copied) *n_copied = c;
  return 0;
}

int mg_lookup_key(mg_ctx* ctx, const char* key, uint32_t key_len, uint64_t* out, uint64_t cap, uint64_t* n_out) {
  if (!ctx) return -1;
  ctx->err.clear();  // (a message left by an earlier failed call is not this call's cause)
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->index_ready) return set_err(ctx, "mg_build_index must run first");
  if (n_out) *n_out = 0;
  if (key_len != ctx->h) return 0;  // no key of another length exists
  if (ctx->nranks > 1) return set_err(ctx, "lookup on a bucket-sharded index");
  if ((!ctx->index_o1 || !ctx->index_o3) && !long_mode(ctx) && !ctx->lookup_ready) {
    // the step's index has no o = 1 keys: file all four once into the lookup table
    MG_ENSURE(d_lkcells, lkcells_cap, ctx->cell_n * kCell);
    MG_TRY(hipMemsetAsync(ctx->d_lkcells, 0xFF, ctx->cell_n * kCell * sizeof(uint64_t), ctx->stream));
    if (ctx->n && dispatch_w<LaunchIndex>(ctx->maxw, ctx, ctx->d_lkcells, true))
      return set_err(ctx, "lookup table build failed");
    ctx->lookup_ready = true;
  }
  const int qwords = (int)((key_len + 31) / 32);
  std::vector<uint64_t> q(qwords + 1, 0);
  for (uint32_t i = 0; i < key_len; i++) {
    const char c = key[i];
    uint64_t code;
    switch (c) {
      case 'A': code = 0; break;
      case 'C': code = 1; break;
      case 'G': code = 2; break;
      case 'T': code = 3; break;
      default: return 0;  // reference keys are ACGT only
    }
    q[i >> 5] |= code << (62 - 2 * (i & 31));
  }
  uint64_t* dq = nullptr;
  unsigned long long* dout = nullptr;
  unsigned int* dn = nullptr;
  const uint32_t dcap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(cap, 1), 1u << 24);
  MG_TRY(hipMalloc(&dq, (qwords + 1) * sizeof(uint64_t)));
  MG_TRY(hipMalloc(&dout, dcap * sizeof(unsigned long long)));
  MG_TRY(hipMalloc(&dn, sizeof(unsigned int)));
  MG_TRY(hipMemcpyAsync(dq, q.data(), (qwords + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipMemsetAsync(dn, 0, sizeof(unsigned int), ctx->stream));
  if (launch_lookup(ctx, dq, qwords, dout, dcap, dn)) return set_err(ctx, "lookup failed");
  unsigned int n = 0;
  MG_TRY(hipMemcpyAsync(&n, dn, sizeof(n), hipMemcpyDeviceToHost, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  std::vector<unsigned long long> res(std::min<uint32_t>(n, dcap));
  if (!res.empty())
    MG_TRY(hipMemcpy(res.data(), dout, res.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  (void)hipFree(dq);
  (void)hipFree(dout);
  (void)hipFree(dn);
  // reference list order: insertion order = ID ascending, then o (HashTable.cpp:58-60, 98-101)
  std::sort(res.begin(), res.end(), [](unsigned long long x, unsigned long long y) {
    const uint64_t ix = x & 0x3FFFFFFFFFFFFFFFULL, iy = y & 0x3FFFFFFFFFFFFFFFULL;
    return ix != iy ? ix < iy : (x >> 62) < (y >> 62);
  });
  for (uint64_t i = 0; i < res.size() && i < cap; i++) out[i] = res[i];
  if (n_out) *n_out = n;
  return 0;
}

static int digest_begin(mg_ctx* ctx) {
  if (!ctx->d_digest) MG_TRY(hipMalloc(&ctx->d_digest, 4 * sizeof(unsigned long long)));
  MG_TRY(hipMemsetAsync(ctx->d_digest, 0, 4 * sizeof(unsigned long long), ctx->stream));
  return 0;
}

static int digest_end(mg_ctx* ctx, uint64_t* out) {
  MG_TRY(hipGetLastError());
  unsigned long long h[4];
  MG_TRY(hipMemcpyAsync(h, ctx->d_digest, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  for (int i = 0; i < 4; ++i) out[i] = h[i];
  return 0;
}

int mg_rows_digest(mg_ctx* ctx, const void* rows, uint64_t n_rows, uint64_t* out) {
  if (!ctx || !out) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (digest_begin(ctx)) return -1;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, ((uint64_t)ctx->n_cu) * 8));
  if (rows) {
    if (n_rows)
      hipLaunchKernelGGL(k_rows_digest, dim3(grid), dim3(kBlock), 0, ctx->stream,
                         reinterpret_cast<const uint32_t*>(rows), (uint64_t)0, nullptr, (uint64_t)0, n_rows,
                         ctx->d_digest);
  } else if (ctx->nreg && ctx->n_rows) {
    hipLaunchKernelGGL(k_rows_digest, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->d_rows,
                       ctx->rows_cap / ctx->nreg, ctx->d_seg, ctx->nreg, (uint64_t)0, ctx->d_digest);
  }
  return digest_end(ctx, out);
}

int mg_slots_digest(mg_ctx* ctx, const void* rows, uint64_t slot, uint32_t rounds, const uint64_t* counts,
                    uint64_t* out) {
  if (!ctx || !out) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (digest_begin(ctx)) return -1;
  const uint64_t nreg = (uint64_t)rounds * ctx->nranks;
  if (nreg && slot) {
    if (!rows || !counts) return set_err(ctx, "mg_slots_digest: null buffer");
    if (slot_regions(ctx, &ctx->d_slot_cnt, &ctx->slot_cnt_cap, reinterpret_cast<const unsigned long long*>(counts),
                     slot, slot, nreg))
      return -1;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, ((uint64_t)ctx->n_cu) * 8));
    hipLaunchKernelGGL(k_rows_digest, dim3(grid), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<const uint32_t*>(rows), slot, ctx->d_slot_cnt, nreg, (uint64_t)0,
                       ctx->d_digest);
    MG_TRY(hipGetLastError());
  }
  return digest_end(ctx, out);
}

int mg_super_digest(mg_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->contained_done) return set_err(ctx, "mg_mark_contained must run first");
  if (digest_begin(ctx)) return -1;
  if (ctx->super_any && ctx->n) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>(4096, (ctx->n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_super_digest, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->d_super, ctx->n, ctx->d_digest, ctx->d_id);
  }
  return digest_end(ctx, out);
}

int mg_get_timings(const mg_ctx* ctx, mg_timings* t) {
  if (!ctx || !t) return -1;
  if (settle_index_times(const_cast<mg_ctx*>(ctx))) return -1;
  *t = ctx->t;
  return 0;
}

int mg_get_counters(const mg_ctx* ctx, mg_counters* c) {
  if (!ctx || !c) return -1;
  *c = ctx->counters;
  c->scan_runs = ctx->scan_runs;
  return 0;
}

}  // extern "C"
