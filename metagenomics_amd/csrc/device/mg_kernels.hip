// mg_kernels.hip — CDNA4 (gfx950) kernels for the read-overlap hot path.
//
// Reference path replaced (paths relative to /root/reference/MetaGenomics):
//   Read::setRead / reverseComplement          Read.cpp:75-82,115-127   -> k_pack_ascii, rc_word
//   HashTable::insertDataset/hashRead/insert   HashTable.cpp:50-195     -> k_index_keys (count/fill) + scan
//   HashTable::getListOfReads                  HashTable.cpp:202-221    -> run lookup inside k_discover, k_lookup_key
//   OverlapGraph::markContainedReads           OverlapGraph.cpp:225-340 -> k_discover<CONTAIN=true> + k_super_finalize
//   OverlapGraph::insertAllEdgesOfRead         OverlapGraph.cpp:529-565 -> k_discover<CONTAIN=false>
//   OverlapGraph::checkOverlap / insertEdge    OverlapGraph.cpp:354-419 -> verify + emit inside k_discover
//
// Design:
//  * reads: AoS 2-bit words (A0 C1 G2 T3, MSB-first), MAXW words per read; the
//    reverse strand is never stored, it is derived in registers (rc_word).
//  * index: every key (the h = l-1 prefix/suffix of both strands, 4 per read)
//    is filed under its m-mer minimizer (m = seed k).  A read's window j
//    matches key K exactly only if both share the minimizer at the same
//    relative offset q, so each exact-key hit of the reference is found once,
//    from the run of windows that share that minimizer; every candidate is
//    then verified over the full overlap, so results are exact.
//  * discovery: one lane per source read; the read's words live in LDS; each
//    loop iteration every lane finds its next candidate (run -> bucket ->
//    entry filter) and verifies it against the partner's words; rows are
//    compacted per wavefront with ballot/popcount into an LDS buffer and
//    flushed with one atomic per >=128 rows.
//  * only half of the symmetric discoveries are verified: o = 1 hits are the
//    twins of the partner's o = 0 hits, o = 2/3 hits are kept only when
//    source <= partner; every verified discovery emits its row and its twin
//    (DESIGN.md §4 proves this reproduces the reference multiset).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "mg_overlap.h"

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kFlush = 128;                 // rows per global reservation (minimum)
constexpr int kBuf = kFlush + 4 * kWave;    // per-wave LDS row buffer capacity
constexpr int kSegs = 64;                   // output segments (one atomic cursor each)
constexpr int kScanPerThread = 16;
constexpr int kScanTile = kBlock * kScanPerThread;
constexpr uint32_t kFpBits = 20;

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

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = __lane_id();
  return lane ? (~0ULL >> (64 - lane)) : 0ULL;
}

// ------------------------------------------------------------ 2-bit pack ---
// One thread per (read, word): ASCII ACGT -> 2-bit codes, MSB-first.
// code = ((c >> 1) ^ (c >> 2)) & 3 maps A,C,G,T (0x41,0x43,0x47,0x54) to 0..3.
__global__ __launch_bounds__(kBlock) void k_pack_ascii(const char* __restrict__ ascii,
                                                      const uint64_t* __restrict__ off, uint64_t n,
                                                      uint32_t maxw, uint64_t* __restrict__ words,
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
  words[r * maxw + k] = wd;
}

// ------------------------------------------------------------ index build ---
struct IndexParams {
  const uint64_t* words;
  const uint16_t* len;
  uint64_t n;
  int h, m, w;
  uint32_t nb_log2;
  uint32_t rank, nranks;
  uint32_t* cnt;        // [NB] per-bucket counts (count pass) / remaining cursor (fill pass)
  const uint32_t* dir;  // [NB+1] exclusive scan of counts
  uint64_t* ent;        // entries: lo32 = read index, hi32 = fp20 | q10 | o2
};

__device__ __forceinline__ bool owned(uint64_t bkt, uint32_t nb_log2, uint32_t rank, uint32_t nranks) {
  return nranks <= 1 || (uint32_t)((bkt * nranks) >> nb_log2) == rank;
}

// Minimizer (leftmost minimum of mix64 over the key's w m-mers) of each of the
// read's 4 keys (hashRead, HashTable.cpp:88-104): o=0 F[0,h), o=1 F[n-h,n),
// o=2 R[0,h), o=3 R[n-h,n).  R m-mer at t = rc(F[n-t-m, n-t)).
// FILL=false: count entries per bucket.  FILL=true: place entries.
template <int MAXW, bool FILL>
__global__ __launch_bounds__(kBlock) void k_index_keys(IndexParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= p.n) return;
  uint64_t* f = smem + threadIdx.x;  // word k at f[k * kBlock]
  const uint64_t* g = p.words + r * MAXW;
#pragma unroll
  for (int k = 0; k < MAXW; ++k) f[k * kBlock] = g[k];
  f[MAXW * kBlock] = 0;
  const int n = p.len[r];
  const int h = p.h, m = p.m, w = p.w;
  const uint64_t mmask = (m == 32) ? ~0ULL : ((1ULL << (2 * m)) - 1);
  const uint64_t nbmask = (1ULL << p.nb_log2) - 1;
#pragma unroll 1
  for (int o = 0; o < 4; ++o) {
    const int kb = (o == 0 || o == 2) ? 0 : n - h;
    uint64_t best = 0;
    int bq = 0;
    for (int i = 0; i < w; ++i) {
      const int t = kb + i;
      uint64_t mm;
      if (o < 2)
        mm = ext_fwd<kBlock>(f, t) >> (64 - 2 * m);
      else
        mm = rc_word(ext_fwd<kBlock>(f, n - t - m)) & mmask;
      const uint64_t v = mix64(mm);
      if (i == 0 || v < best) {
        best = v;
        bq = i;
      }
    }
    const uint64_t bkt = best & nbmask;
    if (!owned(bkt, p.nb_log2, p.rank, p.nranks)) continue;
    if (!FILL) {
      atomicAdd(&p.cnt[bkt], 1u);
    } else {
      const uint32_t fp = (uint32_t)(best >> p.nb_log2) & ((1u << kFpBits) - 1);
      const uint32_t pos = p.dir[bkt] + atomicSub(&p.cnt[bkt], 1u) - 1u;
      const uint32_t hi = (fp << 12) | ((uint32_t)bq << 2) | (uint32_t)o;
      p.ent[pos] = ((uint64_t)hi << 32) | (uint32_t)r;
    }
  }
}

// ------------------------------------------------------------------ scan ---
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total, uint32_t* sh) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  uint32_t wofs = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kWavesPerBlock; ++i) {
    const uint32_t s = sh[i];
    if (i < wv) wofs += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return wofs + x - v;
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t* __restrict__ in, uint64_t n,
                                                       uint32_t* __restrict__ bsum) {
  __shared__ uint32_t sh[kWavesPerBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    const uint64_t idx = base + (uint64_t)i * kBlock + threadIdx.x;
    if (idx < n) s += in[idx];
  }
  uint32_t tot;
  block_excl_scan(s, &tot, sh);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// Single block: exclusive scan of the block sums in place.
__global__ __launch_bounds__(kBlock) void k_scan_bsums(uint32_t* bsum, uint32_t nbs) {
  __shared__ uint32_t sh[kWavesPerBlock];
  uint32_t carry = 0;
  for (uint32_t base = 0; base < nbs; base += kBlock) {
    const uint32_t idx = base + threadIdx.x;
    const uint32_t v = idx < nbs ? bsum[idx] : 0;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, &tot, sh);
    if (idx < nbs) bsum[idx] = carry + ex;
    carry += tot;
  }
}

// Exclusive scan of in[0..n) into out[0..n], out[n] = total.
__global__ __launch_bounds__(kBlock) void k_scan_apply(const uint32_t* __restrict__ in, uint64_t n,
                                                      const uint32_t* __restrict__ bsum,
                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[kWavesPerBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPerThread;
  uint32_t v[kScanPerThread];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    v[i] = (base + i < n) ? in[base + i] : 0;
    s += v[i];
  }
  uint32_t tot;
  uint32_t ex = block_excl_scan(s, &tot, sh) + bsum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    if (base + i < n) out[base + i] = ex;
    if (base + i == n - 1) out[n] = ex + v[i];
    ex += v[i];
  }
}

// ------------------------------------------------------------- discovery ---
struct DiscParams {
  const uint64_t* words;
  const uint16_t* len;
  uint64_t n;
  int h, m, w;
  uint32_t nb_log2;
  uint32_t rank, nranks;
  const uint32_t* dir;
  const uint64_t* ent;
  const uint32_t* super;          // superReadID per read index (nullptr: none contained)
  unsigned long long* superkey;   // CONTAIN: max over containers of (len << 32 | ~index)
  uint64_t a_lo, a_hi;            // source reads handled by this launch
  uint32_t* rows;                 // 3 dwords per row (mg_edge)
  unsigned long long* seg_cnt;    // [kSegs] rows reserved per segment
  uint64_t seg_cap;               // rows per segment
  int uniform_len;                // all reads have the same length
  unsigned long long* stats;      // optional [kSegs*4]: runs probed, entries scanned, partners fetched, rows
};

template <int MAXW>
__device__ __forceinline__ size_t disc_lds_bytes_words() {
  return (size_t)kWavesPerBlock * (MAXW + 1) * kWave * sizeof(uint64_t);
}

// Wave-cooperative flush of the LDS row buffer (all 64 lanes, converged).
__device__ __forceinline__ void flush_rows(const DiscParams& p, uint32_t* obuf, uint32_t nrows,
                                           uint32_t seg, int lane) {
  unsigned long long off = 0;
  if (lane == 0) off = atomicAdd(&p.seg_cnt[seg], (unsigned long long)nrows);
  off = __shfl(off, 0);
  if (off + nrows <= p.seg_cap) {
    uint32_t* dst = p.rows + ((uint64_t)seg * p.seg_cap + off) * 3;
    for (uint32_t i = lane; i < nrows * 3; i += kWave) dst[i] = obuf[i];
  }
  __builtin_amdgcn_wave_barrier();
}

// One lane per source read (insertAllEdgesOfRead, OverlapGraph.cpp:529-565,
// or markContainedReads' inner loop, :239-271, when CONTAIN).
template <int MAXW, bool CONTAIN>
__global__ __launch_bounds__(kBlock) void k_discover(DiscParams p) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t* f1 = smem + (size_t)wv * (MAXW + 1) * kWave + lane;  // word k at f1[k * kWave]
  uint32_t* obuf = reinterpret_cast<uint32_t*>(smem + (size_t)kWavesPerBlock * (MAXW + 1) * kWave) +
                   (size_t)wv * kBuf * 3;
  const uint32_t seg = (blockIdx.x * kWavesPerBlock + wv) & (kSegs - 1);

  const uint64_t a = p.a_lo + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  bool active = a < p.a_hi;
  const int n1 = active ? (int)p.len[a] : 0;
  if (!CONTAIN && active && p.super && p.super[a]) active = false;  // :548 read1 contained
  if (active) {
    const uint64_t* g = p.words + a * MAXW;
#pragma unroll
    for (int k = 0; k < MAXW; ++k) f1[k * kWave] = g[k];
    f1[MAXW * kWave] = 0;
  }
  const int h = p.h, m = p.m, w = p.w;
  const int J = n1 - h - 1;  // windows j = 1 .. n1-h-1 (:534)
  if (J < 1) active = false;
  const uint64_t nbmask = (1ULL << p.nb_log2) - 1;
  const int msh = 64 - 2 * m;

  // sliding-window minimizer state: (cur_p, cur_v) = leftmost argmin of window jn
  int jn = 1, cur_p = 0;
  uint64_t cur_v = 0;
  auto H = [&](int t) -> uint64_t { return mix64(ext_fwd<kWave>(f1, t) >> msh); };
  auto rescan = [&](int j0) {
    for (int t = j0; t < j0 + w; ++t) {
      const uint64_t v = H(t);
      if (t == j0 || v < cur_v) {
        cur_v = v;
        cur_p = t;
      }
    }
  };
  if (active) rescan(1);

  // current run: windows [jlo, jhi] share minimizer position run_p
  int run_p = 0, jlo = 0, jhi = -1;
  uint32_t run_fp = 0, e_idx = 0, e_end = 0;
  uint32_t cnt = 0;  // rows in this wave's LDS buffer (wave-uniform)
  uint32_t st_runs = 0, st_ent = 0, st_ver = 0, st_rows = 0;  // diagnostics (p.stats)

  while (true) {
    // ---- find this lane's next candidate (bucket entry passing the cheap filters)
    bool have = false;
    uint32_t bid = 0;
    int o = 0, j = 0;
    while (active) {
      if (e_idx < e_end) {
        const uint64_t e = p.ent[e_idx++];
        ++st_ent;
#ifdef MG_DEBUG_PRINT
        if (p.n <= 4) printf("scan C=%d a=%d idx=%u e=%llx run_p=%d jlo=%d jhi=%d fp=%x\n", (int)CONTAIN, (int)a, e_idx - 1, (unsigned long long)e, run_p, jlo, jhi, run_fp);
#endif
        const uint32_t hi = (uint32_t)(e >> 32);
        if ((hi >> 12) != run_fp) continue;
        const int q = (int)((hi >> 2) & 1023u);
        const int jj = run_p - q;
        if (jj < jlo || jj > jhi) continue;
        const int oo = (int)(hi & 3u);
        const uint32_t bb = (uint32_t)e;
        // halving: o = 1 hits are the twins of the partner's o = 0
        // hits; o = 2/3 hits are kept only for partner >= source
        const bool keep = CONTAIN || (oo == 0) || (oo >= 2 && (uint64_t)bb >= a);
        if (!keep) continue;
        have = true;
        bid = bb;
        o = oo;
        j = jj;
        break;
      }
      if (jn > J) {
        active = false;
        break;
      }
      // next run of windows sharing one minimizer
      run_p = cur_p;
      const uint64_t rv = cur_v;
      jlo = jn;
      int jj = jn + 1;
      for (; jj <= J; ++jj) {
        if (cur_p < jj) {
          rescan(jj);
        } else {
          const int t = jj + w - 1;
          const uint64_t v = H(t);
          if (v < cur_v) {
            cur_v = v;
            cur_p = t;
          }
        }
        if (cur_p != run_p) break;
      }
      jhi = jj - 1;
      jn = jj;
      const uint64_t bkt = rv & nbmask;
      if (owned(bkt, p.nb_log2, p.rank, p.nranks)) {
        run_fp = (uint32_t)(rv >> p.nb_log2) & ((1u << kFpBits) - 1);
        e_idx = p.dir[bkt];
        e_end = p.dir[bkt + 1];
        ++st_runs;
      } else {
        e_idx = e_end = 0;
      }
    }

    // ---- verify the candidate over the whole overlap (checkOverlap :354-383,
    //      checkOverlapForContainedRead :302-340), partner words from HBM
    int nrec = 0;
    uint32_t r0 = 0, r1 = 0, r2 = 0, t0 = 0, t1 = 0, t2 = 0;
    if (have) {
      const int n2 = p.uniform_len ? n1 : (int)p.len[bid];
      bool cond;
      int x0, y0, L;
      bool rcA;
      if (!CONTAIN) {
        if (o == 0) {        // F1[j, n1) == F2[0, L)
          L = n1 - j; cond = L < n2; x0 = j; y0 = 0; rcA = false;
        } else if (o == 2) { // F1[j, n1) == R2[0, L)  <=>  R1[0, L) == F2[n2-L, n2)
          L = n1 - j; cond = L < n2; x0 = 0; y0 = n2 - L; rcA = true;
        } else {             // F1[0, L) == R2[n2-L, n2)  <=>  R1[n1-L, n1) == F2[0, L)
          L = j + h; cond = j <= n2 - h; x0 = n1 - L; y0 = 0; rcA = true;
        }
        if (cond && p.super && p.super[bid]) cond = false;  // :548 read2 contained
      } else {
        int s;
        cond = n1 > n2;
        if (o == 0 || o == 2) {
          cond = cond && (j <= n1 - n2);
          s = j;
        } else {
          cond = cond && (j >= n2 - h);
          s = j - (n2 - h);
        }
        L = n2; y0 = 0;
        rcA = o >= 2;
        x0 = rcA ? n1 - s - n2 : s;
      }
      if (cond) {
        ++st_ver;
        const uint64_t* bg = p.words + (uint64_t)bid * MAXW + (y0 >> 5);
        const int ys = (y0 & 31) << 1;
        uint64_t y[MAXW + 1];
#pragma unroll
        for (int k = 0; k <= MAXW; ++k) y[k] = bg[k];
        uint64_t diff = 0;
#pragma unroll
        for (int c = 0; c < MAXW; ++c) {
          if (c * 32 < L) {
            const uint64_t av = rcA ? rc_word(ext_fwd<kWave>(f1, n1 - x0 - 32 * c - 32))
                                    : ext_fwd<kWave>(f1, x0 + 32 * c);
            const uint64_t bv = funnel(y[c], y[c + 1], ys);
            const int rem = L - 32 * c;
            const uint64_t mask = rem >= 32 ? ~0ULL : ~(~0ULL >> (2 * rem));
            diff |= (av ^ bv) & mask;
          }
        }
#ifdef MG_DEBUG_PRINT
        if (p.n <= 4) printf("cand C=%d a=%d b=%u o=%d j=%d L=%d x0=%d y0=%d diff=%llx\n", (int)CONTAIN, (int)a, bid, o, j, L, x0, y0, (unsigned long long)diff);
#endif
        if (diff == 0) {
          if (CONTAIN) {
            atomicMax(&p.superkey[bid], ((unsigned long long)n1 << 32) | (0xFFFFFFFFu - (uint32_t)a));
          } else {
            // orientation/offset switch (:550-557) and the twin (:409-412, :841-855)
            const uint32_t orient = (o == 0) ? 3u : (o == 2 ? 2u : 1u);
            const uint32_t off = (o == 3) ? (uint32_t)(n1 - h - j) : (uint32_t)j;
            const uint32_t torient = (orient == 3u) ? 0u : orient;
            const uint32_t toff = (uint16_t)(n2 + off - n1);
            r0 = (uint32_t)a + 1; r1 = bid + 1; r2 = (orient << 16) | off;
            t0 = bid + 1; t1 = (uint32_t)a + 1; t2 = (torient << 16) | toff;
            nrec = (bid == (uint32_t)a && o == 0) ? 4 : 2;  // self o=0 hit: also stands for its o=1 twin
            st_rows += nrec;
          }
        }
      }
    }

#ifdef MG_DEBUG_PRINT
    if (p.n <= 4 && have) printf("have a=%d b=%u o=%d j=%d nrec=%d\n", (int)a, bid, o, j, nrec);
#endif
    // ---- wavefront compaction into the LDS row buffer, flush >= kFlush rows
    if (!CONTAIN) {
      const uint64_t b2 = __ballot(nrec >= 2), b4 = __ballot(nrec == 4);
      const uint32_t total = 2u * (uint32_t)(__popcll(b2) + __popcll(b4));
      if (total) {
        const uint64_t lt = lanemask_lt();
        const uint32_t pre = 2u * (uint32_t)(__popcll(b2 & lt) + __popcll(b4 & lt));
        uint32_t* d = obuf + (cnt + pre) * 3;
        for (int rr = 0; rr < nrec; rr += 2) {
          d[0] = r0; d[1] = r1; d[2] = r2;
          d[3] = t0; d[4] = t1; d[5] = t2;
          d += 6;
        }
        cnt += total;
        __builtin_amdgcn_wave_barrier();
        if (cnt >= (uint32_t)kFlush) {
          flush_rows(p, obuf, cnt, seg, lane);
          cnt = 0;
        }
      }
    }
    if (__ballot(active) == 0) break;
  }
  if (!CONTAIN && cnt) flush_rows(p, obuf, cnt, seg, lane);
  if (p.stats) {
    uint32_t v[4] = {st_runs, st_ent, st_ver, st_rows};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t x = v[i];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
      if (lane == 0) atomicAdd(&p.stats[seg * 4 + i], (unsigned long long)x);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_super_finalize(const unsigned long long* __restrict__ key,
                                                          uint64_t n, uint32_t* __restrict__ super,
                                                          unsigned int* __restrict__ any) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const unsigned long long k = key[i];
  const uint32_t s = k ? (0xFFFFFFFFu - (uint32_t)k) + 1u : 0u;  // container index -> ID
  super[i] = s;
  if (s) atomicOr(any, 1u);
}

// getListOfReads(key) (HashTable.cpp:202-221): scan the minimizer bucket of the
// query key and keep entries whose key string equals it exactly.
template <int MAXW>
__global__ __launch_bounds__(kBlock) void k_lookup_key(IndexParams p, const uint64_t* __restrict__ qkey,
                                                      int qwords, unsigned long long* __restrict__ out,
                                                      uint32_t cap, unsigned int* __restrict__ nout) {
  __shared__ uint64_t q[40];  // h <= 1055 -> at most 33 words + over-read
  __shared__ uint64_t qv;
  __shared__ int qq;
  const int h = p.h, m = p.m, w = p.w;
  if (threadIdx.x < 40) q[threadIdx.x] = threadIdx.x < qwords ? qkey[threadIdx.x] : 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t best = 0;
    int bq = 0;
    for (int i = 0; i < w; ++i) {
      const uint64_t v = mix64(ext_fwd<1>(q, i) >> (64 - 2 * m));
      if (i == 0 || v < best) {
        best = v;
        bq = i;
      }
    }
    qv = best;
    qq = bq;
  }
  __syncthreads();
  const uint64_t bkt = qv & ((1ULL << p.nb_log2) - 1);
  const uint32_t fp = (uint32_t)(qv >> p.nb_log2) & ((1u << kFpBits) - 1);
  const uint32_t s = p.dir[bkt], e = p.dir[bkt + 1];
  for (uint32_t i = s + threadIdx.x; i < e; i += kBlock) {
    const uint64_t en = p.ent[i];
    const uint32_t hi = (uint32_t)(en >> 32);
    if ((hi >> 12) != fp || (int)((hi >> 2) & 1023u) != qq) continue;
    const int o = (int)(hi & 3u);
    const uint32_t r = (uint32_t)en;
    const uint64_t* g = p.words + (uint64_t)r * MAXW;
    const int n = p.len[r];
    // key string of (r, o) vs the query, 32 bases at a time
    uint64_t diff = 0;
    for (int c = 0; c * 32 < h; ++c) {
      uint64_t kv;
      if (o < 2) {
        const int pos = (o == 0 ? 0 : n - h) + 32 * c;
        kv = funnel(g[pos >> 5], g[(pos >> 5) + 1], (pos & 31) << 1);
      } else {
        // R[b, b+32) = rc(F[n-b-32, n-b)), b = (o == 2 ? 0 : n-h) + 32c
        const int b = (o == 2 ? 0 : n - h) + 32 * c;
        const int pos = n - b - 32;
        uint64_t fw;
        if (pos < 0)
          fw = g[0] >> (-pos * 2);
        else
          fw = funnel(g[pos >> 5], g[(pos >> 5) + 1], (pos & 31) << 1);
        kv = rc_word(fw);
      }
      const int rem = h - 32 * c;
      const uint64_t mask = rem >= 32 ? ~0ULL : ~(~0ULL >> (2 * rem));
      diff |= (kv ^ ext_fwd<1>(q, 32 * c)) & mask;
    }
    if (diff) continue;
    const unsigned int slot = atomicAdd(nout, 1u);
    if (slot < cap) out[slot] = ((unsigned long long)(r + 1)) | ((unsigned long long)o << 62);
  }
}

}  // namespace

// ===================================================================== ABI ===
struct mg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // reads
  uint64_t n = 0;
  uint32_t maxw = 0;
  uint32_t minlen = 0, maxlen = 0;
  uint64_t* d_words = nullptr;
  uint16_t* d_len = nullptr;
  size_t words_cap = 0, len_cap = 0;
  // index
  uint32_t l = 0, h = 0, m = 0, w = 0;
  uint32_t nb_log2 = 0, nb_log2_opt = 0;
  bool index_ready = false;
  uint32_t* d_cnt = nullptr;
  uint32_t* d_dir = nullptr;
  uint32_t* d_bsum = nullptr;
  uint64_t* d_ent = nullptr;
  size_t cnt_cap = 0, dir_cap = 0, bsum_cap = 0, ent_cap = 0;
  // containment
  unsigned long long* d_superkey = nullptr;
  uint32_t* d_super = nullptr;
  unsigned int* d_any = nullptr;
  size_t super_cap = 0;
  bool contained_done = false, super_any = false;
  // rows
  uint32_t* d_rows = nullptr;
  uint64_t rows_cap = 0, rows_cap_opt = 0;
  unsigned long long* d_seg = nullptr;
  uint64_t n_rows = 0;
  std::vector<unsigned long long> seg_host;
  bool stats = false;
  unsigned long long* d_stats = nullptr;
  mg_counters counters{};
  // shard
  uint32_t rank = 0, nranks = 1;
  uint64_t read_lo = 0, read_hi = 0;
  // timing
  hipEvent_t ev[8] = {};
  mg_timings t{};
};

namespace {

#define MG_TRY(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ctx->err = std::string(#expr) + " failed: " + hipGetErrorString(e_);            \
      return -1;                                                                      \
    }                                                                                 \
  } while (0)

int set_err(mg_ctx* ctx, const std::string& s) {
  ctx->err = s;
  return -1;
}

template <typename T>
hipError_t ensure(T** p, size_t* cap, size_t count) {
  if (*cap >= count && *p) return hipSuccess;
  if (*p) {
    hipError_t e = hipFree(*p);
    if (e != hipSuccess) return e;
    *p = nullptr;
  }
  const size_t c = std::max<size_t>(count, 1);
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), c * sizeof(T));
  if (e == hipSuccess) *cap = c;
  return e;
}

const uint32_t kSupportedW[] = {1, 2, 3, 4, 5, 6, 8, 12, 16, 32};

uint32_t supported_maxw(uint32_t need) {
  for (uint32_t w : kSupportedW)
    if (w >= need) return w;
  return 0;
}

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
  p.cnt = ctx->d_cnt;
  p.dir = ctx->d_dir;
  p.ent = ctx->d_ent;
  return p;
}

template <int W>
struct LaunchIndex {
  static int run(mg_ctx* ctx, bool fill) {
    IndexParams p = index_params(ctx);
    const uint32_t grid = (uint32_t)((ctx->n + kBlock - 1) / kBlock);
    const size_t lds = (size_t)(W + 1) * kBlock * sizeof(uint64_t);
    if (grid == 0) return 0;
    if (fill) {
      allow_lds(k_index_keys<W, true>, lds);
      hipLaunchKernelGGL((k_index_keys<W, true>), dim3(grid), dim3(kBlock), lds, ctx->stream, p);
    } else {
      allow_lds(k_index_keys<W, false>, lds);
      hipLaunchKernelGGL((k_index_keys<W, false>), dim3(grid), dim3(kBlock), lds, ctx->stream, p);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

template <int W>
struct LaunchDiscover {
  static int run(mg_ctx* ctx, bool contain) {
    DiscParams p{};
    p.words = ctx->d_words;
    p.len = ctx->d_len;
    p.n = ctx->n;
    p.h = (int)ctx->h;
    p.m = (int)ctx->m;
    p.w = (int)ctx->w;
    p.nb_log2 = ctx->nb_log2;
    p.rank = ctx->rank;
    p.nranks = ctx->nranks;
    p.dir = ctx->d_dir;
    p.ent = ctx->d_ent;
    p.super = (ctx->contained_done && ctx->super_any) ? ctx->d_super : nullptr;
    p.superkey = ctx->d_superkey;
    p.rows = ctx->d_rows;
    p.seg_cnt = ctx->d_seg;
    p.seg_cap = ctx->rows_cap / kSegs;
    p.uniform_len = ctx->minlen == ctx->maxlen;
    p.stats = contain ? nullptr : (ctx->stats ? ctx->d_stats : nullptr);
    // containment scans every read as read1 (:235); discovery only this shard's sources
    p.a_lo = contain ? 0 : ctx->read_lo;
    p.a_hi = contain ? ctx->n : (ctx->read_hi ? std::min<uint64_t>(ctx->read_hi, ctx->n) : ctx->n);
    if (p.a_hi <= p.a_lo) return 0;
    const uint32_t grid = (uint32_t)((p.a_hi - p.a_lo + kBlock - 1) / kBlock);
    const size_t lds_words = (size_t)kWavesPerBlock * (W + 1) * kWave * sizeof(uint64_t);
    if (contain) {
      allow_lds(k_discover<W, true>, lds_words);
      hipLaunchKernelGGL((k_discover<W, true>), dim3(grid), dim3(kBlock), lds_words, ctx->stream, p);
    } else {
      const size_t lds = lds_words + (size_t)kWavesPerBlock * kBuf * 3 * sizeof(uint32_t);
      allow_lds(k_discover<W, false>, lds);
      hipLaunchKernelGGL((k_discover<W, false>), dim3(grid), dim3(kBlock), lds, ctx->stream, p);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

template <int W>
struct LaunchLookup {
  static int run(mg_ctx* ctx, const uint64_t* dq, int qwords, unsigned long long* dout, uint32_t cap,
                 unsigned int* dn) {
    IndexParams p = index_params(ctx);
    hipLaunchKernelGGL((k_lookup_key<W>), dim3(1), dim3(kBlock), 0, ctx->stream, p, dq, qwords, dout, cap, dn);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
};

int scan_dir(mg_ctx* ctx, uint64_t nb) {
  const uint64_t nblocks = (nb + kScanTile - 1) / kScanTile;
  MG_TRY(ensure(&ctx->d_bsum, &ctx->bsum_cap, nblocks));
  hipLaunchKernelGGL(k_scan_reduce, dim3((uint32_t)nblocks), dim3(kBlock), 0, ctx->stream, ctx->d_cnt, nb,
                     ctx->d_bsum);
  hipLaunchKernelGGL(k_scan_bsums, dim3(1), dim3(kBlock), 0, ctx->stream, ctx->d_bsum, (uint32_t)nblocks);
  hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nblocks), dim3(kBlock), 0, ctx->stream, ctx->d_cnt, nb,
                     ctx->d_bsum, ctx->d_dir);
  MG_TRY(hipGetLastError());
  return 0;
}

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
  return ms;
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
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
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
  void* bufs[] = {ctx->d_words, ctx->d_len, ctx->d_cnt, ctx->d_dir, ctx->d_bsum, ctx->d_ent,
                  ctx->d_superkey, ctx->d_super, ctx->d_any, ctx->d_rows, ctx->d_seg, ctx->d_stats};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* mg_last_error(const mg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* mg_stream(mg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

uint64_t mg_num_reads(const mg_ctx* ctx) { return ctx ? ctx->n : 0; }

static void reset_derived(mg_ctx* ctx) {
  ctx->index_ready = false;
  ctx->contained_done = false;
  ctx->super_any = false;
  ctx->n_rows = 0;
}

static int finish_upload(mg_ctx* ctx, const uint16_t* lens_host) {
  // min/max length (Dataset::shortestReadLength / longestReadLength, Dataset.h:35-36)
  uint32_t mn = 0xFFFFFFFFu, mx = 0;
  for (uint64_t i = 0; i < ctx->n; i++) {
    mn = std::min<uint32_t>(mn, lens_host[i]);
    mx = std::max<uint32_t>(mx, lens_host[i]);
  }
  ctx->minlen = ctx->n ? mn : 0;
  ctx->maxlen = mx;
  reset_derived(ctx);
  return 0;
}

int mg_upload_reads_packed(mg_ctx* ctx, const uint64_t* words, const uint16_t* lens, uint64_t n_reads,
                           uint32_t words_per_read) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (n_reads >= 0xFFFFFFFFull) return set_err(ctx, "too many reads (max 2^32-2)");
  uint32_t mx = 0;
  for (uint64_t i = 0; i < n_reads; i++) mx = std::max<uint32_t>(mx, lens[i]);
  if (mx > 32u * words_per_read) return set_err(ctx, "read longer than words_per_read * 32");
  const uint32_t maxw = supported_maxw(std::max<uint32_t>(1, words_per_read));
  if (!maxw) return set_err(ctx, "reads longer than 1024 bp are not supported");
  ctx->n = n_reads;
  ctx->maxw = maxw;
  const size_t nw = (size_t)(n_reads + 2) * maxw + 2;  // zero pad for partner over-reads
  MG_TRY(ensure(&ctx->d_words, &ctx->words_cap, nw));
  MG_TRY(ensure(&ctx->d_len, &ctx->len_cap, n_reads + 1));
  MG_TRY(hipMemsetAsync(ctx->d_words, 0, nw * sizeof(uint64_t), ctx->stream));
  if (maxw == words_per_read) {
    MG_TRY(hipMemcpyAsync(ctx->d_words, words, n_reads * maxw * sizeof(uint64_t), hipMemcpyHostToDevice,
                          ctx->stream));
  } else {
    MG_TRY(hipMemcpy2DAsync(ctx->d_words, maxw * sizeof(uint64_t), words, words_per_read * sizeof(uint64_t),
                            words_per_read * sizeof(uint64_t), n_reads, hipMemcpyHostToDevice, ctx->stream));
  }
  if (n_reads)
    MG_TRY(hipMemcpyAsync(ctx->d_len, lens, n_reads * sizeof(uint16_t), hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  return finish_upload(ctx, lens);
}

int mg_upload_reads_ascii(mg_ctx* ctx, const char* concat, const uint64_t* offsets, uint64_t n_reads) {
  if (!ctx) return -1;
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
  const uint32_t maxw = supported_maxw((uint32_t)std::max<uint64_t>(1, (mx + 31) / 32));
  if (!maxw) return set_err(ctx, "reads longer than 1024 bp are not supported");
  ctx->n = n_reads;
  ctx->maxw = maxw;
  const uint64_t total = n_reads ? offsets[n_reads] : 0;
  char* d_ascii = nullptr;
  uint64_t* d_off = nullptr;
  MG_TRY(hipMalloc(&d_ascii, std::max<uint64_t>(total, 1)));
  MG_TRY(hipMalloc(&d_off, (n_reads + 1) * sizeof(uint64_t)));
  const size_t nw = (size_t)(n_reads + 2) * maxw + 2;
  MG_TRY(ensure(&ctx->d_words, &ctx->words_cap, nw));
  MG_TRY(ensure(&ctx->d_len, &ctx->len_cap, n_reads + 1));
  MG_TRY(hipMemsetAsync(ctx->d_words, 0, nw * sizeof(uint64_t), ctx->stream));
  if (total) MG_TRY(hipMemcpyAsync(d_ascii, concat, total, hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipMemcpyAsync(d_off, offsets, (n_reads + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  const uint64_t threads = n_reads * maxw;
  if (threads) {
    hipLaunchKernelGGL(k_pack_ascii, dim3((uint32_t)((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, d_ascii, d_off, n_reads, maxw, ctx->d_words, ctx->d_len);
    MG_TRY(hipGetLastError());
  }
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  MG_TRY(hipStreamSynchronize(ctx->stream));
  ctx->t.pack_ms = elapsed(ctx->ev[0], ctx->ev[1]);
  (void)hipFree(d_ascii);
  (void)hipFree(d_off);
  return finish_upload(ctx, lens.data());
}

int mg_download_reads_packed(mg_ctx* ctx, uint64_t* words, uint16_t* lens, uint32_t* words_per_read) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (words_per_read) *words_per_read = ctx->maxw;
  if (words && ctx->n)
    MG_TRY(hipMemcpy(words, ctx->d_words, ctx->n * ctx->maxw * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (lens && ctx->n) MG_TRY(hipMemcpy(lens, ctx->d_len, ctx->n * sizeof(uint16_t), hipMemcpyDeviceToHost));
  return 0;
}

int mg_set_option(mg_ctx* ctx, const char* name, int64_t value) {
  if (!ctx || !name) return -1;
  if (!strcmp(name, "nb_log2")) {
    if (value != 0 && (value < 10 || value > 31)) return set_err(ctx, "nb_log2 out of range [10,31]");
    ctx->nb_log2_opt = (uint32_t)value;
    ctx->index_ready = false;
    return 0;
  }
  if (!strcmp(name, "stats")) {
    ctx->stats = value != 0;
    return 0;
  }
  if (!strcmp(name, "rows_cap")) {
    ctx->rows_cap_opt = (uint64_t)std::max<int64_t>(0, value);
    return 0;
  }
  return set_err(ctx, std::string("unknown option ") + name);
}

int mg_set_shard(mg_ctx* ctx, uint32_t rank, uint32_t nranks, uint64_t read_lo, uint64_t read_hi) {
  if (!ctx) return -1;
  if (nranks == 0 || rank >= nranks) return set_err(ctx, "bad shard rank/nranks");
  if (read_hi && read_hi < read_lo) return set_err(ctx, "bad read range");
  if (rank != ctx->rank || nranks != ctx->nranks) ctx->index_ready = false;
  ctx->rank = rank;
  ctx->nranks = nranks;
  ctx->read_lo = read_lo;
  ctx->read_hi = read_hi;
  return 0;
}

int mg_build_index(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (min_overlap < 2) return set_err(ctx, "min_overlap must be >= 2");
  const uint32_t h = min_overlap - 1;  // HashTable.cpp:54
  uint32_t m = seed_k ? seed_k : std::min<uint32_t>(31, h);
  if (m > 32 || m > h) return set_err(ctx, "seed k must satisfy 1 <= k <= min(32, l-1)");
  const uint32_t w = h - m + 1;
  if (w > 1024) return set_err(ctx, "l-1 - k + 1 must be <= 1024");
  if (ctx->minlen && ctx->minlen <= min_overlap)
    return set_err(ctx, "every read must be longer than min_overlap (Dataset.cpp:160)");
  ctx->l = min_overlap;
  ctx->h = h;
  ctx->m = m;
  ctx->w = w;
  uint32_t nbl = ctx->nb_log2_opt;
  if (!nbl) {
    // about one bucket per read: 4 keys per read, ~2-3 keys share a minimizer
    nbl = 10;
    while (nbl < 30 && (1ull << nbl) < ctx->n) nbl++;
  }
  ctx->nb_log2 = nbl;
  const uint64_t nb = 1ull << nbl;
  MG_TRY(ensure(&ctx->d_cnt, &ctx->cnt_cap, nb));
  MG_TRY(ensure(&ctx->d_dir, &ctx->dir_cap, nb + 1));
  MG_TRY(ensure(&ctx->d_ent, &ctx->ent_cap, std::max<uint64_t>(4 * ctx->n, 1)));
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  MG_TRY(hipMemsetAsync(ctx->d_cnt, 0, nb * sizeof(uint32_t), ctx->stream));
  if (dispatch_w<LaunchIndex>(ctx->maxw, ctx, false)) return set_err(ctx, "index count launch failed");
  if (scan_dir(ctx, nb)) return -1;
  if (dispatch_w<LaunchIndex>(ctx->maxw, ctx, true)) return set_err(ctx, "index fill launch failed");
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  MG_TRY(hipEventSynchronize(ctx->ev[1]));
  ctx->t.index_ms = elapsed(ctx->ev[0], ctx->ev[1]);
  ctx->index_ready = true;
  ctx->contained_done = false;
  ctx->super_any = false;
  return 0;
}

int mg_mark_contained(mg_ctx* ctx, uint32_t* super_out) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->index_ready) return set_err(ctx, "mg_build_index must run first");
  MG_TRY(ensure(&ctx->d_super, &ctx->super_cap, ctx->n + 1));
  if (!ctx->d_any) MG_TRY(hipMalloc(&ctx->d_any, sizeof(unsigned int)));
  ctx->t.contained_ms = 0.f;
  if (ctx->minlen != ctx->maxlen) {  // OverlapGraph.cpp:228-233
    size_t skcap = 0;
    if (ctx->d_superkey) {
      (void)hipFree(ctx->d_superkey);
      ctx->d_superkey = nullptr;
    }
    MG_TRY(ensure(&ctx->d_superkey, &skcap, ctx->n + 1));
    MG_TRY(hipMemsetAsync(ctx->d_superkey, 0, (ctx->n + 1) * sizeof(unsigned long long), ctx->stream));
    MG_TRY(hipMemsetAsync(ctx->d_any, 0, sizeof(unsigned int), ctx->stream));
    MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
    // sharded contexts still need the full superReadID vector: run over all
    // buckets (the containment pass is small, only for mixed lengths)
    const uint32_t r = ctx->rank, nr = ctx->nranks;
    if (nr > 1) return set_err(ctx, "containment with a bucket-sharded index is not supported yet");
    if (dispatch_w<LaunchDiscover>(ctx->maxw, ctx, true)) return set_err(ctx, "containment launch failed");
    (void)r;
    if (ctx->n)
      hipLaunchKernelGGL(k_super_finalize, dim3((uint32_t)((ctx->n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                         ctx->stream, ctx->d_superkey, ctx->n, ctx->d_super, ctx->d_any);
    MG_TRY(hipGetLastError());
    MG_TRY(hipEventRecord(ctx->ev[3], ctx->stream));
    unsigned int any = 0;
    MG_TRY(hipMemcpyAsync(&any, ctx->d_any, sizeof(any), hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
    ctx->t.contained_ms = elapsed(ctx->ev[2], ctx->ev[3]);
    ctx->super_any = any != 0;
  } else {
    MG_TRY(hipMemsetAsync(ctx->d_super, 0, (ctx->n + 1) * sizeof(uint32_t), ctx->stream));
    ctx->super_any = false;
  }
  ctx->contained_done = true;
  if (super_out) {
    super_out[0] = 0;
    if (ctx->n)
      MG_TRY(hipMemcpyAsync(super_out + 1, ctx->d_super, ctx->n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
  }
  return 0;
}

int mg_find_overlaps(mg_ctx* ctx, uint64_t* n_rows) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->index_ready) return set_err(ctx, "mg_build_index must run first");
  if (!ctx->contained_done && mg_mark_contained(ctx, nullptr)) return -1;
  if (!ctx->d_seg) MG_TRY(hipMalloc(&ctx->d_seg, kSegs * sizeof(unsigned long long)));
  const uint64_t nsrc = (ctx->read_hi ? std::min(ctx->read_hi, ctx->n) : ctx->n) -
                        std::min(ctx->read_lo, ctx->n);
  uint64_t want = ctx->rows_cap_opt ? ctx->rows_cap_opt : std::max<uint64_t>(1u << 20, 48 * nsrc);
  ctx->seg_host.assign(kSegs, 0);
  for (int attempt = 0; attempt < 3; ++attempt) {
    want = (want + kSegs - 1) / kSegs * kSegs;
    if (want > ctx->rows_cap) {
      if (ctx->d_rows) (void)hipFree(ctx->d_rows);
      ctx->d_rows = nullptr;
      MG_TRY(hipMalloc(&ctx->d_rows, want * 3 * sizeof(uint32_t)));
      ctx->rows_cap = want;
    }
    MG_TRY(hipMemsetAsync(ctx->d_seg, 0, kSegs * sizeof(unsigned long long), ctx->stream));
    if (ctx->stats) {
      if (!ctx->d_stats) MG_TRY(hipMalloc(&ctx->d_stats, kSegs * 4 * sizeof(unsigned long long)));
      MG_TRY(hipMemsetAsync(ctx->d_stats, 0, kSegs * 4 * sizeof(unsigned long long), ctx->stream));
    }
    MG_TRY(hipEventRecord(ctx->ev[4], ctx->stream));
    if (dispatch_w<LaunchDiscover>(ctx->maxw, ctx, false)) return set_err(ctx, "discovery launch failed");
    MG_TRY(hipEventRecord(ctx->ev[5], ctx->stream));
    MG_TRY(hipMemcpyAsync(ctx->seg_host.data(), ctx->d_seg, kSegs * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, ctx->stream));
    MG_TRY(hipStreamSynchronize(ctx->stream));
    const uint64_t seg_cap = ctx->rows_cap / kSegs;
    uint64_t total = 0, mx = 0;
    for (auto c : ctx->seg_host) {
      total += c;
      mx = std::max<uint64_t>(mx, c);
    }
    ctx->t.overlap_ms = elapsed(ctx->ev[4], ctx->ev[5]);
    ctx->n_rows = total;
    if (ctx->stats) {
      std::vector<unsigned long long> st(kSegs * 4);
      MG_TRY(hipMemcpy(st.data(), ctx->d_stats, st.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      uint64_t acc[4] = {0, 0, 0, 0};
      for (int s = 0; s < kSegs; ++s)
        for (int i = 0; i < 4; ++i) acc[i] += st[s * 4 + i];
      ctx->counters.runs = acc[0];
      ctx->counters.entries = acc[1];
      ctx->counters.verified = acc[2];
      ctx->counters.rows = acc[3];
      ctx->counters.sources = (ctx->read_hi ? std::min(ctx->read_hi, ctx->n) : ctx->n) - std::min(ctx->read_lo, ctx->n);
    }
    if (mx <= seg_cap) {
      ctx->t.total_ms = ctx->t.index_ms + ctx->t.contained_ms + ctx->t.overlap_ms;
      if (n_rows) *n_rows = total;
      return 0;
    }
    want = (mx + mx / 4 + 1024) * kSegs;  // a segment overflowed: exact need is known now
  }
  return set_err(ctx, "row buffer overflow after resize");
}

int mg_copy_rows(mg_ctx* ctx, mg_edge* out, uint64_t cap, uint64_t* n_copied) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  const uint64_t seg_cap = ctx->rows_cap / kSegs;
  uint64_t done = 0;
  for (int s = 0; s < kSegs && done < cap && !ctx->seg_host.empty(); ++s) {
    const uint64_t c = std::min<uint64_t>(std::min<uint64_t>(ctx->seg_host[s], seg_cap), cap - done);
    if (!c) continue;
    MG_TRY(hipMemcpyAsync(out + done, ctx->d_rows + (uint64_t)s * seg_cap * 3, c * sizeof(mg_edge),
                          hipMemcpyDeviceToHost, ctx->stream));
    done += c;
  }
  MG_TRY(hipStreamSynchronize(ctx->stream));
  if (n_copied) *n_copied = done;
  return 0;
}

int mg_lookup_key(mg_ctx* ctx, const char* key, uint32_t key_len, uint64_t* out, uint64_t cap, uint64_t* n_out) {
  if (!ctx) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->index_ready) return set_err(ctx, "mg_build_index must run first");
  if (n_out) *n_out = 0;
  if (key_len != ctx->h) return 0;  // no key of another length exists
  if (ctx->nranks > 1) return set_err(ctx, "lookup on a bucket-sharded index");
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
  if (dispatch_w<LaunchLookup>(ctx->maxw, ctx, dq, qwords, dout, dcap, dn)) return set_err(ctx, "lookup failed");
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

int mg_get_timings(const mg_ctx* ctx, mg_timings* t) {
  if (!ctx || !t) return -1;
  *t = ctx->t;
  return 0;
}

int mg_get_counters(const mg_ctx* ctx, mg_counters* c) {
  if (!ctx || !c) return -1;
  *c = ctx->counters;
  return 0;
}

}  // extern "C"
