// mg_dataset.hip — the Dataset ingest on the device.
//
// Reference path replaced (paths relative to /root/reference/MetaGenomics):
//   readDataset per-read body: upper-case      Dataset.cpp:158-159
//   testRead: len > l, only ACGT, 80 % rule     Dataset.cpp:160, 398-413
//   canonical strand = min(s, revcomp(s))      Dataset.cpp:163-167, 463-475
//   sortReads (std::sort, std::string order)   Dataset.cpp:197-202 (comparator :16-19)
//   removeDupicateReads: frequency, IDs 1..N   Dataset.cpp:316-345
//
// Pipeline (all in HBM, one stream):
//   k_ingest<W,SRC> : thread per raw read -> filter, 2-bit pack of both strands,
//                     canonical strand (packed-word compare = std::string order
//                     for equal lengths), valid flag, min/max length;
//   select          : indices of the valid reads (hipcub DeviceSelect);
//   LSD sort        : stable radix passes over (length, word W-1, ..., word 0)
//                     = std::string order (zero padding + length tiebreak: a
//                     proper prefix sorts first) (hipcub DeviceRadixSort);
//   k_dedup_*       : run starts of equal reads -> exclusive scan -> unique
//                     reads written in ID order into the context's read slots,
//                     frequency = run length.
// The result is exactly what mg_upload_reads_packed would receive from the
// host Dataset mirror (tests/test_gpu_parity.py::test_device_ingest_*).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "mg_ctx.hpp"
#include "mg_overlap.h"

namespace {

constexpr int kThreads = 256;

// ASCII (concatenated, offsets) or 2-bit codes (fixed stride, lengths) source
struct IngestSrc {
  const char* ascii;
  const uint64_t* off;
  const uint8_t* codes;
  uint64_t stride;
  const uint16_t* lens;
};

template <bool ASCII>
__device__ __forceinline__ uint64_t raw_len(const IngestSrc& s, uint64_t i) {
  return ASCII ? s.off[i + 1] - s.off[i] : s.lens[i];
}

// code of base p of read i: 0..3, or 4 when not A/C/G/T (any case; the
// reference upper-cases the line before testRead, Dataset.cpp:158-159)
template <bool ASCII>
__device__ __forceinline__ uint32_t base_code(const IngestSrc& s, uint64_t i, uint64_t p) {
  if (ASCII) {
    const uint32_t c = (uint8_t)s.ascii[s.off[i] + p] & 0xDFu;  // upper-case letters
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
  }
  const uint32_t c = s.codes[i * s.stride + p];
  return c <= 3u ? c : 4u;
}

// One thread per raw read: testRead + both strands packed (W words each,
// MSB-first, zero padded) + the canonical strand.
template <int W, bool ASCII>
__global__ __launch_bounds__(kThreads) void k_ingest(IngestSrc s, uint64_t n, uint32_t min_overlap,
                                                     uint64_t* __restrict__ canon, uint16_t* __restrict__ len_out,
                                                     uint8_t* __restrict__ valid, unsigned int* __restrict__ lenrange) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t L = raw_len<ASCII>(s, i);
  bool ok = L > min_overlap && L <= 65535 && L <= 32u * W;  // Dataset.cpp:160; UINT16 length
  uint64_t f[W], r[W];
  uint32_t cnt[4] = {0, 0, 0, 0};
  if (ok) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
      uint64_t x = 0, y = 0;
      for (int t = 0; t < 32; ++t) {
        const uint64_t p = 32u * k + t;
        uint32_t cf = 0, cr = 0;
        if (p < L) {
          cf = base_code<ASCII>(s, i, p);
          if (cf > 3u) ok = false;
          else cnt[cf]++;
          const uint32_t cb = base_code<ASCII>(s, i, L - 1 - p);  // reverseComplement (Dataset.cpp:463-475)
          cr = cb > 3u ? 0u : 3u - cb;
        }
        x = (x << 2) | (cf & 3u);
        y = (y << 2) | cr;
      }
      f[k] = x;
      r[k] = y;
    }
  }
  if (ok) {  // 80 % rule (Dataset.cpp:409-411): threshold = (UINT64)(length * .8)
    const uint64_t thr = (uint64_t)((double)L * .8);
    ok = cnt[0] < thr && cnt[1] < thr && cnt[2] < thr && cnt[3] < thr;
  }
  valid[i] = ok ? 1 : 0;
  len_out[i] = (uint16_t)(ok ? L : 0);
  if (!ok) return;
  // std::lexicographical_compare(s, rc): equal lengths -> first differing word
  bool fwd = false;
  bool decided = false;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    if (!decided && f[k] != r[k]) {
      fwd = f[k] < r[k];
      decided = true;
    }
  }
#pragma unroll
  for (int k = 0; k < W; ++k) canon[i * W + k] = fwd ? f[k] : r[k];
  atomicMin(&lenrange[0], (unsigned int)L);
  atomicMax(&lenrange[1], (unsigned int)L);
}

// k_ingest for reads longer than 1,024 bp (up to 65,535, Read.h:62): the same
// filter and canonical strand, but the words are built one at a time from the
// source (no register arrays): pass 1 testRead, pass 2 the first word where
// the strands differ (std::lexicographical_compare), pass 3 the chosen
// strand's CW words.
template <bool ASCII>
__global__ __launch_bounds__(kThreads) void k_ingest_long(IngestSrc s, uint64_t n, uint32_t min_overlap, uint32_t cw,
                                                          uint64_t* __restrict__ canon, uint16_t* __restrict__ len_out,
                                                          uint8_t* __restrict__ valid,
                                                          unsigned int* __restrict__ lenrange) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t L = raw_len<ASCII>(s, i);
  bool ok = L > min_overlap && L <= 65535 && L <= 32u * cw;  // Dataset.cpp:160; UINT16 length
  uint32_t cnt[4] = {0, 0, 0, 0};
  for (uint64_t p = 0; ok && p < L; ++p) {
    const uint32_t c = base_code<ASCII>(s, i, p);
    if (c > 3u) ok = false;
    else cnt[c]++;
  }
  if (ok) {  // 80 % rule (Dataset.cpp:409-411)
    const uint64_t thr = (uint64_t)((double)L * .8);
    ok = cnt[0] < thr && cnt[1] < thr && cnt[2] < thr && cnt[3] < thr;
  }
  valid[i] = ok ? 1 : 0;
  len_out[i] = (uint16_t)(ok ? L : 0);
  if (!ok) return;
  auto word = [&](uint32_t k, bool rc) {
    uint64_t x = 0;
    for (int t = 0; t < 32; ++t) {
      const uint64_t p = 32u * k + t;
      uint32_t c = 0;
      if (p < L) c = rc ? 3u - base_code<ASCII>(s, i, L - 1 - p) : base_code<ASCII>(s, i, p);
      x = (x << 2) | c;
    }
    return x;
  };
  bool fwd = false;
  for (uint32_t k = 0; 32u * k < L; ++k) {
    const uint64_t f = word(k, false), r = word(k, true);
    if (f != r) {
      fwd = f < r;
      break;
    }
  }
  for (uint32_t k = 0; k < cw; ++k) canon[i * cw + k] = 32u * k < L ? word(k, !fwd) : 0ull;
  atomicMin(&lenrange[0], (unsigned int)L);
  atomicMax(&lenrange[1], (unsigned int)L);
}

// key of the current LSD pass for the order so far (W = 0: cw words per read)
template <int W>
__global__ __launch_bounds__(kThreads) void k_gather_word(const uint64_t* __restrict__ canon,
                                                          const uint32_t* __restrict__ idx, uint64_t n, int k,
                                                          uint64_t* __restrict__ key, uint32_t cw) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) key[i] = canon[(uint64_t)idx[i] * (W ? W : cw) + k];
}

__global__ __launch_bounds__(kThreads) void k_gather_len(const uint16_t* __restrict__ len,
                                                         const uint32_t* __restrict__ idx, uint64_t n,
                                                         uint16_t* __restrict__ key) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) key[i] = len[idx[i]];
}

// run starts of equal reads in sorted order (removeDupicateReads, Dataset.cpp:321-339)
template <int W>
__global__ __launch_bounds__(kThreads) void k_dedup_flags(const uint64_t* __restrict__ canon,
                                                          const uint16_t* __restrict__ len,
                                                          const uint32_t* __restrict__ idx, uint64_t n,
                                                          uint32_t* __restrict__ start, uint32_t cw) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  constexpr uint32_t CW0 = W;
  const uint32_t CW = W ? CW0 : cw;
  bool s = i == 0;
  if (!s) {
    const uint64_t a = idx[i - 1], b = idx[i];
    s = len[a] != len[b];
#pragma unroll
    for (uint32_t k = 0; k < CW; ++k) s = s || canon[a * CW + k] != canon[b * CW + k];
  }
  start[i] = s ? 1u : 0u;
}

// unique read u (ID u + 1) = the run starting at sorted position i; its
// frequency is the run length
template <int W>
__global__ __launch_bounds__(kThreads) void k_dedup_write(const uint64_t* __restrict__ canon,
                                                          const uint16_t* __restrict__ len,
                                                          const uint32_t* __restrict__ idx,
                                                          const uint32_t* __restrict__ start,
                                                          const uint32_t* __restrict__ uid, uint64_t n,
                                                          uint32_t maxw, uint32_t stride,
                                                          uint64_t* __restrict__ words, uint16_t* __restrict__ lens,
                                                          uint32_t* __restrict__ first, uint32_t cw) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n || !start[i]) return;
  const uint64_t u = uid[i], a = idx[i];
  constexpr uint32_t CW0 = W;
  const uint32_t CW = W ? CW0 : cw;
#pragma unroll
  for (uint32_t k = 0; k < CW; ++k)
    if (k < maxw) words[u * stride + k] = canon[a * CW + k];
  lens[u] = len[a];
  first[u] = (uint32_t)i;
}

__global__ __launch_bounds__(kThreads) void k_dedup_freq(const uint32_t* __restrict__ first, uint64_t nu,
                                                         uint64_t ngood, uint32_t* __restrict__ freq) {
  const uint64_t u = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (u < nu) freq[u] = (uint32_t)((u + 1 < nu ? first[u + 1] : ngood) - first[u]);
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) { return hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T)); }
};

uint32_t blocks(uint64_t n) { return (uint32_t)((n + kThreads - 1) / kThreads); }

template <int W>
struct Ingest {
  // W = 0: reads longer than 1,024 bp, cw words per read (k_ingest_long)
  static int run(mg_ctx* ctx, const IngestSrc& s, bool ascii, uint64_t n, uint32_t min_overlap, uint64_t* n_unique,
                 uint32_t cw = 0) {
    hipStream_t st = ctx->stream;
    const uint32_t CW = W ? (uint32_t)W : cw;
    DevBuf<uint64_t> canon, key_a, key_b;
    DevBuf<uint16_t> len, lkey_a, lkey_b;
    DevBuf<uint8_t> valid;
    DevBuf<uint32_t> idx_a, idx_b, start, uid, first;
    DevBuf<unsigned int> lr;
    DevBuf<unsigned long long> nsel;
    MG_TRY(canon.alloc(n * CW));
    MG_TRY(len.alloc(n));
    MG_TRY(valid.alloc(n));
    MG_TRY(lr.alloc(2));
    MG_TRY(nsel.alloc(1));
    const unsigned int lr0[2] = {0xFFFFFFFFu, 0u};
    MG_TRY(hipMemcpyAsync(lr.p, lr0, sizeof(lr0), hipMemcpyHostToDevice, st));
    if (n) {
      if (W == 0 && ascii)
        hipLaunchKernelGGL((k_ingest_long<true>), dim3(blocks(n)), dim3(kThreads), 0, st, s, n, min_overlap, CW,
                           canon.p, len.p, valid.p, lr.p);
      else if (W == 0)
        hipLaunchKernelGGL((k_ingest_long<false>), dim3(blocks(n)), dim3(kThreads), 0, st, s, n, min_overlap, CW,
                           canon.p, len.p, valid.p, lr.p);
      else if (ascii)
        hipLaunchKernelGGL((k_ingest<(W ? W : 1), true>), dim3(blocks(n)), dim3(kThreads), 0, st, s, n, min_overlap,
                           canon.p, len.p, valid.p, lr.p);
      else
        hipLaunchKernelGGL((k_ingest<(W ? W : 1), false>), dim3(blocks(n)), dim3(kThreads), 0, st, s, n, min_overlap,
                           canon.p, len.p, valid.p, lr.p);
      MG_TRY(hipGetLastError());
    }
    // indices of the valid reads, in input order
    MG_TRY(idx_a.alloc(n));
    MG_TRY(idx_b.alloc(n));
    size_t tb = 0;
    hipcub::CountingInputIterator<uint32_t> it(0);
    MG_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, it, valid.p, idx_a.p, nsel.p, (int)n, st));
    DevBuf<uint8_t> tmp;
    size_t tmp_bytes = tb;
    {
      size_t t2 = 0;
      MG_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, key_a.p, key_b.p, idx_a.p, idx_b.p, (int)n, 0, 64, st));
      tmp_bytes = std::max(tmp_bytes, t2);
      MG_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, lkey_a.p, lkey_b.p, idx_a.p, idx_b.p, (int)n, 0, 16, st));
      tmp_bytes = std::max(tmp_bytes, t2);
      MG_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, start.p, uid.p, (int)n, st));
      tmp_bytes = std::max(tmp_bytes, t2);
    }
    MG_TRY(tmp.alloc(tmp_bytes));
    tb = tmp_bytes;
    MG_TRY(hipcub::DeviceSelect::Flagged(tmp.p, tb, it, valid.p, idx_a.p, nsel.p, (int)n, st));
    unsigned long long ng = 0;
    unsigned int lrh[2] = {0, 0};
    MG_TRY(hipMemcpyAsync(&ng, nsel.p, sizeof(ng), hipMemcpyDeviceToHost, st));
    MG_TRY(hipMemcpyAsync(lrh, lr.p, sizeof(lrh), hipMemcpyDeviceToHost, st));
    MG_TRY(hipStreamSynchronize(st));
    const uint64_t ngood = ng;
    // LSD: length, then words W-1 .. 0 (stable) = (words, length) order
    MG_TRY(key_a.alloc(ngood));
    MG_TRY(key_b.alloc(ngood));
    MG_TRY(lkey_a.alloc(ngood));
    MG_TRY(lkey_b.alloc(ngood));
    uint32_t* cur = idx_a.p;
    uint32_t* alt = idx_b.p;
    if (ngood) {
      const bool lens_differ = lrh[0] != lrh[1];
      if (lens_differ) {
        hipLaunchKernelGGL(k_gather_len, dim3(blocks(ngood)), dim3(kThreads), 0, st, len.p, cur, ngood, lkey_a.p);
        tb = tmp_bytes;
        MG_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, lkey_a.p, lkey_b.p, cur, alt, (int)ngood, 0, 16, st));
        std::swap(cur, alt);
      }
      const uint32_t wused = (lrh[1] + 31) / 32;  // words past the longest read are all zero
      for (int k = (int)wused - 1; k >= 0; --k) {
        hipLaunchKernelGGL((k_gather_word<W>), dim3(blocks(ngood)), dim3(kThreads), 0, st, canon.p, cur, ngood, k,
                           key_a.p, CW);
        tb = tmp_bytes;
        MG_TRY(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, key_a.p, key_b.p, cur, alt, (int)ngood, 0, 64, st));
        std::swap(cur, alt);
      }
    }
    // dedup + IDs + frequency
    MG_TRY(start.alloc(ngood));
    MG_TRY(uid.alloc(ngood));
    if (ngood) {
      hipLaunchKernelGGL((k_dedup_flags<W>), dim3(blocks(ngood)), dim3(kThreads), 0, st, canon.p, len.p, cur, ngood,
                         start.p, CW);
      tb = tmp_bytes;
      MG_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, start.p, uid.p, (int)ngood, st));
    }
    uint32_t last_uid = 0, last_start = 0;
    if (ngood) {
      MG_TRY(hipMemcpyAsync(&last_uid, uid.p + ngood - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      MG_TRY(hipMemcpyAsync(&last_start, start.p + ngood - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    }
    MG_TRY(hipStreamSynchronize(st));
    const uint64_t nu = ngood ? (uint64_t)last_uid + last_start : 0;
    if (nu >= 0xFFFFFFFFull) return set_err(ctx, "too many reads (max 2^32-2)");
    const uint32_t maxw = slot_maxw(std::max<uint32_t>(1, (lrh[1] + 31) / 32));
    ctx->n = nu;
    ctx->maxw = ngood ? maxw : supported_maxw(1);
    ctx->stride = slot_stride(ctx->maxw);
    const size_t nw = (size_t)(nu + 2) * ctx->stride + 2;  // zero pad for over-reads
    MG_ENSURE(d_words, words_cap, nw);
    MG_ENSURE(d_len, len_cap, nu + 1);
    MG_ENSURE(d_freq, freq_cap, nu + 1);
    MG_TRY(hipMemsetAsync(ctx->d_words, 0, nw * sizeof(uint64_t), st));
    MG_TRY(first.alloc(nu));
    if (ngood) {
      hipLaunchKernelGGL((k_dedup_write<W>), dim3(blocks(ngood)), dim3(kThreads), 0, st, canon.p, len.p, cur, start.p,
                         uid.p, ngood, ctx->maxw, ctx->stride, ctx->d_words, ctx->d_len, first.p, CW);
      hipLaunchKernelGGL(k_dedup_freq, dim3(blocks(nu)), dim3(kThreads), 0, st, first.p, nu, ngood, ctx->d_freq);
      MG_TRY(hipGetLastError());
    }
    MG_TRY(hipStreamSynchronize(st));
    ctx->n_good = ngood;
    ctx->minlen = ngood ? lrh[0] : 0;
    ctx->maxlen = ngood ? lrh[1] : 0;
    if (apply_layout(ctx)) return -1;
    reset_derived(ctx);
    *n_unique = nu;
    return 0;
  }
};

int ingest(mg_ctx* ctx, const IngestSrc& s, bool ascii, uint64_t n, uint64_t maxlen, uint32_t min_overlap,
           uint64_t* n_unique) {
  const uint64_t need = (std::min<uint64_t>(maxlen, 65535) + 31) / 32;
  if (need > 32) return Ingest<0>::run(ctx, s, ascii, n, min_overlap, n_unique, (uint32_t)need);
  const uint32_t w = supported_maxw((uint32_t)std::max<uint64_t>(1, need));
  switch (w) {
    case 1: return Ingest<1>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 2: return Ingest<2>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 3: return Ingest<3>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 4: return Ingest<4>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 5: return Ingest<5>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 6: return Ingest<6>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 8: return Ingest<8>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 12: return Ingest<12>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 16: return Ingest<16>::run(ctx, s, ascii, n, min_overlap, n_unique);
    case 32: return Ingest<32>::run(ctx, s, ascii, n, min_overlap, n_unique);
  }
  return set_err(ctx, "unsupported read length");
}

}  // namespace

extern "C" {

int mg_ingest_ascii(mg_ctx* ctx, const char* concat, const uint64_t* offsets, uint64_t n_raw, uint32_t min_overlap,
                    uint64_t* n_unique) {
  if (!ctx || !n_unique || (n_raw && (!concat || !offsets))) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (n_raw >= 0xFFFFFFFFull) return set_err(ctx, "too many reads (max 2^32-2)");
  uint64_t longest_valid_len = 0;
  for (uint64_t i = 0; i < n_raw; ++i) {
    const uint64_t L = offsets[i + 1] - offsets[i];
    if (L > min_overlap && L <= 65535) longest_valid_len = std::max(longest_valid_len, L);
  }
  const uint64_t total = n_raw ? offsets[n_raw] : 0;
  DevBuf<char> d_ascii;
  DevBuf<uint64_t> d_off;
  MG_TRY(d_ascii.alloc(total));
  MG_TRY(d_off.alloc(n_raw + 1));
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  if (total) MG_TRY(hipMemcpyAsync(d_ascii.p, concat, total, hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipMemcpyAsync(d_off.p, offsets, (n_raw + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  IngestSrc s{d_ascii.p, d_off.p, nullptr, 0, nullptr};
  // slot width from the longest read that can pass testRead's length bounds
  if (ingest(ctx, s, true, n_raw, longest_valid_len, min_overlap, n_unique)) return -1;
  MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
  MG_TRY(hipEventSynchronize(ctx->ev[2]));
  float h2d = 0.f, dev = 0.f;
  (void)hipEventElapsedTime(&h2d, ctx->ev[0], ctx->ev[1]);
  (void)hipEventElapsedTime(&dev, ctx->ev[1], ctx->ev[2]);
  ctx->t.upload_ms = h2d;
  ctx->t.ingest_ms = dev;
  return 0;
}

int mg_ingest_codes(mg_ctx* ctx, const uint8_t* codes, uint64_t n_raw, uint64_t stride, const uint16_t* lens,
                    uint32_t min_overlap, uint64_t* n_unique) {
  if (!ctx || !n_unique || (n_raw && (!codes || !lens))) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (n_raw >= 0xFFFFFFFFull) return set_err(ctx, "too many reads (max 2^32-2)");
  uint64_t maxlen = 0, longest_valid_len = 0;
  for (uint64_t i = 0; i < n_raw; ++i) {
    maxlen = std::max<uint64_t>(maxlen, lens[i]);
    if (lens[i] > min_overlap) longest_valid_len = std::max<uint64_t>(longest_valid_len, lens[i]);
  }
  if (maxlen > stride && n_raw > 1) return set_err(ctx, "read length exceeds the row stride");
  DevBuf<uint8_t> d_codes;
  DevBuf<uint16_t> d_lens;
  MG_TRY(d_codes.alloc(n_raw * stride));
  MG_TRY(d_lens.alloc(n_raw));
  MG_TRY(hipEventRecord(ctx->ev[0], ctx->stream));
  if (n_raw) {
    MG_TRY(hipMemcpyAsync(d_codes.p, codes, n_raw * stride, hipMemcpyHostToDevice, ctx->stream));
    MG_TRY(hipMemcpyAsync(d_lens.p, lens, n_raw * sizeof(uint16_t), hipMemcpyHostToDevice, ctx->stream));
  }
  MG_TRY(hipEventRecord(ctx->ev[1], ctx->stream));
  IngestSrc s{nullptr, nullptr, d_codes.p, stride, d_lens.p};
  if (ingest(ctx, s, false, n_raw, longest_valid_len, min_overlap, n_unique)) return -1;
  MG_TRY(hipEventRecord(ctx->ev[2], ctx->stream));
  MG_TRY(hipEventSynchronize(ctx->ev[2]));
  float h2d = 0.f, dev = 0.f;
  (void)hipEventElapsedTime(&h2d, ctx->ev[0], ctx->ev[1]);
  (void)hipEventElapsedTime(&dev, ctx->ev[1], ctx->ev[2]);
  ctx->t.upload_ms = h2d;
  ctx->t.ingest_ms = dev;
  return 0;
}

int mg_dataset_counts(const mg_ctx* ctx, uint64_t* n_good, uint64_t* n_unique) {
  if (!ctx) return -1;
  if (n_good) *n_good = ctx->n_good;
  if (n_unique) *n_unique = ctx->n;
  return 0;
}

int mg_download_frequency(mg_ctx* ctx, uint32_t* freq) {
  if (!ctx || !freq) return -1;
  MG_TRY(hipSetDevice(ctx->device));
  if (!ctx->d_freq) return set_err(ctx, "no device-ingested Dataset");
  if (ctx->n) MG_TRY(hipMemcpy(freq, ctx->d_freq, ctx->n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return 0;
}

}  // extern "C"
