// Standalone reproducer for the round-4 k_over_heads failure
// (metagenomics_amd/csrc/device/mg_kernels.hip k_over_heads).
//
// k_over_heads marks the first record of each RUN (a cell group's overflow
// records of one fingerprint, adjacent after the exchange mode's sort):
// head[i] = i there, else 0; a max-scan then gives every overflow record its
// run's start.  The round-4 source formed the head with a nested select,
//   head[i] = (over && (first || fp(ent[i]) != fp(ent[i - 1]))) ? i : 0;
// and the shipped source forms it with a multiply over unconditional loads.
// This program runs three forms on the same sorted records and checks each
// against a host restatement (and a fourth, FLAGS, that audits the helpers the
// forms share: rank_in_cell and over_rec's over / first flags, whose own
// short-circuit guards i >= k && key[i - k] are the same pattern):
//   SELECT  the round-4 expression, verbatim;
//   MUL     the shipped expression;
//   GUARD   the nested select with the i - 1 load guarded (ent[i ? i - 1 : 0]).
// The helpers (rank_in_cell, over_rec, entry_fp) are copied from
// mg_kernels.hip.  Inputs: `groups` cell groups of 1..max_group records each;
// inside a group the records of one fingerprint are adjacent, as after the
// sort; n_dev (the device-side record count) on or off as in build_cells.
// Output: one JSON line per (form, n_dev) with the number of wrong heads and
// the first few wrong indices.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 over_heads_repro.hip -o over_heads_repro
//   ISA:   hipcc --offload-arch=gfx950 -O3 -std=c++17 --save-temps -c over_heads_repro.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);    \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

constexpr int kBlock = 256;
constexpr int kCell = 8;

__host__ __device__ __forceinline__ uint32_t entry_fp(unsigned long long e) {
  return (uint32_t)(e >> 44) & ((1u << 19) - 1);
}

__device__ __forceinline__ int rank_in_cell(const uint32_t* __restrict__ key, uint64_t i, uint32_t shift, uint32_t c) {
  bool eq[kCell + 1];
#pragma unroll
  for (int k = 1; k <= kCell; ++k) eq[k] = i >= (uint64_t)k && (key[i - k] >> shift) == c;
  int r = 0;
#pragma unroll
  for (int k = 1; k <= kCell; ++k) r = (r == k - 1 && eq[k]) ? k : r;
  return r;
}

__device__ __forceinline__ bool over_rec(const uint32_t* __restrict__ key, uint64_t i, uint32_t gshift, uint32_t g,
                                         bool* first) {
  if (rank_in_cell(key, i, gshift, g) != kCell) return false;
  *first = !(i >= kCell + 1 && (key[i - kCell - 1] >> gshift) == g);
  return true;
}

enum Form { SELECT = 0, MUL = 1, GUARD = 2, FLAGS = 3 };

template <int F>
__global__ __launch_bounds__(kBlock) void k_over_heads(const uint32_t* __restrict__ key,
                                                      const uint64_t* __restrict__ ent,
                                                      const unsigned long long* __restrict__ n_dev, uint64_t n_host,
                                                      uint32_t gshift, int skip_odd, uint32_t* __restrict__ head) {
  const uint64_t n = n_dev ? *n_dev : n_host;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t g = key[i] >> gshift;
    bool first = false;
    const bool over = !(skip_odd && (g & 1u)) && over_rec(key, i, gshift, g, &first);
    if (F == FLAGS) {  // the audit of the helpers themselves: rank | over << 4 | first << 5
      head[i] = (uint32_t)rank_in_cell(key, i, gshift, g) | (over ? 16u : 0u) | (first ? 32u : 0u);
    } else if (F == SELECT) {
      head[i] = (over && (first || entry_fp(ent[i]) != entry_fp(ent[i - 1]))) ? (uint32_t)i : 0u;
    } else if (F == GUARD) {
      head[i] = (over && (first || entry_fp(ent[i]) != entry_fp(ent[i ? i - 1 : 0]))) ? (uint32_t)i : 0u;
    } else {
      const uint32_t fp_prev = entry_fp(ent[i ? i - 1 : 0]), fp_cur = entry_fp(ent[i]);
      const uint32_t hd = (over ? 1u : 0u) & ((first ? 1u : 0u) | (fp_prev != fp_cur ? 1u : 0u));
      head[i] = (uint32_t)i * hd;
    }
  }
}

int main(int argc, char** argv) {
  const int groups = argc > 1 ? std::atoi(argv[1]) : 200000;
  const int max_group = argc > 2 ? std::atoi(argv[2]) : 40;
  const uint32_t gshift = 3;  // 3 low fingerprint bits under the group, as build_cells' sort key
  std::mt19937_64 rng(12345);
  std::vector<uint32_t> key;
  std::vector<uint64_t> ent;
  for (int gi = 0; gi < groups; ++gi) {
    const int sz = 1 + (int)(rng() % (uint64_t)max_group);
    const int nfp = 1 + (int)(rng() % 3);  // fingerprints per group, each a contiguous run
    std::vector<uint32_t> fps(nfp);
    for (int f = 0; f < nfp; ++f) fps[f] = (uint32_t)(rng() & ((1u << 19) - 1));
    std::sort(fps.begin(), fps.end());
    for (int r = 0; r < sz; ++r) {
      const uint32_t fp = fps[(size_t)r * nfp / sz];
      key.push_back(((uint32_t)gi << (gshift + 1)) | (fp & 7u));  // group 2 gi: even, skip_odd never skips it
      ent.push_back(((uint64_t)fp << 44) | (uint64_t)(key.size() & 0xFFFFFFFFu));
    }
  }
  const uint64_t n = key.size();
  // host restatement
  std::vector<uint32_t> want(n, 0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t g = key[i] >> gshift;
    int r = 0;
    for (int k = 1; k <= kCell; ++k) r = (r == k - 1 && i >= (uint64_t)k && (key[i - k] >> gshift) == g) ? k : r;
    if (r != kCell) continue;
    const bool first = !(i >= kCell + 1 && (key[i - kCell - 1] >> gshift) == g);
    if (first || entry_fp(ent[i]) != entry_fp(ent[i - 1])) want[i] = (uint32_t)i;
  }
  // the helpers' own outputs (rank_in_cell, over_rec's over and first), as FLAGS writes them
  std::vector<uint32_t> want_flags(n, 0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t g = key[i] >> gshift;
    int r = 0;
    for (int k = 1; k <= kCell; ++k) r = (r == k - 1 && i >= (uint64_t)k && (key[i - k] >> gshift) == g) ? k : r;
    const bool over = r == kCell;
    const bool first = over && !(i >= kCell + 1 && (key[i - kCell - 1] >> gshift) == g);
    want_flags[i] = (uint32_t)r | (over ? 16u : 0u) | (first ? 32u : 0u);
  }
  uint32_t *dk = nullptr, *dh = nullptr;
  uint64_t* de = nullptr;
  unsigned long long* dn = nullptr;
  CK(hipMalloc(&dk, n * 4));
  CK(hipMalloc(&de, n * 8));
  CK(hipMalloc(&dh, n * 4));
  CK(hipMalloc(&dn, 8));
  CK(hipMemcpy(dk, key.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(de, ent.data(), n * 8, hipMemcpyHostToDevice));
  const unsigned long long nn = n;
  CK(hipMemcpy(dn, &nn, 8, hipMemcpyHostToDevice));
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + kBlock - 1) / kBlock,
                                                                            (uint64_t)prop.multiProcessorCount * 32));
  uint64_t heads = 0;
  for (uint64_t i = 0; i < n; ++i) heads += want[i] != 0;
  std::printf("{\"records\": %llu, \"heads\": %llu, \"grid\": %u}\n", (unsigned long long)n,
              (unsigned long long)heads, grid);
  std::vector<uint32_t> got(n);
  const char* names[4] = {"select", "mul", "guard", "flags"};
  for (int f = 0; f < 4; ++f)
    for (int use_dev = 0; use_dev < 2; ++use_dev) {
      CK(hipMemset(dh, 0xAB, n * 4));
      const unsigned long long* ndp = use_dev ? dn : nullptr;
      if (f == SELECT) hipLaunchKernelGGL(k_over_heads<SELECT>, dim3(grid), dim3(kBlock), 0, 0, dk, de, ndp, n, gshift, 1, dh);
      if (f == MUL) hipLaunchKernelGGL(k_over_heads<MUL>, dim3(grid), dim3(kBlock), 0, 0, dk, de, ndp, n, gshift, 1, dh);
      if (f == GUARD) hipLaunchKernelGGL(k_over_heads<GUARD>, dim3(grid), dim3(kBlock), 0, 0, dk, de, ndp, n, gshift, 1, dh);
      if (f == FLAGS) hipLaunchKernelGGL(k_over_heads<FLAGS>, dim3(grid), dim3(kBlock), 0, 0, dk, de, ndp, n, gshift, 1, dh);
      const std::vector<uint32_t>& ref = f == FLAGS ? want_flags : want;
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), dh, n * 4, hipMemcpyDeviceToHost));
      uint64_t bad = 0, bad_head = 0, bad_zero = 0;
      std::string first_bad;
      for (uint64_t i = 0; i < n; ++i)
        if (got[i] != ref[i]) {
          ++bad;
          (want[i] ? bad_head : bad_zero) += 1;
          if (bad <= 5)
            first_bad += (bad > 1 ? ", " : "") + std::string("[") + std::to_string(i) + ", " +
                         std::to_string(ref[i]) + ", " + std::to_string(got[i]) + "]";
        }
      std::printf(
          "{\"form\": \"%s\", \"n_dev\": %d, \"wrong\": %llu, \"wrong_at_heads\": %llu, \"wrong_elsewhere\": %llu, "
          "\"first_wrong_i_want_got\": [%s]}\n",
          names[f], use_dev, (unsigned long long)bad, (unsigned long long)bad_head, (unsigned long long)bad_zero,
          first_bad.c_str());
    }
  CK(hipFree(dk));
  CK(hipFree(de));
  CK(hipFree(dh));
  CK(hipFree(dn));
  return 0;
}
