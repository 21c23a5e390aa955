// Random-sector gather ceiling on MI355X: the probe kernel's two dominant
// access kinds are one random 64-B cell line and one random 64-B read slot per
// item.  This measures the chip's rate for uniformly random, 64-B aligned
// 64-B (or 16-B / 128-B) loads from a table larger than the Infinity Cache,
// at several loads-in-flight per lane, so DESIGN.md can state the probe's
// random-access roofline.  Also used to calibrate FETCH_SIZE per request
// (rocprofv3 --pmc FETCH_SIZE on this binary: known bytes per launch).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// each lane performs `per_lane` gathers of BYTES bytes, UNR of them in flight
template <int BYTES, int UNR>
__global__ __launch_bounds__(256) void k_gather(const uint4* __restrict__ tab, uint64_t rows, uint64_t per_lane,
                                                uint64_t seed, uint4* __restrict__ sink) {
  constexpr int V = BYTES / 16;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = 0; i < per_lane; i += UNR) {
    uint4 v[UNR][V];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const uint64_t r = mix64(seed ^ (tid * per_lane + i + u)) % rows;
      const uint4* p = tab + r * V;
#pragma unroll
      for (int k = 0; k < V; ++k) v[u][k] = p[k];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int k = 0; k < V; ++k) { acc.x ^= v[u][k].x; acc.y ^= v[u][k].y; acc.z ^= v[u][k].z; acc.w ^= v[u][k].w; }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[tid] = acc;
}

// 48-B read slots (3 x 16 B) at a STRIDE-byte pitch: 48 B packs slots across
// 64-B / 128-B boundaries (a quarter to a half of them straddle two), 64 B
// keeps every slot inside one 64-B sector
template <int STRIDE, int UNR>
__global__ __launch_bounds__(256) void k_gather_slot(const unsigned char* __restrict__ tab, uint64_t rows,
                                                     uint64_t per_lane, uint64_t seed, uint4* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = 0; i < per_lane; i += UNR) {
    uint4 v[UNR][3];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const uint64_t r = mix64(seed ^ (tid * per_lane + i + u)) % rows;
      const uint4* p = reinterpret_cast<const uint4*>(tab + r * STRIDE);
#pragma unroll
      for (int k = 0; k < 3; ++k) v[u][k] = p[k];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int k = 0; k < 3; ++k) { acc.x ^= v[u][k].x; acc.y ^= v[u][k].y; acc.z ^= v[u][k].z; acc.w ^= v[u][k].w; }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[tid] = acc;
}

template <int STRIDE, int UNR>
void run_slot(const uint4* tab, uint64_t table_bytes, int blocks, uint4* sink, uint64_t total_items) {
  const uint64_t rows = table_bytes / STRIDE - 1;
  const uint64_t lanes = (uint64_t)blocks * 256;
  const uint64_t per_lane = ((total_items / lanes) / UNR) * UNR;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto* t8 = reinterpret_cast<const unsigned char*>(tab);
  hipLaunchKernelGGL((k_gather_slot<STRIDE, UNR>), dim3(blocks), dim3(256), 0, 0, t8, rows, per_lane, 1, sink);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_gather_slot<STRIDE, UNR>), dim3(blocks), dim3(256), 0, 0, t8, rows, per_lane, 7 + rep, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double items = (double)per_lane * lanes;
  printf("{\"slot_bytes\": 48, \"stride\": %d, \"unroll\": %d, \"blocks\": %d, \"table_MB\": %.0f, \"items\": %.0f, "
         "\"ms\": %.4f, \"Gitems_per_s\": %.3f}\n",
         STRIDE, UNR, blocks, table_bytes / 1e6, items, best, items / best / 1e6);
  fflush(stdout);
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

template <int BYTES, int UNR>
void run(const uint4* tab, uint64_t table_bytes, int blocks, uint4* sink, uint64_t total_items) {
  const uint64_t rows = table_bytes / BYTES;
  const uint64_t lanes = (uint64_t)blocks * 256;
  const uint64_t per_lane = ((total_items / lanes) / UNR) * UNR;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_gather<BYTES, UNR>), dim3(blocks), dim3(256), 0, 0, tab, rows, per_lane, 1, sink);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_gather<BYTES, UNR>), dim3(blocks), dim3(256), 0, 0, tab, rows, per_lane, 7 + rep, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double items = (double)per_lane * lanes;
  printf("{\"bytes\": %d, \"unroll\": %d, \"blocks\": %d, \"table_MB\": %.0f, \"items\": %.0f, \"ms\": %.4f, "
         "\"Gitems_per_s\": %.3f, \"GB_per_s\": %.1f}\n",
         BYTES, UNR, blocks, table_bytes / 1e6, items, best, items / best / 1e6, items * BYTES / best / 1e6);
  fflush(stdout);
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const uint64_t table_bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 600ull) << 20;
  const uint64_t items = argc > 2 ? strtoull(argv[2], 0, 10) : 200000000ull;
  int ncu = 256;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  ncu = prop.multiProcessorCount;
  uint4* tab; uint4* sink;
  CK(hipMalloc(&tab, table_bytes));
  CK(hipMemset(tab, 0x5a, table_bytes));
  CK(hipMalloc(&sink, (size_t)ncu * 32 * 256 * sizeof(uint4)));
  if (argc > 3 && argv[3][0] == 's') {  // slot pitch only
    for (int bpc : {8, 16}) {
      run<64, 4>(tab, table_bytes, ncu * bpc, sink, items);
      run_slot<48, 2>(tab, table_bytes, ncu * bpc, sink, items);
      run_slot<64, 2>(tab, table_bytes, ncu * bpc, sink, items);
      run_slot<48, 4>(tab, table_bytes, ncu * bpc, sink, items);
      run_slot<64, 4>(tab, table_bytes, ncu * bpc, sink, items);
    }
    CK(hipFree(tab)); CK(hipFree(sink));
    return 0;
  }
  for (int bpc : {4, 8, 16}) {
    const int blocks = ncu * bpc;
    run<64, 1>(tab, table_bytes, blocks, sink, items);
    run<64, 2>(tab, table_bytes, blocks, sink, items);
    run<64, 4>(tab, table_bytes, blocks, sink, items);
  }
  run<16, 4>(tab, table_bytes, ncu * 8, sink, items);
  run<128, 2>(tab, table_bytes, ncu * 8, sink, items);
  CK(hipFree(tab)); CK(hipFree(sink));
  return 0;
}
