// mg_xchg_local.hip — the one device kernel of LocalTransport (mg_xchg.hpp):
// the MAX all-reduce of P in-process ranks' arrays on one device (u64
// containment keys, u8 prefix marks).  Each rank
// reduces its own slice [lo, hi) of every array and writes the maximum back to
// all of them, so the ranks' slices never overlap and no scratch is needed.
// (The containment keys len << 32 | ~index, OverlapGraph.cpp:259-268: the
// unsigned maximum is the reference's "longest container, lowest ID first".)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "mg_xchg.hpp"

namespace mg {
namespace {
constexpr int kMaxLocal = 16;
template <typename T>
struct Ptrs {
  T* p[kMaxLocal];
};

template <typename T>
__global__ __launch_bounds__(256) void k_local_max(Ptrs<T> a, int P, uint64_t lo, uint64_t hi) {
  for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
       i += (uint64_t)gridDim.x * blockDim.x) {
    T m = a.p[0][i];
    for (int r = 1; r < P; ++r) m = a.p[r][i] > m ? a.p[r][i] : m;
    for (int r = 0; r < P; ++r) a.p[r][i] = m;
  }
}

template <typename T>
void local_max(T* const* ptrs, int P, uint64_t lo, uint64_t hi, hipStream_t s) {
  if (P < 1 || P > kMaxLocal) throw std::runtime_error("local_max: 1..16 ranks");
  if (hi <= lo) return;
  Ptrs<T> a{};
  for (int r = 0; r < P; ++r) a.p[r] = ptrs[r];
  const uint64_t n = hi - lo;
  const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_local_max<T>, dim3(grid), dim3(256), 0, s, a, P, lo, hi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("k_local_max: ") + hipGetErrorString(e));
}
}  // namespace

void local_max_u64(uint64_t* const* ptrs, int P, uint64_t lo, uint64_t hi, hipStream_t s) {
  local_max<uint64_t>(ptrs, P, lo, hi, s);
}
void local_max_u8(uint8_t* const* ptrs, int P, uint64_t lo, uint64_t hi, hipStream_t s) {
  local_max<uint8_t>(ptrs, P, lo, hi, s);
}

}  // namespace mg
