// Experiment (not part of the product library): a side-stream weight prefetcher. While the
// GEMV of linear i runs, a loader kernel on a second stream streams linear i+1's packed weights
// and scales from HBM so they sit in the Infinity Cache (MALL) when GEMV i+1 starts. The
// question it answers: does keeping HBM busy across the launch boundaries shorten the
// 129-launch decode step (bench.py), and by how much.
#include <hip/hip_runtime.h>
#include <stdint.h>

// Each thread loads 16 B per unrolled step, U steps per iteration, grid-stride over the buffer.
// POL: 0 default, 1 non-temporal.
template <int U, int POL>
__global__ __launch_bounds__(256) void pf_kernel(const uint4* __restrict__ p, int64_t n16,
                                                 uint32_t* __restrict__ sink, uint32_t magic) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (U - 1) * T < n16; i += U * T) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4* q = reinterpret_cast<const u32x4*>(p + i + u * T);
      v[u] = POL == 1 ? __builtin_nontemporal_load(q) : *q;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  for (; i < n16; i += T) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == magic) sink[threadIdx.x] = acc;  // keeps the loads live; magic never matches
}

extern "C" int pf_launch(const void* p, int64_t bytes, int grid, int pol, void* sink,
                         void* stream) {
  const int64_t n16 = bytes / 16;
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint32_t* s = reinterpret_cast<uint32_t*>(sink);
  hipStream_t st = (hipStream_t)stream;
  if (pol == 1)
    hipLaunchKernelGGL((pf_kernel<8, 1>), dim3(grid), dim3(256), 0, st, q, n16, s, 0x9E3779B9u);
  else
    hipLaunchKernelGGL((pf_kernel<8, 0>), dim3(grid), dim3(256), 0, st, q, n16, s, 0x9E3779B9u);
  return (int)hipGetLastError();
}
