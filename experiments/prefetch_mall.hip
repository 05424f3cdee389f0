// Experiment (not the product path): a side-stream kernel that reads a byte range with default-
// policy 16-B loads, so the range lands in the MALL (memory-side Infinity Cache) ahead of the
// GEMV that streams it. Grid-stride over `bytes` with `grid` workgroups of 256 threads, four
// loads in flight per thread; a value derived from every load is stored only if it matches a
// constant no data produces.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o experiments/build/libprefetch.so \
//     experiments/prefetch_mall.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void prefetch_kernel(const uint4* __restrict__ p, size_t n16,
                                                       uint32_t* __restrict__ sink) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = i + 256 * j < n16 ? p[i + 256 * j] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;
}

extern "C" int prefetch_launch(const void* p, size_t bytes, int grid, void* sink, void* stream) {
  hipLaunchKernelGGL(prefetch_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)p, bytes / 16, (uint32_t*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
