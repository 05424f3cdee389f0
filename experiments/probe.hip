// Calibration probes (not part of the product library): kernel-duration floors on MI355X for
// an empty launch and for a pure 16-B streaming read, timed by hipExtLaunchKernelGGL events
// (the dispatch's own start/stop timestamps, as rocprofv3 reports them).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void empty_kernel(int* sink) {
  if (sink != nullptr && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 1;
}

// Thread t of T loads p[t + i*T] for i < L (each wave-instruction = 1 KiB contiguous).
template <int L, bool NT>
__global__ void read_kernel(const uint4* __restrict__ p, uint32_t* __restrict__ out, int64_t T) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 v[L];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    if (NT) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + t + i * T));
      v[i] = make_uint4(a[0], a[1], a[2], a[3]);
    } else {
      v[i] = p[t + i * T];
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  if (acc == 0x9E3779B9u) out[t & 1023] = acc;  // keeps the loads live, never taken in practice
}

static float timed(hipEvent_t a, hipEvent_t b) {
  float ms = -1.f;
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

extern "C" {

// Plain (unprofiled) launch of the empty kernel on a stream: for graph-replay timing.
int probe_empty_launch(int grid, int block, void* stream) {
  hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(block), 0, (hipStream_t)stream, (int*)nullptr);
  return (int)hipGetLastError();
}

float probe_empty(int grid, int block) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipExtLaunchKernelGGL(empty_kernel, dim3(grid), dim3(block), 0, 0, a, b, 0, (int*)nullptr);
  float ms = timed(a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms;
}

// bytes must be a multiple of 16 * block * L. Returns kernel ms.
float probe_read(const void* p, int64_t bytes, int block, int L, int nt, void* out) {
  const int64_t n16 = bytes / 16;
  const int64_t T = n16 / L;
  const int grid = (int)(T / block);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
#define RK(LL)                                                                               \
  if (L == LL) {                                                                             \
    if (nt)                                                                                  \
      hipExtLaunchKernelGGL(read_kernel<LL, true>, dim3(grid), dim3(block), 0, 0, a, b, 0, q, o, T); \
    else                                                                                     \
      hipExtLaunchKernelGGL(read_kernel<LL, false>, dim3(grid), dim3(block), 0, 0, a, b, 0, q, o, T); \
  }
  RK(1) RK(2) RK(4) RK(8) RK(16)
#undef RK
  float ms = timed(a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms;
}

// Plain launch of the streaming read on a stream (graph capture). bytes % (16 * block * L) == 0.
int probe_read_launch(const void* p, int64_t bytes, int block, int L, int nt, void* out,
                      void* stream) {
  const int64_t T = bytes / 16 / L;
  const int grid = (int)(T / block);
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  hipStream_t st = (hipStream_t)stream;
#define RL(LL)                                                                               \
  if (L == LL) {                                                                             \
    if (nt)                                                                                  \
      hipLaunchKernelGGL((read_kernel<LL, true>), dim3(grid), dim3(block), 0, st, q, o, T);   \
    else                                                                                     \
      hipLaunchKernelGGL((read_kernel<LL, false>), dim3(grid), dim3(block), 0, st, q, o, T);  \
  }
  RL(1) RL(2) RL(4) RL(8) RL(16)
#undef RL
  return (int)hipGetLastError();
}

}  // extern "C"
