// Per-CU intake of an L2-resident operand vs bytes in flight: does a CU take in more than the
// ~62-73 GB/s the prefill GEMMs and the microarch guide's gather measured, given more waves and
// deeper register rings? 256 workgroups (one per CU), THREADS threads each, every lane DEPTH
// 16-B buffer loads in flight (THREADS x DEPTH x 16 B per CU), each workgroup reading 1 MiB:
//   shared 1: every workgroup reads the same 1 MiB (L2-resident per XCD after the first touch);
//   shared 0: each workgroup streams its own 1 MiB of a 256 MiB buffer (HBM).
// One JSON line per (shared, threads, depth): µs per launch (events over 100 launches).
//
//   hipcc --offload-arch=gfx950 -O3 -o experiments/build/probe_l2_intake2 experiments/probe_l2_intake2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

template <int THREADS, int DEPTH>
__global__ __launch_bounds__(THREADS) void intake(const uint8_t* src, size_t wg_stride,
                                                  uint32_t bytes_per_wg, uint32_t* sink) {
  const uint8_t* base = src + (size_t)blockIdx.x * wg_stride;
  const Rsrc r = make_rsrc(base, bytes_per_wg);
  constexpr uint32_t kStep = THREADS * 16;  // bytes per load round of the workgroup
  const uint32_t lane_off = threadIdx.x * 16;
  uint32_t acc = 0;
  u32x4 v[DEPTH];
  // software pipeline: DEPTH loads in flight per lane at all times
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    v[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, d * kStep, 0));
  const uint32_t rounds = bytes_per_wg / kStep;
  for (uint32_t i = DEPTH; i < rounds; i += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc ^= v[d][0] ^ v[d][3];
      v[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, (i + d) * kStep, 0));
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) acc ^= v[d][0] ^ v[d][3];
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int THREADS, int DEPTH>
static void run(bool shared, const uint8_t* small, const uint8_t* big, uint32_t* sink) {
  const int WG = 256;
  const uint32_t bytes = 1u << 20;
  const uint8_t* src = shared ? small : big;
  const size_t stride = shared ? 0 : (size_t)bytes;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) intake<THREADS, DEPTH><<<WG, THREADS>>>(src, stride, bytes, sink);
  hipEventRecord(a);
  const int iters = 100;
  for (int i = 0; i < iters; ++i) intake<THREADS, DEPTH><<<WG, THREADS>>>(src, stride, bytes, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  printf("{\"shared\": %d, \"threads\": %d, \"depth\": %d, \"in_flight_KiB\": %d, \"us\": %.2f, "
         "\"GBps_per_cu\": %.1f, \"chip_TBps\": %.2f}\n",
         (int)shared, THREADS, DEPTH, THREADS * DEPTH * 16 / 1024, us, bytes / us / 1e3,
         (double)bytes * WG / us / 1e6);
  fflush(stdout);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  uint8_t *small = nullptr, *big = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&small, 1 << 20) != hipSuccess || hipMalloc(&big, (size_t)256 << 20) != hipSuccess ||
      hipMalloc(&sink, 4096) != hipSuccess)
    return 1;
  hipMemset(small, 1, 1 << 20);
  hipMemset(big, 1, (size_t)256 << 20);
  for (int sh = 1; sh >= 0; --sh) {
    run<256, 4>(sh, small, big, sink);
    run<256, 8>(sh, small, big, sink);
    run<256, 16>(sh, small, big, sink);
    run<512, 4>(sh, small, big, sink);
    run<512, 8>(sh, small, big, sink);
    run<512, 16>(sh, small, big, sink);
    run<1024, 2>(sh, small, big, sink);
    run<1024, 4>(sh, small, big, sink);
    run<1024, 8>(sh, small, big, sink);
    run<1024, 16>(sh, small, big, sink);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
