// Per-CU intake rate of an L2-resident operand (the x tile of a prefill GEMM: every workgroup
// re-reads the same rows) vs a streamed-once operand (the weights), on one MI355X.
//
// 256 workgroups x 256 threads (one per CU); each reads BYTES_PER_WG bytes:
//   mode 0: all workgroups read the SAME 1 MiB buffer (L2-resident after the first touch of each
//           XCD) with 16-B buffer loads into registers, DEPTH loads in flight per lane;
//   mode 1: the same reads into LDS with global_load_lds_dwordx4 (LDS-DMA), DEPTH in flight;
//   mode 2: every workgroup streams its own slice of a 1 GiB buffer (HBM), registers;
//   mode 3: mode 2 with LDS-DMA.
// Prints one JSON line per (mode, depth): µs per launch (events over 200 launches) and GB/s per CU.
//
//   hipcc --offload-arch=gfx950 -O3 -o experiments/build/probe_l2_intake experiments/probe_l2_intake.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

template <int DEPTH, bool LDS>
__global__ __launch_bounds__(256) void intake(const uint8_t* src, size_t wg_stride,
                                              uint32_t bytes_per_wg, uint32_t* sink) {
  __shared__ uint4 lds[DEPTH * 256];
  const uint8_t* base = src + (size_t)blockIdx.x * wg_stride;
  const Rsrc r = make_rsrc(base, bytes_per_wg);
  const uint32_t lane_off = threadIdx.x * 16;
  uint32_t acc = 0;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  for (uint32_t off = 0; off < bytes_per_wg; off += DEPTH * 4096) {
    if constexpr (LDS) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(lds + d * 256 + (threadIdx.x & ~63)), 16,
            lane_off, off + d * 4096, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc ^= reinterpret_cast<const uint32_t*>(lds)[threadIdx.x * 4];
    } else {
      u32x4 v[DEPTH];
#pragma unroll
      for (int d = 0; d < DEPTH; ++d)
        v[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, off + d * 4096, 0));
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) acc ^= v[d][0] ^ v[d][3];
    }
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int DEPTH, bool LDS>
static void run(int mode, const uint8_t* small, const uint8_t* big, uint32_t* sink) {
  const int WG = 256;
  const uint32_t bytes = 1u << 20;  // per workgroup
  const bool shared = mode == 0 || mode == 1;
  const uint8_t* src = shared ? small : big;
  const size_t stride = shared ? 0 : (size_t)bytes;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) intake<DEPTH, LDS><<<WG, 256>>>(src, stride, bytes, sink);
  hipEventRecord(a);
  const int iters = 100;
  for (int i = 0; i < iters; ++i) intake<DEPTH, LDS><<<WG, 256>>>(src, stride, bytes, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  printf("{\"mode\": %d, \"lds_dma\": %d, \"depth\": %d, \"us\": %.2f, \"GBps_per_cu\": %.1f, "
         "\"chip_TBps\": %.2f}\n",
         mode, (int)LDS, DEPTH, us, bytes / us / 1e3, (double)bytes * WG / us / 1e6);
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
  for (int mode = 0; mode < 4; ++mode) {
    const bool lds = mode & 1;
    if (lds) {
      run<2, true>(mode, small, big, sink);
      run<4, true>(mode, small, big, sink);
      run<8, true>(mode, small, big, sink);
    } else {
      run<2, false>(mode, small, big, sink);
      run<4, false>(mode, small, big, sink);
      run<8, false>(mode, small, big, sink);
      run<16, false>(mode, small, big, sink);
    }
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
