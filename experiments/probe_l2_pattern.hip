// Per-CU intake of a [64 rows][4096 B] tile (a prefill GEMM's weight tile, row stride 4 KiB) by
// 16-B buffer loads into registers, by load pattern: does an instruction that covers only half
// of each 128-B line it touches (the MFMA fragment order: 16 rows x 64 B) cost intake?
// 256 workgroups (one per CU) x 8 waves, each workgroup reading its tile REPS times, DEPTH loads
// in flight per lane:
//   pattern 0: 1 KiB contiguous per instruction (rows in order, lane l: bytes 16 l of a row run);
//   pattern 1: 8 rows x 128 B per instruction (lane l: row l / 8, bytes 16 (l % 8));
//   pattern 2: 16 rows x 64 B per instruction, the wave's two consecutive instructions covering
//              the two halves of the same 16 lines;
//   pattern 3: 16 rows x 64 B per instruction, 64-B blocks interleaved over the waves (wave w
//              takes blocks w, w + 8, ...: the k-split GEMM's order).
// shared 1: every workgroup reads the same tile (L2-resident); shared 0: 4 workgroups per tile,
// on one XCD as the GEMM's M tiles are (tile = blockIdx % 64).
//
//   hipcc --offload-arch=gfx950 -O3 -o experiments/build/probe_l2_pattern experiments/probe_l2_pattern.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

constexpr int kRows = 64, kRowB = 4096, kTile = kRows * kRowB;  // 256 KiB

// offset of load number i (0 .. kTile / 16 / 512 - 1 = 31 per lane of an 8-wave workgroup)
template <int PAT>
__device__ __forceinline__ uint32_t off(int i, int wave, int lane) {
  if constexpr (PAT == 0) {  // instruction = 1 KiB run; wave w: runs w, w + 8, ...
    const int run = wave + 8 * i;
    return (uint32_t)run * 1024u + 16u * lane;
  } else if constexpr (PAT == 1) {  // instruction = 8 rows x 128 B
    const int blk = wave + 8 * i;   // 0..255: (row group of 8) x (128-B column) = 8 x 32
    const int rg = blk & 7, col = blk >> 3;
    return (uint32_t)(rg * 8 + (lane >> 3)) * kRowB + (uint32_t)col * 128u + 16u * (lane & 7);
  } else if constexpr (PAT == 2) {  // 16 rows x 64 B, halves back to back in the wave
    const int blk = wave + 8 * (i >> 1);  // 0..127: (row group of 16) x (128-B column) = 4 x 32
    const int rg = blk & 3, col = blk >> 2, h = i & 1;
    return (uint32_t)(rg * 16 + (lane & 15)) * kRowB + (uint32_t)col * 128u + 64u * h +
           16u * (lane >> 4);
  } else {  // 16 rows x 64 B, 64-B blocks interleaved over the waves
    const int blk = wave + 8 * i;   // 0..255: (row group of 16) x (64-B column) = 4 x 64
    const int rg = blk & 3, col = blk >> 2;
    return (uint32_t)(rg * 16 + (lane & 15)) * kRowB + (uint32_t)col * 64u + 16u * (lane >> 4);
  }
}

template <int PAT, int DEPTH>
__global__ __launch_bounds__(512) void intake(const uint8_t* src, int shared, int reps,
                                              uint32_t* sink, int call) {
  // shared 2: as 0, the tiles rotating over 1 GiB from call to call (HBM, past the MALL)
  const int tile = shared == 1 ? 0 : (blockIdx.x & 63) + (shared == 2 ? 64 * (call & 63) : 0);
  const Rsrc r = make_rsrc(src + (size_t)tile * kTile, kTile);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  constexpr int kN = kTile / 16 / 512;  // 32 loads per lane per pass
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
    for (int i0 = 0; i0 < kN; i0 += DEPTH) {
      u32x4 v[DEPTH];
#pragma unroll
      for (int d = 0; d < DEPTH; ++d)
        v[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             r, off<PAT>(i0 + d, wave, lane), 0, 0));
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) acc ^= v[d][0] ^ v[d][3];
    }
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int PAT, int DEPTH>
static void run(int shared, const uint8_t* buf, uint32_t* sink) {
  const int WG = 256, reps = shared == 2 ? 1 : 4;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) intake<PAT, DEPTH><<<WG, 512>>>(buf, shared, reps, sink, i);
  hipEventRecord(a);
  const int iters = 100;
  for (int i = 0; i < iters; ++i) intake<PAT, DEPTH><<<WG, 512>>>(buf, shared, reps, sink, i);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double bytes = (double)kTile * reps;
  printf("{\"pattern\": %d, \"shared\": %d, \"depth\": %d, \"us\": %.2f, \"GBps_per_cu\": %.1f}\n",
         PAT, shared, DEPTH, us, bytes / us / 1e3);
  fflush(stdout);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

template <int PAT>
static void pat(const uint8_t* buf, uint32_t* sink) {
  for (int sh = 2; sh >= 0; --sh) {
    run<PAT, 4>(sh, buf, sink);
    run<PAT, 8>(sh, buf, sink);
  }
}

int main() {
  uint8_t* buf = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(&buf, (size_t)4096 * kTile) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess)
    return 1;
  hipMemset(buf, 1, (size_t)4096 * kTile);
  pat<0>(buf, sink);
  pat<1>(buf, sink);
  pat<2>(buf, sink);
  pat<3>(buf, sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
