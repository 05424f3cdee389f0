// Probe (not the product path): does the decode GEMV's second stream, the (scale, zero) words in
// their own array beside the packed nibbles, cost HBM efficiency that one interleaved stream of
// the same bytes would not? Loads only, the GEMV's shape (M = 1, K = 4096, g = 32): a workgroup
// of 4 waves, each wave 4 rows x 2 slices; per row and slice one 16-B-per-lane load of nibbles
// (1 KiB) and one 4-B-per-lane load of (scale, zero) words (256 B), non-temporal, all in flight
// before any is consumed. Modes:
//   0  two arrays: nibbles [N][2048 B], words [N][512 B] (the library's layout)
//   1  one array, each row [2048 B nibbles | 512 B words] (interleaved per row)
//   2  nibbles only (no word loads)
//   3  two arrays, the words of a wave's 4 rows in one 16-B-per-lane load per slice (row-quad)
// A value derived from every load is written to `sink` only if it matches a constant no data
// produces, so nothing is dead-code eliminated.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o experiments/build/libprobe2s.so \
//     experiments/probe_two_streams.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldnt4(const uint4* p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint32_t ldnt1(const uint32_t* p) { return __builtin_nontemporal_load(p); }

template <int MODE>
__global__ __launch_bounds__(256) void probe2s(const uint8_t* __restrict__ w,
                                               const uint8_t* __restrict__ s, int N,
                                               uint32_t* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 16 + wave * 4;
  constexpr int kRowW = 2048, kRowS = 512, kRowI = kRowW + kRowS;
  uint4 wv[8];
  uint32_t sv[8];
  uint4 qv[2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int n = row0 + r < N ? row0 + r : N - 1;
      if constexpr (MODE == 1) {
        const uint8_t* rowp = w + (size_t)n * kRowI;
        wv[r * 2 + sl] = ldnt4(reinterpret_cast<const uint4*>(rowp + sl * 1024) + lane);
        sv[r * 2 + sl] = ldnt1(reinterpret_cast<const uint32_t*>(rowp + kRowW + sl * 256) + lane);
      } else {
        wv[r * 2 + sl] = ldnt4(reinterpret_cast<const uint4*>(w + (size_t)n * kRowW + sl * 1024) + lane);
        if constexpr (MODE == 0)
          sv[r * 2 + sl] = ldnt1(reinterpret_cast<const uint32_t*>(s + (size_t)n * kRowS + sl * 256) + lane);
        else
          sv[r * 2 + sl] = 0u;
      }
    }
  if constexpr (MODE == 3) {  // [N / 4][K / 32][4 rows] words: 16 B per lane per slice
    const int q = (row0 < N ? row0 : N - 4) / 4;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
      qv[sl] = ldnt4(reinterpret_cast<const uint4*>(s + (size_t)q * 4 * kRowS + sl * 1024) + lane);
  } else {
    qv[0] = qv[1] = make_uint4(0, 0, 0, 0);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc ^= wv[i].x ^ wv[i].y ^ wv[i].z ^ wv[i].w ^ sv[i];
  acc ^= qv[0].x ^ qv[0].w ^ qv[1].y ^ qv[1].z;
  if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;
}

extern "C" int probe2s_launch(int mode, const void* w, const void* s, int N, void* sink,
                              void* stream) {
  const dim3 grid((unsigned)((N + 15) / 16)), blk(256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint8_t* wb = reinterpret_cast<const uint8_t*>(w);
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s);
  uint32_t* k = reinterpret_cast<uint32_t*>(sink);
  switch (mode) {
    case 0: hipLaunchKernelGGL(probe2s<0>, grid, blk, 0, st, wb, sb, N, k); break;
    case 1: hipLaunchKernelGGL(probe2s<1>, grid, blk, 0, st, wb, sb, N, k); break;
    case 2: hipLaunchKernelGGL(probe2s<2>, grid, blk, 0, st, wb, sb, N, k); break;
    case 3: hipLaunchKernelGGL(probe2s<3>, grid, blk, 0, st, wb, sb, N, k); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
