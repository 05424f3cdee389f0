// Wave-level reductions shared by the GEMV kernels. Internal header.
#pragma once

#include "tao_common.h"

namespace tao {

template <int V>
struct Log2 {
  static constexpr int value = (V <= 1) ? 0 : 1 + Log2<(V > 1 ? V / 2 : 1)>::value;
};
template <>
struct Log2<1> {
  static constexpr int value = 0;
};

// The value held by a "partner" lane across bit `off` of the lane index, without the LDS pipe
// (ds_bpermute: ~100+ cycles of latency per step on the reduction's critical path):
//   off 32 / 16: v_permlane32_swap / v_permlane16_swap (gfx950) -> exactly lane ^ off;
//   off 8 / 4:   DPP row_mirror / row_half_mirror -> lane ^ 15 / lane ^ 7 (within the row);
//   off 2 / 1:   DPP quad_perm -> lane ^ 2 / lane ^ 1.
// Every partner has the opposite bit `off`, and taken from high `off` to low the masks
// 32, 16, 15, 7, 2, 1 are each outside the span of the ones before, so a high-to-low butterfly
// over them is still a reduction tree over disjoint lane sets (any fixed order: deterministic).
template <int OFF, typename T>
__device__ __forceinline__ T xor_partner(T v, int lane);

template <int OFF>
__device__ __forceinline__ uint64_t xor_partner64(uint64_t v, int lane) {
  const uint64_t lo = xor_partner<OFF>((uint32_t)v, lane);
  const uint64_t hi = xor_partner<OFF>((uint32_t)(v >> 32), lane);
  return lo | (hi << 32);
}

// TAO_REDUCE_BPERMUTE=1 (timing-only variant builds, experiments/ab_gemv.sh): the same
// exchanges through ds_bpermute (__shfl_xor), the pre-DPP code.
#ifndef TAO_REDUCE_BPERMUTE
#define TAO_REDUCE_BPERMUTE 0
#endif

template <int OFF, typename T>
__device__ __forceinline__ T xor_partner(T v, int lane) {
  if constexpr (sizeof(T) == 8) {
    return xor_partner64<OFF>(v, lane);
  } else if constexpr (TAO_REDUCE_BPERMUTE) {
    (void)lane;
    return __shfl_xor(v, OFF, 64);
  } else {
  static_assert(OFF == 32 || OFF == 16 || OFF == 8 || OFF == 4 || OFF == 2 || OFF == 1, "off");
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  uint32_t r;
  if constexpr (OFF == 32 || OFF == 16) {
    const auto sw = OFF == 32 ? __builtin_amdgcn_permlane32_swap(u, u, false, false)
                              : __builtin_amdgcn_permlane16_swap(u, u, false, false);
    r = (lane & OFF) ? sw[0] : sw[1];
  } else {
    constexpr int kCtl = OFF == 8 ? 0x140 : OFF == 4 ? 0x141 : OFF == 2 ? 0x4E : 0xB1;
    r = (uint32_t)__builtin_amdgcn_mov_dpp((int)u, kCtl, 0xF, 0xF, false);
  }
  return __builtin_bit_cast(T, r);
  }
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// All-reduce over lane bits O, 2 O, ... < END (ascending) with a commutative op. Ascending, the
// lanes are uniform across the lower bits before each mirror step, so DPP row_half_mirror /
// row_mirror give exactly the values xor 4 / xor 8 would: the result is bit-identical to the
// __shfl_xor butterfly in the same (ascending) order.
template <int O, int END, typename T, typename F>
__device__ __forceinline__ T wave_bfly(T x, int lane, F op) {
  x = op(x, xor_partner<O>(x, lane));
  if constexpr (O * 2 < END) return wave_bfly<O * 2, END>(x, lane, op);
  return x;
}
__device__ __forceinline__ float wave_sum(float x) {
  return wave_bfly<1, 64>(x, (int)__lane_id(), [](float a, float b) { return a + b; });
}
__device__ __forceinline__ float wave_max(float x) {
  return wave_bfly<1, 64>(x, (int)__lane_id(), [](float a, float b) { return fmaxf(a, b); });
}
__device__ __forceinline__ float wave_min(float x) {
  return wave_bfly<1, 64>(x, (int)__lane_id(), [](float a, float b) { return fminf(a, b); });
}

// One reduce-scatter step at lane bit OFF over the first CUR values: the lanes with the bit
// keep the upper half, the others the lower half, each adding the partner's copy.
template <int OFF, int CUR, int V, typename T>
__device__ __forceinline__ void rs_step(T (&v)[V], int lane) {
  constexpr int half = CUR >> 1;
  // select by bit mask on register values (a select between two array elements can be
  // canonicalised into a dynamically indexed load, which spills the array to scratch)
  const uint32_t m = (lane & OFF) ? ~0u : 0u;
#pragma unroll
  for (int i = 0; i < half; ++i) {
    const uint32_t a = __builtin_bit_cast(uint32_t, v[i]);
    const uint32_t b = __builtin_bit_cast(uint32_t, v[i + half]);
    const T send = __builtin_bit_cast(T, (a & m) | (b & ~m));
    const T keep = __builtin_bit_cast(T, (b & m) | (a & ~m));
    v[i] = keep + xor_partner<OFF>(send, lane);
  }
  if constexpr (half > 1) rs_step<OFF / 2, half>(v, lane);
}

template <int OFF, typename T>
__device__ __forceinline__ void bfly(T& x, int lane) {
  x += xor_partner<OFF>(x, lane);
  if constexpr (OFF > 1) bfly<OFF / 2>(x, lane);
}

// Reduce V values per lane across the 64 lanes of a wave. On return v[0] holds, in every lane
// of each aligned group of 64>>T lanes (T = log2 V), the wave-wide total of value index
// lane >> (6 - T). T is float (the bf16/int4 GEMVs) or int (the exact int8 x int8 GEMV).
// Exchanges go through xor_partner (no LDS pipe).
template <int V, typename T>
__device__ __forceinline__ void wave_reduce_scatter(T (&v)[V], int lane) {
  static_assert(sizeof(T) == 4, "32-bit values");
  constexpr int L = Log2<V>::value;
  static_assert((1 << L) == V && L <= 6, "V must be a power of two <= 64");
  if constexpr (V > 1) rs_step<32, V>(v, lane);
  if constexpr (L < 6) bfly<(32 >> L)>(v[0], lane);
}

}  // namespace tao
