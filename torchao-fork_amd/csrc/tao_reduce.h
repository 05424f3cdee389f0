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

// Reduce V values per lane across the 64 lanes of a wave. On return v[0] holds, in every lane
// of each aligned group of 64>>T lanes (T = log2 V), the wave-wide total of value index
// lane >> (6 - T). T is float (the bf16/int4 GEMVs) or int (the exact int8 x int8 GEMV).
template <int V, typename T>
__device__ __forceinline__ void wave_reduce_scatter(T (&v)[V], int lane) {
  static_assert(sizeof(T) == 4, "32-bit values");
  constexpr int L = Log2<V>::value;
  static_assert((1 << L) == V && L <= 6, "V must be a power of two <= 64");
  int off = 32;
#pragma unroll
  for (int step = 0; step < L; ++step) {
    const int cur = V >> step;
    const int half = cur >> 1;
    const bool up = (lane & off) != 0;
    // select by bit mask on register values (a select between two array elements can be
    // canonicalised into a dynamically indexed load, which spills the array to scratch)
    const uint32_t m = up ? ~0u : 0u;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const uint32_t a = __builtin_bit_cast(uint32_t, v[i]);
      const uint32_t b = __builtin_bit_cast(uint32_t, v[i + half]);
      const T send = __builtin_bit_cast(T, (a & m) | (b & ~m));
      const T keep = __builtin_bit_cast(T, (b & m) | (a & ~m));
      v[i] = keep + __shfl_xor(send, off, 64);
    }
    off >>= 1;
  }
#pragma unroll
  for (int o = 32 >> L; o > 0; o >>= 1) v[0] += __shfl_xor(v[0], o, 64);
}

}  // namespace tao
