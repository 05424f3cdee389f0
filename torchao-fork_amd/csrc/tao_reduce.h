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
// lane >> (6 - T).
template <int V>
__device__ __forceinline__ void wave_reduce_scatter(float (&v)[V], int lane) {
  constexpr int T = Log2<V>::value;
  static_assert((1 << T) == V && T <= 6, "V must be a power of two <= 64");
  int off = 32;
#pragma unroll
  for (int step = 0; step < T; ++step) {
    const int cur = V >> step;
    const int half = cur >> 1;
    const bool up = (lane & off) != 0;
    // select by bit mask on register values (a select between two array elements can be
    // canonicalised into a dynamically indexed load, which spills the array to scratch)
    const uint32_t m = up ? ~0u : 0u;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const uint32_t a = __float_as_uint(v[i]), b = __float_as_uint(v[i + half]);
      const float send = __uint_as_float((a & m) | (b & ~m));
      const float keep = __uint_as_float((b & m) | (a & ~m));
      v[i] = keep + __shfl_xor(send, off, 64);
    }
    off >>= 1;
  }
#pragma unroll
  for (int o = 32 >> T; o > 0; o >>= 1) v[0] += __shfl_xor(v[0], o, 64);
}

}  // namespace tao
