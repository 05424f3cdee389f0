// One 16-key step of the one-pass decode attention, shared by attn_single_kernel
// (decode_ops.hip) and the attention tail of the one-launch wqkv + attention kernel
// (int4_gemv.hip). Layout: lane (g = lane / 8, p8 = lane % 8) holds the bf16 words of keys t0 + g
// (ka) and t0 + 8 + g (kb2), dims 64 hh + 8 p8 .. + 8 (hh < 2); q in the same dims (qw); vv[j]
// is the dword of dims (2 lane, 2 lane + 1) of key t0 + j. Scores by v_dot2_f32_bf16 reduced over
// the 8 lanes of a key, an online-softmax update of (m, l) and of this lane's two output dims
// (o0, o1), the P.V weights broadcast by v_readlane. `prefetch` runs once the step's K / V
// registers are consumed (scores issued, V converted), so the caller can load the next step into
// the same registers under this step's softmax and P.V.
#pragma once

#include "tao_reduce.h"

namespace tao {

template <class Prefetch>
__device__ __forceinline__ void attn_decode_step(const uint32_t (&qw)[8], const uint4 (&ka)[2],
                                                 const uint4 (&kb2)[2], const uint32_t (&vv)[16],
                                                 int t0, int hi, int g, float scale, float& m,
                                                 float& l, float& o0, float& o1,
                                                 Prefetch&& prefetch) {
  float sa = 0.f, sb = 0.f;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const uint32_t wa[4] = {ka[hh].x, ka[hh].y, ka[hh].z, ka[hh].w};
    const uint32_t wb[4] = {kb2[hh].x, kb2[hh].y, kb2[hh].z, kb2[hh].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sa = dot2_bf16(qw[hh * 4 + e], wa[e], sa);
      sb = dot2_bf16(qw[hh * 4 + e], wb[e], sb);
    }
  }
  float vf[32];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    vf[2 * j] = bf16lo_to_f32(vv[j]);
    vf[2 * j + 1] = bf16hi_to_f32(vv[j]);
  }
  prefetch();
  sa = wave_bfly<1, 8>(sa, lane_id(), [](float a, float c) { return a + c; });
  sb = wave_bfly<1, 8>(sb, lane_id(), [](float a, float c) { return a + c; });
  const bool va = t0 + g < hi, vbk = t0 + 8 + g < hi;
  sa = va ? sa * scale : -INFINITY;
  sb = vbk ? sb * scale : -INFINITY;
  float mx = fmaxf(sa, sb);
  mx = wave_bfly<8, 64>(mx, lane_id(), [](float a, float c) { return fmaxf(a, c); });
  const float mn = fmaxf(m, mx);  // finite: key t0 < hi is valid
  const float corr = __expf(m - mn);
  const float ea = va ? __expf(sa - mn) : 0.f, eb = vbk ? __expf(sb - mn) : 0.f;
  float es = ea + eb;  // each key sits in 8 lanes of one group: xor 8..32 counts it once
  es = wave_bfly<8, 64>(es, lane_id(), [](float a, float c) { return a + c; });
  l = fmaf(l, corr, es);
  o0 *= corr;
  o1 *= corr;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float pa =
        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ea), 8 * j));
    const float pb =
        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, eb), 8 * j));
    o0 = fmaf(pa, vf[2 * j], o0);
    o1 = fmaf(pa, vf[2 * j + 1], o1);
    o0 = fmaf(pb, vf[2 * (j + 8)], o0);
    o1 = fmaf(pb, vf[2 * (j + 8) + 1], o1);
  }
  m = mn;
}

}  // namespace tao
