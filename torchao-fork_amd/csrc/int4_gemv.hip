// int4 group-quantised weight-only linear, skinny-M (decode) path: y[M][N] = x[M][K] W^T.
//
// Replaces aten._weight_int4pack_mm at torchao/dtypes/uintx/tensor_core_tiled_layout.py:104
// for M <= 8. HBM-bound: every packed weight byte and every (scale, zero) pair is read exactly
// once, with 16-B non-temporal loads; x (<= 8 x K bf16) stays in L1/L2.
//
// Work decomposition:
//   * a "slice" is 2048 consecutive k of one row = 64 lanes x 32 k = one 1-KiB wave load
//     (16 B of nibbles per lane) + one 256-B (scale, zero) load at group size 32;
//   * a wave owns RPW rows and one slice at a time; a workgroup is G row-groups x Wk waves along
//     K (Wk = min(slices, 8)); slices beyond Wk are looped;
//   * per lane: D = sum x*(128+q) via v_dot2c_f32_bf16 on magic-number bf16 pairs
//     (one v_and_or_b32 per 2 weights), Sx = sum x, then s*(D - 136 Sx) + z*Sx per 32-k chunk —
//     every 32-k chunk lies in exactly one quantisation group because g in {32..256};
//   * cross-lane: reduce-scatter over the RPW*M partials (V/2 + V/4 + ... shuffles), then a
//     butterfly over the remaining lanes; cross-wave: LDS, one wave finishes and writes y.
#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {
namespace {

template <int MT, int RPW>
__global__ __launch_bounds__(512) void int4wo_gemv_kernel(
    const uint16_t* __restrict__ x, const uint4* __restrict__ wq, const uint32_t* __restrict__ sz,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K, int gshift,
    int Wk, int G, int S) {
  constexpr int V = RPW * MT;
  extern __shared__ float red[];  // [G][Wk][V]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wk = wave % Wk;
  const int rg = wave / Wk;
  const int row0 = (blockIdx.x * G + rg) * RPW;
  const int nchunk = K >> 5;               // 32-k chunks per row
  const int ngroups = K >> (5 + gshift);   // quantisation groups per row

  float acc[RPW][MT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;

  for (int s = wk; s < S; s += Wk) {
    const int c = s * 64 + lane;
    const bool cval = c < nchunk;
    const int cc = cval ? c : nchunk - 1;  // clamped: every load stays in bounds, no branches

    uint4 wv[RPW];
    uint32_t szv[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
      const int nn = n < N ? n : N - 1;
      wv[r] = ld_nt_u4(wq + (size_t)nn * nchunk + cc);
      szv[r] = ld_nt(sz + (size_t)nn * ngroups + (cc >> gshift));
    }
    uint4 xv[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int mm = m < M ? m : M - 1;
      const uint4* xp = reinterpret_cast<const uint4*>(x + (size_t)mm * K + (size_t)cc * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[m][j] = xp[j];
    }
    // Lanes past K contribute nothing: zero their (s, z) so the chunk term vanishes.
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const bool ok = cval && (row0 + r) < N;
      szv[r] = ok ? szv[r] : 0u;
    }

    float sx[MT], sx136[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t = dot2_bf16(xv[m][j].x, 0x3F803F80u, t);
        t = dot2_bf16(xv[m][j].y, 0x3F803F80u, t);
        t = dot2_bf16(xv[m][j].z, 0x3F803F80u, t);
        t = dot2_bf16(xv[m][j].w, 0x3F803F80u, t);
      }
      sx[m] = t;
      sx136[m] = 136.f * t;
    }

#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const float sc = bf16lo_to_f32(szv[r]);
      const float zp = bf16hi_to_f32(szv[r]);
      const uint32_t wd[4] = {wv[r].x, wv[r].y, wv[r].z, wv[r].w};
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const uint32_t xd[4][4] = {{xv[m][0].x, xv[m][0].y, xv[m][0].z, xv[m][0].w},
                                   {xv[m][1].x, xv[m][1].y, xv[m][1].z, xv[m][1].w},
                                   {xv[m][2].x, xv[m][2].y, xv[m][2].z, xv[m][2].w},
                                   {xv[m][3].x, xv[m][3].y, xv[m][3].z, xv[m][3].w}};
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) d = dot2_bf16(xd[j][i], nib_pair_bf16(wd[j], i), d);
        acc[r][m] = fmaf(sc, d - sx136[m], fmaf(zp, sx[m], acc[r][m]));
      }
    }
  }

  float v[V];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) v[r * MT + m] = acc[r][m];
  wave_reduce_scatter<V>(v, lane);

  constexpr int T = Log2<V>::value;
  const bool owner = (lane & ((64 >> T) - 1)) == 0;
  const int idx = lane >> (6 - T);

  float total = v[0];
  bool writer = owner;
  int widx = idx;
  if (Wk > 1) {
    if (owner) red[(rg * Wk + wk) * V + idx] = v[0];
    __syncthreads();
    writer = (wk == 0) && (lane < V);
    widx = lane;
    if (writer) {
      total = 0.f;
      for (int kk = 0; kk < Wk; ++kk) total += red[(rg * Wk + kk) * V + widx];
    }
  }
  if (writer) {
    const int r = widx / MT, m = widx % MT;
    const int n = row0 + r;
    if (n < N && m < M) {
      uint16_t out = f32_to_bf16(total);
      if (bias != nullptr) out = f32_to_bf16(bf16_to_f32(out) + bf16_to_f32(bias[n]));
      y[(size_t)m * N + n] = out;
    }
  }
}

int gshift_of(int64_t g) {
  switch (g) {
    case 32: return 0;
    case 64: return 1;
    case 128: return 2;
    case 256: return 3;
    default: return -1;
  }
}

template <int MT, int RPW>
int launch_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, int gshift,
                hipStream_t stream) {
  const int nchunk = K / 32;
  const int S = (nchunk + 63) / 64;
  const int Wk = S < 8 ? S : 8;
  const int G = (8 / Wk) > 0 ? 8 / Wk : 1;
  const int rows_per_wg = G * RPW;
  const int grid = (N + rows_per_wg - 1) / rows_per_wg;
  const int threads = 64 * Wk * G;
  const size_t lds = (size_t)G * Wk * RPW * MT * sizeof(float);
  launch((int4wo_gemv_kernel<MT, RPW>), dim3(grid), dim3(threads), lds, stream, x,
                     reinterpret_cast<const uint4*>(packed),
                     reinterpret_cast<const uint32_t*>(sz), bias, y, M, N, K, gshift, Wk, G, S);
  return check_launch("int4wo_gemv_kernel");
}

}  // namespace

// Internal entry (also used by the MFMA dispatcher for small M).
int int4wo_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                int64_t group_size, hipStream_t stream) {
  const int gs = gshift_of(group_size);
  if (M <= 1) return launch_gemv<1, 4>(x, packed, sz, bias, y, (int)M, (int)N, (int)K, gs, stream);
  if (M <= 2) return launch_gemv<2, 4>(x, packed, sz, bias, y, (int)M, (int)N, (int)K, gs, stream);
  if (M <= 4) return launch_gemv<4, 4>(x, packed, sz, bias, y, (int)M, (int)N, (int)K, gs, stream);
  return launch_gemv<8, 2>(x, packed, sz, bias, y, (int)M, (int)N, (int)K, gs, stream);
}

int int4_check_linear_args(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                           uint16_t* y, int64_t M, int64_t N, int64_t K, int64_t group_size) {
  TAO_CHECK_ARG(gshift_of(group_size) >= 0,
                "int4 linear: qGroupSize must be 32, 64, 128, or 256 (got %lld)",
                (long long)group_size);
  TAO_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "int4 linear: negative size");
  TAO_CHECK_ARG(K % group_size == 0, "int4 linear: K (%lld) %% group_size (%lld) != 0",
                (long long)K, (long long)group_size);
  TAO_CHECK_ARG(N < (1LL << 31) && K < (1LL << 31) && M < (1LL << 31) &&
                    (N * (K / 8)) < (1LL << 40),
                "int4 linear: size out of range");
  if (M == 0 || N == 0) return TAO_OK;
  TAO_CHECK_ARG(K > 0, "int4 linear: K must be > 0");
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(packed, 16, "packed weight");
  TAO_CHECK_ALIGN(sz, 4, "scales_and_zeros");
  TAO_CHECK_ALIGN(y, 2, "y");
  return TAO_OK;
}

}  // namespace tao
