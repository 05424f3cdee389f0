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
#include <atomic>

#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {
namespace {

// WPE: minimum waves per SIMD the register allocation must allow (8 -> <= 64 VGPRs, so four
// 512-thread workgroups fit on a CU and mid-size grids run in a single resident round).
template <int MT, int RPW, int WPE, bool PAIR>
__global__ __launch_bounds__(512, WPE) void int4wo_gemv_kernel(
    const uint16_t* __restrict__ x, const uint4* __restrict__ wq, const uint32_t* __restrict__ sz,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K, int gshift,
    int Wk, int G, int S) {
  constexpr int V = RPW * MT;
  extern __shared__ float red[];  // [G][Wk][V]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
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

  // PAIR (waves owning >= 2 slices): slices are processed two at a time, both slices' weight
  // and (scale, zero) loads issued before either is consumed, so a wave walking two slices pays
  // one memory round trip, not two.
  auto load_slice = [&](int s, uint4 (&wv)[RPW], uint32_t (&szv)[RPW], int& cc, bool& cval)
      __attribute__((always_inline)) {
    const int c = s * 64 + lane;
    cval = s < S && c < nchunk;
    cc = c < nchunk ? c : nchunk - 1;  // clamped: every load stays in bounds, no branches
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
      const int nn = n < N ? n : N - 1;
      wv[r] = ld_nt_u4(wq + (size_t)nn * nchunk + cc);
      szv[r] = ld_nt(sz + (size_t)nn * ngroups + (cc >> gshift));
    }
  };
  auto do_slice = [&](const uint4 (&wv)[RPW], const uint32_t (&szv)[RPW], int cc, bool cval)
      __attribute__((always_inline)) {
    // Lanes past K contribute nothing: zero their (s, z) so the chunk term vanishes.
    float sc[RPW], zp[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const bool ok = cval && (row0 + r) < N;
      const uint32_t v = ok ? szv[r] : 0u;
      sc[r] = bf16lo_to_f32(v);
      zp[r] = bf16hi_to_f32(v);
    }

    // x is streamed one row of M at a time: 16 live VGPRs whatever M is.
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int mm = m < M ? m : M - 1;
      const uint4* xp = reinterpret_cast<const uint4*>(x + (size_t)mm * K + (size_t)cc * 32);
      uint32_t xd[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 t4 = xp[j];
        xd[j][0] = t4.x;
        xd[j][1] = t4.y;
        xd[j][2] = t4.z;
        xd[j][3] = t4.w;
      }
      float sx = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) sx = dot2_bf16(xd[j][i], 0x3F803F80u, sx);
      const float sx136 = 136.f * sx;
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const uint32_t wd[4] = {wv[r].x, wv[r].y, wv[r].z, wv[r].w};
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) d = dot2_bf16(xd[j][i], nib_pair_bf16(wd[j], i), d);
        acc[r][m] = fmaf(sc[r], d - sx136, fmaf(zp[r], sx, acc[r][m]));
      }
    }
  };

  if constexpr (PAIR) {
    for (int s = wk; s < S; s += 2 * Wk) {
      uint4 wv0[RPW], wv1[RPW];
      uint32_t szv0[RPW], szv1[RPW];
      int cc0, cc1;
      bool cv0, cv1;
      load_slice(s, wv0, szv0, cc0, cv0);
      load_slice(s + Wk, wv1, szv1, cc1, cv1);
      do_slice(wv0, szv0, cc0, cv0);
      if (s + Wk < S) do_slice(wv1, szv1, cc1, cv1);  // wave-uniform
    }
  } else {
    for (int s = wk; s < S; s += Wk) {
      uint4 wv0[RPW];
      uint32_t szv0[RPW];
      int cc0;
      bool cv0;
      load_slice(s, wv0, szv0, cc0, cv0);
      do_slice(wv0, szv0, cc0, cv0);
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

// Launch shape: Wk waves split K inside a workgroup (each loops over its slices), G row
// groups of RPW rows per workgroup; <= 8 waves (512 threads) per workgroup.
struct GemvShape {
  int wk, g;
};

GemvShape default_shape(int S) {
  const int wk = S < 8 ? S : 8;
  const int g = (8 / wk) > 0 ? 8 / wk : 1;
  return {wk, g};
}

template <int MT, int RPW, int WPE>
int launch_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, int gshift,
                GemvShape sh, hipStream_t stream) {
  const int nchunk = K / 32;
  const int S = (nchunk + 63) / 64;
  const int wk = sh.wk < S ? sh.wk : S;
  const int rows_per_wg = sh.g * RPW;
  const int grid = (N + rows_per_wg - 1) / rows_per_wg;
  const int threads = 64 * wk * sh.g;
  const size_t lds = (size_t)sh.g * wk * RPW * MT * sizeof(float);
  if (S > wk)
    launch((int4wo_gemv_kernel<MT, RPW, WPE, true>), dim3(grid), dim3(threads), lds, stream, x,
           reinterpret_cast<const uint4*>(packed), reinterpret_cast<const uint32_t*>(sz), bias,
           y, M, N, K, gshift, wk, sh.g, S);
  else
    launch((int4wo_gemv_kernel<MT, RPW, WPE, false>), dim3(grid), dim3(threads), lds, stream,
           x, reinterpret_cast<const uint4*>(packed), reinterpret_cast<const uint32_t*>(sz),
           bias, y, M, N, K, gshift, wk, sh.g, S);
  return check_launch("int4wo_gemv_kernel");
}

// Process-wide override of the M == 1 launch shape (tao_tune_int4_gemv; 0 = heuristic).
std::atomic<int> g_tune_rpw{0}, g_tune_wk{0}, g_tune_g{0}, g_tune_occ{0};

}  // namespace

// Internal entry (also used by the MFMA dispatcher for small M).
int int4wo_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                int64_t group_size, hipStream_t stream) {
  const int gs = gshift_of(group_size);
  const int S = (int)((K / 32 + 63) / 64);
  GemvShape sh = default_shape(S);
  const int iM = (int)M, iN = (int)N, iK = (int)K;
  if (M <= 1) {
    // Measured on MI355X (experiments/sweep_gemv.py, profiles/r1_sweep_gemv.jsonl): the best
    // shapes per (N, K) class, dispatch-event timed over weights rotated past the MALL.
    int rpw, occ = 8;
    if (S <= 2) {  // K <= 4096
      if (N >= 32768) {
        rpw = 4;
        sh = {2, 2};
      } else if (N >= 8192) {  // one wave walks both slices of 4 rows (PAIR)
        rpw = 4;
        occ = 4;
        sh = {1, N >= 16384 ? 4 : 1};
      } else {
        rpw = 2;
        sh = {2, N <= 4096 ? 1 : 4};
      }
    } else {  // K > 4096: waves split K (each walking its slices in pairs) while N is small
      rpw = 4;
      occ = 4;
      sh = {N <= 4096 ? 2 : (S >= 8 ? 1 : 4), 1};
    }
    const int trpw = g_tune_rpw.load(std::memory_order_relaxed);
    const int tocc = g_tune_occ.load(std::memory_order_relaxed);
    const int twk = g_tune_wk.load(std::memory_order_relaxed);
    const int tg = g_tune_g.load(std::memory_order_relaxed);
    if (trpw > 0) rpw = trpw;
    if (tocc > 0) occ = tocc;
    if (twk > 0) sh.wk = twk;
    if (tg > 0) sh.g = tg;
    if (rpw == 1) return launch_gemv<1, 1, 8>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    if (rpw == 2) return launch_gemv<1, 2, 8>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    if (rpw == 8) return launch_gemv<1, 8, 4>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    if (occ == 4) return launch_gemv<1, 4, 4>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    return launch_gemv<1, 4, 8>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
  }
  if (M <= 2) return launch_gemv<2, 4, 1>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
  if (M <= 4) return launch_gemv<4, 4, 1>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
  return launch_gemv<8, 1, 1>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
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

extern "C" int tao_tune_int4_gemv(int rows_per_wave, int waves_k, int row_groups, int occupancy) {
  TAO_CHECK_ARG(rows_per_wave == 0 || rows_per_wave == 1 || rows_per_wave == 2 ||
                    rows_per_wave == 4 || rows_per_wave == 8,
                "tune: rows_per_wave must be 0 (auto), 1, 2, 4 or 8");
  TAO_CHECK_ARG(waves_k >= 0 && row_groups >= 0 && waves_k * (row_groups ? row_groups : 1) <= 8,
                "tune: waves_k * row_groups must be <= 8");
  TAO_CHECK_ARG(occupancy == 0 || occupancy == 4 || occupancy == 8, "tune: occupancy 0, 4 or 8");
  tao::g_tune_rpw.store(rows_per_wave);
  tao::g_tune_wk.store(waves_k);
  tao::g_tune_g.store(row_groups);
  tao::g_tune_occ.store(occupancy);
  return TAO_OK;
}
