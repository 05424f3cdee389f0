// int8 per-channel weight-only linear, skinny-M (decode) path:
//   y[m][n] = bf16( bf16( sum_k x[m][k] * w[n][k] ) * scale[n] ) (+ bias[n])
// Replaces torch.mm(x, w.t().to(bf16)) * scale at torchao/dtypes/uintx/plain_layout.py:256-266,
// which materialises a bf16 copy of W (2x the bytes) before a library GEMM; here W is read once.
//
// Same decomposition as int4_gemv.hip: a slice is 1024 k of one row = 64 lanes x 16 B (int8);
// a wave owns RPW rows; Wk waves split K inside a workgroup; LDS combines the waves.
// Per lane: bytes are biased to unsigned (xor 0x80), converted with v_cvt_f32_ubyte{0..3} and
// FMA'd against x in f32; the bias is removed once per chunk as 128 * sum(x).
#include <atomic>

#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {


namespace {

template <int MT, int RPW>
__global__ __launch_bounds__(512) void int8wo_gemv_kernel(
    const uint16_t* __restrict__ x, const uint4* __restrict__ w,
    const uint16_t* __restrict__ scale, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int Wk, int G, int S) {
  constexpr int V = RPW * MT;
  extern __shared__ float red[];  // [G][Wk][V]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int wk = wave % Wk;
  const int rg = wave / Wk;
  const int row0 = (blockIdx.x * G + rg) * RPW;
  const int nchunk = K >> 4;  // 16-k (16-B) chunks per row

  float acc[RPW][MT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;

  for (int s = wk; s < S; s += Wk) {
    const int c = s * 64 + lane;
    const bool cval = c < nchunk;
    const int cc = cval ? c : nchunk - 1;

    uint4 wv[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
      const int nn = n < N ? n : N - 1;
      wv[r] = ld_nt_u4(w + (size_t)nn * nchunk + cc);
    }
    // x is streamed one row of M at a time: 16 live f32 values whatever M is.
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int mm = m < M ? m : M - 1;
      const uint4* xp = reinterpret_cast<const uint4*>(x + (size_t)mm * K + (size_t)cc * 16);
      const uint4 a = xp[0], b = xp[1];
      const uint32_t d8[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      float xf[16];
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t di = cval ? d8[i] : 0u;
        xf[2 * i] = bf16lo_to_f32(di);
        xf[2 * i + 1] = bf16hi_to_f32(di);
        t = dot2_bf16(di, 0x3F803F80u, t);
      }
      const float sx128 = 128.f * t;
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const uint32_t wd[4] = {wv[r].x ^ 0x80808080u, wv[r].y ^ 0x80808080u,
                                wv[r].z ^ 0x80808080u, wv[r].w ^ 0x80808080u};
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          d = fmaf(xf[4 * j + 0], (float)(wd[j] & 0xFF), d);
          d = fmaf(xf[4 * j + 1], (float)((wd[j] >> 8) & 0xFF), d);
          d = fmaf(xf[4 * j + 2], (float)((wd[j] >> 16) & 0xFF), d);
          d = fmaf(xf[4 * j + 3], (float)(wd[j] >> 24), d);
        }
        acc[r][m] += d - sx128;
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
      // bf16 mm output, then bf16 * scale, then + bias: the reference's three roundings.
      float o = round_bf16(round_bf16(total) * bf16_to_f32(scale[n]));
      if (bias != nullptr) o = round_bf16(o + bf16_to_f32(bias[n]));
      y[(size_t)m * N + n] = f32_to_bf16(o);
    }
  }
}

template <int MT, int RPW>
int launch_gemv(const uint16_t* x, const int8_t* w, const uint16_t* scale, const uint16_t* bias,
                uint16_t* y, int M, int N, int K, hipStream_t stream, int wk = 0, int g = 0) {
  const int nchunk = K / 16;
  const int S = (nchunk + 63) / 64;
  int Wk = S < 8 ? S : 8;
  int G = (8 / Wk) > 0 ? 8 / Wk : 1;
  if (wk > 0) Wk = wk < S ? wk : S;
  if (g > 0) G = g;
  const int rows_per_wg = G * RPW;
  const int grid = (N + rows_per_wg - 1) / rows_per_wg;
  const size_t lds = (size_t)G * Wk * RPW * MT * sizeof(float);
  launch((int8wo_gemv_kernel<MT, RPW>), dim3(grid), dim3(64 * Wk * G), lds, stream,
                     x, reinterpret_cast<const uint4*>(w), scale, bias, y, M, N, K, Wk, G, S);
  return check_launch("int8wo_gemv_kernel");
}

}  // namespace

int int8wo_gemv(const uint16_t* x, const int8_t* w, const uint16_t* scale, const uint16_t* bias,
                uint16_t* y, int64_t M, int64_t N, int64_t K, hipStream_t stream) {
  if (M <= 1) {
    const int rpw = tao::tuning().i8_rpw;
    // one row group per workgroup at M == 1 (experiments/sweep_int8.py,
    // profiles/r1_sweep_int8.jsonl: 4 rows per wave, Wk = min(S, 8), G = 1 is within 1% of the
    // per-shape best on every Llama-3-8B linear; the head 77.8 -> 72.7 us)
    const int wk = tao::tuning().i8_wk;
    const int tg = tao::tuning().i8_g, g = tg > 0 ? tg : 1;
    if (rpw == 2)
      return launch_gemv<1, 2>(x, w, scale, bias, y, (int)M, (int)N, (int)K, stream, wk, g);
    if (rpw == 8)
      return launch_gemv<1, 8>(x, w, scale, bias, y, (int)M, (int)N, (int)K, stream, wk, g);
    return launch_gemv<1, 4>(x, w, scale, bias, y, (int)M, (int)N, (int)K, stream, wk, g);
  }
  if (M <= 2) return launch_gemv<2, 4>(x, w, scale, bias, y, (int)M, (int)N, (int)K, stream);
  if (M <= 4) return launch_gemv<4, 2>(x, w, scale, bias, y, (int)M, (int)N, (int)K, stream);
  return launch_gemv<8, 1>(x, w, scale, bias, y, (int)M, (int)N, (int)K, stream);
}

}  // namespace tao
