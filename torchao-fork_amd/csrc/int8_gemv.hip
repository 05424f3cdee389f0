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

TAO_DECODE_ERROR_WORD(int8gemv_decode_status)

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

// ---- decode-step fusions of the M == 1 int8 weight-only GEMV (tao_int8wo_decode_bf16) -------
// The int4 decode kernel's fusions (int4_gemv.hip) on the int8 weight stream, so
// an int8wo Llama layer is 5 launches per token, as with int4 weights, instead of 9:
//   PRO (NPT > 0)  x -> bf16(bf16(x * rsqrt(mean(x^2) + eps)) * norm_w), normalised once per
//                  workgroup into LDS while the first weight slice is in flight;
//   kI8EpiSwiGLU   rows (2i, 2i+1) = (w1_i, w3_i): y[i] = bf16(bf16(silu(a)) * b);
//   kI8EpiRopeKV   rows = [q | k | v] heads: q rotated into y, k rotated and v stored into the
//                  caches at pos[0] (a position outside [0, T) is reported, no cache row written).
// a and b are the linear's own outputs bf16(bf16(sum) * scale[n]), so every result equals the
// unfused chain (rmsnorm_kernel -> int8wo_gemv_kernel -> silu_mul / rope_kv) bit for bit, up to
// the norm's fp32 sum order.
enum { kI8EpiNone = 0, kI8EpiSwiGLU = 1, kI8EpiRopeKV = 2 };
struct I8Fuse {
  const uint16_t* norm_w;
  float eps;
  const float* freqs;  // [T][D/2] (cos, sin)
  const int64_t* pos;
  uint16_t* k_cache;  // [Hkv][T][D]
  uint16_t* v_cache;
  int H, Hkv, D, T;
};

__device__ __forceinline__ uint32_t i8_rmsnorm_pair(uint32_t xv, uint32_t wv, float r) {
  const float lo = round_bf16(bf16lo_to_f32(xv) * r) * bf16lo_to_f32(wv);
  const float hi = round_bf16(bf16hi_to_f32(xv) * r) * bf16hi_to_f32(wv);
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

template <int RPW, int NPT, int EPI>
__global__ __launch_bounds__(512) void int8wo_decode_kernel(
    const uint16_t* __restrict__ x, const uint4* __restrict__ w,
    const uint16_t* __restrict__ scale, uint16_t* __restrict__ y, int N, int K, int Wk, int G,
    int S, I8Fuse fu) {
  constexpr bool PRO = NPT > 0;
  constexpr int V = RPW;
  static_assert(RPW % 2 == 0, "row pairs stay inside one wave");
  // [G][Wk][V] partials | [16] wave sums of squares | (PRO) normalised x [K / 8] uint4
  extern __shared__ float red[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wk = wave % Wk;
  const int rg = wave / Wk;
  const int row0 = (blockIdx.x * G + rg) * RPW;
  const int nchunk = K >> 4;
  const int nx = K >> 3;
  float* ssr = red + G * Wk * V;
  uint4* xs = reinterpret_cast<uint4*>(red + ((G * Wk * V + 16 + 3) & ~3));

  uint4 xv[PRO ? NPT : 1], gv[PRO ? NPT : 1];
  if constexpr (PRO) {  // x and the norm weight first: their vmcnt wait does not wait for W
    const uint4* xr = reinterpret_cast<const uint4*>(x);
    const uint4* gr = reinterpret_cast<const uint4*>(fu.norm_w);
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      const int ic = i < nx ? i : nx - 1;
      xv[u] = xr[ic];
      gv[u] = gr[ic];
    }
  }
  uint4 wv[RPW];
  auto load_w = [&](int s) __attribute__((always_inline)) {
    const int c = s * 64 + lane;
    const int cc = c < nchunk ? c : nchunk - 1;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
      wv[r] = ld_nt_u4(w + (size_t)(n < N ? n : N - 1) * nchunk + cc);
    }
  };
  load_w(wk);  // Wk <= S: every wave owns a slice
  if constexpr (PRO) {
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const bool ok = threadIdx.x + u * (int)blockDim.x < nx;
      const uint32_t d[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = ok ? bf16lo_to_f32(d[j]) : 0.f, b = ok ? bf16hi_to_f32(d[j]) : 0.f;
        ss = fmaf(a, a, fmaf(b, b, ss));
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) ssr[wave] = ss;
    __syncthreads();
    float t = 0.f;
    for (int q = 0; q < G * Wk; ++q) t += ssr[q];
    const float r = rsqrtf(t / (float)K + fu.eps);
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      // piece i of 16-k chunk c = i >> 1 lands at 2 c + ((i + (c >> 3)) & 1): consecutive lanes
      // read 32-B chunks, the rotation puts the two halves of a pass on distinct bank groups
      if (i < nx)
        xs[(i & ~1) | ((i + (i >> 4)) & 1)] =
            make_uint4(i8_rmsnorm_pair(xv[u].x, gv[u].x, r), i8_rmsnorm_pair(xv[u].y, gv[u].y, r),
                       i8_rmsnorm_pair(xv[u].z, gv[u].z, r), i8_rmsnorm_pair(xv[u].w, gv[u].w, r));
    }
    __syncthreads();
  }

  float acc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) acc[r] = 0.f;
  for (int s = wk; s < S; s += Wk) {
    if (s != wk) load_w(s);
    const int c = s * 64 + lane;
    const bool cval = c < nchunk;
    const int cc = cval ? c : nchunk - 1;
    uint4 a, b;
    if constexpr (PRO) {
      const int rot = (cc >> 3) & 1;
      a = xs[2 * cc + rot];
      b = xs[2 * cc + (rot ^ 1)];
    } else {
      const uint4* xp = reinterpret_cast<const uint4*>(x + (size_t)cc * 16);
      a = xp[0];
      b = xp[1];
    }
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
      acc[r] += d - sx128;
    }
  }

  float v[V];
#pragma unroll
  for (int r = 0; r < RPW; ++r) v[r] = acc[r];
  wave_reduce_scatter<V>(v, lane);
  constexpr int T = Log2<V>::value;
  const bool owner = (lane & ((64 >> T) - 1)) == 0;
  float total = v[0];
  int widx = lane >> (6 - T);  // the row this lane's total belongs to (owner lanes)
  if (Wk > 1) {
    if (owner) red[(rg * Wk + wk) * V + widx] = v[0];
    __syncthreads();
    widx = lane;
    if (wk == 0 && lane < V) {
      total = 0.f;
      for (int kk = 0; kk < Wk; ++kk) total += red[(rg * Wk + kk) * V + lane];
    }
  }
  // the linear's bf16 output of row widx (bf16 mm, then * scale, as int8wo_gemv_kernel)
  const int nrow = row0 + (widx < V ? widx : 0);
  const float o = round_bf16(round_bf16(total) * bf16_to_f32(scale[nrow < N ? nrow : N - 1]));
  if constexpr (EPI == kI8EpiNone) {
    const bool writer = Wk > 1 ? (wk == 0 && lane < V) : owner;
    if (writer && row0 + widx < N) y[row0 + widx] = f32_to_bf16(o);
  } else {
    // row pair (2p, 2p+1) meets in lane p (every lane takes part in the shuffles)
    const int sh = Wk > 1 ? 0 : 6 - T;
    const int pl = lane < RPW / 2 ? lane : 0;
    const float ea = __shfl(o, (2 * pl) << sh);
    const float eb = __shfl(o, (2 * pl + 1) << sh);
    const int n = row0 + 2 * pl;
    if ((Wk == 1 || wk == 0) && lane < RPW / 2 && n < N) {
      if constexpr (EPI == kI8EpiSwiGLU) {
        y[n >> 1] = f32_to_bf16(round_bf16(ea / (1.f + __expf(-ea))) * eb);
      } else {
        const int D = fu.D, HD = fu.H * fu.D, KD = fu.Hkv * fu.D;
        int64_t p = fu.pos[0];
        const bool pok = p >= 0 && p < fu.T;
        if (!pok) {
          flag_decode_error(kDecodeErrKvPos);
          p = p < 0 ? 0 : fu.T - 1;
        }
        uint32_t ov = (uint32_t)f32_to_bf16(ea) | ((uint32_t)f32_to_bf16(eb) << 16);
        if (n < HD + KD) {
          const float2 cs = reinterpret_cast<const float2*>(fu.freqs)[p * (D >> 1) + ((n % D) >> 1)];
          const float o0 = ea * cs.x - eb * cs.y, o1 = eb * cs.x + ea * cs.y;
          ov = (uint32_t)f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
        }
        if (n < HD) {
          reinterpret_cast<uint32_t*>(y)[n >> 1] = ov;
        } else if (pok) {
          const int nk = n < HD + KD ? n - HD : n - HD - KD;
          uint16_t* cache = n < HD + KD ? fu.k_cache : fu.v_cache;
          const size_t off = ((size_t)(nk / D) * fu.T + p) * D + nk % D;
          reinterpret_cast<uint32_t*>(cache)[off >> 1] = ov;
        }
      }
    }
  }
}

template <int RPW, int NPT, int EPI>
int launch_i8_decode(const uint16_t* x, const int8_t* w, const uint16_t* scale, uint16_t* y, int N,
                     int K, int wk, int g, hipStream_t stream, const I8Fuse& fu) {
  const int S = (K / 16 + 63) / 64;
  const int Wk = wk < S ? wk : S;
  const int threads = 64 * Wk * g;
  const int grid = (N + g * RPW - 1) / (g * RPW);
  const size_t lds = (((size_t)g * Wk * RPW + 16 + 3) & ~(size_t)3) * sizeof(float) +
                     (NPT > 0 ? (size_t)K * 2 : 0);
  launch((int8wo_decode_kernel<RPW, NPT, EPI>), dim3(grid), dim3(threads), lds, stream, x,
         reinterpret_cast<const uint4*>(w), scale, y, N, K, Wk, g, S, fu);
  return check_launch("int8wo_decode_kernel");
}

template <int EPI>
int i8_decode(const uint16_t* x, const int8_t* w, const uint16_t* scale, uint16_t* y, int N, int K,
              hipStream_t stream, const I8Fuse& fu) {
  const int S = (K / 16 + 63) / 64;
  // launch shape: Wk = min(S, 4) waves along K, G row groups, RPW rows per wave (tao_tune_int8_gemv
  // overrides); the prologue needs K <= 8 x NPT x threads
  const int trpw = tuning().i8_rpw, twk = tuning().i8_wk, tg = tuning().i8_g;
  const int wk = twk > 0 ? twk : (S < 4 ? S : 4);
  int g = tg > 0 ? tg : 2;
  const int wke = wk < S ? wk : S;
  while (wke * g < 8 && 64 * wke * g * 8 * 4 < K) g *= 2;
  while (g > 1 && wke * g > 8) g /= 2;  // __launch_bounds__(512) and the prologue's 16 slots
  const int threads = 64 * wke * g;
  if (threads > 512)
    return set_error(TAO_ERR_INVALID_ARGUMENT, "int8 decode: %d waves along K exceed 8", wke);
  const bool pro = fu.norm_w != nullptr;
  if (pro && threads * 8 * 4 < K)
    return set_error(TAO_ERR_INVALID_ARGUMENT, "int8 decode: K (%d) too long for the RMSNorm prologue", K);
  const int npt = !pro ? 0 : (threads * 8 >= K ? 1 : threads * 8 * 2 >= K ? 2 : 4);
#define TAO_I8D(R, P) return launch_i8_decode<R, P, EPI>(x, w, scale, y, N, K, wk, g, stream, fu)
  if (trpw == 8) {
    if (npt == 0) TAO_I8D(8, 0);
    if (npt == 1) TAO_I8D(8, 1);
    if (npt == 2) TAO_I8D(8, 2);
    TAO_I8D(8, 4);
  }
  if (trpw == 2) {
    if (npt == 0) TAO_I8D(2, 0);
    if (npt == 1) TAO_I8D(2, 1);
    if (npt == 2) TAO_I8D(2, 2);
    TAO_I8D(2, 4);
  }
  if (npt == 0) TAO_I8D(4, 0);
  if (npt == 1) TAO_I8D(4, 1);
  if (npt == 2) TAO_I8D(4, 2);
  TAO_I8D(4, 4);
#undef TAO_I8D
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

extern "C" int tao_int8wo_decode_bf16(const uint16_t* x, const int8_t* w, const uint16_t* scale,
                                      int64_t N, int64_t K, const uint16_t* norm_weight,
                                      float eps, int epilogue, uint16_t* y, const float* freqs,
                                      const int64_t* pos, uint16_t* k_cache, uint16_t* v_cache,
                                      int64_t n_head, int64_t n_kv_head, int64_t head_dim,
                                      int64_t max_seq, void* stream) {
  using namespace tao;
  TAO_CHECK_ARG(N >= 0 && K > 0 && K % 16 == 0 && N < (1LL << 31) && K < (1LL << 31),
                "int8 decode: K (%lld) must be a positive multiple of 16", (long long)K);
  TAO_CHECK_ARG(epilogue >= kI8EpiNone && epilogue <= kI8EpiRopeKV,
                "int8 decode: epilogue must be 0 (none), 1 (swiglu) or 2 (rope_kv)");
  TAO_CHECK_ARG(epilogue == kI8EpiNone || N % 2 == 0, "int8 decode: N (%lld) must be even",
                (long long)N);
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(y, 2, "y");
  I8Fuse fu{};
  fu.norm_w = norm_weight;
  fu.eps = eps;
  if (norm_weight != nullptr) TAO_CHECK_ALIGN(norm_weight, 16, "norm_weight");
  if (epilogue == kI8EpiRopeKV) {
    TAO_CHECK_ARG(n_head > 0 && n_kv_head > 0 && head_dim > 0 && head_dim % 2 == 0 &&
                      max_seq > 0 && N == (n_head + 2 * n_kv_head) * head_dim,
                  "int8 decode rope_kv: N (%lld) must be (n_head + 2 n_kv_head) * head_dim",
                  (long long)N);
    TAO_CHECK_ARG(freqs != nullptr && pos != nullptr && k_cache != nullptr && v_cache != nullptr,
                  "int8 decode rope_kv: freqs, pos and caches are required");
    TAO_CHECK_ALIGN(k_cache, 4, "k_cache");
    TAO_CHECK_ALIGN(v_cache, 4, "v_cache");
    TAO_CHECK_ALIGN(y, 4, "y");
    fu.freqs = freqs;
    fu.pos = pos;
    fu.k_cache = k_cache;
    fu.v_cache = v_cache;
    fu.H = (int)n_head;
    fu.Hkv = (int)n_kv_head;
    fu.D = (int)head_dim;
    fu.T = (int)max_seq;
  }
  if (N == 0) return TAO_OK;
  const hipStream_t st = as_stream(stream);
  switch (epilogue) {
    case kI8EpiSwiGLU: return i8_decode<kI8EpiSwiGLU>(x, w, scale, y, (int)N, (int)K, st, fu);
    case kI8EpiRopeKV: return i8_decode<kI8EpiRopeKV>(x, w, scale, y, (int)N, (int)K, st, fu);
    default: return i8_decode<kI8EpiNone>(x, w, scale, y, (int)N, (int)K, st, fu);
  }
}
