// int8 dynamic-activation x int8-weight linear (Int8DynamicActivationInt8WeightConfig):
//   1. tao_int8_quant_per_token: x bf16 [M][K] -> (q int8 [M][K], s bf16 [M]), replacing
//      _int8_symm_per_token_reduced_range_quant (torchao/quantization/quant_api.py:1258-1273),
//      which the reference runs as ~6 eager kernels (amin/amax/div/round/clamp/cast);
//   2. tao_int8_scaled_mm_bf16: int32 MFMA GEMM with the fused two-scale epilogue, replacing
//      int_scaled_matmul + the weight-scale multiply (torchao/kernel/intmm.py:108-143,
//      torchao/dtypes/uintx/plain_layout.py:294-315). M > 4: the Int8Dyn instance of the
//      shared skinny-GEMM template in gemm_mfma.hip; M <= 4 (decode): int8dyn_gemv_kernel
//      below, exact int32 dot products (v_dot4_i32_i8) streamed like the int4 / int8 GEMVs;
//   3. tao_int8_dyn_linear_bf16 (M == 1): 1 + 2 in one launch — every workgroup quantises the
//      token into LDS (the per-token kernel's exact arithmetic) while its first weight slice
//      is in flight, then runs the GEMV on it: one launch per linear instead of two.
#include <atomic>

#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {

TAO_DECODE_ERROR_WORD(int8dyn_decode_status)

// Launch shape override of the int8 decode GEMVs (tao_tune_int8_gemv; 0 = heuristic), shared
// with int8wo_gemv (int8_gemv.hip).

namespace {


// ---- int8 x int8 GEMV (decode) ------------------------------------------------------------------
// A slice is 1024 k of one row = 64 lanes x 16 B; a wave owns RPW rows, Wk waves split K inside a
// workgroup, G row groups share it (int8wo_gemv_kernel's decomposition). Per lane and row:
// four v_dot4_i32_i8 per 16-B chunk into an int32 accumulator. Every partial sum is an exact
// integer (|acc| <= 127 * 127 * K < 2^31 for K < 133144), so the cross-lane and cross-wave
// reduction order cannot change the result: bit-identical to the MFMA path and the reference.
// Lanes past K read a clamped in-bounds chunk and a zeroed x, adding exactly 0.
//
// FQ (M == 1): x is the bf16 token. Each workgroup first issues its first slice's weight loads,
// then quantises the token into LDS with int8_quant_per_token_kernel's exact arithmetic (below)
// under their latency, so the per-token quantisation costs no launch of its own.
struct Int8DynGemvArgs {
  const void* x;          // int8 q [M][K] (FQ: bf16 token [K])
  const uint16_t* xs;     // [M] bf16 per-token scales (unused with FQ)
  const uint4* w;         // [N][K/16]
  const uint16_t* ws;     // [N]
  const uint16_t* bias;   // [N] or null
  uint16_t* y;            // [M][N]
  int M, N, K, Wk, G, S;
  // decode-step fusions (tao_int8dq_decode_bf16, FQ only): RMSNorm of the token before its
  // quantisation, SwiGLU / RoPE + KV-write epilogues (int8_gemv.hip's int8wo_decode_kernel)
  const uint16_t* norm_w;
  float eps;
  const float* freqs;
  const int64_t* pos;
  uint16_t* k_cache;
  uint16_t* v_cache;
  int H, Hkv, D, T;
};
enum { kDqEpiNone = 0, kDqEpiSwiGLU = 1, kDqEpiRopeKV = 2 };

__device__ __forceinline__ uint32_t dq_rmsnorm_pair(uint32_t xv, uint32_t wv, float r) {
  const float lo = round_bf16(bf16lo_to_f32(xv) * r) * bf16lo_to_f32(wv);
  const float hi = round_bf16(bf16hi_to_f32(xv) * r) * bf16hi_to_f32(wv);
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

__device__ __forceinline__ int sdot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// per-token scale and its reciprocal from amax (quant_primitives.py:1548-1554, 449-453)
__device__ __forceinline__ float token_scale(float amax) {
  float s = round_bf16(amax / 127.f);
  const float eps = round_bf16(1e-5f);
  return s < eps ? eps : s;
}

// q = clamp(round(bf16(x * r)), -127, 127) for the 8 bf16 of one 16-B piece -> 8 int8 bytes
__device__ __forceinline__ uint2 quant8(const uint4 v, float r) {
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
  uint32_t packed[2] = {0u, 0u};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float xv = (j & 1) ? bf16hi_to_f32(d[j >> 1]) : bf16lo_to_f32(d[j >> 1]);
    float t = rintf(round_bf16(xv * r));
    t = fminf(fmaxf(t, -127.f), 127.f);
    packed[j >> 2] |= ((uint32_t)(int32_t)t & 0xFFu) << (8 * (j & 3));
  }
  return make_uint2(packed[0], packed[1]);
}

__device__ __forceinline__ float bf16_abs_max2(uint32_t d, float m) {
  m = fmaxf(m, fabsf(bf16lo_to_f32(d)));
  return fmaxf(m, fabsf(bf16hi_to_f32(d)));
}

template <int MT, int RPW, int NPT, int EPI = kDqEpiNone>
__global__ __launch_bounds__(512) void int8dyn_gemv_kernel(Int8DynGemvArgs a) {
  constexpr bool FQ = NPT > 0;  // NPT: 16-B pieces of the bf16 token per thread (K <= 8 NPT T)
  static_assert(!FQ || MT == 1, "the fused quantisation is per token, M == 1");
  static_assert(EPI == kDqEpiNone || (FQ && RPW % 2 == 0), "epilogues: fused token, row pairs");
  constexpr int V = RPW * MT;
  // [G][Wk][V] int partials | (FQ) [8] wave maxima | (FQ) token q [K] int8
  extern __shared__ int lds_i[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int wk = wave % a.Wk;
  const int rg = wave / a.Wk;
  const int row0 = (blockIdx.x * a.G + rg) * RPW;
  const int K = a.K, N = a.N, S = a.S, Wk = a.Wk;
  const int nchunk = K >> 4;  // 16-B (16-k) chunks per row
  const int nw = a.G * a.Wk;
  float* wmax = reinterpret_cast<float*>(lds_i + nw * V);
  uint4* xl = reinterpret_cast<uint4*>(lds_i + ((nw * V + 8 + 3) & ~3));

  int acc[RPW][MT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0;

  uint4 wv[RPW];
  auto load_w = [&](int s) __attribute__((always_inline)) {
    const int c = s * 64 + lane;
    const int cc = c < nchunk ? c : nchunk - 1;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int n = row0 + r;
      wv[r] = ld_nt_u4(a.w + (size_t)(n < N ? n : N - 1) * nchunk + cc);
    }
  };

  float sx[MT];
  if constexpr (FQ) {
    // The token's pieces are loaded BEFORE the first slice's weights: vector loads retire in
    // issue order, so the wait for x does not wait for the weights, and the amax, the two
    // barriers and the quantisation into LDS run under the weight loads' latency.
    const uint4* xr = reinterpret_cast<const uint4*>(a.x);
    const int nvec = K >> 3;
    uint4 xv[NPT], gv[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      xv[u] = xr[i < nvec ? i : nvec - 1];  // clamped, masked below
      if (a.norm_w != nullptr) gv[u] = reinterpret_cast<const uint4*>(a.norm_w)[i < nvec ? i : nvec - 1];
    }
    load_w(wk);  // every wave owns at least one slice (Wk <= S)
    if (a.norm_w != nullptr) {  // RMSNorm of the token (the unfused rmsnorm_kernel's roundings)
      float ss = 0.f;
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const bool ok = threadIdx.x + u * (int)blockDim.x < nvec;
        const uint32_t d[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = ok ? bf16lo_to_f32(d[j]) : 0.f, q = ok ? bf16hi_to_f32(d[j]) : 0.f;
          ss = fmaf(p, p, fmaf(q, q, ss));
        }
      }
      ss = wave_sum(ss);
      if (lane == 0) wmax[wave] = ss;
      __syncthreads();
      float t = 0.f;
      for (int q = 0; q < nw; ++q) t += wmax[q];
      const float rn = rsqrtf(t / (float)K + a.eps);
#pragma unroll
      for (int u = 0; u < NPT; ++u)
        xv[u] = make_uint4(dq_rmsnorm_pair(xv[u].x, gv[u].x, rn), dq_rmsnorm_pair(xv[u].y, gv[u].y, rn),
                           dq_rmsnorm_pair(xv[u].z, gv[u].z, rn), dq_rmsnorm_pair(xv[u].w, gv[u].w, rn));
      __syncthreads();  // wmax is reused for the amax below
    }
    // amax over K bf16, then quantise into LDS (int8_quant_per_token_kernel's arithmetic)
    float m = 0.f;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const bool ok = threadIdx.x + u * (int)blockDim.x < nvec;
      const uint4 v = ok ? xv[u] : make_uint4(0u, 0u, 0u, 0u);
      m = bf16_abs_max2(v.x, m);
      m = bf16_abs_max2(v.y, m);
      m = bf16_abs_max2(v.z, m);
      m = bf16_abs_max2(v.w, m);
    }
    m = wave_max(m);
    if (lane == 0) wmax[wave] = m;
    __syncthreads();
    float amax = wmax[0];
    for (int w = 1; w < nw; ++w) amax = fmaxf(amax, wmax[w]);
    const float st = token_scale(amax);
    const float rs = round_bf16(1.f / st);
    uint2* xq = reinterpret_cast<uint2*>(xl);
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      if (i < nvec) xq[i] = quant8(xv[u], rs);
    }
    __syncthreads();
    sx[0] = st;
  } else {
    load_w(wk);
#pragma unroll
    for (int m = 0; m < MT; ++m) sx[m] = bf16_to_f32(a.xs[m < a.M ? m : a.M - 1]);
  }

  for (int s = wk; s < S; s += Wk) {
    if (s != wk) load_w(s);
    const int c = s * 64 + lane;
    const bool cval = c < nchunk;
    const int cc = cval ? c : nchunk - 1;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      uint4 xv;
      if constexpr (FQ) {
        xv = xl[cc];
      } else {
        const int mm = m < a.M ? m : a.M - 1;
        xv = reinterpret_cast<const uint4*>(a.x)[(size_t)mm * nchunk + cc];
      }
      const uint32_t keep = cval ? ~0u : 0u;  // lanes past K add exactly 0
      const uint32_t xd[4] = {xv.x & keep, xv.y & keep, xv.z & keep, xv.w & keep};
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        int d = acc[r][m];
        d = sdot4(xd[0], wv[r].x, d);
        d = sdot4(xd[1], wv[r].y, d);
        d = sdot4(xd[2], wv[r].z, d);
        d = sdot4(xd[3], wv[r].w, d);
        acc[r][m] = d;
      }
    }
  }

  int v[V];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) v[r * MT + m] = acc[r][m];
  wave_reduce_scatter<V>(v, lane);

  constexpr int T = Log2<V>::value;
  const bool owner = (lane & ((64 >> T) - 1)) == 0;
  const int idx = lane >> (6 - T);
  int total = v[0];
  bool writer = owner;
  int widx = idx;
  if (Wk > 1) {
    if (owner) lds_i[(rg * Wk + wk) * V + idx] = v[0];
    __syncthreads();
    writer = (wk == 0) && (lane < V);
    widx = lane;
    if (writer) {
      total = 0;
      for (int kk = 0; kk < Wk; ++kk) total += lds_i[(rg * Wk + kk) * V + widx];
    }
  }
  if constexpr (EPI == kDqEpiNone) {
    if (writer) {
      const int r = widx / MT, m = widx % MT;
      const int n = row0 + r;
      if (n < N && m < a.M) {
        // bf16(c) * x_scale, * w_scale, each rounded (intmm.py:133-137, plain_layout.py:301-315);
        // the MFMA path's Int8Dyn::epilogue
        float o = round_bf16(round_bf16((float)total) * sx[m]);
        o = round_bf16(o * bf16_to_f32(a.ws[n]));
        if (a.bias != nullptr) o = round_bf16(o + bf16_to_f32(a.bias[n]));
        a.y[(size_t)m * N + n] = f32_to_bf16(o);
      }
    }
  } else {
    // the linear's output of this lane's row, then row pair (2p, 2p+1) meets in lane p
    const int nr = row0 + (widx < V ? widx : 0);
    float o = round_bf16(round_bf16((float)total) * sx[0]);
    o = round_bf16(o * bf16_to_f32(a.ws[nr < N ? nr : N - 1]));
    const int sh = Wk > 1 ? 0 : 6 - T;
    const int pl = lane < RPW / 2 ? lane : 0;
    const float ea = __shfl(o, (2 * pl) << sh);
    const float eb = __shfl(o, (2 * pl + 1) << sh);
    const int n = row0 + 2 * pl;
    if ((Wk == 1 || wk == 0) && lane < RPW / 2 && n < N) {
      if constexpr (EPI == kDqEpiSwiGLU) {
        a.y[n >> 1] = f32_to_bf16(round_bf16(ea / (1.f + __expf(-ea))) * eb);
      } else {
        const int D = a.D, HD = a.H * a.D, KD = a.Hkv * a.D;
        int64_t p = a.pos[0];
        const bool pok = p >= 0 && p < a.T;
        if (!pok) {
          flag_decode_error(kDecodeErrKvPos);
          p = p < 0 ? 0 : a.T - 1;
        }
        uint32_t ov = (uint32_t)f32_to_bf16(ea) | ((uint32_t)f32_to_bf16(eb) << 16);
        if (n < HD + KD) {
          const float2 cs = reinterpret_cast<const float2*>(a.freqs)[p * (D >> 1) + ((n % D) >> 1)];
          const float o0 = ea * cs.x - eb * cs.y, o1 = eb * cs.x + ea * cs.y;
          ov = (uint32_t)f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
        }
        if (n < HD) {
          reinterpret_cast<uint32_t*>(a.y)[n >> 1] = ov;
        } else if (pok) {
          const int nk = n < HD + KD ? n - HD : n - HD - KD;
          uint16_t* cache = n < HD + KD ? a.k_cache : a.v_cache;
          const size_t off = ((size_t)(nk / D) * a.T + p) * D + nk % D;
          reinterpret_cast<uint32_t*>(cache)[off >> 1] = ov;
        }
      }
    }
  }
}


template <int MT, int RPW, int NPT, int EPI = kDqEpiNone>
int launch_dyn_gemv_npt(Int8DynGemvArgs a, int grid, int threads, size_t lds, hipStream_t stream) {
  launch((int8dyn_gemv_kernel<MT, RPW, NPT, EPI>), dim3(grid), dim3(threads), lds, stream, a);
  return check_launch("int8dyn_gemv_kernel");
}

template <int MT, int RPW, bool FQ, int EPI = kDqEpiNone>
int launch_dyn_gemv(Int8DynGemvArgs a, int wk, int g, hipStream_t stream) {
  const int nchunk = a.K / 16;
  a.S = (nchunk + 63) / 64;
  a.Wk = wk < a.S ? wk : a.S;
  a.G = g;
  // FQ: the token must fit the workgroup's registers (K <= 8 x 16 pieces x threads)
  while (FQ && 64 * a.Wk * a.G * 8 * 16 < a.K && a.Wk * a.G * 2 <= 8) a.G *= 2;
  const int rows_per_wg = a.G * RPW;
  const int grid = (a.N + rows_per_wg - 1) / rows_per_wg;
  const int nw = a.G * a.Wk;
  const int threads = 64 * nw;
  if (!FQ) {
    const size_t lds = (size_t)nw * RPW * MT * sizeof(int);
    return launch_dyn_gemv_npt<MT, RPW, 0>(a, grid, threads, lds, stream);
  }
  if constexpr (FQ) {
    const size_t lds = (((size_t)nw * RPW * MT + 8 + 3) & ~(size_t)3) * sizeof(int) + (size_t)a.K;
    const int per = (a.K / 8 + threads - 1) / threads;  // pieces per thread
    if (per <= 1) return launch_dyn_gemv_npt<MT, RPW, 1, EPI>(a, grid, threads, lds, stream);
    if (per <= 2) return launch_dyn_gemv_npt<MT, RPW, 2, EPI>(a, grid, threads, lds, stream);
    if (per <= 4) return launch_dyn_gemv_npt<MT, RPW, 4, EPI>(a, grid, threads, lds, stream);
    if (per <= 8) return launch_dyn_gemv_npt<MT, RPW, 8, EPI>(a, grid, threads, lds, stream);
    if (a.norm_w == nullptr && per <= 16)  // (the norm's weight pieces double the registers)
      return launch_dyn_gemv_npt<MT, RPW, 16, EPI>(a, grid, threads, lds, stream);
    TAO_CHECK_ARG(false, "int8 dyn linear: K (%d) too long for the token prologue", a.K);
  }
  return TAO_OK;
}

// M == 1 shape (experiments/sweep_int8.py, profiles/r1_sweep_int8.jsonl, fused path):
// K <= 4096: 4 rows per wave, 2 waves along K, 2 row groups (one for the 128256-row head);
// longer K: 8 rows per wave, 4 waves along K (4096x14336 11.5 us).
template <bool FQ, int EPI = kDqEpiNone>
int dyn_gemv_m1(Int8DynGemvArgs a, hipStream_t stream) {
  const int S = (a.K / 16 + 63) / 64;
  int rpw = 4, wk = S < 2 ? S : 2, g = a.N >= 65536 ? 1 : 2;
  if (S > 4) {
    rpw = 8;
    wk = 4;
    g = 1;
  }
  const int trpw = tao::tuning().i8_rpw;
  const int twk = tao::tuning().i8_wk;
  const int tg = tao::tuning().i8_g;
  if (trpw > 0) rpw = trpw;
  if (twk > 0) wk = twk;
  if (tg > 0) g = tg;
  if (rpw == 2) return launch_dyn_gemv<1, 2, FQ, EPI>(a, wk, g, stream);
  if (rpw == 8) return launch_dyn_gemv<1, 8, FQ, EPI>(a, wk, g, stream);
  return launch_dyn_gemv<1, 4, FQ, EPI>(a, wk, g, stream);
}

int int8dyn_gemv(Int8DynGemvArgs a, hipStream_t stream) {
  const int S = (a.K / 16 + 63) / 64;
  const int wk = S < 8 ? S : 8, g = (8 / wk) > 0 ? 8 / wk : 1;
  if (a.M <= 1) return dyn_gemv_m1<false>(a, stream);
  if (a.M <= 2) return launch_dyn_gemv<2, 4, false>(a, wk, g, stream);
  return launch_dyn_gemv<4, 2, false>(a, wk, g, stream);
}

// ---- per-token quantisation ------------------------------------------------------------------
constexpr int kQBlock = 256;

__global__ __launch_bounds__(kQBlock) void int8_quant_per_token_kernel(
    const uint16_t* __restrict__ x, int8_t* __restrict__ q, uint16_t* __restrict__ scale, int K) {
  __shared__ float wmax[kQBlock / 64];
  const int row = blockIdx.x;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * K);
  const int nvec = K / 8;  // 8 bf16 per 16-B vector
  float m = 0.f;
  for (int i = threadIdx.x; i < nvec; i += kQBlock) {
    const uint4 v = xr[i];
    m = bf16_abs_max2(v.x, m);
    m = bf16_abs_max2(v.y, m);
    m = bf16_abs_max2(v.z, m);
    m = bf16_abs_max2(v.w, m);
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  float amax = wmax[0];
#pragma unroll
  for (int w = 1; w < kQBlock / 64; ++w) amax = fmaxf(amax, wmax[w]);

  // scale = clamp(bf16(amax / 127), min = 1e-5) in bf16 (quant_primitives.py:1548-1554 with
  // quant range [-127, 127]); the clamp minimum is compared after bf16 rounding.
  const float s = token_scale(amax);
  if (threadIdx.x == 0) scale[row] = f32_to_bf16(s);
  // q = clamp(round(bf16(x * bf16(1/s))), -127, 127)  (quant_primitives.py:449-453)
  const float r = round_bf16(1.f / s);
  uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * K);
  for (int i = threadIdx.x; i < nvec; i += kQBlock) qr[i] = quant8(xr[i], r);
}

// One wave per token for K <= 64 * 8 * NV (the prefill shapes): the wave's 16-B pieces of the
// token stay in registers between the amax and the quantisation, so the token is read once
// (the block kernel above re-reads it after its barrier: a second dependent round trip) and the
// amax is a DPP wave reduction with no LDS barrier. Same arithmetic, bit-identical output.
// 4 tokens per 256-thread workgroup.
constexpr int kQWaves = 4;
template <int NV>
__global__ __launch_bounds__(64 * kQWaves) void int8_quant_per_token_wave_kernel(
    const uint16_t* __restrict__ x, int8_t* __restrict__ q, uint16_t* __restrict__ scale, int M,
    int K) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kQWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= M) return;  // wave-uniform
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * K);
  const int nvec = K / 8;
  uint4 v[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = lane + 64 * u;
    v[u] = xr[i < nvec ? i : nvec - 1];  // clamped duplicates do not change the max
  }
  float m = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    m = bf16_abs_max2(v[u].x, m);
    m = bf16_abs_max2(v[u].y, m);
    m = bf16_abs_max2(v[u].z, m);
    m = bf16_abs_max2(v[u].w, m);
  }
  m = wave_max(m);
  const float s = token_scale(m);
  if (lane == 0) scale[row] = f32_to_bf16(s);
  const float r = round_bf16(1.f / s);
  uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * K);
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = lane + 64 * u;
    if (i < nvec) qr[i] = quant8(v[u], r);
  }
}

int launch_quant_per_token(const uint16_t* x, int8_t* q, uint16_t* scale, int M, int K,
                           hipStream_t stream) {
  const int nv = (K / 8 + 63) / 64;
  const dim3 grid((unsigned)((M + kQWaves - 1) / kQWaves)), block(64 * kQWaves);
  if (tuning().quant_block == 0) {
    if (nv <= 2) {
      launch(int8_quant_per_token_wave_kernel<2>, grid, block, 0, stream, x, q, scale, M, K);
      return check_launch("int8_quant_per_token_wave_kernel");
    }
    if (nv <= 4) {
      launch(int8_quant_per_token_wave_kernel<4>, grid, block, 0, stream, x, q, scale, M, K);
      return check_launch("int8_quant_per_token_wave_kernel");
    }
    if (nv <= 8) {
      launch(int8_quant_per_token_wave_kernel<8>, grid, block, 0, stream, x, q, scale, M, K);
      return check_launch("int8_quant_per_token_wave_kernel");
    }
    if (nv <= 16) {
      launch(int8_quant_per_token_wave_kernel<16>, grid, block, 0, stream, x, q, scale, M, K);
      return check_launch("int8_quant_per_token_wave_kernel");
    }
  }
  launch(int8_quant_per_token_kernel, dim3((unsigned)M), dim3(kQBlock), 0, stream, x, q, scale,
         K);
  return check_launch("int8_quant_per_token_kernel");
}

}  // namespace

int int8_scaled_mm_launch(const int8_t* xq, const uint16_t* xs, const int8_t* wq,
                          const uint16_t* ws, const uint16_t* bias, uint16_t* y, int M, int N,
                          int K, hipStream_t stream);  // gemm_mfma.hip

}  // namespace tao

using namespace tao;

extern "C" {

int tao_int8_quant_per_token(const uint16_t* x, int8_t* q, uint16_t* scale, int64_t M,
                             int64_t K, void* stream) {
  TAO_CHECK_ARG(M >= 0 && K >= 0, "int8 quant: negative size");
  TAO_CHECK_ARG(K % 16 == 0, "int8 quant: K (%lld) must be a multiple of 16", (long long)K);
  TAO_CHECK_ARG(M < (1LL << 31) && K < (1LL << 31), "int8 quant: size out of range");
  if (M == 0 || K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(q, 8, "q");
  return launch_quant_per_token(x, q, scale, (int)M, (int)K, as_stream(stream));
}

// per-token quant kernel choice (A/B only): 0 = one wave per token (default), 1 = the
// 256-thread block kernel
int tao_tune_int8_quant(int block) {
  TAO_CHECK_ARG(block == 0 || block == 1, "tune: int8 quant block must be 0 or 1");
  tuning().quant_block = block;
  return TAO_OK;
}

int tao_int8_scaled_mm_bf16(const int8_t* xq, const uint16_t* xs, const int8_t* wq,
                            const uint16_t* ws, const uint16_t* bias, uint16_t* y, int64_t M,
                            int64_t N, int64_t K, void* stream) {
  TAO_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "int8 scaled mm: negative size");
  TAO_CHECK_ARG(K % 16 == 0, "int8 scaled mm: K (%lld) must be a multiple of 16", (long long)K);
  TAO_CHECK_ARG(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31),
                "int8 scaled mm: size out of range");
  if (M == 0 || N == 0) return TAO_OK;
  TAO_CHECK_ARG(K > 0, "int8 scaled mm: K must be > 0");
  TAO_CHECK_ALIGN(xq, 16, "xq");
  TAO_CHECK_ALIGN(wq, 16, "wq");
  if (M <= 4) {
    Int8DynGemvArgs a{xq, xs, reinterpret_cast<const uint4*>(wq), ws, bias, y,
                      (int)M, (int)N, (int)K, 0, 0, 0};
    return int8dyn_gemv(a, as_stream(stream));
  }
  return int8_scaled_mm_launch(xq, xs, wq, ws, bias, y, (int)M, (int)N, (int)K,
                               as_stream(stream));
}

int tao_int8_dyn_linear_bf16(const uint16_t* x, const int8_t* wq, const uint16_t* ws,
                             const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                             void* stream) {
  TAO_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "int8 dyn linear: negative size");
  TAO_CHECK_ARG(M <= 1, "int8 dyn linear: the fused path is one token (M <= 1, got %lld)",
                (long long)M);
  TAO_CHECK_ARG(K % 16 == 0, "int8 dyn linear: K (%lld) must be a multiple of 16", (long long)K);
  TAO_CHECK_ARG(K <= 65536, "int8 dyn linear: K (%lld) must be <= 65536 (token in LDS)",
                (long long)K);
  TAO_CHECK_ARG(N < (1LL << 31), "int8 dyn linear: size out of range");
  if (M == 0 || N == 0) return TAO_OK;
  TAO_CHECK_ARG(K > 0, "int8 dyn linear: K must be > 0");
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(wq, 16, "wq");
  Int8DynGemvArgs a{x, nullptr, reinterpret_cast<const uint4*>(wq), ws, bias, y,
                    1, (int)N, (int)K, 0, 0, 0};
  return dyn_gemv_m1<true>(a, as_stream(stream));
}

int tao_int8dq_decode_bf16(const uint16_t* x, const int8_t* wq, const uint16_t* ws, int64_t N,
                           int64_t K, const uint16_t* norm_weight, float eps, int epilogue,
                           uint16_t* y, const float* freqs, const int64_t* pos, uint16_t* k_cache,
                           uint16_t* v_cache, int64_t n_head, int64_t n_kv_head, int64_t head_dim,
                           int64_t max_seq, void* stream) {
  TAO_CHECK_ARG(N >= 0 && K > 0 && K % 16 == 0 && K <= 32768 && N < (1LL << 31),
                "int8dq decode: K (%lld) must be a positive multiple of 16, <= 32768",
                (long long)K);
  TAO_CHECK_ARG(epilogue >= kDqEpiNone && epilogue <= kDqEpiRopeKV,
                "int8dq decode: epilogue must be 0 (none), 1 (swiglu) or 2 (rope_kv)");
  TAO_CHECK_ARG(epilogue == kDqEpiNone || N % 2 == 0, "int8dq decode: N (%lld) must be even",
                (long long)N);
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(wq, 16, "wq");
  Int8DynGemvArgs a{x, nullptr, reinterpret_cast<const uint4*>(wq), ws, nullptr, y,
                    1, (int)N, (int)K, 0, 0, 0};
  if (norm_weight != nullptr) TAO_CHECK_ALIGN(norm_weight, 16, "norm_weight");
  a.norm_w = norm_weight;
  a.eps = eps;
  if (epilogue == kDqEpiRopeKV) {
    TAO_CHECK_ARG(n_head > 0 && n_kv_head > 0 && head_dim > 0 && head_dim % 2 == 0 &&
                      max_seq > 0 && N == (n_head + 2 * n_kv_head) * head_dim,
                  "int8dq decode rope_kv: N (%lld) must be (n_head + 2 n_kv_head) * head_dim",
                  (long long)N);
    TAO_CHECK_ARG(freqs != nullptr && pos != nullptr && k_cache != nullptr && v_cache != nullptr,
                  "int8dq decode rope_kv: freqs, pos and caches are required");
    TAO_CHECK_ALIGN(k_cache, 4, "k_cache");
    TAO_CHECK_ALIGN(v_cache, 4, "v_cache");
    TAO_CHECK_ALIGN(y, 4, "y");
    a.freqs = freqs;
    a.pos = pos;
    a.k_cache = k_cache;
    a.v_cache = v_cache;
    a.H = (int)n_head;
    a.Hkv = (int)n_kv_head;
    a.D = (int)head_dim;
    a.T = (int)max_seq;
  }
  if (N == 0) return TAO_OK;
  const hipStream_t st = as_stream(stream);
  switch (epilogue) {
    case kDqEpiSwiGLU: return dyn_gemv_m1<true, kDqEpiSwiGLU>(a, st);
    case kDqEpiRopeKV: return dyn_gemv_m1<true, kDqEpiRopeKV>(a, st);
    default: return dyn_gemv_m1<true>(a, st);
  }
}

int tao_tune_int8_gemv(int rows_per_wave, int waves_k, int row_groups) {
  TAO_CHECK_ARG(rows_per_wave == 0 || rows_per_wave == 2 || rows_per_wave == 4 ||
                    rows_per_wave == 8,
                "tune: rows_per_wave must be 0 (auto), 2, 4 or 8");
  TAO_CHECK_ARG(waves_k >= 0 && row_groups >= 0 && waves_k * (row_groups ? row_groups : 1) <= 8,
                "tune: waves_k * row_groups must be <= 8");
  tao::tuning().i8_rpw = rows_per_wave;
  tao::tuning().i8_wk = waves_k;
  tao::tuning().i8_g = row_groups;
  return TAO_OK;
}

}  // extern "C"
