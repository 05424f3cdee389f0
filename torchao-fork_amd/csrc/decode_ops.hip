// Fused decode-step kernels for the end-to-end harness (torchao/_models/llama).
//
// The reference gets these fusions from torch.compile (generate.py:865-875); here each is one
// hand-written gfx950 kernel so a decoded token is ~11 launches per layer instead of ~50 eager
// ones. None is on the int4 hot path; all are tiny and latency-bound (a few KiB per call except
// the KV-cache reads of attention).
//   * RMSNorm:   y = bf16(bf16(x * rsqrt(mean(x^2) + eps)) * w)        (model.py RMSNorm)
//   * RoPE + KV: rotate q, k of the wqkv output in fp32 (interleaved pairs, rotary table row
//                pos[s]), write q as [B][H][S][D] and k, v into the static caches at pos[S]
//   * attention: one query per (batch, head), keys 0..pos. Caches of <= 1024 rows: one kernel,
//                a workgroup per query head (online softmax per wave, LDS merge). Longer:
//                split over 64-key chunks (flash-decoding; GQA: a workgroup serves the G query
//                heads of one kv head), then a combine kernel merges the chunks' (max, sum, o).
//                (Variants measured slower and removed in round 4: the split in one launch merged
//                by the last arriving chunk, 672 vs 700 tokens/s; packed-bf16 math; half-line K
//                loads; 32 keys per wave step; weight prefetch riding on the launch.)
//   * SiLU-mul:  y = bf16(bf16(silu(a)) * b)                             (F.silu(w1 x) * w3 x)
//   * argmax:    greedy next token over bf16 logits, torch.argmax's first-index tie rule
#include <atomic>

#include "tao_common.h"

namespace tao {
// attn_mfma.hip: the MFMA prefill attention (tao_attn_prefill_bf16)
int attn_prefill_mfma(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                      const int64_t* pos, uint16_t* out, int64_t B, int64_t H, int64_t Hkv,
                      int64_t S, int64_t T, float scale, hipStream_t stream);
}  // namespace tao
#include "tao_attn.h"
#include "tao_reduce.h"

#ifndef TAO_ATTN_WAVES
#define TAO_ATTN_WAVES 16  // waves per workgroup of the single-pass decode attention
#endif

namespace tao {

TAO_DECODE_ERROR_WORD(decode_ops_status)
int int4gemv_decode_status(unsigned* bits);
int sf_decode_status(unsigned* bits);
int int8gemv_decode_status(unsigned* bits);
int int8dyn_decode_status(unsigned* bits);
int engine_decode_status(unsigned* bits);

namespace {

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---- RMSNorm (+ residual add): one workgroup per row, 8 bf16 per 16-B piece ---------------------
// The row's pieces stay in registers from the load to the normalised store (NP pieces per thread,
// D <= 8 NP 256), so a row costs one global round trip, the block sum and the stores; the first
// versions re-read x (and the residual) after the block sum, a second dependent round trip in
// every launch. ADD: h = bf16(x + r) stored first (torch's bf16 `x + r`: fp32 sum, RNE), then the
// norm of h; the pair is bit-identical to the two launches it replaces. y = bf16(bf16(h * r) * w).
__device__ __forceinline__ uint32_t add_pair_bf16(uint32_t a, uint32_t b) {
  const float lo = bf16lo_to_f32(a) + bf16lo_to_f32(b);
  const float hi = bf16hi_to_f32(a) + bf16hi_to_f32(b);
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

template <int NP, bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_rows_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
    const uint16_t* __restrict__ w, uint16_t* __restrict__ h, uint16_t* __restrict__ y, int D,
    float eps) {
  __shared__ float red[4];
  const size_t row = (size_t)blockIdx.x * D;
  const uint4* xr = reinterpret_cast<const uint4*>(x + row);
  const uint4* rr = reinterpret_cast<const uint4*>(ADD ? res + row : x + row);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  const int nv = D / 8;
  uint4 v[NP], g[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u) {  // every load of the row (and its norm weights) in one round trip
    const int i = threadIdx.x + 256 * u, ic = i < nv ? i : nv - 1;
    v[u] = xr[ic];
    g[u] = wr[ic];
    if constexpr (ADD) {
      const uint4 b = rr[ic];
      v[u] = make_uint4(add_pair_bf16(v[u].x, b.x), add_pair_bf16(v[u].y, b.y),
                        add_pair_bf16(v[u].z, b.z), add_pair_bf16(v[u].w, b.w));
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i >= nv) continue;
    if constexpr (ADD) reinterpret_cast<uint4*>(h + row)[i] = v[u];
    const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = bf16lo_to_f32(d[j]), b = bf16hi_to_f32(d[j]);
      ss = fmaf(a, a, fmaf(b, b, ss));
    }
  }
  const float r = rsqrtf(block_sum(ss, red) / (float)D + eps);
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i >= nv) continue;
    const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    const uint32_t e[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = round_bf16(bf16lo_to_f32(d[j]) * r) * bf16lo_to_f32(e[j]);
      const float hi = round_bf16(bf16hi_to_f32(d[j]) * r) * bf16hi_to_f32(e[j]);
      o[j] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
    }
    reinterpret_cast<uint4*>(y + row)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// The residual add of a linear whose K slices were NOT reduced in-kernel
// (tao_int4wo_linear_partials_f32): the linear's output is formed here as bf16(sum_z part[z]) in
// slice order from 0 (the single-fetch reducer's order and rounding, so bit-identical to its bf16
// output), then h = bf16(x + that), y = RMSNorm(h) as rmsnorm_rows_kernel<NP, true>.
// SS > 0 (2, 4, 8): S == SS known at compile time, so every slice's loads are issued before the
// first add (one round trip; a runtime S loop waits once per slice). SS == 0: any S, one at a time.
template <int NP, int SS>
__global__ __launch_bounds__(256) void rmsnorm_part_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ part, int S, size_t plane,
    const uint16_t* __restrict__ w, uint16_t* __restrict__ h, uint16_t* __restrict__ y, int D,
    float eps) {
  __shared__ float red[4];
  const size_t row = (size_t)blockIdx.x * D;
  const uint4* xr = reinterpret_cast<const uint4*>(x + row);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  const int nv = D / 8;
  uint4 v[NP], g[NP];
  float a[NP][8];
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = threadIdx.x + 256 * u, ic = i < nv ? i : nv - 1;
    v[u] = xr[ic];
    g[u] = wr[ic];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[u][e] = 0.f;
  }
  auto add_slice = [&](const float4 (&p)[NP][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      a[u][0] += p[u][0].x;
      a[u][1] += p[u][0].y;
      a[u][2] += p[u][0].z;
      a[u][3] += p[u][0].w;
      a[u][4] += p[u][1].x;
      a[u][5] += p[u][1].y;
      a[u][6] += p[u][1].z;
      a[u][7] += p[u][1].w;
    }
  };
  auto load_slice = [&](int z, float4 (&p)[NP][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int i = threadIdx.x + 256 * u, ic = i < nv ? i : nv - 1;
      const float4* pr = reinterpret_cast<const float4*>(part + (size_t)z * plane + row) + 2 * ic;
      p[u][0] = pr[0];
      p[u][1] = pr[1];
    }
  };
  if constexpr (SS > 0) {  // all SS slices in flight, then summed in slice order from 0
    float4 p[SS][NP][2];
#pragma unroll
    for (int z = 0; z < SS; ++z) load_slice(z, p[z]);
#pragma unroll
    for (int z = 0; z < SS; ++z) add_slice(p[z]);
  } else {
    for (int z = 0; z < S; ++z) {
      float4 p[NP][2];
      load_slice(z, p);
      add_slice(p);
    }
  }
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = (uint32_t)f32_to_bf16(a[u][2 * e]) | ((uint32_t)f32_to_bf16(a[u][2 * e + 1]) << 16);
    v[u] = make_uint4(add_pair_bf16(v[u].x, o[0]), add_pair_bf16(v[u].y, o[1]),
                      add_pair_bf16(v[u].z, o[2]), add_pair_bf16(v[u].w, o[3]));
  }
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i >= nv) continue;
    reinterpret_cast<uint4*>(h + row)[i] = v[u];
    const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float p = bf16lo_to_f32(d[j]), q = bf16hi_to_f32(d[j]);
      ss = fmaf(p, p, fmaf(q, q, ss));
    }
  }
  const float r = rsqrtf(block_sum(ss, red) / (float)D + eps);
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i >= nv) continue;
    const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    const uint32_t e[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = round_bf16(bf16lo_to_f32(d[j]) * r) * bf16lo_to_f32(e[j]);
      const float hi = round_bf16(bf16hi_to_f32(d[j]) * r) * bf16hi_to_f32(e[j]);
      o[j] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
    }
    reinterpret_cast<uint4*>(y + row)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// Rows wider than 8 x 4 x 256 bf16: the streaming form (x and the residual re-read after the sum)
template <bool ADD>
__global__ __launch_bounds__(256) void rmsnorm_wide_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
    const uint16_t* __restrict__ w, uint16_t* __restrict__ h, uint16_t* __restrict__ y, int D,
    float eps) {
  __shared__ float red[4];
  const size_t row = (size_t)blockIdx.x * D;
  const uint4* xr = reinterpret_cast<const uint4*>(x + row);
  const uint4* rr = reinterpret_cast<const uint4*>(ADD ? res + row : x + row);
  const uint4* wr = reinterpret_cast<const uint4*>(w);
  const int nv = D / 8;
  auto piece = [&](int i) __attribute__((always_inline)) {
    uint4 a = xr[i];
    if constexpr (ADD) {
      const uint4 b = rr[i];
      a = make_uint4(add_pair_bf16(a.x, b.x), add_pair_bf16(a.y, b.y), add_pair_bf16(a.z, b.z),
                     add_pair_bf16(a.w, b.w));
    }
    return a;
  };
  float ss = 0.f;
  for (int i = threadIdx.x; i < nv; i += 256) {
    const uint4 v = piece(i);
    if constexpr (ADD) reinterpret_cast<uint4*>(h + row)[i] = v;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = bf16lo_to_f32(d[j]), b = bf16hi_to_f32(d[j]);
      ss = fmaf(a, a, fmaf(b, b, ss));
    }
  }
  const float r = rsqrtf(block_sum(ss, red) / (float)D + eps);
  for (int i = threadIdx.x; i < nv; i += 256) {
    const uint4 v = piece(i), g = wr[i];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w}, e[4] = {g.x, g.y, g.z, g.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = round_bf16(bf16lo_to_f32(d[j]) * r) * bf16lo_to_f32(e[j]);
      const float hi = round_bf16(bf16hi_to_f32(d[j]) * r) * bf16hi_to_f32(e[j]);
      o[j] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
    }
    reinterpret_cast<uint4*>(y + row)[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

template <bool ADD>
void launch_rmsnorm(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* h,
                    uint16_t* y, int64_t rows, int64_t dim, float eps, hipStream_t st) {
  const dim3 grid((unsigned)rows), blk(256);
  const int D = (int)dim, nv = D / 8;
  if (nv <= 256) launch(rmsnorm_rows_kernel<1, ADD>, grid, blk, 0, st, x, res, w, h, y, D, eps);
  else if (nv <= 512) launch(rmsnorm_rows_kernel<2, ADD>, grid, blk, 0, st, x, res, w, h, y, D, eps);
  else if (nv <= 1024) launch(rmsnorm_rows_kernel<4, ADD>, grid, blk, 0, st, x, res, w, h, y, D, eps);
  else launch(rmsnorm_wide_kernel<ADD>, grid, blk, 0, st, x, res, w, h, y, D, eps);
}

// ---- RoPE on q, k + KV-cache write: one workgroup per token, one thread per pair -------------
__global__ __launch_bounds__(256) void rope_kv_kernel(
    const uint16_t* __restrict__ qkv, const float* __restrict__ freqs,
    const int64_t* __restrict__ pos, uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc,
    uint16_t* __restrict__ vc, int S, int H, int Hkv, int D, int T) {
  const int tok = blockIdx.x;  // b * S + s
  const int b = tok / S, s = tok % S;
  const int half = D / 2;
  int64_t p = pos[s];
  const bool pok = p >= 0 && p < T;  // KV cache row inside [0, T)
  if (!pok) {  // report (tao_decode_status) and write no cache row
    if (threadIdx.x == 0) flag_decode_error(kDecodeErrKvPos);
    p = p < 0 ? 0 : T - 1;
  }
  const uint32_t* row = reinterpret_cast<const uint32_t*>(qkv + (size_t)tok * (H + 2 * Hkv) * D);
  const float2* f = reinterpret_cast<const float2*>(freqs) + (size_t)p * half;  // table row pos
  const int rot_pairs = (H + Hkv) * half;
  for (int i = threadIdx.x; i < rot_pairs + Hkv * half; i += blockDim.x) {
    const uint32_t w = row[i];  // pairs are interleaved: (x[2j], x[2j+1]) = one dword
    if (i < rot_pairs) {
      const int head = i / half, j = i % half;
      const float2 cs = f[j];
      const float x0 = bf16lo_to_f32(w), x1 = bf16hi_to_f32(w);
      const float o0 = x0 * cs.x - x1 * cs.y, o1 = x1 * cs.x + x0 * cs.y;
      const uint32_t o = (uint32_t)f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
      if (head < H) {
        reinterpret_cast<uint32_t*>(q_out)[(((size_t)b * H + head) * S + s) * half + j] = o;
      } else if (pok) {
        const int kh = head - H;
        reinterpret_cast<uint32_t*>(kc)[(((size_t)b * Hkv + kh) * T + p) * half + j] = o;
      }
    } else if (pok) {
      const int k = i - rot_pairs;
      const int vh = k / half, j = k % half;
      reinterpret_cast<uint32_t*>(vc)[(((size_t)b * Hkv + vh) * T + p) * half + j] = w;
    }
  }
}

// ---- decode attention, phase 1: partial (m, l, o) per 64-key chunk --------------------------
constexpr int kChunk = 64;

template <int G, int D>
__global__ __launch_bounds__(256) void attn_partial_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int64_t* __restrict__ pos, float* __restrict__ part,
    int Hkv, int T, float scale) {
  static_assert(D == 128, "head_dim 128");
  __shared__ float qs[G][D];
  __shared__ float ps[G][kChunk];
  __shared__ float mls[G][2];
  const int bk = blockIdx.x;  // b * Hkv + kvh
  const int b = bk / Hkv, kvh = bk % Hkv;
  const int c = blockIdx.y, NC = gridDim.y;
  const int L = attn_len(pos[0], T);
  const int t0 = c * kChunk;
  if (t0 >= L) return;  // uniform: the combine kernel skips this chunk too
  const int tid = threadIdx.x;
  const int H = Hkv * G;
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    qs[g][d] = bf16_to_f32(q[((size_t)b * H + kvh * G + g) * D + d]);
  }
  __syncthreads();

  // scores: thread = (key j = tid / 4, quarter p = tid % 4 of the 128 dims)
  const int j = tid >> 2, p = tid & 3;
  const int kk = t0 + j;
  float sc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) sc[g] = 0.f;
  if (kk < L) {
    const uint4* kr =
        reinterpret_cast<const uint4*>(kc + (((size_t)b * Hkv + kvh) * T + kk) * D + p * 32);
#pragma unroll
    for (int v4 = 0; v4 < 4; ++v4) {
      const uint4 kv = kr[v4];
      const uint32_t w[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int d = p * 32 + v4 * 8 + 2 * e;
        const float k0 = bf16lo_to_f32(w[e]), k1 = bf16hi_to_f32(w[e]);
#pragma unroll
        for (int g = 0; g < G; ++g) sc[g] = fmaf(qs[g][d], k0, fmaf(qs[g][d + 1], k1, sc[g]));
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    sc[g] += xor_partner<1>(sc[g], lane_id());
    sc[g] += xor_partner<2>(sc[g], lane_id());
  }
  if (p == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) ps[g][j] = kk < L ? sc[g] * scale : -INFINITY;
  }
  __syncthreads();

  // chunk softmax: wave w handles heads w, w + 4, ...
  const int wave = tid >> 6, lane = tid & 63;
  for (int g = wave; g < G; g += 4) {
    const float v = ps[g][lane];
    float m = v;
    m = wave_max(m);
    const float e = lane + t0 < L ? __expf(v - m) : 0.f;
    const float l = wave_sum(e);
    ps[g][lane] = e;
    if (lane == 0) {
      mls[g][0] = m;
      mls[g][1] = l;
    }
  }
  __syncthreads();

  // o[g][d] = sum_j p[g][j] v[j][d]; thread = (dim pair tid % 64, heads tid / 64, +4, ...)
  const int dp = tid & 63;
  const int nk = L - t0 < kChunk ? L - t0 : kChunk;
  const uint32_t* vr =
      reinterpret_cast<const uint32_t*>(vc + (((size_t)b * Hkv + kvh) * T + t0) * D) + dp;
  for (int g = wave; g < G; g += 4) {
    float o0 = 0.f, o1 = 0.f;
    for (int jj = 0; jj < nk; ++jj) {
      const uint32_t w = vr[(size_t)jj * (D / 2)];
      const float pj = ps[g][jj];
      o0 = fmaf(pj, bf16lo_to_f32(w), o0);
      o1 = fmaf(pj, bf16hi_to_f32(w), o1);
    }
    float* dst = part + (((size_t)bk * NC + c) * G + g) * (D + 2);
    dst[2 * dp] = o0;
    dst[2 * dp + 1] = o1;
    if (dp == 0) {
      dst[D] = mls[g][0];
      dst[D + 1] = mls[g][1];
    }
  }
}

// ---- decode attention, phase 2: merge chunks -> bf16 [B][1][H * D] ---------------------------
template <int G, int D>
__global__ __launch_bounds__(64) void attn_combine_kernel(const float* __restrict__ part,
                                                          const int64_t* __restrict__ pos,
                                                          uint16_t* __restrict__ out, int Hkv,
                                                          int NC) {
  const int bh = blockIdx.x;  // b * H + h
  const int H = Hkv * G;
  const int b = bh / H, h = bh % H, kvh = h / G, g = h % G;
  const int L = attn_len(pos[0], NC * kChunk);
  const int nc = (L + kChunk - 1) / kChunk < NC ? (L + kChunk - 1) / kChunk : NC;
  const float* base = part + ((size_t)(b * Hkv + kvh) * NC * G + g) * (D + 2);
  const size_t cstride = (size_t)G * (D + 2);
  float M = -INFINITY;
  for (int c = 0; c < nc; ++c) M = fmaxf(M, base[c * cstride + D]);
  const int dp = threadIdx.x;
  float o0 = 0.f, o1 = 0.f, l = 0.f;
  for (int c = 0; c < nc; ++c) {
    const float* pc = base + c * cstride;
    const float wgt = __expf(pc[D] - M);
    l = fmaf(pc[D + 1], wgt, l);
    o0 = fmaf(pc[2 * dp], wgt, o0);
    o1 = fmaf(pc[2 * dp + 1], wgt, o1);
  }
  const float inv = 1.f / l;
  reinterpret_cast<uint32_t*>(out)[((size_t)b * H + h) * (D / 2) + dp] =
      (uint32_t)f32_to_bf16(o0 * inv) | ((uint32_t)f32_to_bf16(o1 * inv) << 16);
}

// ---- decode attention in one launch (short caches): one workgroup per (batch, query head) -----
// NW waves (16; 8 measured 656 vs 682 tokens/s end to end); wave w takes keys w*16 + 16 NW i.
// Each K load instruction covers 8 keys x 128 B (whole cache lines; lane l: key t0 + 8 i + l / 8,
// dims 64 h + 8 (l % 8) ..; half-line loads moved half the bytes per instruction through the L2,
// profiles/r3_probe_l2_pattern.jsonl), and the 16 keys' V rows are loaded in the same round trip
// (lane = dim pair). The first step's K/V loads are issued before q's, so q (fresh from the wqkv
// kernel) and the first keys arrive together; later steps prefetch the next step's K/V before
// computing the current one. Online softmax per wave in fp32, waves merged through LDS. At
// T <= 1024 the chain is <= 4 round trips; longer caches take the two-kernel split above.
constexpr int kSingleMaxT = 1024;
constexpr int kSingleWaves = TAO_ATTN_WAVES;

// Scores by v_dot2_f32_bf16 on the packed bf16 q and k words (8 ops per key-lane instead of 16
// conversions + 16 fmas; the products are exact in fp32 either way) and the P.V weights
// broadcast by v_readlane (the source lane is uniform) instead of ds_bpermute shuffles: 3.65 /
// 5.52 / 6.54 / 9.85 us per graph launch at 128 / 328 / 512 / 900 keys against 3.80 / 5.63 /
// 7.04 / 10.20 for f32 conversions and shuffles (profiles/r4_attn_time_dot2.jsonl).
// SPLIT (tao_attn_decode_split_bf16): the same kernel over keys [lo, hi) of split blockIdx.y of
// gridDim.y (each split ceil(L / NS) keys rounded up to 16), writing the split's unnormalised
// partial instead of the bf16 output: part [B * H][NS][kPartStride] fp32 = o[D] (sum of
// exp(s - m) v over the split's keys), m, l. An empty split writes m = -inf, l = 0, o = 0.
constexpr int kPartStride = 132;  // o[128], m, l, 2 pad: 16-B aligned records

template <int D, int NW, bool SPLIT = false>
__global__ __launch_bounds__(NW * 64) void attn_single_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int64_t* __restrict__ pos, uint16_t* __restrict__ out,
    int H, int Hkv, int T, float scale, float* __restrict__ part) {
  static_assert(D == 128, "head_dim 128");
  __shared__ float wm[NW], wl[NW];
  __shared__ float wo[NW][D];
  // q [B][H][1][D]: the query at position pos[0] attends keys 0..pos[0]; out [B][1][H * D].
  // (Dealing the G query heads of one kv head to one XCD, so they share its L2 for their common
  // K/V rows, measured no faster: profiles/r4_attn_time_xcd.jsonl, r4_ab_e2e_attn_xcd.jsonl.)
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh % H, kvh = h / (H / Hkv);
  const int L = attn_len(pos[0], T);
  int lo = 0, hi = L;
  if constexpr (SPLIT) {
    const int NS = gridDim.y, C = ((L + NS - 1) / NS + 15) & ~15;
    lo = (int)blockIdx.y * C;
    hi = lo + C < L ? lo + C : L;
    if (lo >= hi) {  // no keys in this split (uniform): the empty partial
      float* pr = part + ((size_t)bh * NS + blockIdx.y) * kPartStride;
      if (threadIdx.x < D) pr[threadIdx.x] = 0.f;
      if (threadIdx.x == D) pr[D] = -INFINITY;
      if (threadIdx.x == D + 1) pr[D + 1] = 0.f;
      return;
    }
  }
  const size_t ooff = (size_t)bh * (D / 2);  // output dword offset
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const size_t head = (size_t)(b * Hkv + kvh) * T;
  const uint32_t* vb = reinterpret_cast<const uint32_t*>(vc + head * D) + lane;
  // lane (g = l / 8, p8 = l % 8): keys t0 + g and t0 + 8 + g, dims 64 h + 8 p8 + e (h < 2, e < 8)
  const int g = lane >> 3, p8 = lane & 7;
  const uint16_t* kbase = kc + head * D + p8 * 8;
  uint4 ka[2], kb2[2];
  uint32_t vv[16];
  auto load_step = [&](int t0) __attribute__((always_inline)) {
    const int ta = t0 + g < hi ? t0 + g : hi - 1, tb = t0 + 8 + g < hi ? t0 + 8 + g : hi - 1;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      ka[hh] = *reinterpret_cast<const uint4*>(kbase + (size_t)ta * D + 64 * hh);
      kb2[hh] = *reinterpret_cast<const uint4*>(kbase + (size_t)tb * D + 64 * hh);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int tj = t0 + j < hi ? t0 + j : hi - 1;
      vv[j] = vb[(size_t)tj * (D / 2)];
    }
  };
  load_step(lo + wave * 16);
  uint32_t qw[8];
  {
    const uint4* qp = reinterpret_cast<const uint4*>(q + (size_t)bh * D + p8 * 8);
    uint4 qv[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) qv[hh] = qp[hh * 8];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint32_t w[4] = {qv[hh].x, qv[hh].y, qv[hh].z, qv[hh].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        qw[hh * 4 + e] = w[e];
      }
    }
  }
  float m = -INFINITY, l = 0.f, o0 = 0.f, o1 = 0.f;
  for (int t0 = lo + wave * 16; t0 < hi; t0 += NW * 16)
    attn_decode_step(qw, ka, kb2, vv, t0, hi, g, scale, m, l, o0, o1, [&]() {
      if (t0 + NW * 16 < hi) load_step(t0 + NW * 16);  // wave-uniform prefetch of the next step
    });
  if (lane == 0) {
    wm[wave] = m;
    wl[wave] = l;
  }
  wo[wave][2 * lane] = o0;
  wo[wave][2 * lane + 1] = o1;
  __syncthreads();
  if (wave == 0) {
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w]);
    float a0 = 0.f, a1 = 0.f, ls = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = wm[w] == -INFINITY ? 0.f : __expf(wm[w] - M);  // waves with no keys
      ls = fmaf(wl[w], f, ls);
      a0 = fmaf(wo[w][2 * lane], f, a0);
      a1 = fmaf(wo[w][2 * lane + 1], f, a1);
    }
    if constexpr (SPLIT) {
      float* pr = part + ((size_t)bh * gridDim.y + blockIdx.y) * kPartStride;
      reinterpret_cast<float2*>(pr)[lane] = make_float2(a0, a1);
      if (lane == 0) reinterpret_cast<float2*>(pr + D)[0] = make_float2(M, ls);
    } else {
      const float inv = 1.f / ls;
      reinterpret_cast<uint32_t*>(out)[ooff + lane] =
          (uint32_t)f32_to_bf16(a0 * inv) | ((uint32_t)f32_to_bf16(a1 * inv) << 16);
    }
  }
}

// ---- merge of the split partials -> bf16 [B][1][H * D] (tao_attn_merge_bf16) --------------------
// One wave per (batch, head), lane = dim pair; attn_merge_pair is also the x prologue of the wo
// GEMV (int4_gemv.hip, tao_int4wo_attn_out_bf16), so both give the same bits.
template <int NS>
__global__ __launch_bounds__(64) void attn_merge_kernel(const float* __restrict__ part,
                                                        uint32_t* __restrict__ out) {
  const float* pr = part + (size_t)blockIdx.x * NS * kPartStride;
  float2 ml[NS], o[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    ml[s] = reinterpret_cast<const float2*>(pr + s * kPartStride + 128)[0];
    o[s] = reinterpret_cast<const float2*>(pr + s * kPartStride)[threadIdx.x];
  }
  float wgt[NS], inv;
  attn_merge_weights<NS>(ml, wgt, inv);
  float r0 = 0.f, r1 = 0.f;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    r0 = fmaf(o[s].x, wgt[s], r0);
    r1 = fmaf(o[s].y, wgt[s], r1);
  }
  out[(size_t)blockIdx.x * 64 + threadIdx.x] =
      (uint32_t)f32_to_bf16(r0 * inv) | ((uint32_t)f32_to_bf16(r1 * inv) << 16);
}

// ---- SiLU(a) * b ----------------------------------------------------------------------------
__device__ __forceinline__ uint16_t silu_mul1(float v, float m) {
  return f32_to_bf16(round_bf16(v / (1.f + __expf(-v))) * m);
}

// b == nullptr: a holds interleaved (gate, up) pairs, the row order of an interleaved w13.
__global__ __launch_bounds__(256) void silu_mul_kernel(const uint32_t* __restrict__ a,
                                                       const uint32_t* __restrict__ b,
                                                       uint32_t* __restrict__ y, int64_t n2) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    uint32_t x, z;
    if (b != nullptr) {
      x = a[i];
      z = b[i];
    } else {
      const uint2 p = reinterpret_cast<const uint2*>(a)[i];  // (g0, u0), (g1, u1)
      x = (p.x & 0xFFFFu) | (p.y << 16);
      z = (p.x >> 16) | (p.y & 0xFFFF0000u);
    }
    y[i] = (uint32_t)silu_mul1(bf16lo_to_f32(x), bf16lo_to_f32(z)) |
           ((uint32_t)silu_mul1(bf16hi_to_f32(x), bf16hi_to_f32(z)) << 16);
  }
}

// ---- greedy argmax over bf16 logits: one workgroup per row ------------------------------------
// bf16 bits b -> signed 16-bit key b ^ (b < 0 ? 0x7FFF : 0), order-preserving (positive-sign NaN
// above +inf, as torch.argmax ranks NaN the maximum; a negative-sign NaN ranks below -inf). Per
// round each thread takes 8 x 16 B: packed v_pk_max_i16 over its words, then a second pass over
// the same registers finds the first index holding that key; across rounds and threads the
// 64-bit (key, ~index) maximum keeps torch's first-index tie rule.
typedef short s16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2_t argmax_keys(uint32_t w) {
  const s16x2_t v = __builtin_bit_cast(s16x2_t, w);
  return v ^ ((v >> (short)15) & (short)0x7FFF);
}

__device__ __forceinline__ uint64_t pack_key(int k, uint32_t idx) {
  return ((uint64_t)(uint32_t)(k + 32768) << 32) | (uint32_t)~idx;
}

__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// With `pos` set (one row): also the decode loop's bookkeeping in the same launch: out (the
// graph's current-token buffer) = the argmax, tokens[pos + 1] = it, pos += 1 (GraphDecoder's
// pos.add_ / tokens.index_copy_ / cur.copy_, three launches, torchao/_models/llama/generate.py).
__global__ __launch_bounds__(1024) void argmax_kernel(const uint16_t* __restrict__ x,
                                                      int64_t* __restrict__ out, int64_t n,
                                                      int64_t* __restrict__ pos,
                                                      int64_t* __restrict__ tokens,
                                                      int64_t max_len) {
  __shared__ uint64_t red[16];
  const uint16_t* row = x + (size_t)blockIdx.x * n;
  uint64_t best = 0;
  const int64_t nv = ((reinterpret_cast<uintptr_t>(row) & 15) == 0) ? n / 8 : 0;
  const uint4* rv = reinterpret_cast<const uint4*>(row);
  constexpr int U = 8;  // 16-B loads in flight per thread per round (a 128K-vocab row: 2 rounds)
  for (int64_t base = 0; base < nv; base += U * 1024) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 1024 + threadIdx.x;
      v[u] = rv[i < nv ? i : nv - 1];  // clamped: a duplicate never beats the first index
    }
    s16x2_t mx = {(short)-32768, (short)-32768};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      mx = __builtin_elementwise_max(mx, argmax_keys(v[u].x));
      mx = __builtin_elementwise_max(mx, argmax_keys(v[u].y));
      mx = __builtin_elementwise_max(mx, argmax_keys(v[u].z));
      mx = __builtin_elementwise_max(mx, argmax_keys(v[u].w));
    }
    const int km = mx.x > mx.y ? mx.x : mx.y;
    uint32_t first = 0xFFFFFFFFu;
#pragma unroll
    for (int u = U - 1; u >= 0; --u) {  // descending, so the last hit written is the first index
      const int64_t i = base + u * 1024 + threadIdx.x;
      const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        const s16x2_t k = argmax_keys(d[j]);
        const uint32_t e = (uint32_t)(i * 8 + 2 * j);
        first = (int)k.y == km ? e + 1 : first;
        first = (int)k.x == km ? e : first;
      }
    }
    best = umax64(best, pack_key(km, first));
  }
  for (int64_t i = nv * 8 + threadIdx.x; i < n; i += 1024) {  // tail (or unaligned rows)
    const s16x2_t k = argmax_keys(row[i]);
    best = umax64(best, pack_key(k.x, (uint32_t)i));
  }
  best = wave_bfly<1, 64>(best, lane_id(), umax64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = umax64(best, red[w]);
    const int64_t idx = (int64_t)(uint32_t)~(uint32_t)best;
    out[blockIdx.x] = idx;
    if (pos != nullptr) {
      const int64_t p = pos[0] + 1;
      if (p >= 0 && p < max_len) tokens[p] = idx;
      pos[0] = p;
    }
  }
}

}  // namespace
}  // namespace tao

using namespace tao;

extern "C" {

int tao_rmsnorm_bf16(const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t rows,
                     int64_t dim, float eps, void* stream) {
  TAO_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0 && dim < (1 << 24),
                "rmsnorm: dim (%lld) must be a positive multiple of 8", (long long)dim);
  if (rows == 0) return TAO_OK;
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(y, 16, "y");
  launch_rmsnorm<false>(x, nullptr, w, nullptr, y, rows, dim, eps, as_stream(stream));
  return check_launch("rmsnorm_kernel");
}

int tao_add_rmsnorm_bf16(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* h,
                         uint16_t* y, int64_t rows, int64_t dim, float eps, void* stream) {
  TAO_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0 && dim < (1 << 24),
                "add_rmsnorm: dim (%lld) must be a positive multiple of 8", (long long)dim);
  if (rows == 0) return TAO_OK;
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(res, 16, "res");
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(h, 16, "h");
  TAO_CHECK_ALIGN(y, 16, "y");
  launch_rmsnorm<true>(x, res, w, h, y, rows, dim, eps, as_stream(stream));
  return check_launch("add_rmsnorm_kernel");
}

int tao_add_rmsnorm_partials_bf16(const uint16_t* x, const float* part, int64_t splits,
                                  const uint16_t* w, uint16_t* h, uint16_t* y, int64_t rows,
                                  int64_t dim, float eps, void* stream) {
  TAO_CHECK_ARG(rows >= 0 && dim > 0 && dim % 8 == 0 && dim <= 8192,
                "add_rmsnorm_partials: dim (%lld) must be a positive multiple of 8, <= 8192",
                (long long)dim);
  TAO_CHECK_ARG(splits >= 1 && splits <= 64, "add_rmsnorm_partials: splits (%lld) out of range",
                (long long)splits);
  if (rows == 0) return TAO_OK;
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(part, 16, "part");
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(h, 16, "h");
  TAO_CHECK_ALIGN(y, 16, "y");
  const dim3 grid((unsigned)rows), blk(256);
  const int D = (int)dim, nv = D / 8, S = (int)splits;
  const size_t plane = (size_t)rows * dim;
  hipStream_t st = as_stream(stream);
#define TAO_PART(NP)                                                                          \
  switch (S) {                                                                                \
    case 2: launch(rmsnorm_part_kernel<NP, 2>, grid, blk, 0, st, x, part, S, plane, w, h, y, D, eps); break; \
    case 4: launch(rmsnorm_part_kernel<NP, 4>, grid, blk, 0, st, x, part, S, plane, w, h, y, D, eps); break; \
    case 8: launch(rmsnorm_part_kernel<NP, 8>, grid, blk, 0, st, x, part, S, plane, w, h, y, D, eps); break; \
    default: launch(rmsnorm_part_kernel<NP, 0>, grid, blk, 0, st, x, part, S, plane, w, h, y, D, eps); \
  }
  if (nv <= 256) TAO_PART(1)
  else if (nv <= 512) TAO_PART(2)
  else TAO_PART(4)
#undef TAO_PART
  return check_launch("rmsnorm_part_kernel");
}

int tao_rope_kv_bf16(const uint16_t* qkv, const float* freqs, const int64_t* pos,
                     uint16_t* q_out, uint16_t* k_cache, uint16_t* v_cache, int64_t B, int64_t S,
                     int64_t H, int64_t Hkv, int64_t D, int64_t T, void* stream) {
  TAO_CHECK_ARG(B > 0 && S > 0 && H > 0 && Hkv > 0 && H % Hkv == 0 && D % 2 == 0 && T >= S,
                "rope_kv: bad sizes");
  TAO_CHECK_ALIGN(qkv, 4, "qkv");
  launch(rope_kv_kernel, dim3((unsigned)(B * S)), dim3(256), 0, as_stream(stream), qkv, freqs,
         pos, q_out, k_cache, v_cache, (int)S, (int)H, (int)Hkv, (int)D, (int)T);
  return check_launch("rope_kv_kernel");
}

static int attn_decode(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                       const int64_t* pos, float* partial, uint16_t* out, int64_t B, int64_t H,
                       int64_t Hkv, int64_t D, int64_t T, float scale, void* stream) {
  TAO_CHECK_ARG(D == 128, "attn_decode: head_dim must be 128 (got %lld)", (long long)D);
  TAO_CHECK_ARG(B > 0 && Hkv > 0 && H % Hkv == 0 && T > 0, "attn_decode: bad sizes");
  const int G = (int)(H / Hkv);
  TAO_CHECK_ARG(G == 1 || G == 2 || G == 4 || G == 8, "attn_decode: H / Hkv must be 1, 2, 4 or 8");
  TAO_CHECK_ALIGN(k_cache, 16, "k_cache");
  TAO_CHECK_ALIGN(q, 16, "q");
  hipStream_t st = as_stream(stream);
  const int mode = tao::tuning().attn_mode;
  // Single pass, a workgroup per query head, whole-line K loads (per graph launch 3.92 / 5.63 /
  // 7.06 / 10.21 us at 128 / 328 / 512 / 900 keys: profiles/r3_attn_time_fullk.jsonl)
  if (T <= kSingleMaxT && mode == 0) {
    launch((attn_single_kernel<128, kSingleWaves>), dim3((unsigned)(B * H)),
           dim3(64 * kSingleWaves), 0, st, q, k_cache, v_cache, pos, out, (int)H, (int)Hkv,
           (int)T, scale, nullptr);
    return check_launch("attn_single_kernel");
  }

  const int NC = (int)((T + kChunk - 1) / kChunk);
  const dim3 g1((unsigned)(B * Hkv), (unsigned)NC), g2((unsigned)(B * H));
  if (partial == nullptr) {  // the library's workspace
    void* ws = nullptr;
    unsigned* cnt = nullptr;
    const int rc = split_workspace(st, (size_t)B * Hkv * NC * G * (D + 2) * sizeof(float), 1,
                                   &ws, &cnt);
    if (rc != TAO_OK) return rc;
    partial = reinterpret_cast<float*>(ws);
  }
  switch (G) {
#define TAO_ATTN(GG)                                                                          \
  case GG:                                                                                    \
    launch(attn_partial_kernel<GG, 128>, g1, dim3(256), 0, st, q, k_cache, v_cache, pos,      \
           partial, (int)Hkv, (int)T, scale);                                                 \
    launch(attn_combine_kernel<GG, 128>, g2, dim3(64), 0, st, partial, pos, out, (int)Hkv, NC); \
    break;
    TAO_ATTN(1)
    TAO_ATTN(2)
    TAO_ATTN(4)
    TAO_ATTN(8)
#undef TAO_ATTN
  }
  return check_launch("attn_decode");
}

int tao_attn_prefill_bf16(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                          const int64_t* pos, uint16_t* out, int64_t B, int64_t H, int64_t Hkv,
                          int64_t D, int64_t S, int64_t T, float scale, void* stream) {
  TAO_CHECK_ARG(D == 128, "attn_prefill: head_dim must be 128 (got %lld)", (long long)D);
  TAO_CHECK_ARG(B > 0 && Hkv > 0 && H % Hkv == 0 && T > 0 && S > 0 && B * H * S < (1LL << 31),
                "attn_prefill: bad sizes");
  TAO_CHECK_ALIGN(q, 16, "q");
  TAO_CHECK_ALIGN(k_cache, 16, "k_cache");
  TAO_CHECK_ALIGN(v_cache, 16, "v_cache");  // V rows are read with 16-B vector loads
  TAO_CHECK_ALIGN(out, 16, "out");
  TAO_CHECK_ARG(B * H <= 65535, "attn_prefill: B * H (%lld) exceeds the grid's y extent",
                (long long)(B * H));
  // MFMA flash-style kernel (attn_mfma.hip): 1-4 waves per 16 queries (key blocks split over
  // them, merged in LDS), K / V read once per block of
  // 16 queries instead of once per query (the single-pass decode kernel generalised, which this
  // replaces, re-read the prefix per query: 24 us per layer at S = 128)
  return tao::attn_prefill_mfma(q, k_cache, v_cache, pos, out, B, H, Hkv, S, T, scale,
                                as_stream(stream));
}

int tao_attn_decode_bf16(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                         const int64_t* pos, float* partial, uint16_t* out, int64_t B, int64_t H,
                         int64_t Hkv, int64_t D, int64_t T, float scale, void* stream) {
  return attn_decode(q, k_cache, v_cache, pos, partial, out, B, H, Hkv, D, T, scale, stream);
}

int tao_attn_decode_split_bf16(const uint16_t* q, const uint16_t* k_cache,
                               const uint16_t* v_cache, const int64_t* pos, float* partial,
                               int64_t B, int64_t H, int64_t Hkv, int64_t D, int64_t T, float scale,
                               int64_t splits, void* stream) {
  TAO_CHECK_ARG(D == 128, "attn_decode_split: head_dim must be 128 (got %lld)", (long long)D);
  TAO_CHECK_ARG(B > 0 && Hkv > 0 && H % Hkv == 0 && T > 0 && B * H < (1LL << 31),
                "attn_decode_split: bad sizes");
  TAO_CHECK_ARG(splits == 2 || splits == 4, "attn_decode_split: splits must be 2 or 4 (got %lld)",
                (long long)splits);
  TAO_CHECK_ARG(partial != nullptr, "attn_decode_split: partial is required");
  TAO_CHECK_ALIGN(q, 16, "q");
  TAO_CHECK_ALIGN(k_cache, 16, "k_cache");
  TAO_CHECK_ALIGN(v_cache, 4, "v_cache");
  TAO_CHECK_ALIGN(partial, 16, "partial");
  launch((attn_single_kernel<128, kSingleWaves, true>), dim3((unsigned)(B * H), (unsigned)splits),
         dim3(64 * kSingleWaves), 0, as_stream(stream), q, k_cache, v_cache, pos, nullptr,
         (int)H, (int)Hkv, (int)T, scale, partial);
  return check_launch("attn_split_kernel");
}

int tao_attn_merge_bf16(const float* partial, uint16_t* out, int64_t B, int64_t H, int64_t D,
                        int64_t splits, void* stream) {
  TAO_CHECK_ARG(D == 128, "attn_merge: head_dim must be 128 (got %lld)", (long long)D);
  TAO_CHECK_ARG(B > 0 && H > 0 && B * H < (1LL << 31), "attn_merge: bad sizes");
  TAO_CHECK_ARG(splits == 2 || splits == 4, "attn_merge: splits must be 2 or 4 (got %lld)",
                (long long)splits);
  TAO_CHECK_ALIGN(partial, 16, "partial");
  TAO_CHECK_ALIGN(out, 4, "out");
  hipStream_t st = as_stream(stream);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  if (splits == 2) launch(attn_merge_kernel<2>, dim3((unsigned)(B * H)), dim3(64), 0, st, partial, o);
  else launch(attn_merge_kernel<4>, dim3((unsigned)(B * H)), dim3(64), 0, st, partial, o);
  return check_launch("attn_merge_kernel");
}

int tao_tune_attn(int mode) {
  TAO_CHECK_ARG(mode == 0 || mode == 1,
                "tune: attention mode must be 0 (auto: single pass up to 1024 keys, else split) "
                "or 1 (two-launch split)");
  tao::tuning().attn_mode = mode;
  return TAO_OK;
}

int tao_silu_mul_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, int64_t n,
                      void* stream) {
  TAO_CHECK_ARG(n >= 0 && n % 2 == 0, "silu_mul: n (%lld) must be even", (long long)n);
  if (n == 0) return TAO_OK;
  TAO_CHECK_ALIGN(a, b != nullptr ? 4 : 8, "a");
  TAO_CHECK_ALIGN(b, 4, "b");
  const int64_t n2 = n / 2;
  int64_t grid = (n2 + 255) / 256;
  if (grid > 4096) grid = 4096;
  launch(silu_mul_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream),
         reinterpret_cast<const uint32_t*>(a), reinterpret_cast<const uint32_t*>(b),
         reinterpret_cast<uint32_t*>(y), n2);
  return check_launch("silu_mul_kernel");
}

int tao_argmax_bf16(const uint16_t* x, int64_t* out, int64_t rows, int64_t n, void* stream) {
  TAO_CHECK_ARG(rows >= 0 && n > 0 && n < (1LL << 31), "argmax: n (%lld) must be in [1, 2^31)",
                (long long)n);
  if (rows == 0) return TAO_OK;
  TAO_CHECK_ALIGN(x, 2, "x");
  launch(argmax_kernel, dim3((unsigned)rows), dim3(1024), 0, as_stream(stream), x, out, n,
         (int64_t*)nullptr, (int64_t*)nullptr, (int64_t)0);
  return check_launch("argmax_kernel");
}

}  // extern "C"

extern "C" int tao_argmax_advance_bf16(const uint16_t* x, int64_t n, int64_t* cur, int64_t* pos,
                                       int64_t* tokens, int64_t max_len, void* stream) {
  TAO_CHECK_ARG(x && cur && pos && tokens && n > 0 && n < (1LL << 31) && max_len > 0,
                "argmax_advance: bad arguments");
  launch(argmax_kernel, dim3(1), dim3(1024), 0, as_stream(stream), x, cur, n, pos, tokens,
         max_len);
  return check_launch("argmax_kernel (advance)");
}

extern "C" int tao_decode_status(int* bits) {
  TAO_CHECK_ARG(bits != nullptr, "decode status: null output");
  unsigned v = 0;
  int rc = tao::decode_ops_status(&v);
  if (rc == TAO_OK) rc = tao::int4gemv_decode_status(&v);
  if (rc == TAO_OK) rc = tao::int8gemv_decode_status(&v);
  if (rc == TAO_OK) rc = tao::int8dyn_decode_status(&v);
  if (rc == TAO_OK) rc = tao::sf_decode_status(&v);
  if (rc == TAO_OK) rc = tao::engine_decode_status(&v);
  unsigned to = 0;  // split-K reducer timeouts of the single-fetch GEMMs (prefill)
  if (rc == TAO_OK) rc = tao_gemm_sf_status(&to);
  if (to != 0) v |= tao::kDecodeErrSplitK;
  *bits = (int)v;
  return rc;
}
