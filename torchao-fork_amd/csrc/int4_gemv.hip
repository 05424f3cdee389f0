// int4 group-quantised weight-only linear, skinny-M (decode) path: y[M][N] = x[M][K] W^T.
//
// Replaces aten._weight_int4pack_mm at torchao/dtypes/uintx/tensor_core_tiled_layout.py:104
// for skinny M: the built-in crossover (gemm_mfma.hip use_gemv) sends M <= 2, or M <= 4 for
// weights of at most 32 Mi elements, here; the kernel itself is instantiated up to M = 8, the
// cap of tao_tune_linear_crossover. HBM-bound: every packed weight byte and every (scale, zero)
// pair is read exactly once, with 16-B non-temporal loads; x (<= 8 x K bf16) stays in L1/L2.
//
// Work decomposition:
//   * a "slice" is 2048 consecutive k of one row = 64 lanes x 32 k = one 1-KiB wave load
//     (16 B of nibbles per lane) + one 256-B (scale, zero) load at group size 32;
//   * a wave owns RPW rows and one slice at a time; a workgroup is G row-groups x Wk waves along
//     K (Wk = min(slices, 8)); slices beyond Wk are looped;
//   * per lane: D = sum x*(128+q) via v_dot2c_f32_bf16 on magic-number bf16 pairs (formed by
//     byte permutes: 7 VALU per 8 weights), Sx = sum x, then s*(D - 136 Sx) + z*Sx per 32-k chunk —
//     every 32-k chunk lies in exactly one quantisation group because g in {32..256};
//   * cross-lane: reduce-scatter over the RPW*M partials (V/2 + V/4 + ... shuffles), then a
//     butterfly over the remaining lanes; cross-wave: LDS, one wave finishes and writes y.
#include <atomic>
#include <type_traits>

#include "tao_common.h"
#include "tao_attn.h"
#include "tao_reduce.h"

// The timing-only variant builds of rounds 1-5 (no x loads, no arithmetic, no (scale, zero)
// loads, no reduction, per-workgroup s_memrealtime stamps, the RMSNorm-prologue variants and the
// both-slices-issued XPRE order) lived in this file behind TAO_GEMV_DEBUG /
// TAO_GEMV_STAMPS / TAO_NORM_DEBUG / GEMV_XPRE up to commit 1bac331; their measurements are in
// profiles/ (r1_gemv_debug*.log, r2/r5g_gemv_stamps.jsonl, r5g_ab_gemv_*.jsonl).

namespace tao {

TAO_DECODE_ERROR_WORD(int4gemv_decode_status)

namespace {

// Decode-step fusions of the M == 1 GEMV (tao_int4wo_decode_bf16). They fold
// the small ops around a Llama block's linears into the linear itself, so a decode token costs
// fewer launches; each keeps the unfused kernels' op order and bf16 roundings
// (decode_ops.hip: rmsnorm_kernel, silu_mul_kernel, rope_kv_kernel).
//   PRO         x -> bf16(bf16(x * rsqrt(mean(x^2) + eps)) * norm_w) on the fly (RMSNorm,
//               reference torchao/_models/llama/model.py RMSNorm.forward);
//   kEpiSwiGLU  rows (2i, 2i+1) hold (w1_i, w3_i): y[i] = bf16(bf16(silu(a)) * b);
//   kEpiRopeKV  rows = [q | k | v] heads of wqkv: q rotated into y, k rotated and v stored
//               into the caches at pos[0] (Attention.forward + KVCache.update).
enum { kEpiNone = 0, kEpiSwiGLU = 1, kEpiRopeKV = 2 };
constexpr int kMaxNormPT = 4;  // max 16-B pieces of x per thread in the RMSNorm prologue
struct GemvFuse {
  const uint16_t* norm_w;  // [K] RMSNorm weight (PRO)
  float eps;
  const float* freqs;      // [T][D/2] (cos, sin) pairs (kEpiRopeKV)
  const int64_t* pos;
  uint16_t* k_cache;       // [Hkv][T][D]
  uint16_t* v_cache;
  int H, Hkv, D, T;
  int norm_deferred;  // PRO: 1 = stage bf16(x * w) and scale the outputs by r (see norm_finish)
  const float* merge;  // MRG: split attention partials [H][MRG][132] (tao_attn_decode_split_bf16)
};

__device__ __forceinline__ uint32_t mul_pair_bf16(uint32_t xv, uint32_t wv) {
  const float lo = bf16lo_to_f32(xv) * bf16lo_to_f32(wv);
  const float hi = bf16hi_to_f32(xv) * bf16hi_to_f32(wv);
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

__device__ __forceinline__ uint32_t rmsnorm_pair(uint32_t xv, uint32_t wv, float r) {
  const float lo = round_bf16(bf16lo_to_f32(xv) * r) * bf16lo_to_f32(wv);
  const float hi = round_bf16(bf16hi_to_f32(xv) * r) * bf16hi_to_f32(wv);
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// WPE: minimum waves per SIMD the register allocation must allow (8 -> <= 64 VGPRs, so four
// 512-thread workgroups fit on a CU and mid-size grids run in a single resident round).
// NPT > 0 enables the RMSNorm prologue with NPT 16-B pieces of x per thread (PRO).
// MRG > 0 (with NPT): x is the merge of MRG split-attention partials per head (fu.merge; head_dim
// 128), formed in the prologue instead of the RMSNorm: tao_int4wo_attn_out_bf16.
// The body of one workgroup: rows row_base + rg RPW .. of row group rg (int4wo_gemv_kernel
// calls it).
// COH (tao_int4wo_qkv_attn_bf16): the RoPE epilogue's q and cache stores are agent-scope (sc1)
// stores, read by the same launch's attention workgroups after their ticket wait.
__device__ __forceinline__ void st_coh(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_coh(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MT, int RPW, bool PAIR, int NPT = 0, int EPI = kEpiNone, int MRG = 0,
          bool COH = false>
__device__ __forceinline__ void gemv_body(
    const uint16_t* __restrict__ x, const uint4* __restrict__ wq, const uint32_t* __restrict__ sz,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K, int gshift,
    int Wk, int G, int S, const GemvFuse& fu, int row_base) {
  constexpr bool PRO = NPT > 0;
  static_assert(MRG == 0 || (PRO && EPI == kEpiNone && MT == 1), "merge prologue: M == 1, NPT");
  static_assert(!(PRO || EPI) || (MT == 1 && RPW % 2 == 0), "fusions are M == 1, row pairs");
  constexpr int V = RPW * MT;
  extern __shared__ float red[];  // [G][Wk][V] (PRO: + [8] partial sums, + normalised x [K])
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int wk = wave % Wk;
  const int rg = wave / Wk;
  const int row0 = row_base + rg * RPW;
  const int nchunk = K >> 5;               // 32-k chunks per row
  const int ngroups = K >> (5 + gshift);   // quantisation groups per row

  float acc[RPW][MT];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[r][m] = 0.f;

  // RMSNorm prologue (PRO): the workgroup normalises x once into LDS. Each thread loads its
  // NPT 16-B pieces of x and of the norm weight (the launcher guarantees
  // K <= 8 * NPT * blockDim.x) BEFORE its first slice's weight loads, so the in-order vmcnt
  // wait for them does not wait for the weights: the sum of squares, the two barriers (reached
  // exactly once by every wave) and the LDS fill all run under the weight-load latency.
  // LDS copy: chunk c (32 k) keeps its four 16-B pieces rotated by c >> 2, so the 16 lanes of a
  // ds_read_b128 pass (consecutive chunks) hit 16 distinct 16-B bank groups.
  uint4* xs = reinterpret_cast<uint4*>(red + ((G * Wk * V + 8 + 3) & ~3));
  uint4 xv[NPT > 0 ? NPT : 1], gv[NPT > 0 ? NPT : 1];
  // MRG: piece i (x[8i .. 8i + 8)) of head i / 16 from the MRG partial records of that head
  constexpr int kMS = MRG > 0 ? MRG : 1;
  float2 mlv[NPT > 0 ? NPT : 1][kMS];
  float4 ov[NPT > 0 ? NPT : 1][kMS][2];
  auto norm_load = [&]() __attribute__((always_inline)) {
    if constexpr (MRG > 0) {
      const int nx = K >> 3;
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int i = threadIdx.x + u * (int)blockDim.x;
        const int ic = i < nx ? i : nx - 1;  // clamped, masked in norm_finish
        const float* rec = fu.merge + (size_t)(ic >> 4) * MRG * 132;  // head ic / 16
        const int d0 = (ic & 15) << 3;
#pragma unroll
        for (int s = 0; s < MRG; ++s) {
          mlv[u][s] = *reinterpret_cast<const float2*>(rec + s * 132 + 128);
          ov[u][s][0] = *reinterpret_cast<const float4*>(rec + s * 132 + d0);
          ov[u][s][1] = *reinterpret_cast<const float4*>(rec + s * 132 + d0 + 4);
        }
      }
      return;
    }
    const uint4* xr = reinterpret_cast<const uint4*>(x);
    const uint4* gr = reinterpret_cast<const uint4*>(fu.norm_w);
    const int nx = K >> 3;
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      const int ic = i < nx ? i : nx - 1;  // clamped, masked below
      xv[u] = xr[ic];
      if (fu.norm_w != nullptr) gv[u] = gr[ic];  // wave-uniform
    }
  };
  auto norm_finish = [&]() __attribute__((always_inline)) {
    const int nx = K >> 3;
    if constexpr (MRG > 0) {  // x = the merged attention output, bf16, as attn_merge_kernel
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int i = threadIdx.x + u * (int)blockDim.x;
        float wgt[MRG], inv;
        attn_merge_weights<MRG>(mlv[u], wgt, inv);
        float r[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = 0.f;
#pragma unroll
        for (int s = 0; s < MRG; ++s) {
          const float4 a = ov[u][s][0], c = ov[u][s][1];
          r[0] = fmaf(a.x, wgt[s], r[0]);
          r[1] = fmaf(a.y, wgt[s], r[1]);
          r[2] = fmaf(a.z, wgt[s], r[2]);
          r[3] = fmaf(a.w, wgt[s], r[3]);
          r[4] = fmaf(c.x, wgt[s], r[4]);
          r[5] = fmaf(c.y, wgt[s], r[5]);
          r[6] = fmaf(c.z, wgt[s], r[6]);
          r[7] = fmaf(c.w, wgt[s], r[7]);
        }
        uint32_t pw[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          pw[e] = (uint32_t)f32_to_bf16(r[2 * e] * inv) |
                  ((uint32_t)f32_to_bf16(r[2 * e + 1] * inv) << 16);
        if (i < nx) {
          const int c = i >> 2;
          xs[c * 4 + (((i & 3) + (c >> 2)) & 3)] = make_uint4(pw[0], pw[1], pw[2], pw[3]);
        }
      }
      __syncthreads();
      return;
    }
    if (fu.norm_w == nullptr) {  // plain x staged in LDS (tao_tune_int4_xlds), no RMSNorm
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int i = threadIdx.x + u * (int)blockDim.x;
        if (i < nx) {
          const int c = i >> 2;
          xs[c * 4 + (((i & 3) + (c >> 2)) & 3)] = xv[u];
        }
      }
      __syncthreads();
      return;
    }
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
    float* ssr = red + G * Wk * V;
    if (lane == 0) ssr[wave] = ss;
    if (fu.norm_deferred) {
      // Deferred normalisation (tao_tune_int4_norm 1): r = rsqrt(mean(x^2) + eps) is one scalar
      // per token, so stage bf16(x * w) now and multiply each output by r at the end. One
      // barrier, no wait for the cross-wave sum before the slices; one bf16 rounding of the
      // normalised input instead of the reference's two (bf16(bf16(x * r) * w)).
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int i = threadIdx.x + u * (int)blockDim.x;
        if (i < nx) {
          const int c = i >> 2;
          xs[c * 4 + (((i & 3) + (c >> 2)) & 3)] =
              make_uint4(mul_pair_bf16(xv[u].x, gv[u].x), mul_pair_bf16(xv[u].y, gv[u].y),
                         mul_pair_bf16(xv[u].z, gv[u].z), mul_pair_bf16(xv[u].w, gv[u].w));
        }
      }
      __syncthreads();
      return;
    }
    __syncthreads();
    float t = 0.f;
    for (int w = 0; w < G * Wk; ++w) t += ssr[w];
    const float r = rsqrtf(t / (float)K + fu.eps);
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = threadIdx.x + u * (int)blockDim.x;
      if (i < nx) {
        const int c = i >> 2;
        xs[c * 4 + (((i & 3) + (c >> 2)) & 3)] =
            make_uint4(rmsnorm_pair(xv[u].x, gv[u].x, r), rmsnorm_pair(xv[u].y, gv[u].y, r),
                       rmsnorm_pair(xv[u].z, gv[u].z, r), rmsnorm_pair(xv[u].w, gv[u].w, r));
      }
    }
    __syncthreads();
  };

  // PAIR (waves owning >= 2 slices): slices are processed two at a time, both slices' weight
  // and (scale, zero) loads issued before either is consumed, so a wave walking two slices pays
  // one memory round trip, not two.
  auto load_slice = [&](int s, uint4 (&wv)[RPW], uint32_t (&szv)[RPW], int& cc,
                        bool& cval) __attribute__((always_inline)) {
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
  auto do_slice = [&](const uint4 (&wv)[RPW], const uint32_t (&szv)[RPW],
                      int cc, bool cval) __attribute__((always_inline)) {
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
        const uint4 t4 = PRO ? xs[cc * 4 + ((j + (cc >> 2)) & 3)] : xp[j];
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
        for (int j = 0; j < 4; ++j) {
          // byte-permute decode (tao_common.h): the same bf16 pairs in 7 VALU instead of 11;
          // bench step 1.098 / 1.116 -> 1.074 / 1.089 ms, 4096x14336 9.3 -> 8.8 us, 28672x4096
          // 14.8 -> 14.1 us (same-box A/B, profiles/r6k_ab_gemv_nibperm.jsonl)
          uint32_t p[4];
          nib_pairs4_bf16(wd[j], p);
#pragma unroll
          for (int i = 0; i < 4; ++i) d = dot2_bf16(xd[j][i], p[i], d);
        }
        acc[r][m] = fmaf(sc[r], d - sx136, fmaf(zp[r], sx, acc[r][m]));
      }
    }
  };

  // With PRO the first slice (every wave has one: Wk <= S) is peeled so the RMSNorm prologue
  // can sit around its loads.
  auto pair_step = [&](int s, auto first) __attribute__((always_inline)) {
    uint4 wv0[RPW], wv1[RPW];
    uint32_t szv0[RPW], szv1[RPW];
    int cc0, cc1;
    bool cv0, cv1;
    if constexpr (PRO && decltype(first)::value) norm_load();
    load_slice(s, wv0, szv0, cc0, cv0);
    load_slice(s + Wk, wv1, szv1, cc1, cv1);
    if constexpr (PRO && decltype(first)::value) norm_finish();
    do_slice(wv0, szv0, cc0, cv0);
    if (s + Wk < S) do_slice(wv1, szv1, cc1, cv1);  // wave-uniform
  };
  auto single_step = [&](int s, auto first) __attribute__((always_inline)) {
    uint4 wv0[RPW];
    uint32_t szv0[RPW];
    int cc0;
    bool cv0;
    if constexpr (PRO && decltype(first)::value) norm_load();
    load_slice(s, wv0, szv0, cc0, cv0);
    if constexpr (PRO && decltype(first)::value) norm_finish();
    do_slice(wv0, szv0, cc0, cv0);
  };
  if constexpr (PAIR && PRO) {
    pair_step(wk, std::true_type{});
    for (int s = wk + 2 * Wk; s < S; s += 2 * Wk) pair_step(s, std::false_type{});
  } else if constexpr (PAIR) {
    for (int s = wk; s < S; s += 2 * Wk) {
      uint4 wv0[RPW], wv1[RPW];
      uint32_t szv0[RPW], szv1[RPW];
      int cc0, cc1;
      bool cv0, cv1;
      load_slice(s, wv0, szv0, cc0, cv0);
      load_slice(s + Wk, wv1, szv1, cc1, cv1);
      do_slice(wv0, szv0, cc0, cv0);
      // wave-uniform. hipcc sinks slice s + Wk's loads into this branch, behind slice s's
      // arithmetic; issuing both slices' loads first (the second do_slice unconditional) measured
      // SLOWER: 28672x4096 14.6-15.0 -> 16.0 us, 4096x14336 9.3 -> 11.4 (every grid is resident
      // at once, and a wave holding less in flight computes while the others' loads stream;
      // profiles/r5g_ab_gemv_pair.jsonl)
      if (s + Wk < S) do_slice(wv1, szv1, cc1, cv1);
    }
  } else if constexpr (PRO) {
    single_step(wk, std::true_type{});
    for (int s = wk + Wk; s < S; s += Wk) single_step(s, std::false_type{});
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
  if constexpr (PRO) {
    if (fu.norm_deferred && fu.norm_w != nullptr) {  // the deferred RMSNorm scale (norm_finish)
      const float* ssr = red + G * Wk * V;
      float t = 0.f;
      for (int w = 0; w < G * Wk; ++w) t += ssr[w];
      const float rn = rsqrtf(t / (float)K + fu.eps);
      total *= rn;
      v[0] *= rn;
    }
  }
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
  if constexpr (EPI == kEpiNone) {
    if (writer) {
      const int r = widx / MT, m = widx % MT;
      const int n = row0 + r;
      if (n < N && m < M) {
        uint16_t out = f32_to_bf16(total);
        if (bias != nullptr) out = f32_to_bf16(bf16_to_f32(out) + bf16_to_f32(bias[n]));
        y[(size_t)m * N + n] = out;
      }
    }
  } else {
    // Row pair (2p, 2p+1) meets in lane p of the writing wave. Row r's total sits in lane r
    // (Wk > 1) or in owner lane r << (6 - T) (Wk == 1); every lane takes part in the shuffles.
    const float o = round_bf16(total);
    const int sh = Wk > 1 ? 0 : 6 - T;
    const int pl = lane < RPW / 2 ? lane : 0;
    const float a = __shfl(o, (2 * pl) << sh);
    const float b = __shfl(o, (2 * pl + 1) << sh);
    const int n = row0 + 2 * pl;
    if ((Wk == 1 || wk == 0) && lane < RPW / 2 && n < N) {
      if constexpr (EPI == kEpiSwiGLU) {
        y[n >> 1] = f32_to_bf16(round_bf16(a / (1.f + __expf(-a))) * b);
      } else {
        const int D = fu.D, HD = fu.H * fu.D, KD = fu.Hkv * fu.D;
        int64_t p = fu.pos[0];
        const bool pok = p >= 0 && p < fu.T;  // KV cache row inside [0, T)
        if (!pok) {  // report (tao_decode_status) and write no cache row
          flag_decode_error(kDecodeErrKvPos);
          p = p < 0 ? 0 : fu.T - 1;
        }
        uint32_t ov = (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
        if (n < HD + KD) {
          const float2 cs = reinterpret_cast<const float2*>(fu.freqs)[p * (D >> 1) + ((n % D) >> 1)];
          const float o0 = a * cs.x - b * cs.y, o1 = b * cs.x + a * cs.y;
          ov = (uint32_t)f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
        }
        if (n < HD) {
          if constexpr (COH) st_coh(reinterpret_cast<uint32_t*>(y) + (n >> 1), ov);
          else reinterpret_cast<uint32_t*>(y)[n >> 1] = ov;
        } else if (pok) {
          const int nk = n < HD + KD ? n - HD : n - HD - KD;
          uint16_t* cache = n < HD + KD ? fu.k_cache : fu.v_cache;
          const size_t off = ((size_t)(nk / D) * fu.T + p) * D + nk % D;
          if constexpr (COH) st_coh(reinterpret_cast<uint32_t*>(cache) + (off >> 1), ov);
          else reinterpret_cast<uint32_t*>(cache)[off >> 1] = ov;
        }
      }
    }
  }
}

template <int MT, int RPW, int WPE, bool PAIR, int NPT = 0, int EPI = kEpiNone, int MRG = 0>
__global__ __launch_bounds__(512, WPE) void int4wo_gemv_kernel(
    const uint16_t* __restrict__ x, const uint4* __restrict__ wq, const uint32_t* __restrict__ sz,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K, int gshift,
    int Wk, int G, int S, GemvFuse fu) {
  gemv_body<MT, RPW, PAIR, NPT, EPI, MRG>(x, wq, sz, bias, y, M, N, K, gshift, Wk, G, S, fu,
                                          (int)blockIdx.x * G * RPW);
}

// ---- wqkv + RoPE / KV write + decode attention in one launch (tao_int4wo_qkv_attn_bf16) -------
// Workgroups [0, ngemv) are the RMSNorm -> wqkv -> RoPE + KV GEMV (kEpiRopeKV, stores agent-scope);
// each then adds one ticket for the q / k / v head its rows belong to. Workgroups past them (the
// grid's tail, so on every XCD they are dispatched after all of that XCD's GEMV workgroups) are
// the decode attention: one per (query head, key split), NW waves. A consumer loads its first
// key step of cache history (rows < pos, written by earlier launches) before its wait, waits for
// the q head's and the kv head's tickets, then reads q and the new row pos with agent-scope loads,
// runs the one-pass attention step (tao_attn.h, as attn_single_kernel) over its key range, stores
// its split's unnormalised partial (sc1) and the split whose ticket comes last merges the head
// (attn_merge_weights) into the bf16 output. No stream-ordered launch between wqkv and the
// attention: the attention launch's fixed cost and its cold history loads overlap the GEMV.
// Tickets: producer counters go back to zero when the last consumer of a kv-head group has passed
// its wait (it subtracts what each counter was owed), so a timed-out wait (reported through
// tao_decode_status bits & 2, that head's output unspecified) still leaves them at zero once
// the late producers have added.
struct QkvAttn {
  uint16_t* out;  // [H * D] bf16 attention output
  float* part;    // [H][NS][kQaRec] fp32 split partials (split workspace slab)
  unsigned* cnt;  // workspace counters, cs words apart: [0, H + 2 Hkv) tickets of the q | k | v
                  // heads, [H + 2 Hkv, + Hkv) consumer arrivals per kv head, then H merge tickets
  int ngemv, need, cs, fenced;
  float scale;
};
constexpr int kQaRec = 132;  // o[128], m, l, 2 pad

template <int NW, int NS>
__device__ __forceinline__ void qkv_attn_tail(const GemvFuse& fu, const QkvAttn& qa,
                                              const uint16_t* __restrict__ qbuf) {
  constexpr int D = 128;
  extern __shared__ float red[];  // [NW] m, [NW] l, [NW][D] o, one flag word
  float* wm = red;
  float* wl = red + NW;
  float* wo = red + 2 * NW;
  unsigned* flag = reinterpret_cast<unsigned*>(red + 2 * NW + NW * D);
  const int c = (int)blockIdx.x - qa.ngemv;
  const int h = c / NS, sp = c % NS;
  const int G = fu.H / fu.Hkv, kvh = h / G, T = fu.T;
  const int64_t p64 = fu.pos[0];
  const int L = attn_len(p64, T);
  const int pk = p64 >= 0 && p64 < T ? (int)p64 : -1;  // the cache row this launch writes
  const int Cn = ((L + NS - 1) / NS + 15) & ~15;
  const int lo = sp * Cn, hi = lo + Cn < L ? lo + Cn : L;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const size_t head = (size_t)kvh * T;  // batch 1
  const uint32_t* vb = reinterpret_cast<const uint32_t*>(fu.v_cache + head * D) + lane;
  // lane (g = l / 8, p8 = l % 8): keys t0 + g and t0 + 8 + g, dims 64 hh + 8 p8 + e
  const int g = lane >> 3, p8 = lane & 7;
  const uint16_t* kbase = fu.k_cache + head * D + p8 * 8;
  uint4 ka[2], kb2[2];
  uint32_t vv[16];
  auto ldk = [&](int t, int hh) __attribute__((always_inline)) {
    const uint16_t* kp = kbase + (size_t)t * D + 64 * hh;
    if (t != pk) return *reinterpret_cast<const uint4*>(kp);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(kp);
    return make_uint4(ld_coh(w), ld_coh(w + 1), ld_coh(w + 2), ld_coh(w + 3));
  };
  auto load_step = [&](int t0) __attribute__((always_inline)) {
    const int ta = t0 + g < hi ? t0 + g : hi - 1, tb = t0 + 8 + g < hi ? t0 + 8 + g : hi - 1;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      ka[hh] = ldk(ta, hh);
      kb2[hh] = ldk(tb, hh);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int tj = t0 + j < hi ? t0 + j : hi - 1;
      vv[j] = tj != pk ? vb[(size_t)tj * (D / 2)] : ld_coh(vb + (size_t)tj * (D / 2));
    }
  };
  // this wave's first step, before the wait when all its rows are history
  const int t0w = lo + wave * 16;
  const int lastw = t0w + 15 < hi - 1 ? t0w + 15 : hi - 1;
  const bool early = t0w < hi && (pk < 0 || lastw < pk);
  if (early) load_step(t0w);

  // wait for the q head's and the kv head's tickets; then count this consumer in (the group's
  // last one returns the producer counters to zero)
  if (tid == 0) {
    const unsigned* cq = qa.cnt + (size_t)h * qa.cs;
    const unsigned* ck = qa.cnt + (size_t)(fu.H + kvh) * qa.cs;
    const unsigned* cv = qa.cnt + (size_t)(fu.H + fu.Hkv + kvh) * qa.cs;
    SeamWait sw;
    while ((int)ld_coh(cq) < qa.need || (int)ld_coh(ck) < qa.need || (int)ld_coh(cv) < qa.need) {
      if (sw.timed_out()) {
        flag_decode_error(kDecodeErrSplitK);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (qa.fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    unsigned* cons = qa.cnt + (size_t)(fu.H + 2 * fu.Hkv + kvh) * qa.cs;
    const unsigned arrivals = (unsigned)(G * NS);
    if (__hip_atomic_fetch_add(cons, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        arrivals - 1) {
      for (int j = 0; j < G; ++j)
        __hip_atomic_fetch_sub(qa.cnt + (size_t)(kvh * G + j) * qa.cs, (unsigned)qa.need,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_sub(qa.cnt + (size_t)(fu.H + kvh) * qa.cs, (unsigned)qa.need,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_sub(qa.cnt + (size_t)(fu.H + fu.Hkv + kvh) * qa.cs, (unsigned)qa.need,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_sub(cons, arrivals, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (t0w < hi && !early) load_step(t0w);
  uint32_t qw[8];
  {
    const uint32_t* qp = reinterpret_cast<const uint32_t*>(qbuf + (size_t)h * D + p8 * 8);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int e = 0; e < 4; ++e) qw[hh * 4 + e] = ld_coh(qp + 32 * hh + e);
  }
  float m = -INFINITY, l = 0.f, o0 = 0.f, o1 = 0.f;
  for (int t0 = t0w; t0 < hi; t0 += NW * 16)
    attn_decode_step(qw, ka, kb2, vv, t0, hi, g, qa.scale, m, l, o0, o1, [&]() {
      if (t0 + NW * 16 < hi) load_step(t0 + NW * 16);  // wave-uniform prefetch of the next step
    });
  if (lane == 0) {
    wm[wave] = m;
    wl[wave] = l;
  }
  wo[wave * D + 2 * lane] = o0;
  wo[wave * D + 2 * lane + 1] = o1;
  __syncthreads();
  float* rec = qa.part + ((size_t)h * NS + sp) * kQaRec;
  if (wave == 0) {  // this split's partial over the NW waves (a wave without keys has m = -inf)
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w]);
    float a0 = 0.f, a1 = 0.f, ls = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = wm[w] == -INFINITY ? 0.f : __expf(wm[w] - M);
      ls = fmaf(wl[w], f, ls);
      a0 = fmaf(wo[w * D + 2 * lane], f, a0);
      a1 = fmaf(wo[w * D + 2 * lane + 1], f, a1);
    }
    if constexpr (NS == 1) {  // the whole head in this workgroup: no partial, no merge ticket
      const float inv = 1.f / ls;
      reinterpret_cast<uint32_t*>(qa.out)[(size_t)h * (D / 2) + lane] =
          (uint32_t)f32_to_bf16(a0 * inv) | ((uint32_t)f32_to_bf16(a1 * inv) << 16);
      return;
    }
    uint32_t* r32 = reinterpret_cast<uint32_t*>(rec);
    st_coh(r32 + 2 * lane, __float_as_uint(a0));
    st_coh(r32 + 2 * lane + 1, __float_as_uint(a1));
    if (lane == 0) {
      st_coh(r32 + D, __float_as_uint(M));
      st_coh(r32 + D + 1, __float_as_uint(ls));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if constexpr (NS == 1) return;
  unsigned* mc = qa.cnt + (size_t)(fu.H + 3 * fu.Hkv + h) * qa.cs;
  if (!last_arriver(mc, (unsigned)NS, flag, qa.fenced)) return;
  if (wave != 0) return;
  float2 ml[NS];
  float ov[NS][2];
#pragma unroll
  for (int s2 = 0; s2 < NS; ++s2) {
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(qa.part + ((size_t)h * NS + s2) * kQaRec);
    ml[s2] = make_float2(__uint_as_float(ld_coh(r32 + D)), __uint_as_float(ld_coh(r32 + D + 1)));
    ov[s2][0] = __uint_as_float(ld_coh(r32 + 2 * lane));
    ov[s2][1] = __uint_as_float(ld_coh(r32 + 2 * lane + 1));
  }
  float wgt[NS], inv;
  attn_merge_weights<NS>(ml, wgt, inv);
  float r0 = 0.f, r1 = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < NS; ++s2) {
    r0 = fmaf(ov[s2][0], wgt[s2], r0);
    r1 = fmaf(ov[s2][1], wgt[s2], r1);
  }
  reinterpret_cast<uint32_t*>(qa.out)[(size_t)h * (D / 2) + lane] =
      (uint32_t)f32_to_bf16(r0 * inv) | ((uint32_t)f32_to_bf16(r1 * inv) << 16);
}

template <int NPT, bool PAIR, int NS>
__global__ __launch_bounds__(256, 4) void int4wo_qkv_attn_kernel(
    const uint16_t* __restrict__ x, const uint4* __restrict__ wq, const uint32_t* __restrict__ sz,
    uint16_t* __restrict__ y, int N, int K, int gshift, int S, GemvFuse fu, QkvAttn qa) {
  if ((int)blockIdx.x < qa.ngemv) {  // 4 waves x 2 rows, whole rows (Wk = 1)
    gemv_body<1, 2, PAIR, NPT, kEpiRopeKV, 0, true>(x, wq, sz, nullptr, y, 1, N, K, gshift, 1, 4,
                                                    S, fu, (int)blockIdx.x * 8);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's q / k / v stores landed
    __syncthreads();
    if (threadIdx.x == 0) {
      if (qa.fenced) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_fetch_add(qa.cnt + (size_t)((int)blockIdx.x * 8 / fu.D) * qa.cs, 1u,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  qkv_attn_tail<4, NS>(fu, qa, y);
}

// ---- grouped (MoE) decode GEMV: A experts' linears of one token in one launch ------------------
// (tao_int4wo_grouped_gemv_bf16). blockIdx.y = activation a: expert e = idx[a] of the [E][N][K]
// stack (packed [E][N][K/8], scales [E][N][K/g]); x row a (x_rows = A) or the shared x
// (x_rows = 1); y [A][N]. Each activation runs the plain M = 1 GEMV body of its expert, so its
// output is bit-identical to that expert's own linear. The expert index is read on the device,
// so the launch is graph-capturable with the router's top-k on the GPU.
template <int RPW, int WPE, bool PAIR>
__global__ __launch_bounds__(512, WPE) void int4wo_grouped_gemv_kernel(
    const uint16_t* __restrict__ x, int x_rows, const uint4* __restrict__ wq,
    const uint32_t* __restrict__ sz, const int64_t* __restrict__ idx, int E,
    uint16_t* __restrict__ y, int N, int K, int gshift, int Wk, int G, int S) {
  const int a = (int)blockIdx.y;
  int64_t e = idx[a];
  if (e < 0 || e >= E) {
    if (threadIdx.x == 0 && blockIdx.x == 0) flag_decode_error(kDecodeErrExpert);
    e = e < 0 ? 0 : E - 1;
  }
  const size_t nchunk = (size_t)K >> 5, ngroups = (size_t)K >> (5 + gshift);
  gemv_body<1, RPW, PAIR>(x + (x_rows > 1 ? (size_t)a * K : 0), wq + (size_t)e * N * nchunk,
                          sz + (size_t)e * N * ngroups, nullptr, y + (size_t)a * N, 1, N, K,
                          gshift, Wk, G, S, GemvFuse{}, (int)blockIdx.x * G * RPW);
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

template <int MT, int RPW, int WPE, int NPT = 0, int EPI = kEpiNone, int MRG = 0>
int launch_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, int gshift,
                GemvShape sh, hipStream_t stream, const GemvFuse& fu = GemvFuse{}) {
  const int nchunk = K / 32;
  const int S = (nchunk + 63) / 64;
  const int wk = sh.wk < S ? sh.wk : S;
  const int rows_per_wg = sh.g * RPW;
  const int grid = (N + rows_per_wg - 1) / rows_per_wg;
  const int threads = 64 * wk * sh.g;
  constexpr bool PRO = NPT > 0;
  size_t lds = PRO ? (((size_t)sh.g * wk * RPW * MT + 8 + 3) & ~(size_t)3) * sizeof(float) +
                         (size_t)K * 2
                   : (size_t)sh.g * wk * RPW * MT * sizeof(float);
  // tao_tune_int4_lds: dynamic LDS of at least this many bytes per workgroup, which caps the
  // workgroups resident per CU (160 KiB / bytes) and so the weight bytes in flight per CU
  if (tao::tuning().gemv_lds > 0 && (size_t)tao::tuning().gemv_lds > lds)
    lds = (size_t)tao::tuning().gemv_lds;
  if (S > wk)
    launch((int4wo_gemv_kernel<MT, RPW, WPE, true, NPT, EPI, MRG>), dim3(grid), dim3(threads), lds,
           stream, x, reinterpret_cast<const uint4*>(packed),
           reinterpret_cast<const uint32_t*>(sz), bias, y, M, N, K, gshift, wk, sh.g, S, fu);
  else
    launch((int4wo_gemv_kernel<MT, RPW, WPE, false, NPT, EPI, MRG>), dim3(grid), dim3(threads), lds,
           stream, x, reinterpret_cast<const uint4*>(packed),
           reinterpret_cast<const uint32_t*>(sz), bias, y, M, N, K, gshift, wk, sh.g, S, fu);
  return check_launch("int4wo_gemv_kernel");
}

// Process-wide override of the M == 1 launch shape (tao_tune_int4_gemv; 0 = heuristic).

// M == 1 launch shape. Measured on MI355X (experiments/sweep_gemv.py,
// profiles/r1_sweep_gemv*.jsonl): the best shapes per (N, K) class, dispatch-event timed over
// weights rotated past the MALL.
struct M1Shape {
  int rpw, occ;
  GemvShape sh;
};

M1Shape m1_shape(int N, int S) {
  M1Shape c{4, 8, default_shape(S)};
  if (S <= 2) {  // K <= 4096
    if (N >= 32768) {
      c.sh = {2, 2};
    } else if (N > 8192 && N < 16384) {  // 11008 (7B-class FFN, BASELINE config 2), 14336:
      // 2 rows per wave, 2 waves along K, 2 row groups (profiles/r2_sweep_gemv_midN.jsonl:
      // 11008x4096 6.91 vs 7.49 µs, 14336x4096 8.12 vs 8.40)
      c.rpw = 2;
      c.sh = {2, 2};
    } else if (N >= 8192) {  // one wave walks both slices of 4 rows (PAIR)
      c.occ = 4;
      c.sh = {1, N >= 16384 ? 4 : 1};
    } else if (N >= 6144) {  // wqkv 6144x4096: one wave walks both slices of 2 rows (PAIR):
      // 4.94 vs 5.18 us for 2 waves along K (same-process A/B after the byte-permute decode,
      // profiles/r6p_ab_wqkv_shape.jsonl)
      c.rpw = 2;
      c.sh = {1, 4};
    } else {
      c.rpw = 2;
      c.sh = {2, N <= 4096 ? 1 : 4};
    }
  } else {  // K > 4096: waves split K (each walking its slices in pairs) while N is small
    // (profiles/r1_sweep_gemv_70b.jsonl, r1_sweep_gemv_shards.jsonl: Llama-3-70B linears and
    // their 2/4/8-way column shards)
    // Round 6 re-sweep after the byte-permute decode (graph-timed, then same-process A/B:
    // profiles/r6r_sweep_gemv_70b.jsonl, r6s_ab_gemv_70b.jsonl; us, old -> new shape): 57344x8192
    // 52.4 -> 46.7, 8192^2 10.3 -> 9.0, 10240x8192 12.1 -> 11.0, 7168x8192 9.4 -> 8.7, 1024x8192
    // 4.0 -> 3.5, 1280x8192 4.1 -> 3.9; 2048x8192, 3584x8192, 1024x28672, 8192x28672 unchanged
    c.occ = 4;
    if (N >= 32768) {  // heads / fused w1||w3: 8 rows per wave (128256x8192 93.9 vs 99.7 µs at 4)
      c.rpw = 8;
      c.sh = {2, 1};
    } else if (N <= 2560 && S <= 4) {
      c.rpw = 2;
      c.sh = {N <= 1536 ? 4 : 2, 1};
    } else if (N <= 2048) {  // few rows, long K: more waves along K (1024x28672 5.7 vs 9.0 µs)
      c.sh = {N <= 1024 ? 8 : 4, 1};
    } else if (N <= 4096 || S > 4) {
      c.sh = {N <= 4096 ? 2 : (S >= 8 ? 1 : 4), 1};
    } else {  // K = 8192, N > 4096: one wave walks the row's 4 slices (two PAIR steps)
      c.sh = N >= 10240 && N < 16384 ? GemvShape{2, 2} : GemvShape{1, 1};
    }
  }
  const int trpw = tao::tuning().rpw;
  const int tocc = tao::tuning().occ;
  const int twk = tao::tuning().wk;
  const int tg = tao::tuning().g;
  if (trpw > 0) c.rpw = trpw;
  if (tocc > 0) c.occ = tocc;
  if (twk > 0) c.sh.wk = twk;
  if (tg > 0) c.sh.g = tg;
  return c;
}

template <int NPT, int EPI>
int launch_decode_rows(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                       uint16_t* y, int N, int K, int gs, hipStream_t stream, const GemvFuse& fu,
                       const M1Shape& c) {
  if constexpr (NPT == 0 && EPI == kEpiNone) {  // the plain linear: the product path's shapes
    if (c.rpw == 8)
      return launch_gemv<1, 8, 4>(x, packed, sz, nullptr, y, 1, N, K, gs, c.sh, stream);
  }
  // row pairs stay inside one wave: 2 or 4 rows per wave; the RMSNorm prologue (the first
  // slices' loads live across it) does not fit 64 VGPRs, so it runs at <= 4 waves per SIMD
  if (c.rpw <= 2) {
    if constexpr (NPT > 0)
      return launch_gemv<1, 2, 4, NPT, EPI>(x, packed, sz, nullptr, y, 1, N, K, gs, c.sh, stream,
                                            fu);
    else
      return launch_gemv<1, 2, 8, NPT, EPI>(x, packed, sz, nullptr, y, 1, N, K, gs, c.sh, stream,
                                            fu);
  }
  if (c.occ == 4 || NPT > 0)
    return launch_gemv<1, 4, 4, NPT, EPI>(x, packed, sz, nullptr, y, 1, N, K, gs, c.sh, stream, fu);
  return launch_gemv<1, 4, 8, 0, EPI>(x, packed, sz, nullptr, y, 1, N, K, gs, c.sh, stream, fu);
}

// Launch shape of the prologue (PRO) paths. Measured (experiments/bench_decode.py,
// profiles/r1_bench_decode*.jsonl): with the prologue a workgroup should own whole rows (no K
// split) and 4 waves of them, so the per-workgroup normalisation is amortised over 8-16 rows; 2
// rows per wave below N = 16384 (Llama-3-70B wqkv 10240x8192: 14.0 vs 18.0 µs at 4 rows).
M1Shape pro_shape(int N, int K) {
  const int S = (K / 32 + 63) / 64;
  M1Shape c = m1_shape(N, S);
  if (tao::tuning().rpw == 0) c.rpw = N < 16384 ? 2 : 4;
  if (tao::tuning().wk == 0) c.sh.wk = 1;
  if (tao::tuning().g == 0) c.sh.g = 4;
  // Round 6, after the byte-permute decode (same-process A/B, profiles/r6z_ab_decode_shape.jsonl):
  // Llama-3-70B's wqkv + RoPE (10240x8192) 15.1 -> 13.9 us on 4 rows per wave and 2 waves along
  // K; its w1||w3 and every Llama-3-8B shape keep the whole-row shape above
  if (K > 4096 && N > 8192 && N < 16384 && tao::tuning().rpw == 0 && tao::tuning().wk == 0 &&
      tao::tuning().g == 0) {
    c.rpw = 4;
    c.sh.wk = 2;
    c.sh.g = 2;
  }
  // enough threads to hold x in the prologue: K <= 8 * NPT * threads, NPT <= kMaxNormPT
  const int wk = c.sh.wk < S ? c.sh.wk : S;
  while (64 * wk * c.sh.g * 8 * kMaxNormPT < K && wk * c.sh.g * 2 <= 8) c.sh.g *= 2;
  return c;
}

// tao_int4wo_attn_out_bf16: the wo GEMV with the split-attention merge as its x prologue, on the
// launch shape of the PRO paths (so tao_tune_int4_xlds 1 gives the unfused reference the same
// per-element sums), bias = the residual
template <int MRG>
int launch_attn_out(const float* part, const uint32_t* packed, const uint16_t* sz,
                    const uint16_t* bias, uint16_t* y, int N, int K, int gs, hipStream_t stream) {
  const M1Shape c = pro_shape(N, K);
  const int wk = c.sh.wk < (K / 32 + 63) / 64 ? c.sh.wk : (K / 32 + 63) / 64;
  const int threads = 64 * wk * c.sh.g;
  GemvFuse fu{};
  fu.merge = part;
  const uint16_t* xn = reinterpret_cast<const uint16_t*>(part);  // unread (the prologue forms x)
  if (threads * 8 * 2 >= K) {
    if (c.rpw <= 2)
      return launch_gemv<1, 2, 4, 2, kEpiNone, MRG>(xn, packed, sz, bias, y, 1, N, K, gs, c.sh,
                                                    stream, fu);
    return launch_gemv<1, 4, 4, 2, kEpiNone, MRG>(xn, packed, sz, bias, y, 1, N, K, gs, c.sh,
                                                  stream, fu);
  }
  if (c.rpw <= 2)
    return launch_gemv<1, 2, 4, 4, kEpiNone, MRG>(xn, packed, sz, bias, y, 1, N, K, gs, c.sh,
                                                  stream, fu);
  return launch_gemv<1, 4, 4, 4, kEpiNone, MRG>(xn, packed, sz, bias, y, 1, N, K, gs, c.sh,
                                                stream, fu);
}

template <bool PRO, int EPI>
int launch_decode(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, uint16_t* y,
                  int N, int K, int gs, hipStream_t stream, const GemvFuse& fu) {
  const int S = (K / 32 + 63) / 64;
  M1Shape c = m1_shape(N, S);
  if constexpr (PRO) {
    c = pro_shape(N, K);
    const int wk = c.sh.wk < S ? c.sh.wk : S;
    const int threads = 64 * wk * c.sh.g;
    if (threads * 8 * 2 >= K)
      return launch_decode_rows<2, EPI>(x, packed, sz, y, N, K, gs, stream, fu, c);
    return launch_decode_rows<4, EPI>(x, packed, sz, y, N, K, gs, stream, fu, c);
  } else {
    return launch_decode_rows<0, EPI>(x, packed, sz, y, N, K, gs, stream, fu, c);
  }
}

}  // namespace

// M == 1 plain linears with x staged once per workgroup in LDS (the RMSNorm prologue's copy,
// without the norm): 0 = off (built-in), 1 = on. tao_tune_int4_xlds.
// RMSNorm prologue mode of the decode GEMV: 0 = exact (the reference's two bf16 roundings,
// normalised before the slices), 1 = deferred (outputs scaled by r). tao_tune_int4_norm.

// Internal entry (also used by the MFMA dispatcher for small M).
int int4wo_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                int64_t group_size, hipStream_t stream) {
  const int gs = gshift_of(group_size);
  const int S = (int)((K / 32 + 63) / 64);
  GemvShape sh = default_shape(S);
  const int iM = (int)M, iN = (int)N, iK = (int)K;
  if (M <= 1 && bias == nullptr && tao::tuning().xlds == 1) {
    GemvFuse fu{};
    fu.norm_w = nullptr;
    return launch_decode<true, kEpiNone>(x, packed, sz, y, iN, iK, gs, stream, fu);
  }
  if (M <= 1) {
    const M1Shape c = m1_shape(iN, S);
    sh = c.sh;
    if (c.rpw == 1) return launch_gemv<1, 1, 8>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    if (c.rpw == 2) return launch_gemv<1, 2, 8>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    if (c.rpw == 8) return launch_gemv<1, 8, 4>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
    if (c.occ == 4) return launch_gemv<1, 4, 4>(x, packed, sz, bias, y, iM, iN, iK, gs, sh, stream);
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

extern "C" int tao_tune_int4_norm(int mode) {
  TAO_CHECK_ARG(mode == 0 || mode == 1, "tune: norm mode must be 0 (exact) or 1 (deferred)");
  tao::tuning().norm = mode;
  return TAO_OK;
}

extern "C" int tao_tune_int4_xlds(int mode) {
  TAO_CHECK_ARG(mode == 0 || mode == 1, "tune: xlds mode must be 0 or 1");
  tao::tuning().xlds = mode;
  return TAO_OK;
}

extern "C" int tao_tune_int4_gemv(int rows_per_wave, int waves_k, int row_groups, int occupancy) {
  TAO_CHECK_ARG(rows_per_wave == 0 || rows_per_wave == 1 || rows_per_wave == 2 ||
                    rows_per_wave == 4 || rows_per_wave == 8,
                "tune: rows_per_wave must be 0 (auto), 1, 2, 4 or 8");
  TAO_CHECK_ARG(waves_k >= 0 && row_groups >= 0 && waves_k * (row_groups ? row_groups : 1) <= 8,
                "tune: waves_k * row_groups must be <= 8");
  TAO_CHECK_ARG(occupancy == 0 || occupancy == 4 || occupancy == 8, "tune: occupancy 0, 4 or 8");
  tao::tuning().rpw = rows_per_wave;
  tao::tuning().wk = waves_k;
  tao::tuning().g = row_groups;
  tao::tuning().occ = occupancy;
  return TAO_OK;
}

extern "C" int tao_int4wo_decode_bf16(const uint16_t* x, const uint32_t* packed,
                                      const uint16_t* scales_and_zeros, int64_t N, int64_t K,
                                      int64_t group_size, const uint16_t* norm_weight, float eps,
                                      int epilogue, uint16_t* y, const float* freqs,
                                      const int64_t* pos, uint16_t* k_cache, uint16_t* v_cache,
                                      int64_t n_head, int64_t n_kv_head, int64_t head_dim,
                                      int64_t max_seq, void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, scales_and_zeros, y, 1, N, K, group_size);
  if (rc != TAO_OK) return rc;
  TAO_CHECK_ARG(epilogue >= tao::kEpiNone && epilogue <= tao::kEpiRopeKV,
                "int4 decode: epilogue must be 0 (none), 1 (swiglu) or 2 (rope_kv)");
  TAO_CHECK_ARG(epilogue == tao::kEpiNone || N % 2 == 0, "int4 decode: N (%lld) must be even",
                (long long)N);
  if (norm_weight != nullptr) {
    TAO_CHECK_ALIGN(norm_weight, 16, "norm_weight");
    TAO_CHECK_ARG(K <= 8 * tao::kMaxNormPT * 512,
                  "int4 decode: RMSNorm prologue needs K <= %d", 8 * tao::kMaxNormPT * 512);
  }
  tao::GemvFuse fu{};
  fu.norm_w = norm_weight;
  fu.eps = eps;
  fu.norm_deferred = tao::tuning().norm;
  if (epilogue == tao::kEpiRopeKV) {
    TAO_CHECK_ARG(n_head > 0 && n_kv_head > 0 && head_dim > 0 && head_dim % 2 == 0 &&
                      max_seq > 0 && N == (n_head + 2 * n_kv_head) * head_dim,
                  "int4 decode rope_kv: N (%lld) must be (n_head + 2 n_kv_head) * head_dim",
                  (long long)N);
    TAO_CHECK_ARG(freqs != nullptr && pos != nullptr && k_cache != nullptr && v_cache != nullptr,
                  "int4 decode rope_kv: freqs, pos and caches are required");
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
  const int gs = tao::gshift_of(group_size);
  hipStream_t st = tao::as_stream(stream);
  const int iN = (int)N, iK = (int)K;
  // without a norm, tao_tune_int4_xlds 1 still takes the prologue path (x staged raw in LDS):
  // the experiment that separates the RMSNorm's cost from the LDS staging's
  const bool pro =
      norm_weight != nullptr || tao::tuning().xlds == 1;
#define TAO_DEC(P, E) \
  return tao::launch_decode<P, E>(x, packed, scales_and_zeros, y, iN, iK, gs, st, fu)
  switch (epilogue) {
    case tao::kEpiSwiGLU:
      if (pro) TAO_DEC(true, tao::kEpiSwiGLU);
      TAO_DEC(false, tao::kEpiSwiGLU);
    case tao::kEpiRopeKV:
      if (pro) TAO_DEC(true, tao::kEpiRopeKV);
      TAO_DEC(false, tao::kEpiRopeKV);
    default:
      if (pro) TAO_DEC(true, tao::kEpiNone);
      TAO_DEC(false, tao::kEpiNone);
  }
#undef TAO_DEC
}

extern "C" int tao_int4wo_attn_out_bf16(const float* partial, int64_t splits, int64_t n_head,
                                        const uint32_t* packed, const uint16_t* scales_and_zeros,
                                        int64_t N, int64_t K, int64_t group_size,
                                        const uint16_t* residual, uint16_t* y, void* stream) {
  TAO_CHECK_ARG(partial != nullptr, "int4 attn_out: partial is required");
  TAO_CHECK_ARG(splits == 2 || splits == 4, "int4 attn_out: splits must be 2 or 4 (got %lld)",
                (long long)splits);
  TAO_CHECK_ARG(n_head > 0 && K == n_head * 128,
                "int4 attn_out: K (%lld) must be n_head * 128", (long long)K);
  TAO_CHECK_ALIGN(partial, 16, "partial");
  int rc = tao::int4_check_linear_args(reinterpret_cast<const uint16_t*>(partial), packed,
                                       scales_and_zeros, y, 1, N, K, group_size);
  if (rc != TAO_OK) return rc;
  TAO_CHECK_ARG(K <= 8 * tao::kMaxNormPT * 512, "int4 attn_out: K must be <= %d",
                8 * tao::kMaxNormPT * 512);
  if (N == 0) return TAO_OK;
  const int gs = tao::gshift_of(group_size);
  hipStream_t st = tao::as_stream(stream);
  if (splits == 2)
    return tao::launch_attn_out<2>(partial, packed, scales_and_zeros, residual, y, (int)N, (int)K,
                                   gs, st);
  return tao::launch_attn_out<4>(partial, packed, scales_and_zeros, residual, y, (int)N, (int)K,
                                 gs, st);
}


extern "C" int tao_tune_int4_lds(int bytes) {
  TAO_CHECK_ARG(bytes >= 0 && bytes <= 160 * 1024, "tune: int4_lds bytes must be 0..163840");
  tao::tuning().gemv_lds = bytes;
  return TAO_OK;
}

namespace tao {
namespace {

// the fused launch's GEMV shape is the RMSNorm-prologue shape of wqkv (pro_shape) when that is
// 4 waves x 2 rows of whole rows; 0 if not (the caller then runs the two launches)
int qkv_attn_npt(int64_t N, int64_t K, int64_t n_head, int64_t n_kv_head, int64_t head_dim) {
  if (head_dim != 128 || n_head <= 0 || n_kv_head <= 0 || n_head % n_kv_head != 0 ||
      N != (n_head + 2 * n_kv_head) * head_dim || K <= 0 || K % 256 != 0 || K > 8192)
    return 0;
  const M1Shape c = pro_shape((int)N, (int)K);
  const int S = (int)((K / 32 + 63) / 64);
  const int wk = c.sh.wk < S ? c.sh.wk : S;
  if (c.rpw != 2 || wk != 1 || c.sh.g != 4) return 0;
  return 256 * 8 * 2 >= K ? 2 : 4;
}

template <int NPT, bool PAIR, int NS>
void launch_qkv_attn(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, uint16_t* y,
                     int N, int K, int gs, int S, const GemvFuse& fu, const QkvAttn& qa,
                     size_t lds, hipStream_t st) {
  launch((int4wo_qkv_attn_kernel<NPT, PAIR, NS>), dim3((unsigned)(qa.ngemv + fu.H * NS)),
         dim3(256), lds, st, x, reinterpret_cast<const uint4*>(packed),
         reinterpret_cast<const uint32_t*>(sz), y, N, K, gs, S, fu, qa);
}

}  // namespace
}  // namespace tao

extern "C" int tao_int4wo_qkv_attn_supported(int64_t N, int64_t K, int64_t n_head,
                                             int64_t n_kv_head, int64_t head_dim) {
  return tao::qkv_attn_npt(N, K, n_head, n_kv_head, head_dim) > 0 ? 1 : 0;
}

extern "C" int tao_int4wo_qkv_attn_bf16(const uint16_t* x, const uint32_t* packed,
                                        const uint16_t* scales_and_zeros, int64_t N, int64_t K,
                                        int64_t group_size, const uint16_t* norm_weight,
                                        float eps, uint16_t* q, uint16_t* out, const float* freqs,
                                        const int64_t* pos, uint16_t* k_cache, uint16_t* v_cache,
                                        int64_t n_head, int64_t n_kv_head, int64_t head_dim,
                                        int64_t max_seq, float scale, int64_t splits,
                                        void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, scales_and_zeros, q, 1, N, K, group_size);
  if (rc != TAO_OK) return rc;
  const int npt = tao::qkv_attn_npt(N, K, n_head, n_kv_head, head_dim);
  TAO_CHECK_ARG(npt > 0,
                "int4 qkv_attn: unsupported shape (N %lld, K %lld, heads %lld / %lld, head_dim "
                "%lld; tao_int4wo_qkv_attn_supported)",
                (long long)N, (long long)K, (long long)n_head, (long long)n_kv_head,
                (long long)head_dim);
  TAO_CHECK_ARG(splits == 1 || splits == 2 || splits == 4,
                "int4 qkv_attn: splits must be 1, 2 or 4 (got %lld)", (long long)splits);
  TAO_CHECK_ARG(norm_weight != nullptr && freqs != nullptr && pos != nullptr &&
                    k_cache != nullptr && v_cache != nullptr && out != nullptr,
                "int4 qkv_attn: norm_weight, freqs, pos, caches and out are required");
  TAO_CHECK_ARG(max_seq > 0 && max_seq < (1LL << 24), "int4 qkv_attn: max_seq out of range");
  TAO_CHECK_ALIGN(norm_weight, 16, "norm_weight");
  TAO_CHECK_ALIGN(k_cache, 16, "k_cache");
  TAO_CHECK_ALIGN(v_cache, 16, "v_cache");
  TAO_CHECK_ALIGN(q, 16, "q");
  TAO_CHECK_ALIGN(out, 4, "out");
  hipStream_t st = tao::as_stream(stream);
  const int H = (int)n_head, Hkv = (int)n_kv_head;
  const int cs = tao::tuning().cnt_stride;
  void* slab = nullptr;
  unsigned* cnt = nullptr;
  rc = tao::split_workspace(st, (size_t)H * splits * tao::kQaRec * sizeof(float),
                            (size_t)(2 * H + 3 * Hkv) * cs, &slab, &cnt);
  if (rc != TAO_OK) return rc;
  tao::GemvFuse fu{};
  fu.norm_w = norm_weight;
  fu.eps = eps;
  fu.norm_deferred = tao::tuning().norm;
  fu.freqs = freqs;
  fu.pos = pos;
  fu.k_cache = k_cache;
  fu.v_cache = v_cache;
  fu.H = H;
  fu.Hkv = Hkv;
  fu.D = (int)head_dim;
  fu.T = (int)max_seq;
  tao::QkvAttn qa{};
  qa.out = out;
  qa.part = static_cast<float*>(slab);
  qa.cnt = cnt;
  qa.ngemv = (int)(N / 8);
  qa.need = (int)(head_dim / 8);
  qa.cs = cs;
  qa.fenced = tao::tuning().splitk_fenced;
  qa.scale = scale;
  const int iN = (int)N, iK = (int)K, gs = tao::gshift_of(group_size);
  const int S = (iK / 32 + 63) / 64;
  // dynamic LDS: the GEMV prologue's ([4][1][2] partials + 8, x [K] bf16) or the attention's
  const size_t lds_gemv = (((size_t)8 + 8 + 3) & ~(size_t)3) * sizeof(float) + (size_t)iK * 2;
  const size_t lds_attn = (size_t)(2 * 4 + 4 * 128 + 1) * sizeof(float);
  const size_t lds = lds_gemv > lds_attn ? lds_gemv : lds_attn;
#define TAO_QA(NPT, PAIR, NS) \
  tao::launch_qkv_attn<NPT, PAIR, NS>(x, packed, scales_and_zeros, q, iN, iK, gs, S, fu, qa, lds, st)
  if (npt == 2) {
    if (S > 1) {
      if (splits == 1) TAO_QA(2, true, 1); else if (splits == 2) TAO_QA(2, true, 2); else TAO_QA(2, true, 4);
    } else {
      if (splits == 1) TAO_QA(2, false, 1); else if (splits == 2) TAO_QA(2, false, 2); else TAO_QA(2, false, 4);
    }
  } else {
    if (splits == 1) TAO_QA(4, true, 1); else if (splits == 2) TAO_QA(4, true, 2); else TAO_QA(4, true, 4);
  }
#undef TAO_QA
  return tao::check_launch("int4wo_qkv_attn_kernel");
}

namespace tao {
namespace {

template <int RPW, int WPE>
void launch_grouped(const uint16_t* x, int x_rows, const uint32_t* packed, const uint16_t* sz,
                    const int64_t* idx, int A, int E, uint16_t* y, int N, int K, int gs,
                    GemvShape sh, hipStream_t st) {
  const int S = (K / 32 + 63) / 64;
  const int wk = sh.wk < S ? sh.wk : S;
  const int rows = sh.g * RPW;
  const dim3 grid((unsigned)((N + rows - 1) / rows), (unsigned)A);
  const size_t lds = (size_t)sh.g * wk * RPW * sizeof(float);
  const uint4* w = reinterpret_cast<const uint4*>(packed);
  const uint32_t* s = reinterpret_cast<const uint32_t*>(sz);
  if (S > wk)
    launch((int4wo_grouped_gemv_kernel<RPW, WPE, true>), grid, dim3(64 * wk * sh.g), lds, st, x,
           x_rows, w, s, idx, E, y, N, K, gs, wk, sh.g, S);
  else
    launch((int4wo_grouped_gemv_kernel<RPW, WPE, false>), grid, dim3(64 * wk * sh.g), lds, st,
           x, x_rows, w, s, idx, E, y, N, K, gs, wk, sh.g, S);
}

}  // namespace
}  // namespace tao

extern "C" int tao_int4wo_grouped_gemv_bf16(const uint16_t* x, int64_t x_rows,
                                            const uint32_t* packed,
                                            const uint16_t* scales_and_zeros,
                                            const int64_t* expert_idx, int64_t A, int64_t E,
                                            int64_t N, int64_t K, int64_t group_size, uint16_t* y,
                                            void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, scales_and_zeros, y, 1, N, K, group_size);
  if (rc != TAO_OK) return rc;
  TAO_CHECK_ARG(A >= 0 && A <= 65535 && E > 0 && E < (1LL << 20),
                "int4 grouped: A (%lld) must be in [0, 65535] and E (%lld) positive",
                (long long)A, (long long)E);
  TAO_CHECK_ARG(x_rows == 1 || x_rows == A, "int4 grouped: x_rows (%lld) must be 1 or A (%lld)",
                (long long)x_rows, (long long)A);
  TAO_CHECK_ARG(expert_idx != nullptr, "int4 grouped: expert_idx is required");
  TAO_CHECK_ARG(E * N * (K / 8) < (1LL << 40), "int4 grouped: weight stack too large");
  if (A == 0 || N == 0) return TAO_OK;
  const int gs = tao::gshift_of(group_size);
  const int S = (int)((K / 32 + 63) / 64);
  const tao::M1Shape c = tao::m1_shape((int)N, S);  // the plain M = 1 linear's launch shape
  hipStream_t st = tao::as_stream(stream);
  const int iN = (int)N, iK = (int)K, iA = (int)A, iE = (int)E, xr = (int)x_rows;
#define TAO_GR(R, W) \
  tao::launch_grouped<R, W>(x, xr, packed, scales_and_zeros, expert_idx, iA, iE, y, iN, iK, gs, c.sh, st)
  if (c.rpw == 1) TAO_GR(1, 8);
  else if (c.rpw == 2) TAO_GR(2, 8);
  else if (c.rpw == 8) TAO_GR(8, 4);
  else if (c.occ == 4) TAO_GR(4, 4);
  else TAO_GR(4, 8);
#undef TAO_GR
  return tao::check_launch("int4wo_grouped_gemv_kernel");
}
