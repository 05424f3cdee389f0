// Prefill attention on MFMA for the e2e harness (gpt-fast's masked SDPA over the KV caches at
// prefill, torchao/_models/llama/model.py:468-470; the reference gets it from
// F.scaled_dot_product_attention): S queries per (batch, head) at positions pos[s], query s
// attending cache keys 0 .. pos[s] (clamped to the cache), GQA, head_dim 128, fp32 softmax.
//
// One wave per (batch, head, 16-query block), a workgroup of its own (S = 128, 32 heads: 256
// workgroups, one per CU). Per 32-key block:
//   * S^T = K Q^T on v_mfma_f32_16x16x32_bf16 (two 16-key tiles x 4 d-chunks): A = K rows, B =
//     Q^T (lane (q, kq) holds Q[q][32 c + 8 kq ..]), both row-contiguous 16-B loads; the result
//     has the query on the lane (q = lane & 15) and 4 keys per tile in registers, so the softmax
//     statistics of a query reduce over its 8 registers and the 4 lane groups (xor 16, 32);
//   * P (bf16) is the A operand of O = P V straight from those registers: lane (q, kq) takes the
//     keys 4 kq + i of tile 0 and 16 + 4 kq + i of tile 1 as its 8 k elements (a k order the V
//     operand follows), no LDS round trip;
//   * V goes through LDS (plain 256-B rows, 16-B chunks XOR-swizzled as the HIP guide's T10 image
//     (b)) and is read transposed with ds_read_b64_tr_b16: 4 keys x 16 d per 16-lane group, two
//     reads per 32-key B fragment, in the same permuted key order;
//   * O (16 queries x 128 d, 8 accumulator tiles) is rescaled by the online-softmax correction of
//     its rows (4 shuffles) before each P V.
// The output tile goes through LDS and leaves in 16-B row pieces: out [B][S][H * D] for wo.
#include "tao_common.h"

namespace tao {
namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t* lds_v4s_ptr;

constexpr int kD = 128;
constexpr int kQB = 16;  // queries per wave
constexpr int kKB = 32;  // keys per block

__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// byte offset of 16-B chunk `ch` (0..15) of V-image row `row` (256-B rows), guide T10 image (b)
__device__ __forceinline__ uint32_t voff(int row, int ch) {
  return 256u * row + 16u * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__global__ __launch_bounds__(64) void attn_prefill_mfma_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int64_t* __restrict__ pos, uint16_t* __restrict__ out,
    int H, int Hkv, int T, int S, float scale) {
  __shared__ uint4 vimg[kKB * kD * 2 / 16];  // 8 KiB: one V block; reused for the output tile
  const int lane = threadIdx.x;
  const int fr = lane & 15, kq = lane >> 4;
  const int bh = blockIdx.y, b = bh / H, h = bh % H, kvh = h / (H / Hkv);
  const int q0 = blockIdx.x * kQB;
  const size_t head = (size_t)(b * Hkv + kvh) * T;

  // this lane's query (column of S^T): row q0 + fr (clamped; outputs of rows >= S dropped)
  const int qs = q0 + fr < S ? q0 + fr : S - 1;
  const int Lq = attn_len(pos[qs], T);  // keys 0 .. Lq - 1
  int Lmax = Lq;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) Lmax = max(Lmax, __shfl_xor(Lmax, o, 64));
  Lmax = __builtin_amdgcn_readfirstlane(Lmax);

  // Q^T B fragments: lane (q, kq) holds Q[q][32 c + 8 kq .. + 8] for d-chunk c
  bf16x8_t qf[4];
  {
    const uint4* qp = reinterpret_cast<const uint4*>(q + ((size_t)bh * S + qs) * kD) + kq;
#pragma unroll
    for (int c = 0; c < 4; ++c) qf[c] = __builtin_bit_cast(bf16x8_t, qp[4 * c]);
  }
  f32x4_t o[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) o[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  const uint8_t* vimg_b = reinterpret_cast<const uint8_t*>(vimg);
  // K A fragments (rows k0 + 16 t + fr, clamped to the cache) and the V block's 16-B pieces. The
  // next block's are loaded into the same registers once this block's have been consumed (S^T
  // MFMAs issued, V stored to LDS), so they arrive under this block's softmax and P V.
  bf16x8_t kf[2][4];
#define ATTN_LOAD_K(K0)                                                                       \
  {                                                                                           \
    _Pragma("unroll") for (int t = 0; t < 2; ++t) {                                           \
      const int key = (K0) + 16 * t + fr < T ? (K0) + 16 * t + fr : T - 1;                   \
      const uint4* kp = reinterpret_cast<const uint4*>(kc + (head + key) * kD) + kq;          \
      _Pragma("unroll") for (int c = 0; c < 4; ++c) kf[t][c] =                                \
          __builtin_bit_cast(bf16x8_t, kp[4 * c]);                                            \
    }                                                                                         \
  }
  ATTN_LOAD_K(0)
  // the V block's 16-B pieces (rows k0 + r, clamped to the cache); ext-vector elements, so a
  // loop-carried copy stays in registers (an array of HIP's uint4 structs went to scratch)
#define ATTN_LOAD_V(K0)                                                                       \
  {                                                                                           \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                           \
      const int r = 4 * i + (lane >> 4);                                                      \
      const int key = (K0) + r < T ? (K0) + r : T - 1;                                        \
      vv[i] = reinterpret_cast<const u32x4_t*>(vc + (head + key) * kD)[lane & 15];            \
    }                                                                                         \
  }
  u32x4_t vv[8];
  ATTN_LOAD_V(0)
  for (int k0 = 0; k0 < Lmax; k0 += kKB) {
    // S^T tiles: lane (q, kq) gets keys 16 t + 4 kq + i of query q
    f32x4_t s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][c], qf[c], s[t], 0, 0, 0);
    }
    // (a one-wave workgroup: its LDS ops execute in program order, so the previous block's
    // transposed reads are done before these writes land, and the writes before the reads below)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 4 * i + (lane >> 4);
      *reinterpret_cast<u32x4_t*>(reinterpret_cast<uint8_t*>(vimg) + voff(r, lane & 15)) = vv[i];
    }
    // this block's K and V are consumed (S^T MFMAs issued, V in LDS): the next block's loads
    // (past the end: clamped rows, unused) arrive under this block's softmax and P V
    ATTN_LOAD_K(k0 + kKB)
    ATTN_LOAD_V(k0 + kKB)
    // online softmax over this block's keys, per query (fp32)
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * t + 4 * kq + i;
        s[t][i] = key < Lq ? s[t][i] * scale : -INFINITY;
        mx = fmaxf(mx, s[t][i]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);  // finite: key k0 < Lmax ... but this query may see none
    const float corr = mn == -INFINITY ? 1.f : __expf(m - mn);
    float ps = 0.f;
    uint32_t pw[4];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        e[i] = s[t][i] == -INFINITY ? 0.f : __expf(s[t][i] - mn);
        ps += e[i];
      }
      pw[2 * t] = pk2(e[0], e[1]);
      pw[2 * t + 1] = pk2(e[2], e[3]);
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
    const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, u32x4_t{pw[0], pw[1], pw[2], pw[3]});
    // rows 4 kq + i of the O tiles take the correction of query 4 kq + i (lane 4 kq + i)
    float cr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) cr[i] = __shfl(corr, 4 * kq + i, 64);
    // V^T B fragments by transposed reads: group kq, lane 4 qq + p supplies row (4 kq + qq) [and
    // 16 + 4 kq + qq], columns 16 dt + 4 p .. + 3 (chunk 2 dt + (p >> 1), half p & 1)
    const int qq = fr >> 2, p = fr & 3;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const int ch = 2 * dt + (p >> 1);
      const uint32_t a0 = voff(4 * kq + qq, ch) + 8u * (p & 1);
      const uint32_t a1 = voff(16 + 4 * kq + qq, ch) + 8u * (p & 1);
      const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)(vimg_b + a0));
      const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)(vimg_b + a1));
      const bf16x8_t vf = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) o[dt][i] *= cr[i];
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[dt], 0, 0, 0);
    }
  }
#undef ATTN_LOAD_K
#undef ATTN_LOAD_V
  // normalise rows 4 kq + i by their query's l, stage the bf16 tile [16][128] in LDS, store rows
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float li = __shfl(l, 4 * kq + i, 64);
    inv[i] = li > 0.f ? 1.f / li : 0.f;
  }
  uint16_t* ot = reinterpret_cast<uint16_t*>(vimg);  // [16][128]
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) ot[(4 * kq + i) * kD + 16 * dt + fr] = f32_to_bf16(o[dt][i] * inv[i]);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = 64 * i + lane;  // 256 pieces of 16 B: row piece / 16, chunk piece % 16
    const int r = piece >> 4, c = piece & 15;
    if (q0 + r < S)
      reinterpret_cast<uint4*>(out + ((size_t)(b * S + q0 + r) * H + h) * kD)[c] =
          reinterpret_cast<const uint4*>(ot)[piece];
  }
}

}  // namespace

int attn_prefill_mfma(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                      const int64_t* pos, uint16_t* out, int64_t B, int64_t H, int64_t Hkv,
                      int64_t S, int64_t T, float scale, hipStream_t stream) {
  const dim3 grid((unsigned)((S + kQB - 1) / kQB), (unsigned)(B * H));
  launch(attn_prefill_mfma_kernel, grid, dim3(64), 0, stream, q, k_cache, v_cache, pos, out,
         (int)H, (int)Hkv, (int)T, (int)S, scale);
  return check_launch("attn_prefill_mfma_kernel");
}

}  // namespace tao
