// Prefill attention on MFMA for the e2e harness (gpt-fast's masked SDPA over the KV caches at
// prefill, torchao/_models/llama/model.py:468-470; the reference gets it from
// F.scaled_dot_product_attention): S queries per (batch, head) at positions pos[s], query s
// attending cache keys 0 .. pos[s] (clamped to the cache), GQA, head_dim 128, fp32 softmax.
//
// One workgroup per (batch, head, 16-query block) of NW waves (round 5; 1 before), wave w taking
// the block's 32-key blocks w, w + NW, ... with its own online softmax, the NW partial states
// merged through LDS at the end (S = 128, 32 heads: 256 workgroups, one per CU, each wave at most
// one key block). Per 32-key block:
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

// NW waves per workgroup share one query block and split its key blocks round-robin (wave w
// takes blocks w, w + NW, ...), each with its own online-softmax state and V image; the NW
// partial (m, l, O) are then merged through LDS. NW = 1 is the one-wave kernel. At short prompts
// (S = 128: at most 4 key blocks per query block) the split turns the wave's serial chain of
// dependent K / V loads into one block per wave.
constexpr int kOStride = kD + 4;                       // fp32 O rows in the merge (padded)
constexpr int kSlab = (16 * kOStride * 4 + 15) / 16;   // uint4s per wave: V image or fp32 O tile

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_prefill_mfma_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
    const uint16_t* __restrict__ vc, const int64_t* __restrict__ pos, uint16_t* __restrict__ out,
    int H, int Hkv, int T, int S, float scale) {
  static_assert(kSlab * 16 >= kKB * kD * 2, "a wave's slab holds its V block");
  // per wave: one V block (8 KiB); reused for the output tile (NW = 1) or the fp32 O (NW > 1)
  __shared__ uint4 slab[NW * kSlab];
  __shared__ float mls[NW > 1 ? NW : 1][2][16];
  const int lane = threadIdx.x & 63, wv = NW > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
  uint4* const vimg = slab + wv * kSlab;
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
  ATTN_LOAD_K(wv * kKB)
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
  ATTN_LOAD_V(wv * kKB)
  for (int k0 = wv * kKB; k0 < Lmax; k0 += NW * kKB) {
    // S^T tiles: lane (q, kq) gets keys 16 t + 4 kq + i of query q
    f32x4_t s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][c], qf[c], s[t], 0, 0, 0);
    }
    // (the wave's own V image: its LDS ops execute in program order, so the previous block's
    // transposed reads are done before these writes land, and the writes before the reads below)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 4 * i + (lane >> 4);
      *reinterpret_cast<u32x4_t*>(reinterpret_cast<uint8_t*>(vimg) + voff(r, lane & 15)) = vv[i];
    }
    // this block's K and V are consumed (S^T MFMAs issued, V in LDS): the next block's loads
    // (past the end: clamped rows, unused) arrive under this block's softmax and P V
    ATTN_LOAD_K(k0 + NW * kKB)
    ATTN_LOAD_V(k0 + NW * kKB)
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
  if constexpr (NW > 1) {
    // publish this wave's (m, l) per query and its unnormalised O rows (fp32, padded rows), then
    // wave w merges rows 16 / NW * w .. over the NW waves: weights exp(m_j - M), M the max
    float* const of = reinterpret_cast<float*>(vimg);
    if (kq == 0) {
      mls[wv][0][fr] = m;
      mls[wv][1][fr] = l;
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) of[(4 * kq + i) * kOStride + 16 * dt + fr] = o[dt][i];
    __syncthreads();
    constexpr int kRows = 16 / NW;  // rows per wave; 16 lanes x 8 columns per row and pass
#pragma unroll
    for (int r0 = 0; r0 < kRows; r0 += 4) {
      const int row = kRows * wv + r0 + (lane >> 4), c8 = 8 * (lane & 15);
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < NW; ++j) mx = fmaxf(mx, mls[j][0][row]);
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ls = 0.f;
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const float mj = mls[j][0][row];
        const float wj = mj == -INFINITY ? 0.f : __expf(mj - mx);
        ls += mls[j][1][row] * wj;
        const float* src = reinterpret_cast<const float*>(slab + j * kSlab) + row * kOStride + c8;
        const f32x4_t a = *reinterpret_cast<const f32x4_t*>(src);
        const f32x4_t b4 = *reinterpret_cast<const f32x4_t*>(src + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] += a[e] * wj;
          acc[4 + e] += b4[e] * wj;
        }
      }
      const float inv = ls > 0.f ? 1.f / ls : 0.f;
      uint32_t w4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w4[e] = (uint32_t)f32_to_bf16(acc[2 * e] * inv) |
                ((uint32_t)f32_to_bf16(acc[2 * e + 1] * inv) << 16);
      if (q0 + row < S)
        *reinterpret_cast<uint4*>(out + ((size_t)(b * S + q0 + row) * H + h) * kD + c8) =
            make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    return;
  }
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
  // waves per query block: the tuning override, else by the grid's query blocks, from HIP-graph
  // timings at Llama-3-8B heads (profiles/r5j_attn_nw_graph.jsonl; us for nw 1 / 2 / 4):
  // S = 128 7.3 / 5.7 / 5.3, 256 13.7 / 9.3 / 9.2, 512 22.4 / 22.8 / 24.4, 1024 75.5 / 72.3 /
  // 70.2, 2048 223 / 204 / 205, 4096 708 / 682 / 677
  int nw = tuning().attn_prefill_nw;
  if (nw == 0) {
    const int64_t blocks = (int64_t)grid.x * grid.y;
    nw = blocks > 512 && blocks <= 1024 ? 2 : 4;
  }
  switch (nw) {
    case 1:
      launch(attn_prefill_mfma_kernel<1>, grid, dim3(64), 0, stream, q, k_cache, v_cache, pos,
             out, (int)H, (int)Hkv, (int)T, (int)S, scale);
      break;
    case 2:
      launch(attn_prefill_mfma_kernel<2>, grid, dim3(128), 0, stream, q, k_cache, v_cache, pos,
             out, (int)H, (int)Hkv, (int)T, (int)S, scale);
      break;
    default:
      launch(attn_prefill_mfma_kernel<4>, grid, dim3(256), 0, stream, q, k_cache, v_cache, pos,
             out, (int)H, (int)Hkv, (int)T, (int)S, scale);
      break;
  }
  return check_launch("attn_prefill_mfma_kernel");
}

}  // namespace tao

// Waves per 16-query block of the prefill attention (key blocks split round-robin, partial
// softmax states merged through LDS): 0 = built-in (2 for 513-1024 query blocks, else 4), 1, 2
// or 4.
extern "C" int tao_tune_attn_prefill_nw(int nw) {
  TAO_CHECK_ARG(nw == 0 || nw == 1 || nw == 2 || nw == 4,
                "tune: attn_prefill_nw must be 0, 1, 2 or 4");
  tao::tuning().attn_prefill_nw = nw;
  return TAO_OK;
}
