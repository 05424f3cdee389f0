// Weight-only quantised linear, batched (prefill) path on bf16 MFMA, for int4 (group-quant,
// float zero) and int8 (per-channel) weights, plus the C-ABI dispatchers
// tao_int4wo_linear_bf16 / tao_int8wo_linear_bf16 that pick GEMV (M <= 8) or MFMA (M > 8).
//
// Replaces aten._weight_int4pack_mm (torchao/dtypes/uintx/tensor_core_tiled_layout.py:104) and
// torch.mm(x, w.t().to(bf16)) * scale (torchao/dtypes/uintx/plain_layout.py:256-266).
//
// Tile: workgroup = 4 waves = BN 64 output columns (16 per wave) x BM rows; K advances in
// macro-steps of 128. v_mfma_f32_16x16x32_bf16 with a permuted k order: in macro-step k0,
// MFMA s (0..3) of lane l (n = l&15, kq = l>>4) covers k = k0 + 32*kq + 8*s + j, j = 0..7.
// So one lane's load of weights (32 consecutive k of row n: 16 B int4 / 32 B int8) feeds its
// B fragment for all four MFMAs, and an int4 lane needs one (scale, zero) dword: every 32-k
// chunk sits inside one quantisation group. The A operand (x) is staged through LDS with the
// same permutation, XOR-swizzled on 16-B slots (cdna guide §5.5 T2). B fragments are
// dequantised once per workgroup, in registers, and reused for BM/16 MFMAs.
#include "tao_common.h"

namespace tao {

int int4wo_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                int64_t group_size, hipStream_t stream);
int int4_check_linear_args(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                           uint16_t* y, int64_t M, int64_t N, int64_t K, int64_t group_size);
int int8wo_gemv(const uint16_t* x, const int8_t* w, const uint16_t* scale, const uint16_t* bias,
                uint16_t* y, int64_t M, int64_t N, int64_t K, hipStream_t stream);

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBN = 64;
constexpr int kKStep = 128;

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// ---- weight-format policies --------------------------------------------------------------
// Each policy loads one lane's 32-k chunk of row n for a macro-step, and turns sub-step s of
// it into an 8-element bf16 B fragment.
struct Int4Policy {
  const uint4* wq;       // [N][K/32] 16-B chunks
  const uint32_t* sz;    // [N][K/g] (scale, zero)
  int gshift;            // log2(g / 32)
  struct Chunk {
    uint4 w;
    uint32_t szw;
  };
  __device__ __forceinline__ Chunk load(int n, int c, int nchunk, bool ok) const {
    Chunk ch;
    ch.w = ld_nt_u4(wq + (size_t)n * nchunk + c);
    const uint32_t v = ld_nt(sz + (size_t)n * (nchunk >> gshift) + (c >> gshift));
    ch.szw = ok ? v : 0u;  // zero (scale, zero) => the fragment is exactly 0
    return ch;
  }
  struct Prep {
    uint32_t w[4];
    float s, zc;
  };
  __device__ __forceinline__ Prep prep(const Chunk& ch) const {
    Prep p;
    p.w[0] = ch.w.x;
    p.w[1] = ch.w.y;
    p.w[2] = ch.w.z;
    p.w[3] = ch.w.w;
    p.s = bf16lo_to_f32(ch.szw);
    p.zc = bf16hi_to_f32(ch.szw) - 136.f * p.s;  // (128+q)*s + zc == (q-8)*s + z
    return p;
  }
  // B fragment = bf16(fma(q - 8, s, z)) for the 8 nibbles of dword s.
  __device__ __forceinline__ bf16x8_t frag(const Prep& p, int sidx) const {
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t pr = nib_pair_bf16(p.w[sidx], i);
      o[i] = pack_bf16x2(fmaf(bf16lo_to_f32(pr), p.s, p.zc), fmaf(bf16hi_to_f32(pr), p.s, p.zc));
    }
    u32x4_t v = {o[0], o[1], o[2], o[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
  // Output epilogue of the int4 path: bf16(acc) (+ bias, tensor_core_tiled_layout.py:112-114).
  __device__ __forceinline__ float epilogue_scale(int) const { return 1.f; }
  static constexpr bool kScaled = false;
};

struct Int8Policy {
  const uint4* w;         // [N][K/16] 16-B chunks of int8
  const uint16_t* scale;  // [N] bf16
  struct Chunk {
    uint4 a, b;
    bool ok;
  };
  __device__ __forceinline__ Chunk load(int n, int c, int nchunk, bool ok) const {
    Chunk ch;
    const uint4* p = w + (size_t)n * (nchunk * 2) + 2 * c;
    ch.a = ld_nt_u4(p);
    ch.b = ld_nt_u4(p + 1);
    ch.ok = ok;
    return ch;
  }
  struct Prep {
    uint32_t w[8];
  };
  __device__ __forceinline__ Prep prep(const Chunk& ch) const {
    Prep p;
    const uint32_t m = ch.ok ? 0xFFFFFFFFu : 0u;
    p.w[0] = ch.a.x & m; p.w[1] = ch.a.y & m; p.w[2] = ch.a.z & m; p.w[3] = ch.a.w & m;
    p.w[4] = ch.b.x & m; p.w[5] = ch.b.y & m; p.w[6] = ch.b.z & m; p.w[7] = ch.b.w & m;
    return p;
  }
  // int8 -> bf16 is exact (|q| <= 128 needs 8 significant bits).
  __device__ __forceinline__ bf16x8_t frag(const Prep& p, int sidx) const {
    uint32_t o[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t d = p.w[2 * sidx + h];
      const float f0 = (float)(int8_t)(d & 0xFF);
      const float f1 = (float)(int8_t)((d >> 8) & 0xFF);
      const float f2 = (float)(int8_t)((d >> 16) & 0xFF);
      const float f3 = (float)(int8_t)(d >> 24);
      o[2 * h] = pack_bf16x2(f0, f1);
      o[2 * h + 1] = pack_bf16x2(f2, f3);
    }
    u32x4_t v = {o[0], o[1], o[2], o[3]};
    return __builtin_bit_cast(bf16x8_t, v);
  }
  static constexpr bool kScaled = true;
  __device__ __forceinline__ float epilogue_scale(int n) const { return bf16_to_f32(scale[n]); }
};

// LDS image of the x tile: [BM rows][16 slots of 16 B], slot XOR-swizzled with row & 15.
__device__ __forceinline__ int lds_slot(int row, int slot) { return row * 16 + (slot ^ (row & 15)); }

template <int BM, class P>
__global__ __launch_bounds__(256) void wo_mfma_kernel(const uint16_t* __restrict__ x, P pol,
                                                      const uint16_t* __restrict__ bias,
                                                      uint16_t* __restrict__ y, int M, int N,
                                                      int K) {
  constexpr int MT = BM / 16;            // m-tiles per wave
  constexpr int XLOADS = BM * 16 / 256;  // 16-B x pieces per thread per macro-step
  __shared__ uint4 xs[BM * 16];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int n_blk = blockIdx.x * kBN;
  const int m_blk = blockIdx.y * BM;
  const int nchunk = K >> 5;
  const int nsteps = (K + kKStep - 1) / kKStep;

  const int bn = n_blk + wave * 16 + (lane & 15);
  const int bnc = bn < N ? bn : N - 1;
  const int kq = lane >> 4;

  f32x4_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 xr[XLOADS];
  typename P::Chunk wr;

  auto load_step = [&](int step) {
    const int k0 = step * kKStep;
#pragma unroll
    for (int i = 0; i < XLOADS; ++i) {
      const int piece = tid + i * 256;
      const int row = piece >> 4, slot = piece & 15;
      const int gm = m_blk + row;
      const int gk = k0 + slot * 8;
      const bool ok = gm < M && gk < K;
      const int gmc = gm < M ? gm : M - 1;
      const int gkc = gk < K ? gk : 0;
      const uint4 v = *reinterpret_cast<const uint4*>(x + (size_t)gmc * K + gkc);
      xr[i] = ok ? v : make_uint4(0, 0, 0, 0);
    }
    const int c = (k0 >> 5) + kq;  // this lane's 32-k chunk
    const bool cok = c < nchunk && bn < N;
    const int cc = c < nchunk ? c : nchunk - 1;
    wr = pol.load(bnc, cc, nchunk, cok);
  };

  load_step(0);
  for (int step = 0; step < nsteps; ++step) {
    __syncthreads();  // all waves finished reading the previous tile
#pragma unroll
    for (int i = 0; i < XLOADS; ++i) {
      const int piece = tid + i * 256;
      xs[lds_slot(piece >> 4, piece & 15)] = xr[i];
    }
    const typename P::Prep pw = pol.prep(wr);
    __syncthreads();
    if (step + 1 < nsteps) load_step(step + 1);  // prefetch under the MFMAs (T14)

#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const bf16x8_t bfrag = pol.frag(pw, sidx);
      const int slot = kq * 4 + sidx;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int row = t * 16 + (lane & 15);
        const bf16x8_t afrag = __builtin_bit_cast(bf16x8_t, xs[lds_slot(row, slot)]);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afrag, bfrag, acc[t], 0, 0, 0);
      }
    }
  }

  // C/D map: col = lane & 15 (n), row = 4*(lane >> 4) + i (m).
  if (bn < N) {
    const float bv = bias != nullptr ? bf16_to_f32(bias[bn]) : 0.f;
    const float sc = pol.epilogue_scale(bn);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m_blk + t * 16 + 4 * (lane >> 4) + i;
        if (m < M) {
          float v = round_bf16(acc[t][i]);
          if (P::kScaled) v = round_bf16(v * sc);
          if (bias != nullptr) v = round_bf16(v + bv);
          y[(size_t)m * N + bn] = f32_to_bf16(v);
        }
      }
    }
  }
}

template <class P>
int launch_wo_mfma(const uint16_t* x, const P& pol, const uint16_t* bias, uint16_t* y, int M,
                   int N, int K, hipStream_t stream) {
  const int bm = M <= 16 ? 16 : (M <= 32 ? 32 : 64);
  dim3 grid((N + kBN - 1) / kBN, (M + bm - 1) / bm);
  if (bm == 16)
    launch((wo_mfma_kernel<16, P>), grid, dim3(256), 0, stream, x, pol, bias, y, M,
                       N, K);
  else if (bm == 32)
    launch((wo_mfma_kernel<32, P>), grid, dim3(256), 0, stream, x, pol, bias, y, M,
                       N, K);
  else
    launch((wo_mfma_kernel<64, P>), grid, dim3(256), 0, stream, x, pol, bias, y, M,
                       N, K);
  return check_launch("wo_mfma_kernel");
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

}  // namespace
}  // namespace tao

extern "C" int tao_int4wo_linear_bf16(const uint16_t* x, const uint32_t* packed,
                                      const uint16_t* sz, const uint16_t* bias, uint16_t* y,
                                      int64_t M, int64_t N, int64_t K, int64_t group_size,
                                      void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, sz, y, M, N, K, group_size);
  if (rc != TAO_OK) return rc;
  if (M == 0 || N == 0) return TAO_OK;
  hipStream_t st = tao::as_stream(stream);
  if (M <= 8) return tao::int4wo_gemv(x, packed, sz, bias, y, M, N, K, group_size, st);
  tao::Int4Policy pol;
  pol.wq = reinterpret_cast<const uint4*>(packed);
  pol.sz = reinterpret_cast<const uint32_t*>(sz);
  pol.gshift = tao::gshift_of(group_size);
  return tao::launch_wo_mfma(x, pol, bias, y, (int)M, (int)N, (int)K, st);
}

extern "C" int tao_int8wo_linear_bf16(const uint16_t* x, const int8_t* w, const uint16_t* scale,
                                      const uint16_t* bias, uint16_t* y, int64_t M, int64_t N,
                                      int64_t K, void* stream) {
  TAO_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "int8 weight-only linear: negative size");
  TAO_CHECK_ARG(K % 32 == 0, "int8 weight-only linear: K (%lld) must be a multiple of 32",
                (long long)K);
  TAO_CHECK_ARG(N < (1LL << 31) && K < (1LL << 31) && M < (1LL << 31),
                "int8 weight-only linear: size out of range");
  if (M == 0 || N == 0) return TAO_OK;
  TAO_CHECK_ARG(K > 0, "int8 weight-only linear: K must be > 0");
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(scale, 2, "scale");
  hipStream_t st = tao::as_stream(stream);
  if (M <= 8) return tao::int8wo_gemv(x, w, scale, bias, y, M, N, K, st);
  tao::Int8Policy pol;
  pol.w = reinterpret_cast<const uint4*>(w);
  pol.scale = scale;
  return tao::launch_wo_mfma(x, pol, bias, y, (int)M, (int)N, (int)K, st);
}
