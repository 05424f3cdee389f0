// Prefill GEMM for the quantized linears at M ~ 17..256 ("k-split" tile):
//   y[M][N] = epilogue(x[M][K] . W[N][K]^T), int4 weight-only (bf16 x) and int8 dynamic (int8 x).
//
// Built on two round-3 measurements:
//   * the prefill tiles are bound by the L2 -> CU intake, and that intake grows with the waves
//     and bytes in flight per CU: 57 GB/s per CU at 4 waves x 16 KiB, 96-104 at 8 waves,
//     107-112 at 16 waves with >= 32 KiB in flight (experiments/probe_l2_intake2.hip,
//     profiles/r3_probe_l2_intake_inflight.jsonl); the 4-wave stream tile spends 8.9 of its
//     10.6 µs (config 3) moving its 384 KiB per CU (profiles/r3_stream_debug_variants.jsonl);
//   * an unsplit 32 x 64 tile needs every x and W byte of the tile exactly once per workgroup,
//     (32 + 64) x K bytes of int8, and no split-K hand-off.
// So one workgroup of NW waves per 32 x 64 output tile, and the waves split K: wave w takes the
// k-blocks w, w + NW, w + 2 NW, ... (neighbouring waves read neighbouring bytes of each row) and
// loads its operands straight into registers in MFMA fragment order, NO LDS staging and no
// barrier in the k loop: each byte of the tile is loaded by exactly one wave. A D-deep register
// ring keeps D k-blocks of loads in flight per wave. At the end every wave's 32 x 64 partial goes
// to LDS ([NW][2048] words) and the workgroup sums the NW partials in wave order (int32 exact;
// fp32 in a fixed order: run-to-run deterministic), then the epilogue.
//
// Fragments (lane l: r = l % 16, q = l / 16; the MFMA's A/B lane layout):
//   int8 dynamic: k-block = 64 k; A[rb] = x[m0 + 16 rb + r][64 kb + 16 q .. +15],
//     B[cb] = W[n0 + 16 cb + r][64 kb + 16 q .. +15]; v_mfma_i32_16x16x64_i8 (exact int32);
//   int4 weight-only: k-block = 128 k; a lane's 16-B nibble load is the 32 k = 128 kb + 32 q ..
//     + 31 of row n0 + 16 cb + r (one (scale, zero) word), dword j of it feeding MFMA j with
//     B = bf16(fma(q, s, z - 8 s)) (gemm_mfma.hip's Int4WO numerics), and A of MFMA j =
//     x[m0 + 16 rb + r][128 kb + 32 q + 8 j .. + 7]; v_mfma_f32_16x16x32_bf16. A and B pair the
//     same k in every lane, so each MFMA's 32 k are a permutation of a contiguous 32-k span.
// Epilogues as gemm_mfma.hip: int4 bf16(acc) (+ bias); int8 dynamic bf16(bf16(bf16(acc) * xs) *
// ws) (+ bias) -- kernel/intmm.py:133-137, plain_layout.py:301-315 (bit-exact).
// Replaces aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104) and int_scaled_matmul
// (plain_layout.py:294-315) at prefill shapes.
#include "tao_common.h"

// Cache policy of the weight loads (timing experiments only): kNT (non-temporal) or 0.
#ifndef TAO_KSPLIT_WAUX
#define TAO_KSPLIT_WAUX kNT
#endif

namespace tao {
namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

// Output tile: RB x 16 rows by CB x 16 columns, RB x CB = 8 MFMA tiles per wave.

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// ---- int8 dynamic activation ------------------------------------------------------------------
template <int RB, int CB>
struct KInt8Dyn {
  static constexpr int kKB = 64;  // k per block
  static constexpr int kRB = RB, kCB = CB;
  typedef i32x4_t Acc;
  struct Frag {
    uint4 a[RB], b[CB];
  };
  struct Args {
    const uint8_t* x;  // [M][K] int8
    const uint8_t* w;  // [N][K] int8
  };
  Rsrc xr, wr;
  uint32_t xoff[RB], woff[CB];  // per-lane byte offsets of the fragments' rows at k = 16 q
  __device__ __forceinline__ void init(const Args& a, int m0, int n0, int M, int N, int K,
                                       int lane) {
    const uint8_t* x = a.x;
    const uint8_t* w = a.w;
    const int r = lane & 15, q = lane >> 4;
    xr = make_rsrc(x, (uint32_t)M * (uint32_t)K);
    wr = make_rsrc(w, (uint32_t)N * (uint32_t)K);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int m = m0 + 16 * rb + r < M ? m0 + 16 * rb + r : M - 1;  // clamped, masked at the end
      xoff[rb] = (uint32_t)m * (uint32_t)K + 16u * (uint32_t)q;
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) woff[cb] = (uint32_t)(n0 + 16 * cb + r) * (uint32_t)K + 16u * q;
  }
  __device__ __forceinline__ void load(Frag& f, int kb) const {
    const uint32_t so = (uint32_t)kb * 64u;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) f.b[cb] = bload16<TAO_KSPLIT_WAUX>(wr, woff[cb], so);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) f.a[rb] = bload16(xr, xoff[rb], so);
  }
  __device__ __forceinline__ void compute(const Frag& f, Acc (&acc)[RB][CB]) const {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int cb = 0; cb < CB; ++cb)
        acc[rb][cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
            __builtin_bit_cast(i32x4_t, f.a[rb]), __builtin_bit_cast(i32x4_t, f.b[cb]),
            acc[rb][cb], 0, 0, 0);
  }
  static __device__ __forceinline__ float epi(int acc, float xs, float ws) {
    const float v = round_bf16(round_bf16((float)acc) * xs);
    return round_bf16(v * ws);
  }
};

// ---- int4 weight-only -------------------------------------------------------------------------
template <int RB, int CB>
struct KInt4 {
  static constexpr int kKB = 128;
  static constexpr int kRB = RB, kCB = CB;
  typedef f32x4_t Acc;
  struct Frag {
    uint4 a[RB][4];  // x: row block rb, MFMA j
    uint4 w[CB];     // nibbles: column block cb
    uint32_t sz[CB]; // (scale, zero) of column block cb
  };
  struct Args {
    const uint16_t* x;   // [M][K] bf16
    const uint32_t* w;   // [N][K/8] row-stream nibbles
    const uint32_t* sz;  // [N][K/g] (scale, zero) bf16 pairs
    int gshift;          // g = 32 << gshift
  };
  Rsrc xr, wr, zr;
  uint32_t xoff[RB], woff[CB], zoff[CB];
  int gshift;
  __device__ __forceinline__ void init(const Args& a, int m0, int n0, int M, int N, int K,
                                       int lane) {
    const uint16_t* x = a.x;
    const uint32_t* w = a.w;
    const uint32_t* sz = a.sz;
    const int gs = a.gshift;
    const int r = lane & 15, q = lane >> 4;
    gshift = gs;
    xr = make_rsrc(x, (uint32_t)M * (uint32_t)K * 2u);
    wr = make_rsrc(w, (uint32_t)N * (uint32_t)(K >> 1));
    const uint32_t zrow = (uint32_t)(K >> (5 + gs)) * 4u;  // bytes of (scale, zero) per row
    zr = make_rsrc(sz, (uint32_t)N * zrow);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int m = m0 + 16 * rb + r < M ? m0 + 16 * rb + r : M - 1;
      xoff[rb] = (uint32_t)m * (uint32_t)K * 2u + 64u * (uint32_t)q;
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const uint32_t n = (uint32_t)(n0 + 16 * cb + r);
      woff[cb] = n * (uint32_t)(K >> 1) + 16u * (uint32_t)q;
      // group of k = 128 kb + 32 q is (4 kb + q) >> gs = ((4 kb) >> gs) + (q >> gs): groups are
      // >= 32 k and 32-aligned, so the lane part never carries into the block part
      zoff[cb] = n * zrow + 4u * (uint32_t)(q >> gs);
    }
  }
  __device__ __forceinline__ void load(Frag& f, int kb) const {
    const uint32_t sw = (uint32_t)kb * 64u, sx = (uint32_t)kb * 256u;
    const uint32_t sz = 4u * (uint32_t)((4 * kb) >> gshift);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) f.w[cb] = bload16<TAO_KSPLIT_WAUX>(wr, woff[cb], sw);
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) f.sz[cb] = bload4<TAO_KSPLIT_WAUX>(zr, zoff[cb], sz);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int j = 0; j < 4; ++j) f.a[rb][j] = bload16(xr, xoff[rb] + 16u * (uint32_t)j, sx);
  }
  static __device__ __forceinline__ uint4 dq8(uint32_t w, float s, float zc) {
    // row-stream nibble order -> 8 bf16 in k order: bf16(fma(q, s, z - 8 s)); a nibble byte b
    // read as OCP e4m3 is b / 512 exactly
    const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
    const f32x2_t q04 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, false);
    const f32x2_t q15 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, true);
    const f32x2_t q26 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, false);
    const f32x2_t q37 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, true);
    const float w0 = __builtin_fmaf(q04[0], s, zc), w4 = __builtin_fmaf(q04[1], s, zc);
    const float w1 = __builtin_fmaf(q15[0], s, zc), w5 = __builtin_fmaf(q15[1], s, zc);
    const float w2 = __builtin_fmaf(q26[0], s, zc), w6 = __builtin_fmaf(q26[1], s, zc);
    const float w3 = __builtin_fmaf(q37[0], s, zc), w7 = __builtin_fmaf(q37[1], s, zc);
    return make_uint4(pk_bf16(w0, w1), pk_bf16(w2, w3), pk_bf16(w4, w5), pk_bf16(w6, w7));
  }
  __device__ __forceinline__ void compute(const Frag& f, Acc (&acc)[RB][CB]) const {
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const float s = bf16lo_to_f32(f.sz[cb]);
      const float zc = bf16hi_to_f32(f.sz[cb]) - 8.f * s;  // q * s + zc == (q - 8) * s + z
      const uint32_t d4[4] = {f.w[cb].x, f.w[cb].y, f.w[cb].z, f.w[cb].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 b = dq8(d4[j], s, zc);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, f.a[rb][j]), __builtin_bit_cast(bf16x8_t, b),
              acc[rb][cb], 0, 0, 0);
      }
    }
  }
  static __device__ __forceinline__ float epi(float acc, float, float) { return round_bf16(acc); }
};

// grid (N / 64, ceil(M / 32)), NW * 64 threads; K = NW * D * kKB * (blocks per wave / D).
template <class P, int NW, int D, bool kRowF, bool kColF>
__global__ __launch_bounds__(NW * 64) void gemm_ksplit_kernel(
    typename P::Args args, const uint16_t* __restrict__ rowf, const uint16_t* __restrict__ colf,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K,
    int rotate) {
  typedef typename P::Acc Acc;
  __shared__ __attribute__((aligned(16))) uint4 red[NW][512];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int RB = P::kRB, CB = P::kCB;
  static_assert(RB * CB == 8, "8 MFMA tiles per wave");
  const int n0 = blockIdx.x * (16 * CB), m0 = blockIdx.y * (16 * RB);
  const int nb = K / (P::kKB * NW);  // k-blocks of this wave: wave + i NW, i < nb
  P pol;
  pol.init(args, m0, n0, M, N, K, lane);

  Acc acc[RB][CB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = Acc{0, 0, 0, 0};

  typename P::Frag f[D];
  // rotate: the workgroup walks its wave's blocks from a rotated start, so that the workgroups
  // sharing an operand tile (the M tiles of one weight tile, the N tiles of one x tile) do not
  // all miss on the same lines at once; wave w still takes exactly the blocks = w mod NW
  const int rot =
      rotate ? (int)((blockIdx.y * (unsigned)((nb + 3) / 4) + blockIdx.x) % (unsigned)nb) : 0;
  auto blk = [&](int i) __attribute__((always_inline)) {
    int j = i + rot;
    j = j >= nb ? j - nb : j;
    return wave + j * NW;
  };
#pragma unroll
  for (int d = 0; d < D; ++d) pol.load(f[d], blk(d));
  int i = 0;
#pragma unroll 1
  for (; i + D < nb; i += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      pol.compute(f[d], acc);
      pol.load(f[d], blk(i + D + d));
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) pol.compute(f[d], acc);

  // the NW partial tiles -> LDS, summed in wave order
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
      red[wave][(rb * CB + cb) * 64 + lane] = __builtin_bit_cast(uint4, acc[rb][cb]);
  __syncthreads();
#pragma unroll
  for (int e = threadIdx.x; e < 512; e += NW * 64) {
    Acc t = __builtin_bit_cast(Acc, red[0][e]);
#pragma unroll
    for (int w = 1; w < NW; ++w) t += __builtin_bit_cast(Acc, red[w][e]);
    const int rc = e >> 6, l = e & 63;
    const int col = n0 + 16 * (rc % CB) + (l & 15);
    const float cf = kColF ? bf16_to_f32(colf[col]) : 1.f;
    const float bv = bias != nullptr ? bf16_to_f32(bias[col]) : 0.f;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int m = m0 + 16 * (rc / CB) + 4 * (l >> 4) + ii;
      if (m < M) {
        float v = P::epi(t[ii], kRowF ? bf16_to_f32(rowf[m]) : 1.f, cf);
        if (bias != nullptr) v = round_bf16(v + bv);
        y[(size_t)m * N + col] = f32_to_bf16(v);
      }
    }
  }
}

// Launch shapes: an RB x CB tile of 16 x 16 MFMA blocks per workgroup, NW waves, D k-blocks in
// flight per wave. K must split into NW x D x kKB pieces; the ring depth is halved until it
// divides the wave's k-blocks.
struct KCfg {
  int rb, cb, nw, d;
};

template <int KB>
bool kcfg_ok(int64_t K, KCfg c) {
  const int64_t per = (int64_t)KB * c.nw;
  return K % per == 0 && (K / per) % c.d == 0 && K / per >= c.d;
}

template <int KB>
KCfg fit_depth(int64_t K, KCfg c) {
  while (c.d > 1 && !kcfg_ok<KB>(K, c)) c.d /= 2;
  return c;
}

// tao_tune_gemm_ksplit shape: 0 built-in; 1 32 x 64 tile, 2 64 x 32, 3 128 x 16, 4 128 x 16 on
// 16 waves (int8) / 32 x 64 with one block in flight (int4)
KCfg kcfg_int8(int64_t K) {
  KCfg c{8, 1, 8, 4};
  switch (tuning().gemm_ksplit_shape) {
    case 1: c = {2, 4, 8, 4}; break;
    case 2: c = {4, 2, 8, 4}; break;
    case 3: c = {8, 1, 8, 4}; break;
    case 4: c = {8, 1, 16, 2}; break;
    default: break;
  }
  return fit_depth<64>(K, c);
}

KCfg kcfg_int4(int64_t K) {  // (64 x 32 with two blocks in flight spills: one)
  KCfg c{4, 2, 8, 1};
  switch (tuning().gemm_ksplit_shape) {
    case 1: c = {2, 4, 8, 2}; break;
    case 2: c = {4, 2, 8, 1}; break;
    case 3: c = {8, 1, 8, 1}; break;
    case 4: c = {2, 4, 8, 1}; break;
    default: break;
  }
  return fit_depth<128>(K, c);
}

}  // namespace

// ---- routing and launchers ------------------------------------------------------------------
// path 0 int4, 2 int8 dynamic. Shapes the kernel covers: N a multiple of the tile's columns, K
// split evenly over the waves (kcfg_ok), operands below 4 GiB. Auto routing
// (tuning().gemm_ksplit == 0): none until measured (profiles/r3_ab_ksplit*.jsonl).
bool use_ksplit(int path, int64_t M, int64_t N, int64_t K, int64_t group_size) {
  const int mode = tuning().gemm_ksplit;
  if (mode == 1) return false;
  if (path != 0 && path != 2) return false;
  if (M < 1 || N * K >= (int64_t(1) << 32) || M * K * 2 >= (int64_t(1) << 32)) return false;
  if (path == 0 && (group_size < 32 || group_size > 256 || (group_size & (group_size - 1))))
    return false;
  const KCfg c = path == 2 ? kcfg_int8(K) : kcfg_int4(K);
  const bool ok = path == 2 ? kcfg_ok<64>(K, c) : kcfg_ok<128>(K, c);
  if (!ok || N % (16 * c.cb) != 0) return false;
  if (mode == 2) return true;
  const Tuning& t = tuning();
  if (t.bm || t.kg || t.splits || t.gemm_nw || t.int4_mfma32 || t.gemm_algo || t.gemm_tile ||
      t.gemm_stream)
    return false;
  return false;
}

template <class P, int NW, int D, bool kRowF, bool kColF>
int launch_ksplit(const typename P::Args& a, const uint16_t* rowf, const uint16_t* colf,
                  const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
                  const char* name) {
  const dim3 grid((unsigned)(N / (16 * P::kCB)), (unsigned)((M + 16 * P::kRB - 1) / (16 * P::kRB)));
  launch(gemm_ksplit_kernel<P, NW, D, kRowF, kColF>, grid, dim3(NW * 64), 0, stream, a, rowf,
         colf, bias, y, M, N, K, tuning().gemm_ksplit_rot);
  return check_launch(name);
}

int ksplit_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int gshift,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  const KCfg c = kcfg_int4(K);
  TAO_CHECK_ARG(N % (16 * c.cb) == 0 && kcfg_ok<128>(K, c) && gshift >= 0 && gshift <= 3,
                "k-split GEMM: N %% %d, K a multiple of %d and g in {32..256} required",
                16 * c.cb, 128 * c.nw * c.d);
  const char* nm = "gemm_ksplit_kernel<int4>";
#define TAO_KS4(RB_, CB_, NW_, D_)                                                              \
  if (c.rb == RB_ && c.cb == CB_ && c.nw == NW_ && c.d == D_) {                                \
    typename KInt4<RB_, CB_>::Args a{x, packed, reinterpret_cast<const uint32_t*>(sz), gshift}; \
    return launch_ksplit<KInt4<RB_, CB_>, NW_, D_, false, false>(a, nullptr, nullptr, bias, y, M, \
                                                                 N, K, stream, nm);            \
  }
  TAO_KS4(2, 4, 8, 2) TAO_KS4(2, 4, 8, 1) TAO_KS4(4, 2, 8, 1) TAO_KS4(8, 1, 8, 1)
#undef TAO_KS4
  TAO_CHECK_ARG(false, "k-split GEMM: no int4 instance for this shape");
  return TAO_ERR_UNSUPPORTED;
}

int ksplit_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
                   const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  const KCfg c = kcfg_int8(K);
  TAO_CHECK_ARG(N % (16 * c.cb) == 0 && kcfg_ok<64>(K, c),
                "k-split GEMM: N %% %d and K a multiple of %d required", 16 * c.cb,
                64 * c.nw * c.d);
  const char* nm = "gemm_ksplit_kernel<int8dyn>";
#define TAO_KS8(RB_, CB_, NW_, D_)                                                              \
  if (c.rb == RB_ && c.cb == CB_ && c.nw == NW_ && c.d == D_) {                                \
    typename KInt8Dyn<RB_, CB_>::Args a{reinterpret_cast<const uint8_t*>(xq),                  \
                                        reinterpret_cast<const uint8_t*>(wq)};                 \
    return launch_ksplit<KInt8Dyn<RB_, CB_>, NW_, D_, true, true>(a, xs, ws, bias, y, M, N, K,  \
                                                                  stream, nm);                 \
  }
  TAO_KS8(2, 4, 8, 4) TAO_KS8(2, 4, 8, 2) TAO_KS8(2, 4, 8, 1)
  TAO_KS8(4, 2, 8, 4) TAO_KS8(4, 2, 8, 2) TAO_KS8(4, 2, 8, 1)
  TAO_KS8(8, 1, 8, 4) TAO_KS8(8, 1, 8, 2) TAO_KS8(8, 1, 8, 1)
  TAO_KS8(8, 1, 16, 2) TAO_KS8(8, 1, 16, 1)
#undef TAO_KS8
  TAO_CHECK_ARG(false, "k-split GEMM: no int8 instance for this shape");
  return TAO_ERR_UNSUPPORTED;
}

}  // namespace tao

extern "C" int tao_tune_gemm_ksplit(int mode, int shape) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 2,
                "tune: gemm k-split mode must be 0 (auto), 1 (off) or 2 (on)");
  TAO_CHECK_ARG((shape & 15) <= 4 && shape >= 0 && shape < 32,
                "tune: gemm k-split shape must be 0..4 (+16: rotated block order)");
  tao::tuning().gemm_ksplit = mode;
  tao::tuning().gemm_ksplit_shape = shape & 15;
  tao::tuning().gemm_ksplit_rot = shape >> 4;
  return TAO_OK;
}
