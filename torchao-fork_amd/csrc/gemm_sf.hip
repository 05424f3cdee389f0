// Single-fetch prefill GEMM for the quantized linears at 64 < M <= 128 (BASELINE config 3 and the
// int4 linears of a 128-token prefill):  y[M][N] = epilogue( x[M][K] . W[N][K]^T )
//   SfI4    : bf16 x, int4 row-stream W + (scale, zero) per group, v_mfma_f32_16x16x32_bf16,
//             B = bf16(fma(q, s, z - 8 s)), y = bf16(acc) (+ bias)
//   SfI8<KS>: int8 x (per-token scale), int8 W (per-channel scale), v_mfma_i32_16x16x64_i8,
//             y = bf16(bf16(bf16(acc) * xs) * ws) (+ bias)     (bit-exact to the reference)
// Replaces aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104) and int_scaled_matmul +
// scales (kernel/intmm.py:82,108-143; plain_layout.py:294-315) at prefill sizes.
//
// What DESIGN §4.2b measured a prefill GEMM on this chip must do, and how this kernel does it:
//   * every weight tile is fetched from HBM by exactly ONE workgroup: the tile covers all 128
//     rows of M (a cold tile read by several workgroups at once streamed at ~36 GB/s per CU,
//     §4.2b pattern table), so HBM traffic is the algorithmic bytes;
//   * full-line loads only: both operands reach LDS by LDS-DMA in whole 128-B lines, XOR-swizzled
//     by choosing each lane's source so that every ds_read_b128 fragment read is conflict-free;
//   * 8 waves and NS-1 stages (32-48 KiB each) in flight per CU: a counted vmcnt + a barrier
//     that does not drain vector memory keep them in flight across every step;
//   * K split S ways over workgroups (the grid fills the 256 CUs) with a fixed reducer: slices
//     0..S-2 publish their fp32 / int32 partial tile (sc1 stores, one ticket add), slice S-1
//     (dispatched last, so a publisher never waits behind it) polls the ticket, sums the slabs
//     in slice order (run-to-run deterministic; int32 exact) and runs the epilogue. Publishers
//     may take fewer K steps than the reducer (`a_steps`) so their publish overlaps its work.
// Wave layout: WM x WN waves over the 128 x BN tile (wave tile 128/WM x BN/WN).
#include <type_traits>

#include "tao_common.h"

// Experiment switch (timing only, experiments/sf_stamps.py): per-workgroup s_memrealtime stamps
// (100 MHz): 0 entry, 1 prologue DMAs issued, 2 first stage landed, 3 k loop done, 4 publish or
// poll done, 5 end; 6 = slice, 7 = 1 for the reducer. Never in the product library.
#ifndef TAO_SF_STAMPS
#define TAO_SF_STAMPS 0
#endif

namespace tao {

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;   // rows per tile
constexpr int kWaves = 8;  // 512 threads

#if TAO_SF_STAMPS
__device__ unsigned long long g_sf_stamps[8192 * 8];
#endif
// reducer poll timeouts (never expected: publishers never wait, and they precede the reducers in
// every XCD's dispatch order); read and cleared by tao_gemm_sf_status()
__device__ unsigned g_sf_err = 0;

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// ---- image swizzles (positions of 16-B granules inside an image row; each is an involution, so
// the DMA lane that fills position p fetches granule pos(row, p)) ---------------------------------
// 256-B rows read in natural k order (lane (r, kq) of k-sub kb reads granule 4 kb + kq): XOR with
// r & 15 puts the 16 lanes of every ds_read_b128 lane group on 16 distinct bank granules.
__device__ __forceinline__ int pos256(int row, int g) { return g ^ (row & 15); }
// 256-B rows read in the int4 order (granule 4 kq + kb): flip bit 2 of r & 15 on rows whose bits
// 2 and 3 differ (gemm_mfma.hip's Int4WO x image mask; checked by tests/test_host_cpu.py).
__device__ __forceinline__ int pos256q(int row, int g) {
  const int m = row & 15;
  return g ^ (m ^ ((m ^ (m >> 1)) & 4));
}
// 128-B rows in natural order (granule 4 kb + kq): XOR with (r >> 1) & 7 (two rows per bank row)
__device__ __forceinline__ int pos128(int row, int g) { return g ^ ((row >> 1) & 7); }
// int4 nibble image [BN][4 granules] read by lane (n, kq) at granule kq: XOR with (4 - (n >> 2)) & 3
__device__ __forceinline__ int pos64(int row, int g) { return g ^ ((4 - ((row >> 2) & 3)) & 3); }
// (scale, zero) image [BN][4 dwords] read by lane (n, kq) at dword kq: XOR with 2 ((n >> 3) & 1)
__device__ __forceinline__ int posz(int row, int q) { return q ^ (((row >> 3) & 1) << 1); }

// ---- policies -----------------------------------------------------------------------------------
template <int KS>
struct SfI8 {
  static constexpr int kXRow = KS;  // x bytes per row per step
  static constexpr int kWRow = KS;  // W bytes per row per step
  static constexpr int kZRow = 0;
  static constexpr int kKStep = KS;
  static constexpr int kKB = KS / 64;  // MFMAs per fragment pair per step
  static constexpr int kABytes = 1;
  typedef i32x4_t Acc;
  const int8_t* w;
  const uint16_t* wscale;
  const uint16_t* xscale;
  static __device__ __forceinline__ int xpos(int row, int g) {
    if constexpr (KS == 256) return pos256(row, g);
    else return pos128(row, g);
  }
  static __device__ __forceinline__ int agran(int kb, int kq) { return 4 * kb + kq; }
  __device__ __forceinline__ Rsrc wrsrc(int N, int K) const {
    return make_rsrc(w, (uint32_t)N * (uint32_t)K);
  }
  __device__ __forceinline__ Rsrc zrsrc(int, int) const { return make_rsrc(w, 0); }
  // W piece i: rows (1024 / KS) i .., lane: row + lane / (KS / 16), granule position lane % (KS / 16)
  __device__ __forceinline__ uint32_t wsrc(int i, int lane, int n_blk, int N, int K) const {
    constexpr int G = KS / 16;
    const int row = i * (1024 / KS) + lane / G, p = lane % G;
    const int gn = n_blk + row < N ? n_blk + row : N - 1;
    return (uint32_t)gn * (uint32_t)K + 16u * (uint32_t)xpos(row, p);
  }
  __device__ __forceinline__ uint32_t wsoff(int st) const { return (uint32_t)st * KS; }
  __device__ __forceinline__ uint32_t zsrc(int, int, int, int, int) const { return 0; }
  __device__ __forceinline__ uint32_t zsoff(int) const { return 0; }
  __device__ __forceinline__ const uint16_t* n_elems() const { return wscale; }  // >= N elements
  __device__ __forceinline__ uint32_t zword(int, int, int) const { return 0; }
};

struct SfI4 {
  static constexpr int kXRow = 256;  // 128 bf16 k
  static constexpr int kWRow = 64;   // 128 nibbles
  static constexpr int kZRow = 16;   // 4 (scale, zero) dwords: the group of each lane's 32 k
  static constexpr int kKStep = 128;
  static constexpr int kABytes = 2;
  typedef f32x4_t Acc;
  const uint32_t* wq;  // [N][K/8] row-stream packed
  const uint32_t* sz;  // [N][K/g] (scale, zero) bf16 pairs
  int lg;              // log2(group size)
  static __device__ __forceinline__ int xpos(int row, int g) { return pos256q(row, g); }
  // MFMA kb of lane kq covers k 32 kq + 8 kb .. + 8 of the step (its nibble dword kb of granule kq)
  static __device__ __forceinline__ int agran(int kb, int kq) { return 4 * kq + kb; }
  __device__ __forceinline__ Rsrc wrsrc(int N, int K) const {
    return make_rsrc(wq, (uint32_t)N * (uint32_t)(K >> 1));
  }
  __device__ __forceinline__ Rsrc zrsrc(int N, int K) const {
    return make_rsrc(sz, (uint32_t)N * (uint32_t)(K >> lg) * 4u);
  }
  // W piece i: 16 rows x 64 B (lane: row 16 i + lane / 4, position lane % 4)
  __device__ __forceinline__ uint32_t wsrc(int i, int lane, int n_blk, int N, int K) const {
    const int row = 16 * i + (lane >> 2), p = lane & 3;
    const int gn = n_blk + row < N ? n_blk + row : N - 1;
    return (uint32_t)gn * (uint32_t)(K >> 1) + 16u * (uint32_t)pos64(row, p);
  }
  __device__ __forceinline__ uint32_t wsoff(int st) const { return (uint32_t)st * 64u; }
  // Z piece i (4-B DMA): 16 rows x 4 dwords; dword q of row n = the group holding k 32 q of the
  // step: ((128 st) >> lg) + ((32 q) >> lg) (exact for every g in 32..256 with g | K)
  __device__ __forceinline__ uint32_t zsrc(int i, int lane, int n_blk, int N, int K) const {
    const int row = 16 * i + (lane >> 2), q = posz(row, lane & 3);
    const int gn = n_blk + row < N ? n_blk + row : N - 1;
    return ((uint32_t)gn * (uint32_t)(K >> lg) + (uint32_t)((32 * q) >> lg)) * 4u;
  }
  __device__ __forceinline__ uint32_t zsoff(int st) const {
    return (uint32_t)(((128 * st) >> lg) * 4);
  }
  // REG staging: byte offset of the (scale, zero) word of row gn for 32-k quarter q of step 0
  __device__ __forceinline__ uint32_t zword(int gn, int q, int K) const {
    return ((uint32_t)gn * (uint32_t)(K >> lg) + (uint32_t)((32 * q) >> lg)) * 4u;
  }
  // >= N bf16 elements: the (scale, zero) array ([N][K/g][2], K >= g)
  __device__ __forceinline__ const uint16_t* n_elems() const {
    return reinterpret_cast<const uint16_t*>(sz);
  }
};

// int4 B fragment: 8 nibbles (row-stream dword: q0,q4,q1,q5 in the bytes of w & 0x0F0F0F0F,
// q2,q6,q3,q7 in those of (w >> 4) & 0x0F0F0F0F) -> bf16(fma(q, s, z - 8 s)) in k order. A byte
// b < 16 read as OCP e4m3 is exactly b / 512: one v_cvt_scalef32_pk_f32_fp8 (scale 512) gives
// two exact fp32 integers (gemm_mfma.hip Int4WO::frag).
__device__ __forceinline__ bf16x8_t deq8(uint32_t w, float sc, float zc) {
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
  const f32x2_t q04 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, false);
  const f32x2_t q15 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, true);
  const f32x2_t q26 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, false);
  const f32x2_t q37 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, true);
  const f32x2_t sv = {sc, sc}, zv = {zc, zc};
  const f32x2_t w04 = q04 * sv + zv, w15 = q15 * sv + zv;
  const f32x2_t w26 = q26 * sv + zv, w37 = q37 * sv + zv;
  const u32x4_t v = {pk_bf16(w04[0], w15[0]), pk_bf16(w26[0], w37[0]), pk_bf16(w04[1], w15[1]),
                     pk_bf16(w26[1], w37[1])};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int N>
__device__ __forceinline__ void wait_ahead(int ahead) {
  // vmcnt(ahead x N): the DMAs of the `ahead` stages issued after the one about to be read
  switch (ahead) {
    case 0: wait_vmcnt<0>(); break;
    case 1: wait_vmcnt<N>(); break;
    case 2: wait_vmcnt<2 * N>(); break;
    default: wait_vmcnt<3 * N>(); break;
  }
}

// REG: register staging instead of LDS-DMA (NS = register ring depth, two LDS buffers). The DMA
// path's per-step time measured 0.59 us for 40 KiB per CU at config 3 (experiments/sf_stamps.py):
// ~68 GB/s per CU, the LDS-DMA intake MI355X_MICROARCH.md's ring-gemm row reports; 16-B loads into
// registers took in 96-112 GB/s per CU at 8-16 waves (DESIGN §4.2b intake table).
template <class P, int BN, int WM, int NS, bool REG = false>
__global__ __launch_bounds__(512) void gemm_sf_kernel(
    const uint8_t* __restrict__ x, P pol, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int a_steps, typename P::Acc* __restrict__ slab,
    unsigned* __restrict__ cnt, int fenced) {
#if TAO_SF_STAMPS
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
  unsigned long long stamp[6] = {t_entry, 0, 0, 0, 0, 0};
#define SF_MARK(i) \
  if (threadIdx.x == 0) stamp[i] = __builtin_amdgcn_s_memrealtime()
#else
#define SF_MARK(i) \
  do {             \
  } while (0)
#endif
  typedef typename P::Acc Acc;
  constexpr int WN = kWaves / WM;
  constexpr int RM = kBM / WM, CN = BN / WN;  // wave tile
  constexpr int MT = RM / 16, NT = CN / 16;
  static_assert(MT >= 1 && NT >= 1, "wave tile");
  constexpr int XB = kBM * P::kXRow, WB = BN * P::kWRow, ZB = BN * P::kZRow;
  constexpr int STAGE = XB + WB + ZB;  // bytes per stage
  constexpr int PX = XB / 1024, PW = WB / 1024, PZ = ZB / 256;
  constexpr int T = PX + PW + PZ;
  static_assert(XB % 1024 == 0 && WB % 1024 == 0 && ZB % 256 == 0, "DMA pieces");
  static_assert(T % kWaves == 0 && PX % kWaves == 0, "DMA pieces per wave");
  constexpr int R = T / kWaves;  // DMA instructions per wave per stage
  constexpr int NB = REG ? 2 : NS;  // LDS stage buffers
  static_assert(NB * STAGE <= 160 * 1024, "LDS");
  static_assert(kBM * BN * 2 <= NB * STAGE, "epilogue image");
  __shared__ uint4 lds[NB * STAGE / 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, kq = lane >> 4;
  const int n_blk = blockIdx.x * BN, m_blk = blockIdx.z * kBM;
  const int S = gridDim.y, z = blockIdx.y;
  const bool reducer = z == S - 1;
  const int nsteps = K / P::kKStep;
  const int s0 = z * a_steps;
  const int J = reducer ? nsteps - s0 : a_steps;  // launcher: every slice >= 1 step
  const uint32_t row_bytes = (uint32_t)K * P::kABytes;

  // ---- DMA slots: this wave's R pieces per stage (piece i = 8 r + wave) --------------------------
  const Rsrc xrs = make_rsrc(x, (uint32_t)M * row_bytes);
  const Rsrc wrs = pol.wrsrc(N, K);
  const Rsrc zrs = pol.zrsrc(N, K);
  uint32_t dv[R];
  int dd[R], dk[R];
  sfor<0, R>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (r < PX / kWaves) {
      constexpr int G = P::kXRow / 16;
      const int i = r * kWaves + wave;
      const int row = i * (1024 / P::kXRow) + lane / G, p = lane % G;
      const int gm = m_blk + row < M ? m_blk + row : M - 1;
      dv[r] = (uint32_t)gm * row_bytes + 16u * (uint32_t)P::xpos(row, p);
      dd[r] = i * 1024;
      dk[r] = 0;
    } else {
      const int i = (r - PX / kWaves) * kWaves + wave;
      if (i < PW) {
        dv[r] = pol.wsrc(i, lane, n_blk, N, K);
        dd[r] = XB + i * 1024;
        dk[r] = 1;
      } else {
        dv[r] = pol.zsrc(i - PW, lane, n_blk, N, K);
        dd[r] = XB + WB + (i - PW) * 256;
        dk[r] = 2;
      }
    }
  });
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    uint8_t* base = reinterpret_cast<uint8_t*>(lds) + buf * STAGE;
    sfor<0, R>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if constexpr (r < PX / kWaves) {
        dma_lds<16>(xrs, dv[r], (uint32_t)st * P::kXRow, base + dd[r]);
      } else {
        if (dk[r] == 1) dma_lds<16, kNT>(wrs, dv[r], pol.wsoff(st), base + dd[r]);
        else if constexpr (PZ > 0) dma_lds<4, kNT>(zrs, dv[r], pol.zsoff(st), base + dd[r]);
      }
    });
  };

  // ---- epilogue operands, loaded ahead of the stream ---------------------------------------------
  // rows of this lane: wm RM + 16 mt + 4 kq + i; columns: wn CN + 16 nt + fr
  constexpr bool kI8 = P::kABytes == 1;
  float xsf[kI8 ? MT * 4 : 1];
  float wsf[NT], bsf[NT];
  if constexpr (kI8) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m_blk + wm * RM + 16 * mt + 4 * kq + i;
        xsf[mt * 4 + i] = bf16_to_f32(pol.xscale[m < M ? m : M - 1]);
      }
  }
  // the bias load is unconditional (from a stand-in array of >= N elements when there is none):
  // a load behind `bias != nullptr` compiles to a branch and a vmcnt(0) at its join, one memory
  // round trip before the first DMA is issued
  const uint16_t* bsrc = bias != nullptr ? bias : pol.n_elems();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = n_blk + wn * CN + 16 * nt + fr;
    const int nn = n < N ? n : N - 1;
    if constexpr (kI8) wsf[nt] = bf16_to_f32(pol.wscale[nn]);
    else wsf[nt] = 1.f;
    bsf[nt] = bf16_to_f32(bsrc[nn]);
  }

  Acc acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = Acc{0, 0, 0, 0};

  // ---- one step: fragments from stage `buf`, MFMAs -------------------------------------------------
  // Every fragment read of the step is issued before the first MFMA (a sched_barrier keeps
  // hipcc from interleaving them one read per MFMA, which exposed each ds_read's latency: one
  // read in flight per wave, lgkmcnt(1) before every MFMA in the first build's ISA).
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const uint4* img = lds + buf * (STAGE / 16);
    if constexpr (kI8) {
      constexpr int G = P::kXRow / 16;  // granules per image row
      i32x4_t bf[P::kKB][NT], af[P::kKB][MT];
#pragma unroll
      for (int kb = 0; kb < P::kKB; ++kb) {
        const int g = P::agran(kb, kq);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = wn * CN + 16 * nt + fr;
          bf[kb][nt] = __builtin_bit_cast(i32x4_t, img[XB / 16 + n * G + P::xpos(n, g)]);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int m = wm * RM + 16 * mt + fr;
          af[kb][mt] = __builtin_bit_cast(i32x4_t, img[m * G + P::xpos(m, g)]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kb = 0; kb < P::kKB; ++kb)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(af[kb][mt], bf[kb][nt], acc[mt][nt], 0, 0, 0);
    } else {
      uint4 wv[NT];
      uint32_t szw[NT];
      bf16x8_t af[4][MT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = wn * CN + 16 * nt + fr;
        wv[nt] = img[XB / 16 + n * 4 + pos64(n, kq)];
        szw[nt] = reinterpret_cast<const uint32_t*>(img)[(XB + WB) / 4 + n * 4 + posz(n, kq)];
      }
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int g = P::agran(kb, kq);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int m = wm * RM + 16 * mt + fr;
          af[kb][mt] = __builtin_bit_cast(bf16x8_t, img[m * 16 + P::xpos(m, g)]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      float sc[NT], zc[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        sc[nt] = bf16lo_to_f32(szw[nt]);
        zc[nt] = bf16hi_to_f32(szw[nt]) - 8.f * sc[nt];  // q*s + zc == (q - 8)*s + z
      }
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        bf16x8_t bf[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint32_t wd = kb == 0 ? wv[nt].x : kb == 1 ? wv[nt].y : kb == 2 ? wv[nt].z : wv[nt].w;
          bf[nt] = deq8(wd, sc[nt], zc[nt]);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kb][mt], bf[nt], acc[mt][nt], 0, 0, 0);
      }
    }
  };

  // ---- the k loop ---------------------------------------------------------------------------------
  if constexpr (!REG) {
    // LDS-DMA: NS-1 stages in flight, one barrier per step
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (p < J) issue(s0 + p, p);
    SF_MARK(1);
    for (int j = 0; j < J; ++j) {
      const int ahead = J - 1 - j < NS - 2 ? J - 1 - j : NS - 2;
      wait_ahead<R>(ahead);  // this wave's DMAs of step j landed
      barrier_lgkm();        // ... and every wave's; step j - 1's fragment reads are done
#if TAO_SF_STAMPS
      if (j == 0) SF_MARK(2);
#endif
      if (j + NS - 1 < J) issue(s0 + j + NS - 1, (j + NS - 1) % NS);
      compute(j % NS);
    }
  } else {
    // Register staging: thread t loads granules t + 512 i of each image in source order (whole
    // lines across consecutive threads) D = NS steps ahead, then writes them at their swizzled
    // image positions (the layout the DMA path builds). Loads past the slice re-read its last
    // step (never predicated: a branch around a load makes hipcc drain vmcnt at the join).
    constexpr int D = NS;
    constexpr int GX = P::kXRow / 16, GW = P::kWRow / 16;
    constexpr int XG = kBM * GX / 512;                    // x granules per thread
    constexpr int WGN = BN * GW, WG = (WGN + 511) / 512;  // W granules (all threads / per thread)
    constexpr int ZGN = BN * P::kZRow / 4, ZG = (ZGN + 511) / 512;  // (scale, zero) dwords
    static_assert(kBM * GX % 512 == 0, "x granules per thread");
    uint32_t xv[XG], wv[WG], zv[ZG > 0 ? ZG : 1];
    int xw[XG], ww[WG], zw[ZG > 0 ? ZG : 1];
#pragma unroll
    for (int i = 0; i < XG; ++i) {
      const int e = tid + 512 * i, row = e / GX, g = e % GX;
      const int gm = m_blk + row < M ? m_blk + row : M - 1;
      xv[i] = (uint32_t)gm * row_bytes + 16u * (uint32_t)g;
      xw[i] = row * P::kXRow + 16 * P::xpos(row, g);
    }
#pragma unroll
    for (int i = 0; i < WG; ++i) {
      const int e0 = tid + 512 * i, e = e0 < WGN ? e0 : WGN - 1;
      const int row = e / GW, g = e % GW;
      const int gn = n_blk + row < N ? n_blk + row : N - 1;
      if constexpr (P::kZRow > 0) {  // int4 nibbles: K / 2 bytes per row
        wv[i] = (uint32_t)gn * (uint32_t)(K >> 1) + 16u * (uint32_t)g;
        ww[i] = e0 < WGN ? XB + row * P::kWRow + 16 * pos64(row, g) : -1;
      } else {
        wv[i] = (uint32_t)gn * (uint32_t)K + 16u * (uint32_t)g;
        ww[i] = e0 < WGN ? XB + row * P::kWRow + 16 * P::xpos(row, g) : -1;
      }
    }
    if constexpr (ZG > 0) {
#pragma unroll
      for (int i = 0; i < ZG; ++i) {
        const int e0 = tid + 512 * i, e = e0 < ZGN ? e0 : ZGN - 1;
        const int row = e >> 2, q = e & 3;
        const int gn = n_blk + row < N ? n_blk + row : N - 1;
        zv[i] = pol.zword(gn, q, K);
        zw[i] = e0 < ZGN ? XB + WB + row * 16 + 4 * posz(row, q) : -1;
      }
    }
    uint4 xr[D][XG], wr[D][WG];
    uint32_t zr[D][ZG > 0 ? ZG : 1];
    auto load = [&](int j, uint4 (&xd)[XG], uint4 (&wd)[WG], uint32_t (&zd)[ZG > 0 ? ZG : 1])
        __attribute__((always_inline)) {
      const int st = s0 + (j < J ? j : J - 1);
#pragma unroll
      for (int i = 0; i < XG; ++i) xd[i] = bload16(xrs, xv[i], (uint32_t)st * P::kXRow);
#pragma unroll
      for (int i = 0; i < WG; ++i) wd[i] = bload16<kNT>(wrs, wv[i], pol.wsoff(st));
      if constexpr (ZG > 0) {
#pragma unroll
        for (int i = 0; i < ZG; ++i) zd[i] = bload4<kNT>(zrs, zv[i], pol.zsoff(st));
      }
    };
    auto store = [&](const uint4 (&xd)[XG], const uint4 (&wd)[WG],
                     const uint32_t (&zd)[ZG > 0 ? ZG : 1], int buf) __attribute__((always_inline)) {
      uint8_t* base = reinterpret_cast<uint8_t*>(lds) + buf * STAGE;
#pragma unroll
      for (int i = 0; i < XG; ++i) *reinterpret_cast<uint4*>(base + xw[i]) = xd[i];
#pragma unroll
      for (int i = 0; i < WG; ++i)
        if (WGN % 512 == 0 || ww[i] >= 0) *reinterpret_cast<uint4*>(base + ww[i]) = wd[i];
      if constexpr (ZG > 0) {
#pragma unroll
        for (int i = 0; i < ZG; ++i)
          if (ZGN % 512 == 0 || zw[i] >= 0) *reinterpret_cast<uint32_t*>(base + zw[i]) = zd[i];
      }
    };
    sfor<0, D>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      load(p, xr[p], wr[p], zr[p]);
    });
    SF_MARK(1);
    store(xr[0], wr[0], zr[0], 0);
    __syncthreads();
#if TAO_SF_STAMPS
    SF_MARK(2);
#endif
    auto body = [&](auto uc, int j) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value;
      load(j + D, xr[u], wr[u], zr[u]);  // ring slot u held step j, already in LDS
      compute(j & 1);
      if (j + 1 < J) store(xr[(u + 1) % D], wr[(u + 1) % D], zr[(u + 1) % D], (j + 1) & 1);
      __syncthreads();
    };
    int j = 0;
    for (; j + D <= J; j += D)
      sfor<0, D>([&](auto uc) { body(uc, j + decltype(uc)::value); });
    sfor<0, D - 1>([&](auto uc) {
      if (j + decltype(uc)::value < J) body(uc, j + decltype(uc)::value);
    });
  }
  barrier_lgkm();  // all fragment reads done: the LDS is free for the epilogue image
  SF_MARK(3);

  // ---- split-K seam -----------------------------------------------------------------------------
  if (S > 1) {
    constexpr uint32_t kSlice = kBM * BN * 4;  // bytes of one slice's partial tile
    const unsigned tile = blockIdx.z * gridDim.x + blockIdx.x;
    const Rsrc srs = make_rsrc(reinterpret_cast<const uint8_t*>(slab) + (size_t)tile * (S - 1) * kSlice,
                               (uint32_t)(S - 1) * kSlice);
    const uint32_t lo = (uint32_t)((wave * MT * NT * 64 + lane) * 16);
    unsigned* word = reinterpret_cast<unsigned*>(lds);
    if (!reducer) {
      // MI355X_MICROARCH.md "Hand-offs measured with sc1 loads in place of the acquire", first row:
      // sc1 16-B stores, every storing wave's vmcnt(0), a workgroup barrier, one agent-scope add
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
          bstore16<kSC1>(srs, lo + (a * NT + b) * 1024, (uint32_t)z * kSlice,
                         __builtin_bit_cast(uint4, acc[a][b]));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (fenced) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        (void)__hip_atomic_fetch_add(&cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#if TAO_SF_STAMPS
      SF_MARK(4);
      SF_MARK(5);
      if (tid < 64) {
        const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        unsigned long long v = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const unsigned l32 = __shfl((unsigned)stamp[i], 0), h32 = __shfl((unsigned)(stamp[i] >> 32), 0);
          if (lane == i) v = ((unsigned long long)h32 << 32) | l32;
        }
        if (lane == 6) v = (unsigned long long)z;
        if (lane == 7) v = 0;
        if (lane < 8 && b < 8192) g_sf_stamps[b * 8 + lane] = v;
      }
#endif
      return;
    }
    // reducer: one lane polls the ticket (sc1 loads), resets it for the next launch, tells the
    // workgroup through LDS; every wave then reads the slabs with sc1 loads
    if (tid == 0) {
      unsigned it = 0, ok = 1;
      while (__hip_atomic_load(&cnt[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
             (unsigned)(S - 1)) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1u << 22)) {  // ~0.3 s: give up, report (outputs of this tile are invalid)
          ok = 0;
          (void)__hip_atomic_fetch_or(&g_sf_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (ok) __hip_atomic_store(&cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fenced) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *word = ok;
    }
    __syncthreads();
    // slices summed in slice order (publishers 0 .. S-2, then this one): deterministic
    Acc sum[MT][NT];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) sum[a][b] = Acc{0, 0, 0, 0};
    // up to 4 slabs' loads in flight before their adds (clamped, then masked): one round trip per
    // 4 publishers instead of one per publisher
    constexpr int kG = MT * NT <= 4 ? 4 : (MT * NT <= 8 ? 2 : 1);
    for (int z0 = 0; z0 < S - 1; z0 += kG) {
      Acc part[kG][MT][NT];
#pragma unroll
      for (int gi = 0; gi < kG; ++gi) {
        const int zz = z0 + gi < S - 1 ? z0 + gi : S - 2;
#pragma unroll
        for (int a = 0; a < MT; ++a)
#pragma unroll
          for (int b = 0; b < NT; ++b)
            part[gi][a][b] = __builtin_bit_cast(
                Acc, bload16<kSC1>(srs, lo + (a * NT + b) * 1024, (uint32_t)zz * kSlice));
      }
#pragma unroll
      for (int gi = 0; gi < kG; ++gi)
        if (z0 + gi < S - 1) {
#pragma unroll
          for (int a = 0; a < MT; ++a)
#pragma unroll
            for (int b = 0; b < NT; ++b) sum[a][b] += part[gi][a][b];
        }
    }
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = sum[a][b] + acc[a][b];
    SF_MARK(4);
  }

  // ---- epilogue: bf16 tile through an LDS image, rows stored in 16-B pieces ------------------------
  uint16_t* out = reinterpret_cast<uint16_t*>(lds);  // [128][BN]
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int c = wn * CN + 16 * nt + fr;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * RM + 16 * mt + 4 * kq + i;
        float v;
        if constexpr (kI8) {
          v = round_bf16(round_bf16((float)acc[mt][nt][i]) * xsf[mt * 4 + i]);
          v = round_bf16(v * wsf[nt]);
        } else {
          v = round_bf16(acc[mt][nt][i]);
        }
        if (bias != nullptr) v = round_bf16(v + bsf[nt]);
        out[r * BN + c] = f32_to_bf16(v);
      }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B pieces per row
  const bool full = n_blk + BN <= N && (N & 7) == 0 && ((uintptr_t)y & 15) == 0;
#pragma unroll
  for (int c = tid; c < kBM * CPR; c += 512) {
    const int r = c / CPR, cc = c % CPR;
    const int m = m_blk + r;
    if (m >= M) continue;
    const uint4 v = reinterpret_cast<const uint4*>(out)[c];
    if (full) {
      *reinterpret_cast<uint4*>(y + (size_t)m * N + n_blk + 8 * cc) = v;
    } else {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
      for (int k = 0; k < 8; ++k)
        if (n_blk + 8 * cc + k < N) y[(size_t)m * N + n_blk + 8 * cc + k] = e[k];
    }
  }
#if TAO_SF_STAMPS
  SF_MARK(5);
  if (tid < 64) {
    const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    unsigned long long v = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const unsigned l32 = __shfl((unsigned)stamp[i], 0), h32 = __shfl((unsigned)(stamp[i] >> 32), 0);
      if (lane == i) v = ((unsigned long long)h32 << 32) | l32;
    }
    if (lane == 6) v = (unsigned long long)z;
    if (lane == 7) v = 1;
    if (lane < 8 && b < 8192) g_sf_stamps[b * 8 + lane] = v;
  }
#endif
#undef SF_MARK
}

// ---- launch ------------------------------------------------------------------------------------
struct SfShape {
  int bn, wm, splits, stages, a_steps;
};

template <class P, int BN, int WM, int NS, bool REG>
bool sf_go(dim3 grid, hipStream_t stream, const uint8_t* x, const P& pol, const uint16_t* bias,
           uint16_t* y, int M, int N, int K, int a, typename P::Acc* slab, unsigned* cnt) {
  constexpr int STAGE = kBM * P::kXRow + BN * P::kWRow + BN * P::kZRow;
  constexpr int NB = REG ? 2 : NS;
  if constexpr (NB * STAGE <= 160 * 1024 && (kBM * P::kXRow + BN * P::kWRow + BN * P::kZRow) > 0) {
    constexpr int T = (kBM * P::kXRow) / 1024 + (BN * P::kWRow) / 1024 + (BN * P::kZRow) / 256;
    if constexpr (T % kWaves == 0 && (BN * P::kWRow) % 1024 == 0 && (BN * P::kZRow) % 256 == 0 &&
                  BN / (kWaves / WM) >= 16)
    {
      launch(gemm_sf_kernel<P, BN, WM, NS, REG>, grid, dim3(512), 0, stream, x, pol, bias, y, M,
             N, K, a, slab, cnt, tuning().splitk_fenced);
      return true;
    }
  }
  return false;  // combination not instantiated (LDS, DMA split or wave tile)
}

template <class P, int BN>
int sf_dispatch_wm(const SfShape& sh, dim3 grid, hipStream_t st, const uint8_t* x, const P& pol,
                   const uint16_t* bias, uint16_t* y, int M, int N, int K, int a,
                   typename P::Acc* slab, unsigned* cnt) {
  bool ok = false;
  const bool reg = tuning().sf_reg != 0;
  auto go = [&](auto wmc, auto nsc) {
    constexpr int W = decltype(wmc)::value, S_ = decltype(nsc)::value;
    ok = reg ? sf_go<P, BN, W, S_, true>(grid, st, x, pol, bias, y, M, N, K, a, slab, cnt)
             : sf_go<P, BN, W, S_, false>(grid, st, x, pol, bias, y, M, N, K, a, slab, cnt);
  };
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  auto by_ns = [&](auto wmc) {
    if (sh.stages == 2) go(wmc, I2{});
    else if (sh.stages == 4) go(wmc, I4{});
    else go(wmc, I3{});
  };
  if (sh.wm == 2) by_ns(I2{});
  else if (sh.wm == 8) by_ns(I8{});
  else by_ns(I4{});
  if (!ok)
    return set_error(TAO_ERR_INVALID_ARGUMENT,
                     "gemm_sf: no kernel for bn %d, wm %d, stages %d with this operand format",
                     BN, sh.wm, sh.stages);
  return check_launch("gemm_sf_kernel");
}

}  // namespace

// Shape for 64 < M <= 128 (per 128-row M tile): the smallest split S (1, 2, 4, 8) whose grid
// (N / BN tiles x S) reaches 256 workgroups, publishers taking an equal share of the steps.
// tao_tune_gemm_sf overrides every field.
static SfShape sf_shape(int path, int M, int N, int K) {
  (void)M;
  const int kstep = path == 0 ? 128 : 256;
  const int nsteps = K / kstep;
  SfShape sh{path == 0 ? 64 : 32, path == 0 ? 2 : 4, 1, 3, 0};
  const Tuning& t = tuning();
  if (t.sf_bn) sh.bn = t.sf_bn;
  if (t.sf_wm) sh.wm = t.sf_wm;
  if (t.sf_stages) sh.stages = t.sf_stages;
  const long tiles = (N + sh.bn - 1) / sh.bn;
  while (tiles * sh.splits < 256 && sh.splits < 8 && nsteps >= 2 * sh.splits * 2) sh.splits *= 2;
  if (t.sf_splits) sh.splits = t.sf_splits;
  if (sh.splits > nsteps) sh.splits = nsteps;
  sh.a_steps = nsteps / sh.splits;
  if (t.sf_a_steps) sh.a_steps = t.sf_a_steps;
  if (sh.splits > 1 && sh.a_steps * (sh.splits - 1) >= nsteps) sh.a_steps = nsteps / sh.splits;
  return sh;
}

bool use_sf(int path, int64_t M, int64_t N, int64_t K, int64_t group_size) {
  const int mode = tuning().gemm_sf;
  if (mode == 1) return false;
  if (path != 0 && path != 2) return false;
  const int kstep = path == 0 ? 128 : 256;
  if (M < 1 || K % kstep != 0 || K < kstep || N < 16 || (uint64_t)M * K >= (1ull << 32) ||
      (uint64_t)N * K >= (1ull << 32))
    return false;
  if (path == 0 && (group_size < 32 || group_size > 256 || K % group_size != 0)) return false;
  if (mode == 2) return M <= 128;
  return false;  // auto: not yet routed
}

int sf_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
               const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  const SfShape sh = sf_shape(2, M, N, K);
  const int ks = tuning().sf_ks == 128 ? 128 : 256;
  const dim3 grid((N + sh.bn - 1) / sh.bn, sh.splits, (M + kBM - 1) / kBM);
  i32x4_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (sh.splits > 1) {
    void* w = nullptr;
    const size_t tiles = (size_t)grid.x * grid.z;
    const int rc = split_workspace(stream, tiles * (sh.splits - 1) * kBM * sh.bn * 4, tiles, &w, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<i32x4_t*>(w);
  }
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(xq);
  // a_steps is in units of the policy's k step (256 k; 128-k steps take twice as many)
  auto run = [&](auto pol, int a) -> int {
    typedef decltype(pol) P;
    switch (sh.bn) {
      case 32: return sf_dispatch_wm<P, 32>(sh, grid, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
      case 128: return sf_dispatch_wm<P, 128>(sh, grid, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
      default: return sf_dispatch_wm<P, 64>(sh, grid, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
    }
  };
  if (ks == 128) {
    SfI8<128> pol{wq, ws, xs};
    return run(pol, sh.a_steps * 2);
  }
  SfI8<256> pol{wq, ws, xs};
  return run(pol, sh.a_steps);
}

int sf32_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int lg,
              const uint16_t* bias, uint16_t* y, int M, int N, int K, int bn, int splits,
              int stages, int a_steps, hipStream_t stream);

int sf_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int lg,
            const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  const SfShape sh = sf_shape(0, M, N, K);
  if (sh.wm == 1)  // one wave along M: the 32x32x16 kernel (gemm_sf32.hip)
    return sf32_int4(x, packed, sz, lg, bias, y, M, N, K, sh.bn, sh.splits, sh.stages,
                     tuning().sf_a_steps, stream);
  const dim3 grid((N + sh.bn - 1) / sh.bn, sh.splits, (M + kBM - 1) / kBM);
  f32x4_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (sh.splits > 1) {
    void* w = nullptr;
    const size_t tiles = (size_t)grid.x * grid.z;
    const int rc = split_workspace(stream, tiles * (sh.splits - 1) * kBM * sh.bn * 4, tiles, &w, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<f32x4_t*>(w);
  }
  if (sh.bn != 64 && sh.bn != 128)
    return set_error(TAO_ERR_INVALID_ARGUMENT, "gemm_sf: int4 takes bn 64 or 128 (got %d)", sh.bn);
  SfI4 pol{packed, reinterpret_cast<const uint32_t*>(sz), lg};
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(x);
  switch (sh.bn) {
    case 128:
      return sf_dispatch_wm<SfI4, 128>(sh, grid, stream, xb, pol, bias, y, M, N, K, sh.a_steps, slab, cnt);
    default:  // 64
      return sf_dispatch_wm<SfI4, 64>(sh, grid, stream, xb, pol, bias, y, M, N, K, sh.a_steps, slab, cnt);
  }
}

}  // namespace tao

// Single-fetch prefill GEMM routing and launch shape (calling thread only; for A/B measurement):
// mode 0 = built-in routing, 1 = never, 2 = whenever the shape is supported (M <= 128 per launch
// tile); bn / wm / splits / stages / a_steps 0 = built-in; ks = int8 k step 128 or 256 (0 = 256).
extern "C" int tao_tune_gemm_sf(int mode, int bn, int wm, int splits, int stages, int a_steps,
                                int ks) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 2, "tune: gemm_sf mode must be 0, 1 or 2");
  TAO_CHECK_ARG(bn == 0 || bn == 32 || bn == 64 || bn == 128, "tune: gemm_sf bn must be 0, 32, 64, 128");
  TAO_CHECK_ARG(wm == 0 || wm == 1 || wm == 2 || wm == 4 || wm == 8,
                "tune: gemm_sf wm must be 0, 1 (int4: the 32x32x16 kernel), 2, 4 or 8");
  TAO_CHECK_ARG(splits >= 0 && splits <= 16, "tune: gemm_sf splits must be in [0, 16]");
  TAO_CHECK_ARG(stages == 0 || (stages >= 2 && stages <= 4), "tune: gemm_sf stages must be 0, 2, 3, 4");
  TAO_CHECK_ARG(a_steps >= 0, "tune: gemm_sf a_steps must be >= 0");
  TAO_CHECK_ARG(ks == 0 || ks == 128 || ks == 256, "tune: gemm_sf ks must be 0, 128 or 256");
  tao::Tuning& t = tao::tuning();
  t.gemm_sf = mode;
  t.sf_bn = bn;
  t.sf_wm = wm;
  t.sf_splits = splits;
  t.sf_stages = stages;
  t.sf_a_steps = a_steps;
  t.sf_ks = ks;
  return TAO_OK;
}

// Register staging instead of LDS-DMA for the single-fetch GEMM (1), or the DMA ring (0, built-in).
extern "C" int tao_tune_gemm_sf_reg(int reg) {
  TAO_CHECK_ARG(reg == 0 || reg == 1, "tune: gemm_sf_reg must be 0 or 1");
  tao::tuning().sf_reg = reg;
  return TAO_OK;
}

// Reducer poll timeouts since the last call (0 = none; a nonzero value means some outputs of a
// split launch were invalid). Synchronous; not capturable.
namespace tao {
int sf32_status(unsigned* bits);
}

extern "C" int tao_gemm_sf_status(unsigned* bits) {
  unsigned v = 0, zero = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(tao::g_sf_err), sizeof(v)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(tao::g_sf_err), &zero, sizeof(zero)) != hipSuccess)
    return tao::set_error(TAO_ERR_HIP, "gemm_sf status: symbol copy failed");
  *bits = v;
  return tao::sf32_status(bits);
}

#if TAO_SF_STAMPS
extern "C" int tao_debug_sf_stamps(unsigned long long* out, int n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tao::g_sf_stamps), (size_t)n * 8 * 8) != hipSuccess)
    return TAO_ERR_HIP;
  static unsigned long long zero[8192 * 8];
  return hipMemcpyToSymbol(HIP_SYMBOL(tao::g_sf_stamps), zero, sizeof(zero)) == hipSuccess
             ? TAO_OK : TAO_ERR_HIP;
}
#endif
