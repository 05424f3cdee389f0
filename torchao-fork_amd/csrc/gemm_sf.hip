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
//   * K split S ways over workgroups (the grid fills the 256 CUs). Spread seam (built-in): each
//     of a tile's S workgroups publishes the fp32 / int32 partials of the waves it does not own
//     (sc1 stores, one ticket add), waits for all S, and its owned 8/S waves sum their fragments
//     over the slices in slice order (run-to-run deterministic; int32 exact) and run the
//     epilogue of their wave tiles. Fixed-reducer seam (tao_tune_gemm_sf_seam 0): slices
//     0..S-2 publish whole tiles, slice S-1 (dispatched last) sums them; publishers may take
//     fewer K steps than the reducer (`a_steps`).
// Wave layout: WM x WN waves over the 128 x BN tile (wave tile 128/WM x BN/WN).
#include <type_traits>

#include "tao_common.h"

// 1: with 3+ stages, each step's DMA pieces are issued between its MFMA groups (after group kb,
// pieces r with r KB / R == kb) instead of all after the step's barrier (gemm_sf32.hip's IL)
#ifndef TAO_SF_IL
#define TAO_SF_IL 0
#endif

namespace tao {

TAO_DECODE_ERROR_WORD(sf_decode_status)

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;   // rows per tile
constexpr int kWaves = 8;  // 512 threads

// reducer poll timeouts (never expected: publishers never wait, and they precede the reducers in
// every XCD's dispatch order); read and cleared by tao_gemm_sf_status()
__device__ unsigned g_sf_err = 0;

// Epilogue folded into the GEMM (kind): 0 = y [M][N] bf16 (+ bias); 1 = SwiGLU of interleaved
// (gate, up) column pairs, y [M][N / 2]; 2 = RoPE + KV-cache write of a wqkv output (the prefill
// rope_kv kernel's math, decode_ops.hip): rows are tokens (b, s) = (m / S, m % S) at position
// pos[s]; columns [q heads | k heads | v heads] of D = 128; q rotated into q_out [B][H][S][D],
// k rotated and v written into the caches [B][Hkv][T][D] at row pos[s]; 3 = int4 only: no seam
// and no bf16 output, every K slice z writes its fp32 partial tile row-major into
// part[z][M][N] (the consumer sums the slices in slice order: tao_add_rmsnorm_partials_bf16).
struct SfEpi {
  int kind;
  float* part;         // kind 3: [S][M][N] fp32
  const float* freqs;  // [T][D / 2] (cos, sin)
  const int64_t* pos;  // [S]
  uint16_t* q_out;
  uint16_t* kc;
  uint16_t* vc;
  int S, H, Hkv, T;
};

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
  // scalar fmas (the Makefile keeps the SLP vectorizer from pairing them into v_pk_fma_f32)
  const float w0 = __builtin_fmaf(q04[0], sc, zc), w4 = __builtin_fmaf(q04[1], sc, zc);
  const float w1 = __builtin_fmaf(q15[0], sc, zc), w5 = __builtin_fmaf(q15[1], sc, zc);
  const float w2 = __builtin_fmaf(q26[0], sc, zc), w6 = __builtin_fmaf(q26[1], sc, zc);
  const float w3 = __builtin_fmaf(q37[0], sc, zc), w7 = __builtin_fmaf(q37[1], sc, zc);
  const u32x4_t v = {pk_bf16(w0, w1), pk_bf16(w2, w3), pk_bf16(w4, w5), pk_bf16(w6, w7)};
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

// Grid: one dimension, ntn N tiles x S slices x M tiles. seam 0 (fixed reducer): N tile fastest,
// so every tile's reducer (slice S-1) is dispatched after all publishers. seam 1 (spread): slice
// fastest, so a tile's S workgroups are dispatched together (they wait for one another: the
// launcher takes this seam only when S divides the 8 waves and the grid's resident set holds S).
// MFMA groups per step: the int8 k blocks, or the 4 nibble dwords of an int4 step
template <class P>
constexpr int mfma_groups() {
  if constexpr (P::kABytes == 1) return P::kKB;
  else return 4;
}

// LDW > 0: LDW dedicated loader waves (one per SIMD) issue every LDS-DMA piece and the 8 compute
// waves only read fragments, dequantise and issue MFMAs (gemm_sf32.hip measured the same split
// 17% faster on its 128-column tile).
template <class P, int BN, int WM, int NS, int LDW = 0>
__global__ __launch_bounds__((kWaves + LDW) * 64) void gemm_sf_kernel(
    const uint8_t* __restrict__ x, P pol, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int a_steps, typename P::Acc* __restrict__ slab,
    unsigned* __restrict__ cnt, int fenced, int S, int ntn, int seam, int cs, SfEpi ep, int xmap) {
  const int epi = ep.kind;
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
  constexpr int DW = LDW > 0 ? LDW : kWaves;  // waves that issue the DMA pieces
  constexpr int NTH = (kWaves + LDW) * 64;      // threads
  static_assert(T % DW == 0 && PX % DW == 0, "DMA pieces per wave");
  constexpr int R = T / DW;  // DMA instructions per DMA wave per stage
  constexpr bool IL = TAO_SF_IL != 0 && NS >= 3 && LDW == 0;
  constexpr int NB = NS;  // LDS stage buffers
  static_assert(NB * STAGE <= 160 * 1024, "LDS");
  static_assert(kBM * BN * 2 <= NB * STAGE, "epilogue image");
  __shared__ uint4 lds[NB * STAGE / 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = LDW > 0 && wave >= kWaves;
  const int dwv = LDW > 0 ? wave - kWaves : wave;  // index among the DMA-issuing waves
  const int wm = loader ? 0 : wave / WN, wn = loader ? 0 : wave % WN;
  const int fr = lane & 15, kq = lane >> 4;
  const int bid = blockIdx.x;
  int z, nb, mb;
  if (seam) {
    z = bid % S;
    nb = (bid / S) % ntn;
    mb = bid / (S * ntn);
  } else if (xmap) {  // slice z on XCDs [z G, (z + 1) G), G = 8 / S (dispatch: block b on XCD b % 8)
    const int G = 8 / S, b = bid % (S * ntn), xcd = b & 7;  // (runtime divisions: VALU, so
    z = __builtin_amdgcn_readfirstlane(xcd / G);            // pinned back to SGPRs)
    nb = __builtin_amdgcn_readfirstlane((b >> 3) * G + xcd % G);
    mb = __builtin_amdgcn_readfirstlane(bid / (S * ntn));
  } else {
    nb = bid % ntn;
    z = (bid / ntn) % S;
    mb = bid / (S * ntn);
  }
  const int n_blk = nb * BN, m_blk = mb * kBM;
  const unsigned tile = (unsigned)(mb * ntn + nb);
  const bool last = z == S - 1;
  const bool reducer = last && !seam;  // fixed-reducer seam: the one workgroup that sums
  const int nsteps = K / P::kKStep;
  const int s0 = z * a_steps;
  const int J = last ? nsteps - s0 : a_steps;  // launcher: every slice >= 1 step
  const uint32_t row_bytes = (uint32_t)K * P::kABytes;

  // ---- DMA slots: this wave's R pieces per stage (piece i = 8 r + wave) --------------------------
  const Rsrc xrs = make_rsrc(x, (uint32_t)M * row_bytes);
  const Rsrc wrs = pol.wrsrc(N, K);
  const Rsrc zrs = pol.zrsrc(N, K);
  uint32_t dv[R];
  int dd[R], dk[R];
  sfor<0, R>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (r < PX / DW) {
      constexpr int G = P::kXRow / 16;
      const int i = r * DW + dwv;
      const int row = i * (1024 / P::kXRow) + lane / G, p = lane % G;
      const int gm = m_blk + row < M ? m_blk + row : M - 1;
      dv[r] = (uint32_t)gm * row_bytes + 16u * (uint32_t)P::xpos(row, p);
      dd[r] = i * 1024;
      dk[r] = 0;
    } else {
      const int i = (r - PX / DW) * DW + dwv;
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
  constexpr bool kI8 = P::kABytes == 1;
  auto issue_piece = [&](auto rc, int st, int buf) __attribute__((always_inline)) {
    constexpr int r = decltype(rc)::value;
    uint8_t* base = reinterpret_cast<uint8_t*>(lds) + buf * STAGE;
    if constexpr (r < PX / DW) {
      dma_lds_ring<16>(xrs, dv[r], (uint32_t)st * P::kXRow, base + dd[r]);
    } else {
      if (dk[r] == 1) dma_lds_ring<16, kNT>(wrs, dv[r], pol.wsoff(st), base + dd[r]);
      else if constexpr (PZ > 0) dma_lds_ring<4, kNT>(zrs, dv[r], pol.zsoff(st), base + dd[r]);
    }
  };
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    sfor<0, R>([&](auto rc) { issue_piece(rc, st, buf); });
  };
  // pieces r with r KB / R == kb, issued after MFMA group kb (IL)
  auto issue_group = [&](auto kbc, int st, int buf) __attribute__((always_inline)) {
    constexpr int kb = decltype(kbc)::value;
    constexpr int KBN = mfma_groups<P>();
    __builtin_amdgcn_sched_barrier(0);
    sfor<0, R>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if constexpr (r * KBN / R == kb) issue_piece(rc, st, buf);
    });
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- epilogue operands, loaded ahead of the stream ---------------------------------------------
  // rows of this lane: wm RM + 16 mt + 4 kq + i; columns: wn CN + 16 nt + fr
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
  auto compute = [&](int buf, auto iss, int st, int ibuf) __attribute__((always_inline)) {
    constexpr bool ISS = decltype(iss)::value;
    if constexpr (ISS && !IL) issue(st, ibuf);
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
      sfor<0, P::kKB>([&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(af[kb][mt], bf[kb][nt], acc[mt][nt], 0, 0, 0);
        if constexpr (ISS && IL) issue_group(kbc, st, ibuf);
      });
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
      sfor<0, 4>([&](auto kbc) {
        constexpr int kb = decltype(kbc)::value;
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
        if constexpr (ISS && IL) issue_group(kbc, st, ibuf);
      });
    }
  };

  // ---- the k loop: LDS-DMA, NS-1 stages in flight, one barrier per step ----------------------------
  // (a register-staged variant -- 16-B loads into a register ring, two LDS buffers -- measured
  // 5-15% slower at every swept shape: profiles/r4_sf_sweep_reg.jsonl)
  if constexpr (LDW > 0) {  // loaders wait for their pieces, join the barrier, refill; compute
    if (loader) {            // waves only read and compute
#pragma unroll
      for (int p = 0; p < NS - 1; ++p)
        if (p < J) issue(s0 + p, p);
      for (int j = 0; j < J; ++j) {
        wait_ahead<R>(J - 1 - j < NS - 2 ? J - 1 - j : NS - 2);
        barrier_lgkm();
        if (j + NS - 1 < J) issue(s0 + j + NS - 1, (j + NS - 1) % NS);
      }
    } else {
      for (int j = 0; j < J; ++j) {
        barrier_lgkm();
        compute(j % NS, std::false_type{}, 0, 0);
      }
    }
  } else {
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < J) issue(s0 + p, p);
  const int jiss = J - (NS - 1);  // steps that issue a stage ahead
  int j = 0;
  for (; j < jiss; ++j) {
    wait_ahead<R>(NS - 2);  // this wave's DMAs of step j landed
    barrier_lgkm();         // ... and every wave's; step j - 1's fragment reads are done
    compute(j % NS, std::true_type{}, s0 + j + NS - 1, (j + NS - 1) % NS);
  }
  for (; j < J; ++j) {
    const int ahead = J - 1 - j < NS - 2 ? J - 1 - j : NS - 2;
    wait_ahead<R>(ahead);
    barrier_lgkm();
    compute(j % NS, std::false_type{}, 0, 0);
  }
  }  // LDW == 0
  barrier_lgkm();  // all fragment reads done: the LDS is free for the epilogue image
  if constexpr (!kI8) {
    if (epi == 3) {  // partials out: this slice's fp32 tile, row-major, no hand-off
      if (!loader) {
        float* dst = ep.part + (size_t)z * M * N;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int c = n_blk + wn * CN + 16 * nt + fr;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = m_blk + wm * RM + 16 * mt + 4 * kq + i;
              if (r < M && c < N) dst[(size_t)r * N + c] = acc[mt][nt][i];
            }
        }
      }
      return;
    }
  }

  // ---- split-K seam -----------------------------------------------------------------------------
  // Slab: S slices' partial tiles per tile, each in the waves' fragment order (granule
  // (wave MT NT + a NT + b) 64 + lane). Spread seam: workgroup z owns waves [z W/S, (z+1) W/S)
  // of the tile (W = 8 waves): it publishes the fragments of the other waves, and its owned
  // waves sum their fragments over the S slices and run the epilogue for their wave tiles, so
  // each workgroup takes in (S-1)/S^2 of the slices' partials instead of one reducer taking in
  // (S-1) whole tiles (the fixed reducer's seam measured 4-11 us at S = 4-8: its intake).
  const int wpo = kWaves / S;  // waves owned per workgroup (spread)
  const bool own = !loader && (S == 1 || !seam || wave / wpo == z);
  if (S > 1) {
    constexpr uint32_t kSlice = kBM * BN * 4;  // bytes of one slice's partial tile
    const Rsrc srs = make_rsrc(reinterpret_cast<const uint8_t*>(slab) + (size_t)tile * S * kSlice,
                               (uint32_t)S * kSlice);
    const uint32_t lo = (uint32_t)((wave * MT * NT * 64 + lane) * 16);
    unsigned* word = reinterpret_cast<unsigned*>(lds);
    if (!reducer && !(seam && own) && !loader) {
      // MI355X_MICROARCH.md "Hand-offs measured with sc1 loads in place of the acquire", first row:
      // sc1 16-B stores, every storing wave's vmcnt(0), a workgroup barrier, one agent-scope add
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
          bstore16<kSC1>(srs, lo + (a * NT + b) * 1024, (uint32_t)z * kSlice,
                         __builtin_bit_cast(uint4, acc[a][b]));
    }
    if (!reducer) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (fenced & 1) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if ((fenced & 2) && z == 0 && !seam) late_publisher_hold(&g_sf_err);
        (void)__hip_atomic_fetch_add(&cnt[tile * cs], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (!seam && !reducer) {
      return;
    }
    // fixed reducer: wait for the S-1 publishers, then take their S-1 arrivals back off the
    // ticket. Spread: every workgroup waits for all S arrivals, then adds a second arrival; the
    // one that completes 2 S resets the ticket (every workgroup has left its wait by then). One
    // lane polls with sc1 loads and tells the workgroup through LDS. A timed-out wait still
    // settles the ticket the same way (the subtraction, or the second arrival), so once the late
    // publishers' adds land it is back at 0 for the next launch on this stream's workspace; the
    // tile itself is skipped and the timeout reported (tao_decode_status bits & 2).
    if (tid == 0) {
      const unsigned need = seam ? (unsigned)S : (unsigned)(S - 1);
      unsigned ok = 1;
      SeamWait sw;
      while (__hip_atomic_load(&cnt[tile * cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        __builtin_amdgcn_s_sleep(1);
        if (sw.timed_out()) {  // give up, report (outputs of this tile are invalid)
          ok = 0;
          (void)__hip_atomic_fetch_or(&g_sf_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (!seam) {
        (void)__hip_atomic_fetch_sub(&cnt[tile * cs], need, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      } else if (__hip_atomic_fetch_add(&cnt[tile * cs], 1u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) == 2u * S - 1u) {
        __hip_atomic_store(&cnt[tile * cs], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (fenced & 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *word = ok;
    }
    __syncthreads();
    if (*word == 0) return;  // timed out: write nothing (uniform over the workgroup)
    if (own) {
      // the other slices' fragments summed with this one's in slice order: deterministic, and
      // the same additions in the same order under both seams
      const int zo = seam ? z : S - 1;  // this workgroup's slice
      Acc sum[MT][NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) sum[a][b] = Acc{0, 0, 0, 0};
      // up to 4 slabs' loads in flight before their adds (clamped, then masked)
      constexpr int kG = MT * NT <= 4 ? 4 : (MT * NT <= 8 ? 2 : 1);
      for (int z0 = 0; z0 < S; z0 += kG) {
        Acc part[kG][MT][NT];
#pragma unroll
        for (int gi = 0; gi < kG; ++gi) {
          const int zz = z0 + gi < S ? z0 + gi : S - 1;
#pragma unroll
          for (int a = 0; a < MT; ++a)
#pragma unroll
            for (int b = 0; b < NT; ++b)
              part[gi][a][b] = zz == zo ? acc[a][b] : __builtin_bit_cast(
                  Acc, bload16<kSC1>(srs, lo + (a * NT + b) * 1024, (uint32_t)zz * kSlice));
        }
#pragma unroll
        for (int gi = 0; gi < kG; ++gi)
          if (z0 + gi < S) {
#pragma unroll
            for (int a = 0; a < MT; ++a)
#pragma unroll
              for (int b = 0; b < NT; ++b) sum[a][b] += part[gi][a][b];
          }
      }
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = sum[a][b];
    }
  }

  // ---- epilogue: bf16 tile through an LDS image, rows stored in 16-B pieces ------------------------
  uint16_t* out = reinterpret_cast<uint16_t*>(lds);  // [128][BN]
  if (own) {
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
  }
  __syncthreads();
  if (epi == 1) {  // SwiGLU over interleaved (gate, up) columns: y [M][N / 2]
    constexpr int OPR = BN / 16;  // 16-B output pieces per row
    const int N2 = N >> 1;
    const bool full2 = n_blk + BN <= N && (N2 & 7) == 0 && ((uintptr_t)y & 15) == 0;
    for (int c = tid; c < kBM * OPR; c += NTH) {
      const int r = c / OPR, cc = c % OPR;
      const int m = m_blk + r;
      if (m >= M) continue;
      if (seam && S > 1 && ((r / RM) * WN + (16 * cc) / CN) / wpo != z) continue;  // not owned
      const uint4* img = reinterpret_cast<const uint4*>(out) + r * (BN / 8) + 2 * cc;
      const uint4 v = swiglu_piece(img[0], img[1]);
      const int n0 = (n_blk >> 1) + 8 * cc;
      if (full2) {
        *reinterpret_cast<uint4*>(y + (size_t)m * N2 + n0) = v;
      } else {
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
        for (int k = 0; k < 8; ++k)
          if (n0 + k < N2) y[(size_t)m * N2 + n0 + k] = e[k];
      }
    }
  }
  if (epi == 2) {  // RoPE + KV-cache write (N = (H + 2 Hkv) 128, 16-B aligned destinations)
    constexpr int CPR = BN / 8;
    const float2* f2 = reinterpret_cast<const float2*>(ep.freqs);
    for (int c = tid; c < kBM * CPR; c += NTH) {
      const int r = c / CPR, cc = c % CPR;
      const int m = m_blk + r, n0 = n_blk + 8 * cc;
      if (m >= M || n0 >= N) continue;
      if (seam && S > 1 && ((r / RM) * WN + (8 * cc) / CN) / wpo != z) continue;  // not owned
      uint4 v = reinterpret_cast<const uint4*>(out)[c];
      const int b = m / ep.S, s = m % ep.S;
      int64_t p = ep.pos[s];
      const bool pok = p >= 0 && p < ep.T;  // KV cache row inside [0, T)
      if (!pok) {  // report (tao_decode_status) and write no cache row
        flag_decode_error(kDecodeErrKvPos);
        p = p < 0 ? 0 : ep.T - 1;
      }
      const int head = n0 >> 7, d0 = n0 & 127;
      if (head < ep.H + ep.Hkv) {  // rotate the 4 interleaved pairs (fp32, bf16 out)
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float2 cs = f2[(size_t)p * 64 + (d0 >> 1) + i];
          const float x0 = bf16lo_to_f32(w[i]), x1 = bf16hi_to_f32(w[i]);
          const float o0 = x0 * cs.x - x1 * cs.y, o1 = x1 * cs.x + x0 * cs.y;
          w[i] = (uint32_t)f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      uint16_t* dst = nullptr;
      if (head < ep.H) {
        dst = ep.q_out + (((size_t)b * ep.H + head) * ep.S + s) * 128 + d0;
      } else if (pok) {
        const bool isk = head < ep.H + ep.Hkv;
        const int kh = isk ? head - ep.H : head - ep.H - ep.Hkv;
        dst = (isk ? ep.kc : ep.vc) + (((size_t)b * ep.Hkv + kh) * ep.T + p) * 128 + d0;
      }
      if (dst != nullptr) *reinterpret_cast<uint4*>(dst) = v;
    }
  }
  constexpr int CPR = BN / 8;  // 16-B pieces per row
  const bool full = n_blk + BN <= N && (N & 7) == 0 && ((uintptr_t)y & 15) == 0;
#pragma unroll
  for (int c = epi != 0 ? kBM * CPR : tid; c < kBM * CPR; c += NTH) {
    const int r = c / CPR, cc = c % CPR;
    const int m = m_blk + r;
    if (m >= M) continue;
    if (seam && S > 1 && ((r / RM) * WN + (8 * cc) / CN) / wpo != z) continue;  // not owned
    const uint4 v = reinterpret_cast<const uint4*>(out)[c];
    if (full) {
      *reinterpret_cast<uint4*>(y + (size_t)m * N + n_blk + 8 * cc) = v;
    } else {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
      for (int k = 0; k < 8; ++k)
        if (n_blk + 8 * cc + k < N) y[(size_t)m * N + n_blk + 8 * cc + k] = e[k];
    }
  }
}

// ---- launch ------------------------------------------------------------------------------------
// the kernels' `fenced` argument: bit 0 agent fences on the hand-off, bit 1 the late-publisher
// test hook (tao_debug_sf_late_publisher)
inline int sk_flags() { return tuning().splitk_fenced | (tuning().sf_late_pub ? 2 : 0); }

struct SfShape {
  int bn, wm, splits, stages, a_steps;
  int seam;    // 0 fixed reducer, 1 spread (see the kernel)
  int kh = 1;  // the 32x32x16 int4 kernel (wm 1): k halves per column group, 1 or 2
  int ld = 0;  // 16x16x32 kernel, 64-column tiles: 4 dedicated LDS-DMA loader waves
  int xm = 0;  // fixed-reducer seam: each K slice's workgroups on their own XCDs (sf_xmap)
};

// loader waves of the 16x16 kernel: tao_tune_gemm_sf_loaders 1 = none, 2 = 4, 3 = 8; 0 = route
int sf_loader_waves(const SfShape& sh) {
  const int m = tuning().sf_loaders;
  return m == 1 ? 0 : m == 2 ? 4 : m == 3 ? 8 : (sh.ld != 0 ? 4 : 0);
}

template <class P, int BN, int WM, int NS>
bool sf_go(const SfShape& sh, hipStream_t stream, const uint8_t* x, const P& pol,
           const uint16_t* bias, uint16_t* y, int M, int N, int K, int a, typename P::Acc* slab,
           unsigned* cnt, const SfEpi& ep, int loaders) {
  constexpr int STAGE = kBM * P::kXRow + BN * P::kWRow + BN * P::kZRow;
  constexpr int NB = NS;
  if constexpr (NB * STAGE <= 160 * 1024 && (kBM * P::kXRow + BN * P::kWRow + BN * P::kZRow) > 0) {
    constexpr int T = (kBM * P::kXRow) / 1024 + (BN * P::kWRow) / 1024 + (BN * P::kZRow) / 256;
    if constexpr (T % kWaves == 0 && (BN * P::kWRow) % 1024 == 0 && (BN * P::kZRow) % 256 == 0 &&
                  BN / (kWaves / WM) >= 16)
    {
      const int ntn = (N + BN - 1) / BN, mtiles = (M + kBM - 1) / kBM;
      const dim3 grid((unsigned)(ntn * sh.splits * mtiles));
      const int xm = tuning().sf_xmap ? tuning().sf_xmap == 2 : sh.xm;
      const int xmap = xm && !sh.seam && (sh.splits == 2 || sh.splits == 4 || sh.splits == 8) &&
                       ntn % (8 / sh.splits) == 0;
      if constexpr (BN <= 64 && T % 4 == 0 && ((kBM * P::kXRow) / 1024) % 4 == 0) {  // wider: spills
        if (loaders == 4) {  // 4 loader waves beside the 8 compute waves
          launch(gemm_sf_kernel<P, BN, WM, NS, 4>, grid, dim3(768), 0, stream, x, pol, bias, y, M,
                 N, K, a, slab, cnt, sk_flags(), sh.splits, ntn, sh.seam,
                 tuning().cnt_stride, ep, xmap);
          return true;
        }
      }
      if constexpr (BN <= 64 && T % 8 == 0 && ((kBM * P::kXRow) / 1024) % 8 == 0 && P::kABytes == 2) {
        if (loaders == 8) {  // 8 loader waves (two per SIMD), 16 waves: <= 128 VGPRs
          launch(gemm_sf_kernel<P, BN, WM, NS, 8>, grid, dim3(1024), 0, stream, x, pol, bias, y, M,
                 N, K, a, slab, cnt, sk_flags(), sh.splits, ntn, sh.seam,
                 tuning().cnt_stride, ep, xmap);
          return true;
        }
      }
      launch(gemm_sf_kernel<P, BN, WM, NS>, grid, dim3(512), 0, stream, x, pol, bias, y, M, N, K,
             a, slab, cnt, sk_flags(), sh.splits, ntn, sh.seam, tuning().cnt_stride,
             ep, xmap);
      return true;
    }
  }
  return false;  // combination not instantiated (LDS, DMA split or wave tile)
}

template <class P, int BN>
int sf_dispatch_wm(const SfShape& sh, hipStream_t st, const uint8_t* x, const P& pol,
                   const uint16_t* bias, uint16_t* y, int M, int N, int K, int a,
                   typename P::Acc* slab, unsigned* cnt, const SfEpi& ep = SfEpi{}) {
  bool ok = false;
  auto go = [&](auto wmc, auto nsc) {
    constexpr int W = decltype(wmc)::value, S_ = decltype(nsc)::value;
    ok = sf_go<P, BN, W, S_>(sh, st, x, pol, bias, y, M, N, K, a, slab, cnt, ep,
                             sf_loader_waves(sh));
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

// Routed shapes (64 < M <= 128, one 128-row M tile), from the sweep against the incumbent
// MFMA GEMM on the same box (experiments/sweep_sf.py, profiles/r4_sf_sweep_cnt_stride.jsonl; us,
// incumbent -> single-fetch): int8 dyn 6144x4096 15.0 -> 12.8, 28672x4096 37.6 -> 31.1 (256-column
// tiles, r4_sf_sweep_bn256.jsonl),
// 4096x14336 23.6 -> 20.4; int4 4096^2 14.6 -> 14.0, 6144x4096 21.6 -> 19.4, 28672x4096
// 59.9 -> 50.0 (the 32x32x16 kernel, one wave along M), 4096x14336 32.6 -> 31.6. Config 3
// (int8 dyn 4096^2: 10.4 vs 10.6) and every M <= 64 stay on the incumbent. Round 5: 4 dedicated
// loader waves on the 64-column int4 tiles where they measured faster (profiles/r5f_ab_loaders*.jsonl,
// same-process alternation; slower at 6144x4096, neutral at 4096^2 and for int8 dyn).
struct SfRoute {
  int path, n, k;
  SfShape sh;
  int ks;
};
constexpr SfRoute kSfRoutes[] = {
    {2, 6144, 4096, {64, 4, 2, 3, 0, 0}, 256},
    {2, 28672, 4096, {256, 4, 2, 3, 0, 1}, 128},
    {2, 4096, 14336, {64, 4, 4, 4, 0, 1}, 128},
    {0, 4096, 4096, {64, 2, 4, 4, 0, 0, 1, 1}, 0},  // r5: 4 stages + loaders 14.6 -> 14.0
    {0, 6144, 4096, {64, 2, 2, 3, 0, 0, 1, 1}, 0},  // r5: S 2, 3 stages + loaders 19.7 -> 18.2
    {0, 28672, 4096, {128, 1, 1, 3, 0, 0}, 0},
    {0, 4096, 14336, {64, 2, 4, 4, 0, 0, 1, 1}, 0},  // loader waves: 31.9 -> 28.7 us
    // Llama-3-70B (profiles/r4_sf_sweep_70b.jsonl; us, incumbent -> single-fetch): int8 dyn
    // 10240x8192 42.6 -> 29.6, 8192^2 27.4 -> 21.6, 57344x8192 145.2 -> 99.2, 8192x28672
    // 68.4 -> 55.8; int4 10240x8192 62.2 -> 48.4, 8192^2 37.8 -> 32.9, 57344x8192 225.9 ->
    // 178.7, 8192x28672 115.1 -> 90.7 (for int4 with wm 1 the ks field is the k halves);
    // int4 57344x8192 on 256-column tiles of the 32x32x16 kernel (8 waves, 224 tiles: one per
    // CU) 171.4 against 213.8 / 195.1 for 128 columns with / without k halves
    // (profiles/r4_sf32_70b.jsonl)
    {2, 10240, 8192, {256, 2, 4, 3, 0, 1}, 128},
    {2, 8192, 8192, {64, 4, 2, 3, 0, 0}, 256},
    {2, 57344, 8192, {256, 2, 1, 3, 0, 0}, 128},
    {2, 8192, 28672, {64, 4, 2, 3, 0, 1}, 256},
    {0, 10240, 8192, {128, 1, 2, 3, 0, 0}, 2},
    {0, 8192, 8192, {64, 2, 2, 3, 0, 0, 1, 1}, 0},  // loader waves: 36.6 -> 33.0 us
    {0, 57344, 8192, {256, 1, 1, 3, 0, 0}, 0},
    {0, 8192, 28672, {128, 2, 4, 3, 0, 1}, 0},
};

static const SfRoute* sf_route(int path, int64_t M, int64_t N, int64_t K) {
  if (M <= 64 || M > 128) return nullptr;
  for (const SfRoute& r : kSfRoutes)
    if (r.path == path && r.n == N && r.k == K) return &r;
  return nullptr;
}

// Launch shape: the routed entry, else (tao_tune_gemm_sf mode 2 on other shapes) the smallest
// split S (1, 2, 4, 8) whose grid (N / BN tiles x S) reaches 256 workgroups, publishers taking
// an equal share of the steps. tao_tune_gemm_sf / _seam override every field.
static SfShape sf_shape(int path, int M, int N, int K, int* ks_out = nullptr) {
  const int kstep = path == 0 ? 128 : 256;
  const int nsteps = K / kstep;
  const Tuning& t = tuning();
  const SfRoute* r = sf_route(path, M, N, K);
  SfShape sh{path == 0 ? 64 : 32, path == 0 ? 2 : 4, 1, 3, 0, 0};
  if (r) sh = r->sh;
  if (ks_out) *ks_out = t.sf_ks ? t.sf_ks : (r && r->ks ? r->ks : 256);
  // int4 (path 0): the route's / tune's ks field is the 32x32x16 kernel's k halves (1, 2)
  if (path == 0) sh.kh = t.sf_ks == 2 ? 2 : t.sf_ks == 1 ? 1 : (r && r->ks == 2 ? 2 : 1);
  if (t.sf_bn) sh.bn = t.sf_bn;
  if (t.sf_wm) sh.wm = t.sf_wm;
  if (t.sf_stages) sh.stages = t.sf_stages;
  if (!r || t.sf_bn) {
    const long tiles = (N + sh.bn - 1) / sh.bn;
    sh.splits = 1;
    while (tiles * sh.splits < 256 && sh.splits < 8 && nsteps >= 2 * sh.splits * 2) sh.splits *= 2;
  }
  if (t.sf_splits) sh.splits = t.sf_splits;
  if (sh.splits > nsteps) sh.splits = nsteps;
  sh.a_steps = nsteps / sh.splits;
  if (t.sf_a_steps) sh.a_steps = t.sf_a_steps;
  if (sh.splits > 1 && sh.a_steps * (sh.splits - 1) >= nsteps) sh.a_steps = nsteps / sh.splits;
  // the spread seam's S workgroups of a tile wait for one another: S must divide the 8 waves,
  // and S consecutive workgroups must be resident together (1 per CU: S <= 8 << 256 CUs)
  if (t.sf_seam >= 0) sh.seam = t.sf_seam;
  if (sh.splits != 2 && sh.splits != 4 && sh.splits != 8) sh.seam = 0;
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
  return sf_route(path, M, N, K) != nullptr;  // auto: the measured shapes
}

int sf_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
               const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  int ks = 256;
  const SfShape sh = sf_shape(2, M, N, K, &ks);
  ks = ks == 128 ? 128 : 256;
  const dim3 grid((N + sh.bn - 1) / sh.bn, 1, (M + kBM - 1) / kBM);  // tiles: grid.x grid.z
  i32x4_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (sh.splits > 1) {
    void* w = nullptr;
    const size_t tiles = (size_t)grid.x * grid.z;
    const int rc = split_workspace(stream, tiles * sh.splits * kBM * sh.bn * 4,
                                   tiles * tuning().cnt_stride, &w, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<i32x4_t*>(w);
  }
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(xq);
  // a_steps is in units of the policy's k step (256 k; 128-k steps take twice as many)
  auto run = [&](auto pol, int a) -> int {
    typedef decltype(pol) P;
    switch (sh.bn) {
      case 32: return sf_dispatch_wm<P, 32>(sh, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
      case 128: return sf_dispatch_wm<P, 128>(sh, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
      case 256: return sf_dispatch_wm<P, 256>(sh, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
      default: return sf_dispatch_wm<P, 64>(sh, stream, xb, pol, bias, y, M, N, K, a, slab, cnt);
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
              int stages, int a_steps, hipStream_t stream, int epi, int kh);

// ep.kind 1: y [M][N / 2] = SwiGLU of the interleaved (gate, up) output pairs; 2: RoPE + KV
// write (y unused). Both need bias == nullptr.
int sf_int4_epi(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int lg,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
                const SfEpi& ep) {
  const SfShape sh = sf_shape(0, M, N, K);
  if (sh.wm == 1) {  // one wave along M: the 32x32x16 kernel (gemm_sf32.hip)
    if (ep.kind == 2)
      return set_error(TAO_ERR_UNSUPPORTED, "gemm_sf: no RoPE epilogue on the 32x32x16 kernel");
    return sf32_int4(x, packed, sz, lg, bias, y, M, N, K, sh.bn, sh.splits, sh.stages,
                     tuning().sf_a_steps, stream, ep.kind, sh.kh);
  }
  // a column tile only a tuning override can ask for: UNSUPPORTED, so the fused-epilogue callers
  // fall back to the plain linear + the separate epilogue kernel (checked before any workspace)
  if (sh.bn != 64 && sh.bn != 128 && sh.bn != 256)
    return set_error(TAO_ERR_UNSUPPORTED, "gemm_sf: int4 takes bn 64, 128 or 256 (got %d)", sh.bn);
  const dim3 grid((N + sh.bn - 1) / sh.bn, 1, (M + kBM - 1) / kBM);  // tiles: grid.x grid.z
  f32x4_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (sh.splits > 1 && ep.kind != 3) {  // (the partials-out launch has no seam)
    void* w = nullptr;
    const size_t tiles = (size_t)grid.x * grid.z;
    const int rc = split_workspace(stream, tiles * sh.splits * kBM * sh.bn * 4,
                                   tiles * tuning().cnt_stride, &w, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<f32x4_t*>(w);
  }
  SfI4 pol{packed, reinterpret_cast<const uint32_t*>(sz), lg};
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(x);
  switch (sh.bn) {
    case 256:
      return sf_dispatch_wm<SfI4, 256>(sh, stream, xb, pol, bias, y, M, N, K, sh.a_steps, slab, cnt,
                                       ep);
    case 128:
      return sf_dispatch_wm<SfI4, 128>(sh, stream, xb, pol, bias, y, M, N, K, sh.a_steps, slab, cnt,
                                       ep);
    default:  // 64
      return sf_dispatch_wm<SfI4, 64>(sh, stream, xb, pol, bias, y, M, N, K, sh.a_steps, slab, cnt,
                                      ep);
  }
}

// The launch shape the single-fetch GEMM takes for (path, M <= 128, N, K) -- 0 int4, 2 int8 dyn
// -- for the LDS-DMA intake probe (probe_intake.hip): column tile, K slices, ring stages, k steps
// per publishing slice, loader waves (0 / 4), k step, one wave along M (the 32x32x16 kernel).
void sf_launch_shape(int path, int M, int N, int K, int* bn, int* splits, int* stages,
                     int* a_steps, int* loaders, int* kstep, int* wm1) {
  int ks = 256;
  const SfShape sh = sf_shape(path, M, N, K, &ks);
  *bn = sh.bn;
  *splits = sh.splits;
  *stages = sh.stages;
  *a_steps = path == 2 && ks == 128 ? sh.a_steps * 2 : sh.a_steps;  // (in units of *kstep)
  *loaders = path == 0 && sh.wm != 1 && sh.bn <= 64 ? sf_loader_waves(sh) : 0;
  *kstep = path == 0 ? 128 : (ks == 128 ? 128 : 256);
  *wm1 = path == 0 && sh.wm == 1;
}

// K slices the partials-out launch of this int4 shape writes (0: not served, the 32x32x16 route)
int sf_int4_partial_slices(int M, int N, int K) {
  const SfShape sh = sf_shape(0, M, N, K);
  if (sh.wm == 1 || (sh.bn != 64 && sh.bn != 128 && sh.bn != 256)) return 0;
  return sh.splits;
}

int sf_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int lg,
            const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
            int epi = 0) {
  SfEpi ep{};
  ep.kind = epi;
  return sf_int4_epi(x, packed, sz, lg, bias, y, M, N, K, stream, ep);
}

}  // namespace tao

// int4 weight-only linear with the SwiGLU of interleaved (gate, up) output rows folded into the
// epilogue (the w1||w3 linear of a prefill and its SiLU-mul in one launch): y [M][N / 2] =
// bf16(bf16(silu(a_i)) * b_i), (a_i, b_i) = bf16 outputs of rows (2i, 2i+1). Served by the
// single-fetch GEMM where it is routed (tao_tune_gemm_sf 2: wherever it applies);
// TAO_ERR_UNSUPPORTED elsewhere (the caller runs the linear and tao_silu_mul_bf16).
namespace tao {
int int4_check_linear_args(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                           uint16_t* y, int64_t M, int64_t N, int64_t K, int64_t group_size);
}  // namespace tao

namespace tao {
bool int4_linear_takes_gemv(int64_t M, int64_t N, int64_t K);
}  // namespace tao

static int lg_of(int64_t g) { return g == 32 ? 5 : g == 64 ? 6 : g == 128 ? 7 : 8; }

extern "C" int tao_int4wo_linear_swiglu_bf16(const uint16_t* x, const uint32_t* packed,
                                             const uint16_t* sz, uint16_t* y, int64_t M,
                                             int64_t N, int64_t K, int64_t group_size,
                                             void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, sz, y, M, N, K, group_size);
  if (rc != TAO_OK) return rc;
  TAO_CHECK_ARG(N % 16 == 0, "int4 swiglu linear: N (%lld) must be a multiple of 16",
                (long long)N);
  if (M == 0) return TAO_OK;
  if (!tao::use_sf(0, M, N, K, group_size) || M > (1 << 20))
    return tao::set_error(TAO_ERR_UNSUPPORTED,
                          "int4 swiglu linear: no fused kernel for M=%lld N=%lld K=%lld",
                          (long long)M, (long long)N, (long long)K);
  return tao::sf_int4(x, packed, sz, lg_of(group_size), nullptr, y, (int)M, (int)N, (int)K,
                      tao::as_stream(stream), 1);
}

// int4 weight-only wqkv linear of a prefill with RoPE and the KV-cache write folded into the
// epilogue (tao_rope_kv_bf16's math and layouts): x [B S][K]; q_out [B][H][S][D] (rotated);
// k (rotated), v -> caches [B][Hkv][T][D] at row pos[s]; D == 128; the weight is [(H + 2 Hkv) D][K].
// Served where the single-fetch GEMM is routed (not its 32x32x16 variant); TAO_ERR_UNSUPPORTED
// elsewhere (the caller runs the linear and tao_rope_kv_bf16).
extern "C" int tao_int4wo_linear_rope_kv_bf16(const uint16_t* x, const uint32_t* packed,
                                              const uint16_t* sz, int64_t K, int64_t group_size,
                                              const float* freqs, const int64_t* pos,
                                              uint16_t* q_out, uint16_t* k_cache,
                                              uint16_t* v_cache, int64_t B, int64_t S, int64_t H,
                                              int64_t Hkv, int64_t D, int64_t T, void* stream) {
  TAO_CHECK_ARG(D == 128, "int4 rope linear: head_dim must be 128 (got %lld)", (long long)D);
  TAO_CHECK_ARG(B > 0 && S > 0 && H > 0 && Hkv > 0 && T > 0 && B * S < (1LL << 30),
                "int4 rope linear: bad sizes");
  const int64_t M = B * S, N = (H + 2 * Hkv) * D;
  int rc = tao::int4_check_linear_args(x, packed, sz, q_out, M, N, K, group_size);
  if (rc != TAO_OK) return rc;
  TAO_CHECK_ALIGN(q_out, 16, "q_out");
  TAO_CHECK_ALIGN(k_cache, 16, "k_cache");
  TAO_CHECK_ALIGN(v_cache, 16, "v_cache");
  TAO_CHECK_ALIGN(freqs, 8, "freqs");
  if (!tao::use_sf(0, M, N, K, group_size))
    return tao::set_error(TAO_ERR_UNSUPPORTED,
                          "int4 rope linear: no fused kernel for M=%lld N=%lld K=%lld",
                          (long long)M, (long long)N, (long long)K);
  tao::SfEpi ep{};
  ep.kind = 2;
  ep.freqs = freqs;
  ep.pos = pos;
  ep.q_out = q_out;
  ep.kc = k_cache;
  ep.vc = v_cache;
  ep.S = (int)S;
  ep.H = (int)H;
  ep.Hkv = (int)Hkv;
  ep.T = (int)T;
  return tao::sf_int4_epi(x, packed, sz, lg_of(group_size), nullptr, q_out, (int)M, (int)N,
                          (int)K, tao::as_stream(stream), ep);
}

// int4 weight-only linear whose K slices hand their fp32 partial tiles to the NEXT launch instead
// of reducing them in-kernel (no split-K seam): part [S][M][N] fp32, S = the routed split count
// (tao_int4wo_linear_partial_slices). The residual add + RMSNorm that follows wo / w2 in a prefill
// sums them (tao_add_rmsnorm_partials_bf16): bf16(sum in slice order) is bit-identical to the
// linear's bf16 output. TAO_ERR_UNSUPPORTED where the shape is not routed to the 16x16 kernel.
extern "C" int tao_int4wo_linear_partial_slices(int64_t M, int64_t N, int64_t K,
                                                int64_t group_size, int* slices) {
  TAO_CHECK_ARG(slices != nullptr, "int4 partials: null output");
  *slices = 0;
  // served only where the plain linear takes this same kernel (not the skinny-M GEMV), so
  // summing the partials reproduces its output bit for bit
  if (M > 0 && M <= (1 << 20) && N > 0 && K > 0 && !tao::int4_linear_takes_gemv(M, N, K) &&
      tao::use_sf(0, M, N, K, group_size))
    *slices = tao::sf_int4_partial_slices((int)M, (int)N, (int)K);
  return TAO_OK;
}

extern "C" int tao_int4wo_linear_partials_f32(const uint16_t* x, const uint32_t* packed,
                                              const uint16_t* sz, float* part, int64_t M,
                                              int64_t N, int64_t K, int64_t group_size,
                                              void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, sz, reinterpret_cast<uint16_t*>(part), M, N, K,
                                       group_size);
  if (rc != TAO_OK) return rc;
  if (M == 0 || N == 0) return TAO_OK;
  TAO_CHECK_ALIGN(part, 4, "part");
  int S = 0;
  tao_int4wo_linear_partial_slices(M, N, K, group_size, &S);
  if (S == 0)
    return tao::set_error(TAO_ERR_UNSUPPORTED,
                          "int4 partials: no 16x16 single-fetch route for M=%lld N=%lld K=%lld",
                          (long long)M, (long long)N, (long long)K);
  tao::SfEpi ep{};
  ep.kind = 3;
  ep.part = part;
  return tao::sf_int4_epi(x, packed, sz, lg_of(group_size), nullptr, nullptr, (int)M, (int)N,
                          (int)K, tao::as_stream(stream), ep);
}

// Single-fetch prefill GEMM routing and launch shape (calling thread only; for A/B measurement):
// mode 0 = built-in routing, 1 = never, 2 = whenever the shape is supported (M <= 128 per launch
// tile); bn / wm / splits / stages / a_steps 0 = built-in; ks = int8 k step 128 or 256 (0 = 256),
// or for int4 with wm 1 (the 32x32x16 kernel) the k halves per column group, 1 or 2.
extern "C" int tao_tune_gemm_sf(int mode, int bn, int wm, int splits, int stages, int a_steps,
                                int ks) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 2, "tune: gemm_sf mode must be 0, 1 or 2");
  TAO_CHECK_ARG(bn == 0 || bn == 32 || bn == 64 || bn == 128 || bn == 256,
                "tune: gemm_sf bn must be 0, 32, 64, 128, 256");
  TAO_CHECK_ARG(wm == 0 || wm == 1 || wm == 2 || wm == 4 || wm == 8,
                "tune: gemm_sf wm must be 0, 1 (int4: the 32x32x16 kernel), 2, 4 or 8");
  TAO_CHECK_ARG(splits >= 0 && splits <= 16, "tune: gemm_sf splits must be in [0, 16]");
  TAO_CHECK_ARG(stages == 0 || (stages >= 2 && stages <= 4), "tune: gemm_sf stages must be 0, 2, 3, 4");
  TAO_CHECK_ARG(a_steps >= 0, "tune: gemm_sf a_steps must be >= 0");
  TAO_CHECK_ARG(ks == 0 || ks == 1 || ks == 2 || ks == 128 || ks == 256,
                "tune: gemm_sf ks must be 0, 128 or 256 (int8 k step) or 1, 2 (int4 wm 1: k halves)");
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

// Dedicated loader waves of the single-fetch kernels: 0 = built-in, 1 = off, 2 = on (4 waves),
// 3 = 8 waves (16x16 int4 kernel, 64-column tiles; elsewhere as 2).
extern "C" int tao_tune_gemm_sf_loaders(int mode) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 3, "tune: gemm_sf_loaders must be 0..3");
  tao::tuning().sf_loaders = mode;
  return TAO_OK;
}

// Test hook: split-K publishers of slice 0 add their ticket only after a reducer has timed out
// (both single-fetch kernels, fixed-reducer seam). 1 = on, 0 = off. Thread-local.
extern "C" int tao_debug_sf_late_publisher(int on) {
  TAO_CHECK_ARG(on == 0 || on == 1, "debug: sf_late_publisher must be 0 or 1");
  tao::tuning().sf_late_pub = on;
  return TAO_OK;
}

// K slice -> XCD block mapping under the fixed-reducer seam: 0 = built-in, 1 = off, 2 = on.
extern "C" int tao_tune_gemm_sf_xmap(int mode) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 2, "tune: gemm_sf_xmap must be 0, 1 or 2");
  tao::tuning().sf_xmap = mode;
  return TAO_OK;
}

// Split-K seam of the single-fetch GEMM: -1 = built-in (per routed shape), 0 = fixed reducer,
// 1 = spread.
extern "C" int tao_tune_gemm_sf_seam(int seam) {
  TAO_CHECK_ARG(seam >= -1 && seam <= 1,
                "tune: gemm_sf_seam must be -1 (built-in), 0 (fixed reducer) or 1 (spread)");
  tao::tuning().sf_seam = seam;
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

