// Single-fetch int4 prefill GEMM on 32x32x16 MFMAs (the int4 member of the gemm_sf family):
//   y[M][N] = bf16( x[M][K] . dequant(W)[N][K]^T ) (+ bias),  bf16 x, int4 row-stream W,
//   B = bf16(fma(q, s, z - 8 s)) as the reference's dequantised weight.
// Replaces aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104) at prefill sizes.
//
// gemm_sf.hip's 16x16x32 int4 tile was bound by its per-wave work, not memory: with 8 waves in a
// 2 (M) x 4 (N) layout every B fragment was dequantised twice (~14 VALU per 8 weights, partly
// v_pk_fma_f32, which stalls beside MFMAs) and every A fragment read from LDS fed 1-2 MFMAs. Here
// each wave owns a 128-row x 32-column output tile (4 accumulators of v_mfma_f32_32x32x16_bf16):
//   * a B fragment (8 weights per lane) is dequantised once per workgroup and feeds 4 MFMAs;
//   * an A fragment read (16 B per lane, 1 KiB per wave) feeds one 32x32x16 MFMA (2x the MACs of
//     a 16x16x32), so LDS bytes per MAC halve;
//   * the k order inside a 128-k step is permuted identically for A and B: lane half h owns k
//     64 h .. 64 h + 63 and MFMA ks takes k 64 h + 8 ks + j, so a lane's B operand for the whole
//     step is 32 contiguous nibble bytes of its column (two ds_read_b128) and its (scale, zero)
//     words are those of groups 2 h and 2 h + 1 of the step (one ds_read_b64);
//   * WV waves (2 or 4) = BN / 32 columns, one wave per SIMD: latency is covered by the LDS-DMA
//     ring (NS stages, counted vmcnt, barriers that do not drain it), not by occupancy.
// Images (16-B granule swizzles; each an involution, so a DMA lane filling position p fetches
// granule pos(row, p)): x [128][256 B] at g ^ (r & 15); W [BN][64 B] at g ^ ((n >> 2) & 3);
// (scale, zero) [BN][4 dwords] at q ^ (2 ((n >> 4) & 1)). All fragment reads conflict-free
// (tests/test_host_cpu.py checks the bank map).
// K split S ways with gemm_sf.hip's fixed-reducer hand-off (sc1 slabs + ticket, slice S - 1 sums
// in slice order).
#include <type_traits>

#include "tao_common.h"

// Timing-only variant builds (experiments/sf32_debug.sh; never the shipped library; results
// wrong): 1 no MFMAs (the B fragment folded into one accumulator lane), 2 no dequantisation (the
// nibble words reinterpreted as bf16), 3 no LDS-DMA after the prologue (steps reuse stale
// stages), 4 no A-fragment LDS reads (one read per step reused), 5 x read as if step-major
// ([K / 128][M][128]: each step's x one contiguous block), 6 / 7 no (scale, zero) / W DMA after
// the prologue (per-instruction vs per-byte cost of the DMA pieces).
// 1: with 3+ stages, each step's DMA pieces are issued between its MFMA k sub-steps (0: all after
// the step's barrier). 2-5% faster at 3 stages, slower at 2 (the stage is needed one step later):
// profiles/r4_sf32_il.jsonl
// 1: 16-B (scale, zero) DMA pieces at group size 32 (the kernel's Z16; 0 for A/B builds)
#ifndef TAO_SF32_Z16
#define TAO_SF32_Z16 1
#endif
#ifndef TAO_SF32_IL
#define TAO_SF32_IL 1
#endif
// A-fragment buffers of the compute waves (1 or 2; measured the same: r5g_ab_sf32_abuf.jsonl)
#ifndef TAO_SF32_ABUF
#define TAO_SF32_ABUF 2
#endif

namespace tao {
namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;
constexpr int kXRow = 256, kWRow = 64, kZRow = 16;  // bytes per row per 128-k step

__device__ unsigned g_sf32_err = 0;

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

__device__ __forceinline__ uint32_t pkb(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ int xpos(int row, int g) { return g ^ (row & 15); }
__device__ __forceinline__ int wpos(int row, int g) { return g ^ ((row >> 2) & 3); }
__device__ __forceinline__ int zpos(int row, int q) { return q ^ (((row >> 4) & 1) << 1); }

// 8 nibbles of a row-stream dword -> bf16(fma(q, s, zc)) in k order; scalar fmas (v_pk_fma_f32
// beside MFMAs costs ~22 extra cycles each: MI355X_MICROARCH.md cycle table; the Makefile builds
// this file with -fno-slp-vectorize, which otherwise paired them back into v_pk_fma_f32)
__device__ __forceinline__ bf16x8_t deq8s(uint32_t w, float sc, float zc) {
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
  const f32x2_t q04 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, false);
  const f32x2_t q15 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, true);
  const f32x2_t q26 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, false);
  const f32x2_t q37 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, true);
  const float w0 = __builtin_fmaf(q04[0], sc, zc), w4 = __builtin_fmaf(q04[1], sc, zc);
  const float w1 = __builtin_fmaf(q15[0], sc, zc), w5 = __builtin_fmaf(q15[1], sc, zc);
  const float w2 = __builtin_fmaf(q26[0], sc, zc), w6 = __builtin_fmaf(q26[1], sc, zc);
  const float w3 = __builtin_fmaf(q37[0], sc, zc), w7 = __builtin_fmaf(q37[1], sc, zc);
  const u32x4_t v = {pkb(w0, w1), pkb(w2, w3), pkb(w4, w5), pkb(w6, w7)};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int N>
__device__ __forceinline__ void wait_ahead(int ahead) {
  switch (ahead) {
    case 0: wait_vmcnt<0>(); break;
    case 1: wait_vmcnt<N>(); break;
    default: wait_vmcnt<2 * N>(); break;
  }
}

// KH = 2: two waves per column group split each step's k (k half kh: MFMA sub-steps 4 kh ..
// 4 kh + 3, one (scale, zero) group pair), so 2 waves share each SIMD and one's MFMAs and
// dequantisation cover the other's LDS waits; the halves' accumulators are summed through LDS
// (in kh order) after the k loop. Same LDS bytes read per step, same dequantisation work.
// Z16 (group size 32): a row's 4 (scale, zero) words of a step are 16 contiguous bytes of the
// [N][K/32][2] array, so they arrive by 16-B DMA, 64 rows per piece, into an unswizzled
// [BN][16 B] image read with one ds_read_b128 per lane (conflict-free: 8 lanes per 128 B); other
// group sizes take the 4-B DMA of a swizzled image. The DMA pieces cost per instruction
// (profiles/r4_sf32_dmacost.jsonl), and Z16 takes a quarter of them for the (scale, zero) words.
// LDW > 0 (KH = 1): LDW dedicated loader waves issue every LDS-DMA piece (they wait for their own
// pieces, join the step barrier and refill the freed stage) and the WV compute waves only read
// LDS, dequantise and issue MFMAs. Per-step stamps (a timing build, round 4) put the one-wave
// kernel at ~2350 of ~2760 cycles per step in its compute phase (32 MFMAs = 1024 cycles), of
// which the DMA pieces issued between the MFMA sub-steps are ~640 (the no-DMA timing build):
// a loader wave on each SIMD takes that issue off the MFMA stream (VMEM and VALU / MFMA issue
// from different waves of a SIMD proceed in parallel).
template <int WV, int NS, int KH = 1, bool Z16 = false, int LDW = 0>
__global__ __launch_bounds__((WV * KH + LDW) * 64) void gemm_sf32_int4_kernel(
    const uint16_t* __restrict__ x, const uint32_t* __restrict__ wq, const uint32_t* __restrict__ sz,
    int lg, const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K,
    int a_steps, f32x16_t* __restrict__ slab, unsigned* __restrict__ cnt, int fenced, int cs,
    int epi) {
  constexpr int BN = 32 * WV;
  constexpr int NW = WV * KH;  // compute waves
  constexpr int NWT = NW + LDW;            // waves of the workgroup
  constexpr int DW = LDW > 0 ? LDW : NW;   // waves that issue the DMA pieces
  constexpr bool IL = TAO_SF32_IL != 0 && NS >= 3 && LDW == 0;
  constexpr int XB = kBM * kXRow, WB = BN * kWRow, ZB = BN * kZRow;
  constexpr int STAGE = XB + WB + ZB;
  constexpr int PX = XB / 1024, PW = WB / 1024, PZ = Z16 ? ZB / 1024 : ZB / 256;
  constexpr int T = PX + PW + PZ;
  static_assert(PX % DW == 0 && (!Z16 || ZB % 1024 == 0), "DMA pieces per wave");
  // piece i = r DW + dma wave: waves below RFULL issue R pieces per stage, the others R - 1
  constexpr int R = (T + DW - 1) / DW, RFULL = T - (R - 1) * DW;
  static_assert(NS * STAGE <= 160 * 1024 && kBM * BN * 2 <= NS * STAGE, "LDS");
  __shared__ uint4 lds[NS * STAGE / 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool loader = LDW > 0 && wave >= NW;
  const int dwv = LDW > 0 ? wave - NW : wave;       // index among the DMA-issuing waves
  const int cw = loader ? 0 : wave % WV, kh = loader ? 0 : wave / WV;  // column group, k half
  const int r32 = lane & 31, h = lane >> 5;
  const int n_blk = blockIdx.x * BN, m_blk = blockIdx.z * kBM;
  const int S = gridDim.y, z = blockIdx.y;
  const bool reducer = z == S - 1;
  const int nsteps = K / 128;
  const int s0 = z * a_steps;
  const int J = reducer ? nsteps - s0 : a_steps;
  const uint32_t row_bytes = (uint32_t)K * 2;

  const Rsrc xrs = make_rsrc(x, (uint32_t)M * row_bytes);
  const Rsrc wrs = make_rsrc(wq, (uint32_t)N * (uint32_t)(K >> 1));
  const Rsrc zrs = make_rsrc(sz, (uint32_t)N * (uint32_t)(K >> lg) * 4u);
  uint32_t dv[R];
  int dd[R], dk[R];
  sfor<0, R>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (r < PX / DW) {  // x: 4 rows x 256 B
      const int i = r * DW + dwv;
      const int row = 4 * i + (lane >> 4), p = lane & 15;
      const int gm = m_blk + row < M ? m_blk + row : M - 1;
      dv[r] = (uint32_t)gm * row_bytes + 16u * (uint32_t)xpos(row, p);
      dd[r] = i * 1024;
      dk[r] = 0;
    } else {
      const int i = (r - PX / DW) * DW + dwv;
      const int row = 16 * (i < PW ? i : i - PW) + (lane >> 2), p = lane & 3;
      const int gn = n_blk + row < N ? n_blk + row : N - 1;
      if (i < PW) {  // W: 16 rows x 64 B
        dv[r] = (uint32_t)gn * (uint32_t)(K >> 1) + 16u * (uint32_t)wpos(row, p);
        dd[r] = XB + i * 1024;
        dk[r] = 1;
      } else if (i >= PW + PZ) {  // past the last piece (T not a multiple of NW)
        dv[r] = 0;
        dd[r] = 0;
        dk[r] = 3;
      } else if constexpr (Z16) {  // (scale, zero): 64 rows x 16 B
        const int zr = 64 * (i - PW) + lane;
        const int gz = n_blk + zr < N ? n_blk + zr : N - 1;
        dv[r] = (uint32_t)gz * (uint32_t)(K >> lg) * 4u;
        dd[r] = XB + WB + (i - PW) * 1024;
        dk[r] = 2;
      } else {  // (scale, zero): 16 rows x 4 dwords, 4-B DMA; dword q = group of k 32 q
        const int q = zpos(row, p);
        dv[r] = ((uint32_t)gn * (uint32_t)(K >> lg) + (uint32_t)((32 * q) >> lg)) * 4u;
        dd[r] = XB + WB + (i - PW) * 256;
        dk[r] = 2;
      }
    }
  });
  auto issue_piece = [&](auto rc, int st, int buf) __attribute__((always_inline)) {
    constexpr int r = decltype(rc)::value;
    uint8_t* base = reinterpret_cast<uint8_t*>(lds) + buf * STAGE;
    if constexpr (r < PX / DW) {
      dma_lds_ring<16>(xrs, dv[r], (uint32_t)st * kXRow, base + dd[r]);
    } else {
      if (dk[r] == 1) dma_lds_ring<16, kNT>(wrs, dv[r], (uint32_t)st * 64u, base + dd[r]);
      else if (dk[r] == 2) {
        if constexpr (Z16) dma_lds_ring<16, kNT>(zrs, dv[r], (uint32_t)st * 16u, base + dd[r]);
        else dma_lds_ring<4, kNT>(zrs, dv[r], (uint32_t)(((128 * st) >> lg) * 4), base + dd[r]);
      }
    }
  };
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    sfor<0, R>([&](auto rc) { issue_piece(rc, st, buf); });
  };

  // bias of this lane's column (unconditional load: see gemm_sf.hip)
  const int ncol = n_blk + 32 * cw + r32;
  const uint16_t* bsrc = bias != nullptr ? bias : reinterpret_cast<const uint16_t*>(sz);
  const float bsf = bf16_to_f32(bsrc[ncol < N ? ncol : N - 1]);

  f32x16_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int wrow = 32 * cw + r32;  // this lane's W row in the images
  // compute(buf, iss, st, ibuf): one step's MFMAs from stage buf; with IL and iss, stage st's
  // DMA pieces into ibuf are issued between its k sub-steps (not all ahead of the MFMAs)
  auto compute = [&](int buf, auto iss, int st, int ibuf) __attribute__((always_inline)) {
    constexpr bool ISS = decltype(iss)::value;
    if constexpr (ISS && !IL) issue(st, ibuf);
    const uint4* img = lds + buf * (STAGE / 16);
    constexpr int KS = 8 / KH;  // MFMA k sub-steps of this wave
    const int ks0 = KH == 2 ? 4 * kh : 0;
    uint32_t wd[8];
    float sf[2], cf[2];
#pragma unroll
    for (int u = 0; u < 2 / KH; ++u) {  // the nibble granules / (scale, zero) words this wave uses
      const int gi = KH == 2 ? kh : u;
      const uint4 b = img[XB / 16 + wrow * 4 + wpos(wrow, 2 * h + gi)];
      wd[4 * u] = b.x;
      wd[4 * u + 1] = b.y;
      wd[4 * u + 2] = b.z;
      wd[4 * u + 3] = b.w;
      uint32_t zw;
      if constexpr (Z16) {
        const uint4 zq = img[(XB + WB) / 16 + wrow];
        zw = h == 0 ? (gi == 0 ? zq.x : zq.y) : (gi == 0 ? zq.z : zq.w);
      } else {
        zw = reinterpret_cast<const uint32_t*>(img)[(XB + WB) / 4 + wrow * 4 + zpos(wrow, 2 * h + gi)];
      }
      sf[u] = bf16lo_to_f32(zw);
      cf[u] = bf16hi_to_f32(zw) - 8.f * sf[u];
    }
    // A fragments of ks and ks + 1 in flight while ks's MFMAs run (TAO_SF32_ABUF 1, variant
    // builds: one buffer, each sub-step's fragments read at its top)
    constexpr int AB = TAO_SF32_ABUF;
    bf16x8_t af[AB][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = 32 * mt + r32;
      af[0][mt] = __builtin_bit_cast(bf16x8_t, img[m * 16 + xpos(m, 8 * h + ks0)]);
    }
    sfor<0, KS>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (AB == 1) {
        if (k > 0) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int m = 32 * mt + r32;
            af[0][mt] = __builtin_bit_cast(bf16x8_t, img[m * 16 + xpos(m, 8 * h + ks0 + k)]);
          }
        }
      } else if (k + 1 < KS) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int m = 32 * mt + r32;
          af[(k + 1) & 1][mt] =
              __builtin_bit_cast(bf16x8_t, img[m * 16 + xpos(m, 8 * h + ks0 + k + 1)]);
        }
      }
      const bf16x8_t bf = deq8s(wd[k], sf[k >> 2], cf[k >> 2]);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[k & (AB - 1)][mt], bf, acc[mt], 0, 0, 0);
      if constexpr (ISS && IL)  // DMA pieces r with r KS / R == k after sub-step k's MFMAs
        sfor<0, R>([&](auto rc) {
          constexpr int r = decltype(rc)::value;
          if constexpr (r * KS / R == k) issue_piece(rc, st, ibuf);
        });
    });
  };

  // this wave's DMAs of the step landed (its own piece count)
  auto wait_own = [&](int ahead) __attribute__((always_inline)) {
    if constexpr (RFULL == DW) {
      wait_ahead<R>(ahead);
    } else {
      if (dwv < RFULL) wait_ahead<R>(ahead);
      else wait_ahead<R - 1>(ahead);
    }
  };
#define SF32_TS(i) \
  do {             \
  } while (0)
  if constexpr (LDW > 0) {
    if (loader) {
#pragma unroll
      for (int p = 0; p < NS - 1; ++p)
        if (p < J) issue(s0 + p, p);
      for (int j = 0; j < J; ++j) {
        const int ahead = J - 1 - j < NS - 2 ? J - 1 - j : NS - 2;
        SF32_TS(0);
        wait_own(ahead);  // this loader's pieces of stage j landed
        SF32_TS(1);
        barrier_lgkm();   // ... every loader's; the compute waves are done with stage j - 1
        SF32_TS(2);
        if (j + NS - 1 < J) issue(s0 + j + NS - 1, (j + NS - 1) % NS);
        SF32_TS(3);
      }
    } else {
      for (int j = 0; j < J; ++j) {
        SF32_TS(0);
        SF32_TS(1);
        barrier_lgkm();
        SF32_TS(2);
        compute(j % NS, std::false_type{}, 0, 0);
        SF32_TS(3);
      }
    }
  }
  if constexpr (LDW == 0) {
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < J) issue(s0 + p, p);
  const int jiss = J - (NS - 1);  // steps that issue a stage ahead
  int j = 0;
  for (; j < jiss; ++j) {
    SF32_TS(0);
    wait_own(NS - 2);
    SF32_TS(1);
    barrier_lgkm();
    SF32_TS(2);
    compute(j % NS, std::true_type{}, s0 + j + NS - 1, (j + NS - 1) % NS);
    SF32_TS(3);
  }
  for (; j < J; ++j) {
    const int ahead = J - 1 - j < NS - 2 ? J - 1 - j : NS - 2;
    SF32_TS(0);
    wait_own(ahead);
    SF32_TS(1);
    barrier_lgkm();
    SF32_TS(2);
    compute(j % NS, std::false_type{}, 0, 0);
    SF32_TS(3);
  }
  }  // LDW == 0
#undef SF32_TS
  barrier_lgkm();
  if constexpr (KH == 2) {  // k half 1's accumulators into k half 0's, through LDS
    uint4* red = lds + (cw * 4 * 64 + lane) * 4;  // [cw][t][lane][16 floats]
    if (kh == 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          red[t * 64 * 4 + q] = make_uint4(__float_as_uint(acc[t][4 * q]), __float_as_uint(acc[t][4 * q + 1]),
                                           __float_as_uint(acc[t][4 * q + 2]), __float_as_uint(acc[t][4 * q + 3]));
    }
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v = red[t * 64 * 4 + q];
          acc[t][4 * q] += __uint_as_float(v.x);
          acc[t][4 * q + 1] += __uint_as_float(v.y);
          acc[t][4 * q + 2] += __uint_as_float(v.z);
          acc[t][4 * q + 3] += __uint_as_float(v.w);
        }
    }
    __syncthreads();
  }
  const bool lead = kh == 0 && !loader;  // the waves holding the summed tile

  if (S > 1) {
    constexpr uint32_t kSlice = kBM * BN * 4;
    const unsigned tile = blockIdx.z * gridDim.x + blockIdx.x;
    const Rsrc srs = make_rsrc(reinterpret_cast<const uint8_t*>(slab) + (size_t)tile * (S - 1) * kSlice,
                               (uint32_t)(S - 1) * kSlice);
    const uint32_t lo = (uint32_t)((cw * 4 * 64 + lane) * 64);  // 4 x 64 B per lane
    unsigned* word = reinterpret_cast<unsigned*>(lds);
    if (!reducer) {
      if (lead)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bstore16<kSC1>(srs, lo + t * 64 * 64 + 16 * q, (uint32_t)z * kSlice,
                         make_uint4(__float_as_uint(acc[t][4 * q]), __float_as_uint(acc[t][4 * q + 1]),
                                    __float_as_uint(acc[t][4 * q + 2]),
                                    __float_as_uint(acc[t][4 * q + 3])));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (fenced & 1) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if ((fenced & 2) && z == 0) late_publisher_hold(&g_sf32_err);
        (void)__hip_atomic_fetch_add(&cnt[tile * cs], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (tid == 0) {
      unsigned ok = 1;
      SeamWait sw;
      while (__hip_atomic_load(&cnt[tile * cs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
             (unsigned)(S - 1)) {
        __builtin_amdgcn_s_sleep(1);
        if (sw.timed_out()) {
          ok = 0;
          (void)__hip_atomic_fetch_or(&g_sf32_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      // take the S-1 arrivals back off the ticket, timed out or not: once a late publisher's add
      // lands the ticket is 0 again for the next launch on this workspace (gemm_sf.hip's seam)
      (void)__hip_atomic_fetch_sub(&cnt[tile * cs], (unsigned)(S - 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      if (fenced & 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *word = ok;
    }
    __syncthreads();
    if (*word == 0) return;  // timed out: write nothing (uniform over the workgroup)
    if constexpr (LDW > 0 && KH == 2) {  // one accumulator tile at a time (the 170-VGPR cap of
      // 12 waves), the same additions in the same order as below
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x16_t st;
#pragma unroll
        for (int i = 0; i < 16; ++i) st[i] = 0.f;
        for (int zz = 0; zz < (lead ? S - 1 : 0); ++zz) {
          uint4 pt[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            pt[q] = bload16<kSC1>(srs, lo + t * 64 * 64 + 16 * q, (uint32_t)zz * kSlice);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            st[4 * q] += __uint_as_float(pt[q].x);
            st[4 * q + 1] += __uint_as_float(pt[q].y);
            st[4 * q + 2] += __uint_as_float(pt[q].z);
            st[4 * q + 3] += __uint_as_float(pt[q].w);
          }
        }
        acc[t] = st + acc[t];
      }
      __syncthreads();  // `word` lives where the output image goes
    } else {
    f32x16_t sum[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) sum[t][i] = 0.f;
    for (int zz = 0; zz < (lead ? S - 1 : 0); ++zz) {
      uint4 part[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          part[t][q] = bload16<kSC1>(srs, lo + t * 64 * 64 + 16 * q, (uint32_t)zz * kSlice);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sum[t][4 * q] += __uint_as_float(part[t][q].x);
          sum[t][4 * q + 1] += __uint_as_float(part[t][q].y);
          sum[t][4 * q + 2] += __uint_as_float(part[t][q].z);
          sum[t][4 * q + 3] += __uint_as_float(part[t][q].w);
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = sum[t] + acc[t];
    __syncthreads();  // `word` lives where the output image goes
    }
  }

  // epilogue: bf16 tile [128][BN] through LDS, rows out in 16-B pieces. C map (32x32x16): column
  // lane & 31, row (i & 3) + 8 (i >> 2) + 4 h of accumulator tile t (rows 32 t ..)
  uint16_t* out = reinterpret_cast<uint16_t*>(lds);
  if (lead)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
      float v = round_bf16(acc[t][i]);
      if (bias != nullptr) v = round_bf16(v + bsf);
      out[r * BN + 32 * cw + r32] = f32_to_bf16(v);
    }
  __syncthreads();
  if (epi == 1) {  // SwiGLU over interleaved (gate, up) columns: y [M][N / 2]
    constexpr int OPR = BN / 16;
    const int N2 = N >> 1;
    const bool full2 = n_blk + BN <= N && (N2 & 7) == 0 && ((uintptr_t)y & 15) == 0;
    for (int c = tid; c < kBM * OPR; c += NWT * 64) {
      const int r = c / OPR, cc = c % OPR;
      const int m = m_blk + r;
      if (m >= M) continue;
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
    return;
  }
  constexpr int CPR = BN / 8;
  const bool full = n_blk + BN <= N && (N & 7) == 0 && ((uintptr_t)y & 15) == 0;
  for (int c = tid; c < kBM * CPR; c += NWT * 64) {
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
}

}  // namespace

// bn 64 (2 waves), 128 (4 waves) or 256 (8 waves, 2 per SIMD); splits S; stages 2-3; a_steps = 128-k steps per publisher
int sf32_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int lg,
              const uint16_t* bias, uint16_t* y, int M, int N, int K, int bn, int splits,
              int stages, int a_steps, hipStream_t stream, int epi, int kh) {
  const int nsteps = K / 128;
  if (splits > nsteps) splits = nsteps;
  if (splits < 1) splits = 1;
  if (a_steps <= 0 || a_steps * (splits - 1) >= nsteps) a_steps = nsteps / splits;
  const dim3 grid((unsigned)((N + bn - 1) / bn), (unsigned)splits, (unsigned)((M + kBM - 1) / kBM));
  f32x16_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (splits > 1) {
    void* w = nullptr;
    const size_t tiles = (size_t)grid.x * grid.z;
    const int rc = split_workspace(stream, tiles * (splits - 1) * kBM * bn * 4,
                                   tiles * tuning().cnt_stride, &w, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<f32x16_t*>(w);
  }
  const int fenced = tuning().splitk_fenced | (tuning().sf_late_pub ? 2 : 0);
  auto go1 = [&](auto kern, int threads) {
    launch(kern, grid, dim3(threads), 0, stream, x, packed, reinterpret_cast<const uint32_t*>(sz),
           lg, bias, y, M, N, K, a_steps, slab, cnt, fenced, tuning().cnt_stride, epi);
  };
  // Z16 at one wave per column group only: with k halves (8 waves, 42 pieces, uneven per wave)
  // it measured 4% slower, at one wave 2-4% faster (profiles/r4_sf32_z16.jsonl)
  const bool z16 = lg == 5 && TAO_SF32_Z16 != 0 && kh != 2;
#define SF32_GO(WV, NS, KH)                                            \
  (z16 ? go1(gemm_sf32_int4_kernel<WV, NS, KH, true>, WV * KH * 64) \
       : go1(gemm_sf32_int4_kernel<WV, NS, KH, false>, WV * KH * 64))
  // dedicated loader waves (one per SIMD): tao_tune_gemm_sf_loaders 2 = on, 1 = off, 0 = built-in
  // (on for 128-column tiles at 3 stages: w1||w3 28672x4096 M = 128 47.4-48.5 -> 39.6 us,
  // 10240x8192 S = 2 48.9 -> 48.7; profiles/r5e_sf32_loaders.jsonl)
  const int ldm = tuning().sf_loaders == 3 ? 2 : tuning().sf_loaders;  // (8 waves: 16x16 only)
  // (k halves + loaders, 12 waves: 70B's 10240x8192 49.4 -> 45.4 us; w1||w3 42.6 -> 44.8, so the
  // one-compute-wave form stays there: profiles/r5g_ab_kh2_loaders.jsonl)
  const bool loaders = (kh == 1 && ((ldm == 2 && (bn == 128 || bn == 64)) ||
                                    (ldm == 0 && bn == 128 && stages == 3))) ||
                       (kh == 2 && bn == 128 && (ldm == 2 || (ldm == 0 && stages == 3)));
  if (loaders) {
    // the loader-wave kernels are instantiated at 3 stages only: a forced loader run at another
    // stage count is refused rather than silently measured at 3
    if (stages != 3)
      return set_error(TAO_ERR_UNSUPPORTED, "gemm_sf32: loader waves need 3 stages, got %d", stages);
    if (kh == 2) {  // two compute waves per column group (k halves) + 4 loader waves
      if (z16) go1(gemm_sf32_int4_kernel<4, 3, 2, true, 4>, 12 * 64);
      else go1(gemm_sf32_int4_kernel<4, 3, 2, false, 4>, 12 * 64);
    } else if (bn == 128) {
      if (z16) go1(gemm_sf32_int4_kernel<4, 3, 1, true, 4>, 8 * 64);
      else go1(gemm_sf32_int4_kernel<4, 3, 1, false, 4>, 8 * 64);
    } else {
      if (z16) go1(gemm_sf32_int4_kernel<2, 3, 1, true, 2>, 4 * 64);
      else go1(gemm_sf32_int4_kernel<2, 3, 1, false, 2>, 4 * 64);
    }
    return check_launch("gemm_sf32_int4_kernel");
  }
  if (bn == 256) {
    if (stages == 2) SF32_GO(8, 2, 1);
    else SF32_GO(8, 3, 1);
  } else if (bn == 128 && kh == 2) {
    if (stages == 2) SF32_GO(4, 2, 2);
    else SF32_GO(4, 3, 2);
  } else if (bn == 128) {
    if (stages == 2) SF32_GO(4, 2, 1);
    else SF32_GO(4, 3, 1);
  } else if (bn == 64) {
    if (stages == 2) SF32_GO(2, 2, 1);
    else SF32_GO(2, 3, 1);
  } else {
    return set_error(TAO_ERR_INVALID_ARGUMENT, "gemm_sf32: bn must be 64, 128 or 256 (got %d)", bn);
  }
#undef SF32_GO
  return check_launch("gemm_sf32_int4_kernel");
}


int sf32_status(unsigned* bits) {
  unsigned v = 0, zero = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_sf32_err), sizeof(v)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_sf32_err), &zero, sizeof(zero)) != hipSuccess)
    return set_error(TAO_ERR_HIP, "gemm_sf32 status: symbol copy failed");
  *bits |= v;
  return TAO_OK;
}

}  // namespace tao
