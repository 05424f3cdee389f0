// Prefill GEMM for the quantized linears at M ~ 64..256 ("stream" tile):
//   y[M][N] = epilogue(x[M][K] . W[N][K]^T), int4 weight-only (bf16 x) and int8 dynamic (int8 x).
//
// Built on what the round-3 streaming probes measured (experiments/probe_stream*.hip, DESIGN
// §4.2c): an unsplit (S = 1) tile whose data movement runs as a per-step LDS ring with a
// workgroup barrier every step streams at only ~43 GB/s per CU (8.5-10 µs for config 3's bytes
// with no math at all), whatever the row run length; the SAME bytes streamed by every wave into a
// wave-private LDS-DMA ring with no barrier take 3.3 µs for the weights alone (5.1 TB/s). Split-K
// variants pay a 3-5 µs slab hand-off tail (profiles/r3_tile_stamps.jsonl). So:
//
//   * one workgroup of 4 waves per 32 x 64 output tile, the whole K (no split, no hand-off);
//     wave w owns output columns 16 w .. 16 w + 15 and all 32 rows (two 16-row blocks);
//   * the x tile is shared: it arrives by LDS-DMA in "phases" of 1 KiB per row (1024 int8 k or
//     512 bf16 k), double-buffered (2 x 32 KiB), one workgroup barrier per phase (4 per config-3
//     launch instead of one per 256 k);
//   * each wave streams ITS OWN 16 weight rows (and, int4, their (scale, zero) words) by LDS-DMA
//     into a private ring of D chunks, D - 1 chunks ahead, with counted vmcnt waits and no
//     barrier: the weight stream never waits for another wave;
//   * every LDS image is XOR-swizzled through the DMA source addresses (LDS-DMA writes
//     lane-linearly, so lane L fetches the chunk that belongs at slot L) so that the fragment
//     reads (ds_read_b128) hit 16 distinct bank groups per lane group;
//   * fragments: int8 dynamic v_mfma_i32_16x16x64_i8 (exact int32); int4 v_mfma_f32_16x16x32_bf16
//     on B = bf16(fma(q, s, z - 8 s)) (gemm_mfma.hip's Int4WO numerics), a lane's 16-B nibble
//     read being one 32-k group = one (scale, zero) word and four MFMAs' B operands.
// Epilogues as gemm_mfma.hip: int4 bf16(acc) (+ bias); int8 dynamic bf16(bf16(bf16(acc) * xs) * ws)
// (+ bias) -- kernel/intmm.py:133-137, plain_layout.py:301-315 (bit-exact).
// Replaces aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104) and int_scaled_matmul
// (plain_layout.py:294-315) at prefill shapes.
#include "tao_common.h"

// Timing-only variant builds (experiments/stream_debug.sh; never the shipped library): 1 no
// fragment reads / MFMAs, 2 no weight DMA, 3 no x (and scale/zero) DMA, 4 no DMA at all.
// Results are wrong in every variant.
#ifndef TAO_STREAM_DEBUG
#define TAO_STREAM_DEBUG 0
#endif

namespace tao {
namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kBM = 32, kBN = 64, kNW = 4;
constexpr int kPhaseRow = 1024;              // x bytes per row per phase
constexpr int kXBuf = kBM * kPhaseRow;       // one x phase buffer (32 KiB)
constexpr int kXI = kBM / kNW;               // x DMA instructions per wave per phase (1 row each)

// LDS-DMA of 64 lanes x SIZE bytes from per-lane buffer offsets into LDS at the wave-uniform `dst`
// + lane * SIZE. Inline asm (gemm_tile.hip's reasoning): hipcc cannot tell which LDS a pending
// intrinsic DMA writes and would wait vmcnt(0) before every ds_read; the waits here are counted
// by hand. M0 is saved and restored around the load.
template <int SIZE, bool NT>
__device__ __forceinline__ void dma(Rsrc r, uint32_t voff, uint32_t soff, const void* dst) {
  static_assert(SIZE == 16 || SIZE == 4, "dma: 16 or 4 bytes per lane");
  // wave-uniform by construction; readfirstlane keeps it in an SGPR for M0
  const uint32_t a =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)(const_cast<void*>(dst)));
  uint32_t keep;
  if constexpr (SIZE == 16 && NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(a), "v"(voff), "s"(r), "s"(soff) : "memory");
  else if constexpr (SIZE == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(a), "v"(voff), "s"(r), "s"(soff) : "memory");
  else if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dword %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(a), "v"(voff), "s"(r), "s"(soff) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dword %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(a), "v"(voff), "s"(r), "s"(soff) : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// vmcnt(n) for a wave-uniform n that the callers keep within {0, 1, ..., 63}: one scalar branch
// tree, each leaf an immediate wait (the counts vary only at the ends of the k loop).
template <int LO, int HI>
__device__ __forceinline__ void vm_wait_dyn(int n) {
  if constexpr (LO == HI) {
    vm_wait<LO>();
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID)
      vm_wait_dyn<LO, MID>(n);
    else
      vm_wait_dyn<MID + 1, HI>(n);
  }
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint4 lds16(const void* base, uint32_t byte_off) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(base) + byte_off);
}

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// ---- int8 dynamic activation -----------------------------------------------------------------
// x int8 [M][K]; W int8 [N][K]. Phase = 1024 k; W chunk = 256 k: 16 rows x 256 B per wave (4 DMA
// instructions of 4 rows x 256 B), slot s of row r holds 16-B chunk s ^ r. x phase row r: slot s
// holds chunk (s & ~15) | ((s & 15) ^ r). Fragment of k-block kb (64 k), lane (r = l % 16, q = l / 16):
// bytes 64 kb + 16 q .. + 15 of row r, for A (x) and B (W) alike.
struct SInt8Dyn {
  static constexpr int kPK = 1024;          // k per phase
  static constexpr int kCK = 256;           // k per weight chunk
  static constexpr int kCPP = kPK / kCK;    // chunks per phase
  static constexpr int kD = kCPP + 1;       // ring depth (chunks)
  static constexpr int kWI = 4;             // DMA instructions per chunk per wave
  static constexpr int kChunk = 16 * 256;   // ring slot bytes
  static constexpr int kZI = 0;             // (scale, zero) instructions per phase
  static constexpr int kZBuf = 0;
  typedef i32x4_t Acc;
  const uint8_t* w;
  const uint16_t* wscale;  // [N]
  const uint16_t* xscale;  // [M]
  int K;
  __device__ __forceinline__ uint32_t x_swz(int r) const { return (uint32_t)r; }
  // weight chunk c of this wave's rows (n_w = first row) into ring slot `dst`
  __device__ __forceinline__ void issue_w(const Rsrc& wr, int n_w, int c, int lane,
                                          uint8_t* dst) const {
#pragma unroll
    for (int i = 0; i < kWI; ++i) {
      const int row = 4 * i + (lane >> 4), s = lane & 15;
      const uint32_t voff = (uint32_t)(n_w + row) * (uint32_t)K + 16u * (uint32_t)(s ^ row);
      dma<16, true>(wr, voff, (uint32_t)c * 256u, dst + i * 1024);
    }
  }
  __device__ __forceinline__ void issue_z(const Rsrc&, int, int, int, uint8_t*) const {}
  // one chunk: 4 k-blocks x 2 row blocks
  __device__ __forceinline__ void compute(const uint8_t* ring, const uint8_t*, const uint8_t* xb,
                                          int cin, int lane, Acc acc[2]) const {
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int ch = 4 * kb + q;
      const uint4 b = lds16(ring, (uint32_t)(r * 256 + 16 * (ch ^ r)));
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int xr = 16 * rb + r;
        const uint4 a = lds16(xb, (uint32_t)(xr * kPhaseRow + 16 * (16 * cin + (ch ^ r))));
        acc[rb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a),
                                                        __builtin_bit_cast(i32x4_t, b), acc[rb], 0,
                                                        0, 0);
      }
    }
  }
  static __device__ __forceinline__ float epi(int acc, float xs, float ws) {
    const float v = round_bf16(round_bf16((float)acc) * xs);
    return round_bf16(v * ws);
  }
};

// ---- int4 weight-only ------------------------------------------------------------------------------
// x bf16 [M][K]; W row-stream nibbles [N][K/8] dwords; sz bf16 (scale, zero) [N][K/g].
// Phase = 512 k (1 KiB of x per row); W chunk = 128 k: 16 rows x 64 B per wave (one DMA
// instruction; slot s of row r holds 16-B chunk s ^ h(r), h from kH4, found by search for
// conflict-free reads), i.e. one k-group of 4 MFMAs: lane (r, q) reads the 32 nibbles k =
// 32 q .. 32 q + 31 of row r (one (scale, zero) word), dword j of them feeding MFMA j; the A operand
// of MFMA j is x[row][32 q + 8 j .. + 7] (chunk 4 q + j of the group's 64 B), so A and B pair the
// same k. x phase row r: slot s holds chunk (s & ~15) | ((s & 15) ^ f(r)), f swapping the two bit
// pairs of r (conflict-free for this read order). (scale, zero) words of a phase and wave: dword
// gg * 16 + r for group gg of the phase, row r (one DMA instruction of 64 dwords per 4 groups).
struct SInt4 {
  static constexpr int kPK = 512;
  static constexpr int kCK = 128;
  static constexpr int kCPP = kPK / kCK;
  static constexpr int kD = 2 * kCPP;       // chunks are small: run further ahead
  static constexpr int kWI = 1;
  static constexpr int kChunk = 16 * 64;
  static constexpr int kH4 = 0x20e30ecd;    // h(r) = (kH4 >> 2r) & 3
  typedef f32x4_t Acc;
  const uint32_t* w;
  const uint32_t* sz;
  int K, gshift;                            // g = 32 << gshift
  int kZI;                                  // (scale, zero) DMA instructions per phase: max(1, 4 >> gshift)
  static constexpr int kZBuf = 4 * 256;     // per wave and phase buffer (4 instructions max)
  __device__ __forceinline__ uint32_t x_swz(int r) const {
    return (uint32_t)(((r & 3) << 2) | (r >> 2));
  }
  __device__ __forceinline__ void issue_w(const Rsrc& wr, int n_w, int c, int lane,
                                          uint8_t* dst) const {
    const int row = lane >> 2, s = lane & 3;
    const int h = (kH4 >> (2 * row)) & 3;
    const uint32_t voff = (uint32_t)(n_w + row) * (uint32_t)(K >> 1) + 16u * (uint32_t)(s ^ h);
    dma<16, true>(wr, voff, (uint32_t)c * 64u, dst);
  }
  // phase p's (scale, zero) words of this wave's 16 rows: group gg of the phase at dword gg * 16 + r
  __device__ __forceinline__ void issue_z(const Rsrc& zr, int n_w, int p, int lane,
                                          uint8_t* dst) const {
    const int gpp = 16 >> gshift;             // groups per phase (g = 32 .. 256: 16 .. 2)
    const uint32_t zrow = (uint32_t)(K >> (5 + gshift));
    for (int i = 0; i < kZI; ++i) {
      const int d = 64 * i + lane, gg = d >> 4, r = d & 15;
      const int g2 = gg < gpp ? gg : gpp - 1;  // lanes past the phase's groups: duplicates
      const uint32_t voff = ((uint32_t)(n_w + r) * zrow + (uint32_t)g2) * 4u;
      dma<4, true>(zr, voff, (uint32_t)(p * gpp) * 4u, dst + i * 256);
    }
  }
  static __device__ __forceinline__ uint4 dq8(uint32_t w, float s, float zc) {
    // row-stream nibble order -> 8 bf16 in k order: bf16(fma(q, s, z - 8 s)); a nibble byte b
    // read as OCP e4m3 is b / 512 exactly (gemm_mfma.hip's Int4WO conversion)
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
  // one chunk = one 128-k group of the phase (cin = its index 0..3): 4 MFMAs x 2 row blocks
  __device__ __forceinline__ void compute(const uint8_t* ring, const uint8_t* zb, const uint8_t* xb,
                                          int cin, int lane, Acc acc[2]) const {
    const int r = lane & 15, q = lane >> 4;
    const int h = (kH4 >> (2 * r)) & 3;
    const uint4 nib = lds16(ring, (uint32_t)(r * 64 + 16 * (q ^ h)));
    // group of k = 128 cin + 32 q within the phase
    const int gg = (4 * cin + q) >> gshift;
    const uint32_t szw = *reinterpret_cast<const uint32_t*>(zb + 4 * (gg * 16 + r));
    const float s = bf16lo_to_f32(szw);
    const float zc = bf16hi_to_f32(szw) - 8.f * s;  // q * s + zc == (q - 8) * s + z
    const uint32_t d4[4] = {nib.x, nib.y, nib.z, nib.w};
    const uint32_t fx = x_swz(r);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 b = dq8(d4[j], s, zc);
      const uint32_t slot = 16u * (uint32_t)cin + ((uint32_t)(4 * q + j) ^ fx);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const uint4 a = lds16(xb, (uint32_t)((16 * rb + r) * kPhaseRow) + 16u * slot);
        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                          __builtin_bit_cast(bf16x8_t, b),
                                                          acc[rb], 0, 0, 0);
      }
    }
  }
  static __device__ __forceinline__ float epi(float acc, float, float) { return round_bf16(acc); }
};

template <class P>
struct StreamLds {
  static constexpr int kX = 2 * kXBuf;                  // double-buffered x phases
  static constexpr int kZ = 2 * kNW * P::kZBuf;         // double-buffered (scale, zero) per wave
  static constexpr int kW = kNW * P::kD * P::kChunk;    // per-wave weight rings
  static constexpr int kTotal = kX + kZ + kW;
  static_assert(kTotal <= 160 * 1024, "LDS budget");
};

// grid (N / 64, ceil(M / 32)), 256 threads. Requires N % 64 == 0, K % P::kPK == 0.
template <class P, bool kRowF, bool kColF>
__global__ __launch_bounds__(256) void gemm_stream_kernel(
    const uint8_t* __restrict__ x, P pol, const uint16_t* __restrict__ rowf,
    const uint16_t* __restrict__ colf, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int rotate) {
  typedef typename P::Acc Acc;
  typedef StreamLds<P> L;
  __shared__ __attribute__((aligned(16))) uint8_t lds[L::kTotal];
  uint8_t* const xs0 = lds;
  uint8_t* const zs0 = lds + L::kX;
  uint8_t* const ws0 = lds + L::kX + L::kZ;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * kBN, m0 = blockIdx.y * kBM;
  const int n_w = n0 + 16 * wave;
  const int nphase = K / P::kPK;
  const int nchunk = nphase * P::kCPP;
  // rotate 1: the workgroup walks the phases from a start set by its M tile (rotate 2: and its
  // N tile), so that the workgroups sharing a weight (x) tile do not all miss on the same lines
  // at once. Only the memory offsets rotate; LDS slots and the k order per phase are unchanged.
  const int rot = rotate == 0 ? 0
                  : (int)((blockIdx.y * (unsigned)((nphase + 3) / 4) +
                           (rotate == 2 ? blockIdx.x : 0u)) % (unsigned)nphase);
  auto phys_p = [&](int p) __attribute__((always_inline)) {
    const int q = p + rot;
    return q >= nphase ? q - nphase : q;
  };
  constexpr int XB = P::kPK == 1024 ? 1 : 2;  // x bytes per element
  const uint32_t xrow = (uint32_t)K * XB;

  // epilogue operands first (their loads retire before every DMA issued after them)
  const int r = lane & 15, q = lane >> 4;
  const int col = n_w + r;
  float cf = 1.f, bv = 0.f, rf[2][4];
  if constexpr (kColF) cf = bf16_to_f32(colf[col]);
  if (bias != nullptr) bv = bf16_to_f32(bias[col]);
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 16 * rb + 4 * q + i;
      rf[rb][i] = kRowF ? bf16_to_f32(rowf[m < M ? m : M - 1]) : 1.f;
    }

  const Rsrc xr = make_rsrc(x, (uint32_t)M * xrow);
  Rsrc wr, zr;
  if constexpr (P::kPK == 1024) {
    wr = make_rsrc(pol.w, (uint32_t)N * (uint32_t)K);
    zr = wr;
  } else {
    wr = make_rsrc(pol.w, (uint32_t)N * (uint32_t)(K >> 1));
    zr = make_rsrc(pol.sz, (uint32_t)N * (uint32_t)(K >> (5 + pol.gshift)) * 4u);
  }
  int zi = 0;
  if constexpr (P::kPK != 1024) zi = pol.kZI;

  // x phase p: this wave's 8 rows (one DMA instruction of 1 KiB each), swizzled slots
  auto issue_x = [&](int p) __attribute__((always_inline)) {
    uint8_t* dst = xs0 + (p & 1) * kXBuf;
    if (TAO_STREAM_DEBUG == 3 || TAO_STREAM_DEBUG == 4) return;
#pragma unroll
    for (int i = 0; i < kXI; ++i) {
      const int row = wave * kXI + i;
      const int m = m0 + row < M ? m0 + row : M - 1;
      const uint32_t ch = ((uint32_t)lane & ~15u) | (((uint32_t)lane & 15u) ^ pol.x_swz(row & 15));
      dma<16, false>(xr, (uint32_t)m * xrow + 16u * ch, (uint32_t)phys_p(p) * kPhaseRow,
                     dst + row * kPhaseRow);
    }
    if constexpr (P::kPK != 1024)
      pol.issue_z(zr, n_w, phys_p(p), lane, zs0 + ((p & 1) * kNW + wave) * P::kZBuf);
  };
  auto issue_chunk = [&](int c) __attribute__((always_inline)) {
    if (TAO_STREAM_DEBUG == 2 || TAO_STREAM_DEBUG == 4) return;
    const int pc = phys_p(c / P::kCPP) * P::kCPP + c % P::kCPP;  // the chunk's memory offset
    pol.issue_w(wr, n_w, pc, lane, ws0 + (wave * P::kD + c % P::kD) * P::kChunk);
  };

  Acc acc[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) acc[rb] = Acc{0, 0, 0, 0};

  // prologue: x phase 0, then weight chunks 0 .. D - 2
  issue_x(0);
  const int pre = P::kD - 1 < nchunk ? P::kD - 1 : nchunk;
  for (int c = 0; c < pre; ++c) issue_chunk(c);
  const int xzi = kXI + zi;  // DMA instructions of one x phase (+ its scale/zero words)

  for (int p = 0; p < nphase; ++p) {
    // x phase p landed for this wave: the instructions issued after it are the weight chunks
    // issued since (prologue: `pre`; later: those of phase p - 1's chunks that were issued)
    {
      int after;
      if (p == 0) {
        after = pre * P::kWI;
      } else {
        const int c_first = P::kCPP * (p - 1);
        int n_iss = nchunk - (P::kD - 1) - c_first;  // chunks c in phase p - 1 with c + D - 1 < nchunk
        n_iss = n_iss < 0 ? 0 : (n_iss > P::kCPP ? P::kCPP : n_iss);
        after = n_iss * P::kWI;
      }
      vm_wait_dyn<0, 31>(after);
    }
    lds_barrier();  // every wave's part of x phase p landed; phase p - 1's buffer is free
    const bool more = p + 1 < nphase;
    if (more) issue_x(p + 1);
    const uint8_t* xb = xs0 + (p & 1) * kXBuf;
    const uint8_t* zb = zs0 + ((p & 1) * kNW + wave) * P::kZBuf;
#pragma unroll
    for (int cin = 0; cin < P::kCPP; ++cin) {
      const int c = p * P::kCPP + cin;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring slot (c - 1) % D read out
      const bool iss = c + P::kD - 1 < nchunk;
      if (iss) issue_chunk(c + P::kD - 1);
      // in flight after chunk c: the chunks c + 1 .. min(c + D - 1, nchunk - 1), and x phase
      // p + 1 (issued after every chunk of phase p: D - 1 >= kCPP)
      const int last = c + P::kD - 1 < nchunk ? c + P::kD - 1 : nchunk - 1;
      vm_wait_dyn<0, 31>((last - c) * P::kWI + (more ? xzi : 0));
      if (TAO_STREAM_DEBUG != 1) pol.compute(ws0 + (wave * P::kD + c % P::kD) * P::kChunk, zb, xb, cin, lane, acc);
    }
  }

  // epilogue: lane (col = n_w + r, rows 4 q + i of each 16-row block)
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 16 * rb + 4 * q + i;
      if (m < M) {
        float v = P::epi(acc[rb][i], rf[rb][i], cf);
        if (bias != nullptr) v = round_bf16(v + bv);
        y[(size_t)m * N + col] = f32_to_bf16(v);
      }
    }
}

}  // namespace

// ---- routing and launchers ------------------------------------------------------------------
// path 0 int4, 2 int8 dynamic. Shapes the kernel covers: N % 64 == 0, K % phase == 0, operands
// below 4 GiB. Auto routing (tuning().gemm_stream == 0) per profiles/r3_ab_stream.jsonl.
bool use_stream(int path, int64_t M, int64_t N, int64_t K, int64_t group_size) {
  const int mode = tuning().gemm_stream;
  if (mode == 1) return false;
  if (path != 0 && path != 2) return false;
  const int64_t pk = path == 2 ? SInt8Dyn::kPK : SInt4::kPK;
  if (N % kBN != 0 || K % pk != 0 || M < 1 || N * K >= (int64_t(1) << 32) ||
      M * K * 2 >= (int64_t(1) << 32))
    return false;
  if (path == 0 && (group_size < 32 || group_size > 256 || (group_size & (group_size - 1))))
    return false;
  if (mode == 2) return true;
  const Tuning& t = tuning();
  if (t.bm || t.kg || t.splits || t.gemm_nw || t.int4_mfma32 || t.gemm_algo || t.gemm_tile)
    return false;
  return false;  // auto routing: set from the A/B once the GPU parity suite is green
}

int stream_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int gshift,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  TAO_CHECK_ARG(N % kBN == 0 && K % SInt4::kPK == 0 && gshift >= 0 && gshift <= 3,
                "stream GEMM: N %% 64, K %% 512 and g in {32..256} required");
  SInt4 pol;
  pol.w = packed;
  pol.sz = reinterpret_cast<const uint32_t*>(sz);
  pol.K = K;
  pol.gshift = gshift;
  pol.kZI = (4 >> gshift) > 0 ? (4 >> gshift) : 1;
  const dim3 grid((unsigned)(N / kBN), (unsigned)((M + kBM - 1) / kBM));
  launch(gemm_stream_kernel<SInt4, false, false>, grid, dim3(256), 0, stream,
         reinterpret_cast<const uint8_t*>(x), pol, (const uint16_t*)nullptr,
         (const uint16_t*)nullptr, bias, y, M, N, K, tuning().gemm_stream_rot);
  return check_launch("gemm_stream_kernel<int4>");
}

int stream_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
                   const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream) {
  TAO_CHECK_ARG(N % kBN == 0 && K % SInt8Dyn::kPK == 0,
                "stream GEMM: N %% 64 and K %% 1024 required");
  SInt8Dyn pol;
  pol.w = reinterpret_cast<const uint8_t*>(wq);
  pol.wscale = ws;
  pol.xscale = xs;
  pol.K = K;
  const dim3 grid((unsigned)(N / kBN), (unsigned)((M + kBM - 1) / kBM));
  launch(gemm_stream_kernel<SInt8Dyn, true, true>, grid, dim3(256), 0, stream,
         reinterpret_cast<const uint8_t*>(xq), pol, xs, ws, bias, y, M, N, K,
         tuning().gemm_stream_rot);
  return check_launch("gemm_stream_kernel<int8dyn>");
}

}  // namespace tao

extern "C" int tao_tune_gemm_stream(int mode) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 5 && mode != 3,
                "tune: gemm stream mode must be 0 (auto), 1 (off), 2 (on), 4 (on, phases rotated by "
                "M tile) or 5 (on, rotated by M and N tile)");
  tao::tuning().gemm_stream = mode <= 2 ? mode : 2;
  tao::tuning().gemm_stream_rot = mode <= 2 ? 0 : mode - 3;
  return TAO_OK;
}
