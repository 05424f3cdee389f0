// Skinny GEMM on MFMA for the quantized linears at M > 4 (prefill / batched decode):
//   y[M][N] = epilogue( x[M][K] . W[N][K]^T )
// three weight/activation formats share one kernel template:
//   Int4WO  : bf16 x, int4 group-quant W (gfx950 row-stream layout), v_mfma_f32_16x16x32_bf16
//   Int8WO  : bf16 x, int8 per-channel W,                            v_mfma_f32_16x16x32_bf16
//   Int8Dyn : int8 x (per-token scale), int8 W (per-channel scale),   v_mfma_i32_16x16x64_i8
// Replaces aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104), mm(x, w.to(bf16)) * s
// (plain_layout.py:256-266) and int_scaled_matmul + scales (plain_layout.py:294-315,
// kernel/intmm.py:108-143).
//
// Tile: 4 waves x 16 output columns (BN = 64) x BM rows per k-group; each wave owns 16 columns
// and all BM rows. K advances in macro-steps (256 bf16 k for int4, 128 bf16 k for int8-WO,
// 256 int8 k for int8-dyn) in which every weight load instruction reads full 128-B lines
// (8 rows x 128 B); a per-wave LDS stage regroups them into the MFMA B layout. The k order
// inside a step is permuted identically for A and B (policy slot(s, kq): the 16-B x slot
// MFMA s of lane l = (n = l & 15, kq = l >> 4) reads).
// x goes global -> registers (D-deep prefetch ring, T14) -> double-buffered, XOR-swizzled LDS
// image -> A fragments; one barrier per step. W goes straight to registers (read once per
// tile, dequantised in registers, reused for BM/16 MFMAs). K is split across k-groups inside
// the workgroup and across workgroups (split-K) so every SIMD holds several waves; the launch
// shape (BM, k-groups, slices) comes from measured sweeps (experiments/sweep_gemm.py).
#include <atomic>
#include <tuple>
#include <type_traits>

#include "tao_common.h"

// Experiment switch: ring depth override (experiments/gemm_depth.sh; 0 = the policy below).
#ifndef TAO_GEMM_DEPTH
#define TAO_GEMM_DEPTH 0
#endif

namespace tao {

int int4wo_gemv(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                int64_t group_size, hipStream_t stream);
int int4_check_linear_args(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                           uint16_t* y, int64_t M, int64_t N, int64_t K, int64_t group_size);
int int8wo_gemv(const uint16_t* x, const int8_t* w, const uint16_t* scale, const uint16_t* bias,
                uint16_t* y, int64_t M, int64_t N, int64_t K, hipStream_t stream);
// gemm_tile.hip: the weight-shared tile GEMM (4 waves split the rows, weights dequantised once per
// workgroup) and its routing rule
int tile_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int gshift,
              const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
              int splits);
int tile_int8wo(const uint16_t* x, const int8_t* w, const uint16_t* scale, const uint16_t* bias,
                uint16_t* y, int M, int N, int K, hipStream_t stream, int splits);
int tile_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
                 const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
                 int splits);
bool use_tile(int path, int64_t M, int64_t N, int64_t K);
// gemm_sf.hip: the single-fetch prefill GEMM (128-row tiles, LDS-DMA, fixed-reducer split-K)
bool use_sf(int path, int64_t M, int64_t N, int64_t K, int64_t group_size);
int sf_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
               const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream);
int sf_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int lg,
            const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
            int epi = 0);

namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBN = 64;

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

__device__ __forceinline__ bf16x8_t as_bf16x8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  u32x4_t v = {a, b, c, d};
  return __builtin_bit_cast(bf16x8_t, v);
}

// Per-wave weight stage of 16 rows x 8 16-B slots (Int4WO, Int8WO). A ds_*_b128 pass is 16
// lanes of 16 B: conflict-free iff the 16 slots land in 16 distinct 16-B bank groups (slot index
// mod 16). The write passes cover rows {2i, 2i+1} x 8 slots; the read passes cover rows 0..15 at
// one slot. Swizzling the slot by (row >> 1) & 7 serves both (the row's parity supplies bit 3);
// the previous row & 7 gave rows n and n + 8 the same bank group on every read pass
// (SQ_LDS_BANK_CONFLICT 1.24-1.33 extra cycles per LDS cycle, profiles/r2_pmc_prefill.jsonl).
__device__ __forceinline__ int stage_slot(int row, int slot) {
  return row * 8 + (slot ^ ((row >> 1) & 7));
}

// Optional XCD-grouped workgroup order (tao_tune_gemm_order 1). Workgroups are dealt
// round-robin over the 8 XCDs (blocks b, b + 8, ... share one L2; which XCD is not fixed:
// MI355X_MICROARCH.md "Workgroup dispatch"). The M tiles of one (column tile, K slice) read the
// same weight bytes; grouped, those ny workgroups run back to back on one XCD and its L2 serves
// the re-reads. Measured (profiles/r2_pmc_prefill*.jsonl, r2_prefill_order_ab.txt): at M = 128,
// N = 28672 it cuts FETCH_SIZE from 2.2x to 1.26x the algorithmic bytes but runs 76 -> 80 us,
// and ties elsewhere: these GEMMs are bound by per-CU ingest, not HBM. So the plain grid order
// is the default. Speed only: any order is correct. Identity unless the grid divides into whole
// groups of 8 x ny.
struct TileId {
  int n, m, z;
};
__device__ __forceinline__ TileId xcd_tile(int order) {
  const int nx = gridDim.x, ny = gridDim.y, nz = gridDim.z;
  const int L = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  const int T = nx * ny * nz;
  if (order != 1 || ny == 1 || T % (8 * ny) != 0)
    return TileId{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const int xcd = L & 7, slot = L >> 3;
  const int gi = (slot / ny) * 8 + xcd;
  return TileId{gi % nx, slot % ny, gi / nx};
}

// ---- policies -------------------------------------------------------------------------------
// setup(): per-lane state for lane (n, kq) — descriptors and voffsets (once per launch).
// load(): the raw bytes of the lane's weight piece for step `st` (wave-uniform, clamped to the
// slice), never predicated: a select on a freshly loaded value makes hipcc wait for the load on
// the spot, or branch around it, which collapses the prefetch pipeline. No weight is masked:
// columns past N (clamped to row N - 1) are computed and dropped, and a K tail reads the next
// row's finite weights against x that the LDS store zeroes. prep()/frag(): B fragments.
struct Int4WO {
  static constexpr int kPathId = 0;   // gemm_table.inc
  static constexpr int kABytes = 2;   // bf16 x
  static constexpr int kKStep = 256;  // 128 B of nibbles per row per step: one full line
  static constexpr int kMfma = 8;
  static constexpr int kMaxBM = 64;  // 512-B x rows: BM 128 would need 64 x VGPRs per stage
  static constexpr int kPrefKG = 2;
  static constexpr int kMinSlice = 4;  // steps per split-K slice (1024 k)
  // Weights in full 128-B lines (8 rows x 128 B per wave instruction: lane l reads row
  // 8 g + l / 8, 16-B chunk l % 8 of the step) regrouped to the MFMA layout through a 2-KiB
  // per-wave LDS stage ([16 rows][8 chunks], XOR-swizzled by row); lane (n, kq) then holds
  // chunks kq and 4 + kq (32 k each, one (scale, zero) dword each).
  static constexpr int kStage = 128;  // uint4 per wave
  typedef f32x4_t Acc;
  const uint4* wq;     // [N][K/32] 16-B chunks
  const uint32_t* sz;  // [N][K/g] (scale, zero)
  int gshift;          // log2(g / 32)
  struct Lane {
    Rsrc w, z;
    uint32_t wv0, wv1, zv0, zv1;
  };
  struct Chunk {
    uint4 a, b;
    uint32_t sz0, sz1;
  };
  struct Prep {
    uint32_t w[8];  // dwords of chunks kq (0..3) and 4 + kq (4..7)
    float s0, zc0, s1, zc1;
  };
  __device__ __forceinline__ Lane setup(int bn, int lane, int N, int K) const {
    const int n = bn < N ? bn : N - 1, kq = lane >> 4;
    Lane L;
    const uint32_t zrow = (uint32_t)(K >> 5 >> gshift);  // (scale, zero) dwords per row
    L.w = make_rsrc(wq, (uint32_t)N * (uint32_t)(K >> 1));
    L.z = make_rsrc(sz, (uint32_t)N * zrow * 4u);
    const int base = bn - (lane & 15);
    const int r0 = base + (lane >> 3), r1 = r0 + 8;
    L.wv0 = (uint32_t)(r0 < N ? r0 : N - 1) * (uint32_t)(K >> 1) + 16 * (lane & 7);
    L.wv1 = (uint32_t)(r1 < N ? r1 : N - 1) * (uint32_t)(K >> 1) + 16 * (lane & 7);
    // chunk 8 st + c -> group ((8 st) >> gshift) + (c >> gshift) (c < 8, gshift <= 3)
    L.zv0 = ((uint32_t)n * zrow + (kq >> gshift)) * 4;
    L.zv1 = ((uint32_t)n * zrow + ((4 + kq) >> gshift)) * 4;
    return L;
  }
  __device__ __forceinline__ Chunk load(const Lane& L, int st) const {
    Chunk ch;
    ch.a = bload16<kNT>(L.w, L.wv0, st * 128);
    ch.b = bload16<kNT>(L.w, L.wv1, st * 128);
    const uint32_t zo = ((8 * st) >> gshift) * 4;
    ch.sz0 = bload4<kNT>(L.z, L.zv0, zo);
    ch.sz1 = bload4<kNT>(L.z, L.zv1, zo);
    return ch;
  }
  __device__ __forceinline__ Prep prep(const Chunk& ch, uint4* stage, int lane) const {
    const int r = lane >> 3, c = lane & 7;
    stage[stage_slot(r, c)] = ch.a;
    stage[stage_slot(r + 8, c)] = ch.b;
    const int n = lane & 15, kq = lane >> 4;
    const uint4 p0 = stage[stage_slot(n, kq)];
    const uint4 p1 = stage[stage_slot(n, 4 + kq)];
    Prep p;
    p.w[0] = p0.x;
    p.w[1] = p0.y;
    p.w[2] = p0.z;
    p.w[3] = p0.w;
    p.w[4] = p1.x;
    p.w[5] = p1.y;
    p.w[6] = p1.z;
    p.w[7] = p1.w;
    p.s0 = bf16lo_to_f32(ch.sz0);
    p.zc0 = bf16hi_to_f32(ch.sz0) - 8.f * p.s0;  // q*s + zc == (q-8)*s + z
    p.s1 = bf16lo_to_f32(ch.sz1);
    p.zc1 = bf16hi_to_f32(ch.sz1) - 8.f * p.s1;
    return p;
  }
  // B fragment of MFMA s (chunk s >> 2, dword s & 3): bf16(fma(q, s, z - 8 s)) for its 8
  // nibbles. Row-stream nibble order (bits 4i: q[2i], bits 16+4i: q[2i+1]) puts q0,q4,q1,q5
  // in the bytes of w & 0x0F0F0F0F and q2,q6,q3,q7 in those of (w >> 4) & 0x0F0F0F0F. A byte
  // b < 16 read as OCP e4m3 is exactly b / 512 (subnormals for b < 8, exponent 1 above), so
  // one v_cvt_scalef32_pk_f32_fp8 with scale 512 turns two of them into exact fp32 integers;
  // then one v_pk_fma_f32 and one v_cvt_pk_bf16_f32 per pair: ~1.9 VALU per weight.
  __device__ __forceinline__ bf16x8_t frag(const Prep& p, int s) const {
    const uint32_t w = p.w[s];
    const float sc = s < 4 ? p.s0 : p.s1, zc = s < 4 ? p.zc0 : p.zc1;
    const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
    const f32x2_t q04 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, false);
    const f32x2_t q15 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, true);
    const f32x2_t q26 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, false);
    const f32x2_t q37 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, true);
    const f32x2_t sv = {sc, sc}, zv = {zc, zc};
    const f32x2_t w04 = q04 * sv + zv, w15 = q15 * sv + zv;  // v_pk_fma_f32 (contracted)
    const f32x2_t w26 = q26 * sv + zv, w37 = q37 * sv + zv;
    return as_bf16x8(pack_bf16x2(w04[0], w15[0]), pack_bf16x2(w26[0], w37[0]),
                     pack_bf16x2(w04[1], w15[1]), pack_bf16x2(w26[1], w37[1]));
  }
  // MFMA s = 4 h + t takes dword t of chunk 4 h + kq: x slot 4 (4 h + kq) + t
  static __device__ __forceinline__ int slot(int s, int kq) {
    return 16 * (s >> 2) + 4 * kq + (s & 3);
  }
  // x image mask (x_slot): m, with bit 2 flipped on rows m & 15 in 4..11 (bits 2 and 3 differ)
  static __device__ __forceinline__ int xswz(int row) {
    const int m = row & 15;
    return m ^ ((m ^ (m >> 1)) & 4);
  }
  static __device__ __forceinline__ Acc mfma(const uint4& a, const bf16x8_t& b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), b, c, 0, 0, 0);
  }
  // int4 output: bf16(acc) (+ bias added by the caller, tensor_core_tiled_layout.py:104-114)
  static constexpr bool kRowF = false, kColF = false;  // no per-row / per-column factor
  __device__ __forceinline__ const uint16_t* row_factor() const { return nullptr; }
  __device__ __forceinline__ const uint16_t* col_factor() const { return nullptr; }
  __device__ __forceinline__ float epi(float acc, float, float) const { return round_bf16(acc); }
};

struct Int8WO {
  static constexpr int kPathId = 1;
  static constexpr int kABytes = 2;
  static constexpr int kKStep = 128;
  static constexpr int kMfma = 4;
  static constexpr int kMaxBM = 128;
  static constexpr int kPrefKG = 2;
  static constexpr int kMinSlice = 8;
  typedef f32x4_t Acc;
  const uint4* w;         // [N][K/16]
  const uint16_t* scale;  // [N]
  // Weights are loaded in full 128-B lines (8 rows x 128 B per wave instruction: lane l reads
  // row 8 g + l / 8, bytes 16 (l % 8) of the step) and regrouped to the MFMA layout through a
  // 2-KiB per-wave LDS stage ([16 rows][8 slots], slot XOR-swizzled by row): measured ~1.4x
  // over 16 rows x 64 B per instruction on the streaming-bound shapes.
  static constexpr int kStage = 128;  // uint4 per wave
  struct Lane {
    Rsrc w;
    uint32_t wv0, wv1;
  };
  struct Chunk {
    uint4 a, b;
  };
  typedef Chunk Prep;
  __device__ __forceinline__ Lane setup(int bn, int lane, int N, int K) const {
    Lane L;
    L.w = make_rsrc(w, (uint32_t)N * (uint32_t)K);
    const int base = bn - (lane & 15);  // the wave's first row
    const int r0 = base + (lane >> 3), r1 = r0 + 8;
    L.wv0 = (uint32_t)(r0 < N ? r0 : N - 1) * (uint32_t)K + 16 * (lane & 7);
    L.wv1 = (uint32_t)(r1 < N ? r1 : N - 1) * (uint32_t)K + 16 * (lane & 7);
    return L;
  }
  __device__ __forceinline__ Chunk load(const Lane& L, int st) const {
    Chunk ch;
    ch.a = bload16<kNT>(L.w, L.wv0, st * 128);
    ch.b = bload16<kNT>(L.w, L.wv1, st * 128);
    return ch;
  }
  // stage: write the two full-line pieces, read back lane (n, kq)'s bytes 16 kq and 64 + 16 kq
  __device__ __forceinline__ Prep prep(const Chunk& ch, uint4* stage, int lane) const {
    const int r = lane >> 3, c = lane & 7;
    stage[stage_slot(r, c)] = ch.a;
    stage[stage_slot(r + 8, c)] = ch.b;
    const int n = lane & 15, kq = lane >> 4;
    Prep p;
    p.a = stage[stage_slot(n, kq)];
    p.b = stage[stage_slot(n, 4 + kq)];
    return p;
  }
  // int8 -> bf16 is exact: (q ^ 0x80) is q + 128 as an unsigned byte (one v_cvt_f32_ubyteN),
  // minus 128 in fp32 (exact), packed.
  __device__ __forceinline__ bf16x8_t frag(const Prep& p, int s) const {
    const uint32_t d0 = ((s == 0) ? p.a.x : (s == 1) ? p.a.z : (s == 2) ? p.b.x : p.b.z) ^ 0x80808080u;
    const uint32_t d1 = ((s == 0) ? p.a.y : (s == 1) ? p.a.w : (s == 2) ? p.b.y : p.b.w) ^ 0x80808080u;
    auto cv = [](uint32_t d, int b) { return (float)((d >> (8 * b)) & 0xFF) - 128.f; };
    return as_bf16x8(pack_bf16x2(cv(d0, 0), cv(d0, 1)), pack_bf16x2(cv(d0, 2), cv(d0, 3)),
                     pack_bf16x2(cv(d1, 0), cv(d1, 1)), pack_bf16x2(cv(d1, 2), cv(d1, 3)));
  }
  // lane (n, kq) holds k 16 kq .. +16 (a) and 64 + 16 kq .. +16 (b): 8-k slots 2 kq, 2 kq + 1,
  // 8 + 2 kq, 9 + 2 kq for MFMA s = 0..3
  static __device__ __forceinline__ int slot(int s, int kq) { return (s >> 1) * 8 + kq * 2 + (s & 1); }
  static __device__ __forceinline__ int xswz(int row) { return row & 15; }
  static __device__ __forceinline__ Acc mfma(const uint4& a, const bf16x8_t& b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), b, c, 0, 0, 0);
  }
  // bf16 mm output, then * scale (plain_layout.py:258-262)
  static constexpr bool kRowF = false, kColF = true;
  __device__ __forceinline__ const uint16_t* row_factor() const { return nullptr; }
  __device__ __forceinline__ const uint16_t* col_factor() const { return scale; }
  __device__ __forceinline__ float epi(float acc, float, float sc) const {
    return round_bf16(round_bf16(acc) * sc);
  }
};

struct Int8Dyn {
  static constexpr int kPathId = 2;
  static constexpr int kABytes = 1;  // int8 x
  static constexpr int kKStep = 256;
  static constexpr int kMfma = 4;
  static constexpr int kMaxBM = 128;
  static constexpr int kPrefKG = 1;
  static constexpr int kMinSlice = 4;
  typedef i32x4_t Acc;
  const uint4* w;           // [N][K/16]
  const uint16_t* wscale;   // [N]
  const uint16_t* xscale;   // [M]
  // Full 128-B lines per wave instruction (lane l: row 8 g + l / 8, bytes 128 h + 16 (l % 8))
  // regrouped to the MFMA layout through a 4-KiB per-wave LDS stage ([16 rows][16 slots],
  // XOR-swizzled by row): 15.1 -> ~11 us at M=128, 4096^2 (experiments/gemm_debug.sh, 5/6).
  static constexpr int kStage = 256;  // uint4 per wave
  struct Lane {
    Rsrc w;
    uint32_t wv0, wv1;
  };
  struct Chunk {
    uint4 v[4];  // (g, h) = (0,0), (1,0), (0,1), (1,1)
  };
  struct Prep {
    uint4 v[4];  // MFMA s: bytes 64 s + 16 kq of row n
  };
  __device__ __forceinline__ Lane setup(int bn, int lane, int N, int K) const {
    Lane L;
    L.w = make_rsrc(w, (uint32_t)N * (uint32_t)K);
    const int base = bn - (lane & 15);
    const int r0 = base + (lane >> 3), r1 = r0 + 8;
    L.wv0 = (uint32_t)(r0 < N ? r0 : N - 1) * (uint32_t)K + 16 * (lane & 7);
    L.wv1 = (uint32_t)(r1 < N ? r1 : N - 1) * (uint32_t)K + 16 * (lane & 7);
    return L;
  }
  __device__ __forceinline__ Chunk load(const Lane& L, int st) const {
    Chunk ch;
    ch.v[0] = bload16<kNT>(L.w, L.wv0, st * 256);
    ch.v[1] = bload16<kNT>(L.w, L.wv1, st * 256);
    ch.v[2] = bload16<kNT>(L.w, L.wv0 + 128, st * 256);
    ch.v[3] = bload16<kNT>(L.w, L.wv1 + 128, st * 256);
    return ch;
  }
  __device__ __forceinline__ Prep prep(const Chunk& ch, uint4* stage, int lane) const {
    const int r = lane >> 3, c = lane & 7;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int row = r + 8 * (x & 1), slot = c + 8 * (x >> 1);
      stage[row * 16 + (slot ^ row)] = ch.v[x];
    }
    const int n = lane & 15, kq = lane >> 4;
    Prep p;
#pragma unroll
    for (int s = 0; s < 4; ++s) p.v[s] = stage[n * 16 + ((4 * s + kq) ^ n)];
    return p;
  }
  __device__ __forceinline__ i32x4_t frag(const Prep& p, int s) const {
    return __builtin_bit_cast(i32x4_t, p.v[s]);
  }
  // load s covers 64 contiguous bytes of each row: lane (n, kq) holds k 64 s + 16 kq .. +16,
  // i.e. MFMA s is the contiguous k block 64 s .. +64 (16-B x slot 4 s + kq)
  static __device__ __forceinline__ int slot(int s, int kq) { return s * 4 + kq; }
  static __device__ __forceinline__ int xswz(int row) { return row & 15; }
  static __device__ __forceinline__ Acc mfma(const uint4& a, const i32x4_t& b, Acc c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a), b, c, 0, 0, 0);
  }
  // bf16(c) * x_scale, * w_scale, each rounded (intmm.py:133-137, plain_layout.py:301-315)
  static constexpr bool kRowF = true, kColF = true;
  __device__ __forceinline__ const uint16_t* row_factor() const { return xscale; }
  __device__ __forceinline__ const uint16_t* col_factor() const { return wscale; }
  __device__ __forceinline__ float epi(int acc, float xs, float ws) const {
    const float v = round_bf16(round_bf16((float)acc) * xs);
    return round_bf16(v * ws);
  }
};

// LDS image of one x tile: [BM rows][16 slots of 16 B], slot XOR-swizzled with row & 15 so the
// 16 rows of an A fragment read spread over all banks (cdna guide §5.5 T2).
template <int SLOTS>
__device__ __forceinline__ int lds_slot(int row, int slot) {
  return row * SLOTS + (slot ^ (row & 15));
}
// gemm_mfma_kernel's x image: the policy picks the row's XOR mask (P::xswz). ds_read_b128
// serves a wave in the lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
// {36-43,48-51,60-63} (MI355X_MICROARCH.md §LDS); an A-fragment read is conflict-free iff the 16
// lanes of each group hit 16 distinct 16-B granules (slot mod 16). Lane (m = l & 15, kq = l >> 4)
// reads slot(s, kq) of row m, so a group holds kq = 2i at rows A = {0-3, 12-15} and kq = 2i + 1
// at rows B = {4-11} (or the reverse). Int8Dyn's slot 4 s + kq and Int8WO's 8 (s >> 1) + 2 kq +
// (s & 1) are conflict-free with mask m; Int4WO's 16 (s >> 2) + 4 kq + (s & 3) is not (A ^ t and
// B ^ 4 ^ t are the same 8 granules: every read 2-way), so it flips bit 2 of the mask on rows B.
// The ds_write_b128 fill (8 lanes = 8 consecutive slots of one row) is conflict-free either way.
template <int SLOTS, class P>
__device__ __forceinline__ int x_slot(int row, int slot) {
  return row * SLOTS + (slot ^ P::xswz(row));
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// One k-step ring of depth D holds both operands' loads: vector-memory loads retire in issue
// order (one vmcnt), so an x ring shallower than the weight ring would drain the weight loads
// issued before each x load anyway. The k loop is unrolled by D so every ring index is a
// compile-time constant (no scratch), and the steady-state body is straight-line code: loads
// past the last step re-read it (clamped), so hipcc counts outstanding loads (vmcnt(N))
// instead of draining them every step.
//
// Latency hiding comes from waves per SIMD, so K is split twice:
//  * inside the workgroup: KG k-groups of 4 waves (256 x KG threads) take interleaved steps
//    (k-group g: steps s0 + g, s0 + g + KG, ...), each with its own double-buffered x tile;
//    their accumulators are summed through LDS in k-group order at the end;
//  * across workgroups (gridDim.z = S slices of `sps` steps): each slice stores its raw
//    accumulator tile to a slab with sc1 (write-through) stores, and the tile's last arriver
//    (agent-scope ticket, told by the value its add returned) reads the S slabs with sc1 loads,
//    sums them in slice order and runs the epilogue. Both sums have a fixed order, so results
//    do not depend on arrival order. Protocol and its hardware assumption: last_arriver()
//    (tao_common.h); `fenced` adds the agent release/acquire fences (tao_tune_splitk_fenced).
// Experiment switch (timing A/B only): minimum waves per SIMD the register allocation must
// allow (amdgpu_waves_per_eu); 0 = the compiler's choice (the product).
#ifndef TAO_GEMM_WPE
#define TAO_GEMM_WPE 0
#endif
#if TAO_GEMM_WPE > 0
#define TAO_GEMM_WPE_ATTR __attribute__((amdgpu_waves_per_eu(TAO_GEMM_WPE)))
#else
#define TAO_GEMM_WPE_ATTR
#endif
template <int BM, int D, int KG, int NW, class P>
__global__ __launch_bounds__(256 * KG) TAO_GEMM_WPE_ATTR void gemm_mfma_kernel(
    const uint8_t* __restrict__ x, P pol, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int sps, typename P::Acc* __restrict__ slab,
    unsigned* __restrict__ cnt, int fenced, int order, int cs) {
  typedef typename P::Acc Acc;
  constexpr int MT = BM / 16;
  constexpr int XSB = P::kABytes * P::kKStep;  // x bytes per row per step (256 or 512)
  constexpr int SLOTS = XSB / 16;               // 16-B x slots per row per step
  constexpr int RPP = 256 / SLOTS;              // x rows loaded per 256-thread pass
  constexpr int XLOADS = BM * SLOTS / 256;      // 16-B x pieces per thread per step
  constexpr int TILE = BM * SLOTS;              // uint4 per x tile
  constexpr int NA = MT * NW;                   // accumulator tiles per wave
  static_assert((KG - 1) * 4 * NA * 64 <= KG * 2 * TILE, "k-group reduction must fit in LDS");
  // one LDS array (a second __shared__ object can de-pipeline the loop, cdna guide §5 item 4a):
  // [KG][2][x tile] then the per-wave weight stages (NW per wave)
  __shared__ uint4 lds[KG * 2 * TILE + KG * 4 * NW * P::kStage + (P::kStage == 0)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int kg = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int wave = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int ktid = tid & 255;
  const TileId tid3 = xcd_tile(order);
  const int n_blk = tid3.n * kBN * NW;
  const int m_blk = tid3.m * BM;
  const int nsteps = (K + P::kKStep - 1) / P::kKStep;
  const int s0 = tid3.z * sps;
  const int s1 = s0 + sps < nsteps ? s0 + sps : nsteps;  // launcher: no empty slice
  const int J = (s1 - s0 + KG - 1) / KG;                 // steps per k-group (all k-groups)
  const int row_bytes = K * P::kABytes;
  uint4* xs = lds + kg * 2 * TILE;

  // the wave's NW 16-column blocks: columns n_blk + 16 (NW wave + c) + (lane & 15)
  int bn[NW];
  typename P::Lane wl[NW];
#pragma unroll
  for (int c = 0; c < NW; ++c) {
    bn[c] = n_blk + (wave * NW + c) * 16 + (lane & 15);
    wl[c] = pol.setup(bn[c], lane, N, K);
  }
  const int kq = lane >> 4;
  uint4* wstage = lds + KG * 2 * TILE + (kg * 4 + wave) * NW * P::kStage;

  // this thread's x pieces: rows row0 + RPP i (i < XLOADS), 16-B slot xslot of each; rows
  // past M are clamped to M - 1 (computed and dropped). A k tail past the row end reads the
  // next row (or 0 past the buffer) and is masked at the LDS store.
  const int row0 = ktid / SLOTS, xslot = ktid % SLOTS;
  const int xslot_b = xslot * 16;
  const Rsrc xrs = make_rsrc(x, (uint32_t)M * (uint32_t)row_bytes);
  uint32_t xv[XLOADS];
  int xlds[XLOADS];
#pragma unroll
  for (int i = 0; i < XLOADS; ++i) {
    const int gm = m_blk + row0 + RPP * i;
    xv[i] = (uint32_t)(gm < M ? gm : M - 1) * (uint32_t)row_bytes + xslot_b;
    xlds[i] = x_slot<SLOTS, P>(row0 + RPP * i, xslot);
  }
  const bool ragged = (row_bytes % XSB) != 0;

  Acc acc[NA];  // [t][c]
#pragma unroll
  for (int t = 0; t < NA; ++t) acc[t] = Acc{0, 0, 0, 0};

  uint4 xr[D][XLOADS];
  typename P::Chunk wr[D][NW];

  // local step j of this k-group -> absolute step (may be >= s1: then inactive)
  auto abs_step = [&](int j) __attribute__((always_inline)) { return s0 + kg + j * KG; };
  auto load_step = [&](int j, uint4 (&xdst)[XLOADS], typename P::Chunk (&wdst)[NW])
      __attribute__((always_inline)) {
    const int st0 = abs_step(j);
    const int st = st0 < s1 ? st0 : s1 - 1;
#pragma unroll
    for (int i = 0; i < XLOADS; ++i) xdst[i] = bload16(xrs, xv[i], st * XSB);
#pragma unroll
    for (int c = 0; c < NW; ++c) wdst[c] = pol.load(wl[c], st);
  };
  auto store_x = [&](const uint4 (&src)[XLOADS], int j) __attribute__((always_inline)) {
    const int st = abs_step(j);
    uint4* dst = xs + (j & 1) * TILE;
    if (!ragged && st < s1) {
#pragma unroll
      for (int i = 0; i < XLOADS; ++i) dst[xlds[i]] = src[i];
    } else {
      // k tail / inactive step -> 0 (an AND mask: a select here compiles to a branch)
      const uint32_t keep = st < s1 && st * XSB + xslot_b < row_bytes ? ~0u : 0u;
#pragma unroll
      for (int i = 0; i < XLOADS; ++i)
        dst[xlds[i]] =
            make_uint4(src[i].x & keep, src[i].y & keep, src[i].z & keep, src[i].w & keep);
    }
  };
  // local step j; u = j % D at compile time
  auto body = [&](auto uc, int j) __attribute__((always_inline)) {
    constexpr int u = decltype(uc)::value;
    load_step(j + D - 1, xr[(u + D - 1) % D], wr[(u + D - 1) % D]);
    if (abs_step(j) < s1) {  // uniform: a k-group's idle tail iterations skip the math
      typename P::Prep pw[NW];
#pragma unroll
      for (int c = 0; c < NW; ++c) pw[c] = pol.prep(wr[u][c], wstage + c * P::kStage, lane);
      const uint4* xb = xs + (j & 1) * TILE;
#pragma unroll
      for (int s = 0; s < P::kMfma; ++s) {
        decltype(pol.frag(pw[0], s)) bfrag[NW];
#pragma unroll
        for (int c = 0; c < NW; ++c) bfrag[c] = pol.frag(pw[c], s);
        const int slot = P::slot(s, kq);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int row = t * 16 + (lane & 15);
          // one A fragment read from LDS feeds the wave's NW column blocks
          const uint4 a = xb[x_slot<SLOTS, P>(row, slot)];
#pragma unroll
          for (int c = 0; c < NW; ++c) acc[t * NW + c] = P::mfma(a, bfrag[c], acc[t * NW + c]);
        }
      }
    }
    if (j + 1 < J) store_x(xr[(u + 1) % D], j + 1);
    __syncthreads();
  };

  // Epilogue operands loaded now, ahead of the weights: loaded in the epilogue, their round
  // trip sat in every workgroup's tail (~1 µs of the int8-dyn M = 128 4096² kernel;
  // experiments/gemm_stamps.py). Per lane: the row factor of its 4 rows per M tile (rows
  // clamped to M - 1, kept as bf16 pairs), the column factor and bias of its NW columns.
  // (the int4 policy has neither factor; its bias stays an epilogue load: prefetching that too
  // measured 1.3 µs slower at M = 128, 4096², profiles/r2_ab_epi.txt)
  constexpr bool kPre = P::kRowF || P::kColF;
  uint2 rowf[P::kRowF ? MT : 1];
  float colf[NW], biasf[NW];
  if constexpr (P::kRowF) {
    const uint16_t* rp = pol.row_factor();
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      uint32_t h[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m_blk + t * 16 + 4 * (lane >> 4) + i;
        h[i] = rp[m < M ? m : M - 1];
      }
      rowf[t] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    }
  }
#pragma unroll
  for (int c = 0; c < NW; ++c) {
    const int nn = bn[c] < N ? bn[c] : N - 1;
    colf[c] = P::kColF ? bf16_to_f32(pol.col_factor()[nn]) : 1.f;
    biasf[c] = (kPre && bias != nullptr) ? bf16_to_f32(bias[nn]) : 0.f;
  }
  static_for<0, D - 1>([&](auto i) __attribute__((always_inline)) {
    load_step(decltype(i)::value, xr[decltype(i)::value], wr[decltype(i)::value]);
  });
  store_x(xr[0], 0);
  __syncthreads();

  int j = 0;
  for (; j + D <= J; j += D)
    static_for<0, D>([&](auto uc) __attribute__((always_inline)) {
      body(uc, j + decltype(uc)::value);
    });
  static_for<0, D - 1>([&](auto uc) __attribute__((always_inline)) {
    if (j + decltype(uc)::value < J) body(uc, j + decltype(uc)::value);
  });

  // k-groups 1..KG-1 hand their accumulators to k-group 0 through LDS (summed in order)
  if constexpr (KG > 1) {
    Acc* red = reinterpret_cast<Acc*>(lds);
    if (kg > 0) {
#pragma unroll
      for (int t = 0; t < NA; ++t) red[(((kg - 1) * 4 + wave) * NA + t) * 64 + lane] = acc[t];
    }
    __syncthreads();
    if (kg == 0) {
      for (int g = 1; g < KG; ++g) {
#pragma unroll
        for (int t = 0; t < NA; ++t) acc[t] += red[(((g - 1) * 4 + wave) * NA + t) * 64 + lane];
      }
    }
    __syncthreads();  // LDS free again (the split-K flag below reuses it)
  }

  const int S = gridDim.z;
  if (S > 1) {
    // Slab hand-off (last_arriver, tao_common.h: MI355X_MICROARCH.md "Hand-offs measured with
    // sc1 loads in place of the acquire", first row): every slab byte is stored sc1 (write-through
    // past the XCD's L2) and read sc1 (L1 bypassed), each storing wave waits for its stores
    // before the workgroup barrier, one lane adds the tile's ticket, and the last arriver is told
    // by the value its add returned. The fences this leaves out by default (buffer_wbl2 +
    // buffer_inv, 1.7-6.5 µs each and serialised per CU) made every split slower than no split;
    // `fenced` puts them back (tao_tune_splitk_fenced).
    const unsigned tile = tid3.m * gridDim.x + tid3.n;
    const size_t tile_bytes = (size_t)S * 4 * NA * 64 * sizeof(Acc);
    const Rsrc srs = make_rsrc(reinterpret_cast<const uint8_t*>(slab) + tile * tile_bytes,
                               (uint32_t)tile_bytes);
    const uint32_t lane_off = (uint32_t)((wave * NA * 64 + lane) * sizeof(Acc));
    constexpr uint32_t kZ = 4 * NA * 64 * sizeof(Acc);  // one slice's slab
    if (kg == 0) {
#pragma unroll
      for (int t = 0; t < NA; ++t)
        bstore16<kSC1>(srs, lane_off + t * 64 * sizeof(Acc), tid3.z * kZ,
                       __builtin_bit_cast(uint4, acc[t]));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool last =
        last_arriver(&cnt[tile * cs], (unsigned)S, reinterpret_cast<unsigned*>(lds), fenced);
    if (!last || kg != 0) {
      return;
    }
#pragma unroll
    for (int t = 0; t < NA; ++t) acc[t] = Acc{0, 0, 0, 0};
    // 4 slabs per round, all loads issued before the first add (clamped, then masked); slices
    // summed in slice order whatever the arrival order
    for (int z0 = 0; z0 < S; z0 += 4) {
      Acc part[4][NA];
#pragma unroll
      for (int zz = 0; zz < 4; ++zz) {
        const int z = z0 + zz < S ? z0 + zz : S - 1;
#pragma unroll
        for (int t = 0; t < NA; ++t)
          part[zz][t] = __builtin_bit_cast(
              Acc, bload16<kSC1>(srs, lane_off + t * 64 * sizeof(Acc), z * kZ));
      }
#pragma unroll
      for (int zz = 0; zz < 4; ++zz) {
        if (z0 + zz < S) {
#pragma unroll
          for (int t = 0; t < NA; ++t) acc[t] += part[zz][t];
        }
      }
    }
  } else if (kg != 0) {
    return;
  }

  // C/D map: col = lane & 15 (n), row = 4*(lane >> 4) + i (m).
#pragma unroll
  for (int c = 0; c < NW; ++c) {
    if (bn[c] < N) {
      if constexpr (!kPre) biasf[c] = bias != nullptr ? bf16_to_f32(bias[bn[c]]) : 0.f;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m_blk + t * 16 + 4 * (lane >> 4) + i;
          if (m < M) {
            float rf = 1.f;
            if constexpr (P::kRowF) {
              const uint32_t w = (i < 2) ? rowf[t].x : rowf[t].y;
              rf = (i & 1) ? bf16hi_to_f32(w) : bf16lo_to_f32(w);
            }
            float v = pol.epi(acc[t * NW + c][i], rf, colf[c]);
            if (bias != nullptr) v = round_bf16(v + biasf[c]);
            y[(size_t)m * N + bn[c]] = f32_to_bf16(v);
          }
        }
      }
    }
  }
}

// Launch shape: M tile, k-groups per workgroup and K slices. Per-workgroup time is set by its
// load latency chain, so the grid should put several waves on every SIMD.
struct GemmShape {
  int bm, kg, splits, nw;
};

GemmShape choose_shape(int M, int N, int nsteps, int max_bm, int xsb, int pref_kg,
                       int min_slice, int nw) {
  // From the sweeps with the fence-free split-K hand-off (experiments/sweep_gemm.py,
  // profiles/r1_sweep_gemm_sc1*.jsonl; the fenced hand-off made every split lose):
  //  * short K (<= 16 steps): the largest M tile (no 2x padding of M) that gives ~one round of
  //    workgroups (>= 224 tiles of 256 CUs) unsplit; 128 gives way to 64 while that still fits
  //    in two rounds (<= 512 tiles);
  //  * otherwise the M tile that covers M up to 64 rows, and K split until the distinct weight
  //    slices (N tiles x K slices) reach one round, <= 512 workgroups, slices >= min_slice
  //    steps (1024 k);
  //  * the policy's preferred k-groups (int4 / int8-WO 2, int8-dyn 1).
  const long nb = (N + kBN * nw - 1) / (kBN * nw);
  auto tiles_of = [&](int bm) { return nb * ((M + bm - 1) / bm); };
  GemmShape sh{16, pref_kg, 1, nw};
  const int cands[4] = {128, 64, 32, 16};
  bool found = false;
  if (nsteps <= 16) {
    for (int bm : cands)
      if (bm <= max_bm && (bm < 2 * M || bm == 16) && tiles_of(bm) >= 224) {
        sh.bm = bm;
        found = true;
        break;
      }
    if (found && sh.bm == 128 && tiles_of(64) <= 512) sh.bm = 64;
  }
  if (!found) {
    const int cap = max_bm < 64 ? max_bm : 64;
    while (sh.bm < cap && sh.bm < M) sh.bm *= 2;
    const long tiles = tiles_of(sh.bm);
    while (nb * sh.splits < 224 && tiles * sh.splits * 2 <= 512 && sh.splits * 2 <= 8 &&
           nsteps >= min_slice * sh.splits * 2)
      sh.splits *= 2;
  }
  // int8-dyn (one k-group by default): two when the launch is unsplit and >= 4 M tiles re-read
  // each weight tile (M = 128, 4096^2: 11.4 vs 11.9 µs; profiles/r1_sweep_gemm_sc1*.jsonl)
  if (pref_kg == 1 && sh.splits == 1 && (M + sh.bm - 1) / sh.bm >= 4) sh.kg = 2;
  const int tb = tao::tuning().bm;
  const int tk = tao::tuning().kg;
  const int ts = tao::tuning().splits;
  if (tb) sh.bm = tb < max_bm ? tb : max_bm;
  if (tk) sh.kg = tk;
  if (ts) sh.splits = ts < nsteps ? ts : nsteps;
  // LDS: KG x 2 x BM x xsb (double-buffered x tiles) <= 64 KiB
  while (sh.kg > 1 && sh.kg * sh.bm * xsb > 32768) sh.kg >>= 1;
  return sh;
}

// Measured launch shapes for the Llama-3 8B / 70B linears (experiments/sweep_nw.py ->
// experiments/gen_gemm_table.py; profiles/r2_sweep_nw_wide*.jsonl): where a swept shape beat
// choose_shape (and, for int8-dyn, the LDS-kernel choice) by >= 7% on the box. M is bucketed up
// to 16 / 32 / ... / 512; other shapes and M > 512 keep the heuristic. Any shape is correct and
// deterministic; a table shape only changes speed (and, through kg / splits, the fixed fp32
// summation order). nw 32 (int4 only) names gemm32_int4_kernel with that (bm, splits).
struct TunedShape {
  int path, m, n, k, bm, kg, splits, nw;
};
constexpr TunedShape kTuned[] = {
#include "gemm_table.inc"
};

const TunedShape* tuned_shape(int path, int M, int N, int K) {
  if (tuning().gemm_table == 1 || tuning().bm || tuning().kg || tuning().splits ||
      tuning().gemm_nw || M > 512)
    return nullptr;
  int mb = 16;
  while (mb < M) mb *= 2;
  for (const TunedShape& t : kTuned)
    if (t.path == path && t.m == mb && t.n == N && t.k == K) return &t;
  return nullptr;
}

template <int BM, int KG, int NW, class P>
void launch_one(dim3 grid, hipStream_t stream, const uint8_t* xb, const P& pol,
                const uint16_t* bias, uint16_t* y, int M, int N, int K, int sps,
                typename P::Acc* slab, unsigned* cnt) {
  if constexpr (BM <= P::kMaxBM) {
    // ring depth: 4 steps, 3 where the per-stage registers grow (int8-dyn's 64-B pieces,
    // int4's 512-B x rows), 2 at BM >= 64
    constexpr bool big = sizeof(typename P::Chunk) > 32 || P::kABytes * P::kKStep > 256;
    constexpr int D = TAO_GEMM_DEPTH > 0 ? TAO_GEMM_DEPTH
                                         : (BM <= 16 ? 4 : (BM <= 32 ? (big ? 3 : 4) : 2));
    launch((gemm_mfma_kernel<BM, D, KG, NW, P>), grid, dim3(256 * KG), 0, stream, xb, pol, bias, y,
           M, N, K, sps, slab, cnt, tuning().splitk_fenced, tuning().gemm_order,
           tuning().cnt_stride);
  }
}

template <class P>
int launch_gemm(const void* x, const P& pol, const uint16_t* bias, uint16_t* y, int M, int N,
                int K, hipStream_t stream) {
  const int nsteps = (K + P::kKStep - 1) / P::kKStep;
  const int nw = tuning().gemm_nw == 2 ? 2 : 1;
  GemmShape sh;
  if (const TunedShape* t = tuned_shape(P::kPathId, M, N, K)) {
    sh = GemmShape{t->bm < P::kMaxBM ? t->bm : P::kMaxBM, t->kg,
                   t->splits < nsteps ? t->splits : nsteps, t->nw};
    // as choose_shape's overrides were applied when the table was measured
    while (sh.kg > 1 && sh.kg * sh.bm * P::kABytes * P::kKStep > 32768) sh.kg >>= 1;
  } else {
    sh = choose_shape(M, N, nsteps, P::kMaxBM, P::kABytes * P::kKStep, P::kPrefKG, P::kMinSlice,
                      nw);
  }
  if (sh.nw == 32) sh.nw = 1;  // (the 32x32x16 kernel's entries are dispatched before this)
  if (sh.nw == 2) {  // instantiated: BM <= 64, KG <= 2 (registers)
    if (sh.bm > 64) sh.bm = 64;
    if (sh.kg > 2) sh.kg = 2;
  }
  const int sps = (nsteps + sh.splits - 1) / sh.splits;
  const int S = (nsteps + sps - 1) / sps;  // no empty slice
  const int bnw = kBN * sh.nw;
  dim3 grid((N + bnw - 1) / bnw, (M + sh.bm - 1) / sh.bm, S);
  typename P::Acc* slab = nullptr;
  unsigned* cnt = nullptr;
  if (S > 1) {
    const size_t tiles = (size_t)grid.x * grid.y;
    void* ws = nullptr;
    const int rc = split_workspace(stream, tiles * S * sh.bm * bnw * sizeof(float),
                                   tiles * tuning().cnt_stride, &ws, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<typename P::Acc*>(ws);
  }
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(x);
  const auto args = std::make_tuple(grid, stream, xb, pol, bias, y, M, N, K, sps, slab, cnt);
  auto go = [&](auto fn) { std::apply(fn, args); };
  if (sh.nw == 2) {  // 32 columns per wave: each A fragment read feeds two MFMAs
    switch (sh.bm * 8 + sh.kg) {
      case 16 * 8 + 1: go(launch_one<16, 1, 2, P>); break;
      case 16 * 8 + 2: go(launch_one<16, 2, 2, P>); break;
      case 32 * 8 + 1: go(launch_one<32, 1, 2, P>); break;
      case 32 * 8 + 2: go(launch_one<32, 2, 2, P>); break;
      case 64 * 8 + 1: go(launch_one<64, 1, 2, P>); break;
      default: go(launch_one<64, 2, 2, P>); break;
    }
    return check_launch("gemm_mfma_kernel");
  }
  switch (sh.bm * 8 + sh.kg) {
    case 16 * 8 + 1: go(launch_one<16, 1, 1, P>); break;
    case 16 * 8 + 2: go(launch_one<16, 2, 1, P>); break;
    case 16 * 8 + 4: go(launch_one<16, 4, 1, P>); break;
    case 32 * 8 + 1: go(launch_one<32, 1, 1, P>); break;
    case 32 * 8 + 2: go(launch_one<32, 2, 1, P>); break;
    case 32 * 8 + 4: go(launch_one<32, 4, 1, P>); break;
    case 64 * 8 + 1: go(launch_one<64, 1, 1, P>); break;
    case 64 * 8 + 2: go(launch_one<64, 2, 1, P>); break;
    default: go(launch_one<128, 1, 1, P>); break;
  }
  return check_launch("gemm_mfma_kernel");
}

// ---- int8 x int8 GEMM with both operands staged through LDS (int8-dyn, M >= 48) -------------
// gemm_mfma_kernel gives each wave 16 columns x all BM rows: every MFMA reads its own 1-KiB A
// fragment from LDS and every 16-column weight piece is regrouped per wave, ~2 KiB of LDS
// traffic per MFMA, so at M = 128 the LDS port, not the MFMA or HBM, sets the pace. Here a
// workgroup tile is BM x 64 with the 4 waves in 2 x 2 (wave (wm, wn): rows wm BM/2 .., columns
// wn 32 ..), so each A fragment feeds 2 MFMAs and each B fragment BM/32: 0.75 KiB per MFMA at
// BM = 128. Per 128-k step the workgroup loads x [BM][128 B] and W [64][128 B] in full 128-B
// lines (8 threads per row) D steps ahead into registers, then stores them to a double-buffered
// LDS image whose 16-B chunks are XOR-swizzled by (row >> 1) & 7: the 16 lanes of each
// ds_write_b128 / ds_read_b128 pass (two rows x 8 chunks; 16 consecutive rows at one chunk) hit
// 16 distinct bank groups. One barrier per step. K is split across workgroups with the same
// fence-free slab hand-off as gemm_mfma_kernel; the epilogue is Int8Dyn's (bit-exact).
constexpr int kI8Step = 128;  // k bytes per step of gemm_i8_lds_kernel

__device__ __forceinline__ int i8_swz(int row, int c) { return row * 8 + (c ^ ((row >> 1) & 7)); }

template <int BM, int D, int BN = 64>
__global__ __launch_bounds__(256) void gemm_i8_lds_kernel(
    const int8_t* __restrict__ x, const int8_t* __restrict__ w, const uint16_t* __restrict__ xscale,
    const uint16_t* __restrict__ wscale, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int sps, i32x4_t* __restrict__ slab,
    unsigned* __restrict__ cnt, int fenced, int order, int cs) {
  constexpr int XL = BM / 32;           // x chunks per thread per step
  constexpr int WL = BN / 32;           // W chunks per thread per step (BN rows x 8 chunks)
  constexpr int MT = BM / 32, NT = BN / 32;  // 16x16 output tiles per wave
  constexpr int XT = BM * 8, WT = BN * 8;    // uint4 per image
  __shared__ uint4 lds[2 * (XT + WT)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const TileId tid3 = xcd_tile(order);
  const int n_blk = tid3.n * BN, m_blk = tid3.m * BM;
  const int nsteps = K / kI8Step;
  const int s0 = tid3.z * sps;
  const int s1 = s0 + sps < nsteps ? s0 + sps : nsteps;  // launcher: no empty slice
  const int J = s1 - s0;

  // load slots: row lr + 32 i, 16-B chunk lc; rows past M / N clamped (computed, dropped)
  const int lr = tid >> 3, lc = tid & 7;
  const Rsrc xrs = make_rsrc(x, (uint32_t)M * (uint32_t)K);
  const Rsrc wrs = make_rsrc(w, (uint32_t)N * (uint32_t)K);
  uint32_t xv[XL], wv[WL];
  int xo[XL], wo[WL];
#pragma unroll
  for (int i = 0; i < XL; ++i) {
    const int r = lr + 32 * i, gm = m_blk + r < M ? m_blk + r : M - 1;
    xv[i] = (uint32_t)gm * (uint32_t)K + 16 * lc;
    xo[i] = i8_swz(r, lc);
  }
#pragma unroll
  for (int i = 0; i < WL; ++i) {
    const int r = lr + 32 * i, gn = n_blk + r < N ? n_blk + r : N - 1;
    wv[i] = (uint32_t)gn * (uint32_t)K + 16 * lc;
    wo[i] = XT + i8_swz(r, lc);
  }

  i32x4_t acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = i32x4_t{0, 0, 0, 0};

  // Epilogue operands loaded up front (gemm_mfma_kernel's reason): the x scales of this lane's
  // 4 rows per M tile as bf16 pairs (rows clamped), the w scale and bias of its NT columns.
  uint2 xsf[MT];
  float wsf[NT], bsf[NT];
  {
    const int q = (lane >> 4) & 3, c16 = lane & 15;
#pragma unroll
    for (int a = 0; a < MT; ++a) {
      uint32_t hh[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m_blk + wm * (BM / 2) + a * 16 + 4 * q + i;
        hh[i] = xscale[m < M ? m : M - 1];
      }
      xsf[a] = make_uint2(hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16));
    }
#pragma unroll
    for (int b = 0; b < NT; ++b) {
      const int n = n_blk + wn * (BN / 2) + b * 16 + c16;
      const int nn = n < N ? n : N - 1;
      wsf[b] = bf16_to_f32(wscale[nn]);
      bsf[b] = bias != nullptr ? bf16_to_f32(bias[nn]) : 0.f;
    }
  }

  uint4 xr[D][XL], wr[D][WL];
  auto load_step = [&](int j, uint4 (&xd)[XL], uint4 (&wd)[WL]) __attribute__((always_inline)) {
    const int st = s0 + j < s1 ? s0 + j : s1 - 1;  // past the slice: re-read (never predicated)
#pragma unroll
    for (int i = 0; i < XL; ++i) xd[i] = bload16(xrs, xv[i], st * kI8Step);
#pragma unroll
    for (int i = 0; i < WL; ++i) wd[i] = bload16<kNT>(wrs, wv[i], st * kI8Step);
  };
  auto store_step = [&](const uint4 (&xd)[XL], const uint4 (&wd)[WL], int buf)
      __attribute__((always_inline)) {
    uint4* img = lds + buf * (XT + WT);
#pragma unroll
    for (int i = 0; i < XL; ++i) img[xo[i]] = xd[i];
#pragma unroll
    for (int i = 0; i < WL; ++i) img[wo[i]] = wd[i];
  };
  const int fr = lane & 15, kq = lane >> 4;
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const uint4* img = lds + buf * (XT + WT);
#pragma unroll
    for (int b = 0; b < 2; ++b) {  // two 64-k blocks per step: chunks 4 b + kq
      const int c = 4 * b + kq;
      i32x4_t bf[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        bf[nt] = __builtin_bit_cast(i32x4_t, img[XT + i8_swz(wn * (BN / 2) + nt * 16 + fr, c)]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const i32x4_t af =
            __builtin_bit_cast(i32x4_t, img[i8_swz(wm * (BM / 2) + mt * 16 + fr, c)]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[nt], acc[mt][nt], 0, 0, 0);
      }
    }
  };
  // slot u holds local step j (j % D == u, compile-time); its registers are free once stored
  auto body = [&](auto uc, int j) __attribute__((always_inline)) {
    constexpr int u = decltype(uc)::value;
    load_step(j + D, xr[u], wr[u]);
    compute(j & 1);
    if (j + 1 < J) store_step(xr[(u + 1) % D], wr[(u + 1) % D], (j + 1) & 1);
    __syncthreads();
  };
  static_for<0, D>([&](auto i) __attribute__((always_inline)) {
    load_step(decltype(i)::value, xr[decltype(i)::value], wr[decltype(i)::value]);
  });
  store_step(xr[0], wr[0], 0);
  __syncthreads();
  int j = 0;
  for (; j + D <= J; j += D)
    static_for<0, D>([&](auto uc) __attribute__((always_inline)) {
      body(uc, j + decltype(uc)::value);
    });
  static_for<0, D - 1>([&](auto uc) __attribute__((always_inline)) {
    if (j + decltype(uc)::value < J) body(uc, j + decltype(uc)::value);
  });

  const int S = gridDim.z;
  if (S > 1) {  // slab hand-off as in gemm_mfma_kernel (last_arriver, tao_common.h)
    const unsigned tile = tid3.m * gridDim.x + tid3.n;
    constexpr uint32_t kZ = 4 * MT * NT * 64 * sizeof(i32x4_t);  // one slice's slab
    const Rsrc srs = make_rsrc(reinterpret_cast<const uint8_t*>(slab) + (size_t)tile * S * kZ,
                               (uint32_t)(S * kZ));
    const uint32_t lo = (uint32_t)((wave * MT * NT * 64 + lane) * sizeof(i32x4_t));
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b)
        bstore16<kSC1>(srs, lo + (a * NT + b) * 64 * sizeof(i32x4_t), tid3.z * kZ,
                       __builtin_bit_cast(uint4, acc[a][b]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!last_arriver(&cnt[tile * cs], (unsigned)S, reinterpret_cast<unsigned*>(lds), fenced)) return;
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[a][b] = i32x4_t{0, 0, 0, 0};
    for (int z = 0; z < S; ++z) {  // slice order
      i32x4_t part[MT][NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b)
          part[a][b] = __builtin_bit_cast(
              i32x4_t, bload16<kSC1>(srs, lo + (a * NT + b) * 64 * sizeof(i32x4_t), z * kZ));
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] += part[a][b];
    }
  }

  // C/D map: col = lane & 15 (n), row = 4 (lane >> 4) + i (m); Int8Dyn's epilogue
#pragma unroll
  for (int b = 0; b < NT; ++b) {
    const int n = n_blk + wn * (BN / 2) + b * 16 + fr;
    if (n >= N) continue;
    const float sw = wsf[b];
    const float bv = bsf[b];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m_blk + wm * (BM / 2) + a * 16 + 4 * kq + i;
        if (m < M) {
          const uint32_t xw = (i < 2) ? xsf[a].x : xsf[a].y;
          const float xsc = (i & 1) ? bf16hi_to_f32(xw) : bf16lo_to_f32(xw);
          float v = round_bf16(round_bf16((float)acc[a][b][i]) * xsc);
          v = round_bf16(v * sw);
          if (bias != nullptr) v = round_bf16(v + bv);
          y[(size_t)m * N + n] = f32_to_bf16(v);
        }
      }
  }
}

// gemm_i8_lds_kernel selection (tao_tune_gemm_algo): 0 = auto, 1 = never, 2 = always (K % 128)
// register-ring depth of gemm_i8_lds_kernel (tao_tune_gemm_depth; 0 = built-in 3 / 4)
// column tile of gemm_i8_lds_kernel (tao_tune_gemm_bn; 0 = built-in 64, or 128)

int launch_i8_lds(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
                  const uint16_t* bias, uint16_t* y, int M, int N, int K, bool auto_mode,
                  hipStream_t stream) {
  const int nsteps = K / kI8Step;
  // auto: 128-column tiles once 128 x 128 tiles alone number >= 256 (M >= 256;
  // profiles/r1_sweep_i8_bn.jsonl: M=512 14336x4096 54.6 vs 70.6 us; no gain at M = 128)
  const int tbn = tao::tuning().i8_bn;
  const int bn = tbn ? (tbn == 128 ? 128 : 64)
                     : (auto_mode && M >= 256 &&
                                (long)((N + 127) / 128) * ((M + 127) / 128) >= 256
                            ? 128
                            : 64);
  const long ntile = (N + bn - 1) / bn;
  // auto (profiles/r1_sweep_i8_lds.jsonl): the M = 128 tile once it alone fills a round of
  // workgroups, else 64; no split (every winning LDS shape ran unsplit). Forced (algo 2, the
  // parity tests' mode): split towards one round, slices of >= 4 steps (512 k).
  int bm = auto_mode ? (bn == 128 || ntile * ((M + 127) / 128) >= 224 ? 128 : 64)
                     : (M > 64 ? 128 : 64);
  const int tb = tao::tuning().bm;
  if (tb == 64 || tb == 128) bm = tb;
  const long tiles = ntile * ((M + bm - 1) / bm);
  int splits = 1;
  while (!auto_mode && tiles * splits < 224 && splits * 2 <= 16 && nsteps >= 4 * splits * 2)
    splits *= 2;
  const int ts = tao::tuning().splits;
  if (ts) splits = ts < nsteps ? ts : nsteps;
  const int sps = (nsteps + splits - 1) / splits;
  const int S = (nsteps + sps - 1) / sps;
  const dim3 grid((N + bn - 1) / bn, (M + bm - 1) / bm, S);
  i32x4_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (S > 1) {
    void* wsp = nullptr;
    const size_t t = (size_t)grid.x * grid.y;
    const int rc = split_workspace(stream, t * S * bm * bn * sizeof(int), t * tuning().cnt_stride,
                                   &wsp, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<i32x4_t*>(wsp);
  }
  const int td = tao::tuning().i8_depth;
  const int d = td ? td : (bm == 128 ? 3 : 4);
  auto go = [&](auto kern) {
    launch(kern, grid, dim3(256), 0, stream, xq, wq, xs, ws, bias, y, M, N, K, sps, slab, cnt,
           tuning().splitk_fenced, tuning().gemm_order, tuning().cnt_stride);
  };
  if (bn == 128) {  // experiment (tao_tune_gemm_bn): ring depth 2 or 3
    if (bm == 128) {
      if (d == 2) go(gemm_i8_lds_kernel<128, 2, 128>);
      else go(gemm_i8_lds_kernel<128, 3, 128>);
    } else {
      if (d == 2) go(gemm_i8_lds_kernel<64, 2, 128>);
      else go(gemm_i8_lds_kernel<64, 3, 128>);
    }
  } else if (bm == 128) {
    if (d == 2) go(gemm_i8_lds_kernel<128, 2>);
    else if (d == 3) go(gemm_i8_lds_kernel<128, 3>);
    else if (d == 4) go(gemm_i8_lds_kernel<128, 4>);
    else go(gemm_i8_lds_kernel<128, 6>);
  } else {
    if (d == 2) go(gemm_i8_lds_kernel<64, 2>);
    else if (d == 3) go(gemm_i8_lds_kernel<64, 3>);
    else if (d == 4) go(gemm_i8_lds_kernel<64, 4>);
    else if (d == 6) go(gemm_i8_lds_kernel<64, 6>);
    else go(gemm_i8_lds_kernel<64, 8>);
  }
  return check_launch("gemm_i8_lds_kernel");
}

// ---- int4 weight-only GEMM on 32x32x16 MFMAs (gemm32_int4_kernel) -----------------------------
// §4.2's variants put the int4 GEMM's time on the per-wave work around each MFMA: an A-fragment
// LDS read (1 KiB) and a B-fragment dequant (8 weights per lane) per 8 K MACs of
// v_mfma_f32_16x16x32_bf16. v_mfma_f32_32x32x16_bf16 does 16 K MACs with the same two fragment
// sizes (cdna guide §MFMA operand maps: lane (r = l & 31, h = l >> 5) holds A[r][8h + j] and
// B[8h + j][r]), so per MAC both halve.
// * Workgroup: 4 waves x 32 columns (128 columns) x BM rows (MT = BM / 32 tiles per wave).
// * Step = 256 k. The k order inside a step is permuted identically for A and B: lane half h
//   owns physical k [128 h, 128 h + 128) of the step, and MFMA s (0..15) takes k 128 h + 8 s + j
//   from each half. So a lane's B operand for the whole step is 64 contiguous nibble bytes of
//   its column (16 dwords, dword s -> MFMA s, already in k order for the fp8 dequant), and its A
//   operand for MFMA s is 16 contiguous bytes of the x image (slot 16 h + s).
// * Weights: full 128-B lines (lane l of load i: row 8 i + l / 8, 16-B chunk l % 8), regrouped
//   through a 4-KiB per-wave LDS stage ([32 rows][8 chunks], stage_slot swizzle: conflict-free
//   for the 2-row write passes and the 16-row read passes).
// * x: the double-buffered [BM][32 slots] image of gemm_mfma_kernel (lds_slot swizzle), one
//   barrier per step; (scale, zero): the lane's 4 groups of 32 k (one 16-B load at g = 32).
// * Split-K over gridDim.z with gemm_mfma_kernel's slab hand-off (last_arriver); bf16(acc)
//   (+ bias, rounded) as the Int4WO epilogue: results within fp32 re-association of it.
typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <int BM, int D, bool G32>
__global__ __launch_bounds__(256) void gemm32_int4_kernel(
    const uint8_t* __restrict__ x, const uint4* __restrict__ wq, const uint32_t* __restrict__ sz,
    int gshift, const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M, int N, int K,
    int sps, f32x16_t* __restrict__ slab, unsigned* __restrict__ cnt, int fenced, int cs) {
  constexpr int MT = BM / 32;
  constexpr int SLOTS = 32;                  // 16-B x slots per row per step (512 B)
  constexpr int RPP = 256 / SLOTS;           // x rows per 256-thread pass
  constexpr int XLOADS = BM * SLOTS / 256;   // x pieces per thread per step
  constexpr int TILE = BM * SLOTS;           // uint4 per x image
  constexpr int STAGE = 256;                 // uint4 per wave weight stage (32 rows x 8 chunks)
  static_assert(BM == 32 || BM == 64 || BM == 128, "BM 32, 64 or 128");
  __shared__ uint4 lds[2 * TILE + 4 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int n_blk = blockIdx.x * 128, m_blk = blockIdx.y * BM;
  const int nw0 = n_blk + wave * 32;
  const int nsteps = (K + 255) / 256;
  const int s0 = blockIdx.z * sps;
  const int s1 = s0 + sps < nsteps ? s0 + sps : nsteps;  // launcher: no empty slice
  const int J = s1 - s0;
  const int row_bytes = K * 2;
  uint4* xs = lds;
  uint4* wstage = lds + 2 * TILE + wave * STAGE;

  // weights: 4 full-line pieces per lane per step; (scale, zero): lane (r, h)'s 4 groups
  const uint32_t wrow = (uint32_t)(K >> 1);
  const Rsrc wrs = make_rsrc(wq, (uint32_t)N * wrow);
  uint32_t wv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = nw0 + 8 * i + (lane >> 3);
    wv[i] = (uint32_t)(n < N ? n : N - 1) * wrow + 16 * (lane & 7);
  }
  const uint32_t zrow = (uint32_t)(K >> 5 >> gshift);  // (scale, zero) dwords per row
  const Rsrc zrs = make_rsrc(sz, (uint32_t)N * zrow * 4u);
  const int ncol = nw0 + r;
  const uint32_t zv = (uint32_t)(ncol < N ? ncol : N - 1) * zrow * 4u;

  // x pieces: rows row0 + RPP i, slot xslot (rows past M clamped, k tail masked at the store)
  const int row0 = tid / SLOTS, xslot = tid % SLOTS;
  const Rsrc xrs = make_rsrc(x, (uint32_t)M * (uint32_t)row_bytes);
  uint32_t xv[XLOADS];
  int xl[XLOADS];
#pragma unroll
  for (int i = 0; i < XLOADS; ++i) {
    const int gm = m_blk + row0 + RPP * i;
    xv[i] = (uint32_t)(gm < M ? gm : M - 1) * (uint32_t)row_bytes + xslot * 16;
    xl[i] = lds_slot<SLOTS>(row0 + RPP * i, xslot);
  }
  const bool ragged = (row_bytes % 512) != 0;

  struct WChunk {
    uint4 p[4];
    uint32_t z[4];
  };
  uint4 xr[D][XLOADS];
  WChunk wr[D];
  f32x16_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  auto load_step = [&](int j, uint4 (&xd)[XLOADS], WChunk& wd) __attribute__((always_inline)) {
    const int st0 = s0 + j;
    const int st = st0 < s1 ? st0 : s1 - 1;
#pragma unroll
    for (int i = 0; i < XLOADS; ++i) xd[i] = bload16(xrs, xv[i], st * 512);
#pragma unroll
    for (int i = 0; i < 4; ++i) wd.p[i] = bload16<kNT>(wrs, wv[i], st * 128);
    if constexpr (G32) {  // groups 8 st + 4 h .. + 3: one 16-B load
      const uint4 z4 = bload16<kNT>(zrs, zv + 16 * h, st * 32);
      wd.z[0] = z4.x;
      wd.z[1] = z4.y;
      wd.z[2] = z4.z;
      wd.z[3] = z4.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        wd.z[c] = bload4<kNT>(zrs, zv, (uint32_t)(((8 * st + 4 * h + c) >> gshift) * 4));
    }
  };
  auto store_x = [&](const uint4 (&src)[XLOADS], int j) __attribute__((always_inline)) {
    const int st = s0 + j;
    uint4* dst = xs + (j & 1) * TILE;
    if (!ragged && st < s1) {
#pragma unroll
      for (int i = 0; i < XLOADS; ++i) dst[xl[i]] = src[i];
    } else {
      const uint32_t keep = st < s1 && st * 512 + xslot * 16 < row_bytes ? ~0u : 0u;
#pragma unroll
      for (int i = 0; i < XLOADS; ++i)
        dst[xl[i]] =
            make_uint4(src[i].x & keep, src[i].y & keep, src[i].z & keep, src[i].w & keep);
    }
  };
  auto body = [&](auto uc, int j) __attribute__((always_inline)) {
    constexpr int u = decltype(uc)::value;
    load_step(j + D - 1, xr[(u + D - 1) % D], wr[(u + D - 1) % D]);
    {
      const WChunk& wc = wr[u];
#pragma unroll
      for (int i = 0; i < 4; ++i) wstage[stage_slot(8 * i + (lane >> 3), lane & 7)] = wc.p[i];
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = wstage[stage_slot(r, 4 * h + q)];
        w[4 * q] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
      }
      float sc[4], zc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sc[c] = bf16lo_to_f32(wc.z[c]);
        zc[c] = bf16hi_to_f32(wc.z[c]) - 8.f * sc[c];  // q*s + zc == (q-8)*s + z
      }
      const uint4* xb = xs + (j & 1) * TILE;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const uint32_t wd = w[s];
        const float scl = sc[s >> 2], zcl = zc[s >> 2];
        const uint32_t lo = wd & 0x0F0F0F0Fu, hi = (wd >> 4) & 0x0F0F0F0Fu;
        const f32x2_t q04 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, false);
        const f32x2_t q15 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(lo, 512.f, true);
        const f32x2_t q26 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, false);
        const f32x2_t q37 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(hi, 512.f, true);
        const f32x2_t sv = {scl, scl}, zvv = {zcl, zcl};
        const f32x2_t w04 = q04 * sv + zvv, w15 = q15 * sv + zvv;
        const f32x2_t w26 = q26 * sv + zvv, w37 = q37 * sv + zvv;
        const bf16x8_t b = as_bf16x8(pack_bf16x2(w04[0], w15[0]), pack_bf16x2(w26[0], w37[0]),
                                     pack_bf16x2(w04[1], w15[1]), pack_bf16x2(w26[1], w37[1]));
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const uint4 a = xb[lds_slot<SLOTS>(32 * t + r, 16 * h + s)];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), b,
                                                           acc[t], 0, 0, 0);
        }
      }
    }
    if (j + 1 < J) store_x(xr[(u + 1) % D], j + 1);
    __syncthreads();
  };

  static_for<0, D - 1>([&](auto i) __attribute__((always_inline)) {
    load_step(decltype(i)::value, xr[decltype(i)::value], wr[decltype(i)::value]);
  });
  store_x(xr[0], 0);
  __syncthreads();
  int j = 0;
  for (; j + D <= J; j += D)
    static_for<0, D>([&](auto uc) __attribute__((always_inline)) {
      body(uc, j + decltype(uc)::value);
    });
  static_for<0, D - 1>([&](auto uc) __attribute__((always_inline)) {
    if (j + decltype(uc)::value < J) body(uc, j + decltype(uc)::value);
  });

  const int S = gridDim.z;
  if (S > 1) {  // gemm_mfma_kernel's slab hand-off, 64-B accumulators
    const unsigned tile = blockIdx.y * gridDim.x + blockIdx.x;
    const size_t tile_bytes = (size_t)S * 4 * MT * 64 * sizeof(f32x16_t);
    const Rsrc srs = make_rsrc(reinterpret_cast<const uint8_t*>(slab) + tile * tile_bytes,
                               (uint32_t)tile_bytes);
    const uint32_t lane_off = (uint32_t)((wave * MT * 64 + lane) * sizeof(f32x16_t));
    constexpr uint32_t kZ = 4 * MT * 64 * sizeof(f32x16_t);
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        bstore16<kSC1>(srs, lane_off + t * 64 * sizeof(f32x16_t) + 16 * q, blockIdx.z * kZ,
                       make_uint4(__float_as_uint(acc[t][4 * q]), __float_as_uint(acc[t][4 * q + 1]),
                                  __float_as_uint(acc[t][4 * q + 2]),
                                  __float_as_uint(acc[t][4 * q + 3])));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool last =
        last_arriver(&cnt[tile * cs], (unsigned)S, reinterpret_cast<unsigned*>(lds), fenced);
    if (!last) return;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    for (int z = 0; z < S; ++z) {  // slices summed in slice order
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v =
              bload16<kSC1>(srs, lane_off + t * 64 * sizeof(f32x16_t) + 16 * q, z * kZ);
          acc[t][4 * q] += __uint_as_float(v.x);
          acc[t][4 * q + 1] += __uint_as_float(v.y);
          acc[t][4 * q + 2] += __uint_as_float(v.z);
          acc[t][4 * q + 3] += __uint_as_float(v.w);
        }
    }
  }

  // C/D map (32x32x16): col = lane & 31, row = (i & 3) + 8 (i >> 2) + 4 h
  if (ncol < N) {
    const float bv = bias != nullptr ? bf16_to_f32(bias[ncol]) : 0.f;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = m_blk + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (m < M) {
          float v = round_bf16(acc[t][i]);
          if (bias != nullptr) v = round_bf16(v + bv);
          y[(size_t)m * N + ncol] = f32_to_bf16(v);
        }
      }
  }
}

// Launch shape of gemm32_int4_kernel: BM 64 where it gives >= 96 tiles of 128 columns, else 32;
// K split until the grid reaches ~256 workgroups with slices of >= 4 steps (1024 k).
int launch_gemm32_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int gshift,
                       const uint16_t* bias, uint16_t* y, int M, int N, int K,
                       hipStream_t stream, int tbm = 0, int tsplits = 0) {
  const int nsteps = (K + 255) / 256;
  const long nb = (N + 127) / 128;
  int bm = (M > 32 && nb * ((M + 63) / 64) >= 96) ? 64 : 32;
  int splits = 1;
  const long tiles = nb * ((M + bm - 1) / bm);
  while (tiles * splits * 2 <= 320 && nsteps >= 4 * splits * 2 && splits < 8) splits *= 2;
  const int tb = tbm ? tbm : tuning().bm, ts = tsplits ? tsplits : tuning().splits;
  if (tb == 32 || tb == 64 || tb == 128) bm = tb;
  if (ts) splits = ts < nsteps ? ts : nsteps;
  const int sps = (nsteps + splits - 1) / splits;
  const int S = (nsteps + sps - 1) / sps;
  const dim3 grid((unsigned)nb, (unsigned)((M + bm - 1) / bm), (unsigned)S);
  f32x16_t* slab = nullptr;
  unsigned* cnt = nullptr;
  if (S > 1) {
    void* ws = nullptr;
    const size_t t = (size_t)grid.x * grid.y;
    const int rc = split_workspace(stream, t * S * bm * 128 * sizeof(float),
                                   t * tuning().cnt_stride, &ws, &cnt);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<f32x16_t*>(ws);
  }
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(x);
  const uint4* w = reinterpret_cast<const uint4*>(packed);
  const uint32_t* z = reinterpret_cast<const uint32_t*>(sz);
  auto go = [&](auto kern) {
    launch(kern, grid, dim3(256), 0, stream, xb, w, z, gshift, bias, y, M, N, K, sps, slab, cnt,
           tuning().splitk_fenced, tuning().cnt_stride);
  };
  if (bm == 128) {  // x ring: one step in flight (2 stages, one live)
    if (gshift == 0) go(gemm32_int4_kernel<128, 2, true>);
    else go(gemm32_int4_kernel<128, 2, false>);
  } else if (bm == 64) {
    if (gshift == 0) go(gemm32_int4_kernel<64, 2, true>);
    else go(gemm32_int4_kernel<64, 2, false>);
  } else {
    if (gshift == 0) go(gemm32_int4_kernel<32, 3, true>);
    else go(gemm32_int4_kernel<32, 3, false>);
  }
  return check_launch("gemm32_int4_kernel");
}

// Largest M served by the GEMV kernels (tao_tune_linear_crossover; 0 = built-in).
// Built-in crossover (experiments/bench_paths.py --crossover): the GEMV wins at M <= 2, and at
// M <= 4 for small weights; the MFMA kernel's per-M cost is nearly flat.
bool use_gemv(int64_t M, int64_t N, int64_t K) {
  const int v = tao::tuning().max_gemv_m;
  if (v > 0) return M <= v;
  return M <= 2 || (M <= 4 && N * K <= (32LL << 20));
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

// the skinny-M crossover, for the single-fetch partials entry (gemm_sf.hip), which serves only
// shapes the plain linear runs on the single-fetch kernel
bool int4_linear_takes_gemv(int64_t M, int64_t N, int64_t K) { return use_gemv(M, N, K); }

int int8_scaled_mm_launch(const int8_t* xq, const uint16_t* xs, const int8_t* wq,
                          const uint16_t* ws, const uint16_t* bias, uint16_t* y, int M, int N,
                          int K, hipStream_t stream) {
  // The LDS-staged kernel where its unsplit 64-row tiles fill >= 192 workgroups (M >= 128):
  // M = 128 N = 6144 14.9 vs 20.0 µs, M = 256 4096^2 14.8 vs 16.5, M = 512 22.5 vs 30.8; ties at
  // N >= 14336; the per-wave-column kernel keeps M = 64..128 at N = 4096 (11.8 vs 12.6 µs).
  if (use_sf(2, M, N, K, 0)) return sf_int8dyn(xq, xs, wq, ws, bias, y, M, N, K, stream);
  if (use_tile(2, M, N, K))
    return tile_int8dyn(xq, xs, wq, ws, bias, y, M, N, K, stream, tuning().tile_splits);
  const int algo = tao::tuning().gemm_algo;
  const long t64 = (long)((N + 63) / 64) * ((M + 63) / 64);
  const bool tuned = algo == 0 && tuned_shape(Int8Dyn::kPathId, M, N, K) != nullptr;
  if (K % kI8Step == 0 && !tuned && (algo == 2 || (algo == 0 && M >= 128 && t64 >= 192)))
    return launch_i8_lds(xq, xs, wq, ws, bias, y, M, N, K, algo == 0, stream);
  Int8Dyn pol;
  pol.w = reinterpret_cast<const uint4*>(wq);
  pol.wscale = ws;
  pol.xscale = xs;
  return launch_gemm(xq, pol, bias, y, M, N, K, stream);
}

}  // namespace tao

extern "C" int tao_int4wo_linear_bf16(const uint16_t* x, const uint32_t* packed,
                                      const uint16_t* sz, const uint16_t* bias, uint16_t* y,
                                      int64_t M, int64_t N, int64_t K, int64_t group_size,
                                      void* stream) {
  int rc = tao::int4_check_linear_args(x, packed, sz, y, M, N, K, group_size);
  if (rc != TAO_OK) return rc;
  if (M == 0 || N == 0) return TAO_OK;
  hipStream_t st = tao::as_stream(stream);
  if (tao::use_gemv(M, N, K))
    return tao::int4wo_gemv(x, packed, sz, bias, y, M, N, K, group_size, st);
  if (tao::use_sf(0, M, N, K, group_size))
    return tao::sf_int4(x, packed, sz, tao::gshift_of(group_size) + 5, bias, y, (int)M, (int)N,
                        (int)K, st);
  if (tao::use_tile(0, M, N, K))
    return tao::tile_int4(x, packed, sz, tao::gshift_of(group_size), bias, y, (int)M, (int)N,
                          (int)K, st, tao::tuning().tile_splits);
  if (tao::tuning().int4_mfma32 == 1)  // 32x32x16 MFMA kernel (tao_tune_int4_mfma32)
    return tao::launch_gemm32_int4(x, packed, sz, tao::gshift_of(group_size), bias, y, (int)M,
                                   (int)N, (int)K, st);
  // measured table entries with nw 32 name the 32x32x16 kernel and its (bm, splits)
  if (const tao::TunedShape* t = tao::tuned_shape(tao::Int4WO::kPathId, (int)M, (int)N, (int)K))
    if (t->nw == 32)
      return tao::launch_gemm32_int4(x, packed, sz, tao::gshift_of(group_size), bias, y, (int)M,
                                     (int)N, (int)K, st, t->bm, t->splits);
  tao::Int4WO pol;
  pol.wq = reinterpret_cast<const uint4*>(packed);
  pol.sz = reinterpret_cast<const uint32_t*>(sz);
  pol.gshift = tao::gshift_of(group_size);
  return tao::launch_gemm(x, pol, bias, y, (int)M, (int)N, (int)K, st);
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
  if (tao::use_gemv(M, N, K)) return tao::int8wo_gemv(x, w, scale, bias, y, M, N, K, st);
  if (tao::use_tile(1, M, N, K))
    return tao::tile_int8wo(x, w, scale, bias, y, (int)M, (int)N, (int)K, st,
                            tao::tuning().tile_splits);
  tao::Int8WO pol;
  pol.w = reinterpret_cast<const uint4*>(w);
  pol.scale = scale;
  return tao::launch_gemm(x, pol, bias, y, (int)M, (int)N, (int)K, st);
}

extern "C" int tao_tune_linear_crossover(int max_gemv_m) {
  TAO_CHECK_ARG(max_gemv_m >= 0 && max_gemv_m <= 8, "tune: max_gemv_m must be in [0, 8]");
  tao::tuning().max_gemv_m = max_gemv_m;
  return TAO_OK;
}

extern "C" int tao_tune_gemm_algo(int algo) {
  TAO_CHECK_ARG(algo >= 0 && algo <= 2,
                "tune: gemm algo must be 0 (auto), 1 (per-wave-column kernel only) or 2 (LDS-staged "
                "int8 kernel whenever K %% 128 == 0)");
  tao::tuning().gemm_algo = algo;
  return TAO_OK;
}

extern "C" int tao_tune_gemm_order(int order) {
  TAO_CHECK_ARG(order == 0 || order == 1,
                "tune: gemm order must be 0 (plain grid order) or 1 (XCD-grouped M tiles)");
  tao::tuning().gemm_order = order;
  return TAO_OK;
}

// Columns per wave of the MFMA GEMMs: 0 = built-in, 1 = 16, 2 = 32 (each A fragment read from
// LDS feeds two MFMAs). Calling thread only; for A/B measurement.
extern "C" int tao_tune_gemm_nw(int nw) {
  TAO_CHECK_ARG(nw >= 0 && nw <= 2, "tune: gemm nw must be 0 (auto), 1 or 2");
  tao::tuning().gemm_nw = nw;
  return TAO_OK;
}

// The measured shape table (gemm_table.inc): 0 = used (built-in), 1 = off (heuristic only).
// Calling thread only; for A/B measurement.
extern "C" int tao_tune_gemm_table(int off) {
  TAO_CHECK_ARG(off == 0 || off == 1, "tune: gemm table must be 0 (on) or 1 (off)");
  tao::tuning().gemm_table = off;
  return TAO_OK;
}

// int4 MFMA GEMM kernel: 0 = built-in (gemm_mfma_kernel), 1 = gemm32_int4_kernel (32x32x16).
// Calling thread only; for A/B measurement.

extern "C" int tao_tune_int4_mfma32(int on) {
  TAO_CHECK_ARG(on == 0 || on == 1, "tune: int4 mfma32 must be 0 or 1");
  tao::tuning().int4_mfma32 = on;
  return TAO_OK;
}

extern "C" int tao_tune_gemm_bn(int bn) {
  TAO_CHECK_ARG(bn == 0 || bn == 64 || bn == 128, "tune: LDS int8 GEMM bn must be 0, 64 or 128");
  tao::tuning().i8_bn = bn;
  return TAO_OK;
}

extern "C" int tao_tune_gemm_depth(int depth) {
  TAO_CHECK_ARG(depth == 0 || depth == 2 || depth == 3 || depth == 4 || depth == 6 || depth == 8,
                "tune: LDS int8 GEMM depth must be 0 (built-in), 2, 3, 4, 6 or 8 (8: M tile 64)");
  tao::tuning().i8_depth = depth;
  return TAO_OK;
}

extern "C" int tao_tune_gemm(int m_tile, int k_groups, int splits) {
  TAO_CHECK_ARG(m_tile == 0 || m_tile == 16 || m_tile == 32 || m_tile == 64 || m_tile == 128,
                "tune: m_tile must be 0 (auto), 16, 32, 64 or 128");
  TAO_CHECK_ARG(k_groups == 0 || k_groups == 1 || k_groups == 2 || k_groups == 4,
                "tune: k_groups must be 0 (auto), 1, 2 or 4");
  TAO_CHECK_ARG(splits >= 0 && splits <= 64, "tune: splits must be in [0, 64]");
  tao::tuning().bm = m_tile;
  tao::tuning().kg = k_groups;
  tao::tuning().splits = splits;
  return TAO_OK;
}
