// Prefill GEMM for the quantized linears at M >= 64: y[M][N] = epilogue(x[M][K] . W[N][K]^T)
// (auto-routed only where measured faster than gemm_mfma.hip, see use_tile),
// built around the bound gemm_mfma.hip measured: there every wave owned 16 columns
// and all BM rows, so each weight fragment was dequantised once per M tile. Here:
//
//   * a workgroup tile is BM (64 or 128) rows x 64 columns, 8 waves in two groups of 4: within a
//     group the waves split the ROWS (BM / 4 each), the two groups split each K step in halves
//     (group-1 accumulators are added into group 0's through LDS once, after the loop). Each
//     step's weight tile is converted ONCE per workgroup (int4 nibbles -> bf16, int8 -> bf16, by
//     waves 0-3) into an LDS B-fragment image that all 8 waves read (int8 dynamic: the int8
//     weight lines are the image);
//   * every operand reaches LDS by LDS-DMA (buffer_load ... lds, 16 B per lane): x in full
//     128-B lines (8 rows x 128 B per wave instruction) into an XOR-swizzled line image, the A
//     fragments then read by ds_read_b128 (fragment-shaped x loads, 16 rows x 64 B per
//     instruction straight to registers, measured ~2x slower through the load path in the first
//     version of this kernel; the HIP guide's projection-GEMM row agrees). Stages ring R deep;
//     counted vmcnt + raw barriers keep R - 1 steps in flight across every barrier (a
//     __syncthreads() would drain them);
//   * K may be split S ways across workgroups (S a power of two): the S partial tiles are then
//     reduced by ALL S workgroups at once, each 1/S of the tile, with a claim word per part so the
//     tile's last arriver takes over any part whose owner did not claim it (slow, or gave up
//     waiting): no workgroup waits on one that might not be resident, the grid always drains, and
//     the slab sum runs in slice order (run-to-run deterministic).
//
// Weights/format policies (same numerics as gemm_mfma.hip's Int4WO / Int8WO / Int8Dyn):
//   TInt4   : bf16 x, int4 row-stream W + (scale, zero) per group, v_mfma_f32_16x16x32_bf16,
//             B = bf16(fma(q, s, z - 8 s)), y = bf16(acc)
//   TInt8WO : bf16 x, int8 W (exact in bf16), y = bf16(bf16(acc) * scale)
//   TInt8Dyn: int8 x, int8 W, v_mfma_i32_16x16x64_i8 (exact int32),
//             y = bf16(bf16(bf16(acc) * xs) * ws) (kernel/intmm.py:133-137, plain_layout.py:301-315)
// Replaces aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104), mm(x, w.to(bf16)) * s
// (plain_layout.py:256-266) and int_scaled_matmul + scales (plain_layout.py:294-315).
#include "tao_common.h"

// The timing-only variant builds (TAO_TILE_DEBUG / TAO_TILE_STAMPS) were removed in round 6;
// their code is in git history (commit 1bac331), their measurements in profiles/r3_*.

namespace tao {
namespace {

typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

constexpr int kTileN = 64;       // columns per workgroup tile (4 blocks of 16)
constexpr int kMaxSplit = 16;    // split-K slices per tile (power of two)
constexpr int kSyncWords = 32;   // u64 per tile: [0] arrivals, [1 + p] claim epoch of part p
constexpr int kStepBytes = 256;  // x bytes per row per step (2 lines), every policy

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// LDS-DMA: 64 lanes x SIZE bytes from per-lane buffer offsets into LDS at the wave-uniform
// `dst` + lane x SIZE (lane-linear). Issued by inline asm: with the intrinsic, hipcc treats every
// pending DMA as a possible writer of any LDS a later ds_read touches and waits vmcnt(0) before
// the first read of every step (it cannot tell the stages of the one LDS array apart), which
// drains the ring. The asm form is invisible to its wait pass; this kernel waits for its DMAs by
// hand (counted vmcnt before each barrier). The compiler's own waits for ordinary loads stay
// correct beside it (unknown VM ops can only make a counted wait stricter). M0 is saved and
// restored around the load (the cdna guide's LDS-DMA recipe).
template <int SIZE, int AUX = 0>
__device__ __forceinline__ void glds(Rsrc r, uint32_t voff, uint32_t soff, uint4* dst) {
  static_assert((SIZE == 16 || SIZE == 4) && (AUX == 0 || AUX == kNT), "glds: 16 / 4 B, nt or not");
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_ptr_t)dst;
  uint32_t keep;
  if constexpr (SIZE == 16 && AUX == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
  else if constexpr (SIZE == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
  else if constexpr (AUX == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dword %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dword %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- line images --------------------------------------------------------------------------------
// A step of ROWS rows x 256 B as [2 lines][ROWS][8 x 16-B chunks], chunk c of row r stored at
// position c ^ ((r >> 1) & 7). Filled by LDS-DMA pieces of 8 rows x one 128-B line (lane l: row
// 8 g + l / 8, position l % 8, so it fetches chunk (l % 8) ^ swz); the A / B fragment reads
// (lane (r, kq): row r of a 16-row block, chunk 4 (kb & 1) + kq of line kb >> 1) hit 16 distinct
// bank groups per ds_read_b128 lane group (checked exhaustively).
__device__ __forceinline__ int line_slot(int rows, int h, int row, int c) {
  return (h * rows + row) * 8 + (c ^ ((row >> 1) & 7));
}

// ---- int4 ----------------------------------------------------------------------------------------
// Raw W per step and wave: 16 rows x 64 B of nibbles (lane l: row 16 w + l % 16, 32-k piece l / 16)
// and the (scale, zero) dword of that piece's group; the same lane converts its piece into the
// bf16 B image (fragment (kb = l / 16, nb = w), slot 16 d + (r ^ 2 kb)).
struct TInt4 {
  static constexpr int kABytes = 2;  // bf16 x
  static constexpr int kKS = 128;    // k per step (256 B of x, 64 B of nibbles per row)
  static constexpr int kKB = 4;      // 32-k MFMA blocks per step
  static constexpr bool kImageW = false;
  static constexpr int kWGlds = 2;         // LDS-DMA instructions per wave per step
  static constexpr int kRawU4 = 256 + 64;  // raw W per stage (uint4): 4 KiB nibbles + 1 KiB sz
  typedef f32x4_t Acc;
  const uint4* wq;     // [N][K/32] 16-B pieces
  const uint32_t* sz;  // [N][K/g] (scale, zero) bf16 pairs
  int gshift;          // log2(g / 32)
  struct Lane {
    Rsrc w, z;
    uint32_t wv, zv;
  };
  __device__ __forceinline__ Lane setup(int n_blk, int wave, int lane, int N, int K) const {
    Lane L;
    int n = n_blk + 16 * wave + (lane & 15);
    n = n < N ? n : N - 1;
    const int c = lane >> 4;
    const uint32_t zrow = (uint32_t)(K >> 5 >> gshift);
    L.w = make_rsrc(wq, (uint32_t)N * (uint32_t)(K >> 1));
    L.z = make_rsrc(sz, (uint32_t)N * zrow * 4u);
    L.wv = (uint32_t)n * (uint32_t)(K >> 1) + 16u * c;
    // group of k = 128 st + 32 c is ((4 st) >> gshift) + (c >> gshift) for gshift <= 3
    L.zv = ((uint32_t)n * zrow + (uint32_t)(c >> gshift)) * 4u;
    return L;
  }
  __device__ __forceinline__ void issue(const Lane& L, int st, int wave, uint4* raw) const {
    glds<16, kNT>(L.w, L.wv, (uint32_t)st * 64u, raw + wave * 64);
    glds<4, kNT>(L.z, L.zv, (uint32_t)(((4 * st) >> gshift) * 4), raw + 256 + wave * 16);
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
  __device__ __forceinline__ void convert(const uint4* raw, uint4* img, int wave, int lane) const {
    const uint4 q = raw[wave * 64 + lane];
    const uint32_t sv = reinterpret_cast<const uint32_t*>(raw + 256)[wave * 64 + lane];
    const int r = lane & 15, kb = lane >> 4;
    const float s = bf16lo_to_f32(sv);
    const float zc = bf16hi_to_f32(sv) - 8.f * s;  // q * s + zc == (q - 8) * s + z
    const uint32_t d4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint4 v = dq8(d4[d], s, zc);
      img[(kb * 4 + wave) * 64 + 16 * d + (r ^ (2 * kb))] = v;
    }
  }
  static __device__ __forceinline__ int rslot(int lane, int kb) {
    return 16 * (lane >> 4) + ((lane & 15) ^ (2 * kb));
  }
  static __device__ __forceinline__ Acc mfma(const uint4& a, const uint4& b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
  __device__ __forceinline__ const void* image_base() const { return nullptr; }
  static constexpr bool kRowF = false, kColF = false;
  __device__ __forceinline__ const uint16_t* row_factor() const { return nullptr; }
  __device__ __forceinline__ const uint16_t* col_factor() const { return nullptr; }
  static __device__ __forceinline__ float epi(float acc, float, float) { return round_bf16(acc); }
};

// ---- int8 weight-only ----------------------------------------------------------------------------
// Raw W per step and wave: 16 rows x 128 B (two DMA pieces of 16 rows x 64 B: lane l row
// 16 w + l % 16, chunk l / 16); the lane converts its two 16-k pieces (int8 -> bf16, exact).
struct TInt8WO {
  static constexpr int kABytes = 2;
  static constexpr int kKS = 128;
  static constexpr int kKB = 4;
  static constexpr bool kImageW = false;
  static constexpr int kWGlds = 2;
  static constexpr int kRawU4 = 512;  // 8 KiB
  typedef f32x4_t Acc;
  const uint8_t* w;       // [N][K]
  const uint16_t* scale;  // [N]
  struct Lane {
    Rsrc w;
    uint32_t wv;
  };
  __device__ __forceinline__ Lane setup(int n_blk, int wave, int lane, int N, int K) const {
    Lane L;
    int n = n_blk + 16 * wave + (lane & 15);
    n = n < N ? n : N - 1;
    L.w = make_rsrc(w, (uint32_t)N * (uint32_t)K);
    L.wv = (uint32_t)n * (uint32_t)K + 16u * (lane >> 4);
    return L;
  }
  __device__ __forceinline__ void issue(const Lane& L, int st, int wave, uint4* raw) const {
    glds<16, kNT>(L.w, L.wv, (uint32_t)st * 128u, raw + wave * 128);
    glds<16, kNT>(L.w, L.wv, (uint32_t)st * 128u + 64u, raw + wave * 128 + 64);
  }
  static __device__ __forceinline__ uint2 cv4(uint32_t d) {
    // 4 int8 -> 4 bf16 (exact): byte ^ 0x80 = q + 128 unsigned, minus 128 in f32
    const uint32_t u = d ^ 0x80808080u;
    auto f = [&](int b) { return (float)((u >> (8 * b)) & 0xFF) - 128.f; };
    return make_uint2(pk_bf16(f(0), f(1)), pk_bf16(f(2), f(3)));
  }
  __device__ __forceinline__ void convert(const uint4* raw, uint4* img, int wave, int lane) const {
    const int r = lane & 15, c = lane >> 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint4 q = raw[wave * 128 + i * 64 + lane];
      const int kb = 2 * i + (c >> 1);
      const uint32_t d4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int d = 2 * (c & 1) + h;
        const uint2 a = cv4(d4[2 * h]), b = cv4(d4[2 * h + 1]);
        const uint4 o = make_uint4(a.x, a.y, b.x, b.y);
        img[(kb * 4 + wave) * 64 + 16 * d + (r ^ ((2 * kb + (c & 1)) & 7))] = o;
      }
    }
  }
  static __device__ __forceinline__ int rslot(int lane, int kb) {
    const int kq = lane >> 4;
    return 16 * kq + ((lane & 15) ^ ((2 * kb + (kq >> 1)) & 7));
  }
  static __device__ __forceinline__ Acc mfma(const uint4& a, const uint4& b, Acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  }
  __device__ __forceinline__ const void* image_base() const { return nullptr; }
  static constexpr bool kRowF = false, kColF = true;
  __device__ __forceinline__ const uint16_t* row_factor() const { return nullptr; }
  __device__ __forceinline__ const uint16_t* col_factor() const { return scale; }
  static __device__ __forceinline__ float epi(float acc, float, float sc) {
    return round_bf16(round_bf16(acc) * sc);
  }
};

// ---- int8 dynamic activation ---------------------------------------------------------------------
// W needs no conversion: its 64 rows x 256 B per step land as a line image like x (4 DMA pieces
// per wave), and the B fragments are read from it.
struct TInt8Dyn {
  static constexpr int kABytes = 1;
  static constexpr int kKS = 256;
  static constexpr int kKB = 4;  // 64-k MFMA blocks
  static constexpr bool kImageW = true;
  static constexpr int kWGlds = 4;
  static constexpr int kRawU4 = kTileN * 16;  // 16 KiB line image
  typedef i32x4_t Acc;
  const uint8_t* w;
  const uint16_t* wscale;  // [N]
  const uint16_t* xscale;  // [M]
  struct Lane {
    Rsrc w;
    uint32_t wv[4];
  };
  __device__ __forceinline__ Lane setup(int n_blk, int wave, int lane, int N, int K) const {
    Lane L;
    L.w = make_rsrc(w, (uint32_t)N * (uint32_t)K);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = wave * 4 + i, h = p >> 3, rg = p & 7;
      const int row = 8 * rg + (lane >> 3);
      int n = n_blk + row;
      n = n < N ? n : N - 1;
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      L.wv[i] = (uint32_t)n * (uint32_t)K + 128u * h + 16u * c;
    }
    return L;
  }
  __device__ __forceinline__ void issue(const Lane& L, int st, int wave, uint4* raw) const {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      glds<16, kNT>(L.w, L.wv[i], (uint32_t)st * 256u, raw + (wave * 4 + i) * 64);
  }
  __device__ __forceinline__ void convert(const uint4*, uint4*, int, int) const {}
  __device__ __forceinline__ const void* image_base() const { return w; }
  static __device__ __forceinline__ int rslot(int, int) { return 0; }
  static __device__ __forceinline__ Acc mfma(const uint4& a, const uint4& b, Acc c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4_t, a),
                                                 __builtin_bit_cast(i32x4_t, b), c, 0, 0, 0);
  }
  static constexpr bool kRowF = true, kColF = true;
  __device__ __forceinline__ const uint16_t* row_factor() const { return xscale; }
  __device__ __forceinline__ const uint16_t* col_factor() const { return wscale; }
  static __device__ __forceinline__ float epi(int acc, float xs, float ws) {
    const float v = round_bf16(round_bf16((float)acc) * xs);
    return round_bf16(v * ws);
  }
};

// ---- the kernel ---------------------------------------------------------------------------------

// LDS: an x ring of R stages, a deeper weight ring (the weights come from HBM: their round trip
// is the long one, and their stages are small) of RW stages, and two B images when the weights are
// converted.
template <int BM, int R, class P>
struct TileLds {
  static constexpr int kX = BM * 16;                        // uint4 per x stage
  static constexpr int kW = P::kRawU4;                      // uint4 per raw-W stage
  static constexpr int kImg = P::kImageW ? 0 : 4 * 4 * 64;  // uint4 per B image (16 fragments)
  static constexpr int kCap = 160 * 1024 / 16;
  static constexpr int kRWFit = (kCap - R * kX - 2 * kImg) / kW;
  static constexpr int RW = kRWFit > 8 ? 8 : kRWFit;
  static constexpr int kTotal = R * kX + RW * kW + 2 * kImg;
  static_assert(RW >= R, "weight ring at least as deep as the x ring");
  static_assert(kTotal <= kCap, "LDS budget");
};

// grid (S, ceil(N / 64), ceil(M / BM)): the S K-slices of a tile are adjacent in dispatch order.
// 512 threads = 8 waves, two per SIMD so one wave's MFMAs cover the other's LDS round trips:
// wave (g = w / 4, wm = w % 4) owns rows wm BM/4 .. of the tile, all 64 columns, and the k-blocks
// of line g of every step (MT x 4 accumulator tiles); the two groups' sums meet in LDS at the end.
template <int BM, int R, class P>
__global__ __launch_bounds__(512) void gemm_tile_kernel(
    const uint8_t* __restrict__ x, P pol, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int M, int N, int K, int sps, typename P::Acc* __restrict__ slab,
    unsigned long long* __restrict__ sync, int fenced) {
  typedef typename P::Acc Acc;
  typedef TileLds<BM, R, P> L;
  constexpr int NW = 8;
  constexpr int MT = BM / 64;   // 16-row subtiles per wave
  constexpr int NT = 16 * MT;   // accumulator tiles per workgroup tile
  constexpr int PX = BM / 4;    // x DMA pieces per step (8 rows x 128 B each)
  // DMA instructions per wave per step (equal for every wave: the counted waits rely on it).
  // Converted weights: waves 0-3 issue their 16 columns' raw W (kWGlds) and fewer x pieces.
  // Line-image weights: x and W pieces dealt out evenly.
  constexpr int NG = P::kImageW ? PX / NW + 2 : (PX + 4 * P::kWGlds) / NW;
  static_assert(P::kImageW ? PX % NW == 0 : (PX + 4 * P::kWGlds) % NW == 0, "DMA split");
  static_assert(NG <= 8, "DMA pieces per wave");
  // ALL LDS in one array (a second __shared__ object can make hipcc wait vmcnt(0) before the
  // ds_reads of every step: cdna guide, projection GEMM item 4a)
  __shared__ uint4 lds[L::kTotal];
  uint4* const xs0 = lds;
  constexpr int RW = L::RW;
  uint4* const ws0 = lds + R * L::kX;
  uint4* const img0 = lds + R * L::kX + RW * L::kW;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wm = wave & 3;
  const int S = gridDim.x, z = blockIdx.x;
  const int n_blk = blockIdx.y * kTileN, m_blk = blockIdx.z * BM;
  const int nsteps = K / P::kKS;
  const int s0 = z * sps;
  const int s1 = s0 + sps < nsteps ? s0 + sps : nsteps;  // launcher: no empty slice
  const int J = s1 - s0;

  // epilogue operands, one per thread, loaded before any DMA and first used after the k loop (the
  // raw bf16 is kept, so no wait for it precedes the DMAs): [0, BM) row factors, [BM, BM + 64)
  // column factors, [BM + 64, BM + 128) bias
  const uint16_t* fsrc = reinterpret_cast<const uint16_t*>(x);  // any readable address
  uint32_t fdef = 0x3F80u;                                      // bf16 1.0
  if (tid < BM) {
    const int m = m_blk + tid;
    if (P::kRowF) fsrc = pol.row_factor() + (m < M ? m : M - 1);
  } else if (tid < BM + 64) {
    const int n = n_blk + tid - BM;
    if (P::kColF) fsrc = pol.col_factor() + (n < N ? n : N - 1);
  } else {
    const int n = n_blk + tid - BM - 64;
    if (bias != nullptr) fsrc = bias + (n < N ? n : N - 1);
    fdef = 0;
  }
  const bool fload = (tid < BM && P::kRowF) || (tid >= BM && tid < BM + 64 && P::kColF) ||
                     (tid >= BM + 64 && bias != nullptr);
  const uint32_t fac_raw = *fsrc;  // unconditional: no branch joins the value before its use

  // this wave's DMA pieces (fixed per wave, no branch per piece): x pieces q = x0 + i (line
  // q / (BM / 8), rows 8 (q % (BM / 8)) ..); line-image weights: pieces qw = 2 wave + i of the
  // 64-row x 256-B weight step; converted weights: waves 0-3 issue their 16 columns' raw W
  // (kWGlds) and XC x pieces, waves 4-7 NG x pieces.
  const uint32_t row_bytes = (uint32_t)K * P::kABytes;
  const Rsrc xrs = make_rsrc(x, (uint32_t)M * row_bytes);
  constexpr int XI = P::kImageW ? PX / NW : NG;       // x pieces per wave (image / waves 4-7)
  constexpr int XC = P::kImageW ? XI : NG - P::kWGlds;  // x pieces of the converting waves 0-3
  const bool wconv = !P::kImageW && wave < 4;           // converts its 16 columns' weights
  const int x0 = P::kImageW ? wave * XI : (wave < 4 ? wave * XC : 4 * XC + (wave - 4) * XI);
  uint32_t xv[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int q = x0 + i < PX ? x0 + i : PX - 1;  // (waves 0-3 use only XC of them)
    const int h = q / (BM / 8), rg = q % (BM / 8);
    const int row = 8 * rg + (lane >> 3);
    const int m = m_blk + row < M ? m_blk + row : M - 1;
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    xv[i] = (uint32_t)m * row_bytes + 128u * h + 16u * c;
  }
  const Rsrc wrs = make_rsrc(P::kImageW ? pol.image_base() : nullptr,
                             P::kImageW ? (uint32_t)N * (uint32_t)K : 0u);
  uint32_t wv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int qw = 2 * wave + i, h = qw >> 3, rg = qw & 7;
    const int row = 8 * rg + (lane >> 3);
    const int n = n_blk + row < N ? n_blk + row : N - 1;
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    wv[i] = (uint32_t)n * (uint32_t)K + 128u * h + 16u * c;
  }
  const typename P::Lane wl = pol.setup(n_blk, wm, lane, N, K);

  // step j's x into x stage j % R, step j's weights into weight stage j % RW; the weights of a
  // step are always issued before its x (so waiting for a step's x also covers its weights)
  auto issue_w = [&](int j) __attribute__((always_inline)) {
    const int st = s0 + j < s1 ? s0 + j : s1 - 1;  // past the slice: re-read (uniform counts)
    uint4* wsg = ws0 + (j % RW) * L::kW;
    const uint32_t so = (uint32_t)st * kStepBytes;
    if constexpr (P::kImageW) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        glds<16, kNT>(wrs, wv[i], so, wsg + (2 * wave + i) * 64);
    } else {
      if (wconv) pol.issue(wl, st, wm, wsg);
    }
  };
  auto issue_x = [&](int j) __attribute__((always_inline)) {
    const int st = s0 + j < s1 ? s0 + j : s1 - 1;
    uint4* xs = xs0 + (j % R) * L::kX;
    const uint32_t so = (uint32_t)st * kStepBytes;
    if (P::kImageW || !wconv) {
#pragma unroll
      for (int i = 0; i < XI; ++i)
        glds<16>(xrs, xv[i], so, xs + (x0 + i) * 64);
    } else {
#pragma unroll
      for (int i = 0; i < XC; ++i)
        glds<16>(xrs, xv[i], so, xs + (x0 + i) * 64);
    }
  };
  // this wave's DMAs of the next step have landed (the wave's DMA count per step is fixed)
  auto wait_next = [&]() __attribute__((always_inline)) {
    wait_vm<(R - 2) * NG>();
  };

  Acc acc[MT][4];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[t][nb] = Acc{0, 0, 0, 0};

  const int arow = wm * (BM / 4) + (lane & 15);  // + 16 t
  // the group's two k-blocks (line grp of the step); every fragment read before the first MFMA
  auto compute = [&](int j) __attribute__((always_inline)) {
    const uint4* xs = xs0 + (j % R) * L::kX;
    const uint4* wsg = ws0 + (j % RW) * L::kW;
    const uint4* img = img0 + (j & 1) * L::kImg;
    uint4 b[2][4], a[2][MT];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kb = 2 * grp + u, c = 4 * u + (lane >> 4);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        if constexpr (P::kImageW)
          b[u][nb] = wsg[line_slot(kTileN, grp, 16 * nb + (lane & 15), c)];
        else
          b[u][nb] = img[(kb * 4 + nb) * 64 + P::rslot(lane, kb)];
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) a[u][t] = xs[line_slot(BM, grp, arow + 16 * t, c)];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          acc[t][nb] = P::mfma(a[u][t], b[u][nb], acc[t][nb]);
        }
  };

  // prologue: weights of steps 0 .. RW - 2 and x of steps 0 .. R - 2 in flight; step 0 landed
  // (this wave's DMAs, then everyone's)
  for (int j = 0; j < RW - 1; ++j) issue_w(j);
  for (int j = 0; j < R - 1; ++j) issue_x(j);
  // step 0's x landed: only x of steps 1 .. R - 2 may be younger (the weights were issued first)
  if (P::kImageW || !wconv) {
    wait_vm<(R - 2) * XI>();
  } else {
    wait_vm<(R - 2) * XC>();
  }
  if constexpr (!P::kImageW) {
    if (wconv) pol.convert(ws0, img0, wm, lane);
  }
  raw_barrier();
  for (int j = 0; j < J; ++j) {
    issue_w(j + RW - 1);
    issue_x(j + R - 1);
    compute(j);
    wait_next();  // this wave's DMAs of step j + 1 landed (its weights were issued earlier still)
    if constexpr (!P::kImageW) {
      if (wconv && j + 1 < J)
        pol.convert(ws0 + ((j + 1) % RW) * L::kW, img0 + ((j + 1) & 1) * L::kImg, wm, lane);
    }
    raw_barrier();
  }
  wait_vm<0>();  // the clamped re-reads past the slice
  __syncthreads();
  // group 1 hands its sums to group 0 (added in group order); the epilogue operand table -> LDS
  {
    Acc* red = reinterpret_cast<Acc*>(lds + 256);
    if (grp == 1) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) red[((wm * MT + t) * 4 + nb) * 64 + lane] = acc[t][nb];
    }
    float* const ft = reinterpret_cast<float*>(lds);
    if (tid < BM + 128) ft[tid] = bf16_to_f32(fload ? fac_raw : fdef);
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[t][nb] += red[((wm * MT + t) * 4 + nb) * 64 + lane];
    }
  }
  const float* const ftab = reinterpret_cast<const float*>(lds);

  // ---- epilogue of one 16 x 16 accumulator tile: rows r0 + 4 (lane >> 4) + i, column c0 + lane % 16
  auto emit = [&](const Acc& v, int r0, int c0) __attribute__((always_inline)) {
    const int col = n_blk + c0 + (lane & 15);
    if (col >= N) return;
    const float cf = ftab[BM + c0 + (lane & 15)];
    const float bv = ftab[BM + 64 + c0 + (lane & 15)];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = r0 + 4 * (lane >> 4) + i, m = m_blk + rl;
      if (m < M) {
        float o = P::epi(v[i], ftab[rl], cf);
        if (bias != nullptr) o = round_bf16(o + bv);
        y[(size_t)m * N + col] = f32_to_bf16(o);
      }
    }
  };

  if (S == 1) {
    if (grp == 0) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) emit(acc[t][nb], wm * (BM / 4) + 16 * t, 16 * nb);
    }
    return;
  }

  // ---- split-K: every slice publishes its partial tile, then the parts are reduced --------------
  // Slab of tile T: [S][NT accumulator tiles][64 lanes] x 16 B; accumulator tile
  // idx = (wm MT + t) 4 + nb. Stores and loads all sc1, every storing wave drains (vmcnt(0))
  // before the barrier, one lane adds the arrival (MI355X_MICROARCH.md hand-off table, first row:
  // agent-scope add, the consumer told by an sc1 poll or by the value its add returned).
  const unsigned tile = blockIdx.y + gridDim.y * blockIdx.z;
  const uint32_t tile_bytes = (uint32_t)S * NT * 64 * 16;
  const Rsrc srs =
      make_rsrc(reinterpret_cast<const uint8_t*>(slab) + (size_t)tile * tile_bytes, tile_bytes);
  if (grp == 0) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int idx = (wm * MT + t) * 4 + nb;
        bstore16<kSC1>(srs, (uint32_t)(idx * 64 + lane) * 16u, (uint32_t)z * NT * 1024u,
                       __builtin_bit_cast(uint4, acc[t][nb]));
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned long long* tsync = sync + (size_t)tile * kSyncWords;
  // flag words after the epilogue table: [0] last, [1..2] epoch, [3] go, [4 + p] last's claims
  unsigned* word = reinterpret_cast<unsigned*>(lds) + 512;
  if (tid == 0) {
    if (fenced) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // arrivals advance by 64 per launch whatever S (S | 64): the base of this launch's tickets is
    // a multiple of 64 and the epoch numbers the launch for the claim words (never reset)
    const unsigned long long t =
        __hip_atomic_fetch_add(&tsync[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long base = t & ~63ull;
    const bool last = (t & 63ull) == (unsigned long long)(S - 1);
    if (last)
      (void)__hip_atomic_fetch_add(&tsync[0], (unsigned long long)(64 - S), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long epoch = (base >> 6) + 1;
    unsigned go = 0;
    if (last) {
      go = 1;
    } else {
      // wait (bounded) for the other slices, then claim this slice's part
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const unsigned long long v =
            __hip_atomic_load(&tsync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v - base >= (unsigned long long)S) {
          go = 1;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000) break;  // 20 µs: leave it to the last
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (go) {
      if (fenced) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const unsigned long long prev = __hip_atomic_fetch_max(&tsync[1 + z], epoch, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
      go = prev < epoch ? 1u : 0u;
    }
    word[0] = last ? 1u : 0u;
    word[1] = (unsigned)epoch;
    word[2] = (unsigned)(epoch >> 32);
    word[3] = go;
  }
  __syncthreads();
  const bool last = word[0] != 0;
  const unsigned long long epoch = ((unsigned long long)word[2] << 32) | word[1];
  const int per = NT / S;  // accumulator tiles per part
  // every slab load of an accumulator tile in flight before the first add (no per-load branch:
  // the slice count is dispatched to a constant), summed in slice order
  auto reduce_part = [&](int p) __attribute__((always_inline)) {
    auto run = [&](auto sc) __attribute__((always_inline)) {
      constexpr int SS = decltype(sc)::value;
      for (int i = wave; i < per; i += NW) {
        const int idx = p * per + i;
        const uint32_t off = (uint32_t)(idx * 64 + lane) * 16u;
        uint4 v[SS];
#pragma unroll
        for (int zz = 0; zz < SS; ++zz) v[zz] = bload16<kSC1>(srs, off, (uint32_t)zz * NT * 1024u);
        Acc sum = Acc{0, 0, 0, 0};
#pragma unroll
        for (int zz = 0; zz < SS; ++zz) sum += __builtin_bit_cast(Acc, v[zz]);
        const int src = idx / (4 * MT), t = (idx >> 2) % MT, nb = idx & 3;
        emit(sum, src * (BM / 4) + 16 * t, 16 * nb);
      }
    };
    switch (S) {
      case 2: run(std::integral_constant<int, 2>{}); break;
      case 4: run(std::integral_constant<int, 4>{}); break;
      case 8: run(std::integral_constant<int, 8>{}); break;
      default: run(std::integral_constant<int, 16>{}); break;
    }
  };
  if (word[3]) reduce_part(z);
  if (!last) return;
  // the last arriver: claim, in one round trip, every part whose owner has not claimed it
  if (tid < S && tid != z)
    word[4 + tid] = __hip_atomic_fetch_max(&tsync[1 + tid], epoch, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) < epoch ? 1u : 0u;
  __syncthreads();
  for (int p = 0; p < S; ++p)
    if (p != z && word[4 + p]) reduce_part(p);
}

}  // namespace

// Routing (path 0 int4, 1 int8 weight-only, 2 int8 dynamic); callers have already sent M at or
// below the GEMV crossover to the GEMVs.
bool use_tile(int path, int64_t M, int64_t N, int64_t K) {
  const int mode = tuning().gemm_tile;
  const int ks = path == 2 ? TInt8Dyn::kKS : TInt4::kKS;
  if (mode == 1 || K % ks != 0 || M > (1 << 20) || N > (1 << 24)) return false;
  if (mode == 2) return true;
  // an explicit override of the older kernels' launch shapes keeps them (their tests and sweeps)
  const Tuning& t = tuning();
  if (t.bm || t.kg || t.splits || t.gemm_nw || t.int4_mfma32 || t.gemm_algo) return false;
  // auto: only where profiles/r3_ab_tile.jsonl measured this kernel ahead of gemm_mfma.hip's —
  // int8 dynamic with a long reduction (K >= 8192: 1.09-1.16x at M 128..512). Everywhere else
  // this kernel ran at 0.5-0.99x of the older kernels' speed.
  return path == 2 && K >= 8192 && M >= 128;
}

// ---- launcher ------------------------------------------------------------------------------------
// Tile rows BM = 64 at M <= 64, else 128; split-K S (power of two, <= 16, >= 2 steps per slice)
// until the grid reaches ~one workgroup per CU.
template <class P>
int launch_tile(const void* x, const P& pol, const uint16_t* bias, uint16_t* y, int M, int N,
                int K, hipStream_t stream, int force_splits) {
  TAO_CHECK_ARG(K % P::kKS == 0, "tile GEMM: K (%d) must be a multiple of %d", K, P::kKS);
  const int nsteps = K / P::kKS;
  const int bm = M <= 64 ? 64 : 128;
  const long tiles = (long)((N + kTileN - 1) / kTileN) * ((M + bm - 1) / bm);
  int S = 1;
  if (force_splits > 0) {
    while (S * 2 <= force_splits && S * 2 <= kMaxSplit && nsteps >= 2 * S * 2) S *= 2;
  } else {
    while (tiles * S < 224 && S * 2 <= kMaxSplit && nsteps >= 2 * S * 2) S *= 2;
  }
  const int sps = (nsteps + S - 1) / S;
  const dim3 grid((unsigned)S, (unsigned)((N + kTileN - 1) / kTileN), (unsigned)((M + bm - 1) / bm));
  typename P::Acc* slab = nullptr;
  unsigned long long* sync = nullptr;
  if (S > 1) {
    const size_t ntiles = (size_t)grid.y * grid.z;
    void* ws = nullptr;
    const int rc = split_workspace_epoch(stream, ntiles * S * (bm / 64) * 16 * 1024,
                                         ntiles * kSyncWords, &ws, &sync);
    if (rc != TAO_OK) return rc;
    slab = reinterpret_cast<typename P::Acc*>(ws);
  }
  const uint8_t* xb = reinterpret_cast<const uint8_t*>(x);
  const int fenced = tuning().splitk_fenced;
  if (bm == 64)
    launch(gemm_tile_kernel<64, 3, P>, grid, dim3(512), 0, stream, xb, pol, bias, y, M, N, K, sps,
           slab, sync, fenced);
  else
    launch(gemm_tile_kernel<128, 3, P>, grid, dim3(512), 0, stream, xb, pol, bias, y, M, N, K, sps,
           slab, sync, fenced);
  return check_launch("gemm_tile_kernel");
}

int tile_int4(const uint16_t* x, const uint32_t* packed, const uint16_t* sz, int gshift,
              const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
              int splits) {
  TInt4 pol;
  pol.wq = reinterpret_cast<const uint4*>(packed);
  pol.sz = reinterpret_cast<const uint32_t*>(sz);
  pol.gshift = gshift;
  return launch_tile(x, pol, bias, y, M, N, K, stream, splits);
}

int tile_int8wo(const uint16_t* x, const int8_t* w, const uint16_t* scale, const uint16_t* bias,
                uint16_t* y, int M, int N, int K, hipStream_t stream, int splits) {
  TInt8WO pol;
  pol.w = reinterpret_cast<const uint8_t*>(w);
  pol.scale = scale;
  return launch_tile(x, pol, bias, y, M, N, K, stream, splits);
}

int tile_int8dyn(const int8_t* xq, const uint16_t* xs, const int8_t* wq, const uint16_t* ws,
                 const uint16_t* bias, uint16_t* y, int M, int N, int K, hipStream_t stream,
                 int splits) {
  TInt8Dyn pol;
  pol.w = reinterpret_cast<const uint8_t*>(wq);
  pol.wscale = ws;
  pol.xscale = xs;
  return launch_tile(xq, pol, bias, y, M, N, K, stream, splits);
}

}  // namespace tao


extern "C" int tao_tune_gemm_tile(int mode, int splits) {
  TAO_CHECK_ARG(mode >= 0 && mode <= 2, "tune: gemm tile mode must be 0 (auto), 1 (off) or 2 (on)");
  TAO_CHECK_ARG(splits >= 0 && splits <= 64, "tune: tile splits must be in [0, 64]");
  tao::tuning().gemm_tile = mode;
  tao::tuning().tile_splits = splits;
  return TAO_OK;
}
