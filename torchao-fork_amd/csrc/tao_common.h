// Shared helpers for the gfx950 kernels behind include/torchao_mi355x.h.
// Internal header: not part of the C-ABI.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/torchao_mi355x.h"
#include "../../include/torchao_mi355x_llama.h"
#include "../../include/torchao_mi355x_tune.h"

namespace tao {

// ---- error reporting (defined in capi.cpp) ------------------------------------------------
int set_error(int code, const char* fmt, ...);
void clear_error();

#define TAO_CHECK_ARG(cond, ...)                                             \
  do {                                                                       \
    if (!(cond)) return ::tao::set_error(TAO_ERR_INVALID_ARGUMENT, __VA_ARGS__); \
  } while (0)

#define TAO_CHECK_ALIGN(ptr, bytes, name)                                            \
  TAO_CHECK_ARG((reinterpret_cast<uintptr_t>(ptr) % (bytes)) == 0,                   \
                "%s must be %d-byte aligned (got %p)", name, (int)(bytes), (const void*)(ptr))

// Check the launch of the kernel just enqueued (no synchronisation: capture-safe).
int check_launch(const char* what);
const char* last_kernel();  // name given to the last successful check_launch of this thread

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- split-K workspace (capi.cpp) ------------------------------------------------------------
// Scratch for the partial-sum slabs of split-K launches plus zeroed counter arrays: `cnt` (u32
// tickets, each reset by its tile's last arriver: gemm_mfma.hip) or `sync` (u64 epoch counters and
// claim words, never reset: gemm_tile.hip). Eager calls use one workspace per (device, stream),
// grown after a synchronisation of that stream (nothing else ever holds its pointers). A graph
// capture gets a workspace of its own, per capture sequence, allocated during the capture (relaxed
// capture mode) and owned by the graph through a user object: a replay never shares scratch with
// eager work or another graph, and the buffers are released when the graph is destroyed.
int split_workspace(hipStream_t stream, size_t slab_bytes, size_t counters, void** slab,
                    unsigned** cnt);
int split_workspace_epoch(hipStream_t stream, size_t slab_bytes, size_t sync_words, void** slab,
                          unsigned long long** sync);
int graph_workspace_count();

// ---- launch-shape overrides (tao_tune_*, tao_tune_reset) --------------------------------------
// Zero means "built-in choice". Thread-local: a tao_tune_* call re-routes only launches issued
// from the calling thread, and tao_tune_reset() (torchao.kernel.tuning() on exit) restores the
// built-in shapes, so sweeps cannot re-route another thread's model.
// The fence-free split-K hand-off (last_arriver, fenced == 0) rests on sc1 stores / loads as
// measured on gfx950 under the HIP runtimes this library was validated with (torch's bundled 7.0
// and /opt/rocm's 7.2). Under any other runtime major.minor the fenced form is the
// default instead.
bool fence_free_validated();

struct Tuning {
  int rpw = 0, wk = 0, g = 0, occ = 0;           // int4 GEMV (tao_tune_int4_gemv)
  int xlds = 0, norm = 0;                        // int4 GEMV x staging / deferred norm
  int bm = 0, kg = 0, splits = 0;                // MFMA GEMM (tao_tune_gemm)
  int gemm_algo = 0, i8_depth = 0, i8_bn = 0;    // int8 LDS GEMM
  int max_gemv_m = 0;                            // GEMV <-> MFMA crossover
  int i8_rpw = 0, i8_wk = 0, i8_g = 0;           // int8 GEMVs (tao_tune_int8_gemv)
  int attn_mode = 0;                             // decode attention (tao_tune_attn)
  int splitk_fenced = fence_free_validated() ? 0 : 1;  // split-K hand-off with agent fences
  int gemm_order = 0;                            // MFMA GEMM tile order: 0 plain, 1 XCD-grouped
  int gemm_nw = 0;                               // MFMA GEMM 16-col blocks per wave: 0 auto, 1, 2
  int gemm_table = 0;                            // MFMA GEMM measured-shape table: 0 on, 1 off
  int int4_mfma32 = 0;                           // int4 GEMM on 32x32x16 MFMAs: 0 off, 1 on
  int quant_block = 0;                           // per-token int8 quant: 0 wave kernel, 1 block
  int gemm_tile = 0, tile_splits = 0;            // weight-shared tile GEMM: 0 auto, 1 off, 2 on
  int gemm_sf = 0;                               // single-fetch GEMM: 0 auto, 1 off, 2 on
  int sf_bn = 0, sf_wm = 0, sf_splits = 0;       // single-fetch GEMM shape overrides
  int sf_stages = 0, sf_a_steps = 0, sf_ks = 0;
  int cnt_stride = 32;  // split-K tickets: unsigned words between tiles' counters (32 = a 128-B line each)
  int sf_seam = -1;  // single-fetch GEMM split-K seam: -1 built-in, 0 fixed reducer, 1 spread
  int sf_late_pub = 0;  // robustness test hook: slice-0 publishers add after the reducer timed out
  int sf_xmap = 0;     // fixed-reducer seam: K slices on their own XCDs (0 built-in, 1 off, 2 on)
  int sf_loaders = 0;  // single-fetch GEMMs: loader waves (0 built-in, 1 off, 2 on, 3 eight)
  int attn_prefill_nw = 0;  // prefill attention: waves per query block (0 built-in, 1, 2, 4)
  int gemv_lds = 0;  // int4 GEMV: minimum dynamic LDS per workgroup (caps residency; tao_tune_int4_lds)
};
Tuning& tuning();

// ---- optional per-kernel timing (tao_profile_begin / tao_profile_end, capi.cpp) ---------------
// While a profile session is open on this thread, each launch gets a start/stop hipEvent pair
// recorded by the kernel's own dispatch packet (hipExtLaunchKernelGGL): the same interval
// rocprofv3 reports as the kernel's duration. Outside a session launches are plain.
bool profile_slot(hipEvent_t* start, hipEvent_t* stop);

// Enqueue a kernel (callers then check_launch(name)).
template <typename K, typename... Args>
void launch(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t stream, Args... args) {
  hipEvent_t a = nullptr, b = nullptr;
  if (profile_slot(&a, &b))
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, stream, a, b, 0, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, lds, stream, args...);
}

// ---- device numerics --------------------------------------------------------------------
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float bf16lo_to_f32(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16hi_to_f32(uint32_t w) {
  return __uint_as_float(w & 0xFFFF0000u);
}

// Round-to-nearest-even f32 -> bf16 (v_cvt_pk_bf16_f32 on gfx950; keeps NaN a NaN).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
__device__ __forceinline__ float round_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }

// acc + a.lo*b.lo + a.hi*b.hi on bf16 pairs (v_dot2c_f32_bf16).
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a),
                                         __builtin_bit_cast(bf16x2_t, b), acc, false);
}

// Two nibbles (bits 4i and 16+4i) -> bf16 pair (128+q_lo, 128+q_hi): the exact "magic number"
// conversion (0x4300 = 128.0 in bf16, q fills the low mantissa bits).
__device__ __forceinline__ uint32_t nib_pair_bf16(uint32_t w, int i) {
  return ((w >> (4 * i)) & 0x000F000Fu) | 0x43004300u;
}
// All four pairs of a word, p[i] == nib_pair_bf16(w, i), by byte permutes: lo = w & 0x0F0F0F0F
// holds q0, q4, q1, q5 in its bytes and hi = (w >> 4) & 0x0F0F0F0F holds q2, q6, q3, q7; one
// v_perm_b32 puts two of them under 0x43 bytes ([q_a, 0x43, q_b, 0x43] = (128 + q_a, 128 + q_b)):
// 7 VALU per 4 pairs instead of 11 (3 shifts + 4 ands + 4 ors)
__device__ __forceinline__ void nib_pairs4_bf16(uint32_t w, uint32_t (&p)[4]) {
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
  p[0] = __builtin_amdgcn_perm(0x43434343u, lo, 0x04020400u);
  p[1] = __builtin_amdgcn_perm(0x43434343u, hi, 0x04020400u);
  p[2] = __builtin_amdgcn_perm(0x43434343u, lo, 0x04030401u);
  p[3] = __builtin_amdgcn_perm(0x43434343u, hi, 0x04030401u);
}

template <typename T>
__device__ __forceinline__ T ld_nt(const T* p) {
  return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ uint4 ld_nt_u4(const uint4* p) {
  // Non-temporal 16-B load of streamed-once weights (MI355X_MICROARCH "nt-weights").
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void st_nt_u4(uint4* p, uint4 v) {  // 16-B non-temporal vector store
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

// ---- split-K seam waits ------------------------------------------------------------------------
// A reducer gives up on its tile's publishers once BOTH kSeamTimeoutTicks of the 100 MHz
// s_memrealtime clock (0.25 s) have passed AND it has polled kSeamMinPolls times itself, reports,
// and writes nothing for that tile. The poll count only advances while the waiting wave runs, so
// time the GPU spends on other work (a shared or preempted card, e.g. every rank of a gloo
// rehearsal on one device) does not count toward a timeout.
constexpr unsigned long long kSeamTimeoutTicks = 25000000ull;
constexpr unsigned kSeamMinPolls = 200000u;

struct SeamWait {
  unsigned long long t0;
  unsigned polls;
  __device__ __forceinline__ SeamWait() : t0(__builtin_amdgcn_s_memrealtime()), polls(0u) {}
  __device__ __forceinline__ bool timed_out() {
    return ++polls > kSeamMinPolls && __builtin_amdgcn_s_memrealtime() - t0 > kSeamTimeoutTicks;
  }
};

// Test hook (tao_debug_sf_late_publisher): a slice-0 publisher holds its ticket add until some
// reducer has timed out (its error word set) or 2 s passed, so a test can check that the
// ticket is back at 0 after such a launch.
__device__ __forceinline__ void late_publisher_hold(const unsigned* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
         __builtin_amdgcn_s_memrealtime() - t0 < 8 * kSeamTimeoutTicks)
    __builtin_amdgcn_s_sleep(127);
}

// ---- buffer resources --------------------------------------------------------------------------
// All operand loads are raw buffer loads: a wave-uniform 128-bit descriptor, a per-lane 32-bit
// voffset fixed for the whole launch and a per-step wave-uniform soffset, so the k loop spends
// no VALU on 64-bit address arithmetic (cdna guide T8/T20). Loads past the descriptor's byte
// count return 0; callers keep every operand below 4 GiB.
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int kNT = 2;    // aux: non-temporal (streamed-once weights)
constexpr int kSC1 = 16;  // aux: sc1 (device scope: L1 bypassed, stores written through L2)

__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  // readfirstlane on the inputs makes the descriptor provably uniform (no waterfall loops)
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  void* p = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}
template <int AUX = 0>
__device__ __forceinline__ uint4 bload16(Rsrc r, uint32_t voff, uint32_t soff) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v =
      __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX));
  return make_uint4(v[0], v[1], v[2], v[3]);
}
template <int AUX = 0>
__device__ __forceinline__ void bstore16(Rsrc r, uint32_t voff, uint32_t soff, uint4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 d = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(d, r, voff, soff, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ uint32_t bload4(Rsrc r, uint32_t voff, uint32_t soff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX);
}

constexpr int kWave = 64;

// ---- LDS-DMA (buffer_load ... lds) ------------------------------------------------------------
// 64 lanes x SIZE bytes from per-lane buffer offsets into LDS at the wave-uniform `dst` + lane x
// SIZE (lane-linear; swizzled images are made by choosing each lane's SOURCE). Issued by inline
// asm: with the intrinsic, hipcc treats every pending DMA as a writer of any LDS a later ds_read
// touches and waits vmcnt(0) before the first read of every step, which drains a ring. The caller
// waits for its DMAs by hand (counted vmcnt before a barrier). M0 is saved and restored.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
// dma_lds_ring: the same DMA without the asm's "memory" clobber, for rings whose every refill
// targets a stage no ds_read of the current barrier interval touches (the stage was last read
// before the barrier_lgkm() that precedes the refill, and barrier_lgkm() is itself a compiler
// memory barrier; volatile asm statements keep their order). The clobber otherwise pins every
// LDS fragment read of the step on one side of every DMA piece, so hipcc cannot issue a step's
// reads ahead of the MFMAs that need them.
template <int SIZE, int AUX = 0>
__device__ __forceinline__ void dma_lds_ring(Rsrc r, uint32_t voff, uint32_t soff, void* dst) {
  static_assert((SIZE == 16 || SIZE == 4) && (AUX == 0 || AUX == kNT), "dma_lds: 16 / 4 B, nt or not");
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_ptr_t)dst;
  uint32_t keep;
  if constexpr (SIZE == 16 && AUX == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff));
  else if constexpr (SIZE == 16)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff));
  else if constexpr (AUX == 0)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dword %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff));
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dword %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff));
}

template <int SIZE, int AUX = 0>
__device__ __forceinline__ void dma_lds(Rsrc r, uint32_t voff, uint32_t soff, void* dst) {
  static_assert((SIZE == 16 || SIZE == 4) && (AUX == 0 || AUX == kNT), "dma_lds: 16 / 4 B, nt or not");
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

// Workgroup barrier that leaves vector-memory ops (LDS-DMA included) in flight: only this wave's
// LDS ops are drained (a __syncthreads() would also wait vmcnt(0) while a DMA is pending).
__device__ __forceinline__ void barrier_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// SwiGLU of an interleaved (gate, up) bf16 pair word: bf16(bf16(silu(a)) * b), the roundings of
// decode_ops.hip's silu_mul kernel (F.silu(w1 x) * w3 x on bf16 tensors); used by the GEMM
// epilogues that fold the prefill SiLU-mul into the w1||w3 linear
__device__ __forceinline__ uint16_t swiglu_pair(uint32_t ab) {
  const float a = __uint_as_float(ab << 16), b = __uint_as_float(ab & 0xFFFF0000u);
  const float sa = __uint_as_float((uint32_t)f32_to_bf16(a / (1.f + __expf(-a))) << 16);
  return f32_to_bf16(sa * b);
}
// 16 bf16 columns (8 pairs) of an epilogue image -> 8 bf16 outputs
__device__ __forceinline__ uint4 swiglu_piece(uint4 lo, uint4 hi) {
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    o[i] = (uint32_t)swiglu_pair(w[2 * i]) | ((uint32_t)swiglu_pair(w[2 * i + 1]) << 16);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- decode-step error word ------------------------------------------------------------------
// Device-side argument faults of the decode kernels (a KV position outside [0, T)) are not
// trapped: the kernel skips the out-of-range cache write, clamps what it reads, and ORs a bit
// into a per-translation-unit error word that the host reads and clears with
// tao_decode_status() (a synchronous read, made outside graph capture; the decode harness does
// it after every generate()). The reference's index_put KV cache device-asserts instead.
constexpr unsigned kDecodeErrKvPos = 1u;
// tao_decode_status bits & 2: a single-fetch GEMM's split-K reducer timed out waiting for its
// publishers (that tile was not written; never expected)
constexpr unsigned kDecodeErrSplitK = 2u;
// tao_decode_status bits & 4: a grouped (MoE) GEMV read an expert index outside [0, E) (clamped)
constexpr unsigned kDecodeErrExpert = 4u;
#define TAO_DECODE_ERROR_WORD(reader)                                                        \
  static __device__ unsigned g_decode_err = 0;                                                \
  __device__ __forceinline__ void flag_decode_error(unsigned bits) {                          \
    (void)__hip_atomic_fetch_or(&g_decode_err, bits, __ATOMIC_RELAXED,                        \
                                __HIP_MEMORY_SCOPE_AGENT);                                    \
  }                                                                                           \
  int reader(unsigned* bits) {                                                                \
    unsigned v = 0, zero = 0;                                                                 \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_decode_err), sizeof(v)) != hipSuccess ||         \
        hipMemcpyToSymbol(HIP_SYMBOL(g_decode_err), &zero, sizeof(zero)) != hipSuccess)       \
      return set_error(TAO_ERR_HIP, "decode status: symbol copy failed");                     \
    *bits |= v;                                                                               \
    return TAO_OK;                                                                            \
  }

// Split decode attention: the merge weights of NS partials (m_s, l_s) of one head (an empty split
// has m = -inf, l = 0; split 0 is never empty): wgt_s = exp(m_s - max m), inv = 1 / sum l_s wgt_s.
// Shared by the merge kernel (decode_ops.hip) and the wo GEMV's merge prologue (int4_gemv.hip).
template <int NS>
__device__ __forceinline__ void attn_merge_weights(const float2 (&ml)[NS], float (&wgt)[NS],
                                                   float& inv) {
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < NS; ++s) M = fmaxf(M, ml[s].x);
  float L = 0.f;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    wgt[s] = ml[s].x == -INFINITY ? 0.f : __expf(ml[s].x - M);
    L = fmaf(ml[s].y, wgt[s], L);
  }
  inv = 1.f / L;
}

// keys attended at query position p of a cache of T rows: p + 1, clamped to [1, T] (a p
// outside [0, T) was reported by the KV-writing kernel of the same step)
__device__ __forceinline__ int attn_len(int64_t p, int T) {
  return p < 0 ? 1 : (p >= T ? T : (int)p + 1);
}

// ---- last-arriver hand-off (split-K slabs, decode-attention chunks) ------------------------------
// Call after every storing wave of the workgroup has stored its share of the hand-off (all with
// kSC1) and run `s_waitcnt vmcnt(0)`, from all threads (contains a workgroup barrier). One lane
// adds to the tile's arrival counter; every thread learns whether this workgroup arrived last
// (then the counter is reset for the next launch) and may load the others' bytes with kSC1 loads.
//
// fenced == 0 (default): no agent fences. This is MI355X_MICROARCH.md's "Hand-offs measured with
// sc1 loads in place of the acquire", first row: one lane per storing workgroup signals with an
// agent-scope atomic add to one unsharded counter, the workgroup whose add came last is told by
// the value it returned, its other waves load after a workgroup barrier joined behind an LDS
// word, sc1 stores and sc1 loads of 16 B (and 8 B in decode attention), hipMalloc'd memory. That
// row is a measured gfx950 / ROCm 7.0-7.2 behaviour, not an HIP memory-model guarantee (the guide
// says so); the fences it removes cost 1.7-6.5 µs each.
// fenced == 1 (tao_tune_splitk_fenced): the memory-model form on top of the same stores and
// loads: release fence (buffer_wbl2 sc1 + asm vmcnt(0), the guide's compiler-hazard fix) before
// the add, acquire fence (buffer_inv sc1 + vmcnt(0)) in the last arriver before the barrier.
// tests/test_gpu_gemm_tiles.py checks both give bit-identical results.
__device__ __forceinline__ bool last_arriver(unsigned* counter, unsigned arrivals,
                                             unsigned* lds_word, int fenced) {
  if (threadIdx.x == 0 && threadIdx.y == 0) {
    if (fenced) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned ticket =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = ticket == arrivals - 1;
    if (last) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fenced) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    *lds_word = last ? 1u : 0u;
  }
  __syncthreads();
  return *lds_word != 0;
}

}  // namespace tao
