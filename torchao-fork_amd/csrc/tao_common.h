// Shared helpers for the gfx950 kernels behind include/torchao_mi355x.h.
// Internal header: not part of the C-ABI.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/torchao_mi355x.h"

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

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- split-K workspace (capi.cpp) ------------------------------------------------------------
// Per (device, stream) scratch for the partial-sum slabs of split-K launches plus a zeroed array
// of arrival counters (each reset by its tile's last arriver). Grows outside graph capture
// only: a capture borrows a large-enough workspace reserved on the device by an earlier eager
// call (on any stream), else it is an error (run the op once at that shape before capturing).
int split_workspace(hipStream_t stream, size_t slab_bytes, size_t counters, void** slab,
                    unsigned** cnt);

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

}  // namespace tao
