// Measurement kernel used by bench.py (not on the product path): a pure streaming read of a buffer
// with 16-B non-temporal loads, one load per thread, 512-thread workgroups (each wave-instruction
// 1 KiB contiguous). It is the best of the read variants DESIGN §5.0 measured
// (experiments/probe_graph_read.py): replaying one such launch per linear from a HIP graph gives
// the floor any one-kernel-per-linear GEMV step can reach on this chip, measured in the same run
// as the GEMV step (bench.py roofline.pure_read_ms_per_step).
#include "tao_common.h"

namespace tao {
namespace {

__global__ __launch_bounds__(512) void read_probe_kernel(const uint4* __restrict__ p,
                                                         uint32_t* __restrict__ sink) {
  const size_t t = (size_t)blockIdx.x * 512 + threadIdx.x;
  const uint4 v = ld_nt_u4(p + t);
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x9E3779B9u) sink[t & 1023] = acc;  // keeps the load live; never taken in practice
}

// Streaming copy for the bench's ceiling calibration (MI355X_MICROARCH.md "HBM": a float4 copy
// measured at 6.29 TB/s read + write). mode 0: each thread moves 4 x 16 B per grid-stride round
// with all four loads in flight before the stores, default cache policy; mode 1: the same with
// non-temporal loads and stores; mode 2: one 16-B element per thread, no loop (grid covers the
// buffer: bytes / 16 / 256 workgroups), non-temporal.
template <int MODE>
__global__ __launch_bounds__(256) void copy_probe_kernel(const uint4* __restrict__ src,
                                                         uint4* __restrict__ dst, size_t n16) {
  if constexpr (MODE == 2) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) st_nt_u4(dst + i, ld_nt_u4(src + i));
    return;
  } else {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = i + 256 * j < n16 ? (MODE == 1 ? ld_nt_u4(src + i + 256 * j) : src[i + 256 * j])
                                 : uint4{};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i + 256 * j < n16) {
          if constexpr (MODE == 1) st_nt_u4(dst + i + 256 * j, v[j]);
          else dst[i + 256 * j] = v[j];
        }
    }
  }
}

}  // namespace
}  // namespace tao

extern "C" int tao_hbm_copy_probe(const void* src, void* dst, int64_t bytes, int grid, int mode,
                                  void* stream) {
  TAO_CHECK_ARG(src != nullptr && dst != nullptr, "copy probe: null pointer");
  TAO_CHECK_ARG(bytes > 0 && bytes % 16 == 0, "copy probe: bytes (%lld) must be a positive "
                "multiple of 16", (long long)bytes);
  TAO_CHECK_ARG(mode >= 0 && mode <= 2, "copy probe: mode (%d) must be 0, 1 or 2", mode);
  TAO_CHECK_ARG(mode == 2 || (grid > 0 && grid <= (1 << 20)), "copy probe: grid (%d) out of range",
                grid);
  TAO_CHECK_ARG(mode != 2 || bytes / 4096 < (1LL << 31), "copy probe: bytes too large for mode 2");
  TAO_CHECK_ALIGN(src, 16, "src");
  TAO_CHECK_ALIGN(dst, 16, "dst");
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const size_t n16 = (size_t)(bytes / 16);
  hipStream_t st = tao::as_stream(stream);
  if (mode == 2)
    tao::launch(tao::copy_probe_kernel<2>, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st,
                s, d, n16);
  else if (mode == 1)
    tao::launch(tao::copy_probe_kernel<1>, dim3((unsigned)grid), dim3(256), 0, st, s, d, n16);
  else
    tao::launch(tao::copy_probe_kernel<0>, dim3((unsigned)grid), dim3(256), 0, st, s, d, n16);
  return tao::check_launch("copy_probe_kernel");
}

extern "C" int tao_hbm_read_probe(const void* buf, int64_t bytes, void* sink, void* stream) {
  TAO_CHECK_ARG(buf != nullptr && sink != nullptr, "read probe: null pointer");
  TAO_CHECK_ARG(bytes > 0 && bytes % 8192 == 0 && bytes / 8192 < (1LL << 31),
                "read probe: bytes (%lld) must be a positive multiple of 8192",
                (long long)bytes);
  TAO_CHECK_ALIGN(buf, 16, "buf");
  tao::launch(tao::read_probe_kernel, dim3((unsigned)(bytes / 8192)), dim3(512), 0,
              tao::as_stream(stream), reinterpret_cast<const uint4*>(buf),
              reinterpret_cast<uint32_t*>(sink));
  return tao::check_launch("read_probe_kernel");
}
