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

}  // namespace
}  // namespace tao

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
