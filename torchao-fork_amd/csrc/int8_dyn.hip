// int8 dynamic-activation x int8-weight linear (Int8DynamicActivationInt8WeightConfig):
//   1. tao_int8_quant_per_token: x bf16 [M][K] -> (q int8 [M][K], s bf16 [M]), replacing
//      _int8_symm_per_token_reduced_range_quant (torchao/quantization/quant_api.py:1258-1273),
//      which the reference runs as ~6 eager kernels (amin/amax/div/round/clamp/cast);
//   2. tao_int8_scaled_mm_bf16: int32 MFMA GEMM with the fused two-scale epilogue, replacing
//      int_scaled_matmul + the weight-scale multiply (torchao/kernel/intmm.py:108-143,
//      torchao/dtypes/uintx/plain_layout.py:294-315). The GEMM is the Int8Dyn instance of the
//      shared skinny-GEMM template in gemm_mfma.hip.
#include "tao_common.h"

namespace tao {
namespace {

// ---- per-token quantisation ------------------------------------------------------------------
constexpr int kQBlock = 256;

__device__ __forceinline__ float bf16_abs_max2(uint32_t d, float m) {
  m = fmaxf(m, fabsf(bf16lo_to_f32(d)));
  return fmaxf(m, fabsf(bf16hi_to_f32(d)));
}

__global__ __launch_bounds__(kQBlock) void int8_quant_per_token_kernel(
    const uint16_t* __restrict__ x, int8_t* __restrict__ q, uint16_t* __restrict__ scale, int K) {
  __shared__ float wmax[kQBlock / 64];
  const int row = blockIdx.x;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * K);
  const int nvec = K / 8;  // 8 bf16 per 16-B vector
  float m = 0.f;
  for (int i = threadIdx.x; i < nvec; i += kQBlock) {
    const uint4 v = xr[i];
    m = bf16_abs_max2(v.x, m);
    m = bf16_abs_max2(v.y, m);
    m = bf16_abs_max2(v.z, m);
    m = bf16_abs_max2(v.w, m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  float amax = wmax[0];
#pragma unroll
  for (int w = 1; w < kQBlock / 64; ++w) amax = fmaxf(amax, wmax[w]);

  // scale = clamp(bf16(amax / 127), min = 1e-5) in bf16 (quant_primitives.py:1548-1554 with
  // quant range [-127, 127]); the clamp minimum is compared after bf16 rounding.
  float s = round_bf16(amax / 127.f);
  const float eps = round_bf16(1e-5f);
  s = s < eps ? eps : s;
  if (threadIdx.x == 0) scale[row] = f32_to_bf16(s);
  // q = clamp(round(bf16(x * bf16(1/s))), -127, 127)  (quant_primitives.py:449-453)
  const float r = round_bf16(1.f / s);
  uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * K);
  for (int i = threadIdx.x; i < nvec; i += kQBlock) {
    const uint4 v = xr[i];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    uint32_t packed[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = (j & 1) ? bf16hi_to_f32(d[j >> 1]) : bf16lo_to_f32(d[j >> 1]);
      float t = rintf(round_bf16(xv * r));
      t = fminf(fmaxf(t, -127.f), 127.f);
      const uint32_t b = (uint32_t)(int32_t)t & 0xFFu;
      packed[j >> 2] |= b << (8 * (j & 3));
    }
    qr[i] = make_uint2(packed[0], packed[1]);
  }
}

}  // namespace

int int8_scaled_mm_launch(const int8_t* xq, const uint16_t* xs, const int8_t* wq,
                          const uint16_t* ws, const uint16_t* bias, uint16_t* y, int M, int N,
                          int K, hipStream_t stream);  // gemm_mfma.hip

}  // namespace tao

using namespace tao;

extern "C" {

int tao_int8_quant_per_token(const uint16_t* x, int8_t* q, uint16_t* scale, int64_t M,
                             int64_t K, void* stream) {
  TAO_CHECK_ARG(M >= 0 && K >= 0, "int8 quant: negative size");
  TAO_CHECK_ARG(K % 16 == 0, "int8 quant: K (%lld) must be a multiple of 16", (long long)K);
  TAO_CHECK_ARG(M < (1LL << 31) && K < (1LL << 31), "int8 quant: size out of range");
  if (M == 0 || K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(x, 16, "x");
  TAO_CHECK_ALIGN(q, 8, "q");
  launch(int8_quant_per_token_kernel, dim3((unsigned)M), dim3(kQBlock), 0,
                     as_stream(stream), x, q, scale, (int)K);
  return check_launch("int8_quant_per_token_kernel");
}

int tao_int8_scaled_mm_bf16(const int8_t* xq, const uint16_t* xs, const int8_t* wq,
                            const uint16_t* ws, const uint16_t* bias, uint16_t* y, int64_t M,
                            int64_t N, int64_t K, void* stream) {
  TAO_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "int8 scaled mm: negative size");
  TAO_CHECK_ARG(K % 16 == 0, "int8 scaled mm: K (%lld) must be a multiple of 16", (long long)K);
  TAO_CHECK_ARG(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31),
                "int8 scaled mm: size out of range");
  if (M == 0 || N == 0) return TAO_OK;
  TAO_CHECK_ARG(K > 0, "int8 scaled mm: K must be > 0");
  TAO_CHECK_ALIGN(xq, 16, "xq");
  TAO_CHECK_ALIGN(wq, 16, "wq");
  return int8_scaled_mm_launch(xq, xs, wq, ws, bias, y, (int)M, (int)N, (int)K,
                               as_stream(stream));
}

}  // extern "C"
