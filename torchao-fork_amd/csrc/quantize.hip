// On-GPU weight quantizers: bf16 weight -> the packed operands the linears read,
// in one pass over the weight, bit-exact to the reference's bf16 op order.
//
//   int4 tinygemm (Int4WeightOnlyConfig; reference quant_primitives.py:1238-1307 qparams,
//   :461-573 quantize, tensor_core_tiled_layout.py:262-307 pack), per (row, group of g):
//     s = bf16(max(bf16(bf16(max - min) / 15), eps))      z = bf16(min + 8 s)
//     q = clamp(rint(bf16(bf16(w - bf16(z - 8 s)) / s)), 0, 15)
//   then nibbles into the gfx950 row-stream dword (bits 4i / 16+4i = q[8d+2i] / q[8d+2i+1])
//   and (s, z) into scales_and_zeros [rows][K/g][2]. Every bf16 op is its fp32 result rounded
//   to nearest even (torch's opmath for bf16 tensors); division is IEEE-correct.
//
//   int8 symmetric per-row (Int8WeightOnlyConfig, Int8DynamicActivationInt8WeightConfig weight;
//   quant_api.py:1200-1255 / :1352-1430 through choose_qparams_affine SYMMETRIC):
//     s = bf16(max(bf16(amax / 127.5), eps))   q = clamp(rint(bf16(w * bf16(1 / s))), -128, 127)
//
// Both are HBM-bound byte work: 16-B loads of the weight, one thread per 8 weights; the int4
// group reductions are lane shuffles (g / 8 lanes per group), the int8 row reduction a
// workgroup per row.
#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {
namespace {

template <int LPG>  // lanes per quantisation group (g / 8)
__global__ __launch_bounds__(256) void int4_quantize_kernel(const uint4* __restrict__ w,
                                                            uint32_t* __restrict__ packed,
                                                            uint32_t* __restrict__ sz,
                                                            int64_t total8, float eps) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const uint4 v = w[i < total8 ? i : total8 - 1];  // clamped: tail lanes still shuffle
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
  float f[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = bf16lo_to_f32(d[j]);
    f[2 * j + 1] = bf16hi_to_f32(d[j]);
  }
  float mn = f[0], mx = f[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) {
    mn = fminf(mn, f[j]);
    mx = fmaxf(mx, f[j]);
  }
#pragma unroll
  for (int o = 1; o < LPG; o <<= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  const float rng = round_bf16(mx - mn);
  const float s = round_bf16(fmaxf(round_bf16(rng / 15.0f), eps));
  const float z = round_bf16(mn + s * 8.0f);  // s * 8 is exact
  const float lo = round_bf16(z - s * 8.0f);
  uint32_t out = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float t = round_bf16(f[j] - lo);
    const float q = fminf(fmaxf(rintf(round_bf16(t / s)), 0.f), 15.f);
    out |= (uint32_t)q << ((j & 1) * 16 + (j >> 1) * 4);
  }
  if (i < total8) {
    packed[i] = out;
    if ((i & (LPG - 1)) == 0)
      sz[i / LPG] = (uint32_t)f32_to_bf16(s) | ((uint32_t)f32_to_bf16(z) << 16);
  }
}

// One workgroup per row; K % 8 == 0. Pass 1: amax; pass 2 (the row again, from L2): quantise.
__global__ __launch_bounds__(256) void int8_quantize_rows_kernel(const uint4* __restrict__ w,
                                                                 uint2* __restrict__ q,
                                                                 uint16_t* __restrict__ scale,
                                                                 int K8, float eps) {
  __shared__ float red[4];
  const uint4* row = w + (size_t)blockIdx.x * K8;
  float amax = 0.f;  // max(-min(mn, 0), max(mx, 0)) == max |w| with 0 included
  for (int i = threadIdx.x; i < K8; i += 256) {
    const uint4 v = row[i];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      amax = fmaxf(amax, fmaxf(fabsf(bf16lo_to_f32(d[j])), fabsf(bf16hi_to_f32(d[j]))));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = round_bf16(fmaxf(round_bf16(amax / 127.5f), eps));
  const float r = round_bf16(1.0f / s);
  if (threadIdx.x == 0) scale[blockIdx.x] = f32_to_bf16(s);
  uint2* qr = q + (size_t)blockIdx.x * K8;
  for (int i = threadIdx.x; i < K8; i += 256) {
    const uint4 v = row[i];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = (j & 1) ? bf16hi_to_f32(d[j >> 1]) : bf16lo_to_f32(d[j >> 1]);
      const float qf = fminf(fmaxf(rintf(round_bf16(x * r)), -128.f), 127.f);
      o[j >> 2] |= ((uint32_t)(int)qf & 0xFFu) << (8 * (j & 3));
    }
    qr[i] = make_uint2(o[0], o[1]);
  }
}

}  // namespace
}  // namespace tao

using namespace tao;

extern "C" {

int tao_int4_quantize_bf16(const uint16_t* w, uint32_t* packed, uint16_t* scales_and_zeros,
                           int64_t rows, int64_t K, int64_t group_size, float eps,
                           void* stream) {
  TAO_CHECK_ARG(group_size == 32 || group_size == 64 || group_size == 128 || group_size == 256,
                "int4 quantize: group_size must be 32, 64, 128 or 256 (got %lld)",
                (long long)group_size);
  TAO_CHECK_ARG(rows >= 0 && K >= 0 && K % group_size == 0,
                "int4 quantize: K (%lld) %% group_size (%lld) != 0", (long long)K,
                (long long)group_size);
  const int64_t total8 = rows * (K / 8);
  if (total8 == 0) return TAO_OK;
  TAO_CHECK_ARG(total8 / 256 < (1LL << 31), "int4 quantize: tensor too large");
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(packed, 4, "packed");
  TAO_CHECK_ALIGN(scales_and_zeros, 4, "scales_and_zeros");
  const dim3 grid((unsigned)((total8 + 255) / 256));
  hipStream_t st = as_stream(stream);
  const uint4* wv = reinterpret_cast<const uint4*>(w);
  uint32_t* szv = reinterpret_cast<uint32_t*>(scales_and_zeros);
  switch (group_size) {
    case 32: launch(int4_quantize_kernel<4>, grid, dim3(256), 0, st, wv, packed, szv, total8, eps); break;
    case 64: launch(int4_quantize_kernel<8>, grid, dim3(256), 0, st, wv, packed, szv, total8, eps); break;
    case 128: launch(int4_quantize_kernel<16>, grid, dim3(256), 0, st, wv, packed, szv, total8, eps); break;
    default: launch(int4_quantize_kernel<32>, grid, dim3(256), 0, st, wv, packed, szv, total8, eps); break;
  }
  return check_launch("int4_quantize_kernel");
}

int tao_int8_quantize_rows_bf16(const uint16_t* w, int8_t* q, uint16_t* scale, int64_t rows,
                                int64_t K, float eps, void* stream) {
  TAO_CHECK_ARG(rows >= 0 && rows < (1LL << 31) && K >= 0 && K % 8 == 0 && K < (1LL << 31),
                "int8 quantize: K (%lld) must be a multiple of 8", (long long)K);
  if (rows == 0 || K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(q, 8, "q");
  TAO_CHECK_ALIGN(scale, 2, "scale");
  launch(int8_quantize_rows_kernel, dim3((unsigned)rows), dim3(256), 0, as_stream(stream),
         reinterpret_cast<const uint4*>(w), reinterpret_cast<uint2*>(q), scale, (int)(K / 8),
         eps);
  return check_launch("int8_quantize_rows_kernel");
}

}  // extern "C"
