// int8 dynamic-activation x int8-weight linear (Int8DynamicActivationInt8WeightConfig):
//   1. tao_int8_quant_per_token: x bf16 [M][K] -> (q int8 [M][K], s bf16 [M]), replacing
//      _int8_symm_per_token_reduced_range_quant (torchao/quantization/quant_api.py:1258-1273),
//      which the reference runs as ~6 eager kernels (amin/amax/div/round/clamp/cast);
//   2. tao_int8_scaled_mm_bf16: int32 MFMA GEMM with the fused two-scale epilogue, replacing
//      int_scaled_matmul + the weight-scale multiply (torchao/kernel/intmm.py:108-143,
//      torchao/dtypes/uintx/plain_layout.py:294-315).
//
// GEMM tile: 4 waves x 16 output columns = BN 64, BM rows; macro-step 256 k;
// v_mfma_i32_16x16x64_i8 with a permuted k order: MFMA s of lane l (r = l&15, kq = l>>4) uses
// k = k0 + 64*kq + 16*s + (0..15), identically for A and B, so a lane's 64-B weight load
// feeds all four MFMAs. x (int8) is staged through LDS with 16-B slots XOR-swizzled by row.
#include "tao_common.h"

namespace tao {
namespace {

typedef int i32x4_t __attribute__((ext_vector_type(4)));

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

// ---- int8 x int8 -> int32 MFMA GEMM ----------------------------------------------------------
constexpr int kBN = 64;
constexpr int kKStep = 256;

__device__ __forceinline__ int lds_slot(int row, int slot) { return row * 16 + (slot ^ (row & 15)); }

template <int BM>
__global__ __launch_bounds__(256) void int8_scaled_mm_kernel(
    const int8_t* __restrict__ xq, const uint16_t* __restrict__ xs, const uint4* __restrict__ wq,
    const uint16_t* __restrict__ ws, const uint16_t* __restrict__ bias, uint16_t* __restrict__ y,
    int M, int N, int K) {
  constexpr int MT = BM / 16;
  constexpr int XLOADS = BM * 16 / 256;
  __shared__ uint4 xsm[BM * 16];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int n_blk = blockIdx.x * kBN;
  const int m_blk = blockIdx.y * BM;
  const int nvec = K >> 4;  // 16-B vectors per row
  const int nsteps = (K + kKStep - 1) / kKStep;

  const int bn = n_blk + wave * 16 + (lane & 15);
  const int bnc = bn < N ? bn : N - 1;
  const int kq = lane >> 4;

  i32x4_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = i32x4_t{0, 0, 0, 0};

  uint4 xr[XLOADS];
  uint4 wr[4];

  auto load_step = [&](int step) {
    const int k0 = step * kKStep;
#pragma unroll
    for (int i = 0; i < XLOADS; ++i) {
      const int piece = tid + i * 256;
      const int row = piece >> 4, slot = piece & 15;
      const int gm = m_blk + row;
      const int gk = k0 + slot * 16;
      const bool ok = gm < M && gk < K;
      const int gmc = gm < M ? gm : M - 1;
      const int gkc = gk < K ? gk : 0;
      const uint4 v = *reinterpret_cast<const uint4*>(xq + (size_t)gmc * K + gkc);
      xr[i] = ok ? v : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int vec = (k0 >> 4) + kq * 4 + s;
      const bool ok = vec < nvec && bn < N;
      const int vc = vec < nvec ? vec : nvec - 1;
      const uint4 v = ld_nt_u4(wq + (size_t)bnc * nvec + vc);
      wr[s] = ok ? v : make_uint4(0, 0, 0, 0);
    }
  };

  load_step(0);
  for (int step = 0; step < nsteps; ++step) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < XLOADS; ++i) {
      const int piece = tid + i * 256;
      xsm[lds_slot(piece >> 4, piece & 15)] = xr[i];
    }
    uint4 wcur[4] = {wr[0], wr[1], wr[2], wr[3]};
    __syncthreads();
    if (step + 1 < nsteps) load_step(step + 1);

#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const i32x4_t bfrag = __builtin_bit_cast(i32x4_t, wcur[s]);
      const int slot = kq * 4 + s;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int row = t * 16 + (lane & 15);
        const i32x4_t afrag = __builtin_bit_cast(i32x4_t, xsm[lds_slot(row, slot)]);
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag, bfrag, acc[t], 0, 0, 0);
      }
    }
  }

  if (bn < N) {
    const float wsc = bf16_to_f32(ws[bn]);
    const float bv = bias != nullptr ? bf16_to_f32(bias[bn]) : 0.f;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m_blk + t * 16 + 4 * (lane >> 4) + i;
        if (m < M) {
          // bf16(c) * x_scale, * w_scale, + bias: each rounded to bf16, the op order of the
          // reference (intmm.py:133-137 then plain_layout.py:301-315).
          float v = round_bf16(round_bf16((float)acc[t][i]) * bf16_to_f32(xs[m]));
          v = round_bf16(v * wsc);
          if (bias != nullptr) v = round_bf16(v + bv);
          y[(size_t)m * N + bn] = f32_to_bf16(v);
        }
      }
    }
  }
}

}  // namespace
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
  hipStream_t st = as_stream(stream);
  const int bm = M <= 16 ? 16 : (M <= 32 ? 32 : 64);
  dim3 grid((unsigned)((N + kBN - 1) / kBN), (unsigned)((M + bm - 1) / bm));
  const uint4* w4 = reinterpret_cast<const uint4*>(wq);
  if (bm == 16)
    launch(int8_scaled_mm_kernel<16>, grid, dim3(256), 0, st, xq, xs, w4, ws, bias, y,
                       (int)M, (int)N, (int)K);
  else if (bm == 32)
    launch(int8_scaled_mm_kernel<32>, grid, dim3(256), 0, st, xq, xs, w4, ws, bias, y,
                       (int)M, (int)N, (int)K);
  else
    launch(int8_scaled_mm_kernel<64>, grid, dim3(256), 0, st, xq, xs, w4, ws, bias, y,
                       (int)M, (int)N, (int)K);
  return check_launch("int8_scaled_mm_kernel");
}

}  // extern "C"
