// int4 pack / unpack / dequant helpers for the gfx950 row-stream layout, and the reference
// tile-format compat ops (torchao::unpack/dequantize_tensor_core_tiled_layout).
//
// All kernels are HBM-bound elementwise byte work: one thread per packed dword (8 weights),
// 16-B vector loads/stores, grid-stride loops capped at 256 CUs x 8 blocks (cdna guide G11).
#include "tao_common.h"

namespace tao {
namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t work) {
  int64_t g = (work + kBlock - 1) / kBlock;
  if (g > 2048) g = 2048;
  return g < 1 ? 1 : (int)g;
}

// packed[n][d] <- q[n][8d .. 8d+7]  (int32 nibbles)
__global__ void int4_pack_kernel(const int4* __restrict__ q, uint32_t* __restrict__ packed,
                                 int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int4 a = q[2 * i], b = q[2 * i + 1];  // k = 8d+0..3, 8d+4..7
    uint32_t v[8] = {(uint32_t)a.x, (uint32_t)a.y, (uint32_t)a.z, (uint32_t)a.w,
                     (uint32_t)b.x, (uint32_t)b.y, (uint32_t)b.z, (uint32_t)b.w};
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w |= (v[2 * j] & 0xF) << (4 * j);
      w |= (v[2 * j + 1] & 0xF) << (16 + 4 * j);
    }
    packed[i] = w;
  }
}

// packed[n][d] <- u8[n][4d .. 4d+3], byte j = q[8d+2j] << 4 | q[8d+2j+1]
__global__ void int4_pack_u8_kernel(const uint32_t* __restrict__ u8, uint32_t* __restrict__ packed,
                                    int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t b = u8[i];
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t byte = (b >> (8 * j)) & 0xFF;
      w |= (byte >> 4) << (4 * j);
      w |= (byte & 0xF) << (16 + 4 * j);
    }
    packed[i] = w;
  }
}

__global__ void int4_unpack_kernel(const uint32_t* __restrict__ packed, int4* __restrict__ q,
                                   int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t w = packed[i];
    int v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = (w >> (4 * j)) & 0xF;
      v[2 * j + 1] = (w >> (16 + 4 * j)) & 0xF;
    }
    q[2 * i] = make_int4(v[0], v[1], v[2], v[3]);
    q[2 * i + 1] = make_int4(v[4], v[5], v[6], v[7]);
  }
}

// One dequantised value. MODE 0: two bf16 roundings as _dequantize_affine_tinygemm
// (quant_primitives.py:1019-1023: (q-8).to(bf16) * s, then + z). MODE 1: single rounding of
// fma(q-8, s, z) as the reference tile dequant (tensor_core_tiled_layout.cu:184-190).
template <int MODE>
__device__ __forceinline__ uint16_t deq1(uint32_t q, float s, float z) {
  const float qf = (float)((int)q - 8);
  if (MODE == 0) {
    return f32_to_bf16(round_bf16(qf * s) + z);
  } else {
    return f32_to_bf16(fmaf(qf, s, z));
  }
}

template <int MODE>
__global__ void int4_dequant_kernel(const uint32_t* __restrict__ packed,
                                    const uint32_t* __restrict__ sz, uint4* __restrict__ w,
                                    int64_t total, int64_t KD, int64_t ngroups, int gshift) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / KD, d = i - n * KD;
    const uint32_t p = packed[i];
    const uint32_t szw = sz[n * ngroups + ((d * 8) >> gshift)];
    const float s = bf16lo_to_f32(szw), z = bf16hi_to_f32(szw);
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t lo = deq1<MODE>((p >> (4 * j)) & 0xF, s, z);
      uint32_t hi = deq1<MODE>((p >> (16 + 4 * j)) & 0xF, s, z);
      o[j] = lo | (hi << 16);
    }
    w[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ---- reference tile format: [N/8][K/(ikt*16)][32][ikt/2] int32, two nibble maps --------------
// fmt 0 (kTileCuda), the semantics of the reference's unpack kernel
//   (tensor_core_tiled_layout.cu:131-215): P[nt][kt][t][j]: n = 8nt + t/4;
//   kb0 = (kt*ikt + 2j)*16; ks = {kb0+2(t%4), +8, kb0+16+2(t%4), +8}.
// fmt 1 (kTileRocm), what PyTorch-ROCm's aten._convert_weight_to_int4pack writes on gfx950
//   (recovered on the box by experiments/probe_aten_tile_map.py, pinned by
//   tests/golden/aten_tile_map_rocm.npz): the same bytes seen flat as [N/16][K/(ikt*16)][64][ikt/2]
//   for wave64 lanes l: n = 16nb + l%16; b = kb*ikt*16 + 32j + 4(l/16); ks = {b, b+2, b+16, b+18}.
// Both: bits 4i hold q[n][ks_i], bits 16+4i hold q[n][ks_i + 1].
constexpr int kTileCuda = 0, kTileRocm = 1;

__device__ __host__ __forceinline__ void tile_coords(int64_t idx, int ikt, int64_t KT, int fmt,
                                                     int64_t* n, int64_t ks[4]) {
  const int half = ikt / 2;
  const int j = (int)(idx % half);
  int64_t r = idx / half;
  if (fmt == kTileRocm) {
    const int l = (int)(r % 64);
    r /= 64;
    const int64_t kb = r % KT, nb = r / KT;
    *n = nb * 16 + l % 16;
    const int64_t b = kb * ikt * 16 + 32 * j + 4 * (l / 16);
    ks[0] = b;
    ks[1] = b + 2;
    ks[2] = b + 16;
    ks[3] = b + 18;
  } else {
    const int t = (int)(r % 32);
    r /= 32;
    const int64_t kt = r % KT, nt = r / KT;
    *n = nt * 8 + t / 4;
    const int64_t kb = (kt * ikt + 2 * j) * 16;
    const int t4 = t % 4;
    ks[0] = kb + 2 * t4;
    ks[1] = kb + 2 * t4 + 8;
    ks[2] = kb + 16 + 2 * t4;
    ks[3] = kb + 16 + 2 * t4 + 8;
  }
}

template <int OUT>  // 0: int32 unpack, 1: bf16 dequant
__global__ void tile_unpack_kernel(const int32_t* __restrict__ in, void* __restrict__ out,
                                   const uint16_t* __restrict__ sz, int64_t total, int ikt,
                                   int64_t KT, int64_t N, int64_t K, int g, int fmt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t n, ks[4];
    tile_coords(i, ikt, KT, fmt, &n, ks);
    const uint32_t p = (uint32_t)in[i];
    if (OUT == 0) {
      int32_t* o = reinterpret_cast<int32_t*>(out) + n * K;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        *reinterpret_cast<int2*>(o + ks[q]) =
            make_int2((p >> (4 * q)) & 0xF, (p >> (16 + 4 * q)) & 0xF);
      }
    } else {
      const int64_t grp = ks[0] / g;  // the 4 pairs lie in one 32-k window: one group
      const uint16_t* psz = sz + (grp * N + n) * 2;
      const float s = bf16_to_f32(psz[0]), z = bf16_to_f32(psz[1]);
      uint16_t* o = reinterpret_cast<uint16_t*>(out) + n * K;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t lo = deq1<1>((p >> (4 * q)) & 0xF, s, z);
        uint32_t hi = deq1<1>((p >> (16 + 4 * q)) & 0xF, s, z);
        *reinterpret_cast<uint32_t*>(o + ks[q]) = lo | (hi << 16);
      }
    }
  }
}

__global__ void tile_pack_kernel(const int32_t* __restrict__ q, int32_t* __restrict__ out,
                                 int64_t total, int ikt, int64_t KT, int64_t K, int fmt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t n, ks[4];
    tile_coords(i, ikt, KT, fmt, &n, ks);
    const int32_t* row = q + n * K;
    uint32_t p = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      int2 v = *reinterpret_cast<const int2*>(row + ks[s]);
      p |= ((uint32_t)v.x & 0xF) << (4 * s);
      p |= ((uint32_t)v.y & 0xF) << (16 + 4 * s);
    }
    out[i] = (int32_t)p;
  }
}

int gshift_of(int64_t g) {
  switch (g) {
    case 32: return 5;
    case 64: return 6;
    case 128: return 7;
    case 256: return 8;
    default: return -1;
  }
}

}  // namespace
}  // namespace tao

using namespace tao;

extern "C" {

int tao_int4_pack(const int32_t* q, uint32_t* packed, int64_t N, int64_t K, void* stream) {
  TAO_CHECK_ARG(N >= 0 && K >= 0 && K % 8 == 0, "int4 pack: need K %% 8 == 0 (K=%lld)",
                (long long)K);
  if (N * K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(q, 16, "q");
  const int64_t total = N * (K / 8);
  launch(int4_pack_kernel, dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream),
                     reinterpret_cast<const int4*>(q), packed, total);
  return check_launch("int4_pack_kernel");
}

int tao_int4_pack_u8(const uint8_t* q_u8, uint32_t* packed, int64_t N, int64_t K,
                     void* stream) {
  TAO_CHECK_ARG(N >= 0 && K >= 0 && K % 8 == 0, "int4 pack_u8: need K %% 8 == 0 (K=%lld)",
                (long long)K);
  if (N * K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(q_u8, 4, "q_u8");
  const int64_t total = N * (K / 8);
  launch(int4_pack_u8_kernel, dim3(grid_for(total)), dim3(kBlock), 0,
                     as_stream(stream), reinterpret_cast<const uint32_t*>(q_u8), packed, total);
  return check_launch("int4_pack_u8_kernel");
}

int tao_int4_unpack(const uint32_t* packed, int32_t* q, int64_t N, int64_t K, void* stream) {
  TAO_CHECK_ARG(N >= 0 && K >= 0 && K % 8 == 0, "int4 unpack: need K %% 8 == 0 (K=%lld)",
                (long long)K);
  if (N * K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(q, 16, "q");
  const int64_t total = N * (K / 8);
  launch(int4_unpack_kernel, dim3(grid_for(total)), dim3(kBlock), 0,
                     as_stream(stream), packed, reinterpret_cast<int4*>(q), total);
  return check_launch("int4_unpack_kernel");
}

int tao_int4_dequant(const uint32_t* packed, const uint16_t* sz, uint16_t* w, int64_t N,
                     int64_t K, int64_t group_size, int mode, void* stream) {
  const int gs = gshift_of(group_size);
  TAO_CHECK_ARG(gs > 0, "int4 dequant: group_size must be 32/64/128/256 (got %lld)",
                (long long)group_size);
  TAO_CHECK_ARG(N >= 0 && K >= 0 && K % group_size == 0,
                "int4 dequant: K (%lld) %% group_size (%lld) != 0", (long long)K,
                (long long)group_size);
  TAO_CHECK_ARG(mode == 0 || mode == 1, "int4 dequant: mode must be 0 or 1");
  if (N * K == 0) return TAO_OK;
  TAO_CHECK_ALIGN(w, 16, "w");
  TAO_CHECK_ALIGN(sz, 4, "sz");
  const int64_t total = N * (K / 8);
  if (mode == 0)
    launch(int4_dequant_kernel<0>, dim3(grid_for(total)), dim3(kBlock), 0,
                       as_stream(stream), packed, reinterpret_cast<const uint32_t*>(sz),
                       reinterpret_cast<uint4*>(w), total, K / 8, K / group_size, gs);
  else
    launch(int4_dequant_kernel<1>, dim3(grid_for(total)), dim3(kBlock), 0,
                       as_stream(stream), packed, reinterpret_cast<const uint32_t*>(sz),
                       reinterpret_cast<uint4*>(w), total, K / 8, K / group_size, gs);
  return check_launch("int4_dequant_kernel");
}

static int check_tile_args(int64_t N, int64_t K, int64_t ikt, int fmt, const char* who) {
  TAO_CHECK_ARG(ikt == 2 || ikt == 4 || ikt == 8, "%s: inner_k_tiles must be 2, 4, or 8", who);
  TAO_CHECK_ARG(fmt == kTileCuda || fmt == kTileRocm, "%s: tile_format must be 0 or 1", who);
  const int nm = fmt == kTileRocm ? 16 : 8;
  TAO_CHECK_ARG(N >= 0 && N % nm == 0, "%s: N (%lld) must be a multiple of %d", who, (long long)N,
                nm);
  TAO_CHECK_ARG(K >= 0 && K % (ikt * 16) == 0, "%s: K (%lld) must be a multiple of %lld", who,
                (long long)K, (long long)(ikt * 16));
  return TAO_OK;
}

int tao_unpack_tensor_core_tiled_layout(const int32_t* packed_w, int32_t* out, int64_t N,
                                        int64_t K, int64_t inner_k_tiles, int tile_format,
                                        void* stream) {
  int rc = check_tile_args(N, K, inner_k_tiles, tile_format, "unpack_tensor_core_tiled_layout");
  if (rc) return rc;
  if (N * K == 0) return TAO_OK;
  const int64_t KT = K / (inner_k_tiles * 16);
  const int64_t total = N * K / 8;
  launch(tile_unpack_kernel<0>, dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream),
         packed_w, (void*)out, (const uint16_t*)nullptr, total, (int)inner_k_tiles, KT, N, K, 32,
         tile_format);
  return check_launch("tile_unpack_kernel");
}

int tao_dequantize_tensor_core_tiled_layout(const int32_t* packed_w,
                                            const uint16_t* scales_and_zeros, uint16_t* out,
                                            int64_t N, int64_t K, int64_t group_size,
                                            int64_t inner_k_tiles, int tile_format,
                                            void* stream) {
  int rc = check_tile_args(N, K, inner_k_tiles, tile_format,
                           "dequantize_tensor_core_tiled_layout");
  if (rc) return rc;
  TAO_CHECK_ARG(gshift_of(group_size) > 0,
                "dequantize_tensor_core_tiled_layout: qGroupSize must be 32, 64, 128, or 256");
  TAO_CHECK_ARG(K % group_size == 0, "dequantize_tensor_core_tiled_layout: K %% group_size != 0");
  if (N * K == 0) return TAO_OK;
  const int64_t KT = K / (inner_k_tiles * 16);
  const int64_t total = N * K / 8;
  launch(tile_unpack_kernel<1>, dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream),
         packed_w, (void*)out, scales_and_zeros, total, (int)inner_k_tiles, KT, N, K,
         (int)group_size, tile_format);
  return check_launch("tile_dequant_kernel");
}

int tao_pack_tensor_core_tiled_layout(const int32_t* q, int32_t* packed_w, int64_t N, int64_t K,
                                      int64_t inner_k_tiles, int tile_format, void* stream) {
  int rc = check_tile_args(N, K, inner_k_tiles, tile_format, "pack_tensor_core_tiled_layout");
  if (rc) return rc;
  if (N * K == 0) return TAO_OK;
  const int64_t KT = K / (inner_k_tiles * 16);
  const int64_t total = N * K / 8;
  launch(tile_pack_kernel, dim3(grid_for(total)), dim3(kBlock), 0, as_stream(stream), q,
         packed_w, total, (int)inner_k_tiles, KT, K, tile_format);
  return check_launch("tile_pack_kernel");
}

// Host unpack of either tile format (checkpoints loaded on the CPU, tensor_core_tiled_layout.py)
int tao_unpack_tensor_core_tiled_layout_host(const int32_t* packed_w, int32_t* out, int64_t N,
                                             int64_t K, int64_t inner_k_tiles,
                                             int tile_format) {
  int rc = check_tile_args(N, K, inner_k_tiles, tile_format,
                           "unpack_tensor_core_tiled_layout (host)");
  if (rc) return rc;
  const int64_t KT = K / (inner_k_tiles * 16);
  const int64_t total = N * K / 8;
  for (int64_t i = 0; i < total; ++i) {
    int64_t n, ks[4];
    tile_coords(i, (int)inner_k_tiles, KT, tile_format, &n, ks);
    const uint32_t p = (uint32_t)packed_w[i];
    for (int q = 0; q < 4; ++q) {
      out[n * K + ks[q]] = (int32_t)((p >> (4 * q)) & 0xF);
      out[n * K + ks[q] + 1] = (int32_t)((p >> (16 + 4 * q)) & 0xF);
    }
  }
  return TAO_OK;
}

}  // extern "C"
