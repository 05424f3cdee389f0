/*
 * torchao_mi355x.h — C-ABI of the MI355X (gfx950) weight-only quantized linear path.
 *
 * This is the drop-in boundary. Every entry point takes plain device pointers, sizes and a
 * hipStream_t passed as `void*` (NULL = the legacy default stream); no torch types appear here.
 * Each function replaces one call site of the reference (torchao 0.13.0, cited file:line) —
 * the aten/torchao op that the reference's Python layout `impl` functions invoke.
 *
 * Conventions (mirroring the reference op conventions):
 *   - inputs are borrowed, contiguous, row-major; outputs are caller-allocated;
 *   - no entry point allocates, synchronises or copies host<->device, so every call is
 *     hipGraph-capturable (reference compiles decode with mode="reduce-overhead",
 *     torchao/_models/llama/generate.py:865-872);
 *   - bf16 tensors are passed as uint16_t bit patterns;
 *   - return value is TAO_OK (0) or a TAO_ERR_* code; tao_last_error() gives the message for the
 *     calling thread (the reference raises RuntimeError via TORCH_CHECK with the same meaning).
 *
 * int4 weight layout ("gfx950 row-stream layout"):
 *   packed : uint32 [N][K/8]; dword d of row n holds k = 8d..8d+7 with
 *            bits 4i..4i+3 = q[n][8d+2i], bits 16+4i..16+4i+3 = q[n][8d+2i+1]   (i = 0..3)
 *   sz     : bf16 [N][K/group][2] = (scale, zero) interleaved per (row, group)
 *   dequant: w = (q - 8) * scale + zero        (tinygemm float-zero domain)
 *
 * Companion headers of the same library: torchao_mi355x_llama.h (the fused kernels of the
 * end-to-end gpt-fast harness, BASELINE config 4) and torchao_mi355x_tune.h (internal: launch-shape
 * overrides, profiling and diagnostics for bench.py / tests / experiments; not a boundary).
 */
#ifndef TORCHAO_MI355X_H_
#define TORCHAO_MI355X_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  TAO_OK = 0,
  TAO_ERR_INVALID_ARGUMENT = 1, /* shape / alignment / group-size check failed   */
  TAO_ERR_UNSUPPORTED = 2,      /* valid request this build does not implement     */
  TAO_ERR_HIP = 3               /* a HIP runtime call or kernel launch failed      */
};

/* ---- library ------------------------------------------------------------------------------ */

/* Version string of this library ("torchao-mi355x <ver> gfx950"). */
const char* tao_version(void);
/* Message describing the last failed call on this thread ("" if none). */
const char* tao_last_error(void);
/* Number of hipDevices visible (0 if no GPU / runtime unavailable). Never fails. */
int tao_device_count(void);

/* ---- int4 weight-only (tinygemm-equivalent) ----------------------------------------------- */

/* y[M][N] = x[M][K] @ dequant(packed, sz)^T (+ bias[N]), bf16 in/out, fp32 accumulate.
 * Replaces aten._weight_int4pack_mm(x, packed, qGroupSize, qScaleAndZeros) called at
 * torchao/dtypes/uintx/tensor_core_tiled_layout.py:104 (plus the bias add at :112-113).
 * group_size in {32,64,128,256}; K % group_size == 0; M >= 0 (M == 0 is a no-op).
 * x, y: 16-B aligned rows. bias may be NULL. */
int tao_int4wo_linear_bf16(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                           const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                           int64_t group_size, void* stream);

/* packed[N][K/8] <- q[N][K] (int32 values 0..15).
 * Replaces aten._convert_weight_to_int4pack(u8, inner_k_tiles) at
 * torchao/dtypes/uintx/tensor_core_tiled_layout.py:279 (device kernel). K % 8 == 0. */
int tao_int4_pack(const int32_t* q, uint32_t* packed, int64_t N, int64_t K, void* stream);

/* packed[N][K/8] <- u8[N][K/2] where u8 = q[:, 0::2] << 4 | q[:, 1::2]
 * (the operand the reference builds at tensor_core_tiled_layout.py:276). */
int tao_int4_pack_u8(const uint8_t* q_u8, uint32_t* packed, int64_t N, int64_t K,
                     void* stream);

/* q[N][K] (int32 0..15) <- packed. Exact inverse of tao_int4_pack.
 * Replaces the identity-matmul recovery in get_plain (tensor_core_tiled_layout.py:465-517). */
int tao_int4_unpack(const uint32_t* packed, int32_t* q, int64_t N, int64_t K, void* stream);

/* w[N][K] bf16 <- dequant(packed, sz).
 * mode 0: bf16((q-8)*s) then bf16(+z) — the two roundings of _dequantize_affine_tinygemm
 *         (torchao/quantization/quant_primitives.py:1019-1023), bit-exact to AQT.dequantize();
 * mode 1: one rounding of fma(q-8, s, z) — the semantics of the reference dequant kernel
 *         (torchao/csrc/cuda/tensor_core_tiled_layout/tensor_core_tiled_layout.cu:184-190). */
int tao_int4_dequant(const uint32_t* packed, const uint16_t* sz, uint16_t* w, int64_t N,
                     int64_t K, int64_t group_size, int mode, void* stream);

/* Host (CPU) versions of pack / unpack for weights that are quantized on the CPU before being
 * moved to the GPU (quantize_ on a CPU model). Plain C++; identical bytes to the device kernels. */
int tao_int4_pack_host(const int32_t* q, uint32_t* packed, int64_t N, int64_t K);
int tao_int4_unpack_host(const uint32_t* packed, int32_t* q, int64_t N, int64_t K);

/* ---- reference tile-format compat (torchao::*_tensor_core_tiled_layout) ------------------- */

/* The reference tile format: int32 [N/8][K/(ikt*16)][32][ikt/2], inner_k_tiles (ikt) in {2,4,8}.
 * Two nibble maps share that shape (tile_format):
 *   0 = CUDA: the semantics of the reference's own kernels (tensor_core_tiled_layout.cu:131-215),
 *       i.e. what aten._convert_weight_to_int4pack writes on CUDA builds of PyTorch;
 *   1 = ROCm: what aten._convert_weight_to_int4pack writes on PyTorch-ROCm (gfx950, measured:
 *       experiments/probe_aten_tile_map.py, tests/golden/aten_tile_map_rocm.npz), the bytes seen
 *       flat as [N/16][K/(ikt*16)][64][ikt/2] for wave64 lanes; needs N % 16 == 0.
 * A checkpoint saved by torchao holds whichever format its producing build wrote. */

/* out[N][K] int32 <- tile-format packed_w.
 * Replaces torchao::unpack_tensor_core_tiled_layout (torchao/ops.py:255-296,
 * tensor_core_tiled_layout.cu:320-368). */
int tao_unpack_tensor_core_tiled_layout(const int32_t* packed_w, int32_t* out, int64_t N,
                                        int64_t K, int64_t inner_k_tiles, int tile_format,
                                        void* stream);

/* The same on the host (checkpoint conversion of CPU-resident state dicts). */
int tao_unpack_tensor_core_tiled_layout_host(const int32_t* packed_w, int32_t* out, int64_t N,
                                             int64_t K, int64_t inner_k_tiles, int tile_format);

/* out[N][K] bf16 <- fma(q-8, s, z) with scales_and_zeros [K/g][N][2] bf16 (tinygemm packing,
 * torchao/quantization/utils.py:395-409). Replaces torchao::dequantize_tensor_core_tiled_layout
 * (torchao/ops.py:299-377, tensor_core_tiled_layout.cu:223-316). */
int tao_dequantize_tensor_core_tiled_layout(const int32_t* packed_w,
                                            const uint16_t* scales_and_zeros, uint16_t* out,
                                            int64_t N, int64_t K, int64_t group_size,
                                            int64_t inner_k_tiles, int tile_format,
                                            void* stream);

/* Tile-format packer (the inverse of the unpack above): packed_w <- q[N][K] int32; with
 * tile_format 1 bit-identical to PyTorch-ROCm's aten._convert_weight_to_int4pack (the call at
 * torchao/dtypes/uintx/tensor_core_tiled_layout.py:279). K % (ikt*16) == 0. */
int tao_pack_tensor_core_tiled_layout(const int32_t* q, int32_t* packed_w, int64_t N, int64_t K,
                                      int64_t inner_k_tiles, int tile_format, void* stream);

/* ---- int8 weight-only ---------------------------------------------------------------------- */

/* y[M][N] = bf16( bf16(x @ w^T) * scale[n] ) (+ bias), w int8 [N][K], scale bf16 [N].
 * Replaces torch.mm(x, w.t().to(bf16)) * scale at torchao/dtypes/uintx/plain_layout.py:256-266. */
int tao_int8wo_linear_bf16(const uint16_t* x, const int8_t* w, const uint16_t* scale,
                           const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                           void* stream);

/* ---- int8 dynamic activation x int8 weight -------------------------------------------------- */

/* Per-token symmetric reduced-range int8 quantization of x [M][K] bf16:
 *   s[m] = max(bf16(amax(|x[m]|) / 127), bf16(1e-5)); q = clamp(rne(bf16(x * bf16(1/s))), -127, 127)
 * Replaces _int8_symm_per_token_reduced_range_quant (torchao/quantization/quant_api.py:1258-1273). */
int tao_int8_quant_per_token(const uint16_t* x, int8_t* q, uint16_t* scale, int64_t M,
                             int64_t K, void* stream);

/* y[M][N] = bf16( bf16( bf16(xq @ wq^T) * xs[m] ) * ws[n] ) (+ bias), exact int32 accumulation.
 * Replaces int_scaled_matmul + the weight-scale epilogue at
 * torchao/dtypes/uintx/plain_layout.py:294-315 and torchao/kernel/intmm.py:108-143. */
int tao_int8_scaled_mm_bf16(const int8_t* xq, const uint16_t* xs, const int8_t* wq,
                            const uint16_t* ws, const uint16_t* bias, uint16_t* y, int64_t M,
                            int64_t N, int64_t K, void* stream);

/* One token (M <= 1) through both steps above in ONE launch: every workgroup quantises x [K]
 * bf16 per token into LDS (tao_int8_quant_per_token's arithmetic) and runs the int8 x int8 GEMV
 * on it. Bit-identical to tao_int8_quant_per_token + tao_int8_scaled_mm_bf16 (K % 16 == 0,
 * K <= 65536). Replaces LinearActivationQuantizedTensor's quantize-then-F.linear for the default
 * Int8DynamicActivationInt8WeightConfig recipe at decode (linear_activation_quantized_tensor.py
 * _quantized_linear_op; quant_api.py:1258-1273 + plain_layout.py:294-315). */
int tao_int8_dyn_linear_bf16(const uint16_t* x, const int8_t* wq, const uint16_t* ws,
                             const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                             void* stream);

/* Device-side faults of the decode kernels since the last call, read and cleared (synchronous:
 * call outside graph capture). bits & 1: a KV-cache position outside [0, T) reached
 * tao_rope_kv_bf16 / tao_int4wo_decode_bf16's rope_kv epilogue; those launches wrote no cache
 * row and tao_attn_decode_bf16 clamped its key count to T. (The reference's index_put KV cache
 * device-asserts in this case, torchao/_models/llama/model.py KVCache.update.) bits & 2: a split-K
 * reducer of the prefill GEMMs timed out waiting for its publishers; that output tile was not
 * written (never expected; the ticket is left consistent for later launches). */
int tao_decode_status(int* bits);

/* Fused int4 weight quantizer (Int4WeightOnlyConfig's from_hp_to_intx in one pass):
 * w [rows][K] bf16 -> packed [rows][K/8] (row-stream nibbles, as tao_int4_pack) and
 * scales_and_zeros [rows][K/g][2] bf16, per group of g: s = clamp(bf16(bf16(max-min)/15), eps),
 * z = bf16(min + 8 s), q = clamp(rint(bf16(bf16(w - bf16(z - 8 s)) / s)), 0, 15), each step
 * rounded to bf16 as the reference's torch ops do (_choose_qparams_affine_tinygemm
 * quant_primitives.py:1238-1307, _quantize_affine_tinygemm :461-573). g in {32,64,128,256}. */
int tao_int4_quantize_bf16(const uint16_t* w, uint32_t* packed, uint16_t* scales_and_zeros,
                           int64_t rows, int64_t K, int64_t group_size, float eps, void* stream);

/* Fused symmetric per-row int8 weight quantizer (Int8WeightOnlyConfig /
 * Int8DynamicActivationInt8WeightConfig weights; choose_qparams_affine SYMMETRIC +
 * quantize_affine, quant_primitives.py): s[r] = bf16(max(bf16(max|w[r]| / 127.5), eps)),
 * q = clamp(rint(bf16(w * bf16(1 / s))), -128, 127). K % 8 == 0. Replaces the torch-op
 * quantisation behind to_affine_quantized_intx in _int8_weight_only_quantize_tensor
 * (torchao/quantization/quant_api.py:1223-1240) for bf16 GPU weights. */
int tao_int8_quantize_rows_bf16(const uint16_t* w, int8_t* q, uint16_t* scale, int64_t rows,
                                int64_t K, float eps, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TORCHAO_MI355X_H_ */
