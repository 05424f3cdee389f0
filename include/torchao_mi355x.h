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
/* Name of the last kernel this thread launched through the library (its routing decision, for
 * measurement labels); "" before the first launch. */
const char* tao_last_kernel(void);
/* Number of hipDevices visible (0 if no GPU / runtime unavailable). Never fails. */
int tao_device_count(void);

/* Per-kernel timing for benchmarks (not used on the inference path). Between begin and end,
 * the calling thread's next `capacity` kernel launches carry a start/stop hipEvent pair written
 * by the kernel's own dispatch packet (hipExtLaunchKernelGGL) — the interval rocprofv3 reports
 * as the kernel duration. end() synchronises on the events and writes one duration (ms) per
 * recorded launch, in launch order; *count receives how many. Do not open a session while
 * capturing a hipGraph. */
int tao_profile_begin(int capacity);
int tao_profile_end(float* durations_ms, int capacity, int* count);

/* ---- int4 weight-only (tinygemm-equivalent) ----------------------------------------------- */

/* y[M][N] = x[M][K] @ dequant(packed, sz)^T (+ bias[N]), bf16 in/out, fp32 accumulate.
 * Replaces aten._weight_int4pack_mm(x, packed, qGroupSize, qScaleAndZeros) called at
 * torchao/dtypes/uintx/tensor_core_tiled_layout.py:104 (plus the bias add at :112-113).
 * group_size in {32,64,128,256}; K % group_size == 0; M >= 0 (M == 0 is a no-op).
 * x, y: 16-B aligned rows. bias may be NULL. */
int tao_int4wo_linear_bf16(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                           const uint16_t* bias, uint16_t* y, int64_t M, int64_t N, int64_t K,
                           int64_t group_size, void* stream);

/* tao_int4wo_linear_bf16 (no bias) with the SwiGLU of interleaved (gate, up) output rows folded
 * into the epilogue: y [M][N/2] = bf16(bf16(silu(a_i)) * b_i), (a_i, b_i) = the bf16 outputs of
 * rows (2i, 2i+1) (a w1||w3 weight merged row-interleaved; N % 16 == 0). Replaces the prefill's
 * `F.silu(w1(x)) * w3(x)` (gpt-fast model.py FeedForward.forward) as one launch. Served where
 * the single-fetch GEMM is routed; TAO_ERR_UNSUPPORTED elsewhere (the caller then runs the linear
 * and tao_silu_mul_bf16). */
int tao_int4wo_linear_swiglu_bf16(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                                  uint16_t* y, int64_t M, int64_t N, int64_t K,
                                  int64_t group_size, void* stream);

/* The prefill's wqkv linear (int4 weight-only, no bias) with RoPE and the KV-cache write of
 * tao_rope_kv_bf16 folded into the epilogue: x [B*S][K] bf16; weight [(H + 2 Hkv) D][K]; q
 * rotated into q_out [B][H][S][D]; k rotated and v written into the caches [B][Hkv][T][D] at row
 * pos[s] (a position outside [0, T) writes no cache row and sets tao_decode_status bit 1).
 * D == 128; q_out and the caches 16-B aligned. Replaces wqkv + apply_rotary_emb +
 * KVCache.update (gpt-fast model.py Attention.forward) at prefill as one launch. Served where
 * the single-fetch GEMM is routed; TAO_ERR_UNSUPPORTED elsewhere. */
int tao_int4wo_linear_rope_kv_bf16(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                                   int64_t K, int64_t group_size, const float* freqs,
                                   const int64_t* pos, uint16_t* q_out, uint16_t* k_cache,
                                   uint16_t* v_cache, int64_t B, int64_t S, int64_t H,
                                   int64_t Hkv, int64_t D, int64_t T, void* stream);

/* Tuning hooks (tao_tune_*). Every override is THREAD-LOCAL: it re-routes only launches issued
 * from the thread that set it, never another thread's model. tao_tune_reset() restores every
 * built-in choice for the calling thread (torchao.kernel.tuning(...) wraps set + reset). */
int tao_tune_reset(void);

/* Split-K / last-arriver hand-off form for the calling thread: 0 = fence-free sc1 protocol
 * (built-in under the HIP 7.0 / 7.2 runtimes it was validated on; MI355X_MICROARCH.md "Hand-offs
 * measured with sc1 loads in place of the acquire", first row), 1 = the same plus agent release /
 * acquire fences (the HIP memory-model form; built-in under any other runtime version).
 * Both give bit-identical results (tests/test_gpu_gemm_tiles.py). */
int tao_tune_splitk_fenced(int fenced);

/* The calling thread's current split-K hand-off form (0 fence-free, 1 fenced): the built-in
 * choice unless tao_tune_splitk_fenced overrode it. No device work. */
int tao_query_splitk_fenced(void);
/* Split-K ticket layout: unsigned words between consecutive tiles' counters, 32 (built-in: each
 * tile's ticket on its own 128-B line, so the S workgroups of one tile do not contend with other
 * tiles' arrivals) or 1 (packed). Thread-local; for measurement. */
int tao_tune_cnt_stride(int stride);

/* Tuning hook (benchmarks / autotuning sweeps): override the M == 1 int4 GEMV launch shape,
 * for the calling thread. rows_per_wave in {1,2,4,8}; waves_k = waves splitting K inside a workgroup
 * (1..8); row_groups = row groups per workgroup; waves_k * row_groups <= 8; occupancy in {4,8}
 * = minimum waves per SIMD the register budget targets (rows_per_wave 4 only).
 * 0 for any field keeps the built-in choice; all zeros restores the defaults. */
int tao_tune_int4_gemv(int rows_per_wave, int waves_k, int row_groups, int occupancy);

/* Tuning hook: the weight-only linears (int4 and int8) use the GEMV kernels for M <= max_gemv_m
 * and the MFMA skinny GEMM above it. 0 restores the built-in crossover (M <= 2, or M <= 4 for
 * weights of at most 32 Mi elements). Calling thread only. */
int tao_tune_linear_crossover(int max_gemv_m);

/* Tuning hook: force the MFMA skinny GEMM's M tile (16/32/64/128), k-groups per workgroup
 * (1/2/4; 4 waves each) and K slices across workgroups (1..64); 0 = the built-in choice for
 * each. Calling thread only. */
int tao_tune_gemm(int m_tile, int k_groups, int splits);

/* Calling thread's choice of the int8 dynamic-activation GEMM kernel (M above the GEMV crossover):
 * 0 = auto (the LDS-staged int8 kernel when K % 128 == 0, M >= 128 and its 64-row tiles number
 * >= 192, unsplit; else the per-wave-column MFMA kernel), 1 = always the per-wave-column kernel,
 * 2 = the LDS-staged kernel whenever K % 128 == 0. tao_tune_gemm's m_tile (64 / 128) and
 * splits also apply to the LDS kernel. */
int tao_tune_gemm_algo(int algo);

/* Register-ring depth (k steps in flight) of the LDS-staged int8 GEMM: 0 = built-in (3 at M tile
 * 128, 4 at 64), else 2, 3, 4, 6 or 8 (8 only at M tile 64; 128 takes 6). Calling thread only. */
int tao_tune_gemm_depth(int depth);

/* Column tile of the LDS-staged int8 GEMM: 0 = built-in (128 when M >= 256 and 128 x 128 tiles
 * number >= 256, else 64), 64, or 128 (each wave 2 x 4 16x16 tiles per M half; ring depth 2 or
 * 3). Calling thread only; for sweeps. */
int tao_tune_gemm_bn(int bn);

/* Workgroup order of the MFMA GEMMs: 0 = plain grid order (built-in), 1 = the M tiles that share
 * a weight tile back to back on one XCD (its L2 serves the re-reads: fewer HBM bytes, measured
 * no faster). Calling thread only; for A/B measurement. */
int tao_tune_gemm_order(int order);
/* Columns per wave of the MFMA GEMMs: 0 = built-in, 1 = 16, 2 = 32 (one A-fragment LDS read
 * feeds two MFMAs; the workgroup tile is 128 columns wide). Calling thread only; for A/B
 * measurement. */
int tao_tune_gemm_nw(int nw);
/* The MFMA GEMMs' measured launch-shape table for the Llama-3 linears (csrc/gemm_table.inc):
 * 0 = used (built-in), 1 = off (heuristic only). Calling thread only; for A/B measurement. */
int tao_tune_gemm_table(int off);
/* int4 MFMA GEMM kernel: 0 = built-in, 1 = the 32x32x16-MFMA kernel (gemm32_int4_kernel).
 * Calling thread only; for A/B measurement. */
int tao_tune_int4_mfma32(int on);
/* Weight-shared tile GEMM (csrc/gemm_tile.hip: 4 waves split the rows of a 64/128 x 64 tile, each
 * weight dequantised once per workgroup into LDS, x fragments straight from global, split-K
 * reduced by every slice): mode 0 = built-in routing, 1 = never (the MFMA kernels above),
 * 2 = wherever it applies (K a multiple of its step, M above the GEMV crossover); splits 0 =
 * built-in, else the largest power of two <= splits (<= 16). Calling thread only. */
int tao_tune_gemm_tile(int mode, int splits);

/* The single-fetch prefill GEMM (csrc/gemm_sf.hip: 128-row tiles so each weight tile is fetched by
 * one workgroup, 8 waves, both operands by LDS-DMA in full lines, K split over workgroups; for
 * int4 with wm 1 the 32x32x16 kernel of csrc/gemm_sf32.hip) for the int4 weight-only and int8
 * dynamic linears. mode 0 = built-in routing (64 < M <= 128 at the Llama-3-8B and -70B shapes
 * where it measured faster than the MFMA GEMMs), 1 = never, 2 = wherever the shape is supported
 * (K % 128 (int4) / 256 (int8) == 0; M <= 128 per 128-row tile). bn (32 / 64 / 128 / 256), wm
 * (waves along M: 2 / 4 / 8; int4: 1 = the 32x32x16 kernel, one wave per 32 columns), splits,
 * stages (2-4), a_steps (K steps of each publishing slice) and ks (int8 k step 128 / 256; int4
 * with wm 1: 1 or 2 waves per 32-column group, splitting each step's k): 0 = built-in.
 * Thread-local; for measurement. */
int tao_tune_gemm_sf(int mode, int bn, int wm, int splits, int stages, int a_steps, int ks);
/* Single-fetch GEMM split-K seam: -1 = built-in (per routed shape), 1 = spread (each of a tile's
 * S workgroups sums and stores 1/S of the tile; splits 2 / 4 / 8 only, others take 0), 0 = fixed
 * reducer (slice S-1 sums the whole tile). Thread-local; for measurement. */
int tao_tune_gemm_sf_seam(int seam);
/* Reducer poll timeouts of the single-fetch GEMM since the last call (*bits != 0: some split
 * launch's outputs are invalid; never expected, see gemm_sf.hip). Synchronous. */
int tao_gemm_sf_status(unsigned* bits);

/* Measurement kernel (bench.py, not the product path): a pure streaming read of `bytes` (a
 * positive multiple of 8192) from `buf` (16-B aligned) with 16-B non-temporal loads; `sink` is
 * >= 4 KiB of device memory the kernel may write (it never does in practice). Graph-capturable. */
int tao_hbm_read_probe(const void* buf, int64_t bytes, void* sink, void* stream);
/* Number of split-K workspaces currently owned by captured graphs (each is released with its
 * graph). Diagnostic for tests; never fails. */
int tao_graph_workspace_count(void);

/* M == 1 int4 linears without bias: 1 = stage x once per workgroup in LDS (the decode RMSNorm
 * prologue's copy, without the norm), 0 = built-in policy. Calling thread only; for sweeps. */
int tao_tune_int4_xlds(int mode);

/* RMSNorm prologue of tao_int4wo_decode_bf16: 0 = exact (normalise x with the reference's two
 * bf16 roundings before the slices; built-in), 1 = deferred (stage bf16(x * norm_weight), scale
 * each output by rsqrt(mean(x^2) + eps) at the end). Calling thread only; for measurement. */
int tao_tune_int4_norm(int mode);

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

/* Tuning hook: M == 1 launch shape of the int8 decode GEMVs (int8 weight-only and int8 x int8:
 * rows per wave 2/4/8, waves along K, row groups per workgroup; 0 = built-in heuristic).
 * Calling thread only; for sweeps (experiments/sweep_int8.py). */
int tao_tune_int8_gemv(int rows_per_wave, int waves_k, int row_groups);
/* Per-token int8 quantisation kernel (A/B only): 0 = one wave per token, the token held in
 * registers (default, K <= 8192); 1 = one 256-thread workgroup per token. Bit-identical. */
int tao_tune_int8_quant(int block);

/* ---- fused decode-step kernels of the end-to-end harness (torchao/_models/llama) -------------
 * Not on the int4 path: the fusions the reference gets from torch.compile in its gpt-fast
 * harness (torchao/_models/llama/generate.py:865-875, model.py:405-501). */

/* y[r] = bf16(bf16(x[r] * rsqrt(mean(x[r]^2) + eps)) * w), rows of `dim` bf16 (dim % 8 == 0).
 * Replaces RMSNorm.forward (torchao/_models/llama/model.py:489-501). */
int tao_rmsnorm_bf16(const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t rows,
                     int64_t dim, float eps, void* stream);

/* h = x + res (bf16, rounded as torch's bf16 add), stored, then y = RMSNorm(h) as
 * tao_rmsnorm_bf16: the residual add and the next norm of a prefill block in one launch,
 * bit-identical to the two. rows x dim, dim % 8 == 0. */
int tao_add_rmsnorm_bf16(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* h,
                         uint16_t* y, int64_t rows, int64_t dim, float eps, void* stream);

/* qkv [B*S][(H + 2 Hkv) * D] bf16 -> q_out [B][H][S][D] rotated; k (rotated) and v written to
 * k_cache / v_cache [B][Hkv][T][D] at positions pos[S] (int64). freqs: rotary table
 * [rows][D/2][2] fp32 (cos, sin), row pos[s]. Replaces apply_rotary_emb + KVCache.update
 * (model.py:547-557, 175-196). */
int tao_rope_kv_bf16(const uint16_t* qkv, const float* freqs, const int64_t* pos,
                     uint16_t* q_out, uint16_t* k_cache, uint16_t* v_cache, int64_t B, int64_t S,
                     int64_t H, int64_t Hkv, int64_t D, int64_t T, void* stream);

/* One-query attention over keys 0..pos[0] of the caches, GQA (H % Hkv == 0, H/Hkv <= 8),
 * D == 128: out [B][1][H*D] bf16. partial: fp32 workspace of B*Hkv*ceil(T/64)*(H/Hkv)*(D+2)
 * for the two-launch split (T > 1024, or tao_tune_attn 1); NULL = the library's per-stream
 * workspace (run once eagerly before graph capture). Shorter caches run one single-pass kernel
 * and do not touch it.
 * Replaces F.scaled_dot_product_attention at decode (model.py:441-476). */
int tao_attn_decode_bf16(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                         const int64_t* pos, float* partial, uint16_t* out, int64_t B, int64_t H,
                         int64_t Hkv, int64_t D, int64_t T, float scale, void* stream);

/* Prefill attention: S queries per (batch, head), q [B][H][S][D] bf16 (RoPE applied), query s at
 * position pos[s] attending cache keys 0..pos[s] (the causal mask of a prompt written into the
 * caches at pos), GQA (H % Hkv == 0), D == 128: out [B][S][H*D] bf16, fp32 softmax. Replaces the
 * masked F.scaled_dot_product_attention over the caches of the reference's Attention.forward
 * (gpt-fast model.py) at prefill. */
int tao_attn_prefill_bf16(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                          const int64_t* pos, uint16_t* out, int64_t B, int64_t H, int64_t Hkv,
                          int64_t D, int64_t S, int64_t T, float scale, void* stream);

/* Calling thread's choice of the decode-attention kernel: 0 = single-pass workgroup per query head
 * (f32 math, whole-line K loads) for T <= 1024, else the two-launch split (default); 1 = two-launch
 * split. */
int tao_tune_attn(int mode);

/* Device-side faults of the decode kernels since the last call, read and cleared (synchronous:
 * call outside graph capture). bits & 1: a KV-cache position outside [0, T) reached
 * tao_rope_kv_bf16 / tao_int4wo_decode_bf16's rope_kv epilogue; those launches wrote no cache
 * row and tao_attn_decode_bf16 clamped its key count to T. (The reference's index_put KV cache
 * device-asserts in this case, torchao/_models/llama/model.py KVCache.update.) */
int tao_decode_status(int* bits);

/* y = bf16(bf16(silu(a)) * b) elementwise over n bf16 (n even). Replaces FeedForward's
 * F.silu(w1(x)) * w3(x) (model.py:485-486). b == NULL: a holds n interleaved (gate, up) pairs
 * (2n bf16, the output of an interleaved w13 linear) and y[i] = silu(a[2i]) * a[2i+1]. */
int tao_silu_mul_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, int64_t n,
                      void* stream);

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
 * q = clamp(rint(bf16(w * bf16(1 / s))), -128, 127). K % 8 == 0. */
int tao_int8_quantize_rows_bf16(const uint16_t* w, int8_t* q, uint16_t* scale, int64_t rows,
                                int64_t K, float eps, void* stream);

/* out[r] = argmax over n bf16 logits of row r (first index of the maximum; a positive-sign NaN
 * counts as the maximum, as in torch.argmax) as int64. Replaces logits.argmax(dim=-1) of the greedy decode
 * (generate.py:111-142, sample with temperature 0). */
int tao_argmax_bf16(const uint16_t* x, int64_t* out, int64_t rows, int64_t n, void* stream);

/* One decode step's greedy bookkeeping in one launch (batch 1): cur[0] = argmax of x[n] (the
 * rule of tao_argmax_bf16), then tokens[pos[0] + 1] = cur[0] (when inside [0, max_len)) and
 * pos[0] += 1. Replaces the harness's argmax + pos.add_ + tokens.index_copy_ + cur.copy_
 * (torchao/_models/llama/generate.py decode loop, reference generate.py:111-142). */
int tao_argmax_advance_bf16(const uint16_t* x, int64_t n, int64_t* cur, int64_t* pos,
                            int64_t* tokens, int64_t max_len, void* stream);

/* One token through an int8 weight-only linear with its decode-step neighbours fused (the
 * int8 counterpart of tao_int4wo_decode_bf16; csrc/int8_gemv.hip). Operands of
 * tao_int8wo_linear_bf16 at M == 1 (x [K] bf16, w [N][K] int8, scale [N] bf16, no bias).
 *   norm_weight  NULL: x as is; else [K] bf16, x -> bf16(bf16(x * rsqrt(mean(x^2) + eps)) * w).
 *   epilogue 0: y [N] = the linear; 1 (swiglu): rows (2i, 2i+1) = (w1_i, w3_i), y [N/2] =
 *   bf16(bf16(silu(a)) * b); 2 (rope_kv): rows [q | k | v] heads, y [n_head * head_dim] = rotated
 *   q, rotated k and v written to k_cache / v_cache [n_kv_head][max_seq][head_dim] at pos[0]
 *   (outside [0, max_seq): no cache row written, reported by tao_decode_status).
 * Each result equals rmsnorm -> tao_int8wo_linear_bf16 -> silu_mul / rope_kv. Replaces, at
 * decode, the RMSNorm / SiLU-mul / RoPE + KVCache.update ops around the reference's int8
 * weight-only linears (torchao/_models/llama/model.py). */
int tao_int8wo_decode_bf16(const uint16_t* x, const int8_t* w, const uint16_t* scale, int64_t N,
                           int64_t K, const uint16_t* norm_weight, float eps, int epilogue,
                           uint16_t* y, const float* freqs, const int64_t* pos, uint16_t* k_cache,
                           uint16_t* v_cache, int64_t n_head, int64_t n_kv_head, int64_t head_dim,
                           int64_t max_seq, void* stream);

/* The same decode-step fusions on the int8 dynamic-activation linear (one token; the per-token
 * int8 quantisation of the normalised token inside the kernel, as tao_int8_dyn_linear_bf16
 * does for the plain token). Operands and epilogues as tao_int8wo_decode_bf16; equals
 * rmsnorm -> tao_int8_dyn_linear_bf16 -> silu_mul / rope_kv up to the norm's fp32 sum order.
 * K <= 32768 (<= 16384 with norm_weight). Replaces, at decode, the ops around the reference's
 * Int8DynamicActivationInt8WeightConfig linears (model.py, quant_api.py:1258-1273). */
int tao_int8dq_decode_bf16(const uint16_t* x, const int8_t* w, const uint16_t* scale, int64_t N,
                           int64_t K, const uint16_t* norm_weight, float eps, int epilogue,
                           uint16_t* y, const float* freqs, const int64_t* pos, uint16_t* k_cache,
                           uint16_t* v_cache, int64_t n_head, int64_t n_kv_head, int64_t head_dim,
                           int64_t max_seq, void* stream);

/* Decode-step fused int4 linear, M = 1: y = epilogue(rmsnorm(x) W^T) in one launch, with the
 * operands of tao_int4wo_linear_bf16 (x [K] bf16, packed [N][K/8], scales_and_zeros [N][K/g]).
 *   norm_weight  NULL: x is used as is; else [K] bf16 and x -> bf16(bf16(x * rsqrt(mean(x^2) +
 *                eps)) * norm_weight) first (= tao_rmsnorm_bf16; RMSNorm, model.py:489-501).
 *   epilogue 0   y [N] bf16 (the plain linear).
 *   epilogue 1   rows (2i, 2i+1) are (w1_i, w3_i): y [N/2] = bf16(bf16(silu(a)) * b)
 *                (= tao_silu_mul_bf16 over w1 and w3 outputs; FeedForward, model.py:485-486).
 *   epilogue 2   rows are wqkv's [q | k | v] heads, N = (n_head + 2 n_kv_head) * head_dim:
 *                y [n_head * head_dim] = rotated q, k rotated and v stored into k_cache /
 *                v_cache [n_kv_head][max_seq][head_dim] at pos[0] (= tao_rope_kv_bf16 with
 *                B = S = 1; Attention.forward, model.py:547-557).
 * freqs/pos/caches/head sizes are read only by epilogue 2. Same bf16 roundings as the unfused
 * kernels; the one difference is the order of the fp32 sum of squares in the RMSNorm. */
int tao_int4wo_decode_bf16(const uint16_t* x, const uint32_t* packed,
                           const uint16_t* scales_and_zeros, int64_t N, int64_t K,
                           int64_t group_size, const uint16_t* norm_weight, float eps,
                           int epilogue, uint16_t* y, const float* freqs, const int64_t* pos,
                           uint16_t* k_cache, uint16_t* v_cache, int64_t n_head,
                           int64_t n_kv_head, int64_t head_dim, int64_t max_seq, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TORCHAO_MI355X_H_ */
