/*
 * torchao_mi355x_llama.h — fused kernels of the end-to-end decode / prefill harness
 * (torchao/_models/llama, BASELINE config 4). They replace the ops around the quantized linears
 * of the reference's gpt-fast model (torchao/_models/llama/model.py), which the reference gets
 * from torch.compile (generate.py:865-875). Same conventions as include/torchao_mi355x.h.
 */
#ifndef TORCHAO_MI355X_LLAMA_H_
#define TORCHAO_MI355X_LLAMA_H_

#include "torchao_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

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
/* The residual add + RMSNorm after a linear whose K slices were NOT reduced in-kernel
 * (tao_int4wo_linear_partials_f32): part [splits][rows][dim] fp32; the linear's output is
 * bf16(sum over slices, in slice order) (bit-identical to the single-fetch GEMM's own bf16
 * output), h = bf16(x + it), y = RMSNorm(h) * w as tao_add_rmsnorm_bf16. dim <= 8192. */
int tao_add_rmsnorm_partials_bf16(const uint16_t* x, const float* part, int64_t splits,
                                  const uint16_t* w, uint16_t* h, uint16_t* y, int64_t rows,
                                  int64_t dim, float eps, void* stream);
/* int4 weight-only linear (x [M][K] bf16, the library's packed layout) whose K slices write fp32
 * partial tiles part [S][M][N] for the NEXT launch to sum instead of meeting at an in-kernel
 * split-K seam; S from tao_int4wo_linear_partial_slices (0 = not served for this shape: run the
 * plain linear). Replaces the prefill's wo / w2 `F.linear` + residual add
 * (torchao/_models/llama/model.py TransformerBlock.forward) together with the add + norm above. */
int tao_int4wo_linear_partial_slices(int64_t M, int64_t N, int64_t K, int64_t group_size,
                                     int* slices);
int tao_int4wo_linear_partials_f32(const uint16_t* x, const uint32_t* packed, const uint16_t* sz,
                                   float* part, int64_t M, int64_t N, int64_t K,
                                   int64_t group_size, void* stream);

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

/* Split decode attention (the first half of the decode attention + wo pair): the single-pass
 * kernel of tao_attn_decode_bf16 over `splits` (2 or 4) key ranges of each query head, one
 * workgroup per (batch, head, split), each range ceil(L / splits) keys rounded up to 16 (L =
 * pos[0] + 1 clamped to [1, T]). Writes the unnormalised partials: partial [B * H][splits][132]
 * fp32 = o[128] (sum over the range of exp(s - m) v), m, l, 2 pad (an empty range: o = 0,
 * m = -inf, l = 0). D == 128; partial 16-B aligned. tao_attn_merge_bf16 (or the wo linear
 * tao_int4wo_attn_out_bf16) finishes it. Replaces F.scaled_dot_product_attention at decode
 * (model.py:441-476), spread over splits x the workgroups of the one-pass kernel. */
int tao_attn_decode_split_bf16(const uint16_t* q, const uint16_t* k_cache,
                               const uint16_t* v_cache, const int64_t* pos, float* partial,
                               int64_t B, int64_t H, int64_t Hkv, int64_t D, int64_t T, float scale,
                               int64_t splits, void* stream);

/* out [B][1][H * D] bf16 = the merged split partials of tao_attn_decode_split_bf16:
 * bf16(sum_s o_s w_s * (1 / sum_s l_s w_s)), w_s = exp(m_s - max m). D == 128. */
int tao_attn_merge_bf16(const float* partial, uint16_t* out, int64_t B, int64_t H, int64_t D,
                        int64_t splits, void* stream);

/* The attention output linear of a decode step with the split merge folded into its x load: y [N]
 * = bf16(bf16(W x) + residual[n]) with x = tao_attn_merge_bf16(partial) (batch 1, K = n_head *
 * 128), W int4 (the operands of tao_int4wo_linear_bf16); residual may be NULL. Every workgroup
 * merges x into LDS while its first weight slices are in flight. Bit-identical to
 * tao_attn_merge_bf16 -> tao_int4wo_linear_bf16 (bias = residual) up to the GEMV's launch shape.
 * Replaces the wo linear + residual add after attention (model.py Attention.forward,
 * TransformerBlock.forward) at decode. */
int tao_int4wo_attn_out_bf16(const float* partial, int64_t splits, int64_t n_head,
                             const uint32_t* packed, const uint16_t* scales_and_zeros, int64_t N,
                             int64_t K, int64_t group_size, const uint16_t* residual, uint16_t* y,
                             void* stream);

/* Prefill attention: S queries per (batch, head), q [B][H][S][D] bf16 (RoPE applied), query s at
 * position pos[s] attending cache keys 0..pos[s] (the causal mask of a prompt written into the
 * caches at pos), GQA (H % Hkv == 0), D == 128: out [B][S][H*D] bf16, fp32 softmax. Replaces the
 * masked F.scaled_dot_product_attention over the caches of the reference's Attention.forward
 * (gpt-fast model.py) at prefill. */
int tao_attn_prefill_bf16(const uint16_t* q, const uint16_t* k_cache, const uint16_t* v_cache,
                          const int64_t* pos, uint16_t* out, int64_t B, int64_t H, int64_t Hkv,
                          int64_t D, int64_t S, int64_t T, float scale, void* stream);

/* y = bf16(bf16(silu(a)) * b) elementwise over n bf16 (n even). Replaces FeedForward's
 * F.silu(w1(x)) * w3(x) (model.py:485-486). b == NULL: a holds n interleaved (gate, up) pairs
 * (2n bf16, the output of an interleaved w13 linear) and y[i] = silu(a[2i]) * a[2i+1]. */
int tao_silu_mul_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, int64_t n,
                      void* stream);

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

/* Decode step, batch 1: one Llama block's feed-forward in ONE persistent launch (the LDS-DMA
 * engine, csrc/decode_engine.hip): out [dim] = h + w2(swiglu(w13(rmsnorm(h)))) with the roundings
 * of tao_int4wo_decode_bf16 (norm_weight, epilogue 1) followed by tao_int4wo_linear_bf16 with h as
 * its bias. w13 / sz13: the fused (w1_i, w3_i)-interleaved int4 linear [2 inter][dim/8] /
 * [2 inter][dim/32][2]; w2 / sz2: [dim][inter/8] / [dim][inter/32][2]; group size 32. The
 * summation order differs from the two launches (not bit-identical; within the oracle bars).
 * `ctl` / `payload`: a device workspace of tao_int4wo_ffn_engine_workspace_bytes(inter) bytes,
 * zeroed, then ctl[0] = 1 (an epoch the kernel advances per launch; one workspace per stream,
 * shared by every layer); ctl is its first 2 KiB (128-B aligned), payload the rest. One workgroup per CU, all co-resident: shapes and devices
 * tao_int4wo_ffn_engine_supported() accepts (1 / 0, not a status); a timed-out in-launch wait
 * sets tao_decode_status bit 2. Replaces FeedForward.forward's w1 / w3 / silu / w2 around the
 * reference's int4 linears at decode (torchao/_models/llama/model.py:481-492). */
int tao_int4wo_ffn_engine_supported(int64_t dim, int64_t inter, int64_t group_size);
int64_t tao_int4wo_ffn_engine_workspace_bytes(int64_t inter);
int tao_int4wo_ffn_engine_bf16(const uint16_t* h, const uint16_t* norm_weight, float eps,
                               const uint32_t* w13, const uint16_t* sz13, const uint32_t* w2,
                               const uint16_t* sz2, uint16_t* out, int64_t dim, int64_t inter,
                               int64_t group_size, unsigned* ctl, uint32_t* payload,
                               void* stream);

/* MoE decode: the A activated experts' int4 linears of one token in one launch. packed
 * [E][N][K/8] and scales_and_zeros [E][N][K/g][2] are a 3-D Int4WeightOnlyConfig weight (the
 * reference packs 3-D weights per expert, tensor_core_tiled_layout.py:283-294); expert_idx [A]
 * int64 on the device; x [x_rows][K] bf16 with x_rows 1 (every expert reads the same token) or A
 * (row a for expert a); y [A][N] bf16. Row a is bit-identical to tao_int4wo_linear_bf16 of expert
 * expert_idx[a] alone. Replaces the per-expert F.linear(x, w[expert_indices][i]) loop of
 * ConditionalFeedForwardAOQuantizable's one-token branch (_models/mixtral-moe/model.py:360-384).
 * An index outside [0, E) is clamped and reported by tao_decode_status (bits & 4). */
int tao_int4wo_grouped_gemv_bf16(const uint16_t* x, int64_t x_rows, const uint32_t* packed,
                                 const uint16_t* scales_and_zeros, const int64_t* expert_idx,
                                 int64_t A, int64_t E, int64_t N, int64_t K, int64_t group_size,
                                 uint16_t* y, void* stream);

/* Decode step, batch 1: RMSNorm -> int4 wqkv -> RoPE + KV-cache write (= tao_int4wo_decode_bf16
 * with norm_weight and epilogue 2, q into `q` [n_head * 128]) AND the decode attention of the
 * rotated q over cache keys 0..pos[0] (= tao_attn_decode_bf16) in ONE launch: out [n_head * 128]
 * bf16. Replaces, at decode, the Attention.forward sequence wqkv -> apply_rotary_emb ->
 * KVCache.update -> F.scaled_dot_product_attention (model.py:547-562). The attention workgroups
 * (n_head x `splits` key ranges, splits 1, 2 or 4) follow the GEMV's in the grid and start on
 * per-head tickets; a ticket wait that times out sets tao_decode_status bit 2. head_dim 128,
 * caches [1][n_kv_head][max_seq][128]; shapes tao_int4wo_qkv_attn_supported() accepts (returns
 * 1 / 0, not a status). */
int tao_int4wo_qkv_attn_supported(int64_t N, int64_t K, int64_t n_head, int64_t n_kv_head,
                                  int64_t head_dim);
int tao_int4wo_qkv_attn_bf16(const uint16_t* x, const uint32_t* packed,
                             const uint16_t* scales_and_zeros, int64_t N, int64_t K,
                             int64_t group_size, const uint16_t* norm_weight, float eps,
                             uint16_t* q, uint16_t* out, const float* freqs, const int64_t* pos,
                             uint16_t* k_cache, uint16_t* v_cache, int64_t n_head,
                             int64_t n_kv_head, int64_t head_dim, int64_t max_seq, float scale,
                             int64_t splits, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TORCHAO_MI355X_LLAMA_H_ */
