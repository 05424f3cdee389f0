/*
 * torchao_mi355x_tune.h — internal measurement and tuning entry points of libtorchao_mi355x.so.
 *
 * Not part of the drop-in boundary (include/torchao_mi355x.h): nothing here replaces a reference
 * call. These are the launch-shape overrides (tao_tune_*, thread-local), the routing label, the
 * per-dispatch profiler, the HBM read probe and diagnostics used by bench.py, tests/ and
 * experiments/. Same conventions and error codes as the public header.
 */
#ifndef TORCHAO_MI355X_TUNE_H_
#define TORCHAO_MI355X_TUNE_H_

#include "torchao_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Name of the last kernel this thread launched through the library (its routing decision, for
 * measurement labels); "" before the first launch. */
const char* tao_last_kernel(void);
/* Per-kernel timing for benchmarks (not used on the inference path). Between begin and end,
 * the calling thread's next `capacity` kernel launches carry a start/stop hipEvent pair written
 * by the kernel's own dispatch packet (hipExtLaunchKernelGGL) — the interval rocprofv3 reports
 * as the kernel duration. end() synchronises on the events and writes one duration (ms) per
 * recorded launch, in launch order; *count receives how many. Do not open a session while
 * capturing a hipGraph. */
int tao_profile_begin(int capacity);
int tao_profile_end(float* durations_ms, int capacity, int* count);

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
/* int4 GEMV launches: reserve at least `bytes` of LDS per workgroup (0 = built-in: what the kernel
 * uses), which caps the workgroups resident per CU at 160 KiB / bytes and with them the weight
 * bytes each CU has in flight. Calling thread only; for measurement. */
int tao_tune_int4_lds(int bytes);

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
/* Single-fetch GEMMs: dedicated LDS-DMA loader waves beside the compute waves (0 = built-in,
 * 1 = off, 2 = on, 3 = 8 loader waves on the 16x16 int4 kernel, else as 2). 32x32x16 int4 kernel:
 * one per SIMD, bn 64 / 128, one wave per column group; 16x16 kernel: 4 (or 8) beside its 8
 * compute waves, 64-column tiles. Thread-local; for measurement. */
int tao_tune_gemm_sf_loaders(int mode);
/* Single-fetch GEMM, fixed-reducer seam: place each K slice's workgroups on their own XCDs
 * (slice z on XCDs [8z/S, 8(z+1)/S)), so each XCD's L2 takes in 1/S of x. 0 = built-in,
 * 1 = off, 2 = on. */
int tao_tune_gemm_sf_xmap(int mode);
/* Prefill attention: waves per 16-query block, each taking every nw-th 32-key block, partial
 * softmax states merged through LDS (0 = built-in: 2 for 513-1024 query blocks, else 4;
 * 1, 2 or 4). Thread-local; for measurement. */
int tao_tune_attn_prefill_nw(int nw);
/* Test hook for the single-fetch split-K seam (fixed reducer): with `on` = 1, slice-0 publishers
 * add their ticket only after a reducer has given up waiting (0.25 s) or 2 s passed, so tests can
 * check that a timed-out launch is reported (tao_gemm_sf_status, tao_decode_status bits & 2), writes
 * nothing for its tiles, and leaves the tickets at 0 for the next launch. Thread-local. */
int tao_debug_sf_late_publisher(int on);
/* Reducer poll timeouts of the single-fetch GEMM since the last call (*bits != 0: some split
 * launch's outputs are invalid; never expected, see gemm_sf.hip). Synchronous. */
int tao_gemm_sf_status(unsigned* bits);

/* Measurement hook (experiments/engine_stamps.py): the following tao_int4wo_ffn_engine_bf16
 * launches of this process write per-workgroup phase stamps (s_memrealtime, 100 MHz; 64 u64 per
 * workgroup, layout in csrc/decode_engine.hip) into `buf` (>= 256 x 64 x 8 bytes of device
 * memory); NULL turns it off. */
int tao_debug_ffn_engine_stamps(void* buf);
/* A/B knobs of the decode FFN engine: consumer waves per workgroup (3 or 7, built-in 7), the
 * nibble decode (0 shift + and + or, 1 byte permutes, built-in 1), the loader's slots in flight
 * (1..3, built-in 3) and the w1||w3 block assignment (0 static rows per workgroup, built-in;
 * 1 per-XCD queues fed by a dispatcher wave, which runs 7 consumers, decode 1, 2 slots). */
int tao_tune_ffn_engine(int consumers, int dq, int ahead, int dyn);
/* Measurement kernel (bench.py, not the product path): a pure streaming read of `bytes` (a
 * positive multiple of 8192) from `buf` (16-B aligned) with 16-B non-temporal loads; `sink` is
 * >= 4 KiB of device memory the kernel may write (it never does in practice). Graph-capturable. */
int tao_hbm_read_probe(const void* buf, int64_t bytes, void* sink, void* stream);
/* Measurement kernel (bench.py ceiling calibration): dst <- src, `bytes` (multiple of 16), 16-B
 * loads and stores. mode 0: `grid` 256-thread workgroups striding over the buffer (4 x 16 B in
 * flight per thread), default cache policy; 1: the same, non-temporal loads and stores; 2: one
 * 16-B element per thread, one pass (`grid` ignored), non-temporal. Graph-capturable. */
int tao_hbm_copy_probe(const void* src, void* dst, int64_t bytes, int grid, int mode,
                       void* stream);
/* Measurement kernel (bench.py prefill_mfma intake ceiling, not the product path): the LDS-DMA
 * intake of the single-fetch prefill GEMM's launch shape at (path 0 int4 / 2 int8 dyn, 64 < M <=
 * 128, N, K): every workgroup streams exactly its tile's x, weight and (scale, zero) bytes per k
 * step through the kernel's LDS ring, counted waits and barriers, and computes nothing. x / w / z
 * as the GEMM's operands (z: int4 (scale, zero) words; unused for int8). shape_out[0..6] <- bn,
 * K slices, stages, k steps per slice, loader waves, k step, bytes per workgroup per step. `sink`
 * >= 4 KiB of device memory (never written in practice). mode 0 is that intake; 1..3 attribute it
 * (int4 route with loader waves only): 1 weight + (scale, zero) pieces only, 2 x pieces only,
 * 3 every piece with x read from a private [grid][128][K] copy per workgroup, 4 every piece with
 * the k steps of each workgroup rotated to start at step (block / 8) mod steps, 5 x pieces only,
 * rotated. Graph-capturable. */
int tao_sf_intake_probe(int path, int mode, const void* x, const void* w, const void* z,
                        int64_t M, int64_t N, int64_t K, int64_t group_size, int* shape_out,
                        void* sink, void* stream);
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

/* Tuning hook: M == 1 launch shape of the int8 decode GEMVs (int8 weight-only and int8 x int8:
 * rows per wave 2/4/8, waves along K, row groups per workgroup; 0 = built-in heuristic).
 * Calling thread only; for sweeps (experiments/sweep_int8.py). */
int tao_tune_int8_gemv(int rows_per_wave, int waves_k, int row_groups);
/* Per-token int8 quantisation kernel (A/B only): 0 = one wave per token, the token held in
 * registers (default, K <= 8192); 1 = one 256-thread workgroup per token. Bit-identical. */
int tao_tune_int8_quant(int block);

/* Calling thread's choice of the decode-attention kernel: 0 = single-pass workgroup per query head
 * (f32 math, whole-line K loads) for T <= 1024, else the two-launch split (default); 1 = two-launch
 * split. */
int tao_tune_attn(int mode);

#ifdef __cplusplus
}
#endif

#endif /* TORCHAO_MI355X_TUNE_H_ */
