// probe_stream3: probe_stream.hip with the run length of a row per wave instruction as a parameter
// (XRL for x, WRL for the weights: 1024 / RL rows per instruction, RL / 16 lanes per row), to
// separate the per-step barrier from the access pattern (probe_stream2 measured 1 KiB row runs
// ~1.4-1.9x faster than 64-B runs).
// Streaming skeleton of an unsplit (S = 1) prefill GEMM tile, no math: what the per-CU intake of
// the x rows (L2-resident, shared by every workgroup of an M tile) plus the weight rows (streamed
// from HBM: 20 copies rotated past the 256 MiB Infinity Cache) costs when it is the ONLY work.
//
// grid (N / BN, M / BM), NW waves; per k step every workgroup LDS-DMAs BM rows x XS bytes of x and
// BN rows x WS bytes of weights (full 128-B lines, 8 rows x 128 B per wave instruction) into stage
// j % R of an R-deep ring; one barrier per step (wait own DMAs of step j -> barrier -> issue step
// j + R - 1 into the stage step j - 1 used -> read one dword of step j). Prints µs per launch
// (events over 50 launches) and GB/s per CU of algorithmic bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -o experiments/build/probe_stream experiments/probe_stream.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void glds16(Rsrc r, uint32_t voff, uint32_t soff, void* dst, bool nt) {
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_ptr_t)dst;
  uint32_t keep;
  if (nt)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// pieces of 8 rows x 128 B: x has BM * XS / 1024 per step, W BN * WS / 1024 (WS >= 128), or for
// WS = 64: BN / 16 pieces of 16 rows x 64 B
template <int BM, int BN, int XS, int WS, int XRL, int WRL, int R, int NW>
__global__ __launch_bounds__(NW * 64) void stream_kernel(const uint8_t* __restrict__ x,
                                                         const uint8_t* __restrict__ w, int K,
                                                         int N, uint32_t* sink) {
  constexpr int PX = BM * XS / 1024, PW = BN * WS / 1024, P = PX + PW;
  static_assert(P % NW == 0, "pieces per wave");
  constexpr int PPW = P / NW;
  constexpr int STAGE = P * 1024;
  static_assert(R * STAGE <= 160 * 1024, "LDS");
  __shared__ uint4 lds[R * STAGE / 16];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int nsteps = K / (XS);  // x bytes per row = K (int8 x) -- XS bytes of x per step
  const uint32_t xrow = (uint32_t)K, wrow = (uint32_t)(K / XS) * WS;
  const Rsrc xr = make_rsrc(x, 0x7fffffff), wr = make_rsrc(w, 0x7fffffff);
  uint32_t voff[PPW];
  bool isw[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wave * PPW + i;
    const bool w_ = p >= PX;
    const int q = w_ ? p - PX : p;
    const int RL = w_ ? WRL : XRL, SB = w_ ? WS : XS;  // run length, step bytes per row
    const int cols = SB / RL;                          // pieces across a row's step
    const int rpp = 1024 / RL;                         // rows per piece
    const int row = (q / cols) * rpp + lane / (RL / 16);
    const uint32_t cb = (uint32_t)((q % cols) * RL + 16 * (lane % (RL / 16)));
    voff[i] = w_ ? (uint32_t)(n0 + row) * wrow + cb : (uint32_t)(m0 + row) * xrow + cb;
    isw[i] = w_;
  }
  auto issue = [&](int j) __attribute__((always_inline)) {
    const int st = j < nsteps ? j : nsteps - 1;
    uint8_t* stage = reinterpret_cast<uint8_t*>(lds) + (j % R) * STAGE;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wave * PPW + i;
      glds16(isw[i] ? wr : xr, voff[i], (uint32_t)st * (isw[i] ? WS : XS), stage + p * 1024, isw[i]);
    }
  };
  for (int j = 0; j < R - 1; ++j) issue(j);
  uint32_t acc = 0;
  for (int j = 0; j < nsteps; ++j) {
    wait_vm<(R - 2) * PPW>();
    raw_barrier();
    issue(j + R - 1);
    acc ^= reinterpret_cast<const uint32_t*>(lds)[((j % R) * STAGE) / 4 + threadIdx.x];
  }
  wait_vm<0>();
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int BM, int BN, int XS, int WS, int XRL, int WRL, int R, int NW>
static void run(const char* tag, const uint8_t* x, const uint8_t* wbig, size_t wcopy, int copies,
                int M, int N, int K, uint32_t* sink) {
  const dim3 grid(N / BN, M / BM);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i)
    stream_kernel<BM, BN, XS, WS, XRL, WRL, R, NW><<<grid, NW * 64>>>(x, wbig + (i % copies) * wcopy, K, N, sink);
  hipEventRecord(a);
  const int iters = 50;
  for (int i = 0; i < iters; ++i)
    stream_kernel<BM, BN, XS, WS, XRL, WRL, R, NW><<<grid, NW * 64>>>(x, wbig + (i % copies) * wcopy, K, N, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double wg_bytes = (double)BM * K + (double)BN * (K / XS) * WS;
  const int wgs = grid.x * grid.y;
  printf("{\"probe\": \"%s\", \"BM\": %d, \"BN\": %d, \"XS\": %d, \"WS\": %d, \"XRL\": %d, \"WRL\": %d, \"R\": %d, \"waves\": %d, "
         "\"workgroups\": %d, \"KB_per_wg\": %.0f, \"us\": %.2f, \"GBps_per_wg\": %.1f, "
         "\"weight_TBps\": %.2f}\n",
         tag, BM, BN, XS, WS, XRL, WRL, R, NW, wgs, wg_bytes / 1024, us, wg_bytes / us / 1e3,
         (double)N * (K / XS) * WS / us / 1e6);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const int M = 128, N = 4096, K = 4096;
  uint8_t *x = nullptr, *w = nullptr;
  uint32_t* sink = nullptr;
  const size_t wcopy = (size_t)N * K;  // 16 MiB (int8); int4 uses the first quarter
  const int copies = 20;
  if (hipMalloc(&x, (size_t)M * K * 2) != hipSuccess || hipMalloc(&w, wcopy * copies) != hipSuccess ||
      hipMalloc(&sink, 1 << 16) != hipSuccess)
    return 1;
  hipMemset(x, 1, (size_t)M * K * 2);
  hipMemset(w, 1, wcopy * copies);
  // int8 dynamic (config 3): x int8 rows of K bytes, W int8 rows of K bytes
  run<32, 64, 256, 256, 128, 128, 4, 4>("i8", x, w, wcopy, copies, M, N, K, sink);
  run<32, 64, 256, 256, 256, 256, 6, 4>("i8", x, w, wcopy, copies, M, N, K, sink);
  run<32, 64, 512, 512, 512, 512, 3, 4>("i8", x, w, wcopy, copies, M, N, K, sink);
  run<32, 64, 512, 512, 512, 512, 3, 8>("i8", x, w, wcopy, copies, M, N, K, sink);
  // int4 weight-only: bf16 x ("K" = x row bytes = 8 KiB), nibble rows of 2 KiB
  run<32, 64, 256, 64, 128, 64, 4, 4>("i4", x, w, wcopy, copies, M, N, 2 * K, sink);
  run<16, 128, 512, 128, 512, 128, 6, 4>("i4", x, w, wcopy, copies, M, N, 2 * K, sink);
  run<16, 128, 1024, 256, 1024, 256, 3, 4>("i4", x, w, wcopy, copies, M, N, 2 * K, sink);
  run<16, 128, 1024, 256, 1024, 128, 3, 4>("i4", x, w, wcopy, copies, M, N, 2 * K, sink);
  run<32, 64, 512, 128, 512, 128, 4, 4>("i4", x, w, wcopy, copies, M, N, 2 * K, sink);
  run<16, 128, 1024, 256, 1024, 256, 3, 8>("i4", x, w, wcopy, copies, M, N, 2 * K, sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
