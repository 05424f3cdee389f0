// Streaming skeleton of an x-resident prefill tile, no math (companion of probe_stream.hip, whose
// per-step LDS ring + barrier structure measured ~43 GB/s per CU): the workgroup LDS-DMAs its whole
// x tile (BM rows x XB bytes, L2-resident) once, then every wave streams ITS OWN weight rows into
// registers with no barrier, DEPTH chunks of (rows x 1 KiB) in flight, in one of two patterns:
//   PAT 0: a wave instruction reads 16 rows x 64 B (lane l: row l % 16, bytes 16 (l / 16)) -- the
//          MFMA 16x16x64-i8 / 16x16x32-bf16 B-fragment order, no regrouping needed;
//   PAT 1: a wave instruction reads 1 row x 1 KiB (the GEMV pattern; needs an LDS regroup).
// Weights rotate over 20 copies (past the 256 MiB Infinity Cache). µs per launch over 50 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -o experiments/build/probe_stream2 experiments/probe_stream2.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ Rsrc make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void glds16(Rsrc r, uint32_t voff, uint32_t soff, void* dst) {
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_ptr_t)dst;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(lds_addr), "v"(voff), "s"(r), "s"(soff) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// RW = weight rows per wave (16 or 32), chunk = RW rows x 1 KiB = RW wave instructions
template <int BM, int BN, int XB, int WB, int PAT, int DEPTH, int NT>
__global__ __launch_bounds__(256) void xres_kernel(const uint8_t* __restrict__ x,
                                                   const uint8_t* __restrict__ w, uint32_t* sink) {
  constexpr int RW = BN / 4;
  constexpr int XP = BM * XB / 1024;  // x DMA pieces (8 rows x 128 B)
  static_assert(XP % 4 == 0 && BM * XB <= 160 * 1024, "x tile");
  constexpr int NCH = WB / 1024;      // chunks per row
  constexpr int IPC = RW;             // instructions per chunk (PAT 0: RW/16 groups x 16 64-B
                                      // columns; PAT 1: one per row)
  __shared__ uint4 xs[BM * XB / 16];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * BN + wave * RW, m0 = blockIdx.y * BM;
  const Rsrc xr = make_rsrc(x, 0x7fffffff), wr = make_rsrc(w, 0x7fffffff);
  // x tile once
#pragma unroll
  for (int i = 0; i < XP / 4; ++i) {
    const int p = wave * (XP / 4) + i;
    const int h = p / (BM / 8), rg = p % (BM / 8);
    const int row = 8 * rg + (lane >> 3);
    glds16(xr, (uint32_t)(m0 + row) * XB + 128u * h + 16u * (lane & 7), 0,
           reinterpret_cast<uint8_t*>(xs) + p * 1024);
  }
  // per-instruction lane offsets within a chunk
  auto voff = [&](int i) __attribute__((always_inline)) -> uint32_t {
    if (PAT == 0) {
      const int grp = i / 16, col = i % 16;  // 16-row group, 64-B column of the 1 KiB chunk
      return (uint32_t)(n0 + 16 * grp + (lane & 15)) * WB + 64u * col + 16u * (lane >> 4);
    }
    return (uint32_t)(n0 + i) * WB + 16u * lane;
  };
  u32x4 buf[DEPTH][IPC];
  auto issue = [&](int c, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < IPC; ++i)
      buf[slot][i] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, voff(i), c * 1024, NT ? 2 : 0));
  };
  // chunks still in flight after chunk c's issue window: min(NCH - 1, c + DEPTH - 1) - c
  auto wait_chunks = [&](int pending) __attribute__((always_inline)) {
    switch (pending) {
      case 0: wait_vm<0>(); break;
      case 1: wait_vm<IPC>(); break;
      case 2: wait_vm<2 * IPC>(); break;
      default: wait_vm<3 * IPC>(); break;
    }
  };
#pragma unroll
  for (int c = 0; c < DEPTH - 1 && c < NCH; ++c) issue(c, c % DEPTH);
  uint32_t acc = 0;
  {
    const int pend = (DEPTH - 1 < NCH ? DEPTH - 1 : NCH);  // W chunks issued after x
    wait_chunks(pend);                                     // x landed (issued first)
  }
  __syncthreads();
  acc ^= reinterpret_cast<const uint32_t*>(xs)[threadIdx.x];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c + DEPTH - 1 < NCH) issue(c + DEPTH - 1, (c + DEPTH - 1) % DEPTH);
    const int last = (c + DEPTH - 1 < NCH ? c + DEPTH - 1 : NCH - 1);
    wait_chunks(last - c);
#pragma unroll
    for (int i = 0; i < IPC; ++i) acc ^= buf[c % DEPTH][i][0] ^ buf[c % DEPTH][i][3];
  }
  wait_vm<0>();
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int BM, int BN, int XB, int WB, int PAT, int DEPTH, int NT>
static void run(const char* tag, const uint8_t* x, const uint8_t* wbig, size_t wcopy, int copies,
                int M, int N, uint32_t* sink) {
  const dim3 grid(N / BN, M / BM);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i)
    xres_kernel<BM, BN, XB, WB, PAT, DEPTH, NT><<<grid, 256>>>(x, wbig + (i % copies) * wcopy, sink);
  hipEventRecord(a);
  const int iters = 50;
  for (int i = 0; i < iters; ++i)
    xres_kernel<BM, BN, XB, WB, PAT, DEPTH, NT><<<grid, 256>>>(x, wbig + (i % copies) * wcopy, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / iters;
  const double wg_bytes = (double)BM * XB + (double)BN * WB;
  printf("{\"probe\": \"%s\", \"BM\": %d, \"BN\": %d, \"x_row_B\": %d, \"w_row_B\": %d, \"pat\": %d, "
         "\"depth\": %d, \"nt\": %d, \"workgroups\": %d, \"KB_per_wg\": %.0f, \"us\": %.2f, "
         "\"GBps_per_wg\": %.1f, \"weight_TBps\": %.2f}\n",
         tag, BM, BN, XB, WB, PAT, DEPTH, NT, (int)(grid.x * grid.y), wg_bytes / 1024, us,
         wg_bytes / us / 1e3, (double)N * WB / us / 1e6);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  const int M = 128, N = 4096;
  uint8_t *x = nullptr, *w = nullptr;
  uint32_t* sink = nullptr;
  const size_t wcopy = (size_t)N * 4096;
  const int copies = 20;
  if (hipMalloc(&x, (size_t)M * 8192) != hipSuccess || hipMalloc(&w, wcopy * copies) != hipSuccess ||
      hipMalloc(&sink, 1 << 16) != hipSuccess)
    return 1;
  hipMemset(x, 1, (size_t)M * 8192);
  hipMemset(w, 1, wcopy * copies);
  // int8 dynamic (config 3): x 32 rows x 4 KiB (128 KiB of LDS), W 64 rows x 4 KiB per workgroup
  run<32, 64, 4096, 4096, 0, 1, 0>("i8", x, w, wcopy, copies, M, N, sink);
  run<32, 64, 4096, 4096, 0, 2, 0>("i8", x, w, wcopy, copies, M, N, sink);
  run<32, 64, 4096, 4096, 0, 2, 1>("i8", x, w, wcopy, copies, M, N, sink);
  run<32, 64, 4096, 4096, 0, 4, 0>("i8", x, w, wcopy, copies, M, N, sink);
  run<32, 64, 4096, 4096, 1, 2, 0>("i8", x, w, wcopy, copies, M, N, sink);
  run<32, 64, 4096, 4096, 1, 4, 0>("i8", x, w, wcopy, copies, M, N, sink);
  // int4 weight-only: x 16 rows x 8 KiB bf16 (128 KiB), W 128 rows x 2 KiB nibbles
  run<16, 128, 8192, 2048, 0, 1, 0>("i4", x, w, wcopy, copies, M, N, sink);
  run<16, 128, 8192, 2048, 0, 2, 0>("i4", x, w, wcopy, copies, M, N, sink);
  run<16, 128, 8192, 2048, 1, 2, 0>("i4", x, w, wcopy, copies, M, N, sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
