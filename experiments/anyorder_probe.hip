// Does hipExtAnyOrderLaunch (AQL barrier bit clear) let a kernel start before its stream
// predecessor has finished on gfx950, eagerly and inside a captured hipGraph, and does the
// dispatcher hand out the successor's workgroups only after all of the predecessor's (so a
// successor that waits for the predecessor cannot starve it)? Every wait is bounded.
//
//   hipcc -O2 --offload-arch=gfx950 experiments/anyorder_probe.hip -o experiments/build/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// A: each workgroup spins `ticks` of the constant clock, then counts itself done.
__global__ void kernel_a(unsigned long long* t_start, unsigned long long* t_end, unsigned* done,
                         unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) t_start[blockIdx.x] = t0;
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (threadIdx.x == 0) {
    t_end[blockIdx.x] = wall_clock64();
    __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// B: records when it started, then waits (bounded) until all of A's workgroups are done.
__global__ void kernel_b(unsigned long long* t_start, unsigned long long* t_pass, unsigned* done,
                         unsigned need, unsigned long long timeout, unsigned* timed_out) {
  const unsigned long long t0 = wall_clock64();
  __shared__ unsigned ok;
  if (threadIdx.x == 0) {
    t_start[blockIdx.x] = t0;
    unsigned v = 0;
    while ((v = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < need &&
           wall_clock64() - t0 < timeout)
      __builtin_amdgcn_s_sleep(2);
    ok = v >= need;
    t_pass[blockIdx.x] = wall_clock64();
    if (!ok) __hip_atomic_fetch_add(timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}

struct Buf {
  unsigned long long *as, *ae, *bs, *bp;
  unsigned *done, *to;
};

static void run(const char* tag, int ga, int gb, int threads, double a_us, unsigned flags,
                bool graph, double tick_mhz) {
  Buf b;
  CK(hipMalloc(&b.as, ga * 8));
  CK(hipMalloc(&b.ae, ga * 8));
  CK(hipMalloc(&b.bs, gb * 8));
  CK(hipMalloc(&b.bp, gb * 8));
  CK(hipMalloc(&b.done, 4));
  CK(hipMalloc(&b.to, 4));
  CK(hipMemset(b.done, 0, 4));
  CK(hipMemset(b.to, 0, 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const unsigned long long ticks = (unsigned long long)(a_us * tick_mhz);
  const unsigned long long timeout = (unsigned long long)(200000.0 * tick_mhz);  // 200 ms
  auto enqueue = [&]() {
    hipLaunchKernelGGL(kernel_a, dim3(ga), dim3(threads), 0, s, b.as, b.ae, b.done, ticks);
    hipExtLaunchKernelGGL(kernel_b, dim3(gb), dim3(threads), 0, s, nullptr, nullptr, flags, b.bs,
                          b.bp, b.done, (unsigned)ga, timeout, b.to);
  };
  if (graph) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    enqueue();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
  } else {
    enqueue();
  }
  CK(hipStreamSynchronize(s));
  unsigned long long *as = (unsigned long long*)malloc(ga * 8), *ae = (unsigned long long*)malloc(ga * 8);
  unsigned long long *bs = (unsigned long long*)malloc(gb * 8), *bp = (unsigned long long*)malloc(gb * 8);
  unsigned to = 0;
  CK(hipMemcpy(as, b.as, ga * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ae, b.ae, ga * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(bs, b.bs, gb * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(bp, b.bp, gb * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&to, b.to, 4, hipMemcpyDeviceToHost));
  unsigned long long a0 = ~0ull, a_end = 0, a_last_start = 0, b0 = ~0ull, b_last = 0;
  for (int i = 0; i < ga; ++i) {
    a0 = as[i] < a0 ? as[i] : a0;
    a_end = ae[i] > a_end ? ae[i] : a_end;
    a_last_start = as[i] > a_last_start ? as[i] : a_last_start;
  }
  for (int i = 0; i < gb; ++i) {
    b0 = bs[i] < b0 ? bs[i] : b0;
    b_last = bp[i] > b_last ? bp[i] : b_last;
  }
  auto us = [&](long long t) { return (double)t / tick_mhz; };
  printf("{\"case\": \"%s\", \"graph\": %d, \"flags\": %u, \"ga\": %d, \"gb\": %d, \"a_us\": %.1f, "
         "\"a_span_us\": %.2f, \"b_first_start_minus_a_end_us\": %.2f, "
         "\"b_first_start_minus_a_last_start_us\": %.2f, \"b_pass_minus_a_end_us\": %.2f, "
         "\"b_timeouts\": %u}\n",
         tag, (int)graph, flags, ga, gb, a_us, us(a_end - a0), us((long long)(b0 - a_end)),
         us((long long)(b0 - a_last_start)), us((long long)(b_last - a_end)), to);
  fflush(stdout);
  free(as); free(ae); free(bs); free(bp);
  CK(hipFree(b.as)); CK(hipFree(b.ae)); CK(hipFree(b.bs)); CK(hipFree(b.bp));
  CK(hipFree(b.done)); CK(hipFree(b.to));
  CK(hipStreamDestroy(s));
}

int main() {
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const double mhz = rate_khz / 1000.0;
  printf("{\"wall_clock_mhz\": %.1f}\n", mhz);
  // A fits on the chip (256 WGs), B small: does B start before A ends?
  run("fit_default", 256, 256, 256, 30.0, 0, false, mhz);
  run("fit_anyorder", 256, 256, 256, 30.0, hipExtAnyOrderLaunch, false, mhz);
  run("fit_anyorder_graph", 256, 256, 256, 30.0, hipExtAnyOrderLaunch, true, mhz);
  // A oversubscribes the chip (8192 WGs of 256 threads, several dispatch rounds): with the
  // barrier bit clear, are B's waiting workgroups dispatched only after all of A's?
  run("oversub_anyorder", 8192, 2048, 256, 5.0, hipExtAnyOrderLaunch, false, mhz);
  run("oversub_anyorder_graph", 8192, 2048, 256, 5.0, hipExtAnyOrderLaunch, true, mhz);
  return 0;
}
