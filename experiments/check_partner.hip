// GPU check of tao::xor_partner (tao_reduce.h) against __shfl_xor: for off 32/16/2/1 the
// partner must be lane ^ off, for off 8/4 lane ^ 15 / lane ^ 7. Prints PASS/FAIL per offset.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../torchao-fork_amd/csrc/tao_reduce.h"

__global__ void k(int* out) {
  const int lane = threadIdx.x;
  const int v = lane * 7 + 1000;
  out[0 * 64 + lane] = tao::xor_partner<32>(v, lane);
  out[1 * 64 + lane] = tao::xor_partner<16>(v, lane);
  out[2 * 64 + lane] = tao::xor_partner<8>(v, lane);
  out[3 * 64 + lane] = tao::xor_partner<4>(v, lane);
  out[4 * 64 + lane] = tao::xor_partner<2>(v, lane);
  out[5 * 64 + lane] = tao::xor_partner<1>(v, lane);
}

int main() {
  int* d;
  int h[6 * 64];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  const int offs[6] = {32, 16, 8, 4, 2, 1}, mask[6] = {32, 16, 15, 7, 2, 1};
  int bad = 0;
  for (int i = 0; i < 6; ++i) {
    int e = 0;
    for (int l = 0; l < 64; ++l) e += h[i * 64 + l] != (l ^ mask[i]) * 7 + 1000;
    printf("off %d (lane ^ %d): %s\n", offs[i], mask[i], e ? "FAIL" : "PASS");
    bad += e;
  }
  (void)hipFree(d);
  return bad ? 1 : 0;
}
