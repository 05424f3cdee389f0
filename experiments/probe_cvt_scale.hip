// Probe (not the product path): does v_cvt_scalef32_pk_bf16_fp8 apply the full f32 scale (so a
// nibble byte b < 16 read as e4m3 = b / 512, scaled by 512 s, gives bf16(b s) in one instruction
// per two weights), or only the scale's exponent? Prints the mismatch count against bf16(b * s)
// rounded on the host (RNE), over b = 0..15 and 4096 scales.
//   hipcc --offload-arch=gfx950 -O2 experiments/probe_cvt_scale.hip -o experiments/build/probe_cvt
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__global__ void probe(const float* scales, uint32_t* out, int ns) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ns * 8) return;
  const int si = i / 8, bp = i % 8;  // byte pair (2 bp, 2 bp + 1)
  const uint32_t b0 = 2 * bp, b1 = 2 * bp + 1;
  const uint32_t src = b0 | (b1 << 8) | (b0 << 16) | (b1 << 24);
  const bf16x2_t lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(src, 512.f * scales[si], false);
  out[i] = __builtin_bit_cast(uint32_t, lo);
}

static uint16_t host_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

int main() {
  const int ns = 4096;
  float* hs = new float[ns];
  uint32_t seed = 12345;
  for (int i = 0; i < ns; ++i) {
    seed = seed * 1664525u + 1013904223u;
    const uint32_t bits = (0x3A00u + (seed >> 20) % 0x0600u) << 16;  // bf16 scales ~1e-3..1
    memcpy(&hs[i], &bits, 4);
  }
  float* ds;
  uint32_t* dout;
  hipMalloc(&ds, ns * 4);
  hipMalloc(&dout, ns * 8 * 4);
  hipMemcpy(ds, hs, ns * 4, hipMemcpyHostToDevice);
  probe<<<(ns * 8 + 255) / 256, 256>>>(ds, dout, ns);
  uint32_t* ho = new uint32_t[ns * 8];
  hipMemcpy(ho, dout, ns * 8 * 4, hipMemcpyDeviceToHost);
  int bad = 0, shown = 0;
  for (int i = 0; i < ns * 8; ++i) {
    const int si = i / 8, bp = i % 8;
    const uint16_t e0 = host_bf16((float)(2 * bp) * hs[si]), e1 = host_bf16((float)(2 * bp + 1) * hs[si]);
    const uint16_t g0 = ho[i] & 0xFFFF, g1 = ho[i] >> 16;
    if (g0 != e0 || g1 != e1) {
      ++bad;
      if (shown++ < 8)
        printf("scale %g b %d,%d: got %04x %04x expected %04x %04x\n", hs[si], 2 * bp, 2 * bp + 1,
               g0, g1, e0, e1);
    }
  }
  printf("{\"probe\": \"cvt_scalef32_pk_bf16_fp8\", \"cases\": %d, \"mismatches\": %d}\n", ns * 16,
         bad);
  return 0;
}
