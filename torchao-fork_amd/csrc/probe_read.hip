// Measurement kernel used by bench.py (not on the product path): a pure streaming read of a buffer
// with 16-B non-temporal loads, one load per thread, 512-thread workgroups (each wave-instruction
// 1 KiB contiguous). It is the best of the read variants DESIGN §5.0 measured
// (experiments/probe_graph_read.py): replaying one such launch per linear from a HIP graph gives
// the floor any one-kernel-per-linear GEMV step can reach on this chip, measured in the same run
// as the GEMV step (bench.py roofline.pure_read_ms_per_step).
#include "tao_common.h"

namespace tao {
namespace {

__global__ __launch_bounds__(512) void read_probe_kernel(const uint4* __restrict__ p,
                                                         uint32_t* __restrict__ sink) {
  const size_t t = (size_t)blockIdx.x * 512 + threadIdx.x;
  const uint4 v = ld_nt_u4(p + t);
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x9E3779B9u) sink[t & 1023] = acc;  // keeps the load live; never taken in practice
}

// Streaming copy for the bench's ceiling calibration (MI355X_MICROARCH.md "HBM": a float4 copy
// measured at 6.29 TB/s read + write). mode 0: each thread moves 4 x 16 B per grid-stride round
// with all four loads in flight before the stores, default cache policy; mode 1: the same with
// non-temporal loads and stores; mode 2: one 16-B element per thread, no loop (grid covers the
// buffer: bytes / 16 / 256 workgroups), non-temporal.
template <int MODE>
__global__ __launch_bounds__(256) void copy_probe_kernel(const uint4* __restrict__ src,
                                                         uint4* __restrict__ dst, size_t n16) {
  if constexpr (MODE == 2) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) st_nt_u4(dst + i, ld_nt_u4(src + i));
    return;
  } else {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = i + 256 * j < n16 ? (MODE == 1 ? ld_nt_u4(src + i + 256 * j) : src[i + 256 * j])
                                 : uint4{};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i + 256 * j < n16) {
          if constexpr (MODE == 1) st_nt_u4(dst + i + 256 * j, v[j]);
          else dst[i + 256 * j] = v[j];
        }
    }
  }
}

// LDS-DMA intake probe of the single-fetch prefill GEMM's tile family (bench.py prefill_mfma
// intake ceiling): each workgroup of a launch shape takes in exactly the bytes
// its tile does per k step -- the 128 x rows of its K slice, the tile's BN weight rows, their
// (scale, zero) words -- as 1-KiB (16 B / lane) and 256-B (4 B / lane) LDS-DMA pieces into an NS-stage
// ring, with the kernel's counted vmcnt wait and one barrier per step, issued by 4 loader waves
// beside 8 waves that only join the barriers (LDW) or by all 8 waves, and computes nothing. Its
// time is the intake-bound floor of that tile on this chip (gemm_sf.hip's per-step DMA).
// R = pieces per issuing wave per stage (compile time, for the counted wait). MODE (attribution
// of the intake, experiments only): 0 the tile's pieces; 1 its weight and (scale, zero) pieces
// only; 2 its x pieces only; 3 all pieces, x read from a private copy per workgroup (x holds
// grid x 128 rows: no two workgroups request the same x lines); 4 the tile's pieces with each
// workgroup starting its k steps at a different step (rot = (block / 8) mod steps: the workgroups
// of one XCD that share a K slice first request different x lines); 5 x pieces only, rotated.
template <int NS, int R, int LDW, int MODE>
__global__ __launch_bounds__((8 + LDW) * 64) void sf_intake_probe_kernel(
    const uint8_t* __restrict__ x, uint32_t x_bytes, uint32_t x_row, int kx,
    const uint8_t* __restrict__ w, uint32_t w_bytes, uint32_t w_row, int kw,
    const uint8_t* __restrict__ z, uint32_t z_bytes, uint32_t z_row, int kz, int zgs,
    int px, int pw, int pz, int ntn, int S, int a_steps, int nsteps, uint32_t* __restrict__ sink) {
  constexpr int DW = LDW > 0 ? LDW : 8;
  constexpr int STAGE_MAX = 160 * 1024 / NS;
  __shared__ uint4 lds[160 * 1024 / 16];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool issuer = LDW == 0 || wave >= 8;
  const int dwv = LDW > 0 ? wave - 8 : wave;
  const int bid = blockIdx.x;
  const int nb = bid % ntn, sl = (bid / ntn) % S;
  const int s0 = sl * a_steps, J = sl == S - 1 ? nsteps - s0 : a_steps;
  const int stage = px * 1024 + pw * 1024 + pz * 256;
  const Rsrc xr = make_rsrc(x, x_bytes), wr = make_rsrc(w, w_bytes), zr = make_rsrc(z, z_bytes);
  // piece r of this wave: index i = r DW + dwv over [x pieces | w pieces | z pieces]
  uint32_t dv[R];
  int dd[R], dk[R];
  const int xrow0 = MODE == 3 ? bid * 128 : 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int i = r * DW + dwv;
    if (MODE == 1) i += px;                    // no x pieces
    if ((MODE == 2 || MODE == 5) && i >= px) i = px + pw + pz;  // x pieces only
    if (i < px) {  // 1024 / kx rows per piece, kx / 16 lanes per row
      const int g = kx / 16, row = xrow0 + i * (1024 / kx) + lane / g;
      dv[r] = (uint32_t)row * x_row + 16u * (uint32_t)(lane % g);
      dd[r] = i * 1024;
      dk[r] = 0;
    } else if (i < px + pw) {
      const int j = i - px, g = kw / 16, row = nb * (pw * 1024 / kw) + j * (1024 / kw) + lane / g;
      dv[r] = (uint32_t)row * w_row + 16u * (uint32_t)(lane % g);
      dd[r] = px * 1024 + j * 1024;
      dk[r] = 1;
    } else if (i < px + pw + pz) {  // 4 B per lane: 256 / kz rows per piece
      const int j = i - px - pw, g = kz / 4, row = nb * (pz * 256 / kz) + j * (256 / kz) + lane / g;
      dv[r] = (uint32_t)row * z_row + 4u * (uint32_t)(lane % g);
      dd[r] = px * 1024 + pw * 1024 + j * 256;
      dk[r] = 2;
    } else {
      dk[r] = 3;  // no piece (the issuing waves' share is uneven)
    }
  }
  const int rot = MODE >= 4 ? (bid >> 3) % J : 0;
  auto issue = [&](int stp, int buf) __attribute__((always_inline)) {
    const int st = MODE >= 4 ? s0 + (stp - s0 + rot) % J : stp;
    uint8_t* base = reinterpret_cast<uint8_t*>(lds) + buf * (stage < STAGE_MAX ? stage : STAGE_MAX);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (dk[r] == 0) dma_lds_ring<16>(xr, dv[r], (uint32_t)st * (uint32_t)kx, base + dd[r]);
      else if (dk[r] == 1) dma_lds_ring<16, kNT>(wr, dv[r], (uint32_t)st * (uint32_t)kw, base + dd[r]);
      else if (dk[r] == 2)
        dma_lds_ring<4, kNT>(zr, dv[r], (uint32_t)(st * (kx / 2) / zgs) * 4u, base + dd[r]);
      else  // keep the per-wave count of vector-memory ops at R per stage
        dma_lds_ring<4>(xr, 0u, 0u, base);
    }
  };
  if (issuer) {
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (p < J) issue(s0 + p, p);
  }
  for (int j = 0; j < J; ++j) {
    if (issuer) {
      if (J - 1 - j >= NS - 2) wait_vmcnt<(NS - 2) * R>();
      else wait_vmcnt<0>();
    }
    barrier_lgkm();
    if (issuer && j + NS - 1 < J) issue(s0 + j + NS - 1, (j + NS - 1) % NS);
  }
  wait_vmcnt<0>();
  barrier_lgkm();
  if (threadIdx.x == 0) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(lds)[bid & 1023];
    if (v == 0x9E3779B9u) sink[bid & 1023] = v;  // keeps the ring live; never taken in practice
  }
}

}  // namespace

void sf_launch_shape(int path, int M, int N, int K, int* bn, int* splits, int* stages,
                     int* a_steps, int* loaders, int* kstep, int* wm1);

}  // namespace tao

// The intake probe for the single-fetch launch shape the GEMM takes at (path, M <= 128, N, K):
// path 0 = int4 (x bf16 [M][K], w packed [N][K/2] bytes, z (scale, zero) [N][K/g] dwords), 2 =
// int8 dyn (x int8 [M][K], w int8 [N][K], z unused). Writes the launch shape it streamed to
// shape_out[0..6] (bn, splits, stages, a_steps, loaders, kstep, bytes per workgroup per step).
extern "C" int tao_sf_intake_probe(int path, int mode, const void* x, const void* w,
                                   const void* z, int64_t M, int64_t N, int64_t K,
                                   int64_t group_size, int* shape_out, void* sink, void* stream) {
  TAO_CHECK_ARG(path == 0 || path == 2, "intake probe: path must be 0 (int4) or 2 (int8 dyn)");
  TAO_CHECK_ARG(mode >= 0 && mode <= 5, "intake probe: mode (%d) must be 0..5", mode);
  TAO_CHECK_ARG(x != nullptr && w != nullptr && sink != nullptr && shape_out != nullptr &&
                    (path == 2 || z != nullptr),
                "intake probe: null pointer");
  TAO_CHECK_ARG(M > 64 && M <= 128 && N > 0 && K > 0 && N * K < (1LL << 32),
                "intake probe: one 128-row tile (64 < M <= 128), N x K < 2^32");
  TAO_CHECK_ARG(path == 2 || (group_size >= 32 && group_size <= 256 && K % group_size == 0),
                "intake probe: bad group size %lld", (long long)group_size);
  int bn, S, ns, a, ld, ks, wm1;
  tao::sf_launch_shape(path, (int)M, (int)N, (int)K, &bn, &S, &ns, &a, &ld, &ks, &wm1);
  const int kx = path == 0 ? 256 : ks, kw = path == 0 ? 64 : ks, kz = path == 0 ? 16 : 0;
  TAO_CHECK_ARG(K % ks == 0 && N % bn == 0, "intake probe: N (%lld) / K (%lld) off the tile grid",
                (long long)N, (long long)K);
  const int px = 128 * kx / 1024, pw = bn * kw / 1024, pz = bn * kz / 256;
  const int T = px + pw + pz, DW = ld ? ld : 8, R = (T + DW - 1) / DW;
  if (ns < 2) ns = 2;
  if (ns > 4) ns = 4;
  shape_out[0] = bn;
  shape_out[1] = S;
  shape_out[2] = ns;
  shape_out[3] = a;
  shape_out[4] = ld;
  shape_out[5] = ks;
  shape_out[6] = px * 1024 + pw * 1024 + pz * 256;
  TAO_CHECK_ARG((int64_t)ns * shape_out[6] <= 160 * 1024, "intake probe: %d stages of %d B exceed LDS",
                ns, shape_out[6]);
  const int ntn = (int)(N / bn), nsteps = (int)(K / ks);
  const uint8_t* xb = static_cast<const uint8_t*>(x);
  const uint8_t* wb = static_cast<const uint8_t*>(w);
  const uint8_t* zb = static_cast<const uint8_t*>(z != nullptr ? z : w);
  const uint32_t xrow = (uint32_t)(K * (path == 0 ? 2 : 1)), wrow = (uint32_t)(path == 0 ? K / 2 : K);
  const uint32_t zrow = path == 0 ? (uint32_t)(K / group_size * 4) : 4u;
  const int64_t xrows = mode == 3 ? 128LL * (N / bn) * S : M;  // mode 3: a private x per workgroup
  TAO_CHECK_ARG(xrows * xrow < (1LL << 32), "intake probe: x too large");
  const uint32_t xbytes = (uint32_t)(xrows * xrow), wbytes = (uint32_t)(N * wrow);
  const uint32_t zbytes = path == 0 ? (uint32_t)(N * zrow) : 4u;
  const int zgs = path == 0 ? (int)group_size : 32;
  const dim3 grid((unsigned)(ntn * S));
  hipStream_t st = tao::as_stream(stream);
  uint32_t* sk = static_cast<uint32_t*>(sink);
#define TAO_IP(NS_, R_, LDW_, MODE_)                                                               \
  tao::launch(tao::sf_intake_probe_kernel<NS_, R_, LDW_, MODE_>, grid, dim3((8 + LDW_) * 64), 0,  \
              st, xb, xbytes, xrow, kx, wb, wbytes, wrow, kw, zb, zbytes, zrow, kz, zgs, px, pw,   \
              pz, ntn, S, a, nsteps, sk)
  if (mode == 0 && ld == 8 && R == 5 && ns == 4) TAO_IP(4, 5, 8, 0);
  else if (mode == 2 && ld == 8 && R == 5 && ns == 4) TAO_IP(4, 4, 8, 2);
  else if (mode == 0 && ld && R == 10 && ns == 4) TAO_IP(4, 10, 4, 0);
  else if (mode == 0 && ld && R == 10 && ns == 3) TAO_IP(3, 10, 4, 0);
  else if (mode == 0 && !ld && R == 5 && ns == 4) TAO_IP(4, 5, 0, 0);
  else if (mode == 2 && !ld && R == 5 && ns == 4) TAO_IP(4, 4, 0, 2);  // 32 x pieces, 8 waves
  else if (mode == 0 && !ld && R == 5 && ns == 3) TAO_IP(3, 5, 0, 0);
  else if (mode == 0 && !ld && R == 5 && ns == 2) TAO_IP(2, 5, 0, 0);
  else if (mode == 0 && !ld && R == 6 && ns == 3) TAO_IP(3, 6, 0, 0);
  else if (mode == 0 && !ld && R == 6 && ns == 2) TAO_IP(2, 6, 0, 0);
  else if (mode == 1 && ld && R == 10 && ns == 4) TAO_IP(4, 2, 4, 1);  // 8 w / z pieces
  else if (mode == 2 && ld && R == 10 && ns == 4) TAO_IP(4, 8, 4, 2);  // 32 x pieces
  else if (mode == 3 && ld && R == 10 && ns == 4) TAO_IP(4, 10, 4, 3);
  else if (mode == 4 && ld && R == 10 && ns == 4) TAO_IP(4, 10, 4, 4);
  else if (mode == 5 && ld && R == 10 && ns == 4) TAO_IP(4, 8, 4, 5);
  else
    return tao::set_error(TAO_ERR_UNSUPPORTED,
                          "intake probe: no instance for %d pieces per wave, %d stages, loaders %d",
                          R, ns, ld);
#undef TAO_IP
  return tao::check_launch("sf_intake_probe_kernel");
}

extern "C" int tao_hbm_copy_probe(const void* src, void* dst, int64_t bytes, int grid, int mode,
                                  void* stream) {
  TAO_CHECK_ARG(src != nullptr && dst != nullptr, "copy probe: null pointer");
  TAO_CHECK_ARG(bytes > 0 && bytes % 16 == 0, "copy probe: bytes (%lld) must be a positive "
                "multiple of 16", (long long)bytes);
  TAO_CHECK_ARG(mode >= 0 && mode <= 2, "copy probe: mode (%d) must be 0, 1 or 2", mode);
  TAO_CHECK_ARG(mode == 2 || (grid > 0 && grid <= (1 << 20)), "copy probe: grid (%d) out of range",
                grid);
  TAO_CHECK_ARG(mode != 2 || bytes / 4096 < (1LL << 31), "copy probe: bytes too large for mode 2");
  TAO_CHECK_ALIGN(src, 16, "src");
  TAO_CHECK_ALIGN(dst, 16, "dst");
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const size_t n16 = (size_t)(bytes / 16);
  hipStream_t st = tao::as_stream(stream);
  if (mode == 2)
    tao::launch(tao::copy_probe_kernel<2>, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st,
                s, d, n16);
  else if (mode == 1)
    tao::launch(tao::copy_probe_kernel<1>, dim3((unsigned)grid), dim3(256), 0, st, s, d, n16);
  else
    tao::launch(tao::copy_probe_kernel<0>, dim3((unsigned)grid), dim3(256), 0, st, s, d, n16);
  return tao::check_launch("copy_probe_kernel");
}

extern "C" int tao_hbm_read_probe(const void* buf, int64_t bytes, void* sink, void* stream) {
  TAO_CHECK_ARG(buf != nullptr && sink != nullptr, "read probe: null pointer");
  TAO_CHECK_ARG(bytes > 0 && bytes % 8192 == 0 && bytes / 8192 < (1LL << 31),
                "read probe: bytes (%lld) must be a positive multiple of 8192",
                (long long)bytes);
  TAO_CHECK_ALIGN(buf, 16, "buf");
  tao::launch(tao::read_probe_kernel, dim3((unsigned)(bytes / 8192)), dim3(512), 0,
              tao::as_stream(stream), reinterpret_cast<const uint4*>(buf),
              reinterpret_cast<uint32_t*>(sink));
  return tao::check_launch("read_probe_kernel");
}
