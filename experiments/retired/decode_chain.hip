// Persistent int4 decode chain: a sequence of DEPENDENT M = 1 int4 weight-only linears (a Llama
// decoder's wqkv -> wo -> w1||w3 -> w2 per layer, then the output head) in ONE launch.
//
// Why: one kernel per linear pays, per linear, the dispatch ramp, the
// first weight round trip and the last wave's arithmetic/reduction tail, and between linears a
// kernel boundary (2.8 µs end-of-last-wave to start-of-next measured on this MI355X,
// experiments/anyorder_probe.hip). Here each workgroup issues the weight loads of its share of
// the NEXT linear before it waits for that linear's input, so the weight stream of linear p+1
// overlaps linear p's tail and the hand-off between them.
//
// Geometry: one 1024-thread workgroup per CU (grid = CU count, all resident: every wait below
// is on work of strictly earlier phases, and every wait is bounded). Phase p's N rows are split
// over the workgroups in blocks of multiples of 4 rows; inside a workgroup, tasks of 4 rows x
// a strided subset of the 2048-k slices go round-robin over the 16 waves (the int4 GEMV's lane
// math: 16-B nibble loads, magic-number bf16 pairs, v_dot2c; reduce-scatter across lanes;
// k-parts summed through LDS in a fixed order — deterministic).
//
// Hand-off (MI355X_MICROARCH.md "Hand-offs measured with sc1 loads in place of the acquire",
// first row; the same protocol as the split-K slabs, tao_common.h last_arriver): a phase's
// outputs are stored sc1 (4- / 8-B), every storing wave waits vmcnt(0), a workgroup barrier,
// then ONE lane adds 1 to the phase's counter shard (8 shards, one per blockIdx % 8 = one per
// XCD under round-robin placement; an agent-scope atomic add). A consumer's wave 0 polls every
// shard with sc1 loads (s_sleep between polls) until each reaches (epoch + 1) x its producer
// count, then a workgroup barrier, and every load of the handed-off vector is an sc1 buffer
// load. Counters are monotonic across launches: the epoch advances when the last workgroup of
// a launch exits, so a graph replays with no host work and no reset kernel.
// Every poll is bounded (wall clock); a timeout sets the abort word, which every other poll
// sees, so all workgroups drain and the host reads the failure (tao_chain_status).
#include <vector>

#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {
namespace {

constexpr int kChainThreads = 1024;
constexpr int kChainWaves = kChainThreads / 64;
constexpr int kRPW = 4;       // rows per task
constexpr int kShards = 8;    // counter shards per phase

struct DevPhase {
  const uint4* wq;          // [N][K/32] 16-B chunks
  const uint32_t* sz;       // [N][K/g] (scale, zero)
  const uint16_t* x;        // [K] input
  const uint16_t* norm_w;   // [K] or null
  const uint16_t* res;      // [N] (or [N/2] with SwiGLU) residual, or null
  uint16_t* y;              // output
  int N, K, gshift, x_phase, epi, x_ext;  // x_ext: x written before the launch
  float eps;
};

struct ChainCtl {
  unsigned epoch;       // launches completed
  unsigned exit_count;  // workgroups of the current launch that have exited
  unsigned abort;       // set by a timed-out poll
  unsigned err_phase;   // first phase that timed out (+1)
};

__device__ __forceinline__ unsigned ld_sc1_u32(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int row_split(int N, int b, int G) {
  return (int)(((long long)(N >> 2) * b / G) << 2);
}

__device__ __forceinline__ float silu_bf16(float a) { return round_bf16(a / (1.f + __expf(-a))); }

// The control wave polls until phase q is complete (every shard at (epoch + 1) x its
// producer count). Returns false if the wait timed out or the launch was aborted.
__device__ __forceinline__ bool poll_phase(const unsigned* cnt, ChainCtl* ctl, int q,
                                           unsigned epoch, int G, uint64_t timeout, int lane) {
  const int shard = lane & (kShards - 1);
  const unsigned per = (unsigned)(G / kShards + (shard < G % kShards ? 1 : 0));
  const unsigned target = (epoch + 1u) * per;
  const uint64_t t0 = wall_clock64();
  for (int it = 0;; ++it) {
    const unsigned v = ld_sc1_u32(cnt + q * kShards + shard);
    const bool done = lane >= kShards || v >= target;
    if (__ballot(!done) == 0) return true;
    if ((it & 15) == 15) {
      if (ld_sc1_u32(&ctl->abort) != 0u) return false;
      if (wall_clock64() - t0 > timeout) {
        if (lane == 0) {
          __hip_atomic_store(&ctl->err_phase, (unsigned)q + 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ctl->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Roles: waves 0..14 stream weights and compute (kCompute); wave 15 (the poller) issues no
// weight loads, so its in-order vmcnt waits see only its own polls: it alone waits for the input
// phase's counters while the compute waves' first weight loads are in flight. Then every wave
// gathers its share of the input (sc1 loads) and the RMSNorm runs across the workgroup; the
// norm weights and the residual rows (complete since an earlier phase) are loaded at phase
// start, off the critical path.
//   all:      [norm_w, residual -> regs/LDS] [compute waves: first weights in flight]
//   poller:   poll(p) | A0 |  all: gather x(p) (+ norm) -> LDS | A | compute: tasks -> partials
//   | B | all: epilogue + sc1 stores, vmcnt(0) | C | one lane signals
constexpr int kCompute = kChainWaves - 1;
constexpr int kXPT = 4;  // 16-B x pieces per thread (K <= 8 x 4 x 1024)

__global__ __launch_bounds__(kChainThreads, 1) void chain_kernel(const DevPhase* __restrict__ phases,
                                                                 int nph, unsigned* cnt,
                                                                 ChainCtl* ctl, uint64_t timeout,
                                                                 uint64_t* prof) {
  extern __shared__ uint4 smem[];  // x image [Kmax/8] uint4, then partials [tasks][4] floats
  __shared__ unsigned s_epoch, s_abort;
  __shared__ float s_ss[kChainWaves];
  __shared__ uint32_t s_res[kChainThreads * 2];  // residual rows of this workgroup (<= 4096)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool poller = wave == kCompute;
  const int G = gridDim.x, b = blockIdx.x;
  if (tid == 0) {
    s_epoch = ld_sc1_u32(&ctl->epoch);
    s_abort = 0u;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;

  auto stamp = [&](int p, int k) __attribute__((always_inline)) {
    if (prof != nullptr && tid == 0) prof[((size_t)p * G + b) * 4 + k] = wall_clock64();
  };

  for (int p = 0; p < nph; ++p) {
    stamp(p, 0);
    const DevPhase P = phases[p];
    const int N = P.N, K = P.K, gshift = P.gshift;
    const int nchunk = K >> 5, ngroups = K >> (5 + gshift);
    const int S = (nchunk + 63) >> 6;
    const int r0 = row_split(N, b, G), r1 = row_split(N, b + 1, G);
    const int R = r1 - r0;
    const int nrg = (R + kRPW - 1) / kRPW;
    int KP = nrg >= kCompute ? 1 : kCompute / (nrg > 0 ? nrg : 1);
    KP = KP < S ? KP : S;
    const int ntask = nrg * KP;
    const int nx = K >> 3;
    uint4* xs = smem;
    uint4* gs = smem + (K >> 3);  // norm weight image (same element order as the x pieces)
    float* part = reinterpret_cast<float*>(smem + 2 * (K >> 3));

    // ---- phase start, poller wave: static operands (norm weights, residual rows) -> LDS -----
    if (poller) {
      if (P.norm_w != nullptr) {
        const uint4* gw = reinterpret_cast<const uint4*>(P.norm_w);
        for (int i = lane; i < nx; i += 64) gs[i] = gw[i];
      }
      const int rwords = (P.epi == 1 ? R : 2 * R) >> 2;  // residual dwords of this workgroup
      if (P.res != nullptr) {
        const Rsrc rr = make_rsrc(P.res, (uint32_t)(P.epi == 1 ? N : 2 * N));
        const uint32_t base = (uint32_t)(P.epi == 1 ? r0 : 2 * r0);
        for (int i = lane; i < rwords; i += 64) s_res[i] = bload4<kSC1>(rr, base + i * 4u, 0);
      }
    }

    uint4 wv[2][kRPW];
    uint32_t szv[2][kRPW];
    int ccs[2];
    bool cvs[2];
    auto load_slice = [&](int u, int rowb, int s) __attribute__((always_inline)) {
      const int c = s * 64 + lane;
      cvs[u] = s < S && c < nchunk;
      ccs[u] = c < nchunk ? c : nchunk - 1;
#pragma unroll
      for (int r = 0; r < kRPW; ++r) {
        const int n = rowb + r;
        const int nn = n < r1 ? n : (r1 > 0 ? r1 - 1 : 0);
        wv[u][r] = ld_nt_u4(P.wq + (size_t)nn * nchunk + ccs[u]);
        szv[u][r] = ld_nt(P.sz + (size_t)nn * ngroups + (ccs[u] >> gshift));
      }
    };
    if (!poller && wave < ntask) {  // the first task's first slice pair in flight
      const int rg = wave / KP, kp = wave % KP;
      load_slice(0, r0 + rg * kRPW, kp);
      load_slice(1, r0 + rg * kRPW, kp + KP);
    }

    // ---- wait for the input (the poller), then gather it across the workgroup ----------------
    if (poller && P.x_phase >= 0) {
      if (!poll_phase(cnt, ctl, P.x_phase, epoch, G, timeout, lane) && lane == 0) s_abort = 1u;
    }
    __syncthreads();  // A0
    if (s_abort) break;
    stamp(p, 1);
    {
      // raw x -> LDS image (sc1 loads, all issued before the first use), sum of squares
      const Rsrc xr = make_rsrc(P.x, (uint32_t)K * 2u);
      uint4 xv[kXPT];
#pragma unroll
      for (int u = 0; u < kXPT; ++u) {
        const int i = tid + u * kChainThreads;
        xv[u] = i < nx ? bload16<kSC1>(xr, (uint32_t)i * 16u, 0) : make_uint4(0, 0, 0, 0);
      }
      float ss = 0.f;
#pragma unroll
      for (int u = 0; u < kXPT; ++u) {
        const int i = tid + u * kChainThreads;
        const uint32_t d[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float a = bf16lo_to_f32(d[j]), c = bf16hi_to_f32(d[j]);
          ss = fmaf(a, a, fmaf(c, c, ss));
        }
        if (i < nx) {
          const int c = i >> 2;
          xs[c * 4 + (((i & 3) + (c >> 2)) & 3)] = xv[u];
        }
      }
      if (P.norm_w != nullptr) {  // in place over the image: bf16(bf16(x r) w)
        ss = wave_sum(ss);
        if (lane == 0) s_ss[wave] = ss;
        __syncthreads();
        float t = 0.f;
        for (int w = 0; w < kChainWaves; ++w) t += s_ss[w];
        const float rn = rsqrtf(t / (float)K + P.eps);
        for (int i = tid; i < nx; i += kChainThreads) {
          const int c = i >> 2;
          uint4& slot = xs[c * 4 + (((i & 3) + (c >> 2)) & 3)];
          const uint4 xq = slot, gv = gs[i];
          const uint32_t xd[4] = {xq.x, xq.y, xq.z, xq.w};
          const uint32_t gd[4] = {gv.x, gv.y, gv.z, gv.w};
          uint32_t o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float lo = round_bf16(bf16lo_to_f32(xd[j]) * rn) * bf16lo_to_f32(gd[j]);
            const float hi = round_bf16(bf16hi_to_f32(xd[j]) * rn) * bf16hi_to_f32(gd[j]);
            o[j] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
          }
          slot = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    __syncthreads();  // A: x image ready

    if (!poller) {
      auto do_slice = [&](int u, float (&acc)[kRPW], int rowb) __attribute__((always_inline)) {
        const int cc = ccs[u];
        float sc[kRPW], zp[kRPW];
#pragma unroll
        for (int r = 0; r < kRPW; ++r) {
          const bool ok = cvs[u] && rowb + r < r1;
          const uint32_t v = ok ? szv[u][r] : 0u;
          sc[r] = bf16lo_to_f32(v);
          zp[r] = bf16hi_to_f32(v);
        }
        uint32_t xd[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4 t4 = xs[cc * 4 + ((j + (cc >> 2)) & 3)];
          xd[j][0] = t4.x;
          xd[j][1] = t4.y;
          xd[j][2] = t4.z;
          xd[j][3] = t4.w;
        }
        float sx = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) sx = dot2_bf16(xd[j][i], 0x3F803F80u, sx);
        const float sx136 = 136.f * sx;
#pragma unroll
        for (int r = 0; r < kRPW; ++r) {
          const uint32_t wd[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
          float d = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) d = dot2_bf16(xd[j][i], nib_pair_bf16(wd[j], i), d);
          acc[r] = fmaf(sc[r], d - sx136, fmaf(zp[r], sx, acc[r]));
        }
      };
      bool first = true;
      for (int t = wave; t < ntask; t += kCompute) {
        const int rg = t / KP, kp = t % KP;
        const int rowb = r0 + rg * kRPW;
        float acc[kRPW] = {0.f, 0.f, 0.f, 0.f};
        for (int s2 = kp; s2 < S; s2 += 2 * KP) {
          if (!first) {
            load_slice(0, rowb, s2);
            load_slice(1, rowb, s2 + KP);
          }
          first = false;
          do_slice(0, acc, rowb);
          if (s2 + KP < S) do_slice(1, acc, rowb);  // wave-uniform
        }
        wave_reduce_scatter<kRPW>(acc, lane);
        if ((lane & 15) == 0) part[t * kRPW + (lane >> 4)] = acc[0];
      }
    }
    __syncthreads();  // B: partials complete
    stamp(p, 2);

    // ---- epilogue: 4 rows per thread, k-parts summed in order, sc1 stores ----------------------
    const int nq = R >> 2;
    const Rsrc yr = make_rsrc(P.y, (uint32_t)(P.epi == 1 ? N : 2 * N));
    for (int i = tid; i < nq; i += kChainThreads) {
      float tot[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 4 * i + q;
        const int rg = row / kRPW, ri = row % kRPW;
        float sacc = 0.f;
        for (int kp = 0; kp < KP; ++kp) sacc += part[(rg * KP + kp) * kRPW + ri];
        tot[q] = sacc;
      }
      const int n0 = r0 + 4 * i;
      if (P.epi == 1) {  // SwiGLU over (w1, w3) row pairs -> two outputs, one 4-B store
        const float a0 = round_bf16(tot[0]), b0 = round_bf16(tot[1]);
        const float a1 = round_bf16(tot[2]), b1 = round_bf16(tot[3]);
        uint32_t o = (uint32_t)f32_to_bf16(silu_bf16(a0) * b0) |
                     ((uint32_t)f32_to_bf16(silu_bf16(a1) * b1) << 16);
        if (P.res != nullptr) {
          const uint32_t rv = s_res[i];
          o = (uint32_t)f32_to_bf16(bf16lo_to_f32(o) + bf16lo_to_f32(rv)) |
              ((uint32_t)f32_to_bf16(bf16hi_to_f32(o) + bf16hi_to_f32(rv)) << 16);
        }
        __builtin_amdgcn_raw_buffer_store_b32(o, yr, (uint32_t)n0, 0, kSC1);
      } else {
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = f32_to_bf16(tot[q]);
        if (P.res != nullptr) {
          const uint32_t rv0 = s_res[2 * i], rv1 = s_res[2 * i + 1];
          const uint32_t rv[4] = {rv0 & 0xFFFFu, rv0 >> 16, rv1 & 0xFFFFu, rv1 >> 16};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            o[q] = f32_to_bf16(bf16_to_f32(o[q]) + bf16_to_f32(rv[q]));
        }
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 d = {o[0] | (o[1] << 16), o[2] | (o[3] << 16)};
        __builtin_amdgcn_raw_buffer_store_b64(d, yr, (uint32_t)n0 * 2u, 0, kSC1);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // C: every storing wave has drained its sc1 stores
    if (tid == 0)
      __hip_atomic_fetch_add(cnt + p * kShards + (b & (kShards - 1)), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    stamp(p, 3);
  }

  // ---- launch end: the last workgroup out advances the epoch ---------------------------------
  __syncthreads();
  if (tid == 0) {
    const unsigned old =
        __hip_atomic_fetch_add(&ctl->exit_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)G - 1u) {
      __hip_atomic_store(&ctl->exit_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&ctl->epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct Chain {
  DevPhase* phases = nullptr;
  unsigned* cnt = nullptr;
  ChainCtl* ctl = nullptr;
  int nph = 0, grid = 0, device = 0;
  size_t lds = 0;
  uint64_t timeout_ticks = 0;
  uint64_t* prof = nullptr;  // tao_chain_profile buffer (caller-owned), or null
};

int gshift_of_g(int64_t g) {
  switch (g) {
    case 32: return 0;
    case 64: return 1;
    case 128: return 2;
    case 256: return 3;
    default: return -1;
  }
}

}  // namespace
}  // namespace tao

using namespace tao;

extern "C" {

int tao_chain_create(const TaoChainPhase* phases, int n, void** handle) {
  TAO_CHECK_ARG(handle != nullptr && phases != nullptr && n > 0 && n <= 4096,
                "chain: need 1..4096 phases and a handle");
  *handle = nullptr;
  std::vector<DevPhase> dev(n);
  int64_t kmax = 0, lds_part = 0;
  for (int p = 0; p < n; ++p) {
    const TaoChainPhase& s = phases[p];
    const int gs = gshift_of_g(s.group_size);
    TAO_CHECK_ARG(gs >= 0, "chain phase %d: group_size must be 32/64/128/256", p);
    TAO_CHECK_ARG(s.N > 0 && s.N % 4 == 0 && s.N < (1 << 30),
                  "chain phase %d: N (%lld) must be a positive multiple of 4", p, (long long)s.N);
    TAO_CHECK_ARG(s.K > 0 && s.K % s.group_size == 0 && s.K <= 8 * 4 * kChainThreads,
                  "chain phase %d: K (%lld) must be a multiple of the group and <= %d", p,
                  (long long)s.K, 8 * 4 * kChainThreads);
    TAO_CHECK_ARG(s.residual == nullptr || (s.N + 255) / 256 * 4 * 2 <= 4 * 2 * kChainThreads,
                  "chain phase %d: too many rows per workgroup for the residual stage", p);
    TAO_CHECK_ARG(s.epilogue == 0 || s.epilogue == 1, "chain phase %d: epilogue 0 or 1", p);
    TAO_CHECK_ARG(s.x_phase >= -1 && s.x_phase < p,
                  "chain phase %d: x_phase must name an earlier phase or be -1", p);
    TAO_CHECK_ARG(s.packed && s.sz && s.x && s.y, "chain phase %d: null operand", p);
    TAO_CHECK_ALIGN(s.x, 16, "chain x");
    TAO_CHECK_ALIGN(s.packed, 16, "chain packed");
    TAO_CHECK_ALIGN(s.y, 8, "chain y");
    if (s.norm_w) TAO_CHECK_ALIGN(s.norm_w, 16, "chain norm_w");
    if (s.residual) TAO_CHECK_ALIGN(s.residual, 8, "chain residual");
    DevPhase& d = dev[p];
    d.wq = reinterpret_cast<const uint4*>(s.packed);
    d.sz = reinterpret_cast<const uint32_t*>(s.sz);
    d.x = s.x;
    d.norm_w = s.norm_w;
    d.res = s.residual;
    d.y = s.y;
    d.N = (int)s.N;
    d.K = (int)s.K;
    d.gshift = gs;
    d.x_phase = s.x_phase;
    d.epi = s.epilogue;
    d.x_ext = s.x_phase < 0;
    d.eps = s.eps;
    kmax = s.K > kmax ? s.K : kmax;
  }
  Chain* c = new Chain();
  if (hipGetDevice(&c->device) != hipSuccess) {
    delete c;
    return set_error(TAO_ERR_HIP, "chain: hipGetDevice failed");
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) {
    delete c;
    return set_error(TAO_ERR_HIP, "chain: hipGetDeviceProperties failed");
  }
  c->grid = prop.multiProcessorCount;
  // partials: per phase at most ceil(rows/4) x KP tasks (<= max(16, rows/4)) x 4 floats
  for (int p = 0; p < n; ++p) {
    const int64_t rows = (phases[p].N / 4 / c->grid + 1) * 4;
    const int64_t tasks = ((rows + kRPW - 1) / kRPW) * kCompute;
    lds_part = tasks * kRPW * 4 > lds_part ? tasks * kRPW * 4 : lds_part;
  }
  c->lds = (size_t)(kmax * 4 + lds_part);
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, chain_kernel, kChainThreads, c->lds) !=
          hipSuccess ||
      occ < 1) {
    delete c;
    return set_error(TAO_ERR_UNSUPPORTED, "chain: %zu B of LDS per workgroup does not fit a CU",
                     c->lds);
  }
  if (c->lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(chain_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->lds) != hipSuccess) {
    delete c;
    return set_error(TAO_ERR_HIP, "chain: cannot raise the dynamic LDS limit to %zu B", c->lds);
  }
  int rate_khz = 0;
  (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->device);
  c->timeout_ticks = (uint64_t)(rate_khz > 0 ? rate_khz : 100000) * 200ull;  // 200 ms per wait
  c->nph = n;
  if (hipMalloc(&c->phases, sizeof(DevPhase) * n) != hipSuccess ||
      hipMalloc(&c->cnt, sizeof(unsigned) * kShards * n) != hipSuccess ||
      hipMalloc(&c->ctl, sizeof(ChainCtl)) != hipSuccess ||
      hipMemcpy(c->phases, dev.data(), sizeof(DevPhase) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->cnt, 0, sizeof(unsigned) * kShards * n) != hipSuccess ||
      hipMemset(c->ctl, 0, sizeof(ChainCtl)) != hipSuccess) {
    (void)hipFree(c->phases);
    (void)hipFree(c->cnt);
    (void)hipFree(c->ctl);
    delete c;
    return set_error(TAO_ERR_HIP, "chain: device allocation failed");
  }
  *handle = c;
  return TAO_OK;
}

int tao_chain_run(void* handle, void* stream) {
  TAO_CHECK_ARG(handle != nullptr, "chain: null handle");
  Chain* c = static_cast<Chain*>(handle);
  launch(chain_kernel, dim3(c->grid), dim3(kChainThreads), c->lds, as_stream(stream), c->phases,
         c->nph, c->cnt, c->ctl, c->timeout_ticks, c->prof);
  return check_launch("chain_kernel");
}

int tao_chain_status(void* handle, int* aborted_phase, unsigned* launches) {
  TAO_CHECK_ARG(handle != nullptr && aborted_phase != nullptr, "chain: null argument");
  Chain* c = static_cast<Chain*>(handle);
  ChainCtl h;
  if (hipMemcpy(&h, c->ctl, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
    return set_error(TAO_ERR_HIP, "chain: status read failed");
  *aborted_phase = h.abort ? (int)h.err_phase : 0;
  if (launches) *launches = h.epoch;
  return TAO_OK;
}

int tao_chain_reset(void* handle) {
  TAO_CHECK_ARG(handle != nullptr, "chain: null handle");
  Chain* c = static_cast<Chain*>(handle);
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemset(c->cnt, 0, sizeof(unsigned) * kShards * c->nph) != hipSuccess ||
      hipMemset(c->ctl, 0, sizeof(ChainCtl)) != hipSuccess)
    return set_error(TAO_ERR_HIP, "chain: reset failed");
  return TAO_OK;
}

int tao_chain_profile(void* handle, uint64_t* stamps, int* grid) {
  TAO_CHECK_ARG(handle != nullptr && grid != nullptr, "chain: null argument");
  Chain* c = static_cast<Chain*>(handle);
  c->prof = stamps;
  *grid = c->grid;
  return TAO_OK;
}

int tao_chain_destroy(void* handle) {
  if (handle == nullptr) return TAO_OK;
  Chain* c = static_cast<Chain*>(handle);
  (void)hipFree(c->phases);
  (void)hipFree(c->cnt);
  (void)hipFree(c->ctl);
  delete c;
  return TAO_OK;
}

}  // extern "C"
