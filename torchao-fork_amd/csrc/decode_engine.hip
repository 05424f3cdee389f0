// Persistent LDS-DMA decode engine (MI355X_MICROARCH.md rows ldsdma-fill,
// prefetch-credit, gather-pass, engine-vs-launches): one Llama decode block's feed-forward at
// batch 1 — RMSNorm -> int4 w1||w3 -> SwiGLU -> int4 w2 -> + residual — in ONE launch, with the
// real data dependency (w2 reads every SwiGLU output) kept inside it.
//
// Replaces, at decode, FeedForward.forward's w1 / w3 / silu / w2 sequence around the reference's
// int4 linears (torchao/_models/llama/model.py:481-492, tensor_core_tiled_layout.py:104 for each
// linear), which the launch path runs as two launches (tao_int4wo_decode_bf16 with the RMSNorm
// prologue and SwiGLU epilogue, then the w2 GEMV with the residual on its bias).
//
// Geometry: kNWG = 256 workgroups, one per CU (123 KiB LDS each: all resident), C + 1 waves:
//   wave 0 (loader)    streams this CU's weight rows of BOTH linears, in order, into a ring of
//                      kRing LDS slots with non-temporal LDS-DMA (buffer_load ... lds), kAhead
//                      slots in flight; it never waits for an activation, so w2's rows stream in
//                      while w1||w3's outputs are still being gathered (prefetch credit);
//   waves 1..C         consume slots round-robin (slot g -> consumer g % C; C = 7 consumer waves,
//                      two per SIMD, or 3 with tao_tune_ffn_engine):
//     phase 1  x = RMSNorm(h) held in registers (each consumer wave normalises the whole h,
//              so no cross-wave exchange); a slot is 8 rows (4 (w1_i, w3_i) pairs) x 4096 k;
//              per row the GEMV's lane math (v_dot2c_f32_bf16 on magic-number nibble pairs),
//              a reduce-scatter, then SwiGLU -> 4 outputs stored sc1 (write-through);
//     edge     every storing wave drains (vmcnt(0)) and counts itself in LDS; the last one adds
//              the workgroup's arrival to one of 8 shard counters (agent-scope atomic). The
//              counters only grow (32 arrivals per launch each), so a launch with epoch E waits
//              for 32 E on all 8 (MI355X_MICROARCH.md hand-offs with sc1 loads, first row);
//     phase 2  a slot is 16 rows x one 2048-k unit of w2; after the counters match, a consumer
//              loads the SwiGLU outputs of ITS units with 16-B sc1 loads straight into registers,
//              accumulates its units' partial dot products, and the consumers' partials meet in
//              LDS (fixed order) -> + h -> out.
// In-CU hand-offs are LDS words: FULL[slot] (loader, after a counted vmcnt wait) and FREE[slot]
// (consumer, after its reads of the slot). The epoch lives on the device (ctl[0]); the last
// workgroup out advances it, so HIP-graph replays need no reset.
// Every wait is bounded (SeamWait): a timeout sets tao_decode_status bit 2 and the grid drains.
#include <type_traits>

#include "tao_common.h"
#include "tao_reduce.h"

namespace tao {

TAO_DECODE_ERROR_WORD(engine_decode_status)

namespace {

constexpr int kNWG = 256;            // one workgroup per CU
constexpr int kSlotB = 20 * 1024;    // slot: 16 KiB of nibbles + 4 KiB of (scale, zero) words
constexpr int kScaleOff = 16 * 1024;
constexpr int kRing = 7;             // 140 KiB of ring: w2's 7 slots all fit behind w1||w3's
constexpr int kPieces = 20;          // DMA wave-instructions per slot (1 KiB each)
constexpr int kShards = 8;           // phase-1 arrival counters (workgroup wg -> shard wg % 8)
constexpr int kShard0 = 64;          // word offset of shard 0 in ctl
constexpr int kHeads = 8;            // DYN: w1||w3 block queues (workgroup wg -> queue wg % 8)
constexpr int kHead0 = 320;          // word offset of queue 0's head in ctl
constexpr int kCtlBytes = 4096;      // ctl words; the SwiGLU payload follows
constexpr int kTq = 8;               // DYN: LDS ticket ring
constexpr int kTqAhead = 2;          // DYN: tickets the dispatcher holds beyond the loader's

struct FfnArgs {
  const uint16_t* h;       // [4096] residual stream (the FFN's input and residual)
  const uint16_t* norm_w;  // [4096] ffn_norm weight
  float eps;
  const uint32_t* w13;     // [2I][512] nibbles (row-stream layout), rows (w1_i, w3_i) interleaved
  const uint32_t* sz13;    // [2I][128] (scale, zero) bf16 pairs, group size 32
  const uint32_t* w2;      // [4096][I/8]
  const uint32_t* sz2;     // [4096][I/32]
  uint16_t* out;           // [4096] h + w2(swiglu(w13(rmsnorm(h))))
  unsigned* ctl;           // [0] epoch (>= 1), [32] workgroups done, [kShard0 + 32 s] shard s
                           // arrival counters (each on its own 128-B line)
  uint32_t* pay;           // [I/2] the SwiGLU output, bf16 pairs
  int inter;               // I (multiple of 2048)
  unsigned long long* stamps;  // measurement hook (tao_debug_ffn_engine_stamps), else null
  uint32_t nib_mask, nib_magic;  // 0x000F000F, 0x43004300 (see NibConst)
};

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }
// per workgroup 64 x u64 (lane 0 of the stamping wave): [0] loader entry, [1] last phase-1 slot
// issued, [2] every slot issued, [3] last FULL, [4] loader time waiting on FREE; consumer c at
// 8 + 6 c: [0] x normalised, [1] phase 1 done, [2] gather done, [3] phase 2 done, [4] end,
// [5] time waiting on FULL
__device__ __forceinline__ void stamp(const FfnArgs& a, int slot, unsigned long long v) {
  if (a.stamps != nullptr && slot < 64 && (threadIdx.x & 63) == 0) a.stamps[blockIdx.x * 64 + slot] = v;
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ unsigned lds_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// one 2048-k unit of one row for this lane: 16 B of nibbles (32 k), its (scale, zero) word and
// the lane's 32 x values (16 bf16 pairs) with their sum sx: s (D - 136 sx) + z sx, D = sum x (128 + q)
// The magic-number pair of nibble pair i of a word, ((w >> 4 i) & 0x000F000F) | 0x43004300, is one
// v_and_or_b32 (mask in an SGPR, magic in a VGPR: a VOP3 takes no literal here) after the shift:
// 7 VALU per 8 weights before the 4 dot2s instead of 11 (the engine's consumers are VALU-bound;
// same bits as nib_pair_bf16, so the same results)
struct NibConst {
  uint32_t mask, magic;
  // the constants come in as kernel arguments (0x000F000F, 0x43004300), opaque to the compiler,
  // so it cannot fold them into literals (it still splits the and-or into two VOP2s)
  __device__ __forceinline__ NibConst(uint32_t m, uint32_t g) : mask(m), magic(g) {}
  __device__ __forceinline__ uint32_t pair(uint32_t t) const { return (t & mask) | magic; }
};

// DQ 0: the four magic-number pairs of a word by shift + and + or (11 VALU per 8 weights before
// the dot2s). DQ 1: byte permutes: lo = w & 0x0F0F0F0F holds q0, q4, q1, q5 in its bytes and
// hi = (w >> 4) & 0x0F0F0F0F holds q2, q6, q3, q7; v_perm_b32 puts two of them under 0x43 bytes,
// [q_a, 0x43, q_b, 0x43] = the bf16 pair (128 + q_a, 128 + q_b): 7 VALU per 8 weights, the same
// bits as DQ 0.
template <int DQ>
__device__ __forceinline__ void nib_pairs(const NibConst& nc, uint32_t w, uint32_t (&p)[4]) {
  if constexpr (DQ == 0) {
    p[0] = nc.pair(w);
    p[1] = nc.pair(w >> 4);
    p[2] = nc.pair(w >> 8);
    p[3] = nc.pair(w >> 12);
  } else {
    const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
    p[0] = __builtin_amdgcn_perm(0x43434343u, lo, 0x04020400u);
    p[1] = __builtin_amdgcn_perm(0x43434343u, hi, 0x04020400u);
    p[2] = __builtin_amdgcn_perm(0x43434343u, lo, 0x04030401u);
    p[3] = __builtin_amdgcn_perm(0x43434343u, hi, 0x04030401u);
  }
}

template <int DQ>
__device__ __forceinline__ float unit_dot(const NibConst& nc, const uint4 w, uint32_t szw,
                                          const uint32_t (&x)[16], float sx) {
  const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
  float d = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t p[4];
    nib_pairs<DQ>(nc, wd[j], p);
#pragma unroll
    for (int i = 0; i < 4; ++i) d = dot2_bf16(x[4 * j + i], p[i], d);
  }
  return fmaf(bf16lo_to_f32(szw), d - 136.f * sx, bf16hi_to_f32(szw) * sx);
}

__device__ __forceinline__ float pair_sum(const uint32_t (&x)[16]) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s = dot2_bf16(x[i], 0x3F803F80u, s);
  return s;
}

template <int NS1, int NS2, int kCons, int DQ, int kAhead, bool DYN>
__global__ __launch_bounds__(64 * (kCons + 1 + DYN), 1) void ffn_engine_kernel(FfnArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 ring[kRing * kSlotB / 16];
  __shared__ unsigned full[kRing], freew[kRing], blk[kRing], tq[kTq], done_lds, p1_lds, p2go, n1w,
      tqn, ldr_g;
  __shared__ float red[kCons][16];
  constexpr int NSL = NS1 + NS2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wg = blockIdx.x;
  constexpr int kRows13 = NS1 * 8;   // w1||w3 rows of this workgroup
  constexpr int kRows2 = 16;         // w2 rows of this workgroup
  constexpr int kK2B = NS2 * 1024;   // bytes of one w2 row's nibbles (NS2 units of 2048 k)
  constexpr int kS2B = NS2 * 256;    // bytes of one w2 row's (scale, zero) words

  if (threadIdx.x < kRing) {
    full[threadIdx.x] = 0u;
    freew[threadIdx.x] = 0u;
  }
  if (threadIdx.x == 0) {
    done_lds = 0u;
    p1_lds = 0u;
    p2go = 0u;
    n1w = DYN ? ~0u : (unsigned)NS1;
    tqn = 0u;
    ldr_g = 0u;
  }
  __syncthreads();  // the only workgroup barrier: the roles below never meet again

  if (wave == 0) {
    // ---------------------------------- loader ----------------------------------------------
    stamp(a, 0, now());
    unsigned long long t_free = 0;
    const Rsrc r13 = make_rsrc(a.w13, (uint32_t)((size_t)kNWG * kRows13 * 2048));
    const Rsrc rz13 = make_rsrc(a.sz13, (uint32_t)((size_t)kNWG * kRows13 * 512));
    const Rsrc r2 = make_rsrc(a.w2, (uint32_t)((size_t)kNWG * kRows2 * kK2B));
    const Rsrc rz2 = make_rsrc(a.sz2, (uint32_t)((size_t)kNWG * kRows2 * kS2B));
    const uint32_t v16 = 16u * lane;
    // phase-2 (scale, zero) pieces: 4 rows x 256 B per wave-instruction
    const uint32_t vz2 = (uint32_t)(lane >> 4) * kS2B + 16u * (lane & 15);
    const uint32_t base13 = (uint32_t)wg * kRows13;
    const uint32_t base2 = (uint32_t)wg * kRows2;
    // phase-1 slot: block b = rows 8 b .. 8 b + 7 of w1||w3 (8 x 2048 B contiguous, then their
    // 8 x 512 B of words); phase-2 slot: unit u of this workgroup's 16 w2 rows (one 1 KiB piece per
    // row, words 4 rows per piece)
    auto issue1 = [&](int g, uint32_t b) __attribute__((always_inline)) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(ring) + (g % kRing) * kSlotB;
      const uint32_t r0 = 8u * b;
#pragma unroll
      for (int p = 0; p < 16; ++p)
        dma_lds_ring<16, kNT>(r13, v16, r0 * 2048u + 1024u * p, dst + 1024 * p);
#pragma unroll
      for (int p = 0; p < 4; ++p)
        dma_lds_ring<16, kNT>(rz13, v16, r0 * 512u + 1024u * p, dst + kScaleOff + 1024 * p);
    };
    auto issue2 = [&](int g, uint32_t u) __attribute__((always_inline)) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(ring) + (g % kRing) * kSlotB;
#pragma unroll
      for (int p = 0; p < 16; ++p)
        dma_lds_ring<16, kNT>(r2, v16, (base2 + p) * (uint32_t)kK2B + 1024u * u, dst + 1024 * p);
#pragma unroll
      for (int p = 0; p < 4; ++p)
        dma_lds_ring<16, kNT>(rz2, vz2, (base2 + 4u * p) * (uint32_t)kS2B + 256u * u,
                              dst + kScaleOff + 1024 * p);
    };
    auto wait_free = [&](int g) __attribute__((always_inline)) {
      if (g < kRing) return;  // slot g % kRing free again (consumer of slot g - kRing done)
      const unsigned long long tw = a.stamps ? now() : 0;
      SeamWait sw;
      while (lds_ld(&freew[g % kRing]) != (unsigned)(g - kRing + 1)) {
        if (sw.timed_out()) {
          flag_decode_error(kDecodeErrSplitK);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (a.stamps) t_free += now() - tw;
    };
    auto publish = [&](int g) __attribute__((always_inline)) {
      lds_st(&full[g % kRing], (unsigned)(g + 1));
    };
    int n1 = NS1;
    if constexpr (DYN) {
      // w1||w3 blocks come from a queue per blockIdx % 8 (kHeads heads of NS1 kNWG / kHeads
      // blocks each), two blocks per ticket, taken by this workgroup's dispatcher wave into the
      // LDS ticket ring tq: a CU whose stream runs slow takes fewer blocks, so the phase-1 finish
      // lines up across CUs (what the all-to-all edge waits for)
      constexpr unsigned kLimit = (unsigned)(NS1 * kNWG / kHeads);
      const uint32_t qbase = (uint32_t)(wg % kHeads) * kLimit;
      for (int g = 0;; ++g) {
        const int i = g >> 1;
        {
          SeamWait sw;
          while ((int)lds_ld(&tqn) <= i) {
            if (sw.timed_out()) {
              flag_decode_error(kDecodeErrSplitK);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const uint32_t t = lds_ld(&tq[i % kTq]);
        if (t >= kLimit) {  // queue empty: this workgroup's phase 1 is slots 0 .. g - 1
          n1 = g;
          wait_vmcnt<0>();
          for (int k = g - kAhead > 0 ? g - kAhead : 0; k < g; ++k) publish(k);
          lds_st(&n1w, (unsigned)g);
          break;
        }
        lds_st(&ldr_g, (unsigned)(g + 1));
        const uint32_t blockid = qbase + t + (uint32_t)(g & 1);
        wait_free(g);
        lds_st(&blk[g % kRing], blockid);
        issue1(g, blockid);
        if (g >= kAhead) {
          wait_vmcnt<kAhead * kPieces>();
          publish(g - kAhead);
        }
      }
      stamp(a, 1, now());
      for (int j = 0; j < NS2; ++j) {
        const int g = n1 + j;
        wait_free(g);
        issue2(g, (uint32_t)j);
        if (j >= kAhead) {
          wait_vmcnt<kAhead * kPieces>();
          publish(g - kAhead);
        }
      }
      stamp(a, 2, now());
      static_for<0, kAhead>([&](auto kc) __attribute__((always_inline)) {  // drain, oldest first
        constexpr int k = kAhead - 1 - decltype(kc)::value;
        wait_vmcnt<k * kPieces>();
        publish(n1 + NS2 - 1 - k);
      });
    } else {
      for (int g = 0; g < NSL; ++g) {
        wait_free(g);
        if (g < NS1) {
          lds_st(&blk[g % kRing], base13 / 8u + (uint32_t)g);
          issue1(g, base13 / 8u + (uint32_t)g);
        } else {
          issue2(g, (uint32_t)(g - NS1));
        }
        if (g == NS1 - 1) stamp(a, 1, now());
        if (g >= kAhead) {  // slot g - kAhead has landed: kAhead slots' pieces may still be out
          wait_vmcnt<kAhead * kPieces>();
          publish(g - kAhead);
        }
      }
      stamp(a, 2, now());
      static_for<0, kAhead>([&](auto kc) __attribute__((always_inline)) {  // drain, oldest first
        constexpr int k = kAhead - 1 - decltype(kc)::value;
        wait_vmcnt<k * kPieces>();
        publish(NSL - 1 - k);
      });
    }
    stamp(a, 3, now());
    stamp(a, 4, t_free);
    return;
  }

  if (DYN && wave == kCons + 1) {
    // ---------------------------------- dispatcher ------------------------------------------
    // one returning agent-scope atomic per two w1||w3 blocks, at most kTqAhead tickets ahead of
    // the loader (tickets taken early could leave another CU idle)
    constexpr unsigned kLimit = (unsigned)(NS1 * kNWG / kHeads);
    unsigned* head = a.ctl + kHead0 + 32 * (wg % kHeads);
    for (int i = 0;; ++i) {
      {
        SeamWait sw;
        while (2 * i > (int)lds_ld(&ldr_g) + 2 * kTqAhead) {
          if (sw.timed_out()) {
            flag_decode_error(kDecodeErrSplitK);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      unsigned t = 0;
      if (lane == 0)
        t = __hip_atomic_fetch_add(head, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = __shfl(t, 0);
      if (lane == 0) {
        lds_st(&tq[i % kTq], t);
        lds_st(&tqn, (unsigned)(i + 1));
      }
      if (t >= kLimit) break;
    }
    return;
  }

  // ------------------------------------ consumers -------------------------------------------
  const int c = wave - 1;
  const NibConst nc(a.nib_mask, a.nib_magic);
  const unsigned epoch = a.ctl[0];
  const uint8_t* ringb = reinterpret_cast<const uint8_t*>(ring);
  unsigned long long t_full = 0;
  auto wait_full = [&](int g) __attribute__((always_inline)) {
    const unsigned long long tw = a.stamps ? now() : 0;
    SeamWait sw;
    while (lds_ld(&full[g % kRing]) != (unsigned)(g + 1)) {
      if (sw.timed_out()) {
        flag_decode_error(kDecodeErrSplitK);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (a.stamps) t_full += now() - tw;
    asm volatile("" ::: "memory");
  };
  auto release = [&](int g) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot are back
    if (lane == 0) lds_st(&freew[g % kRing], (unsigned)(g + 1));
  };

  // phase-1 input: x = bf16(bf16(h * r) * w), r = rsqrt(mean(h^2) + eps); lane l holds
  // k = 32 l .. 32 l + 31 (unit 0) and 2048 + 32 l .. (unit 1)
  uint32_t x1[2][16];
  float sx1[2];
  {
    const uint4* hp = reinterpret_cast<const uint4*>(a.h);
    const uint4* wp = reinterpret_cast<const uint4*>(a.norm_w);
    uint4 hv[2][4], gv[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hv[u][j] = hp[u * 256 + lane * 4 + j];
        gv[u][j] = wp[u * 256 + lane * 4 + j];
      }
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t d[4] = {hv[u][j].x, hv[u][j].y, hv[u][j].z, hv[u][j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float lo = bf16lo_to_f32(d[i]), hi = bf16hi_to_f32(d[i]);
          ss = fmaf(lo, lo, fmaf(hi, hi, ss));
        }
      }
    ss = wave_sum(ss);
    const float r = rsqrtf(ss / 4096.f + a.eps);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t d[4] = {hv[u][j].x, hv[u][j].y, hv[u][j].z, hv[u][j].w};
        const uint32_t w[4] = {gv[u][j].x, gv[u][j].y, gv[u][j].z, gv[u][j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float lo = round_bf16(bf16lo_to_f32(d[i]) * r) * bf16lo_to_f32(w[i]);
          const float hi = round_bf16(bf16hi_to_f32(d[i]) * r) * bf16hi_to_f32(w[i]);
          x1[u][4 * j + i] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
        }
      }
      sx1[u] = pair_sum(x1[u]);
    }
  }

  stamp(a, 8 + 6 * c, now());
  // ---- phase 1: w1||w3 rows -> SwiGLU granules ----
  int n1 = NS1;
#pragma unroll 1
  for (int g = c;; g += kCons) {
    if constexpr (DYN) {  // slot g holds a block, or the loader has closed phase 1 before it
      const unsigned long long tw = a.stamps ? now() : 0;
      SeamWait sw;
      bool have = false;
      while (true) {
        // FULL first, then the phase-1 count: the loader sets n1w before it publishes any
        // phase-2 slot (whose FULL value g + 1 a phase-1 wait could otherwise mistake), and LDS
        // keeps one wave's writes in order
        const bool f = lds_ld(&full[g % kRing]) == (unsigned)(g + 1);
        const unsigned n = lds_ld(&n1w);
        if (n != ~0u && g >= (int)n) {
          n1 = (int)n;
          break;
        }
        if (f) {
          have = true;
          break;
        }
        if (sw.timed_out()) {
          flag_decode_error(kDecodeErrSplitK);
          n1 = g;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (a.stamps) t_full += now() - tw;
      asm volatile("" ::: "memory");
      if (!have) break;
    } else {
      if (g >= NS1) break;
      wait_full(g);
    }
    const uint32_t blkid = lds_ld(&blk[g % kRing]);
    const uint8_t* sl = ringb + (g % kRing) * kSlotB;
    // the slot's 8 rows x 2 units into registers, then the slot is released before the
    // arithmetic: a slot is held for its landing plus one LDS pass, not for the dot products
    uint4 w[8][2];
    uint32_t szw[8][2];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        w[r][u] = *reinterpret_cast<const uint4*>(sl + r * 2048 + u * 1024 + 16 * lane);
        szw[r][u] =
            *reinterpret_cast<const uint32_t*>(sl + kScaleOff + r * 512 + u * 256 + 4 * lane);
      }
    release(g);
    float v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      v[r] = unit_dot<DQ>(nc, w[r][0], szw[r][0], x1[0], sx1[0]) +
             unit_dot<DQ>(nc, w[r][1], szw[r][1], x1[1], sx1[1]);
    }
    wave_reduce_scatter<8>(v, lane);  // v[0] = total of row lane >> 3
    const float o = round_bf16(v[0]);
    const int b = (lane & 1) * 32;    // lane 0: rows 0..3, lane 1: rows 4..7
    const float a0 = __shfl(o, b), b0 = __shfl(o, b + 8), a1 = __shfl(o, b + 16),
                b1 = __shfl(o, b + 24);
    if (lane < 2) {
      const uint32_t s0 = f32_to_bf16(round_bf16(a0 / (1.f + __expf(-a0))) * b0);
      const uint32_t s1 = f32_to_bf16(round_bf16(a1 / (1.f + __expf(-a1))) * b1);
      const size_t gi = (size_t)2 * blkid + lane;
      __hip_atomic_store(a.pay + gi, s0 | (s1 << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  // publish: every storing wave drains its sc1 stores, counts itself in LDS, and the last of
  // the workgroup's consumer waves adds the workgroup's arrival to its shard counter
  // (MI355X_MICROARCH.md hand-offs with sc1 loads, first row: one signal per storing workgroup,
  // sc1 payload stores and loads, the polling wave loads only after its poll matched)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bool signaller;
  {
    unsigned arrived = 0;
    if (lane == 0)
      arrived = __hip_atomic_fetch_add(&p1_lds, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    signaller = __shfl(arrived, 0) == kCons - 1;
    if (signaller && lane == 0)
      (void)__hip_atomic_fetch_add(a.ctl + kShard0 + 32 * (wg % kShards), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  stamp(a, 9 + 6 * c, now());
  // ---- phase 2: wait for every workgroup's SwiGLU outputs, load this consumer's units, w2 ----
  // phase-2 slots g = n1 + u; consumer c owns the units u with (n1 + u) % kCons == c
  constexpr int kMaxU = (NS2 + kCons - 1) / kCons;
  const int u0 = ((c - n1) % kCons + kCons) % kCons;  // first unit of this consumer
  const int nu = u0 < NS2 ? (NS2 - u0 + kCons - 1) / kCons : 0;
  uint32_t x2[kMaxU][16];
  float sx2[kMaxU];
  {
    // ONE poller per workgroup (the wave that signalled it) reads the 8 shard counters, sleeping
    // ~0.05 us between polls; the counters only grow (kNWG / kShards arrivals per launch), so this
    // launch's are complete at (kNWG / kShards) x epoch. It then sets an LDS word the other
    // consumer waves poll (the table row's "after an LDS word it then sets").
    SeamWait sw;
    if (signaller) {
      const unsigned need = (unsigned)(kNWG / kShards) * epoch;
      while (true) {
        bool ok = true;
        if (lane < kShards)
          ok = __hip_atomic_load(a.ctl + kShard0 + 32 * lane, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) >= need;
        if (__all(ok)) break;
        if (sw.timed_out()) {
          flag_decode_error(kDecodeErrSplitK);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (lane == 0) lds_st(&p2go, 1u);
    } else {
      while (lds_ld(&p2go) == 0u) {
        if (sw.timed_out()) {
          flag_decode_error(kDecodeErrSplitK);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    asm volatile("" ::: "memory");
    const Rsrc rp = make_rsrc(a.pay, (uint32_t)((size_t)a.inter * 2));
#pragma unroll
    for (int ui = 0; ui < kMaxU; ++ui) {
      const int u = ui < nu ? u0 + kCons * ui : u0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 v = bload16<kSC1>(rp, (uint32_t)(64 * lane + 16 * i), (uint32_t)(4096 * u));
        x2[ui][4 * i] = v.x;
        x2[ui][4 * i + 1] = v.y;
        x2[ui][4 * i + 2] = v.z;
        x2[ui][4 * i + 3] = v.w;
      }
      sx2[ui] = pair_sum(x2[ui]);
    }
  }
  stamp(a, 10 + 6 * c, now());
  float acc2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
#pragma unroll
  for (int ui = 0; ui < kMaxU; ++ui) {
    if (ui < nu) {
      const int g = n1 + u0 + kCons * ui;
      wait_full(g);
      const uint8_t* sl = ringb + (g % kRing) * kSlotB;
      // computed straight from LDS: with kRing = 7 the phase-2 slots never wait for one another,
      // so holding the slot through the arithmetic delays nothing
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint4 w = *reinterpret_cast<const uint4*>(sl + r * 1024 + 16 * lane);
        const uint32_t szw = *reinterpret_cast<const uint32_t*>(sl + kScaleOff + r * 256 + 4 * lane);
        acc2[r] += unit_dot<DQ>(nc, w, szw, x2[ui], sx2[ui]);
      }
      release(g);
    }
  }
  stamp(a, 11 + 6 * c, now());
  stamp(a, 13 + 6 * c, t_full);
  wave_reduce_scatter<16>(acc2, lane);  // acc2[0] = this wave's total of row lane >> 2
  if ((lane & 3) == 0) red[c][lane >> 2] = acc2[0];
  unsigned last = 0;
  if (lane == 0) last = __hip_atomic_fetch_add(&done_lds, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) == kCons - 1;
  last = __shfl(last, 0);
  if (!last) {
    stamp(a, 12 + 6 * c, now());
    return;
  }
  asm volatile("" ::: "memory");
  if (lane < 16) {
    float t = red[0][lane];
#pragma unroll
    for (int k = 1; k < kCons; ++k) t += red[k][lane];
    const int n = wg * kRows2 + lane;
    a.out[n] = f32_to_bf16(round_bf16(t) + bf16_to_f32(a.h[n]));
  }
  if (lane == 0) {  // epoch hand-over: the last workgroup out advances it for the next launch
    const unsigned prev =
        __hip_atomic_fetch_add(a.ctl + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == kNWG - 1) {  // every workgroup is done: the queues start empty again
      if constexpr (DYN)
        for (int q = 0; q < kHeads; ++q)
          __hip_atomic_store(a.ctl + kHead0 + 32 * q, 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctl + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctl, epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  stamp(a, 12 + 6 * c, now());
}

}  // namespace

int ffn_engine_cus() {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
    cus = n;
  }
  return cus;
}

}  // namespace tao

static unsigned long long* g_engine_stamps = nullptr;
static int g_engine_consumers = 7;
static int g_engine_dq = 1;
static int g_engine_ahead = 3;
static int g_engine_dyn = 0;

// A/B knobs: consumer waves per workgroup (3: 256-thread workgroups, one consumer per SIMD
// beside the loader's; 7: 512 threads, two per SIMD) and the nibble decode (0: shift, and, or;
// 1: byte permutes), and the loader's slots in flight beyond the last published one (1..3; 3
// consumers run 1 / 2, dq 0 runs 2)
extern "C" int tao_tune_ffn_engine(int consumers, int dq, int ahead, int dyn) {
  TAO_CHECK_ARG(dyn == 0 || dyn == 1, "tune: ffn engine dyn must be 0 or 1");
  g_engine_dyn = dyn;
  TAO_CHECK_ARG(consumers == 3 || consumers == 7, "tune: ffn engine consumers must be 3 or 7");
  TAO_CHECK_ARG(dq == 0 || dq == 1, "tune: ffn engine decode must be 0 or 1");
  TAO_CHECK_ARG(ahead >= 1 && ahead <= 3, "tune: ffn engine slots ahead must be 1..3");
  g_engine_consumers = consumers;
  g_engine_dq = dq;
  g_engine_ahead = ahead;
  return TAO_OK;
}

// measurement hook: per-workgroup phase stamps of the following engine launches into `buf`
// (256 x 32 u64 device memory; NULL turns it off)
extern "C" int tao_debug_ffn_engine_stamps(void* buf) {
  g_engine_stamps = reinterpret_cast<unsigned long long*>(buf);
  return TAO_OK;
}

extern "C" int tao_int4wo_ffn_engine_supported(int64_t dim, int64_t inter, int64_t group_size) {
  return dim == 4096 && inter == 14336 && group_size == 32 && tao::ffn_engine_cus() >= tao::kNWG;
}

extern "C" int tao_int4wo_ffn_engine_bf16(const uint16_t* h, const uint16_t* norm_weight,
                                          float eps, const uint32_t* w13, const uint16_t* sz13,
                                          const uint32_t* w2, const uint16_t* sz2, uint16_t* out,
                                          int64_t dim, int64_t inter, int64_t group_size,
                                          unsigned* ctl, uint32_t* payload, void* stream) {
  using namespace tao;
  TAO_CHECK_ARG(h && norm_weight && w13 && sz13 && w2 && sz2 && out && ctl && payload,
                "ffn engine: null operand");
  TAO_CHECK_ARG(tao_int4wo_ffn_engine_supported(dim, inter, group_size),
                "ffn engine: shape (dim %lld, inter %lld, g %lld) or device (%d CUs) unsupported",
                (long long)dim, (long long)inter, (long long)group_size, ffn_engine_cus());
  TAO_CHECK_ARG(out != h, "ffn engine: out must not alias h");
  TAO_CHECK_ALIGN(h, 16, "h");
  TAO_CHECK_ALIGN(norm_weight, 16, "norm_weight");
  TAO_CHECK_ALIGN(w13, 16, "w13");
  TAO_CHECK_ALIGN(sz13, 16, "sz13");
  TAO_CHECK_ALIGN(w2, 16, "w2");
  TAO_CHECK_ALIGN(sz2, 16, "sz2");
  TAO_CHECK_ALIGN(payload, 16, "payload");
  TAO_CHECK_ALIGN(ctl, 128, "ctl");
  FfnArgs a{h, norm_weight, eps, w13, reinterpret_cast<const uint32_t*>(sz13), w2,
            reinterpret_cast<const uint32_t*>(sz2), out, ctl, payload, (int)inter,
            g_engine_stamps, 0x000F000Fu, 0x43004300u};
  const int nc = g_engine_consumers, dq = g_engine_dq, ah = g_engine_ahead;
#define TAO_FFN_GO(NC, DQ, AH, DY)                                                             \
  hipLaunchKernelGGL((ffn_engine_kernel<14, 7, NC, DQ, AH, DY>), dim3(kNWG),                 \
                     dim3(64 * (NC + 1 + DY)), 0, (hipStream_t)stream, a)
  if (g_engine_dyn) {
    TAO_FFN_GO(7, 1, 2, true);
  } else if (nc == 3) {
    TAO_FFN_GO(3, 1, 2, false);
  } else if (dq == 0) {
    TAO_FFN_GO(7, 0, 2, false);
  } else if (ah == 3) {
    TAO_FFN_GO(7, 1, 3, false);
  } else if (ah == 1) {
    TAO_FFN_GO(7, 1, 1, false);
  } else {
    TAO_FFN_GO(7, 1, 2, false);
  }
#undef TAO_FFN_GO
  return check_launch("ffn_engine_kernel");
}

// workspace: ctl (kCtlBytes: epoch at word 0 = 1, done counter at 32, shard counters at
// 64 + 32 s, queue heads at 320 + 32 q, all zero otherwise) + the SwiGLU payload [inter / 2] u32
extern "C" int64_t tao_int4wo_ffn_engine_workspace_bytes(int64_t inter) {
  return tao::kCtlBytes + inter / 2 * 4;
}
