// Library-level C-ABI entry points (version, error state, device count) and the host-side
// int4 packers. Kernel entry points live next to their kernels (int4_*.hip, int8_*.hip).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "tao_common.h"

namespace tao {

static thread_local char g_err[512] = {0};

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { g_err[0] = 0; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TAO_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return TAO_OK;
}

// ---- per-kernel timing sessions --------------------------------------------------------------
struct ProfileSession {
  bool active = false;
  std::vector<hipEvent_t> start, stop;
  size_t used = 0;
};
static thread_local ProfileSession g_prof;

bool profile_slot(hipEvent_t* a, hipEvent_t* b) {
  if (!g_prof.active || g_prof.used >= g_prof.start.size()) return false;
  *a = g_prof.start[g_prof.used];
  *b = g_prof.stop[g_prof.used];
  ++g_prof.used;
  return true;
}

static void profile_release() {
  for (hipEvent_t e : g_prof.start) (void)hipEventDestroy(e);
  for (hipEvent_t e : g_prof.stop) (void)hipEventDestroy(e);
  g_prof.start.clear();
  g_prof.stop.clear();
  g_prof.used = 0;
  g_prof.active = false;
}

Tuning& tuning() {
  static thread_local Tuning t;
  return t;
}

// ---- split-K workspace --------------------------------------------------------------------------
struct Workspace {
  void* slab = nullptr;
  size_t slab_cap = 0;
  unsigned* cnt = nullptr;
  size_t cnt_cap = 0;
};
static std::mutex g_ws_mu;
// eager: one per (device, stream); graphs: one per (device, capture sequence id), never freed
static std::map<std::pair<int, hipStream_t>, Workspace> g_ws;
static std::map<std::pair<int, unsigned long long>, Workspace> g_ws_graph;

// Allocate zeroed counters without touching any stream that may be capturing: a private
// non-blocking stream does the memset (it does not synchronise with the capturing stream).
static int alloc_counters(unsigned** cnt, size_t n) {
  if (hipMalloc(reinterpret_cast<void**>(cnt), n * sizeof(unsigned)) != hipSuccess)
    return set_error(TAO_ERR_HIP, "split-K counter allocation failed");
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return set_error(TAO_ERR_HIP, "split-K counter init: stream creation failed");
  const bool ok = hipMemsetAsync(*cnt, 0, n * sizeof(unsigned), s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess;
  (void)hipStreamDestroy(s);
  return ok ? TAO_OK : set_error(TAO_ERR_HIP, "split-K counter init failed");
}

int split_workspace(hipStream_t stream, size_t slab_bytes, size_t counters, void** slab,
                    unsigned** cnt) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(TAO_ERR_HIP, "hipGetDevice failed");
  std::lock_guard<std::mutex> lock(g_ws_mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cap_id = 0;
  if (hipStreamGetCaptureInfo(stream, &cs, &cap_id) != hipSuccess)
    return set_error(TAO_ERR_HIP, "hipStreamGetCaptureInfo failed");
  if (cs == hipStreamCaptureStatusActive) {
    // This capture's own workspace. Allocation is not a stream operation; relaxed mode lets
    // this thread make it while a global-mode capture is open. A larger request later in the
    // same capture retires the smaller buffers (kept: earlier nodes of this graph use them).
    Workspace& w = g_ws_graph[{dev, cap_id}];
    if (w.slab_cap < slab_bytes || w.cnt_cap < counters) {
      hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
      (void)hipThreadExchangeStreamCaptureMode(&mode);
      int rc = TAO_OK;
      Workspace n;
      n.slab_cap = std::max(slab_bytes, w.slab_cap);
      n.cnt_cap = std::max(counters, w.cnt_cap);
      if (hipMalloc(&n.slab, n.slab_cap) != hipSuccess)
        rc = set_error(TAO_ERR_HIP, "hipMalloc of %zu B split-K slabs (capture) failed",
                       n.slab_cap);
      if (rc == TAO_OK) rc = alloc_counters(&n.cnt, n.cnt_cap);
      (void)hipThreadExchangeStreamCaptureMode(&mode);
      if (rc != TAO_OK) return rc;
      w = n;  // the previous buffers are intentionally leaked: the graph references them
    }
    *slab = w.slab;
    *cnt = w.cnt;
    return TAO_OK;
  }
  if (cs != hipStreamCaptureStatusNone)
    return set_error(TAO_ERR_HIP, "split-K launch on an invalidated capture");
  Workspace& w = g_ws[{dev, stream}];
  if (w.slab_cap < slab_bytes || w.cnt_cap < counters) {
    // only work queued on this stream can hold the old buffers (graphs never borrow them)
    if (hipStreamSynchronize(stream) != hipSuccess)
      return set_error(TAO_ERR_HIP, "hipStreamSynchronize failed");
    const size_t sb = std::max(slab_bytes, w.slab_cap);
    const size_t nc = std::max(counters, w.cnt_cap);
    if (w.slab_cap < sb) {
      (void)hipFree(w.slab);
      w.slab = nullptr;
      w.slab_cap = 0;
      if (hipMalloc(&w.slab, sb) != hipSuccess)
        return set_error(TAO_ERR_HIP, "hipMalloc of %zu B split-K slabs failed", sb);
      w.slab_cap = sb;
    }
    if (w.cnt_cap < nc) {
      (void)hipFree(w.cnt);
      w.cnt = nullptr;
      w.cnt_cap = 0;
      const int rc = alloc_counters(&w.cnt, nc);
      if (rc != TAO_OK) return rc;
      w.cnt_cap = nc;
    }
  }
  *slab = w.slab;
  *cnt = w.cnt;
  return TAO_OK;
}

}  // namespace tao

extern "C" {

const char* tao_version(void) { return "torchao-mi355x 0.1.0 gfx950"; }

const char* tao_last_error(void) { return tao::g_err; }

int tao_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int tao_tune_reset(void) {
  tao::tuning() = tao::Tuning{};
  return TAO_OK;
}

int tao_tune_splitk_fenced(int fenced) {
  TAO_CHECK_ARG(fenced == 0 || fenced == 1, "tune: splitk_fenced must be 0 or 1");
  tao::tuning().splitk_fenced = fenced;
  return TAO_OK;
}

int tao_profile_begin(int capacity) {
  TAO_CHECK_ARG(capacity > 0 && capacity <= (1 << 20), "profile: capacity out of range");
  tao::profile_release();
  tao::g_prof.start.resize(capacity, nullptr);
  tao::g_prof.stop.resize(capacity, nullptr);
  for (int i = 0; i < capacity; ++i) {
    if (hipEventCreate(&tao::g_prof.start[i]) != hipSuccess ||
        hipEventCreate(&tao::g_prof.stop[i]) != hipSuccess) {
      tao::profile_release();
      return tao::set_error(TAO_ERR_HIP, "profile: hipEventCreate failed");
    }
  }
  tao::g_prof.active = true;
  return TAO_OK;
}

int tao_profile_end(float* durations_ms, int capacity, int* count) {
  TAO_CHECK_ARG(count != nullptr, "profile: null count");
  *count = 0;
  if (!tao::g_prof.active) return tao::set_error(TAO_ERR_INVALID_ARGUMENT, "profile: no session");
  const int n = (int)tao::g_prof.used;
  int rc = TAO_OK;
  for (int i = 0; i < n && i < capacity; ++i) {
    float ms = 0.f;
    if (hipEventSynchronize(tao::g_prof.stop[i]) != hipSuccess ||
        hipEventElapsedTime(&ms, tao::g_prof.start[i], tao::g_prof.stop[i]) != hipSuccess) {
      rc = tao::set_error(TAO_ERR_HIP, "profile: event timing failed for launch %d", i);
      break;
    }
    durations_ms[i] = ms;
    *count = i + 1;
  }
  tao::profile_release();
  return rc;
}

// Host packer: identical bytes to int4_pack_kernel (int4_pack.hip). Used when quantize_ runs on
// a CPU-resident model (the reference quantizes on whatever device the weight lives on,
// torchao/quantization/quant_api.py:173-222).
int tao_int4_pack_host(const int32_t* q, uint32_t* packed, int64_t N, int64_t K) {
  TAO_CHECK_ARG(N >= 0 && K >= 0 && K % 8 == 0, "int4 pack: need K %% 8 == 0 (K=%lld)",
                (long long)K);
  TAO_CHECK_ARG(q != nullptr || N * K == 0, "int4 pack: null q");
  const int64_t KD = K / 8;
  for (int64_t n = 0; n < N; ++n) {
    const int32_t* row = q + n * K;
    for (int64_t d = 0; d < KD; ++d) {
      uint32_t w = 0;
      for (int i = 0; i < 4; ++i) {
        int32_t a = row[8 * d + 2 * i], b = row[8 * d + 2 * i + 1];
        if ((uint32_t)a > 15u || (uint32_t)b > 15u)
          return tao::set_error(TAO_ERR_INVALID_ARGUMENT,
                                "int4 pack: value out of [0,15] at row %lld", (long long)n);
        w |= (uint32_t)a << (4 * i);
        w |= (uint32_t)b << (16 + 4 * i);
      }
      packed[n * KD + d] = w;
    }
  }
  return TAO_OK;
}

int tao_int4_unpack_host(const uint32_t* packed, int32_t* q, int64_t N, int64_t K) {
  TAO_CHECK_ARG(N >= 0 && K >= 0 && K % 8 == 0, "int4 unpack: need K %% 8 == 0 (K=%lld)",
                (long long)K);
  const int64_t KD = K / 8;
  for (int64_t n = 0; n < N; ++n) {
    for (int64_t d = 0; d < KD; ++d) {
      uint32_t w = packed[n * KD + d];
      int32_t* out = q + n * K + 8 * d;
      for (int i = 0; i < 4; ++i) {
        out[2 * i] = (w >> (4 * i)) & 0xF;
        out[2 * i + 1] = (w >> (16 + 4 * i)) & 0xF;
      }
    }
  }
  return TAO_OK;
}

}  // extern "C"
