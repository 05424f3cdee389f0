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

static thread_local const char* g_last_kernel = "";

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(TAO_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  g_last_kernel = what;
  return TAO_OK;
}

const char* last_kernel() { return g_last_kernel; }

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

bool fence_free_validated() {
  static const bool ok = [] {
    int v = 0;
    if (hipRuntimeGetVersion(&v) != hipSuccess) return false;
    // HIP_VERSION = major * 10^7 + minor * 10^5 + patch. Inside a PyTorch process the runtime is
    // the one torch bundles (7.0 for torch 2.10+rocm7.0, the runtime every GPU test of rounds 1-3
    // ran under); standalone C-ABI programs load /opt/rocm's 7.2. Both are validated.
    const int mm = v / 100000;
    return mm == 700 || mm == 702;
  }();
  return ok;
}

Tuning& tuning() {
  static thread_local Tuning t;
  return t;
}

// ---- split-K workspace --------------------------------------------------------------------------
// Two counter arrays, both zeroed once:
//  * cnt  (u32): gemm_mfma.hip's last-arriver tickets, each reset to 0 by its tile's last arriver;
//  * sync (u64): gemm_tile.hip's epoch counters (arrivals advance by 64 per launch, claim words hold
//    launch epochs; never reset). Separate arrays, so neither protocol sees the other's values.
struct Workspace {
  void* slab = nullptr;
  size_t slab_cap = 0;
  unsigned* cnt = nullptr;
  size_t cnt_cap = 0;
  unsigned long long* sync = nullptr;
  size_t sync_cap = 0;
};
static std::recursive_mutex g_ws_mu;
// eager: one per (device, stream); graphs: one per (device, capture sequence id), owned by the graph
static std::map<std::pair<int, hipStream_t>, Workspace> g_ws;
static std::map<std::pair<int, unsigned long long>, Workspace> g_ws_graph;
// buffers of destroyed graphs, freed by the next eager call (a user-object destructor may not call
// HIP; it runs once the graph, its executable copies and their pending launches are gone)
static std::vector<void*> g_ws_retired;

// Allocate zeroed counters without touching any stream that may be capturing: a private
// non-blocking stream does the memset (it does not synchronise with the capturing stream).
static int alloc_zeroed(void** p, size_t bytes) {
  if (hipMalloc(p, bytes) != hipSuccess)
    return set_error(TAO_ERR_HIP, "split-K counter allocation failed");
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    return set_error(TAO_ERR_HIP, "split-K counter init: stream creation failed");
  const bool ok = hipMemsetAsync(*p, 0, bytes, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  (void)hipStreamDestroy(s);
  return ok ? TAO_OK : set_error(TAO_ERR_HIP, "split-K counter init failed");
}

static int alloc_set(Workspace& n, size_t slab_bytes, size_t counters, size_t sync_words) {
  if (slab_bytes && hipMalloc(&n.slab, slab_bytes) != hipSuccess)
    return set_error(TAO_ERR_HIP, "hipMalloc of %zu B split-K slabs failed", slab_bytes);
  n.slab_cap = slab_bytes;
  if (counters) {
    const int rc = alloc_zeroed(reinterpret_cast<void**>(&n.cnt), counters * sizeof(unsigned));
    if (rc != TAO_OK) return rc;
  }
  n.cnt_cap = counters;
  if (sync_words) {
    const int rc =
        alloc_zeroed(reinterpret_cast<void**>(&n.sync), sync_words * sizeof(unsigned long long));
    if (rc != TAO_OK) return rc;
  }
  n.sync_cap = sync_words;
  return TAO_OK;
}

// One allocation set of a captured graph: released when the graph is destroyed (the
// buffers used to live forever, so every re-capture leaked device memory).
struct GraphBuffers {
  std::pair<int, unsigned long long> key;
  void* ptrs[3];
};
static void graph_buffers_release(void* arg) {
  GraphBuffers* gb = static_cast<GraphBuffers*>(arg);
  std::lock_guard<std::recursive_mutex> lock(g_ws_mu);
  for (void* p : gb->ptrs)
    if (p) g_ws_retired.push_back(p);
  auto it = g_ws_graph.find(gb->key);
  if (it != g_ws_graph.end() && it->second.slab == gb->ptrs[0] && it->second.cnt == gb->ptrs[1] &&
      it->second.sync == gb->ptrs[2])
    g_ws_graph.erase(it);
  delete gb;
}

static void free_retired_locked() {
  for (void* p : g_ws_retired) (void)hipFree(p);
  g_ws_retired.clear();
}

static int get_workspace(hipStream_t stream, size_t slab_bytes, size_t counters, size_t sync_words,
                         Workspace* out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(TAO_ERR_HIP, "hipGetDevice failed");
  std::lock_guard<std::recursive_mutex> lock(g_ws_mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cap_id = 0;
  hipGraph_t graph = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  if (hipStreamGetCaptureInfo_v2(stream, &cs, &cap_id, &graph, &deps, &ndeps) != hipSuccess)
    return set_error(TAO_ERR_HIP, "hipStreamGetCaptureInfo failed");
  if (cs == hipStreamCaptureStatusActive) {
    // This capture's own workspace. Allocation is not a stream operation; relaxed mode lets this
    // thread make it while a global-mode capture is open. A larger request later in the same
    // capture allocates a new set; the graph owns every set (earlier nodes use the older ones).
    const std::pair<int, unsigned long long> key{dev, cap_id};
    Workspace& w = g_ws_graph[key];
    if (w.slab_cap < slab_bytes || w.cnt_cap < counters || w.sync_cap < sync_words) {
      hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
      (void)hipThreadExchangeStreamCaptureMode(&mode);
      Workspace n;
      int rc = alloc_set(n, std::max(slab_bytes, w.slab_cap), std::max(counters, w.cnt_cap),
                         std::max(sync_words, w.sync_cap));
      if (rc == TAO_OK) {
        GraphBuffers* gb = new GraphBuffers{key, {n.slab, n.cnt, n.sync}};
        hipUserObject_t obj = nullptr;
        if (hipUserObjectCreate(&obj, gb, graph_buffers_release, 1,
                                hipUserObjectNoDestructorSync) != hipSuccess ||
            hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
          delete gb;
          rc = set_error(TAO_ERR_HIP, "split-K workspace: graph user object failed");
        }
      }
      (void)hipThreadExchangeStreamCaptureMode(&mode);
      if (rc != TAO_OK) return rc;
      w = n;
    }
    *out = w;
    return TAO_OK;
  }
  if (cs != hipStreamCaptureStatusNone)
    return set_error(TAO_ERR_HIP, "split-K launch on an invalidated capture");
  free_retired_locked();
  Workspace& w = g_ws[{dev, stream}];
  if (w.slab_cap < slab_bytes || w.cnt_cap < counters || w.sync_cap < sync_words) {
    // only work queued on this stream can hold the old buffers (graphs never borrow them)
    if (hipStreamSynchronize(stream) != hipSuccess)
      return set_error(TAO_ERR_HIP, "hipStreamSynchronize failed");
    if (w.slab_cap < slab_bytes) {
      (void)hipFree(w.slab);
      w.slab = nullptr;
      w.slab_cap = 0;
      if (hipMalloc(&w.slab, slab_bytes) != hipSuccess)
        return set_error(TAO_ERR_HIP, "hipMalloc of %zu B split-K slabs failed", slab_bytes);
      w.slab_cap = slab_bytes;
    }
    if (w.cnt_cap < counters) {
      (void)hipFree(w.cnt);
      w.cnt = nullptr;
      w.cnt_cap = 0;
      const int rc = alloc_zeroed(reinterpret_cast<void**>(&w.cnt), counters * sizeof(unsigned));
      if (rc != TAO_OK) return rc;
      w.cnt_cap = counters;
    }
    if (w.sync_cap < sync_words) {
      // epoch counters: a grown array restarts at zero, which the protocol allows (every tile
      // counter is a multiple of 64 between launches and claim epochs only need to increase per
      // counter; the old array is gone with its values)
      (void)hipFree(w.sync);
      w.sync = nullptr;
      w.sync_cap = 0;
      const int rc =
          alloc_zeroed(reinterpret_cast<void**>(&w.sync), sync_words * sizeof(unsigned long long));
      if (rc != TAO_OK) return rc;
      w.sync_cap = sync_words;
    }
  }
  *out = w;
  return TAO_OK;
}

int split_workspace(hipStream_t stream, size_t slab_bytes, size_t counters, void** slab,
                    unsigned** cnt) {
  Workspace w;
  const int rc = get_workspace(stream, slab_bytes, counters, 0, &w);
  if (rc != TAO_OK) return rc;
  *slab = w.slab;
  *cnt = w.cnt;
  return TAO_OK;
}

int split_workspace_epoch(hipStream_t stream, size_t slab_bytes, size_t sync_words, void** slab,
                          unsigned long long** sync) {
  Workspace w;
  const int rc = get_workspace(stream, slab_bytes, 0, sync_words, &w);
  if (rc != TAO_OK) return rc;
  *slab = w.slab;
  *sync = w.sync;
  return TAO_OK;
}

// Graph workspaces alive (for tests: re-capturing and destroying graphs must not grow this).
int graph_workspace_count() {
  std::lock_guard<std::recursive_mutex> lock(g_ws_mu);
  return (int)g_ws_graph.size();
}

}  // namespace tao

extern "C" {

const char* tao_version(void) { return "torchao-mi355x 0.1.0 gfx950"; }

const char* tao_last_error(void) { return tao::g_err; }

const char* tao_last_kernel(void) { return tao::last_kernel(); }

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

int tao_graph_workspace_count(void) { return tao::graph_workspace_count(); }

int tao_tune_splitk_fenced(int fenced) {
  TAO_CHECK_ARG(fenced == 0 || fenced == 1, "tune: splitk_fenced must be 0 or 1");
  tao::tuning().splitk_fenced = fenced;
  return TAO_OK;
}

int tao_query_splitk_fenced(void) { return tao::tuning().splitk_fenced; }

int tao_tune_cnt_stride(int stride) {
  TAO_CHECK_ARG(stride == 1 || stride == 32, "tune: cnt_stride must be 1 or 32");
  tao::tuning().cnt_stride = stride;
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
