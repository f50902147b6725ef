// Context lifetime, error reporting and the RANSAC table upload of the kcmc C ABI.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_ext.h>

#include "kcmc_internal.h"

namespace kcmc {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return KCMC_OK;
  return fail(KCMC_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

int launch_check(const char* what) { return hip_check(hipGetLastError(), what); }

// Defined in hostalg.cpp.
int hypothesis_table_impl(int n, int trials, uint32_t seed, int min_samples, int32_t* out);

}  // namespace kcmc

using namespace kcmc;

static void free_tables(kcmc_ctx* ctx);

extern "C" int kcmc_abi_version(void) { return KCMC_ABI_VERSION; }

extern "C" const char* kcmc_last_error(void) { return g_last_error.c_str(); }

extern "C" int kcmc_memcpy_async(void* dst, const void* src, size_t bytes, kcmc_stream_t stream) {
  if (bytes == 0) return KCMC_OK;
  if (!dst || !src) return fail(KCMC_EINVAL, "kcmc_memcpy_async: NULL pointer");
  return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream), "hipMemcpyAsync");
}

extern "C" int kcmc_create(int device, kcmc_ctx** out) {
  if (!out) return fail(KCMC_EINVAL, "kcmc_create: out is NULL");
  int n = 0;
  KCMC_TRY(hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount"));
  if (device < 0 || device >= n)
    return fail(KCMC_EINVAL, "kcmc_create: device " + std::to_string(device) + " out of range");
  auto* c = new (std::nothrow) kcmc_ctx();
  if (!c) return fail(KCMC_ENOMEM, "kcmc_create: out of host memory");
  c->device = device;
  *out = c;
  return KCMC_OK;
}

static void free_model_tables(HypTables& t) {
  if (t.dev) hipFree(t.dev);
  if (t.off) hipFree(t.off);
  t.dev = nullptr;
  t.off = nullptr;
  t.off_len = 0;
}

extern "C" int kcmc_destroy(kcmc_ctx* ctx) {
  if (!ctx) return KCMC_OK;
  bool any_model = false;
  for (const auto& t : ctx->mhyp) any_model = any_model || t.dev || t.off;
  if (ctx->hyp || ctx->hyp_off || ctx->ws_pool || any_model) {
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(ctx->device);
    free_tables(ctx);
    for (auto& t : ctx->mhyp) free_model_tables(t);
    if (ctx->ws_pool) {
      hipDeviceSynchronize();
      // the device is idle: free on the null stream (a cached block's own stream may
      // already be gone when the context is destroyed at interpreter exit)
      for (auto& kv : ctx->stream_ws)
        if (kv.second.ptr) hipFreeAsync(kv.second.ptr, nullptr);
      hipDeviceSynchronize();  // pending stream-ordered frees return to the pool first
      hipMemPoolDestroy(ctx->ws_pool);
    }
    hipSetDevice(prev);
  }
  delete ctx;
  return KCMC_OK;
}

namespace kcmc {

// The per-stream cache is used only on a stream that names one ordered queue and is not
// being captured: a block baked into a hipGraph must never be swapped or freed by later
// eager calls, and hipStreamPerThread is one handle shared by every thread's stream.
static bool cacheable_stream(hipStream_t s) {
  if (s == hipStreamPerThread) return false;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) {
    hipGetLastError();
    return false;
  }
  return st == hipStreamCaptureStatusNone;
}

int workspace_alloc(kcmc_ctx* ctx, void** p, size_t bytes, hipStream_t s) {
  const bool cacheable = cacheable_stream(s);
  {
    std::lock_guard<std::mutex> lk(ctx->ws_mutex);
    if (!ctx->ws_pool) {
      hipMemPoolProps props = {};
      props.allocType = hipMemAllocationTypePinned;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = ctx->device;
      KCMC_TRY(hip_check(hipMemPoolCreate(&ctx->ws_pool, &props), "hipMemPoolCreate"));
      uint64_t keep = UINT64_MAX;  // never trim: the same sizes come back every call
      KCMC_TRY(hip_check(hipMemPoolSetAttribute(ctx->ws_pool, hipMemPoolAttrReleaseThreshold, &keep),
                         "hipMemPoolSetAttribute"));
    }
    if (cacheable) {
      auto it = ctx->stream_ws.find(s);
      if (it != ctx->stream_ws.end() && !it->second.busy && it->second.bytes >= bytes) {
        it->second.busy = true;
        *p = it->second.ptr;
        return KCMC_OK;
      }
    }
  }
  // a stream-ordered pool allocation (under capture: the graph's own allocation node)
  if (hipMallocFromPoolAsync(p, bytes, ctx->ws_pool, s) != hipSuccess) {
    hipGetLastError();
    return fail(KCMC_ENOMEM, "workspace: device out of memory (" + std::to_string(bytes) + " bytes)");
  }
  return KCMC_OK;
}

int workspace_free(kcmc_ctx* ctx, void* p, hipStream_t s, size_t bytes) {
  void* drop = p;
  if (cacheable_stream(s)) {
    std::lock_guard<std::mutex> lk(ctx->ws_mutex);
    kcmc_ctx::StreamScratch& c = ctx->stream_ws[s];
    if (c.ptr == p) {  // the stream's cached block: keep it
      c.busy = false;
      return KCMC_OK;
    }
    if (!c.busy && bytes > c.bytes) {  // a larger block becomes the stream's cache
      drop = c.ptr;
      c.ptr = p;
      c.bytes = bytes;
    }
  }
  return drop ? hip_check(hipFreeAsync(drop, s), "hipFreeAsync") : KCMC_OK;
}

}  // namespace kcmc

static void free_tables(kcmc_ctx* ctx) {
  if (ctx->hyp) hipFree(ctx->hyp);
  if (ctx->hyp_off) hipFree(ctx->hyp_off);
  ctx->hyp = nullptr;
  ctx->hyp_off = nullptr;
  ctx->hyp_off_len = 0;
}

extern "C" int kcmc_ransac_prepare(kcmc_ctx* ctx, const int32_t* n_values, int count, int trials, uint32_t seed) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_ransac_prepare: ctx is NULL");
  if (count < 0 || (count > 0 && !n_values) || trials < 1)
    return fail(KCMC_EINVAL, "kcmc_ransac_prepare: bad arguments");
  // one (trials, seed) table set per context: another seed or trial count replaces it, and
  // the device copy must follow even when no count is new
  bool changed = ctx->hyp == nullptr;
  if (ctx->hyp_trials != trials || ctx->hyp_seed != seed) {
    ctx->hyp_host.clear();
    ctx->hyp_trials = trials;
    ctx->hyp_seed = seed;
    changed = true;
  }
  std::vector<int32_t> tab((size_t)trials * 2);
  for (int k = 0; k < count; ++k) {
    const int n = n_values[k];
    if (n < 3 || n > 65535) return fail(KCMC_EINVAL, "kcmc_ransac_prepare: point counts must be in [3, 65535]");
    if (ctx->hyp_host.count(n)) continue;
    KCMC_TRY(hypothesis_table_impl(n, trials, seed, 2, tab.data()));
    std::vector<uint32_t> packed((size_t)trials);
    for (int t = 0; t < trials; ++t) packed[(size_t)t] = (uint32_t)tab[2 * t] | ((uint32_t)tab[2 * t + 1] << 16);
    ctx->hyp_host.emplace(n, std::move(packed));
    changed = true;
  }
  if (!changed) return KCMC_OK;
  // (re)upload every cached table
  const int off_len = ctx->hyp_host.empty() ? 1 : ctx->hyp_host.rbegin()->first + 1;
  std::vector<int32_t> off((size_t)off_len, -1);
  std::vector<uint32_t> all;
  all.reserve(ctx->hyp_host.size() * (size_t)trials);
  for (const auto& kv : ctx->hyp_host) {
    off[(size_t)kv.first] = (int32_t)all.size();
    all.insert(all.end(), kv.second.begin(), kv.second.end());
  }
  if (all.size() > (size_t)INT32_MAX) return fail(KCMC_EUNSUPPORTED, "kcmc_ransac_prepare: tables too large");
  if (all.empty()) all.push_back(0);
  int prev = 0;
  hipGetDevice(&prev);
  KCMC_TRY(hip_check(hipSetDevice(ctx->device), "hipSetDevice"));
  free_tables(ctx);
  int rc = hip_check(hipMalloc(&ctx->hyp, all.size() * sizeof(uint32_t)), "hipMalloc(hyp)");
  if (rc == KCMC_OK) rc = hip_check(hipMalloc(&ctx->hyp_off, off.size() * sizeof(int32_t)), "hipMalloc(hyp_off)");
  if (rc == KCMC_OK)
    rc = hip_check(hipMemcpy(ctx->hyp, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice),
                   "hipMemcpy(hyp)");
  if (rc == KCMC_OK)
    rc = hip_check(hipMemcpy(ctx->hyp_off, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice),
                   "hipMemcpy(hyp_off)");
  hipSetDevice(prev);
  if (rc != KCMC_OK) {
    free_tables(ctx);
    ctx->hyp_host.clear();
    return rc;
  }
  ctx->hyp_off_len = off_len;
  return KCMC_OK;
}

extern "C" int kcmc_ransac_prepare_samples(kcmc_ctx* ctx, int min_samples, const int32_t* n_values, int count,
                                           int trials, uint32_t seed) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_ransac_prepare_samples: ctx is NULL");
  if (min_samples == 2) return kcmc_ransac_prepare(ctx, n_values, count, trials, seed);
  if (min_samples != 3 && min_samples != 4)
    return fail(KCMC_EINVAL, "kcmc_ransac_prepare_samples: min_samples must be 2, 3 or 4");
  if (count < 0 || (count > 0 && !n_values) || trials < 1)
    return fail(KCMC_EINVAL, "kcmc_ransac_prepare_samples: bad arguments");
  HypTables& T = ctx->mhyp[min_samples];
  bool changed = T.dev == nullptr;
  if (T.trials != trials || T.seed != seed) {
    T.host.clear();
    T.trials = trials;
    T.seed = seed;
    changed = true;
  }
  std::vector<int32_t> tab((size_t)trials * min_samples);
  for (int k = 0; k < count; ++k) {
    const int n = n_values[k];
    if (n <= min_samples || n > 65535)
      return fail(KCMC_EINVAL, "kcmc_ransac_prepare_samples: point counts must be in [min_samples + 1, 65535]");
    if (T.host.count(n)) continue;
    KCMC_TRY(hypothesis_table_impl(n, trials, seed, min_samples, tab.data()));
    std::vector<uint64_t> packed((size_t)trials);
    for (int t = 0; t < trials; ++t) {
      uint64_t w = ~0ull;
      for (int s = 0; s < min_samples; ++s) {
        w &= ~(0xffffull << (16 * s));
        w |= (uint64_t)(uint32_t)tab[(size_t)t * min_samples + s] << (16 * s);
      }
      packed[(size_t)t] = w;
    }
    T.host.emplace(n, std::move(packed));
    changed = true;
  }
  if (!changed) return KCMC_OK;
  const int off_len = T.host.empty() ? 1 : T.host.rbegin()->first + 1;
  std::vector<int32_t> off((size_t)off_len, -1);
  std::vector<uint64_t> all;
  all.reserve(T.host.size() * (size_t)trials);
  for (const auto& kv : T.host) {
    off[(size_t)kv.first] = (int32_t)all.size();
    all.insert(all.end(), kv.second.begin(), kv.second.end());
  }
  if (all.size() > (size_t)INT32_MAX) return fail(KCMC_EUNSUPPORTED, "kcmc_ransac_prepare_samples: tables too large");
  if (all.empty()) all.push_back(~0ull);
  int prev = 0;
  hipGetDevice(&prev);
  KCMC_TRY(hip_check(hipSetDevice(ctx->device), "hipSetDevice"));
  free_model_tables(T);
  int rc = hip_check(hipMalloc(&T.dev, all.size() * sizeof(uint64_t)), "hipMalloc(model hyp)");
  if (rc == KCMC_OK) rc = hip_check(hipMalloc(&T.off, off.size() * sizeof(int32_t)), "hipMalloc(model hyp_off)");
  if (rc == KCMC_OK)
    rc = hip_check(hipMemcpy(T.dev, all.data(), all.size() * sizeof(uint64_t), hipMemcpyHostToDevice),
                   "hipMemcpy(model hyp)");
  if (rc == KCMC_OK)
    rc = hip_check(hipMemcpy(T.off, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice),
                   "hipMemcpy(model hyp_off)");
  hipSetDevice(prev);
  if (rc != KCMC_OK) {
    free_model_tables(T);
    T.host.clear();
    return rc;
  }
  T.off_len = off_len;
  return KCMC_OK;
}
