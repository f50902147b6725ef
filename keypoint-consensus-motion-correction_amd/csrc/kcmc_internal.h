// Internal helpers shared by the kcmc translation units (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kcmc.h"


// Hypothesis tables of the min_samples-point models (3: affine, 4: projective): per
// point count n, `trials` samples packed as four 16-bit indices in a u64 (unused slots
// 0xffff).  dev = all tables back to back, off[n] = start of n's table or -1.
struct HypTables {
  std::map<int, std::vector<uint64_t>> host;
  uint64_t* dev = nullptr;
  int32_t* off = nullptr;
  int off_len = 0;
  int trials = 0;
  uint32_t seed = 0;
};

struct kcmc_ctx {
  int device = 0;
  HypTables mhyp[5];  // indexed by min_samples (3 and 4 used)
  // RANSAC hypothesis tables, built on demand per point count n: `hyp_trials` packed
  // (i | j << 16) u32 samples per n.  Device: hyp (all tables back to back) and
  // hyp_off[n] = start of n's table in hyp, or -1 (n in [0, hyp_off_len)).
  std::map<int, std::vector<uint32_t>> hyp_host;
  uint32_t* hyp = nullptr;
  int32_t* hyp_off = nullptr;
  int hyp_off_len = 0;
  int hyp_trials = 0;
  uint32_t hyp_seed = 0;
  // Stream-ordered scratch (per-call workspaces, e.g. the warp's tile plans): a private
  // memory pool that keeps its pages between calls.
  hipMemPool_t ws_pool = nullptr;
  // One cached workspace per stream, reused by the next call on that stream without
  // touching the pool (stream order makes the reuse safe; a pool allocation while the
  // previous warp still runs blocked the host for the rest of that warp).  Assumes a
  // stream handle names one stream for the context's lifetime (torch's pooled streams);
  // never used for hipStreamPerThread or a capturing stream (capi.cpp cacheable_stream).
  struct StreamScratch {
    void* ptr = nullptr;
    size_t bytes = 0;
    bool busy = false;
  };
  std::map<hipStream_t, StreamScratch> stream_ws;
  std::mutex ws_mutex;
};

namespace kcmc {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
// Check a HIP call / the last launch; on failure record the message and return KCMC_EHIP.
int hip_check(hipError_t e, const char* what);
int launch_check(const char* what);

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// CU count of the calling thread's current HIP device (cached per device id; match.hip).
int device_cus();

// XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (speed only, never
// relied on for correctness), so give each XCD a contiguous run of ids (bijective also
// when n % 8 != 0): neighbouring tiles that share input then share one XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int q8 = n >> 3, r8 = n & 7, xcd = bid & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// Stream-ordered workspace from the context's pool (valid for work enqueued on `s`
// until workspace_free, which is itself stream-ordered).
int workspace_alloc(kcmc_ctx* ctx, void** p, size_t bytes, hipStream_t s);
// bytes > 0: the block may be kept as the stream's cached workspace (see kcmc_ctx).
int workspace_free(kcmc_ctx* ctx, void* p, hipStream_t s, size_t bytes = 0);

// VA:196-214 per frame on knn output (match.hip): reorder, ratio and displacement
// filters, survivor bitmask, log counts.  Shared by the uint8 and float32 matchers.
int launch_match_filter(const int32_t* idx, const float* dist, const double* kp_tpl, const double* kp_q,
                        const int32_t* q_off, int n_frames, int n_tpl, double ratio, double d_lo, double d_hi,
                        double* kp_ordered, uint32_t* keep_bits, int32_t* counts, hipStream_t s);

}  // namespace kcmc

#define KCMC_TRY(expr)            \
  do {                            \
    int _rc = (expr);             \
    if (_rc != KCMC_OK) return _rc; \
  } while (0)
