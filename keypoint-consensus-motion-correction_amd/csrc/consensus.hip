// The keypoint consensus of VA:224-286 on the device, in the three parts of
// hostalg.cpp (vote / merge / lookup): the per-frame parts run here, over the survivor
// bitmasks kcmc_match_frames leaves in HBM, so a step moves O(n_tpl) vote numbers to the
// host instead of every frame's bitmask, and a frame-sharded job exchanges only the votes.
//
//   vote:   Counter([x for s in kp_idxs_list for x in s]) (VA:239) = per template a count
//           and the position of its first occurrence: (frame, slot of the template in that
//           frame's CPython set table).  vote_count_kernel (atomics over frame chunks) +
//           vote_key_kernel (one workgroup: flags the first frames and writes the keys).
//   lookup: list(consensus_idxs.intersection(kp_idxs_list[i])) (VA:274) per frame:
//           lookup_count_kernel (counts + exclusive scan = CSR offsets, one workgroup) +
//           lookup_order_kernel (one wave per frame writes its list in set order).
//
// CPython set order: a set of non-negative ints (hash(k) == k) built by insertions only
// iterates in table-slot order.  When every key is below the final table size (which
// depends on the number of keys only) each key sits in its home slot and the order is
// ascending; otherwise the insertions are replayed exactly (DevPySet, the rules of
// Objects/setobject.c: 9 linear probes, then perturbed probing, resize at fill*5 >= mask*3
// to the smallest power of two > 4*used) in a per-thread scratch table.
#include <climits>

#include "kcmc_internal.h"

namespace kcmc {
namespace {

// Table size of a set after m insertions of distinct keys into an empty set (no deletions,
// so fill == used): resizes happen when used reaches ceil(3*mask/5).
__host__ __device__ inline uint32_t pyset_table_size(uint32_t m) {
  uint32_t mask = 7;
  while (true) {
    const uint32_t u = (3 * mask + 4) / 5;
    if (m < u) return mask + 1;
    const uint32_t minused = u > 50000 ? u * 2 : u * 4;
    uint32_t ns = 8;
    while (ns <= minused) ns <<= 1;
    mask = ns - 1;
  }
}

// CPython set insertions (set_add_entry / set_table_resize / set_insert_clean) on two
// caller-provided ping-pong tables of at least pyset_table_size(final size) entries.
struct DevPySet {
  int32_t* b0;
  int32_t* b1;
  int32_t* t;
  uint32_t mask, fill, used;

  __device__ void init(int32_t* a, int32_t* b) {
    b0 = a;
    b1 = b;
    t = a;
    mask = 7;
    fill = used = 0;
    for (int i = 0; i < 8; ++i) t[i] = -1;
  }
  __device__ void add(int32_t key) {
    uint32_t i = (uint32_t)key & mask;
    if (t[i] == -1) return store(i, key);
    uint64_t perturb = (uint64_t)key;
    while (true) {
      if (t[i] == key) return;
      if (i + 9 <= mask) {
        for (uint32_t j = 1; j <= 9; ++j) {
          const int32_t v = t[i + j];
          if (v == -1) return store(i + j, key);
          if (v == key) return;
        }
      }
      perturb >>= 5;
      i = (uint32_t)(((uint64_t)i * 5 + 1 + perturb) & mask);
      if (t[i] == -1) return store(i, key);
    }
  }

 private:
  __device__ void store(uint32_t slot, int32_t key) {
    t[slot] = key;
    ++fill;
    ++used;
    if (fill * 5 < mask * 3) return;
    const uint32_t minused = used > 50000 ? used * 2 : used * 4;
    uint32_t ns = 8;
    while (ns <= minused) ns <<= 1;
    int32_t* old = t;
    const uint32_t oldmask = mask;
    t = (t == b0) ? b1 : b0;
    for (uint32_t k = 0; k < ns; ++k) t[k] = -1;
    mask = ns - 1;
    fill = used;
    for (uint32_t k = 0; k <= oldmask; ++k)
      if (old[k] != -1) insert_clean(old[k]);
  }
  __device__ void insert_clean(int32_t key) {
    uint64_t perturb = (uint64_t)key;
    uint32_t i = (uint32_t)key & mask;
    while (true) {
      if (t[i] == -1) {
        t[i] = key;
        return;
      }
      if (i + 9 <= mask) {
        for (uint32_t j = 1; j <= 9; ++j)
          if (t[i + j] == -1) {
            t[i + j] = key;
            return;
          }
      }
      perturb >>= 5;
      i = (uint32_t)(((uint64_t)i * 5 + 1 + perturb) & mask);
    }
  }
};

constexpr int kVoteChunk = 64;    // frames per vote_count_kernel thread
constexpr int kVoteThreads = 256;
constexpr int kKeyThreads = 256;
constexpr int kEmuLanes = 64;     // vote_key_kernel replays of non-ascending first frames
constexpr int kCountThreads = 64;
constexpr uint32_t kOrderLdsCap = 2048;  // lookup_order_kernel keeps set tables up to this size in LDS

// lookup_order_kernel's set tables: R (the result, 2 cap words) in LDS when cap <= kOrderLdsCap,
// S (the frame's own set, 2 cap words) when cap <= kOrderLdsCap / 2; the tables that do not
// fit live in a per-frame global scratch of this many words
__host__ __device__ inline uint32_t lookup_scratch_words(uint32_t cap) {
  return (cap <= kOrderLdsCap ? 0u : 2u * cap) + (cap <= kOrderLdsCap / 2 ? 0u : 2u * cap);
}

// cnt[t] += frames of the chunk holding t; first_enc[t] = max(0x7fffffff - first frame):
// scratch in the key row of the output (zeroed before the launch).
__global__ __launch_bounds__(kVoteThreads) void vote_count_kernel(const uint32_t* __restrict__ keep, int F, int n_tpl,
                                                                  int W, int32_t* __restrict__ cnt,
                                                                  int32_t* __restrict__ first_enc) {
  const int t = blockIdx.x * kVoteThreads + threadIdx.x;
  if (t >= n_tpl) return;
  const int f0 = blockIdx.y * kVoteChunk, f1 = min(F, f0 + kVoteChunk);
  const uint32_t* p = keep + (size_t)f0 * W + (t >> 5);
  const int sh = t & 31;
  int c = 0, first = -1;
#pragma unroll 8
  for (int f = f0; f < f1; ++f, p += W) {
    const int on = (int)((*p >> sh) & 1u);
    c += on;
    first = (first < 0 && on) ? f : first;
  }
  if (c) {
    atomicAdd(&cnt[t], c);
    atomicMax(&first_enc[t], 0x7fffffff - first);
  }
}

// One workgroup: out row 0 = counts; row 1 = first-occurrence keys.  Frames that are some
// template's first frame are flagged; an ascending frame set gives slot = key, the others are
// replayed by the first kEmuLanes threads in their scratch tables.
__global__ __launch_bounds__(kKeyThreads) void vote_key_kernel(const uint32_t* __restrict__ keep, int F, int n_tpl,
                                                               int W, long long frame_base, long long* __restrict__ out,
                                                               int32_t* __restrict__ scratch, uint32_t emu_cap) {
  extern __shared__ uint32_t lds[];
  int32_t* first = reinterpret_cast<int32_t*>(lds);  // [n_tpl]
  int32_t* count = first + n_tpl;                    // [n_tpl]
  uint32_t* flag = reinterpret_cast<uint32_t*>(count + n_tpl);  // [ceil(F/32)]
  const int FW = (F + 31) / 32;
  int32_t* queue = reinterpret_cast<int32_t*>(flag + FW);  // [min(F, n_tpl)]
  __shared__ int qn;
  const int32_t* cnt = reinterpret_cast<const int32_t*>(out + n_tpl);
  const int32_t* first_enc = cnt + n_tpl;
  for (int i = threadIdx.x; i < FW; i += kKeyThreads) flag[i] = 0u;
  if (threadIdx.x == 0) qn = 0;
  __syncthreads();
  for (int t = threadIdx.x; t < n_tpl; t += kKeyThreads) {
    const int32_t e = first_enc[t];
    const int f = e ? 0x7fffffff - e : -1;
    first[t] = f;
    count[t] = cnt[t];
    if (f >= 0) atomicOr(&flag[f >> 5], 1u << (f & 31));
  }
  // every count / first frame is in LDS before the key row (which held them) is overwritten
  __syncthreads();
  for (int t = threadIdx.x; t < n_tpl; t += kKeyThreads) {
    out[t] = count[t];
    out[n_tpl + t] = INT64_MAX;
  }
  // first frames whose set iterates in ascending order (slot = key) are marked in `flag`
  // again (bit cleared = ascending), the others queued for a replay
  for (int f = threadIdx.x; f < F; f += kKeyThreads) {
    if (!((flag[f >> 5] >> (f & 31)) & 1u)) continue;
    const uint32_t* row = keep + (size_t)f * W;
    uint32_t flen = 0;
    int top = -1;
    for (int w = 0; w < W; ++w) {
      const uint32_t v = row[w];
      flen += __popc(v);
      if (v) top = 32 * w + 31 - __clz(v);
    }
    if ((uint32_t)top >= pyset_table_size(flen)) queue[atomicAdd(&qn, 1)] = f;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < qn; q += kKeyThreads) {
    const int f = queue[q];
    atomicAnd(&flag[f >> 5], ~(1u << (f & 31)));
  }
  __syncthreads();
  for (int t = threadIdx.x; t < n_tpl; t += kKeyThreads) {
    const int f = first[t];
    if (f >= 0 && ((flag[f >> 5] >> (f & 31)) & 1u)) out[n_tpl + t] = ((frame_base + f) << 32) | t;
  }
  if (threadIdx.x < kEmuLanes) {
    int32_t* sc = scratch + (size_t)threadIdx.x * 2 * emu_cap;
    for (int q = threadIdx.x; q < qn; q += kEmuLanes) {
      const int f = queue[q];
      const uint32_t* row = keep + (size_t)f * W;
      DevPySet s;
      s.init(sc, sc + emu_cap);
      for (int w = 0; w < W; ++w)
        for (uint32_t b = row[w]; b; b &= b - 1) s.add(32 * w + __ffs(b) - 1);
      const long long base = (frame_base + f) << 32;
      for (uint32_t slot = 0; slot <= s.mask; ++slot) {
        const int32_t key = s.t[slot];
        if (key >= 0 && first[key] == f) out[n_tpl + key] = base | (long long)slot;
      }
    }
  }
}

// Per-frame counts |consensus & frame| into pt_off[f + 1] (one thread per frame).
__global__ __launch_bounds__(kCountThreads) void lookup_count_kernel(const uint32_t* __restrict__ keep, int F, int W,
                                                                     const uint32_t* __restrict__ cons_bits,
                                                                     int32_t* __restrict__ pt_off) {
  const int f = blockIdx.x * kCountThreads + threadIdx.x;
  if (f >= F) return;
  const uint32_t* row = keep + (size_t)f * W;
  int m = 0;
  for (int w = 0; w < W; ++w) m += __popc(row[w] & cons_bits[w]);
  pt_off[f + 1] = m;
}

// In-place inclusive scan of pt_off[1..F], pt_off[0] = 0: CSR offsets.  ONE wave: the
// lookup runs beside the warp, whose tiles fill every CU; a single-wave workgroup gets a
// slot as soon as one tile retires, a 1024-thread one waited ~0.43 ms for 16 free slots on
// one CU (c3 trace).
__global__ __launch_bounds__(64) void lookup_scan_kernel(int F, int32_t* __restrict__ pt_off) {
  // 1024 frames per pass, 16 consecutive ones per lane: the 16 loads of a lane are in
  // flight together (a pass per 64 frames waited on one load at a time: ~40 us at F = 2500)
  constexpr int kPer = 16;
  const int lane = threadIdx.x;
  if (lane == 0) pt_off[0] = 0;
  int32_t* c = pt_off + 1;
  int carry = 0;
  for (int base = 0; base < F; base += 64 * kPer) {
    const int f0 = base + lane * kPer;
    int v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) v[k] = f0 + k < F ? c[f0 + k] : 0;
#pragma unroll
    for (int k = 1; k < kPer; ++k) v[k] += v[k - 1];
    int x = v[kPer - 1];  // inclusive prefix of the lane totals
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    const int before = carry + x - v[kPer - 1];
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (f0 + k < F) c[f0 + k] = before + v[k];
    carry += __shfl(x, 63, 64);
  }
}

__device__ __forceinline__ int wave_sum(int x) {
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return x;
}
__device__ __forceinline__ int wave_max(int x) {
  for (int d = 32; d >= 1; d >>= 1) x = max(x, __shfl_xor(x, d, 64));
  return x;
}

// One wave per frame: its consensus points in CPython set-iteration order at pt_off[f].
// Ascending results (every key below the final table size) are written by the whole wave
// (lane = bitmask word, wave prefix sums).  The others are replayed by lane 0 in set tables
// in LDS (global scratch when they do not fit), fed from a list of keys the whole wave
// stages in LDS in insertion order first: the serial part then touches only LDS (round 3:
// the replay loop's own global loads, two per consensus key, were most of the kernel's
// time -- c2 lookup 51.6 us).  The insertion order is set_intersection's (VA:274): the
// consensus in its own iteration order when the frame's set is larger, else the frame's
// set in its table order (ascending, or replayed first when its keys exceed its table).
__device__ __forceinline__ int wave_compact(bool take, int32_t key, int32_t* dst, int n, uint64_t below) {
  const uint64_t hit = __ballot(take);
  if (take) dst[n + __popcll(hit & below)] = key;
  return n + __popcll(hit);
}

__global__ __launch_bounds__(64) void lookup_order_kernel(
    const uint32_t* __restrict__ keep, int F, int W, const int32_t* __restrict__ cons_iter, int nc,
    const uint32_t* __restrict__ cons_bits, const int32_t* __restrict__ pt_off, int32_t* __restrict__ pt_idx,
    int32_t* __restrict__ scratch, uint32_t cap, int r_lds, int s_lds) {
  // LDS: [W] frame words, [W] consensus words, [nc] staged keys, then the R tables
  // [2 cap] when r_lds and the S tables [2 cap] when s_lds
  extern __shared__ uint32_t lds[];
  uint32_t* rowS = lds;
  uint32_t* consS = rowS + W;
  int32_t* keyS = reinterpret_cast<int32_t*>(lds + 2 * W);
  int32_t* tabS = keyS + nc;
  const int f = blockIdx.x;
  const int lane = threadIdx.x;
  const int o = pt_off[f];
  const int m = pt_off[f + 1] - o;
  if (m == 0) return;
  const uint32_t* row = keep + (size_t)f * W;
  int flen = 0, fmax = -1, top = -1;
  for (int w = lane; w < W; w += 64) {
    const uint32_t v = row[w], cb = cons_bits[w];
    rowS[w] = v;
    consS[w] = cb;
    flen += __popc(v);
    if (v) fmax = 32 * w + 31 - __clz(v);
    const uint32_t h = v & cb;
    if (h) top = 32 * w + 31 - __clz(h);
  }
  flen = wave_sum(flen);
  fmax = wave_max(fmax);
  top = wave_max(top);
  __syncthreads();  // one wave: the staged words are visible to every lane
  int32_t* out = pt_idx + o;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  // the bits of rowS & mask in ascending key order, compacted into dst (returns the count)
  auto stage_bits = [&](const uint32_t* mask, int32_t* dst) {
    int n = 0;
    for (int w0 = 0; w0 < W; w0 += 64) {
      const int w = w0 + lane;
      uint32_t h = w < W ? rowS[w] & (mask ? mask[w] : ~0u) : 0u;
      const int c = __popc(h);
      int x = c;  // inclusive prefix over the lanes
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      int k = n + x - c;
      for (; h; h &= h - 1) dst[k++] = 32 * w + __ffs(h) - 1;
      n += __shfl(x, 63, 64);
    }
    return n;
  };
  if ((uint32_t)top < pyset_table_size((uint32_t)m)) {  // every key in its home slot: ascending
    stage_bits(consS, out);
    return;
  }
  int32_t* fscr = scratch + (size_t)f * lookup_scratch_words(cap);  // r_lds / s_lds follow the same rule
  int32_t* R0 = r_lds ? tabS : fscr;
  int32_t* R1 = R0 + cap;
  int32_t* S0 = s_lds ? tabS + 2 * cap : fscr + (r_lds ? 0 : 2 * cap);
  // ---- the result's keys in insertion order -> keyS[0, m)
  if ((uint32_t)flen > (uint32_t)nc) {  // set_intersection iterates the smaller set: the consensus
    int n = 0;
    for (int k0 = 0; k0 < nc; k0 += 64) {
      const int k = k0 + lane;
      const int32_t key = k < nc ? cons_iter[k] : 0;
      n = wave_compact(k < nc && ((rowS[key >> 5] >> (key & 31)) & 1u), key, keyS, n, below);
    }
  } else if ((uint32_t)fmax < pyset_table_size((uint32_t)flen)) {  // the frame's set, ascending
    stage_bits(consS, keyS);
  } else {  // the frame's set in its own table order: replay it, then read its slots
    int32_t* fk = keyS;  // the frame's keys ascending (flen <= nc entries), then reused
    stage_bits(nullptr, fk);
    __syncthreads();
    uint32_t smask = 0;
    int ssel = 0;
    if (lane == 0) {
      DevPySet S;
      S.init(S0, S0 + cap);
      for (int i = 0; i < flen; ++i) S.add(fk[i]);
      smask = S.mask;
      ssel = S.t != S0;
    }
    __syncthreads();
    smask = __shfl(smask, 0, 64);
    ssel = __shfl(ssel, 0, 64);
    const int32_t* T = ssel ? S0 + cap : S0;
    int n = 0;
    for (uint32_t s0 = 0; s0 <= smask; s0 += 64) {
      const uint32_t slot = s0 + lane;
      const int32_t key = slot <= smask ? T[slot] : -1;
      n = wave_compact(key >= 0 && ((consS[key >> 5] >> (key & 31)) & 1u), key, keyS, n, below);
    }
  }
  __syncthreads();
  uint32_t rmask = 0;
  int rsel = 0;
  if (lane == 0) {
    DevPySet R;
    R.init(R0, R1);
    for (int i = 0; i < m; ++i) R.add(keyS[i]);
    rmask = R.mask;
    rsel = R.t == R1;
  }
  __syncthreads();  // one wave: lane 0's table writes are visible to every lane
  rmask = __shfl(rmask, 0, 64);
  rsel = __shfl(rsel, 0, 64);
  const int32_t* T = rsel ? R1 : R0;
  int n = 0;
  for (uint32_t s0 = 0; s0 <= rmask; s0 += 64) {
    const uint32_t slot = s0 + lane;
    const int32_t key = slot <= rmask ? T[slot] : -1;
    n = wave_compact(key >= 0, key, out, n, below);
  }
}

// First / last frame without NaN among params [F, E] and their parameters.
constexpr int kBoundThreads = 256;
__global__ __launch_bounds__(kBoundThreads) void params_boundary_kernel(const double* __restrict__ params, int F, int E,
                                                                        double* __restrict__ out) {
  __shared__ int lo, hi;
  if (threadIdx.x == 0) {
    lo = INT_MAX;
    hi = -1;
  }
  __syncthreads();
  int my_lo = INT_MAX, my_hi = -1;
  for (int f = threadIdx.x; f < F; f += kBoundThreads) {
    bool ok = true;
    for (int e = 0; e < E; ++e) ok = ok && !isnan(params[(size_t)f * E + e]);
    if (ok) {
      my_lo = min(my_lo, f);
      my_hi = max(my_hi, f);
    }
  }
  if (my_hi >= 0) {
    atomicMin(&lo, my_lo);
    atomicMax(&hi, my_hi);
  }
  __syncthreads();
  const bool any = hi >= 0;
  if (threadIdx.x == 0) {
    out[0] = any ? (double)lo : -1.0;
    out[1] = any ? (double)hi : -1.0;
  }
  for (int e = threadIdx.x; e < 2 * E; e += kBoundThreads) {
    const int f = e < E ? lo : hi;
    out[2 + e] = any ? params[(size_t)f * E + (e % E)] : __builtin_nan("");
  }
}

}  // namespace
}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_consensus_vote(kcmc_ctx* ctx, const uint32_t* keep_bits, int n_frames, int n_tpl,
                                   long long frame_base, int64_t* out_votes, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_consensus_vote: ctx is NULL");
  if (n_frames < 0 || n_tpl < 0 || frame_base < 0 || frame_base + (long long)n_frames > (long long)INT32_MAX)
    return fail(KCMC_EINVAL, "kcmc_consensus_vote: bad sizes");
  if (n_tpl == 0) return KCMC_OK;
  if (!out_votes || (n_frames > 0 && !keep_bits)) return fail(KCMC_EINVAL, "kcmc_consensus_vote: NULL pointer");
  const int W = (n_tpl + 31) / 32;
  const size_t lds = (size_t)n_tpl * 8 + (size_t)((n_frames + 31) / 32) * 4 + (size_t)std::min(n_frames, n_tpl) * 4;
  if (lds > 150 * 1024) return fail(KCMC_EUNSUPPORTED, "kcmc_consensus_vote: too many frames / templates for one launch");
  hipStream_t s = (hipStream_t)stream;
  int32_t* cnt = reinterpret_cast<int32_t*>(out_votes + n_tpl);
  KCMC_TRY(hip_check(hipMemsetAsync(cnt, 0, (size_t)n_tpl * sizeof(int64_t), s), "hipMemsetAsync(votes)"));
  if (n_frames > 0) {
    hipLaunchKernelGGL(vote_count_kernel, dim3(ceil_div(n_tpl, kVoteThreads), ceil_div(n_frames, kVoteChunk)),
                       dim3(kVoteThreads), 0, s, keep_bits, n_frames, n_tpl, W, cnt, cnt + n_tpl);
    KCMC_TRY(launch_check("vote_count_kernel"));
  }
  const uint32_t emu_cap = pyset_table_size((uint32_t)n_tpl);
  const size_t sbytes = (size_t)kEmuLanes * 2 * emu_cap * sizeof(int32_t);
  void* scratch = nullptr;
  KCMC_TRY(workspace_alloc(ctx, &scratch, sbytes, s));
  hipLaunchKernelGGL(vote_key_kernel, dim3(1), dim3(kKeyThreads), lds, s, keep_bits, n_frames, n_tpl, W, frame_base,
                     reinterpret_cast<long long*>(out_votes), reinterpret_cast<int32_t*>(scratch), emu_cap);
  const int rc = launch_check("vote_key_kernel");
  KCMC_TRY(workspace_free(ctx, scratch, s, sbytes));
  return rc;
}

extern "C" long long kcmc_consensus_lookup_scratch_bytes(int n_frames, int nc) {
  if (n_frames < 0 || nc < 0) return -1;
  return (long long)n_frames * (long long)lookup_scratch_words(pyset_table_size((uint32_t)nc)) *
         (long long)sizeof(int32_t);
}

namespace kcmc {
namespace {
// the lookup with the consensus size nc, the bitmask at cons_pack + nc
int launch_lookup(const uint32_t* keep_bits, int n_frames, int n_tpl, const int32_t* cons_pack, int nc,
                  int32_t* out_pt_off, int32_t* out_pt_idx, void* scratch, hipStream_t s) {
  if (n_frames == 0) return hip_check(hipMemsetAsync(out_pt_off, 0, sizeof(int32_t), s), "hipMemsetAsync(pt_off)");
  if (nc == 0 || n_tpl == 0)
    return hip_check(hipMemsetAsync(out_pt_off, 0, (size_t)(n_frames + 1) * sizeof(int32_t), s),
                     "hipMemsetAsync(pt_off)");
  const uint32_t cap = pyset_table_size((uint32_t)nc);
  if (!keep_bits || !cons_pack || !out_pt_idx || (!scratch && lookup_scratch_words(cap) > 0))
    return fail(KCMC_EINVAL, "kcmc_consensus_lookup: NULL pointer");
  const int W = (n_tpl + 31) / 32;
  const uint32_t* cons_bits = reinterpret_cast<const uint32_t*>(cons_pack + nc);
  hipLaunchKernelGGL(lookup_count_kernel, dim3(ceil_div(n_frames, kCountThreads)), dim3(kCountThreads), 0, s, keep_bits,
                     n_frames, W, cons_bits, out_pt_off);
  KCMC_TRY(launch_check("lookup_count_kernel"));
  hipLaunchKernelGGL(lookup_scan_kernel, dim3(1), dim3(64), 0, s, n_frames, out_pt_off);
  KCMC_TRY(launch_check("lookup_scan_kernel"));
  const int r_lds = cap <= kOrderLdsCap, s_lds = cap <= kOrderLdsCap / 2;
  const size_t lds = ((size_t)2 * W + nc + (r_lds ? 2 * cap : 0) + (s_lds ? 2 * cap : 0)) * sizeof(int32_t);
  hipLaunchKernelGGL(lookup_order_kernel, dim3(n_frames), dim3(64), lds, s, keep_bits, n_frames, W, cons_pack, nc,
                     cons_bits, out_pt_off, out_pt_idx, reinterpret_cast<int32_t*>(scratch), cap, r_lds, s_lds);
  return launch_check("lookup_order_kernel");
}
}  // namespace
}  // namespace kcmc

extern "C" int kcmc_consensus_lookup(kcmc_ctx* ctx, const uint32_t* keep_bits, int n_frames, int n_tpl,
                                     const int32_t* cons_pack, int nc, int32_t* out_pt_off, int32_t* out_pt_idx,
                                     void* scratch, kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_consensus_lookup: ctx is NULL");
  if (n_frames < 0 || n_tpl < 0 || nc < 0 || nc > n_tpl) return fail(KCMC_EINVAL, "kcmc_consensus_lookup: bad sizes");
  if (!out_pt_off) return fail(KCMC_EINVAL, "kcmc_consensus_lookup: NULL pointer");
  return launch_lookup(keep_bits, n_frames, n_tpl, cons_pack, nc, out_pt_off, out_pt_idx, scratch, (hipStream_t)stream);
}

extern "C" int kcmc_params_boundary(kcmc_ctx* ctx, const double* params, int n_frames, int E, double* out,
                                    kcmc_stream_t stream) {
  if (!ctx) return fail(KCMC_EINVAL, "kcmc_params_boundary: ctx is NULL");
  if (n_frames < 0 || E < 1 || !out || (n_frames > 0 && !params))
    return fail(KCMC_EINVAL, "kcmc_params_boundary: bad arguments");
  hipLaunchKernelGGL(params_boundary_kernel, dim3(1), dim3(kBoundThreads), 0, (hipStream_t)stream, params, n_frames, E,
                     out);
  return launch_check("params_boundary_kernel");
}
