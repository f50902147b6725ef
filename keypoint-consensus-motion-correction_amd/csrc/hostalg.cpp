// Host-side algorithms of the hot path that have to reproduce CPython / numpy
// behaviour bit for bit:
//   * the legacy numpy MT19937 sample stream skimage 0.18.3's ransac consumes
//     (RandomState(seed).choice(n, k, replace=False) == permutation(n)[:k]);
//   * the keypoint consensus of VA:224-286, whose RANSAC point order is the
//     iteration order of CPython `set` objects (VA:214, VA:248, VA:274) and whose
//     selection is Counter.most_common (stable by first occurrence).
#include <algorithm>
#include <array>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "kcmc_internal.h"

namespace kcmc {

// ------------------------------------------------------------------ MT19937
namespace {
struct MT19937 {
  uint32_t key[624];
  int pos;
  explicit MT19937(uint32_t seed) {  // numpy mt19937_seed == init_genrand
    for (int i = 0; i < 624; ++i) {
      key[i] = seed;
      seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
    }
    pos = 624;
  }
  void regen() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int i = 0;
    for (; i < 624 - 397; ++i) {
      uint32_t y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
      key[i] = key[i + 397] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; i < 623; ++i) {
      uint32_t y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
      key[i] = key[i + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    uint32_t y = (key[623] & 0x80000000u) | (key[0] & 0x7fffffffu);
    key[623] = key[396] ^ (y >> 1) ^ mag01[y & 1u];
    pos = 0;
  }
  uint32_t next32() {
    if (pos == 624) regen();
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // numpy legacy random_interval(max): rejection on the smallest enclosing mask.
  uint32_t interval(uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > max) {
    }
    return v;
  }
};
}  // namespace

int hypothesis_table_impl(int n, int trials, uint32_t seed, int min_samples, int32_t* out) {
  if (n < 1 || trials < 0 || min_samples < 1 || min_samples > n || !out)
    return fail(KCMC_EINVAL, "kcmc_hypothesis_table: need 1 <= min_samples <= n, trials >= 0");
  MT19937 rng(seed);
  std::vector<int32_t> perm((size_t)n);
  for (int t = 0; t < trials; ++t) {
    std::iota(perm.begin(), perm.end(), 0);
    for (int i = n - 1; i > 0; --i) {  // RandomState.shuffle (_shuffle_raw)
      uint32_t j = rng.interval((uint32_t)i);
      std::swap(perm[(size_t)i], perm[j]);
    }
    for (int k = 0; k < min_samples; ++k) out[(size_t)t * min_samples + k] = perm[(size_t)k];
  }
  return KCMC_OK;
}

// ------------------------------------------------------- CPython set emulation
namespace {
// A set of non-negative Python ints (hash(k) == k) built by insertions only, as
// Objects/setobject.c does it: open addressing, LINEAR_PROBES = 9 then perturbed
// probing (PERTURB_SHIFT = 5), resize when fill*5 >= mask*3 to the smallest power
// of two > used*4 (used*2 above 50000).  Iteration order == table slot order.
class PySet {
 public:
  static constexpr int64_t kEmpty = -1;
  PySet() : table_(8, kEmpty), mask_(7), fill_(0), used_(0) {}

  size_t size() const { return used_; }

  // Table sizes after m = 0..max_m insertions of distinct keys into an empty set (no
  // deletions): the same fill/resize rule as store().
  static std::vector<size_t> table_sizes(size_t max_m) {
    std::vector<size_t> out(max_m + 1);
    size_t mask = 7, fill = 0;
    out[0] = 8;
    for (size_t used = 1; used <= max_m; ++used) {
      ++fill;
      if (fill * 5 >= mask * 3) {
        const size_t minused = used > 50000 ? used * 2 : used * 4;
        size_t newsize = 8;
        while (newsize <= minused) newsize <<= 1;
        mask = newsize - 1;
        fill = used;
      }
      out[used] = mask + 1;
    }
    return out;
  }

  void add(int64_t key) {
    size_t mask = mask_;
    size_t i = (size_t)key & mask;
    if (table_[i] == kEmpty) return store(i, key);
    size_t perturb = (size_t)key;
    while (true) {
      if (table_[i] == key) return;
      if (i + kLinearProbes <= mask) {
        for (size_t j = 1; j <= kLinearProbes; ++j) {
          if (table_[i + j] == kEmpty) return store(i + j, key);
          if (table_[i + j] == key) return;
        }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
      if (table_[i] == kEmpty) return store(i, key);
    }
  }

  bool contains(int64_t key) const {
    size_t mask = mask_;
    size_t i = (size_t)key & mask;
    size_t perturb = (size_t)key;
    while (true) {
      if (table_[i] == kEmpty) return false;
      if (table_[i] == key) return true;
      if (i + kLinearProbes <= mask) {
        for (size_t j = 1; j <= kLinearProbes; ++j) {
          if (table_[i + j] == kEmpty) return false;
          if (table_[i + j] == key) return true;
        }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }

  template <class F>
  void for_each(F&& f) const {
    for (int64_t k : table_)
      if (k != kEmpty) f(k);
  }
  // f(key, slot) in iteration (= slot) order
  template <class F>
  void for_each_slot(F&& f) const {
    for (size_t s = 0; s < table_.size(); ++s)
      if (table_[s] != kEmpty) f(table_[s], s);
  }

 private:
  static constexpr size_t kLinearProbes = 9;
  static constexpr int kPerturbShift = 5;

  void store(size_t slot, int64_t key) {
    table_[slot] = key;
    ++fill_;
    ++used_;
    if (fill_ * 5 < mask_ * 3) return;
    resize(used_ > 50000 ? used_ * 2 : used_ * 4);
  }

  void resize(size_t minused) {
    size_t newsize = 8;
    while (newsize <= minused) newsize <<= 1;
    std::vector<int64_t> old;
    old.swap(table_);
    table_.assign(newsize, kEmpty);
    mask_ = newsize - 1;
    fill_ = used_;
    for (int64_t k : old)
      if (k != kEmpty) insert_clean(k);
  }

  void insert_clean(int64_t key) {
    size_t mask = mask_;
    size_t perturb = (size_t)key;
    size_t i = (size_t)key & mask;
    while (true) {
      if (table_[i] == kEmpty) {
        table_[i] = key;
        return;
      }
      if (i + kLinearProbes <= mask) {
        for (size_t j = 1; j <= kLinearProbes; ++j)
          if (table_[i + j] == kEmpty) {
            table_[i + j] = key;
            return;
          }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }

  std::vector<int64_t> table_;
  size_t mask_, fill_, used_;
};

// PySet's insertion/resize/probe rules on two fixed buffers (no allocation): the replay
// of a per-frame intersection result, whose final table has at most kMax slots.
class SmallPySet {
 public:
  static constexpr size_t kMax = 2048;  // holds up to 1228 keys (next resize at fill 1229)
  SmallPySet() : t_(a_), mask_(7), fill_(0), used_(0) {
    for (size_t i = 0; i < 8; ++i) t_[i] = kEmpty;
  }
  void add(int32_t key) {
    size_t mask = mask_;
    size_t i = (size_t)key & mask;
    if (t_[i] == kEmpty) return store(i, key);
    size_t perturb = (size_t)key;
    while (true) {
      if (t_[i] == key) return;
      if (i + kLinearProbes <= mask) {
        for (size_t j = 1; j <= kLinearProbes; ++j) {
          if (t_[i + j] == kEmpty) return store(i + j, key);
          if (t_[i + j] == key) return;
        }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
      if (t_[i] == kEmpty) return store(i, key);
    }
  }
  template <class F>
  void for_each(F&& f) const {
    for (size_t i = 0; i <= mask_; ++i)
      if (t_[i] != kEmpty) f(t_[i]);
  }

 private:
  static constexpr int32_t kEmpty = -1;
  static constexpr size_t kLinearProbes = 9;
  static constexpr int kPerturbShift = 5;
  void store(size_t slot, int32_t key) {
    t_[slot] = key;
    ++fill_;
    ++used_;
    if (fill_ * 5 < mask_ * 3) return;
    size_t newsize = 8;
    const size_t minused = used_ > 50000 ? used_ * 2 : used_ * 4;
    while (newsize <= minused) newsize <<= 1;
    int32_t* old = t_;
    const size_t oldmask = mask_;
    t_ = (t_ == a_) ? b_ : a_;
    for (size_t i = 0; i < newsize; ++i) t_[i] = kEmpty;
    mask_ = newsize - 1;
    fill_ = used_;
    for (size_t i = 0; i <= oldmask; ++i)
      if (old[i] != kEmpty) insert_clean(old[i]);
  }
  void insert_clean(int32_t key) {
    size_t mask = mask_;
    size_t perturb = (size_t)key;
    size_t i = (size_t)key & mask;
    while (true) {
      if (t_[i] == kEmpty) {
        t_[i] = key;
        return;
      }
      if (i + kLinearProbes <= mask) {
        for (size_t j = 1; j <= kLinearProbes; ++j)
          if (t_[i + j] == kEmpty) {
            t_[i + j] = key;
            return;
          }
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }
  int32_t* t_;
  size_t mask_, fill_, used_;
  int32_t a_[kMax], b_[kMax];
};

// Persistent workers for the per-step host loops (the consensus replays and vote counts
// run every step, and spawning 8-16 threads per call costs a few hundred microseconds).
// run(tasks, fn) calls fn(0..tasks-1) on the workers and the calling thread and returns
// when all have finished; concurrent callers are serialised.
class WorkerPool {
 public:
  explicit WorkerPool(int n_workers) : pid_(getpid()) {
    for (int i = 0; i < n_workers; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)workers_.size() + 1; }
  pid_t pid() const { return pid_; }
  void run(int tasks, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> caller(run_m_);
    {
      std::lock_guard<std::mutex> lk(m_);
      job_.store(&fn, std::memory_order_relaxed);
      n_tasks_.store(tasks, std::memory_order_relaxed);
      pending_.store(tasks, std::memory_order_relaxed);
      next_.store(0, std::memory_order_release);
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return pending_.load(std::memory_order_acquire) == 0; });
    next_.store(INT_MAX / 2, std::memory_order_relaxed);
  }

 private:
  void work() {
    while (true) {
      const int t = next_.fetch_add(1, std::memory_order_acq_rel);
      if (t >= n_tasks_.load(std::memory_order_relaxed)) return;
      (*job_.load(std::memory_order_relaxed))(t);
      if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> lk(m_);
        done_cv_.notify_all();
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  std::atomic<const std::function<void(int)>*> job_{nullptr};
  std::atomic<int> n_tasks_{0};
  std::atomic<int> next_{INT_MAX / 2}, pending_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
  pid_t pid_;
};

WorkerPool& worker_pool() {
  static std::mutex m;
  static WorkerPool* pool = nullptr;
  std::lock_guard<std::mutex> lk(m);
  if (!pool || pool->pid() != getpid()) {  // a forked child has none of the parent's threads
    unsigned hw = std::thread::hardware_concurrency();
    pool = new WorkerPool((int)std::min<unsigned>(hw ? hw : 1, 16) - 1);  // never joined: lives with the process
  }
  return *pool;
}

// f(i) for i in [0, n) in contiguous blocks, one per pool thread (no false sharing between
// the blocks' per-index outputs)
template <class F>
void parallel_for(int n, F&& f) {
  if (n < 64) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  WorkerPool& pool = worker_pool();
  const int nt = std::min(pool.size(), n / 32);
  if (nt <= 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  pool.run(nt, [&](int t) {
    const int b = (int)((long long)n * t / nt), e = (int)((long long)n * (t + 1) / nt);
    for (int i = b; i < e; ++i) f(i);
  });
}
}  // namespace

}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_hypothesis_table(int n, int trials, uint32_t seed, int min_samples, int32_t* out_host) {
  return hypothesis_table_impl(n, trials, seed, min_samples, out_host);
}

// ------------------------------------------------------------- consensus, in three parts
// The consensus of VA:224-286 split so that a frame-sharded job exchanges O(n_tpl) data per
// rank instead of every frame's bitmask:
//   vote   (per rank, over its own frames)  Counter counts + each template's first occurrence
//   merge  (every rank, O(world * n_tpl))   Counter.most_common + set(consensus) iteration order
//   lookup (per rank, over its own frames)  list(consensus & frame_set) per frame (VA:274)
// The device kernels (consensus.hip) compute vote and lookup with the same definitions.
namespace kcmc {

// kp_idxs = set([m.queryIdx for m in distance_matches]) (VA:214): insertions in ascending
// template order.
static PySet frame_set_of(const uint32_t* w, int words) {
  PySet s;
  for (int k = 0; k < words; ++k)
    for (uint32_t b = w[k]; b; b &= b - 1) s.add(32 * k + __builtin_ctz(b));
  return s;
}

// votes [2][n_tpl]: row 0 = Counter count of every template over frames [0, n_frames); row 1
// = its first-occurrence key (frame_base + f) << 32 | slot: f the first frame whose set holds
// it, slot its position in that set's table (iteration order = slot order), INT64_MAX if no
// frame holds it.  Counter([x for s in kp_idxs_list for x in s]) (VA:239) inserts keys in
// exactly the order of these keys, so merging ranks = summing counts + taking the min key.
int vote_impl(const uint32_t* keep_bits, int n_frames, int n_tpl, int64_t frame_base, int64_t* out) {
  const int words = (n_tpl + 31) / 32;
  auto frame_bits = [&](int f) { return keep_bits + (size_t)f * words; };
  // Vertical counting in byte lanes: spread[byte] holds the byte's 8 bits as 8 bytes of
  // 0/1, so one 64-bit add counts 8 template indices; flushed every 255 frames.
  static const std::array<uint64_t, 256> spread = [] {
    std::array<uint64_t, 256> t{};
    for (int v = 0; v < 256; ++v)
      for (int b = 0; b < 8; ++b) t[(size_t)v] |= (uint64_t)((v >> b) & 1) << (8 * b);
    return t;
  }();
  std::vector<int32_t> count((size_t)words * 32, 0);
  std::vector<uint32_t> seen((size_t)words, 0u), any((size_t)words, 0u);
  // frames [fb, fe) into cnt / anym; integer sums, so splitting the frames over threads is exact
  auto vote = [&](int fb, int fe, int32_t* cnt, uint32_t* anym) {
    std::vector<uint64_t> acc((size_t)words * 4, 0);
    auto flush = [&] {
      for (size_t q = 0; q < acc.size(); ++q) {
        for (int b = 0; b < 8; ++b) cnt[8 * q + (size_t)b] += (int32_t)((acc[q] >> (8 * b)) & 0xff);
        acc[q] = 0;
      }
    };
    for (int f = fb; f < fe; ++f) {
      const uint32_t* w = frame_bits(f);
      for (int k = 0; k < words; ++k) {
        const uint32_t wk = w[k];
        anym[k] |= wk;
        uint64_t* a = acc.data() + 4 * (size_t)k;
        a[0] += spread[wk & 0xff];
        a[1] += spread[(wk >> 8) & 0xff];
        a[2] += spread[(wk >> 16) & 0xff];
        a[3] += spread[wk >> 24];
      }
      if ((f - fb) % 255 == 254) flush();
    }
    flush();
  };
  const int vote_chunks = n_frames >= 8192 ? std::min(8, n_frames / 2048) : 1;
  if (vote_chunks == 1) {
    vote(0, n_frames, count.data(), any.data());
  } else {
    std::vector<int32_t> cnt_p((size_t)vote_chunks * count.size(), 0);
    std::vector<uint32_t> any_p((size_t)vote_chunks * any.size(), 0u);
    worker_pool().run(vote_chunks, [&](int t) {
      vote((int)((long long)n_frames * t / vote_chunks), (int)((long long)n_frames * (t + 1) / vote_chunks),
           cnt_p.data() + (size_t)t * count.size(), any_p.data() + (size_t)t * any.size());
    });
    for (int t = 0; t < vote_chunks; ++t) {
      for (size_t q = 0; q < count.size(); ++q) count[q] += cnt_p[(size_t)t * count.size() + q];
      for (size_t q = 0; q < any.size(); ++q) any[q] |= any_p[(size_t)t * any.size() + q];
    }
  }
  for (int t = 0; t < n_tpl; ++t) {
    out[t] = count[(size_t)t];
    out[n_tpl + t] = INT64_MAX;
  }
  // a frame's set iteration order only matters for the keys it holds first: only those
  // frames are replayed
  size_t remaining = 0;
  for (int k = 0; k < words; ++k) remaining += (size_t)__builtin_popcount(any[(size_t)k]);
  for (int f = 0; f < n_frames && remaining; ++f) {
    const uint32_t* w = frame_bits(f);
    bool fresh = false;
    for (int k = 0; k < words && !fresh; ++k) fresh = (w[k] & ~seen[(size_t)k]) != 0;
    if (!fresh) continue;
    frame_set_of(w, words).for_each_slot([&](int64_t key, size_t slot) {
      uint32_t& sw = seen[(size_t)(key >> 5)];
      const uint32_t bit = 1u << (key & 31);
      if (!(sw & bit)) {
        sw |= bit;
        out[n_tpl + key] = ((frame_base + f) << 32) | (int64_t)slot;
        --remaining;
      }
    });
  }
  return KCMC_OK;
}

// votes [world][2][n_tpl] -> the consensus (Counter.most_common(n_kp_global) order + counts)
// and the iteration order of set(consensus) (VA:248).  out_cons_pack [n_kp_global + words]:
// the set's iteration order in [0, nc), its bitmask (words u32) in [nc, nc + words).
int merge_impl(const int64_t* votes, int world, int n_tpl, int n_kp_global, int n_min, int32_t* out_consensus,
               int32_t* out_votes, int* out_n, int32_t* out_cons_pack) {
  std::vector<int64_t> cnt((size_t)n_tpl, 0), key((size_t)n_tpl, INT64_MAX);
  for (int r = 0; r < world; ++r) {
    const int64_t* v = votes + (size_t)r * 2 * (size_t)n_tpl;
    for (int t = 0; t < n_tpl; ++t) {
      cnt[(size_t)t] += v[t];
      key[(size_t)t] = std::min(key[(size_t)t], v[n_tpl + t]);
    }
  }
  std::vector<int32_t> order;
  for (int t = 0; t < n_tpl; ++t) {
    if (cnt[(size_t)t] < 0) return fail(KCMC_EINVAL, "kcmc_consensus_merge: negative vote count");
    if (cnt[(size_t)t] == 0) continue;
    if (key[(size_t)t] == INT64_MAX)
      return fail(KCMC_EINVAL, "kcmc_consensus_merge: a voted template has no first-occurrence key");
    order.push_back(t);
  }
  // most_common(n) == sort by count desc over first-occurrence order (heapq.nlargest is
  // stable); first-occurrence keys are distinct, so the order is total and only the first
  // n need sorting (n_tpl 4096, n 200: a full sort cost ~0.5 ms of host time per slab)
  const int nc = std::min<int>(n_kp_global, (int)order.size());
  auto before = [&](int32_t a, int32_t b) {
    return cnt[(size_t)a] != cnt[(size_t)b] ? cnt[(size_t)a] > cnt[(size_t)b] : key[(size_t)a] < key[(size_t)b];
  };
  std::partial_sort(order.begin(), order.begin() + nc, order.end(), before);
  *out_n = nc;
  for (int k = 0; k < nc; ++k) {
    if (out_consensus) out_consensus[k] = order[(size_t)k];
    if (out_votes) out_votes[k] = (int32_t)cnt[(size_t)order[(size_t)k]];
  }
  if (nc < n_min)
    return fail(KCMC_EALIGN,
                "Too few keypoints found. Try a higher quality video, or decrease "
                "`VideoAligner.N_KP_GLOBAL_MIN`");
  if (out_cons_pack) {
    PySet cons;
    for (int k = 0; k < nc; ++k) cons.add(order[(size_t)k]);
    int n = 0;
    cons.for_each([&](int64_t k) { out_cons_pack[n++] = (int32_t)k; });
    const int words = (n_tpl + 31) / 32;
    uint32_t* bits = reinterpret_cast<uint32_t*>(out_cons_pack + nc);
    for (int k = 0; k < words; ++k) bits[k] = 0u;
    for (int k = 0; k < nc; ++k) bits[order[(size_t)k] >> 5] |= 1u << (order[(size_t)k] & 31);
  }
  return KCMC_OK;
}

// list(consensus_idxs.intersection(kp_idxs_list[f])) (VA:274) for frames [f_begin, f_end):
// out_pt_off [f_end - f_begin + 1] (from 0), out_pt_idx [(f_end - f_begin) * nc].
// set_intersection iterates the smaller set (the frame's when len(frame) <= len(consensus))
// and inserts the hits into a fresh set, whose iteration order is the result.
int lookup_impl(const uint32_t* keep_bits, int f_begin, int f_end, int n_tpl, const int32_t* cons_iter, int nc,
                int32_t* out_pt_off, int32_t* out_pt_idx) {
  const int words = (n_tpl + 31) / 32;
  auto frame_bits = [&](int f) { return keep_bits + (size_t)f * words; };
  std::vector<uint32_t> cons_bits((size_t)words, 0u);
  for (int k = 0; k < nc; ++k) {
    const int32_t key = cons_iter[k];
    if (key < 0 || key >= n_tpl) return fail(KCMC_EINVAL, "consensus lookup: consensus index out of range");
    cons_bits[(size_t)(key >> 5)] |= 1u << (key & 31);
  }
  // Shortcut: without deletions a set's table size after m insertions depends on m only
  // (PySet::table_sizes), and when every key is below that size each key sits in its own
  // home slot (hash(i) = i), so the iteration order is ascending whatever the insertion and
  // resize history.  Only frames whose result keeps a key >= its final table size replay.
  const std::vector<size_t> tsize = PySet::table_sizes((size_t)nc);
  const int nf = f_end - f_begin;
  // per-frame results into a [nf, nc] scratch (no per-frame allocation), compacted below
  std::vector<int32_t> scratch((size_t)nf * (size_t)std::max(nc, 1));
  std::vector<int32_t> len((size_t)nf, 0);
  // pass 1 (serial, a few dozen operations per frame): frames whose result keeps every
  // key in its home slot list it in ascending order; the others are replayed in parallel
  std::vector<int> replay;
  for (int r = 0; r < nf; ++r) {
    const uint32_t* w = frame_bits(f_begin + r);
    size_t m = 0;
    int top = -1;
    for (int k = 0; k < words; ++k) {
      const uint32_t hit = w[k] & cons_bits[(size_t)k];
      m += (size_t)__builtin_popcount(hit);
      if (hit) top = 32 * k + 31 - __builtin_clz(hit);
    }
    if (top >= 0 && (size_t)top >= tsize[m]) {
      replay.push_back(r);
      continue;
    }
    int32_t* L = scratch.data() + (size_t)r * (size_t)std::max(nc, 1);
    int n = 0;
    for (int k = 0; k < words; ++k)
      for (uint32_t b = w[k] & cons_bits[(size_t)k]; b; b &= b - 1) L[n++] = 32 * k + __builtin_ctz(b);
    len[(size_t)r] = n;
  }
  parallel_for((int)replay.size(), [&](int q) {
    const int r = replay[(size_t)q], f = f_begin + r;
    const uint32_t* w = frame_bits(f);
    int32_t* L = scratch.data() + (size_t)r * (size_t)std::max(nc, 1);
    size_t flen = 0;
    for (int k = 0; k < words; ++k) flen += (size_t)__builtin_popcount(w[k]);
    int n = 0;
    if (flen > (size_t)nc && (size_t)nc <= 1228) {
      // the common replay: iterate the consensus set, insert the frame's keys
      SmallPySet result;
      for (int k = 0; k < nc; ++k) {
        const int32_t key = cons_iter[k];
        if ((w[key >> 5] >> (key & 31)) & 1u) result.add(key);
      }
      result.for_each([&](int32_t key) { L[n++] = key; });
    } else {
      PySet result;
      if (flen > (size_t)nc) {
        for (int k = 0; k < nc; ++k) {
          const int32_t key = cons_iter[k];
          if ((w[key >> 5] >> (key & 31)) & 1u) result.add(key);
        }
      } else {
        frame_set_of(w, words).for_each([&](int64_t key) {
          if ((cons_bits[(size_t)(key >> 5)] >> (key & 31)) & 1u) result.add(key);
        });
      }
      result.for_each([&](int64_t key) { L[n++] = (int32_t)key; });
    }
    len[(size_t)r] = n;
  });
  out_pt_off[0] = 0;
  for (int r = 0; r < nf; ++r) {
    if (out_pt_idx)
      std::copy(scratch.begin() + (ptrdiff_t)r * std::max(nc, 1),
                scratch.begin() + (ptrdiff_t)r * std::max(nc, 1) + len[(size_t)r], out_pt_idx + out_pt_off[r]);
    out_pt_off[r + 1] = out_pt_off[r] + len[(size_t)r];
  }
  return KCMC_OK;
}

}  // namespace kcmc

extern "C" int kcmc_consensus_vote_host(const uint32_t* keep_bits, int n_frames, int n_tpl, long long frame_base,
                                        int64_t* out_votes) {
  if (n_frames < 0 || n_tpl < 0 || (!keep_bits && n_frames > 0 && n_tpl > 0) || (!out_votes && n_tpl > 0) ||
      frame_base < 0 || frame_base + (long long)n_frames > (long long)INT32_MAX)
    return fail(KCMC_EINVAL, "kcmc_consensus_vote_host: bad arguments");
  return vote_impl(keep_bits, n_frames, n_tpl, (int64_t)frame_base, out_votes);
}

extern "C" int kcmc_consensus_merge(const int64_t* votes, int world, int n_tpl, int n_kp_global, int n_min,
                                    int32_t* out_consensus, int32_t* out_votes, int* out_n_consensus,
                                    int32_t* out_cons_pack) {
  if (world < 1 || n_tpl < 0 || n_kp_global < 0 || (!votes && n_tpl > 0) || !out_n_consensus)
    return fail(KCMC_EINVAL, "kcmc_consensus_merge: bad arguments");
  return merge_impl(votes, world, n_tpl, n_kp_global, n_min, out_consensus, out_votes, out_n_consensus,
                    out_cons_pack);
}

extern "C" int kcmc_consensus_lookup_host(const uint32_t* keep_bits, int n_frames, int n_tpl, const int32_t* cons_iter,
                                          int nc, int32_t* out_pt_off, int32_t* out_pt_idx) {
  if (n_frames < 0 || n_tpl < 0 || nc < 0 || (!keep_bits && n_frames > 0 && n_tpl > 0) ||
      (!cons_iter && nc > 0) || !out_pt_off)
    return fail(KCMC_EINVAL, "kcmc_consensus_lookup_host: bad arguments");
  return lookup_impl(keep_bits, 0, n_frames, n_tpl, cons_iter, nc, out_pt_off, out_pt_idx);
}

extern "C" int kcmc_consensus_slice(const uint32_t* keep_bits, int n_frames, int n_tpl, int n_kp_global,
                                    int n_min, int f_begin, int f_end, int32_t* out_consensus,
                                    int32_t* out_votes, int* out_n_consensus, int32_t* out_pt_off,
                                    int32_t* out_pt_idx) {
  if (n_frames < 0 || n_tpl < 0 || n_kp_global < 0 || (!keep_bits && n_frames > 0) ||
      !out_n_consensus || !out_pt_off || f_begin < 0 || f_end < f_begin || f_end > n_frames)
    return fail(KCMC_EINVAL, "kcmc_consensus: bad arguments");
  std::vector<int64_t> votes((size_t)2 * (size_t)n_tpl);
  KCMC_TRY(vote_impl(keep_bits, n_frames, n_tpl, 0, votes.data()));
  const int words = (n_tpl + 31) / 32;
  std::vector<int32_t> pack((size_t)n_kp_global + (size_t)words);
  KCMC_TRY(merge_impl(votes.data(), 1, n_tpl, n_kp_global, n_min, out_consensus, out_votes, out_n_consensus,
                      pack.data()));
  return lookup_impl(keep_bits, f_begin, f_end, n_tpl, pack.data(), *out_n_consensus, out_pt_off, out_pt_idx);
}

extern "C" int kcmc_consensus(const uint32_t* keep_bits, int n_frames, int n_tpl, int n_kp_global,
                              int n_min, int32_t* out_consensus, int32_t* out_votes,
                              int* out_n_consensus, int32_t* out_pt_off, int32_t* out_pt_idx) {
  return kcmc_consensus_slice(keep_bits, n_frames, n_tpl, n_kp_global, n_min, 0, n_frames < 0 ? 0 : n_frames,
                              out_consensus, out_votes, out_n_consensus, out_pt_off, out_pt_idx);
}
