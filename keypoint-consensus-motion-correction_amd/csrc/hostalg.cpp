// Host-side algorithms of the hot path that have to reproduce CPython / numpy
// behaviour bit for bit:
//   * the legacy numpy MT19937 sample stream skimage 0.18.3's ransac consumes
//     (RandomState(seed).choice(n, k, replace=False) == permutation(n)[:k]);
//   * the keypoint consensus of VA:224-286, whose RANSAC point order is the
//     iteration order of CPython `set` objects (VA:214, VA:248, VA:274) and whose
//     selection is Counter.most_common (stable by first occurrence).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

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

template <class F>
void parallel_for(int n, F&& f) {
  unsigned hw = std::thread::hardware_concurrency();
  int nt = (int)std::min<unsigned>(hw ? hw : 1, 16);
  if (n < 64 || nt <= 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  nt = std::min(nt, n / 32);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int i = t; i < n; i += nt) f(i);
    });
  for (auto& x : th) x.join();
}
}  // namespace

}  // namespace kcmc

using namespace kcmc;

extern "C" int kcmc_hypothesis_table(int n, int trials, uint32_t seed, int min_samples, int32_t* out_host) {
  return hypothesis_table_impl(n, trials, seed, min_samples, out_host);
}

extern "C" int kcmc_consensus(const uint32_t* keep_bits, int n_frames, int n_tpl, int n_kp_global,
                              int n_min, int32_t* out_consensus, int32_t* out_votes,
                              int* out_n_consensus, int32_t* out_pt_off, int32_t* out_pt_idx) {
  if (n_frames < 0 || n_tpl < 0 || n_kp_global < 0 || (!keep_bits && n_frames > 0) ||
      !out_n_consensus || !out_pt_off)
    return fail(KCMC_EINVAL, "kcmc_consensus: bad arguments");
  const int words = (n_tpl + 31) / 32;
  auto frame_bits = [&](int f) { return keep_bits + (size_t)f * words; };
  // kp_idxs = set([m.queryIdx for m in distance_matches]) (VA:214): insertions in
  // ascending template order.  Only needed where its iteration order is observable.
  auto frame_set = [&](int f) {
    PySet s;
    const uint32_t* w = frame_bits(f);
    for (int k = 0; k < words; ++k)
      for (uint32_t b = w[k]; b; b &= b - 1) s.add(32 * k + __builtin_ctz(b));
    return s;
  };
  // Counter([x for s in kp_idxs_list for x in s]) (VA:239): vote counts, and the
  // first-occurrence order (dict insertion order) -- a frame's set iteration order only
  // matters for the elements it contributes first, so only those frames are replayed.
  std::vector<int32_t> count((size_t)n_tpl, 0);
  std::vector<uint32_t> seen((size_t)words, 0u), any((size_t)words, 0u);
  for (int f = 0; f < n_frames; ++f) {
    const uint32_t* w = frame_bits(f);
    for (int k = 0; k < words; ++k) {
      any[(size_t)k] |= w[k];
      for (uint32_t b = w[k]; b; b &= b - 1) ++count[(size_t)(32 * k + __builtin_ctz(b))];
    }
  }
  size_t remaining = 0;
  for (int k = 0; k < words; ++k) remaining += (size_t)__builtin_popcount(any[(size_t)k]);
  std::vector<int32_t> order;
  order.reserve(remaining);
  for (int f = 0; f < n_frames && remaining; ++f) {
    const uint32_t* w = frame_bits(f);
    bool fresh = false;
    for (int k = 0; k < words && !fresh; ++k) fresh = (w[k] & ~seen[(size_t)k]) != 0;
    if (!fresh) continue;
    frame_set(f).for_each([&](int64_t key) {
      uint32_t& sw = seen[(size_t)(key >> 5)];
      const uint32_t bit = 1u << (key & 31);
      if (!(sw & bit)) {
        sw |= bit;
        order.push_back((int32_t)key);
        --remaining;
      }
    });
  }
  // most_common(n) == stable sort by count desc over first-occurrence order (heapq.nlargest).
  std::stable_sort(order.begin(), order.end(),
                   [&](int32_t a, int32_t b) { return count[(size_t)a] > count[(size_t)b]; });
  const int nc = std::min<int>(n_kp_global, (int)order.size());
  *out_n_consensus = nc;
  for (int k = 0; k < nc; ++k) {
    if (out_consensus) out_consensus[k] = order[(size_t)k];
    if (out_votes) out_votes[k] = count[(size_t)order[(size_t)k]];
  }
  if (nc < n_min)
    return fail(KCMC_EALIGN,
                "Too few keypoints found. Try a higher quality video, or decrease "
                "`VideoAligner.N_KP_GLOBAL_MIN`");
  // consensus_idxs = set(consensus_idxs) (VA:248)
  PySet cons;
  for (int k = 0; k < nc; ++k) cons.add(order[(size_t)k]);
  std::vector<int32_t> cons_iter;
  cons_iter.reserve((size_t)nc);
  cons.for_each([&](int64_t key) { cons_iter.push_back((int32_t)key); });
  std::vector<uint32_t> cons_bits((size_t)words, 0u);
  for (int32_t key : cons_iter) cons_bits[(size_t)(key >> 5)] |= 1u << (key & 31);
  // list(consensus_idxs.intersection(kp_idxs_list[i])) (VA:274): set_intersection
  // iterates the smaller set (the frame's when len(frame) <= len(consensus)) and
  // inserts the hits into a fresh set, whose iteration order is the result.
  std::vector<std::vector<int32_t>> lists((size_t)n_frames);
  parallel_for(n_frames, [&](int f) {
    const uint32_t* w = frame_bits(f);
    size_t len = 0;
    for (int k = 0; k < words; ++k) len += (size_t)__builtin_popcount(w[k]);
    PySet result;
    if (len > (size_t)nc) {
      for (int32_t key : cons_iter)
        if ((w[key >> 5] >> (key & 31)) & 1u) result.add(key);
    } else {
      frame_set(f).for_each([&](int64_t key) {
        if ((cons_bits[(size_t)(key >> 5)] >> (key & 31)) & 1u) result.add(key);
      });
    }
    auto& L = lists[(size_t)f];
    L.reserve(result.size());
    result.for_each([&](int64_t key) { L.push_back((int32_t)key); });
  });
  out_pt_off[0] = 0;
  for (int f = 0; f < n_frames; ++f) {
    const auto& L = lists[(size_t)f];
    if (out_pt_idx) std::copy(L.begin(), L.end(), out_pt_idx + out_pt_off[f]);
    out_pt_off[f + 1] = out_pt_off[f] + (int32_t)L.size();
  }
  return KCMC_OK;
}
