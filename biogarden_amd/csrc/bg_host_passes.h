// Host-side byte passes behind the C ABI (bg_host.cpp): validation and staging of a batch's
// residues, the reference aligner's scratch history, and the unpacking of fetched strings, with
// the worker pool they run on.  Plain C++17 with no HIP dependency, so the pointer and offset
// arithmetic can be exercised under AddressSanitizer / UBSan on a CPU-only host
// (tests/cpp/test_host_passes.cpp, tests/test_sanitizers.py).
//
// Reference behaviour mirrored here:
//   argument checks      aligner.rs:87-89, 153-155, 219-225 (status 1 / 2, in that order)
//   score closure domain score.rs:38-41 (a byte outside the table panics: status 3)
//   scratch history      aligner.rs:92-94, 594-602 (resize to (n1+1, n2+1) iff n1 > rows || n2 > cols)
#pragma once
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "biogarden_gpu.h"

namespace bgh {

// CPUs this process may run on: its affinity mask, bounded by the cgroup's CPU quota (threads
// beyond the quota only time-share it, and a burst over it is throttled for the rest of the
// scheduler period).  The MI355X boxes show 256 CPUs with a 16-CPU quota per GPU.
inline int usable_cpus() {
  static const int n = [] {
    int c = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = CPU_COUNT(&set);
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long per = 0;
      if (std::fscanf(f, "%31s %ld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0)
        c = std::min(c, std::max(1, (int)(std::atol(q) / per)));
      std::fclose(f);
    }
    return std::max(1, c);
  }();
  return n;
}

// Host threads for the byte passes of prepare / fetch: at most 16 (a GPU's share of the host's
// cores on the MI355X nodes) and the usable CPUs, one per ~256 KiB of input; BG_HOST_THREADS
// overrides.
inline int host_threads(uint64_t bytes) {
  int t = std::min(16, usable_cpus());
  if (const char* e = std::getenv("BG_HOST_THREADS")) t = std::max(1, std::atoi(e));
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)t, bytes / (256 << 10) + 1));
}

// A persistent pool of host worker threads for the byte passes (created once, reused by every
// handle): a parallel region costs two condition-variable hand-offs instead of a thread
// creation and join per worker per call (16 of them per prepare and per fetch, ~1 ms a batch on
// the streaming path).  One region at a time; the calling thread takes a share of the tasks.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();   // never destroyed: workers may outlive static dtors
    return *p;
  }
  // runs f(0) .. f(n - 1), at most one task per thread at a time, returns when all are done
  template <class F>
  void run(int n, const F& f) {
    if (n <= 1) { if (n == 1) f(0); return; }
    std::lock_guard<std::mutex> region(callM_);
    const int want = n - 1;
    {
      std::lock_guard<std::mutex> g(m_);
      while ((int)th_.size() < want) th_.emplace_back([this] { worker(); });
      task_ = [&f](int k) { f(k); };
      ntasks_ = n;
      next_ = 0;
      finished_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return finished_ == ntasks_; });
    task_ = nullptr;
  }

 private:
  void drain() {
    for (;;) {
      int k;
      {
        std::lock_guard<std::mutex> g(m_);
        if (next_ >= ntasks_) return;
        k = next_++;
      }
      task_(k);
      std::lock_guard<std::mutex> g(m_);
      if (++finished_ == ntasks_) done_.notify_all();
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
      }
      drain();
    }
  }
  std::mutex callM_, m_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  std::function<void(int)> task_;
  int ntasks_ = 0, next_ = 0, finished_ = 0;
  uint64_t gen_ = 0;
};

// Runs fn(lo, hi) over [0, n) split into contiguous ranges of about equal weight
// (weight(i) = bytes of item i), one per pool task; inline when one thread suffices.
template <class Wt, class F>
void par_ranges(size_t n, Wt weight, F fn) {
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += weight(i);
  const int T = host_threads(total);
  if (T <= 1 || n < 2) { fn((size_t)0, n); return; }
  std::vector<size_t> cut(1, 0);
  size_t lo = 0;
  uint64_t acc = 0;
  for (int k = 0; k < T && lo < n; ++k) {
    const uint64_t goal = total * (uint64_t)(k + 1) / (uint64_t)T;
    size_t hi = lo;
    while (hi < n && (acc < goal || hi == lo)) acc += weight(hi++);
    if (k == T - 1) hi = n;
    cut.push_back(hi);
    lo = hi;
  }
  if (cut.back() < n) cut.back() = n;
  HostPool::get().run((int)cut.size() - 1, [&](int k) { fn(cut[k], cut[k + 1]); });
}

// The score closure tabulated over the codes a batch may use: code[byte] (0xFFFF:
// the closure panics on that byte, score.rs:40), tab[q * K + c].  The 32 x 32 bg_scoring and the
// wide table of bg_batch_prepare_table (up to 256 codes: any byte alphabet, as the reference's
// &dyn Fn(&u8, &u8) -> i32 and analysis::seq's raw-byte equality allow) both become this.
struct HScore {
  uint16_t code[256];
  int K = 0;
  std::vector<int32_t> tab;
  int32_t at(int q, int c) const { return tab[(size_t)q * K + c]; }
};

// ---- prepare, part 1: per-pair argument checks in the reference's order (status 1 before 2),
// and the caller-order offsets of the residues that will be staged (pairs with a status are not).
// Returns BG_OK or BG_E_ARG (a null pointer with a nonzero length, a length beyond 2^30 - 1).
inline int stage_validate(int mode, size_t npairs, const uint8_t* const* s1, const size_t* n1,
                          const uint8_t* const* s2, const size_t* n2, int32_t a, int32_t b,
                          std::vector<int>& prestatus, std::vector<uint64_t>& coff1,
                          std::vector<uint64_t>& coff2) {
  const bool needNonPos = mode == BG_GLOBAL || mode == BG_LOCAL || mode == BG_FITTING;
  prestatus.assign(npairs, -1);
  for (size_t p = 0; p < npairs; ++p) {
    if ((n1[p] && !s1[p]) || (n2[p] && !s2[p])) return BG_E_ARG;
    if (n1[p] > 0x3FFFFFFF || n2[p] > 0x3FFFFFFF) return BG_E_ARG;
    if (needNonPos && (a > 0 || b > 0)) { prestatus[p] = BG_INVALID_ARGUMENT_RANGE; continue; }
    if (mode == BG_FITTING && n1[p] < n2[p]) { prestatus[p] = BG_INVALID_INPUT_SIZE; continue; }
  }
  coff1.resize(npairs + 1);
  coff2.resize(npairs + 1);
  coff1[0] = coff2[0] = 0;
  for (size_t p = 0; p < npairs; ++p) {
    const bool stage = prestatus[p] < 0;
    coff1[p + 1] = coff1[p] + (stage ? n1[p] : 0);
    coff2[p + 1] = coff2[p] + (stage ? n2[p] : 0);
  }
  return BG_OK;
}

// ---- prepare, part 2: one pass over the caller's bytes, split over the pool by bytes: the raw
// residues of every pair without a status go to st1 / st2 at coff1 / coff2 (caller order), and
// each such pair's set of score codes is computed — pmask (codes < 32; bit 31 marks a byte the
// closure panics on) or, for alphabets beyond 32 codes, pmaskW (4 x 64 bits per pair).  A pair
// touching an unscorable byte gets status 3 (score.rs:40 panics; never for an empty side: the
// closure is not called).  present[c] = some staged pair uses code c.
inline void stage_copy(size_t npairs, const uint8_t* const* s1, const size_t* n1,
                       const uint8_t* const* s2, const size_t* n2, const HScore& S,
                       std::vector<int>& prestatus, const std::vector<uint64_t>& coff1,
                       const std::vector<uint64_t>& coff2, uint8_t* st1, uint8_t* st2,
                       std::vector<uint32_t>& pmask, std::vector<uint64_t>& pmaskW,
                       std::vector<char>& present) {
  uint32_t bitOf[256];
  for (int x = 0; x < 256; ++x) {
    const uint16_t c = S.code[x];
    bitOf[x] = (c < 32 && c < S.K) ? (1u << c) : 0x80000000u;
  }
  bool codeBad = false;                 // a byte coded 31 collides with the marker: scan exactly
  for (int x = 0; x < 256; ++x) codeBad |= S.code[x] == 31;
  const bool wideK = S.K > 32;          // codes beyond 31: 256-bit sets per pair
  pmask.assign(npairs, 0);
  if (wideK) pmaskW.assign(npairs * 4, 0);
  present.assign(S.K, 0);
  par_ranges(npairs, [&](size_t p) -> uint64_t { return (uint64_t)n1[p] + n2[p]; },
             [&](size_t lo, size_t hi) {
    for (size_t p = lo; p < hi; ++p) {
      if (prestatus[p] >= 0) continue;
      if (n1[p]) std::memcpy(st1 + coff1[p], s1[p], n1[p]);
      if (n2[p]) std::memcpy(st2 + coff2[p], s2[p], n2[p]);
      if (n1[p] == 0 || n2[p] == 0) continue;   // the score closure is never called
      const uint8_t* x1 = st1 + coff1[p];
      const uint8_t* x2 = st2 + coff2[p];
      bool bad = false;
      if (wideK) {
        uint64_t m4[4] = {0, 0, 0, 0};
        for (int side = 0; side < 2 && !bad; ++side) {
          const uint8_t* x = side ? x2 : x1;
          const size_t n = side ? n2[p] : n1[p];
          for (size_t i = 0; i < n; ++i) {
            const uint16_t c = S.code[x[i]];
            if (c >= S.K) { bad = true; break; }
            m4[c >> 6] |= 1ull << (c & 63);
          }
        }
        if (bad) prestatus[p] = BG_UNSCORABLE;
        else for (int w = 0; w < 4; ++w) pmaskW[p * 4 + w] = m4[w];
        continue;
      }
      uint32_t m = 0;
      for (size_t i = 0; i < n1[p]; ++i) m |= bitOf[x1[i]];
      for (size_t j = 0; j < n2[p]; ++j) m |= bitOf[x2[j]];
      if (codeBad) {
        for (size_t i = 0; i < n1[p] && !bad; ++i) bad = S.code[x1[i]] >= 32 || S.code[x1[i]] >= S.K;
        for (size_t j = 0; j < n2[p] && !bad; ++j) bad = S.code[x2[j]] >= 32 || S.code[x2[j]] >= S.K;
      } else {
        bad = (m & 0x80000000u) != 0;
      }
      if (bad) prestatus[p] = BG_UNSCORABLE;
      else pmask[p] = m;
    }
  });
  for (size_t p = 0; p < npairs; ++p) {
    if (prestatus[p] >= 0) continue;
    if (wideK) {
      for (int c = 0; c < S.K; ++c) present[c] |= ((pmaskW[p * 4 + (c >> 6)] >> (c & 63)) & 1u) != 0;
    } else {
      for (int c = 0; c < 32 && c < S.K; ++c) present[c] |= ((pmask[p] >> c) & 1u) != 0;
    }
  }
}

// ---- the reference's scratch history over a batch's calls (aligner.rs:92-94): bufAt[p] = the
// dims call p starts from.  The argument errors return before the resize; everything else (the
// score panic included) resizes first.  `given` (npairs entries, or empty): per-pair start dims
// of a shard (bg_aligner_set_call_dims).  `noAligner` (edit distance, LCS): no history.
// Updates rows / cols to the dims after the last call.
inline void call_history(size_t npairs, const size_t* n1, const size_t* n2,
                         const std::vector<int>& prestatus,
                         const std::vector<std::pair<long, long>>& given, bool noAligner,
                         long& rows, long& cols, std::vector<std::pair<long, long>>& bufAt) {
  bufAt.assign(npairs, std::make_pair(rows, cols));
  for (size_t p = 0; p < npairs; ++p) {
    if (!given.empty()) { rows = given[p].first; cols = given[p].second; }
    bufAt[p] = std::make_pair(rows, cols);
    if (noAligner || prestatus[p] == BG_INVALID_ARGUMENT_RANGE || prestatus[p] == BG_INVALID_INPUT_SIZE)
      continue;
    if ((long)n1[p] > rows || (long)n2[p] > cols) { rows = (long)n1[p] + 1; cols = (long)n2[p] + 1; }
  }
}

// ---- multi-device batches (bg_group, bg_group.cpp): a batch split over shards by cells,
// largest pair first, each to the least-loaded shard (ties: the lower index), as
// biogarden_amd/shard.py lpt_shards does for ranks.  shard_of[p] = the shard of pair p.
inline void lpt_plan(size_t npairs, const size_t* n1, const size_t* n2, int nshards, int32_t* shard_of) {
  std::vector<size_t> order(npairs);
  for (size_t p = 0; p < npairs; ++p) order[p] = p;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
    return (uint64_t)n1[x] * n2[x] > (uint64_t)n1[y] * n2[y];
  });
  std::vector<uint64_t> load((size_t)std::max(nshards, 1), 0);
  for (size_t p : order) {
    int best = 0;
    for (int r = 1; r < nshards; ++r)
      if (load[r] < load[best]) best = r;
    shard_of[p] = best;
    load[best] += (uint64_t)n1[p] * n2[p];
  }
}

// The scratch dims each call of a batch starts from, in caller order, for ONE reference aligner
// running the whole batch (biogarden_amd/shard.py call_dims): the argument errors return before
// the resize (aligner.rs:87-89, 153-155, 219-225), every other call resizes to (n1 + 1, n2 + 1)
// when n1 > rows || n2 > cols (:92-94, 594-602).  rows / cols: in, the dims before the batch;
// out, after it.
inline void batch_call_dims(int mode, size_t npairs, const size_t* n1, const size_t* n2, int32_t a,
                            int32_t b, long& rows, long& cols, std::vector<std::pair<long, long>>& dims) {
  const bool badArgs = (mode == BG_GLOBAL || mode == BG_LOCAL || mode == BG_FITTING) && (a > 0 || b > 0);
  dims.resize(npairs);
  for (size_t p = 0; p < npairs; ++p) {
    dims[p] = std::make_pair(rows, cols);
    if (badArgs || (mode == BG_FITTING && n1[p] < n2[p])) continue;
    if ((long)n1[p] > rows || (long)n2[p] > cols) { rows = (long)n1[p] + 1; cols = (long)n2[p] + 1; }
  }
}

// ---- fetch: copy each pair's aligned strings from the downloaded slot buffers to the caller's
// output, over the pool: job q copies len bytes at src of h1 / h2 to dst of out1 / out2.
struct UnpackJob {
  uint64_t src, dst;
  uint32_t len;
};
inline void unpack_strings(const std::vector<UnpackJob>& jobs, const uint8_t* h1, const uint8_t* h2,
                           uint8_t* out1, uint8_t* out2) {
  par_ranges(jobs.size(), [&](size_t q) -> uint64_t { return 2ull * jobs[q].len + 64; },
             [&](size_t lo, size_t hi) {
    for (size_t q = lo; q < hi; ++q) {
      const UnpackJob& j = jobs[q];
      if (!j.len) continue;
      std::memcpy(out1 + j.dst, h1 + j.src, j.len);
      std::memcpy(out2 + j.dst, h2 + j.src, j.len);
    }
  });
}

// ---- the compact export record (include/biogarden_gpu.h bg_batch_export_compact) expanded on
// the host into bg_batch_fetch's output, over the pool.  Every header is range-checked against
// its pair before any byte is written; returns BG_OK or BG_E_ARG.
// One or several records (bg_group: one per member) in ONE pass over the pool: the pairs of every
// record are the work items, so a group's members expand side by side instead of one after the
// other.  Record r covers rp[r] of the caller's pairs: s1 / n1 / s2 / n2 / res are indexed through
// idx (nullptr: the records' pairs are 0, 1, 2, ... in order), dstoff[q] (nullptr: packed back to
// back in that order, as bg_batch_fetch does) is where item q's strings go in out1 / out2.
struct CompactRec {
  const uint8_t* rec;
  size_t bytes;
  size_t np;
};
inline int compact_expand_multi(const CompactRec* recs, size_t nrec, const uint8_t* const* s1,
                                const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                                const size_t* idx, bg_pair_result* res, uint8_t* out1, uint8_t* out2,
                                size_t out_cap, const uint64_t* dstoff) {
  struct Item {
    bg_compact_hdr h;
    const uint8_t* ops;     // the record's ops area
    uint64_t opsBytes;
    size_t p;               // caller pair
    uint64_t off;           // output offset
    bool semi;
  };
  size_t total = 0;
  for (size_t r = 0; r < nrec; ++r) total += recs[r].np;
  if (total && (!res || !n1 || !n2 || !s1 || !s2)) return BG_E_ARG;
  std::vector<Item> it(total);
  uint64_t end = 0, pos = 0;
  size_t q = 0;
  for (size_t r = 0; r < nrec; ++r) {
    const CompactRec& R = recs[r];
    if (!R.rec || R.bytes < 32) return BG_E_ARG;
    uint64_t head[4];
    std::memcpy(head, R.rec, 32);
    if (head[0] != 0x31434742ull || head[1] != R.np || head[3] > 4) return BG_E_ARG;
    if (R.bytes < 32 + R.np * sizeof(bg_compact_hdr) + head[2]) return BG_E_ARG;
    const uint8_t* ops = R.rec + 32 + R.np * sizeof(bg_compact_hdr);
    for (size_t k = 0; k < R.np; ++k, ++q) {
      Item& I = it[q];
      std::memcpy(&I.h, R.rec + 32 + k * sizeof(bg_compact_hdr), sizeof(bg_compact_hdr));
      I.ops = ops;
      I.opsBytes = head[2];
      I.semi = head[3] == 4;                             // bg_mode of the batch (BG_SEMIGLOBAL)
      I.p = idx ? idx[q] : q;
      I.off = dstoff ? dstoff[q] : pos;
      pos += n1[I.p] + n2[I.p];
      end = std::max<uint64_t>(end, I.off + n1[I.p] + n2[I.p]);
      if (dstoff && I.off > (uint64_t)out_cap) return BG_E_ARG;
    }
  }
  if (end && (!out1 || !out2 || out_cap < end)) return BG_E_ARG;
  // every pair checked (over the pool) before any byte is written
  std::atomic<int> fail{BG_OK};
  par_ranges(total, [&](size_t x) -> uint64_t { return it[x].h.len / 4 + 64; }, [&](size_t lo, size_t hi) {
  for (size_t x = lo; x < hi && fail.load(std::memory_order_relaxed) == BG_OK; ++x) {
    const bg_compact_hdr& h = it[x].h;
    const size_t p = it[x].p;
    const uint64_t ncore = (uint64_t)h.len - h.npre - h.ntail;
    auto bad = [&]() { fail.store(BG_E_ARG, std::memory_order_relaxed); };
    if ((uint64_t)h.npre + h.ntail > h.len || h.len > n1[p] + n2[p] || h.ops_off + (ncore + 3) / 4 > it[x].opsBytes ||
        h.start1 > n1[p] || h.start2 > n2[p] || h.end_i > n1[p] || h.end_j > n2[p] ||
        (n1[p] && !s1[p]) || (n2[p] && !s2[p])) {
      bad();
      continue;
    }
    // the core consumes exactly s1[start1, end_i) and s2[start2, end_j): op 0 (diagonal) takes
    // both, 1 (up) s1 only, 2 (left) s2 only, 3 is invalid — counted 32 ops per 64-bit word from
    // the ops' low and high bit planes
    uint64_t c1 = 0, c2 = 0;
    bool three = false;
    const uint8_t* po = it[x].ops + h.ops_off;
    const uint64_t kLo = 0x5555555555555555ull;
    uint64_t y = 0;
    for (; y + 32 <= ncore; y += 32) {
      uint64_t w;
      std::memcpy(&w, po + y / 4, 8);
      const uint64_t lo = w & kLo, hi = (w >> 1) & kLo;
      three |= (lo & hi) != 0;
      c1 += 32 - (uint64_t)__builtin_popcountll(hi);
      c2 += 32 - (uint64_t)__builtin_popcountll(lo);
    }
    for (; y < ncore; ++y) {
      const int op = (po[y / 4] >> (2 * (y % 4))) & 3;
      three |= op == 3;
      c1 += op != 2;
      c2 += op != 1;
    }
    if (three) { bad(); continue; }
    if (h.start1 + c1 != h.end_i || h.start2 + c2 != h.end_j) { bad(); continue; }
    // the reference's semiglobal assembly (aligner.rs:389-428): the tail gap columns run from the
    // end cell to the last row / column, and a walk that returned (status 0) is preceded by the
    // prefix of the sequence it stopped in, exactly up to its start cell (row case: s2[0, start2),
    // column case: s1[0, start1)); the other modes have neither
    const bool colcase = h.end_i < n1[p];
    if (!it[x].semi) {
      if (h.npre || h.ntail) bad();
    } else {
      const uint64_t tail = colcase ? n1[p] - h.end_i : n2[p] - h.end_j;
      const uint64_t pre = colcase ? h.start1 : h.start2;
      // status 4 is either a walk that stopped at an index underflow (no prefix) or a complete
      // walk the host flagged BG_REF_DIVERGENT (bg_ref_divergent: prefix and tail as status 0)
      const bool whole = h.npre == pre && h.ntail == tail;
      const bool stopped = h.npre == 0 && (h.ntail == 0 || h.ntail == tail);
      if (h.status == 0 ? !whole : h.status == BG_REF_DIVERGENT ? !(whole || stopped) : !stopped)
        bad();
    }
  }
  });
  if (fail.load() != BG_OK) return fail.load();
  par_ranges(total, [&](size_t x) -> uint64_t { return 2ull * it[x].h.len + 64; }, [&](size_t lo, size_t hi) {
    for (size_t x = lo; x < hi; ++x) {
      const bg_compact_hdr& h = it[x].h;
      const size_t p = it[x].p;
      bg_pair_result& o = res[p];
      std::memset(&o, 0, sizeof(o));
      o.status = h.status; o.score = h.score; o.offset = it[x].off; o.len = h.len;
      o.end_i = h.end_i; o.end_j = h.end_j; o.start1 = h.start1; o.start2 = h.start2;
      uint8_t* a1 = out1 + it[x].off;
      uint8_t* a2 = out2 + it[x].off;
      const uint8_t* r1 = s1[p];
      const uint8_t* r2 = s2[p];
      const bool colcase = h.end_i < n1[p];
      uint64_t y = 0;
      if (h.npre) {
        if (colcase) { std::memcpy(a1, r1, h.npre); std::memset(a2, '-', h.npre); }
        else { std::memset(a1, '-', h.npre); std::memcpy(a2, r2, h.npre); }
        y = h.npre;
      }
      const uint64_t ncore = (uint64_t)h.len - h.npre - h.ntail;
      const uint8_t* po = it[x].ops + h.ops_off;
      size_t i = h.start1, j = h.start2;
      // four columns per ops byte: diagonal bytes (0x00, the common case) copy four residues of
      // each sequence, the others go column by column
      uint64_t q0 = 0;
      for (; q0 + 4 <= ncore; q0 += 4, y += 4) {
        const uint8_t ob = po[q0 / 4];
        if (ob == 0) {
          std::memcpy(a1 + y, r1 + i, 4);
          std::memcpy(a2 + y, r2 + j, 4);
          i += 4;
          j += 4;
          continue;
        }
        for (int k = 0; k < 4; ++k) {
          const int op = (ob >> (2 * k)) & 3;
          a1[y + k] = op != 2 ? r1[i] : (uint8_t)'-';
          a2[y + k] = op != 1 ? r2[j] : (uint8_t)'-';
          i += op != 2;
          j += op != 1;
        }
      }
      for (; q0 < ncore; ++q0, ++y) {
        const int op = (po[q0 / 4] >> (2 * (q0 % 4))) & 3;
        a1[y] = op != 2 ? r1[i] : (uint8_t)'-';
        a2[y] = op != 1 ? r2[j] : (uint8_t)'-';
        i += op != 2;
        j += op != 1;
      }
      if (h.ntail) {
        if (colcase) { std::memcpy(a1 + y, r1 + h.end_i, h.ntail); std::memset(a2 + y, '-', h.ntail); }
        else { std::memset(a1 + y, '-', h.ntail); std::memcpy(a2 + y, r2 + h.end_j, h.ntail); }
      }
    }
  });
  return BG_OK;
}

// One record of np pairs (pairs 0 .. np-1 of the arrays); dstoff as above.
inline int compact_expand(const uint8_t* rec, size_t bytes, size_t np, const uint8_t* const* s1,
                          const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                          bg_pair_result* res, uint8_t* out1, uint8_t* out2, size_t out_cap,
                          const uint64_t* dstoff = nullptr) {
  if (!rec || bytes < 32 || (np && (!res || !n1 || !n2 || !s1 || !s2))) return BG_E_ARG;
  const CompactRec R{rec, bytes, np};
  return compact_expand_multi(&R, 1, s1, n1, s2, n2, nullptr, res, out1, out2, out_cap, dstoff);
}

}  // namespace bgh
