// The host byte passes of bg_batch_prepare / bg_batch_fetch (biogarden_amd/csrc/bg_host_passes.h)
// against straightforward restatements, on random batches: empty sides, unscorable bytes,
// 26-code and wide (40 / 256-code) closures, a byte coded 31, argument errors, shard call dims,
// 1 / 3 / 16 pool threads.  Built with -fsanitize=address,undefined by tests/test_sanitizers.py
// so the offset and pointer arithmetic of those passes runs under the sanitizers.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../biogarden_amd/csrc/bg_host_passes.h"

#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static bgh::HScore make_score(int kind, std::mt19937_64& rng) {
  bgh::HScore S;
  for (int x = 0; x < 256; ++x) S.code[x] = 0xFFFF;
  if (kind == 0) {            // 'A'..'Z' (score.rs's tables)
    S.K = 32;
    for (int c = 0; c < 26; ++c) S.code['A' + c] = (uint16_t)c;
  } else if (kind == 1) {     // a byte coded 31 (collides with the unscorable marker bit)
    S.K = 32;
    for (int c = 0; c < 32; ++c) S.code['@' + c] = (uint16_t)c;
  } else if (kind == 2) {     // 40 codes
    S.K = 40;
    for (int c = 0; c < 40; ++c) S.code['0' + c] = (uint16_t)c;
  } else {                    // every byte
    S.K = 256;
    for (int c = 0; c < 256; ++c) S.code[c] = (uint16_t)c;
  }
  S.tab.resize((size_t)S.K * S.K);
  for (auto& v : S.tab) v = (int32_t)(rng() % 21) - 10;
  return S;
}

int main() {
  std::mt19937_64 rng(12345);
  const char* threads[] = {"1", "3", "16"};
  int batches = 0;
  for (int it = 0; it < 120; ++it) {
    setenv("BG_HOST_THREADS", threads[it % 3], 1);
    const int kind = it % 4;
    bgh::HScore S = make_score(kind, rng);
    const size_t np = rng() % 40;
    std::vector<std::string> a(np), b(np);
    std::vector<const uint8_t*> p1(np), p2(np);
    std::vector<size_t> n1(np), n2(np);
    for (size_t p = 0; p < np; ++p) {
      const size_t lens[] = {0, 1, 2, 63, 64, 65, 700, 3000};
      n1[p] = lens[rng() % 8];
      n2[p] = lens[rng() % 8];
      auto fill = [&](std::string& s, size_t n) {
        s.resize(n);
        for (size_t i = 0; i < n; ++i) {
          int c;
          do { c = (int)(rng() % 256); } while (S.code[c] >= S.K && rng() % 512);  // rare unscorable
          s[i] = (char)c;
        }
      };
      fill(a[p], n1[p]);
      fill(b[p], n2[p]);
      p1[p] = n1[p] ? reinterpret_cast<const uint8_t*>(a[p].data()) : nullptr;   // null when empty
      p2[p] = n2[p] ? reinterpret_cast<const uint8_t*>(b[p].data()) : nullptr;
    }
    const int mode = (int)(rng() % 5);
    const int32_t ga = (it % 7 == 0) ? 1 : -(int32_t)(rng() % 12);
    const int32_t gb = -(int32_t)(rng() % 3);
    std::vector<int> pre;
    std::vector<uint64_t> c1, c2;
    CHECK(bgh::stage_validate(mode, np, p1.data(), n1.data(), p2.data(), n2.data(), ga, gb, pre, c1, c2) == BG_OK);
    // restated checks
    const bool nonpos = mode == BG_GLOBAL || mode == BG_LOCAL || mode == BG_FITTING;
    uint64_t o1 = 0, o2 = 0;
    for (size_t p = 0; p < np; ++p) {
      int want = -1;
      if (nonpos && (ga > 0 || gb > 0)) want = BG_INVALID_ARGUMENT_RANGE;
      else if (mode == BG_FITTING && n1[p] < n2[p]) want = BG_INVALID_INPUT_SIZE;
      CHECK(pre[p] == want);
      CHECK(c1[p] == o1 && c2[p] == o2);
      if (want < 0) { o1 += n1[p]; o2 += n2[p]; }
    }
    CHECK(c1[np] == o1 && c2[np] == o2);
    std::vector<uint8_t> stage(o1 + o2 + 16 + 1);
    uint8_t* st1 = stage.data();
    uint8_t* st2 = st1 + o1 + 16;
    std::vector<uint32_t> pm;
    std::vector<uint64_t> pw;
    std::vector<char> present;
    bgh::stage_copy(np, p1.data(), n1.data(), p2.data(), n2.data(), S, pre, c1, c2, st1, st2, pm, pw, present);
    std::vector<char> want_present(S.K, 0);
    for (size_t p = 0; p < np; ++p) {
      if (pre[p] == BG_INVALID_ARGUMENT_RANGE || pre[p] == BG_INVALID_INPUT_SIZE) continue;
      CHECK(std::string(reinterpret_cast<char*>(st1 + c1[p]), n1[p]) == a[p]);
      CHECK(std::string(reinterpret_cast<char*>(st2 + c2[p]), n2[p]) == b[p]);
      bool bad = false;
      std::vector<char> used(S.K, 0);
      if (n1[p] && n2[p])
        for (const std::string* s : {&a[p], &b[p]})
          for (unsigned char ch : *s) {
            if (S.code[ch] >= S.K) bad = true;
            else used[S.code[ch]] = 1;
          }
      CHECK(pre[p] == (bad ? BG_UNSCORABLE : -1));
      if (bad || !n1[p] || !n2[p]) continue;
      for (int c = 0; c < S.K; ++c) {
        const bool got = S.K > 32 ? ((pw[p * 4 + (c >> 6)] >> (c & 63)) & 1) : ((pm[p] >> c) & 1);
        CHECK(got == (used[c] != 0));
        want_present[c] |= used[c];
      }
    }
    CHECK(present == want_present);
    // call history: plain and with per-pair dims
    for (int given = 0; given < 2; ++given) {
      std::vector<std::pair<long, long>> dims;
      if (given)
        for (size_t p = 0; p < np; ++p) dims.emplace_back((long)(rng() % 4000), (long)(rng() % 4000));
      long rows = 1024, cols = 1024;
      std::vector<std::pair<long, long>> at;
      bgh::call_history(np, n1.data(), n2.data(), pre, dims, false, rows, cols, at);
      long r = 1024, c = 1024;
      for (size_t p = 0; p < np; ++p) {
        if (given) { r = dims[p].first; c = dims[p].second; }
        CHECK(at[p].first == r && at[p].second == c);
        if (pre[p] == BG_INVALID_ARGUMENT_RANGE || pre[p] == BG_INVALID_INPUT_SIZE) continue;
        if ((long)n1[p] > r || (long)n2[p] > c) { r = (long)n1[p] + 1; c = (long)n2[p] + 1; }
      }
      CHECK(rows == r && cols == c);
    }
    // fetch unpack: random slot layout -> caller layout
    std::vector<bgh::UnpackJob> jobs;
    uint64_t src = 0, dst = 0;
    for (size_t p = 0; p < np; ++p) {
      const uint32_t cap = (uint32_t)(n1[p] + n2[p]);
      const uint32_t len = cap ? (uint32_t)(rng() % (cap + 1)) : 0;
      jobs.push_back({src + (cap - len), dst, len});
      src += cap;
      dst += cap;
    }
    std::vector<uint8_t> h1(src + 1), h2(src + 1), out1(dst + 1, 0), out2(dst + 1, 0);
    for (auto& x : h1) x = (uint8_t)rng();
    for (auto& x : h2) x = (uint8_t)rng();
    bgh::unpack_strings(jobs, h1.data(), h2.data(), out1.data(), out2.data());
    for (const auto& j : jobs)
      for (uint32_t k = 0; k < j.len; ++k) CHECK(out1[j.dst + k] == h1[j.src + k] && out2[j.dst + k] == h2[j.src + k]);
    ++batches;
  }
  // argument errors
  {
    const size_t n1[] = {3}, n2[] = {2};
    const uint8_t* p1[] = {nullptr};
    const uint8_t* p2[] = {reinterpret_cast<const uint8_t*>("AC")};
    std::vector<int> pre;
    std::vector<uint64_t> c1, c2;
    CHECK(bgh::stage_validate(BG_GLOBAL, 1, p1, n1, p2, n2, -1, -1, pre, c1, c2) == BG_E_ARG);
    const size_t big[] = {(size_t)1 << 30};
    CHECK(bgh::stage_validate(BG_GLOBAL, 1, p2, big, p2, n2, -1, -1, pre, c1, c2) == BG_E_ARG);
  }
  // compact export records (bg_batch_export_compact's format): random alignments encoded as
  // headers + 2-bit cores, expanded, checked against a direct construction; malformed records
  // (bad magic, truncation, op 3, inconsistent consumption, out-of-range fields) are refused
  int records = 0;
  for (int it = 0; it < 60; ++it) {
    setenv("BG_HOST_THREADS", threads[it % 3], 1);
    const size_t np = rng() % 30;
    const uint64_t mode = (it % 3 == 0) ? (uint64_t)(rng() % 4) : 4;   // mostly semiglobal
    const bool semi = mode == 4;
    std::vector<std::string> a(np), b(np), w1(np), w2(np);
    std::vector<bg_compact_hdr> hd(np);
    std::vector<uint8_t> ops;
    for (size_t p = 0; p < np; ++p) {
      const size_t n1 = rng() % 300, n2 = rng() % 300;
      a[p].resize(n1); b[p].resize(n2);
      for (auto& c : a[p]) c = (char)(rng() % 256);      // any byte, '-' included
      for (auto& c : b[p]) c = (char)(rng() % 256);
      bg_compact_hdr h;
      std::memset(&h, 0, sizeof(h));
      h.status = (int)(rng() % 5);
      h.score = (int)(rng() % 1000) - 500;
      // a core from (s1, s2) to (e1, e2), then optional semiglobal prefix / tail runs
      size_t s1 = n1 ? rng() % (n1 + 1) : 0, s2 = n2 ? rng() % (n2 + 1) : 0;
      size_t i = s1, j = s2;
      std::vector<int> core;
      while ((i < n1 || j < n2) && rng() % 50) {
        int op = (int)(rng() % 3);
        if (op != 2 && i >= n1) op = 2;
        if (op != 1 && j >= n2) op = (i < n1) ? 1 : -1;
        if (op < 0) break;
        core.push_back(op);
        i += op != 2;
        j += op != 1;
      }
      h.start1 = (uint32_t)s1; h.start2 = (uint32_t)s2; h.end_i = (uint32_t)i; h.end_j = (uint32_t)j;
      const bool colcase = i < n1;
      // semiglobal assembly (aligner.rs:389-428): the tail runs to the last row / column; a
      // returned walk (status 0) has the prefix up to its start cell; other modes have neither
      // (status 4 is also a complete walk the host flagged BG_REF_DIVERGENT: prefix and tail too)
      const bool whole = h.status == 0 || (h.status == BG_REF_DIVERGENT && rng() % 2);
      h.npre = (uint32_t)(semi && whole ? (colcase ? s1 : s2) : 0);
      h.ntail = (uint32_t)(semi && (whole || rng() % 2) ? (colcase ? n1 - i : n2 - j) : 0);
      h.len = (uint32_t)(h.npre + core.size() + h.ntail);
      h.ops_off = ops.size();
      for (size_t q = 0; q < core.size(); q += 4) {
        uint8_t v = 0;
        for (size_t r = 0; r < 4 && q + r < core.size(); ++r) v |= (uint8_t)(core[q + r] << (2 * r));
        ops.push_back(v);
      }
      // the expected strings
      for (uint32_t q = 0; q < h.npre; ++q) {
        w1[p] += colcase ? a[p][q] : '-';
        w2[p] += colcase ? '-' : b[p][q];
      }
      size_t ii = s1, jj = s2;
      for (int op : core) { w1[p] += op != 2 ? a[p][ii++] : '-'; w2[p] += op != 1 ? b[p][jj++] : '-'; }
      for (uint32_t q = 0; q < h.ntail; ++q) {
        w1[p] += colcase ? a[p][i + q] : '-';
        w2[p] += colcase ? '-' : b[p][j + q];
      }
      hd[p] = h;
    }
    std::vector<uint8_t> rec(32 + np * sizeof(bg_compact_hdr) + ops.size());
    const uint64_t head[4] = {0x31434742ull, np, ops.size(), mode};
    std::memcpy(rec.data(), head, 32);
    if (np) std::memcpy(rec.data() + 32, hd.data(), np * sizeof(bg_compact_hdr));
    if (!ops.empty()) std::memcpy(rec.data() + 32 + np * sizeof(bg_compact_hdr), ops.data(), ops.size());
    std::vector<const uint8_t*> p1(np), p2(np);
    std::vector<size_t> n1(np), n2(np);
    size_t cap = 0;
    for (size_t p = 0; p < np; ++p) {
      p1[p] = reinterpret_cast<const uint8_t*>(a[p].data()); n1[p] = a[p].size();
      p2[p] = reinterpret_cast<const uint8_t*>(b[p].data()); n2[p] = b[p].size();
      cap += n1[p] + n2[p];
    }
    std::vector<bg_pair_result> res(np + 1);
    std::vector<uint8_t> o1(cap + 1), o2(cap + 1);
    CHECK(bgh::compact_expand(rec.data(), rec.size(), np, p1.data(), n1.data(), p2.data(), n2.data(),
                              res.data(), o1.data(), o2.data(), cap) == BG_OK);
    size_t off = 0;
    for (size_t p = 0; p < np; ++p) {
      CHECK(res[p].offset == off && res[p].len == hd[p].len && res[p].status == hd[p].status);
      CHECK(std::string(reinterpret_cast<char*>(o1.data() + off), res[p].len) == w1[p]);
      CHECK(std::string(reinterpret_cast<char*>(o2.data() + off), res[p].len) == w2[p]);
      off += n1[p] + n2[p];
    }
    // malformed: truncated, bad magic, and one corrupted header field
    if (np) {
      CHECK(bgh::compact_expand(rec.data(), rec.size() - 1, np, p1.data(), n1.data(), p2.data(), n2.data(),
                                res.data(), o1.data(), o2.data(), cap) == BG_E_ARG);
      std::vector<uint8_t> bad = rec;
      bad[0] ^= 1;
      CHECK(bgh::compact_expand(bad.data(), bad.size(), np, p1.data(), n1.data(), p2.data(), n2.data(),
                                res.data(), o1.data(), o2.data(), cap) == BG_E_ARG);
      bad = rec;
      bg_compact_hdr h0;
      std::memcpy(&h0, bad.data() + 32, sizeof(h0));
      h0.end_i += 1;                                   // consumption no longer matches
      std::memcpy(bad.data() + 32, &h0, sizeof(h0));
      CHECK(bgh::compact_expand(bad.data(), bad.size(), np, p1.data(), n1.data(), p2.data(), n2.data(),
                                res.data(), o1.data(), o2.data(), cap) == BG_E_ARG);
      // a prefix / tail inconsistent with the start / end cells (or present outside semiglobal)
      for (int kind = 0; kind < 2; ++kind) {
        bad = rec;
        std::memcpy(&h0, bad.data() + 32, sizeof(h0));
        if (kind == 0) {
          const bool cc0 = h0.end_i < n1[0];
          const uint32_t pre0 = (uint32_t)(cc0 ? h0.start1 : h0.start2);
          if (!semi || (h0.status != 0 && h0.status != BG_REF_DIVERGENT)) h0.npre += 1;
          else if (h0.status == 0) h0.npre = h0.npre ? h0.npre - 1 : 1;
          else h0.npre = pre0 + 1;                           // neither 0 nor the prefix
        } else {
          const bool cc0 = h0.end_i < n1[0];
          h0.ntail = (uint32_t)((cc0 ? n1[0] - h0.end_i : n2[0] - h0.end_j) + 1);   // past the end
        }
        h0.len = h0.npre + h0.ntail + (hd[0].len - hd[0].npre - hd[0].ntail);
        std::memcpy(bad.data() + 32, &h0, sizeof(h0));
        CHECK(bgh::compact_expand(bad.data(), bad.size(), np, p1.data(), n1.data(), p2.data(), n2.data(),
                                  res.data(), o1.data(), o2.data(), cap) == BG_E_ARG);
      }
      bad = rec;
      reinterpret_cast<uint64_t*>(bad.data())[3] = 7;  // no such mode
      CHECK(bgh::compact_expand(bad.data(), bad.size(), np, p1.data(), n1.data(), p2.data(), n2.data(),
                                res.data(), o1.data(), o2.data(), cap) == BG_E_ARG);
    }
    ++records;
  }
  std::printf("host passes ok (%d batches, %d compact records)\n", batches, records);
  return 0;
}
