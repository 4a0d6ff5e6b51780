// biogarden.hpp — C++17 host facade over the C ABI (biogarden_gpu.h), mirroring the surface of
// robsndr/biogarden that the aligner's callers use (header-only; link -lbiogarden_gpu):
//
//   biogarden::alignment::SequenceAligner   src/alignment/aligner.rs:28-55, 84-435
//   biogarden::score::{blosum62,pam250,unit} src/alignment/score.rs:38, 78, 114
//   biogarden::ds::Sequence                  src/ds/sequence.rs:10-257
//   biogarden::ds::Tile                      src/ds/tile.rs:9-177
//   biogarden::io::fasta::{Reader,Record}    src/io/fasta.rs:95-135, 205-272
//   biogarden::BioError / Result             src/error.rs:8-14, 46
//
// Same method names, argument meaning and error behaviour: Err(InvalidArgumentRange) and
// Err(InvalidInputSize) exactly where the reference returns them; ReferencePanic (an exception,
// the analogue of a Rust panic) where the reference panics or hangs.  Every alignment runs the
// HIP kernels of libbiogarden_gpu.so; there is no CPU path.
#pragma once

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <istream>
#include <optional>
#include <ostream>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <variant>
#include <vector>

#include "biogarden_gpu.h"

namespace biogarden {

// ------------------------------------------------------------------ errors (error.rs:8-14)
enum class BioError { InvalidArgumentRange, InvalidInputSize };

inline const char* to_string(BioError e) {
  return e == BioError::InvalidArgumentRange ? "The provided has is within an unsupported range!"
                                             : "Provided inputs have invalid size!";
}

// Rust `Result<T, BioError>`
template <class T>
class Result {
 public:
  Result(T v) : v_(std::move(v)) {}
  Result(BioError e) : v_(e) {}
  bool is_ok() const { return v_.index() == 0; }
  bool is_err() const { return !is_ok(); }
  const T& unwrap() const {
    if (!is_ok()) throw std::logic_error(std::string("called unwrap on Err: ") + to_string(error()));
    return std::get<0>(v_);
  }
  BioError error() const { return std::get<1>(v_); }

 private:
  std::variant<T, BioError> v_;
};

// The reference panics (or hangs): unscorable byte, buffer-edge index, traceback underflow.
struct ReferencePanic : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// HIP / allocation failure below the ABI (no reference analogue).
struct DeviceError : std::runtime_error {
  int code;
  DeviceError(int c) : std::runtime_error(bg_status_string(c)), code(c) {}
};

inline int check(int rc) {
  if (rc < 0) throw DeviceError(rc);
  return rc;
}

namespace ds {

// ------------------------------------------------------------------ Sequence (sequence.rs)
class Sequence {
 public:
  std::vector<uint8_t> chain;
  std::optional<std::string> id;

  Sequence() = default;
  Sequence(const std::string& s) : chain(s.begin(), s.end()) {}
  Sequence(const char* s) : Sequence(std::string(s)) {}
  Sequence(std::vector<uint8_t> v) : chain(std::move(v)) {}
  Sequence(std::vector<uint8_t> v, std::string ident) : chain(std::move(v)), id(std::move(ident)) {}

  size_t len() const { return chain.size(); }
  bool is_empty() const { return chain.empty(); }
  void push(uint8_t c) { chain.push_back(c); }
  void extend(const Sequence& o) { chain.insert(chain.end(), o.chain.begin(), o.chain.end()); }
  void reverse() { std::reverse(chain.begin(), chain.end()); }
  uint8_t operator[](size_t i) const { return chain.at(i); }
  std::string to_string() const { return std::string(chain.begin(), chain.end()); }
  // equality ignores the id (sequence.rs:113-117)
  bool operator==(const Sequence& o) const { return chain == o.chain; }
  bool operator!=(const Sequence& o) const { return !(*this == o); }
};

inline std::ostream& operator<<(std::ostream& os, const Sequence& s) { return os << s.to_string(); }

// ------------------------------------------------------------------ Tile (tile.rs)
class Tile {
 public:
  Tile() = default;
  explicit Tile(std::vector<Sequence> v) : v_(std::move(v)) {}
  void push(Sequence s) { v_.push_back(std::move(s)); }
  size_t len() const { return v_.size(); }
  bool is_empty() const { return v_.empty(); }
  const Sequence& operator[](size_t i) const { return v_.at(i); }
  Sequence& operator[](size_t i) { return v_.at(i); }
  std::vector<Sequence>::const_iterator begin() const { return v_.begin(); }
  std::vector<Sequence>::const_iterator end() const { return v_.end(); }

 private:
  std::vector<Sequence> v_;
};

}  // namespace ds

namespace io {
namespace fasta {

// ------------------------------------------------------------------ FASTA (fasta.rs)
struct Record {
  std::string id;
  std::optional<std::string> desc;
  std::vector<uint8_t> seq;
  bool is_empty() const { return id.empty() && !desc && seq.empty(); }
};

class Reader {
 public:
  explicit Reader(std::istream& in) : in_(in) {}

  // Reads the next record into rec; returns false (rec empty) at end of input.  A record must
  // start with '>' (fasta.rs:104-109, io error otherwise); the header is right-trimmed, id = the
  // text before its first whitespace character and desc = everything after that character
  // (splitn(2, char::is_whitespace), :110-112); the sequence is the concatenation of the
  // right-trimmed lines up to the next '>' or EOF (:113-121).
  bool read(Record& rec) {
    rec = Record();
    std::string line;
    if (!have_) {
      if (!std::getline(in_, line)) return false;
    } else {
      line = std::move(pending_);
      have_ = false;
    }
    if (line.empty() || line[0] != '>') throw std::ios_base::failure("Expected > at record start.");
    std::string head = line.substr(1);
    while (!head.empty() && std::isspace((unsigned char)head.back())) head.pop_back();
    size_t cut = 0;
    while (cut < head.size() && !std::isspace((unsigned char)head[cut])) ++cut;
    rec.id = head.substr(0, cut);
    if (cut < head.size()) rec.desc = head.substr(cut + 1);
    while (std::getline(in_, line)) {
      if (!line.empty() && line[0] == '>') {
        pending_ = std::move(line);
        have_ = true;
        break;
      }
      size_t e = line.size();
      while (e > 0 && std::isspace((unsigned char)line[e - 1])) --e;
      rec.seq.insert(rec.seq.end(), line.begin(), line.begin() + e);
    }
    return true;
  }

  std::vector<Record> read_all() {
    std::vector<Record> out;
    Record r;
    while (read(r)) out.push_back(r);
    return out;
  }

 private:
  std::istream& in_;
  std::string pending_;
  bool have_ = false;
};

inline ds::Tile read_tile(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::ios_base::failure("cannot open " + path);
  Reader r(f);
  ds::Tile t;
  for (auto& rec : r.read_all()) t.push(ds::Sequence(rec.seq, rec.id));
  return t;
}

}  // namespace fasta
}  // namespace io

namespace score {

// ------------------------------------------------------------------ score (score.rs)
using ScoreFn = std::function<int32_t(const uint8_t&, const uint8_t&)>;

namespace detail {
inline const bg_scoring& builtin(int which) {
  static bg_scoring tabs[3];
  static bool init[3] = {false, false, false};
  if (!init[which]) {
    check(bg_scoring_builtin(which, &tabs[which]));
    init[which] = true;
  }
  return tabs[which];
}
inline int32_t lookup(int which, uint8_t a, uint8_t b) {
  if (a < 'A' || a > 'Z' || b < 'A' || b > 'Z')
    throw ReferencePanic("index out of bounds: score table (score.rs:40)");
  const bg_scoring& s = builtin(which);
  return s.table[s.code[a] * 32 + s.code[b]];
}
}  // namespace detail

inline int32_t blosum62(const uint8_t& a, const uint8_t& b) { return detail::lookup(BG_BLOSUM62, a, b); }
inline int32_t pam250(const uint8_t& a, const uint8_t& b) { return detail::lookup(BG_PAM250, a, b); }
inline int32_t unit(const uint8_t& a, const uint8_t& b) { return detail::lookup(BG_UNIT, a, b); }

// The device form of a score closure: the built-in tables directly; any other
// callable is evaluated once per distinct (byte of a seq1, byte of a seq2) of the batch.  The
// (byte1, byte2) on which it throws are kept: a pair whose set(seq1) x set(seq2) meets them is
// one on which the reference DP panics (status BG_UNSCORABLE, see pair_panics).
struct Tabulated {
  bg_scoring sc;
  std::set<std::pair<uint8_t, uint8_t>> panics;
  // more than 32 distinct bytes: the k x k form of bg_batch_prepare_table (code[byte] >= k:
  // a byte the closure is never evaluated on, status BG_UNSCORABLE if a pair's DP reaches it)
  bool wide = false;
  std::vector<uint16_t> code;
  int32_t k = 0;
  std::vector<int32_t> table;
};

using PairRef = std::pair<const std::vector<uint8_t>*, const std::vector<uint8_t>*>;

inline Tabulated tabulate(const ScoreFn& fn, const std::vector<PairRef>& pairs) {
  using Builtin = int32_t (*)(const uint8_t&, const uint8_t&);
  Tabulated t;
  if (const Builtin* p = fn.target<Builtin>()) {
    if (*p == &blosum62) { t.sc = detail::builtin(BG_BLOSUM62); return t; }
    if (*p == &pam250) { t.sc = detail::builtin(BG_PAM250); return t; }
    if (*p == &unit) { t.sc = detail::builtin(BG_UNIT); return t; }
  }
  std::set<uint8_t> xs, ys;
  for (const auto& pr : pairs) {
    xs.insert(pr.first->begin(), pr.first->end());
    ys.insert(pr.second->begin(), pr.second->end());
  }
  std::set<uint8_t> syms(xs);
  syms.insert(ys.begin(), ys.end());
  if (syms.size() > 32) {
    t.wide = true;
    t.k = (int32_t)syms.size();
    t.code.assign(256, 0xFFFF);
    int c = 0;
    for (uint8_t x : syms) t.code[x] = (uint16_t)c++;
    t.table.assign((size_t)t.k * t.k, 0);
    for (uint8_t x : xs)
      for (uint8_t y : ys) {
        try {
          t.table[(size_t)t.code[x] * t.k + t.code[y]] = fn(x, y);
        } catch (...) {
          t.panics.insert({x, y});
        }
      }
    return t;
  }
  std::memset(&t.sc, 0, sizeof(t.sc));
  std::memset(t.sc.code, 0xFF, sizeof(t.sc.code));
  t.sc.alphabet_size = (int32_t)syms.size();
  int c = 0;
  for (uint8_t x : syms) t.sc.code[x] = (uint8_t)c++;
  for (uint8_t x : xs)
    for (uint8_t y : ys) {
      try {
        t.sc.table[t.sc.code[x] * 32 + t.sc.code[y]] = fn(x, y);
      } catch (...) {
        t.panics.insert({x, y});
      }
    }
  return t;
}

inline bool pair_panics(const Tabulated& t, const std::vector<uint8_t>& s1, const std::vector<uint8_t>& s2) {
  if (t.panics.empty() || s1.empty() || s2.empty()) return false;
  bool in1[256] = {false}, in2[256] = {false};
  for (uint8_t x : s1) in1[x] = true;
  for (uint8_t y : s2) in2[y] = true;
  for (const auto& pr : t.panics)
    if (in1[pr.first] && in2[pr.second]) return true;
  return false;
}

}  // namespace score

namespace alignment {

using Alignment = std::tuple<int32_t, ds::Sequence, ds::Sequence>;

// Batch result: the alignment plus the per-pair status and cells (bg_pair_result).
struct PairAlignment {
  int status;
  int32_t score;
  ds::Sequence aligned1, aligned2;
  uint32_t end_i, end_j, start1, start2;
};

// ------------------------------------------------------------------ SequenceAligner
class SequenceAligner {
 public:
  explicit SequenceAligner(int device = 0) : h_(bg_aligner_new(device)) {
    if (!h_) throw DeviceError(BG_E_HIP);
  }
  static SequenceAligner new_(int device = 0) { return SequenceAligner(device); }  // aligner.rs:44
  ~SequenceAligner() {
    if (h_) bg_aligner_free(h_);
  }
  SequenceAligner(const SequenceAligner&) = delete;
  SequenceAligner& operator=(const SequenceAligner&) = delete;
  SequenceAligner(SequenceAligner&& o) noexcept : h_(o.h_) { o.h_ = nullptr; }

  Result<Alignment> global_alignment(const ds::Sequence& s1, const ds::Sequence& s2,
                                     const score::ScoreFn& score, int32_t a, int32_t b) {
    return one(BG_GLOBAL, s1, s2, score, a, b);
  }
  Result<Alignment> local_alignment(const ds::Sequence& s1, const ds::Sequence& s2,
                                    const score::ScoreFn& score, int32_t a, int32_t b) {
    return one(BG_LOCAL, s1, s2, score, a, b);
  }
  Result<Alignment> fitting_alignment(const ds::Sequence& s1, const ds::Sequence& s2,
                                      const score::ScoreFn& score, int32_t a, int32_t b) {
    return one(BG_FITTING, s1, s2, score, a, b);
  }
  Result<Alignment> overlap_alignment(const ds::Sequence& s1, const ds::Sequence& s2,
                                      const score::ScoreFn& score, int32_t a, int32_t b) {
    return one(BG_OVERLAP, s1, s2, score, a, b);
  }
  Result<Alignment> semiglobal_alignment(const ds::Sequence& s1, const ds::Sequence& s2,
                                         const score::ScoreFn& score, int32_t a, int32_t b) {
    return one(BG_SEMIGLOBAL, s1, s2, score, a, b);
  }

  // Many pairs, one call (the Tile form): no exception for per-pair statuses, see .status.
  std::vector<PairAlignment> align_batch(bg_mode mode,
                                         const std::vector<std::pair<ds::Sequence, ds::Sequence>>& pairs,
                                         const score::ScoreFn& score, int32_t a, int32_t b) {
    const size_t n = pairs.size();
    std::vector<const uint8_t*> p1(n), p2(n);
    std::vector<size_t> n1(n), n2(n);
    std::vector<score::PairRef> refs(n);
    size_t cap = 0;
    for (size_t i = 0; i < n; ++i) {
      p1[i] = pairs[i].first.chain.data();
      p2[i] = pairs[i].second.chain.data();
      n1[i] = pairs[i].first.len();
      n2[i] = pairs[i].second.len();
      cap += n1[i] + n2[i];
      refs[i] = {&pairs[i].first.chain, &pairs[i].second.chain};
    }
    const score::Tabulated tab = score::tabulate(score, refs);
    const bg_scoring& sc = tab.sc;
    std::vector<bg_pair_result> res(n ? n : 1);
    std::vector<uint8_t> o1(cap ? cap : 1), o2(cap ? cap : 1);
    if (tab.wide) {
      check(bg_batch_prepare_table(h_, mode, n, p1.data(), n1.data(), p2.data(), n2.data(),
                                   tab.code.data(), tab.k, tab.table.data(), a, b));
      check(bg_batch_execute(h_));
      check(bg_batch_fetch(h_, res.data(), o1.data(), o2.data(), cap));
    } else {
      check(bg_align_batch(h_, mode, n, p1.data(), n1.data(), p2.data(), n2.data(), &sc, a, b,
                           res.data(), o1.data(), o2.data(), cap));
    }
    std::vector<PairAlignment> out(n);
    for (size_t i = 0; i < n; ++i) {
      const bg_pair_result& r = res[i];
      out[i].status = r.status;
      if (r.status == BG_OK && score::pair_panics(tab, pairs[i].first.chain, pairs[i].second.chain))
        out[i].status = BG_UNSCORABLE;
      out[i].score = r.score;
      out[i].aligned1 = ds::Sequence(std::vector<uint8_t>(o1.begin() + r.offset, o1.begin() + r.offset + r.len));
      out[i].aligned2 = ds::Sequence(std::vector<uint8_t>(o2.begin() + r.offset, o2.begin() + r.offset + r.len));
      out[i].end_i = r.end_i;
      out[i].end_j = r.end_j;
      out[i].start1 = r.start1;
      out[i].start2 = r.start2;
    }
    return out;
  }

  bg_aligner* handle() { return h_; }

 private:
  Result<Alignment> one(bg_mode mode, const ds::Sequence& s1, const ds::Sequence& s2,
                        const score::ScoreFn& score, int32_t a, int32_t b) {
    auto r = align_batch(mode, {{s1, s2}}, score, a, b);
    const PairAlignment& p = r[0];
    switch (p.status) {
      case BG_OK: return Alignment(p.score, p.aligned1, p.aligned2);
      case BG_INVALID_ARGUMENT_RANGE: return BioError::InvalidArgumentRange;
      case BG_INVALID_INPUT_SIZE: return BioError::InvalidInputSize;
      case BG_UNSCORABLE: throw ReferencePanic("score closure panics on an input byte");
      case BG_INTERNAL: throw std::runtime_error("biogarden_gpu: traceback recomputation timed out");
      default: throw ReferencePanic("the reference SequenceAligner panics or hangs on this input");
    }
  }

  bg_aligner* h_;
};

}  // namespace alignment

// ------------------------------------------------------------------ the DP's other callers
// The reference's free functions that are alignment DPs, on the same GPU kernels.  They take an
// explicit device handle (a SequenceAligner-owned bg_aligner would do as well); one call = one
// GPU batch.
namespace detail {
struct PairArrays {            // one pair as the C ABI's pointer / length arrays
  const uint8_t* p1[1];
  const uint8_t* p2[1];
  size_t n1[1], n2[1];
  PairArrays(const ds::Sequence& a, const ds::Sequence& b)
      : p1{a.chain.data()}, p2{b.chain.data()}, n1{a.chain.size()}, n2{b.chain.size()} {}
};
class Device {
 public:
  static bg_aligner* get() {
    static Device d;
    if (!d.h_) throw DeviceError(BG_E_HIP);
    return d.h_;
  }
 private:
  Device() : h_(bg_aligner_new(0)) {}
  ~Device() { if (h_) bg_aligner_free(h_); }
  bg_aligner* h_;
};
}  // namespace detail

namespace analysis {
namespace seq {
// analysis::seq::edit_distance (src/analysis/seq.rs:105-130)
inline Result<size_t> edit_distance(const ds::Sequence& seq1, const ds::Sequence& seq2) {
  detail::PairArrays a(seq1, seq2);
  uint64_t d = 0;
  check(bg_edit_distance_batch(detail::Device::get(), 1, a.p1, a.n1, a.p2, a.n2, &d));
  return Result<size_t>((size_t)d);
}
}  // namespace seq
}  // namespace analysis

namespace processing {
namespace patterns {
// processing::patterns::longest_common_subsequence (src/processing/patterns.rs:82-118)
inline ds::Sequence longest_common_subsequence(const ds::Sequence& seq1, const ds::Sequence& seq2) {
  detail::PairArrays a(seq1, seq2);
  std::vector<uint8_t> out(std::min(seq1.len(), seq2.len()) + 1);
  uint64_t off = 0, len = 0;
  check(bg_lcs_batch(detail::Device::get(), 1, a.p1, a.n1, a.p2, a.n2, out.data(), out.size(), &off, &len));
  return ds::Sequence(std::vector<uint8_t>(out.begin() + off, out.begin() + off + len));
}
// processing::patterns::shortest_common_supersequence (:198-235): both sequences interleaved
// around their LCS, residues differing from the next LCS residue first
inline ds::Sequence shortest_common_supersequence(const ds::Sequence& seq1, const ds::Sequence& seq2) {
  const ds::Sequence lcs = longest_common_subsequence(seq1, seq2);
  std::vector<uint8_t> out;
  size_t i = 0, j = 0;
  for (uint8_t c : lcs.chain) {
    while (i < seq1.len()) { const uint8_t x = seq1.chain[i++]; if (x == c) break; out.push_back(x); }
    while (j < seq2.len()) { const uint8_t x = seq2.chain[j++]; if (x == c) break; out.push_back(x); }
    out.push_back(c);
  }
  out.insert(out.end(), seq1.chain.begin() + i, seq1.chain.end());
  out.insert(out.end(), seq2.chain.begin() + j, seq2.chain.end());
  return ds::Sequence(std::move(out));
}
}  // namespace patterns
}  // namespace processing
}  // namespace biogarden
