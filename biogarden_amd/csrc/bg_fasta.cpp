// Streaming FASTA reader behind the C ABI (include/biogarden_gpu.h, bg_fasta_*): the ingest side
// of the batch aligner.  Records come out in batches, their residues packed back to back in one
// reader-owned buffer with an offset per record, ready to hand to bg_batch_prepare as pointer +
// length arrays without a per-record allocation.
//
// Record semantics are the reference reader's (src/io/fasta.rs:95-135):
//   * a record starts at a line beginning with '>' (else the read fails: "Expected > at record
//     start.");
//   * the header after '>' is trim_end'ed and split once at its first whitespace character:
//     id = the part before it, desc = the rest (absent when the header has no whitespace);
//   * the sequence is the concatenation of the following lines, each trim_end'ed, up to EOF or
//     the next line beginning with '>';
//   * read_all (:125-135) stops at the first empty record (no id, no desc, no residues), which is
//     also what EOF returns.
// Whitespace is Rust's char::is_whitespace (Unicode White_Space) on UTF-8 text.  Every line is
// UTF-8 validated as BufRead::read_line does (:97, :115): an invalid line fails the read with
// BG_E_UTF8 (io::ErrorKind::InvalidData, "stream did not contain valid UTF-8").
//
// Input is read in large blocks (BG_FASTA_BLOCK bytes, default 4 MiB) and split into lines with
// memchr; a line spanning two blocks is carried over.
#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "biogarden_gpu.h"

namespace {

// byte length of the Unicode White_Space character starting at p (< end), or 0
inline size_t ws_at(const uint8_t* p, const uint8_t* end) {
  const uint8_t c = p[0];
  if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
  if (c == 0xC2 && p + 1 < end && (p[1] == 0x85 || p[1] == 0xA0)) return 2;
  if (p + 2 < end) {
    if (c == 0xE1 && p[1] == 0x9A && p[2] == 0x80) return 3;                     // U+1680
    if (c == 0xE2 && p[1] == 0x80 && ((p[2] >= 0x80 && p[2] <= 0x8A) || p[2] == 0xA8 ||
                                      p[2] == 0xA9 || p[2] == 0xAF)) return 3;    // U+2000-200A, 2028, 2029, 202F
    if (c == 0xE2 && p[1] == 0x81 && p[2] == 0x9F) return 3;                     // U+205F
    if (c == 0xE3 && p[1] == 0x80 && p[2] == 0x80) return 3;                     // U+3000
  }
  return 0;
}

// str::from_utf8's rules (no overlong forms, no surrogates, nothing above U+10FFFF)
inline bool utf8_valid(const uint8_t* p, size_t n) {
  size_t i = 0;
  while (i < n) {
    // ASCII fast path, 8 bytes at a time
    while (i + 8 <= n) {
      uint64_t w;
      std::memcpy(&w, p + i, 8);
      if (w & 0x8080808080808080ull) break;
      i += 8;
    }
    if (i >= n) break;
    const uint8_t c = p[i];
    if (c < 0x80) { ++i; continue; }
    size_t len;
    uint8_t lo = 0x80, hi = 0xBF;                      // bounds of the second byte
    if (c >= 0xC2 && c <= 0xDF) len = 2;
    else if (c == 0xE0) { len = 3; lo = 0xA0; }
    else if (c == 0xED) { len = 3; hi = 0x9F; }
    else if (c >= 0xE1 && c <= 0xEF) len = 3;
    else if (c == 0xF0) { len = 4; lo = 0x90; }
    else if (c == 0xF4) { len = 4; hi = 0x8F; }
    else if (c >= 0xF1 && c <= 0xF3) len = 4;
    else return false;
    if (i + len > n || p[i + 1] < lo || p[i + 1] > hi) return false;
    for (size_t k = 2; k < len; ++k)
      if ((p[i + k] & 0xC0) != 0x80) return false;
    i += len;
  }
  return true;
}

// str::trim_end: the length of [b, e) without its trailing whitespace characters
inline size_t trim_end_len(const uint8_t* b, const uint8_t* e) {
  while (e > b) {
    const uint8_t c = e[-1];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) { --e; continue; }
    if (e - b >= 2 && ws_at(e - 2, e) == 2) { e -= 2; continue; }
    if (e - b >= 3 && ws_at(e - 3, e) == 3) { e -= 3; continue; }
    break;
  }
  return (size_t)(e - b);
}

}  // namespace

struct bg_fasta {
  FILE* f = nullptr;
  std::vector<uint8_t> blk;        // current input block
  size_t pos = 0, len = 0;
  bool eof = false;
  std::string carry;               // a line split over two blocks
  std::string pending;             // the header line read ahead (fasta.rs `self.line`)
  bool havePending = false;
  bool done = false;               // an empty record was returned: read_all has stopped
  // the last batch
  std::vector<uint8_t> seq;
  std::vector<uint64_t> seqOff, idOff, descOff;
  std::vector<uint8_t> hasDesc;
  std::vector<char> text;          // ids and descriptions, each NUL-terminated

  // next line (including its '\n' when present) into `out`; false at EOF with nothing read
  bool next_line(std::string& out) {
    out.clear();
    for (;;) {
      if (pos >= len) {
        if (eof) return !out.empty();
        len = std::fread(blk.data(), 1, blk.size(), f);
        pos = 0;
        if (len == 0) { eof = true; return !out.empty(); }
      }
      const uint8_t* b = blk.data() + pos;
      const uint8_t* nl = static_cast<const uint8_t*>(std::memchr(b, '\n', len - pos));
      if (nl) {
        out.append(reinterpret_cast<const char*>(b), (size_t)(nl - b) + 1);
        pos += (size_t)(nl - b) + 1;
        return true;
      }
      out.append(reinterpret_cast<const char*>(b), len - pos);
      pos = len;
    }
  }
};

extern "C" bg_fasta* bg_fasta_open(const char* path, int* err) {
  if (err) *err = 0;
  if (!path) { if (err) *err = BG_E_ARG; return nullptr; }
  FILE* f = std::fopen(path, "rb");
  if (!f) { if (err) *err = BG_E_IO; return nullptr; }
  bg_fasta* r = new bg_fasta;
  r->f = f;
  size_t block = 4u << 20;
  if (const char* e = std::getenv("BG_FASTA_BLOCK")) block = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
  r->blk.resize(block);
  return r;
}

extern "C" void bg_fasta_close(bg_fasta* r) {
  if (!r) return;
  if (r->f) std::fclose(r->f);
  delete r;
}

extern "C" long bg_fasta_next_batch(bg_fasta* r, size_t max_records, size_t max_residues,
                                    bg_fasta_batch* out) {
  // max_residues == 0 could never hold a record: refused rather than read as end of file
  if (!r || !out || max_records == 0 || max_residues == 0) return BG_E_ARG;
  r->seq.clear();
  r->text.clear();
  r->seqOff.assign(1, 0);
  r->idOff.clear();
  r->descOff.clear();
  r->hasDesc.clear();
  std::string line;
  size_t n = 0;
  while (!r->done && n < max_records && r->seq.size() < max_residues) {
    // Reader::read (fasta.rs:95-123)
    if (!r->havePending) {
      if (!r->next_line(r->pending)) { r->done = true; break; }   // EOF: the empty record
      r->havePending = true;
    }
    const std::string& hl = r->pending;
    if (!utf8_valid(reinterpret_cast<const uint8_t*>(hl.data()), hl.size())) return BG_E_UTF8;
    if (hl.empty() || hl[0] != '>') return BG_E_FORMAT;            // "Expected > at record start."
    const uint8_t* hb = reinterpret_cast<const uint8_t*>(hl.data()) + 1;
    const uint8_t* he = hb + trim_end_len(hb, reinterpret_cast<const uint8_t*>(hl.data()) + hl.size());
    // splitn(2, char::is_whitespace)
    const uint8_t* cut = nullptr;
    size_t cutLen = 0;
    for (const uint8_t* p = hb; p < he; ++p)
      if ((cutLen = ws_at(p, he)) != 0) { cut = p; break; }
    const uint64_t idAt = r->text.size();
    r->text.insert(r->text.end(), hb, cut ? cut : he);
    r->text.push_back('\0');
    uint64_t descAt = r->text.size();
    if (cut) {
      r->text.insert(r->text.end(), cut + cutLen, he);
      r->text.push_back('\0');
    }
    const size_t seqAt = r->seq.size();
    r->havePending = false;
    for (;;) {
      if (!r->next_line(line)) break;
      // read_line fails on the line it reads, the next record's header included (:115)
      if (!utf8_valid(reinterpret_cast<const uint8_t*>(line.data()), line.size())) return BG_E_UTF8;
      if (line[0] == '>') { r->pending.swap(line); r->havePending = true; break; }
      const uint8_t* lb = reinterpret_cast<const uint8_t*>(line.data());
      r->seq.insert(r->seq.end(), lb, lb + trim_end_len(lb, lb + line.size()));
    }
    // Record::is_empty: read_all stops here (and would at EOF)
    if (idAt + 1 == r->text.size() && !cut && r->seq.size() == seqAt) {
      r->text.resize(idAt);
      r->done = true;
      break;
    }
    r->idOff.push_back(idAt);
    r->descOff.push_back(cut ? descAt : (uint64_t)-1);
    r->hasDesc.push_back(cut ? 1 : 0);
    r->seqOff.push_back(r->seq.size());
    ++n;
  }
  out->n = n;
  out->seq = r->seq.data();
  out->seq_off = r->seqOff.data();
  out->text = r->text.data();
  out->id_off = r->idOff.data();
  out->desc_off = r->descOff.data();
  return (long)n;
}
