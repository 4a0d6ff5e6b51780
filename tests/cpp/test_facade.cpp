// CPU checks of the C++ facade (include/biogarden.hpp): data types, FASTA, scoring, errors.
// No GPU needed: bg_scoring_builtin touches no device; bg_aligner_new fails cleanly without one.
#include <cstdio>
#include <sstream>

#include "biogarden.hpp"

using namespace biogarden;

static int fails = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

int main(int argc, char** argv) {
  const std::string fix = argc > 1 ? argv[1] : "tests/golden/reference_fixtures";
  // Sequence: equality ignores id (sequence.rs:113-117)
  ds::Sequence a("ACGT"), b(std::vector<uint8_t>{'A', 'C', 'G', 'T'}, "x");
  CHECK(a == b);
  b.push('A');
  CHECK(a != b && b.len() == 5);
  b.reverse();
  CHECK(b.to_string() == "ATGCA");

  // FASTA (fasta.rs:95-135): id/desc split, trimmed lines, '>' required
  {
    std::istringstream in(">id1 some desc  \nACG \nTT\r\n>id2\n\n>id3\tx y\nG\n");
    io::fasta::Reader r(in);
    auto recs = r.read_all();
    CHECK(recs.size() == 3);
    CHECK(recs[0].id == "id1" && recs[0].desc && *recs[0].desc == "some desc");
    CHECK(std::string(recs[0].seq.begin(), recs[0].seq.end()) == "ACGTT");
    CHECK(recs[1].id == "id2" && !recs[1].desc && recs[1].seq.empty());
    CHECK(recs[2].id == "id3" && *recs[2].desc == "x y");
    std::istringstream bad("ACGT\n");
    io::fasta::Reader rb(bad);
    io::fasta::Record rec;
    bool threw = false;
    try { rb.read(rec); } catch (const std::ios_base::failure&) { threw = true; }
    CHECK(threw);
  }
  for (const char* name : {"global", "local", "fitting", "overlap", "semiglobal"}) {
    auto in = io::fasta::read_tile(fix + "/input/" + name + "_alignment.fasta");
    auto out = io::fasta::read_tile(fix + "/output/" + name + "_alignment.fasta");
    CHECK(in.len() == 2 && out.len() == 2);
    CHECK(out[0].len() == out[1].len());
  }

  // score (score.rs): table values, panics outside 'A'..'Z'
  CHECK(score::blosum62('A', 'A') == 4 && score::blosum62('C', 'C') == 9 && score::blosum62('W', 'W') == 11);
  CHECK(score::blosum62('C', 'G') == -3 && score::unit('A', 'A') == 1 && score::unit('A', 'C') == -1);
  bool panicked = false;
  try { score::blosum62('a', 'A'); } catch (const ReferencePanic&) { panicked = true; }
  CHECK(panicked);
  // tabulate: built-ins skip the closure, other callables are evaluated per (seq1, seq2) byte
  {
    std::vector<uint8_t> s1{'A', 'C'}, s2{'G', '*'}, s3{'G'};
    std::vector<score::PairRef> v{{&s1, &s2}};
    score::Tabulated t = score::tabulate(score::blosum62, v);
    CHECK(t.sc.alphabet_size == 26 && t.panics.empty());
    score::ScoreFn f = [](const uint8_t& x, const uint8_t& y) -> int32_t {
      if (x == 'A' && y == '*') throw std::out_of_range("panic");
      return x == y ? 3 : -2;
    };
    score::Tabulated c = score::tabulate(f, v);
    CHECK(c.sc.alphabet_size == 4 && c.panics.size() == 1);
    CHECK(c.sc.table[c.sc.code['C'] * 32 + c.sc.code['G']] == -2);
    CHECK(score::pair_panics(c, s1, s2) && !score::pair_panics(c, s1, s3));
    // more than 32 distinct bytes: the k x k form for bg_batch_prepare_table
    std::vector<uint8_t> w1, w2{'!'};
    for (int i = 0; i < 40; ++i) w1.push_back((uint8_t)(100 + i));
    std::vector<score::PairRef> vw{{&w1, &w2}};
    score::Tabulated wt = score::tabulate(f, vw);
    CHECK(wt.wide && wt.k == 41 && wt.code.size() == 256 && wt.table.size() == 41u * 41u);
    CHECK(wt.code['!'] == 0 && wt.code[100] == 1 && wt.code['A'] == 0xFFFF);
    CHECK(wt.table[(size_t)wt.code[100] * wt.k + wt.code['!']] == -2);
  }

  // Result / errors
  Result<int> ok(5), err(BioError::InvalidInputSize);
  CHECK(ok.is_ok() && ok.unwrap() == 5 && err.is_err() && err.error() == BioError::InvalidInputSize);
  CHECK(bg_abi_version() == BG_ABI_VERSION);

  // without a GPU the aligner cannot be created: a DeviceError, never a CPU fallback
  if (argc > 2 && std::string(argv[2]) == "--no-gpu") {
    bool dev = false;
    try { alignment::SequenceAligner al(0); } catch (const DeviceError&) { dev = true; }
    CHECK(dev);
  }
  std::printf("%s (%d failures)\n", fails ? "FAILED" : "facade ok", fails);
  return fails ? 1 : 0;
}
