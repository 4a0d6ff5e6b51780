// The reference's alignment integration tests (tests/integration.rs:234-312) through the C++
// facade on the GPU: same inputs, same calls, same expected scores and aligned strings.
#include <cstdio>

#include "biogarden.hpp"

using namespace biogarden;

int main(int argc, char** argv) {
  const std::string fix = argc > 1 ? argv[1] : "tests/golden/reference_fixtures";
  int fails = 0;
  alignment::SequenceAligner aligner(0);   // SequenceAligner::new()
  struct Case {
    const char* name;
    score::ScoreFn scoring;
    int32_t a, b, expect;
  } cases[] = {
      {"global", score::blosum62, -11, -1, 232},
      {"local", score::blosum62, -11, -1, 20431},
      {"fitting", score::unit, -1, -1, 145},
      {"overlap", score::unit, -2, -2, 698},
      {"semiglobal", score::unit, -1, -1, 982},
  };
  for (auto& c : cases) {
    auto inputs = io::fasta::read_tile(fix + "/input/" + c.name + "_alignment.fasta");
    auto outputs = io::fasta::read_tile(fix + "/output/" + c.name + "_alignment.fasta");
    const std::string n = c.name;
    auto r = n == "global"    ? aligner.global_alignment(inputs[0], inputs[1], c.scoring, c.a, c.b)
             : n == "local"   ? aligner.local_alignment(inputs[0], inputs[1], c.scoring, c.a, c.b)
             : n == "fitting" ? aligner.fitting_alignment(inputs[0], inputs[1], c.scoring, c.a, c.b)
             : n == "overlap" ? aligner.overlap_alignment(inputs[0], inputs[1], c.scoring, c.a, c.b)
                              : aligner.semiglobal_alignment(inputs[0], inputs[1], c.scoring, c.a, c.b);
    const auto& [score, s1, s2] = r.unwrap();
    const bool ok = score == c.expect && s1 == outputs[0] && s2 == outputs[1];
    std::printf("%-10s score %d (expect %d) %s\n", c.name, score, c.expect, ok ? "ok" : "MISMATCH");
    fails += !ok;
  }
  // error behaviour (aligner.rs:87-89, 223-225)
  auto e1 = aligner.global_alignment(ds::Sequence("ACGT"), ds::Sequence("ACG"), score::blosum62, 1, -1);
  auto e2 = aligner.fitting_alignment(ds::Sequence("AC"), ds::Sequence("ACG"), score::unit, -1, -1);
  fails += !(e1.is_err() && e1.error() == BioError::InvalidArgumentRange);
  fails += !(e2.is_err() && e2.error() == BioError::InvalidInputSize);
  bool panicked = false;
  try { aligner.global_alignment(ds::Sequence("ACgT"), ds::Sequence("ACG"), score::blosum62, -1, -1); }
  catch (const ReferencePanic&) { panicked = true; }
  fails += !panicked;
  // tests/integration.rs:69-74 and :135-149 (edit distance, LCS, SCS)
  {
    auto ed = io::fasta::read_tile(fix + "/input/edit_distance.fasta");
    const size_t d = analysis::seq::edit_distance(ed[0], ed[1]).unwrap();
    std::printf("edit_distance %zu (expect 299)\n", d);
    fails += d != 299;
    auto li = io::fasta::read_tile(fix + "/input/longest_common_subseq.fasta");
    auto lo = io::fasta::read_tile(fix + "/output/longest_common_subseq.fasta");
    const bool lok = processing::patterns::longest_common_subsequence(li[0], li[1]) == lo[0];
    auto si = io::fasta::read_tile(fix + "/input/shortest_common_superseq.fasta");
    auto so = io::fasta::read_tile(fix + "/output/shortest_common_superseq.fasta");
    const bool sok = processing::patterns::shortest_common_supersequence(si[0], si[1]) == so[0];
    std::printf("lcs %s scs %s\n", lok ? "ok" : "MISMATCH", sok ? "ok" : "MISMATCH");
    fails += !lok + !sok;
  }
  // a closure over more than 32 distinct bytes (score.rs:38-41 takes any &dyn Fn): the facade
  // tabulates it k x k for bg_batch_prepare_table.  40 distinct bytes, seq2 = seq1 less byte 17:
  // the one optimal global alignment opens one gap there (score 5 * 39 + a)
  {
    std::vector<uint8_t> x;
    for (int i = 0; i < 40; ++i) x.push_back((uint8_t)(200 + i));
    std::vector<uint8_t> y(x);
    y.erase(y.begin() + 17);
    score::ScoreFn f = [](const uint8_t& p, const uint8_t& q) -> int32_t { return p == q ? 5 : -4; };
    auto r = aligner.global_alignment(ds::Sequence(x), ds::Sequence(y), f, -11, -1);
    const auto& [sc, a1, a2] = r.unwrap();
    std::vector<uint8_t> gy(y);
    gy.insert(gy.begin() + 17, (uint8_t)'-');
    const bool wok = sc == 5 * 39 - 11 && a1 == ds::Sequence(x) && a2 == ds::Sequence(gy);
    std::printf("wide alphabet score %d (expect %d) %s\n", sc, 5 * 39 - 11, wok ? "ok" : "MISMATCH");
    fails += !wok;
  }
  std::printf("%s\n", fails ? "FAILED" : "integration ok");
  return fails ? 1 : 0;
}
