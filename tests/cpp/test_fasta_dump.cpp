// Dumps every record the native FASTA batch reader (biogarden_amd/csrc/bg_fasta.cpp) returns, for
// tests/test_sanitizers.py, which builds it with -fsanitize=address,undefined around the reader's
// sources and compares the dump with the Python mirror of the reference reader (fasta.rs:95-135).
//   test_fasta_dump FILE MAX_RECORDS MAX_RESIDUES
// One line per record: id, TAB, description or "-", TAB, residues; "ERR <code>" on an error.
#include <cstdio>
#include <cstdlib>

#include "biogarden_gpu.h"

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  int err = 0;
  bg_fasta* r = bg_fasta_open(argv[1], &err);
  if (!r) { std::printf("ERR %d\n", err); return 0; }
  const size_t maxr = std::strtoull(argv[2], nullptr, 10), maxres = std::strtoull(argv[3], nullptr, 10);
  for (;;) {
    bg_fasta_batch b;
    const long n = bg_fasta_next_batch(r, maxr, maxres, &b);
    if (n < 0) { std::printf("ERR %ld\n", n); break; }
    if (n == 0) break;
    for (long k = 0; k < n; ++k) {
      std::fputs(b.text + b.id_off[k], stdout);
      std::fputc('\t', stdout);
      std::fputs(b.desc_off[k] == (uint64_t)-1 ? "-" : b.text + b.desc_off[k], stdout);
      std::fputc('\t', stdout);
      const size_t len = b.seq_off[k + 1] - b.seq_off[k];
      if (len) std::fwrite(b.seq + b.seq_off[k], 1, len, stdout);   // seq may be NULL when empty
      std::fputc('\n', stdout);
    }
  }
  bg_fasta_close(r);
  return 0;
}
