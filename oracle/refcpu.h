/*
 * refcpu — CPU restatement of the reference aligner.  TEST INFRASTRUCTURE ONLY.
 *
 * This is the parity oracle for the MI355X aligner.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker (or as the timed
 * CPU baseline).  The product path (biogarden_amd / libbiogarden_gpu.so) never calls it.
 *
 * It restates, in plain C, the semantics of the reference Rust crate robsndr/biogarden
 * (src/alignment/aligner.rs, score.rs), INCLUDING its scratch-buffer model:
 *   - SequenceAligner::new() allocates six 1024x1024 matrices        (aligner.rs:44-55)
 *   - a call resizes ONLY when len1 > rows || len2 > cols, to (len1+1, len2+1) (:92-94, 594-602)
 *   - every matrix access is bounds-checked like ndarray (an out-of-bounds index = panic)
 *   - release-mode integer semantics: wrapping i32 adds, saturating add on the extend term
 * so it reproduces the reference's panics/hangs as status codes.  An "exact" aligner instead
 * allocates exactly (len1+1)x(len2+1) fresh buffers per call (border writes restricted to that
 * region): the product's documented semantics (DESIGN.md "Buffer semantics"), equal to the
 * reference wherever it returns.
 *
 * Parity pinning: the restatement reproduces the reference's 5 integration goldens
 * (tests/integration.rs:234-312, fixtures tests/golden/reference_fixtures/) and the 5 aligner
 * doctests (aligner.rs:75-82,141-148,206-214,281-288,342-349) byte for byte — see
 * tests/test_oracle.py.  The Rust reference itself cannot be compiled here (no cargo/rustc).
 */
#ifndef BIOGARDEN_REFCPU_H
#define BIOGARDEN_REFCPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_GLOBAL = 0, OR_LOCAL = 1, OR_FITTING = 2, OR_OVERLAP = 3, OR_SEMIGLOBAL = 4 };

enum {
  OR_OK = 0,
  OR_INVALID_ARGUMENT_RANGE = 1, /* BioError::InvalidArgumentRange */
  OR_INVALID_INPUT_SIZE = 2,     /* BioError::InvalidInputSize    */
  OR_PANIC_SCORE = 3,            /* score table index out of range -> panic (score.rs:40) */
  OR_PANIC_INDEX = 4,            /* matrix / sequence index out of bounds -> panic */
  OR_HANG = 5                    /* backtrack loops forever (aligner.rs:549 `_ => {}`) */
};

/* Scoring closure as data: code[byte] = 0..k-1, or 0xFF when the closure panics on it;
 * table[c1*32 + c2] = S(byte1, byte2).  Same layout as bg_scoring in include/biogarden_gpu.h.
 * wide_k > 0 instead tabulates a closure over up to 256 codes (the form of
 * bg_batch_prepare_table): wide_code[byte] (>= wide_k: panics), wide_table[c1*wide_k + c2]. */
typedef struct or_scoring {
  int32_t alphabet_size;
  uint8_t code[256];
  int32_t table[32 * 32];
  int32_t wide_k;
  const uint16_t* wide_code;
  const int32_t* wide_table;
} or_scoring;

typedef struct or_aligner or_aligner;

or_aligner* or_aligner_new(void);        /* reference SequenceAligner::new()  */
or_aligner* or_aligner_new_exact(void);  /* product semantics: exact-size buffers per call */
or_aligner* or_aligner_new_dims(size_t rows, size_t cols);  /* reference aligner after a resize */
void or_aligner_free(or_aligner* A);
void or_buffer_size(const or_aligner* A, size_t* rows, size_t* cols);

/* 0 = blosum62, 1 = pam250, 2 = unit (score.rs:38,78,114) */
void or_scoring_builtin(int which, or_scoring* out);

/* Runs one alignment.  out1/out2 need capacity n1+n2.  Returns an OR_* status. */
int or_align(or_aligner* A, int mode, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
             const or_scoring* sc, int32_t a, int32_t b, int32_t* score, uint8_t* out1,
             uint8_t* out2, size_t* out_len);

/* CPU baseline: align npairs pairs (one aligner per thread, pairs taken dynamically) on
 * nthreads threads; exact=0 uses reference-style reused aligners.  Returns seconds. */
double or_align_batch(int mode, size_t npairs, const uint8_t* const* s1, const size_t* n1,
                      const uint8_t* const* s2, const size_t* n2, const or_scoring* sc, int32_t a,
                      int32_t b, int nthreads, int exact, int32_t* scores, int* statuses);

/* analysis::seq::edit_distance (src/analysis/seq.rs:105-130) */
uint64_t or_edit_distance(const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2);
/* processing::patterns::longest_common_subsequence (src/processing/patterns.rs:82-118);
 * out capacity >= min(n1, n2); returns the subsequence length */
size_t or_lcs(const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
