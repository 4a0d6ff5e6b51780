/* The CPU oracle (oracle/refcpu.c) on random small pairs in every mode, scoring and gap setting,
 * through one reused reference-faithful aligner (its resizes, panics and stale-scratch answers)
 * and an exact-size one, for tests/test_sanitizers.py, which builds it with
 * -fsanitize=address,undefined.  Checks the invariants every answer must keep (equal string
 * lengths within n1 + n2, de-gapped strings are substrings of the inputs) and that both aligners
 * agree wherever the faithful one returns cleanly from a buffer it just resized. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/refcpu.h"

static unsigned long long st = 88172645463325252ull;
static unsigned rnd(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (unsigned)st; }

static int sub_of(const unsigned char* al, size_t L, const unsigned char* s, size_t n) {
  unsigned char* d = malloc(L + 1);
  size_t k = 0;
  for (size_t i = 0; i < L; ++i) if (al[i] != '-') d[k++] = al[i];
  int ok = 0;
  if (k <= n)
    for (size_t o = 0; o + k <= n && !ok; ++o) ok = memcmp(s + o, d, k) == 0;
  free(d);
  return ok;
}

int main(void) {
  or_scoring sc[2];
  or_scoring_builtin(0, &sc[0]);
  or_scoring_builtin(2, &sc[1]);
  const int gaps[][2] = {{-11, -1}, {-1, -2}, {-1, -1}, {-2, -2}, {0, 0}, {2, 1}};
  const size_t lens[] = {0, 1, 2, 5, 31, 64, 200, 1023, 1024, 1025};
  or_aligner* faithful = or_aligner_new();
  int runs = 0, agree = 0;
  for (int it = 0; it < 400; ++it) {
    const size_t n1 = lens[rnd() % 10], n2 = lens[rnd() % 10];
    unsigned char* s1 = malloc(n1 + 1);
    unsigned char* s2 = malloc(n2 + 1);
    const char* alpha = (rnd() % 4) ? "ACGT" : "ACDEFGHIKLMNPQRSTVWYBZX";
    const size_t na = strlen(alpha);
    for (size_t i = 0; i < n1; ++i) s1[i] = (unsigned char)alpha[rnd() % na];
    for (size_t i = 0; i < n2; ++i) s2[i] = (rnd() % 3 && i < n1) ? s1[i] : (unsigned char)alpha[rnd() % na];
    if (rnd() % 50 == 0 && n1) s1[rnd() % n1] = 'a';          /* unscorable byte */
    const int mode = (int)(rnd() % 5), g = (int)(rnd() % 6);
    const or_scoring* S = &sc[rnd() % 2];
    unsigned char* o1 = malloc(n1 + n2 + 1);
    unsigned char* o2 = malloc(n1 + n2 + 1);
    unsigned char* e1 = malloc(n1 + n2 + 1);
    unsigned char* e2 = malloc(n1 + n2 + 1);
    size_t r0 = 0, c0 = 0;
    or_buffer_size(faithful, &r0, &c0);
    int32_t fs = 0, es = 0;
    size_t fl = 0, el = 0;
    const int fst = or_align(faithful, mode, s1, n1, s2, n2, S, gaps[g][0], gaps[g][1], &fs, o1, o2, &fl);
    or_aligner* exact = or_aligner_new_exact();
    const int est = or_align(exact, mode, s1, n1, s2, n2, S, gaps[g][0], gaps[g][1], &es, e1, e2, &el);
    or_aligner_free(exact);
    if (est == OR_OK) {
      if (el > n1 + n2 || !sub_of(e1, el, s1, n1) || !sub_of(e2, el, s2, n2)) {
        fprintf(stderr, "bad exact answer it=%d mode=%d n=%zu,%zu\n", it, mode, n1, n2);
        return 1;
      }
    }
    if (fst == OR_OK && fl > n1 + n2) { fprintf(stderr, "bad faithful length\n"); return 1; }
    /* a faithful call that resized to exactly (n1+1, n2+1) is the exact-size DP */
    if (fst == OR_OK && (n1 > r0 || n2 > c0) && est == OR_OK) {
      if (fs != es || fl != el || memcmp(o1, e1, el) || memcmp(o2, e2, el)) {
        fprintf(stderr, "faithful != exact after a resize it=%d mode=%d\n", it, mode);
        return 1;
      }
      ++agree;
    }
    ++runs;
    free(s1); free(s2); free(o1); free(o2); free(e1); free(e2);
  }
  or_aligner_free(faithful);
  printf("oracle fuzz ok (%d runs, %d resized agreements)\n", runs, agree);
  return 0;
}
