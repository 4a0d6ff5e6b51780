/*
 * refcpu.c — CPU restatement of robsndr/biogarden's SequenceAligner.  TEST INFRASTRUCTURE ONLY
 * (parity oracle + timed CPU baseline); see refcpu.h for the rules and the pinning evidence.
 *
 * Every function cites the reference lines it restates (paths relative to the reference root).
 */
#include "refcpu.h"

#include <pthread.h>
#include <setjmp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "score_tables.inc"

struct or_aligner {
  size_t rows, cols;            /* buffer_size (aligner.rs:30) */
  int32_t *m, *x, *y;           /* cost buffers (:32-34) */
  uint8_t *mt, *xt, *yt;        /* trace buffers (:36-38) */
  int exact;
  jmp_buf jb;
};

/* ---------------------------------------------------------------- helpers ------------ */

static void or_panic(or_aligner* A, int code) { longjmp(A->jb, code); }

/* Release-mode `+` on i32 wraps (Cargo.toml has no overflow-checks profile). */
static inline int32_t wadd(int32_t p, int32_t q) { return (int32_t)((uint32_t)p + (uint32_t)q); }
/* i32::saturating_add (aligner.rs:443,447,477,483). */
static inline int32_t sadd(int32_t p, int32_t q) {
  int64_t s = (int64_t)p + (int64_t)q;
  return s > INT32_MAX ? INT32_MAX : (s < INT32_MIN ? INT32_MIN : (int32_t)s);
}
static inline int32_t imax(int32_t p, int32_t q) { return p > q ? p : q; }

/* ndarray [[i,j]] on a (rows, cols) standard-layout array: bounds-checked, row-major. */
static inline size_t IX(or_aligner* A, size_t i, size_t j) {
  if (i >= A->rows || j >= A->cols) or_panic(A, OR_PANIC_INDEX);
  return i * A->cols + j;
}
/* Sequence Index (sequence.rs:119-127): Vec indexing, panics out of range. `k - 1` with k == 0
 * wraps to usize::MAX in release mode, which is out of range too. */
static inline uint8_t SQ(or_aligner* A, const uint8_t* s, size_t n, size_t idx_plus_1_minus_1) {
  if (idx_plus_1_minus_1 >= n) or_panic(A, OR_PANIC_INDEX);
  return s[idx_plus_1_minus_1];
}
/* score closure, e.g. blosum62 (score.rs:38-41): table[(a-65),(b-65)], panics outside 'A'..'Z'. */
static inline int32_t SC(or_aligner* A, const or_scoring* sc, uint8_t p, uint8_t q) {
  if (sc->wide_k > 0) {
    const int k = sc->wide_k, wp = sc->wide_code[p], wq = sc->wide_code[q];
    if (wp >= k || wq >= k) or_panic(A, OR_PANIC_SCORE);
    return sc->wide_table[(size_t)wp * k + wq];
  }
  uint8_t cp = sc->code[p], cq = sc->code[q];
  if (cp == 0xFF || cq == 0xFF) or_panic(A, OR_PANIC_SCORE);
  return sc->table[cp * 32 + cq];
}

static void free_buffers(or_aligner* A) {
  free(A->m); free(A->x); free(A->y); free(A->mt); free(A->xt); free(A->yt);
  A->m = A->x = A->y = NULL; A->mt = A->xt = A->yt = NULL;
}

/* resize_buffers (aligner.rs:594-602) / new (:44-55): m = 0, x = y = i32::MIN, m_trace = 0,
 * x_trace = y_trace = 'I'. */
static int alloc_buffers(or_aligner* A, size_t r, size_t c) {
  free_buffers(A);
  size_t N = r * c;
  A->rows = r; A->cols = c;
  A->m = (int32_t*)calloc(N ? N : 1, 4);
  A->x = (int32_t*)malloc((N ? N : 1) * 4);
  A->y = (int32_t*)malloc((N ? N : 1) * 4);
  A->mt = (uint8_t*)calloc(N ? N : 1, 1);
  A->xt = (uint8_t*)malloc(N ? N : 1);
  A->yt = (uint8_t*)malloc(N ? N : 1);
  if (!A->m || !A->x || !A->y || !A->mt || !A->xt || !A->yt) return -1;
  for (size_t t = 0; t < N; ++t) { A->x[t] = INT32_MIN; A->y[t] = INT32_MIN; }
  memset(A->xt, 'I', N);
  memset(A->yt, 'I', N);
  return 0;
}

or_aligner* or_aligner_new(void) {
  or_aligner* A = (or_aligner*)calloc(1, sizeof(or_aligner));
  if (!A) return NULL;
  if (alloc_buffers(A, 1024, 1024)) { free_buffers(A); free(A); return NULL; }
  return A;
}

/* A reference aligner whose scratch is rows x cols (as after resize_buffers(rows, cols),
 * aligner.rs:594-602): the state a reused SequenceAligner reaches; tests mirror a product
 * handle's modelled history with it. */
or_aligner* or_aligner_new_dims(size_t rows, size_t cols) {
  or_aligner* A = (or_aligner*)calloc(1, sizeof(or_aligner));
  if (!A) return NULL;
  if (alloc_buffers(A, rows, cols)) { free_buffers(A); free(A); return NULL; }
  return A;
}

or_aligner* or_aligner_new_exact(void) {
  or_aligner* A = or_aligner_new();
  if (A) A->exact = 1;
  return A;
}

void or_aligner_free(or_aligner* A) {
  if (!A) return;
  free_buffers(A);
  free(A);
}

void or_buffer_size(const or_aligner* A, size_t* rows, size_t* cols) {
  *rows = A->rows; *cols = A->cols;
}

void or_scoring_builtin(int which, or_scoring* out) {
  const int* T = which == 0 ? BLOSUM62_COLMAJOR : which == 1 ? PAM250_COLMAJOR : UNIT_COLMAJOR;
  memset(out, 0, sizeof(*out));
  out->alphabet_size = 26;
  memset(out->code, 0xFF, 256);
  for (int c = 0; c < 26; ++c) out->code['A' + c] = (uint8_t)c;
  for (int r = 0; r < 26; ++r)
    for (int c = 0; c < 26; ++c) out->table[r * 32 + c] = T[c * 26 + r];
}

/* "Allocate a larger buffer if sequences cannot fit" (aligner.rs:92-94 and its copies). */
static void maybe_resize(or_aligner* A, size_t n1, size_t n2) {
  if (A->exact || n1 > A->rows || n2 > A->cols)
    if (alloc_buffers(A, n1 + 1, n2 + 1)) or_panic(A, OR_PANIC_INDEX);
}

/* m_trace.column_mut(0).fill('X'); m_trace.row_mut(0).fill('Y') (e.g. aligner.rs:107-108). */
static void trace_borders(or_aligner* A) {
  for (size_t i = 0; i < A->rows; ++i) A->mt[i * A->cols] = 'X';
  memset(A->mt, 'Y', A->cols);
}

/* ---------------------------------------------------------------- DP ----------------- */

/* compute_scores_global (aligner.rs:437-469) and compute_scores_local (:471-509).
 * Checked variant: literal restatement with every index bounds-checked, in program order. */
static void dp_checked(or_aligner* A, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
                       const or_scoring* sc, int32_t a, int32_t b, int local) {
  for (size_t i = 1; i < n1 + 1; ++i) {
    for (size_t j = 1; j < n2 + 1; ++j) {
      int32_t xo = wadd(A->m[IX(A, i - 1, j)], a);
      int32_t xv = imax(xo, sadd(A->x[IX(A, i - 1, j)], b));
      A->x[IX(A, i, j)] = xv;
      A->xt[IX(A, i, j)] = (xv == wadd(A->m[IX(A, i - 1, j)], a)) ? 'M' : 'I';
      if (local) A->x[IX(A, i, j)] = xv < 0 ? 0 : xv;          /* :480 */
      int32_t yo = wadd(A->m[IX(A, i, j - 1)], a);
      int32_t yv = imax(yo, sadd(A->y[IX(A, i, j - 1)], b));
      A->y[IX(A, i, j)] = yv;
      A->yt[IX(A, i, j)] = (yv == wadd(A->m[IX(A, i, j - 1)], a)) ? 'M' : 'I';
      if (local) A->y[IX(A, i, j)] = yv < 0 ? 0 : yv;          /* :486 */
      int32_t d = wadd(A->m[IX(A, i - 1, j - 1)], SC(A, sc, SQ(A, s1, n1, i - 1), SQ(A, s2, n2, j - 1)));
      int32_t X = A->x[IX(A, i, j)], Y = A->y[IX(A, i, j)];
      int32_t best = imax(d, imax(X, Y));
      A->mt[IX(A, i, j)] = best == Y ? 'Y' : (best == X ? 'X' : 'R');   /* :455-463 */
      A->m[IX(A, i, j)] = (local && best < 0) ? 0 : best;           /* :466 / :506 */
    }
  }
}

/* Fast variant, valid when every index of the loop nest is in bounds and every byte scores. */
static void dp_fast(or_aligner* A, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
                    const or_scoring* sc, int32_t a, int32_t b, int local) {
  const size_t C = A->cols;
  uint8_t* c2 = (uint8_t*)malloc(n2 + 1);
  for (size_t j = 0; j < n2; ++j) c2[j] = sc->code[s2[j]];
  for (size_t i = 1; i <= n1; ++i) {
    const int32_t* Mp = A->m + (i - 1) * C;
    int32_t* Mc = A->m + i * C;
    const int32_t* Xp = A->x + (i - 1) * C;
    int32_t* Xc = A->x + i * C;
    int32_t* Yc = A->y + i * C;
    uint8_t* MTc = A->mt + i * C;
    uint8_t* XTc = A->xt + i * C;
    uint8_t* YTc = A->yt + i * C;
    const int32_t* row = sc->table + 32 * sc->code[s1[i - 1]];
    for (size_t j = 1; j <= n2; ++j) {
      int32_t xo = wadd(Mp[j], a);
      int32_t xv = imax(xo, sadd(Xp[j], b));
      XTc[j] = xv == xo ? 'M' : 'I';
      int32_t yo = wadd(Mc[j - 1], a);
      int32_t yv = imax(yo, sadd(Yc[j - 1], b));
      YTc[j] = yv == yo ? 'M' : 'I';
      if (local) { xv = xv < 0 ? 0 : xv; yv = yv < 0 ? 0 : yv; }
      Xc[j] = xv;
      Yc[j] = yv;
      int32_t d = wadd(Mp[j - 1], row[c2[j - 1]]);
      int32_t best = imax(d, imax(xv, yv));
      MTc[j] = best == yv ? 'Y' : (best == xv ? 'X' : 'R');
      Mc[j] = (local && best < 0) ? 0 : best;
    }
  }
  free(c2);
}

static void dp(or_aligner* A, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
               const or_scoring* sc, int32_t a, int32_t b, int local) {
  int fast = n1 < A->rows && n2 < A->cols && sc->wide_k == 0;   /* wide tables: checked loop */
  if (fast && n1 > 0 && n2 > 0) {
    for (size_t i = 0; i < n1 && fast; ++i) fast = sc->code[s1[i]] != 0xFF;
    for (size_t j = 0; j < n2 && fast; ++j) fast = sc->code[s2[j]] != 0xFF;
  }
  if (fast) dp_fast(A, s1, n1, s2, n2, sc, a, b, local);
  else dp_checked(A, s1, n1, s2, n2, sc, a, b, local);
}

/* ---------------------------------------------------------------- traceback ---------- */

typedef struct { uint8_t *o1, *o2; size_t len, cap; } outbuf;

static inline void push(or_aligner* A, outbuf* o, uint8_t c1, uint8_t c2) {
  if (o->len >= o->cap) or_panic(A, OR_PANIC_INDEX);  /* unreachable: every column consumes */
  o->o1[o->len] = c1; o->o2[o->len] = c2; o->len++;
}

enum { TV_GLOBAL, TV_LOCAL, TV_L_NONZERO, TV_KL_NONZERO };

static inline int trace_valid(or_aligner* A, int kind, size_t k, size_t l) {
  switch (kind) {
    case TV_GLOBAL: return k != 0 || l != 0;                                    /* :117 */
    case TV_LOCAL: return (k != 0 || l != 0) && A->m[IX(A, k, l)] > 0;          /* :181 */
    case TV_L_NONZERO: return l != 0;                                           /* :256,:317 */
    default: return k * l != 0;                                                 /* :409 */
  }
}

/* backtrack (aligner.rs:511-592).  Columns are pushed in walk (backward) order; the caller
 * reverses once at the end, which composes to the reference's reverse/extend sequence. */
static void backtrack(or_aligner* A, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
                      size_t* k, size_t* l, int kind, outbuf* o) {
  uint8_t cur = 'M';
  while (trace_valid(A, kind, *k, *l)) {
    if (cur == 'M') {
      uint8_t t = A->mt[IX(A, *k, *l)];
      if (t == 'R') {
        push(A, o, SQ(A, s1, n1, *k - 1), SQ(A, s2, n2, *l - 1));
        *k -= 1; *l -= 1;
      } else if (t == 'X') {
        cur = 'X';
        push(A, o, SQ(A, s1, n1, *k - 1), '-');
        *k -= 1;
      } else if (t == 'Y') {
        cur = 'Y';
        push(A, o, '-', SQ(A, s2, n2, *l - 1));
        *l -= 1;
      } else {
        or_panic(A, OR_HANG); /* `_ => {}` (:549): state and position never change again */
      }
    } else if (cur == 'X') {
      if (A->xt[IX(A, *k, *l)] == 'M') cur = 'M';
      else { push(A, o, SQ(A, s1, n1, *k - 1), '-'); *k -= 1; }
    } else {
      if (A->yt[IX(A, *k, *l)] == 'M') cur = 'M';
      else { push(A, o, '-', SQ(A, s2, n2, *l - 1)); *l -= 1; }
    }
  }
}

static void reverse_out(outbuf* o) {
  for (size_t i = 0, j = o->len; i + 1 < j; ++i, --j) {
    uint8_t t = o->o1[i]; o->o1[i] = o->o1[j - 1]; o->o1[j - 1] = t;
    t = o->o2[i]; o->o2[i] = o->o2[j - 1]; o->o2[j - 1] = t;
  }
}

/* ---------------------------------------------------------------- modes -------------- */

static int32_t run_mode(or_aligner* A, int mode, const uint8_t* s1, size_t n1, const uint8_t* s2,
                        size_t n2, const or_scoring* sc, int32_t a, int32_t b, outbuf* o) {
  size_t k = 0, l = 0;
  int32_t score = 0;
  switch (mode) {
    case OR_GLOBAL: {                                          /* aligner.rs:84-121 */
      maybe_resize(A, n1, n2);
      /* exact mode restricts the border writes to the pair's region: row0[1] / col0[1] of an
       * exactly (n1+1)x(n2+1) scratch do not exist when n2 == 0 / n1 == 0 */
      if (!(A->exact && n2 == 0)) A->m[IX(A, 0, 1)] = a;
      for (size_t j = 2; j < n2 + 1; ++j) A->m[IX(A, 0, j)] = wadd(A->m[IX(A, 0, j - 1)], b);
      if (!(A->exact && n1 == 0)) A->m[IX(A, 1, 0)] = a;
      for (size_t i = 2; i < n1 + 1; ++i) A->m[IX(A, i, 0)] = wadd(A->m[IX(A, i - 1, 0)], b);
      trace_borders(A);
      dp(A, s1, n1, s2, n2, sc, a, b, 0);
      score = A->m[IX(A, n1, n2)];
      k = n1; l = n2;
      backtrack(A, s1, n1, s2, n2, &k, &l, TV_GLOBAL, o);
      break;
    }
    case OR_LOCAL: {                                           /* :150-185 */
      maybe_resize(A, n1, n2);
      memset(A->m, 0, A->rows * A->cols * 4);
      trace_borders(A);
      dp(A, s1, n1, s2, n2, sc, a, b, 1);
      int32_t best = INT32_MIN;
      size_t bi = 0, bj = 0;
      for (size_t i = 0; i < A->rows; ++i)          /* indexed_iter fold, strict > (:173-174) */
        for (size_t j = 0; j < A->cols; ++j) {
          int32_t v = A->m[i * A->cols + j];
          if (v > best) { best = v; bi = i; bj = j; }
        }
      score = best;
      k = bi; l = bj;
      backtrack(A, s1, n1, s2, n2, &k, &l, TV_LOCAL, o);
      break;
    }
    case OR_FITTING: {                                         /* :216-260 */
      maybe_resize(A, n1, n2);
      memset(A->m, 0, A->rows * A->cols * 4);
      if (!(A->exact && n2 == 0)) A->m[IX(A, 0, 1)] = a;
      for (size_t j = 2; j < n2 + 1; ++j) A->m[IX(A, 0, j)] = wadd(A->m[IX(A, 0, j - 1)], b);
      trace_borders(A);
      dp(A, s1, n1, s2, n2, sc, a, b, 0);
      if (n2 >= A->cols) or_panic(A, OR_PANIC_INDEX);        /* column(n2) */
      int32_t best = INT32_MIN;
      size_t bi = 0;
      for (size_t i = 0; i < A->rows; ++i) {
        int32_t v = A->m[i * A->cols + n2];
        if (v > best) { best = v; bi = i; }
      }
      score = best;
      k = bi; l = n2;
      backtrack(A, s1, n1, s2, n2, &k, &l, TV_L_NONZERO, o);
      break;
    }
    case OR_OVERLAP: {                                         /* :290-321 */
      maybe_resize(A, n1, n2);
      memset(A->m, 0, A->rows * A->cols * 4);
      trace_borders(A);
      dp(A, s1, n1, s2, n2, sc, a, b, 0);
      if (n1 >= A->rows) or_panic(A, OR_PANIC_INDEX);        /* row(n1) */
      int32_t best = INT32_MIN;
      size_t bj = 0;
      for (size_t j = 0; j < A->cols; ++j) {
        int32_t v = A->m[n1 * A->cols + j];
        if (v >= best) { best = v; bj = j; }
      }
      score = best;
      k = n1; l = bj;
      backtrack(A, s1, n1, s2, n2, &k, &l, TV_L_NONZERO, o);
      break;
    }
    default: {                                                 /* semiglobal :351-435 */
      maybe_resize(A, n1, n2);
      memset(A->m, 0, A->rows * A->cols * 4);
      trace_borders(A);
      dp(A, s1, n1, s2, n2, sc, a, b, 0);
      if (n1 >= A->rows) or_panic(A, OR_PANIC_INDEX);
      int32_t mr = INT32_MIN; size_t mrj = 0;
      for (size_t j = 0; j < A->cols; ++j) {                   /* last row, >= (:369-371) */
        int32_t v = A->m[n1 * A->cols + j];
        if (v >= mr) { mr = v; mrj = j; }
      }
      if (n2 >= A->cols) or_panic(A, OR_PANIC_INDEX);
      int32_t mc = INT32_MIN; size_t mci = 0;
      for (size_t i = 0; i < A->rows; ++i) {                   /* last column, > (:376-378) */
        int32_t v = A->m[i * A->cols + n2];
        if (v > mc) { mc = v; mci = i; }
      }
      int colcase = mc > mr;                                   /* :389 */
      if (colcase) {
        k = mci; l = n2; score = mc;
        for (size_t i = n1; i >= mci + 1 && i > 0; --i) push(A, o, SQ(A, s1, n1, i - 1), '-');
      } else {
        k = n1; l = mrj; score = mr;
        for (size_t j = n2; j >= mrj + 1 && j > 0; --j) push(A, o, '-', SQ(A, s2, n2, j - 1));
      }
      backtrack(A, s1, n1, s2, n2, &k, &l, TV_KL_NONZERO, o);
      if (colcase) {                                           /* :417-422 */
        for (size_t i = k; i > 0; --i) push(A, o, SQ(A, s1, n1, i - 1), '-');
      } else {                                                 /* :423-428 */
        for (size_t j = l; j > 0; --j) push(A, o, '-', SQ(A, s2, n2, j - 1));
      }
      break;
    }
  }
  reverse_out(o);
  return score;
}

int or_align(or_aligner* A, int mode, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
             const or_scoring* sc, int32_t a, int32_t b, int32_t* score, uint8_t* out1,
             uint8_t* out2, size_t* out_len) {
  *score = 0;
  *out_len = 0;
  if (mode == OR_GLOBAL || mode == OR_LOCAL || mode == OR_FITTING)
    if (a > 0 || b > 0) return OR_INVALID_ARGUMENT_RANGE;      /* :87-89 ,:153-155, :219-221 */
  if (mode == OR_FITTING && n1 < n2) return OR_INVALID_INPUT_SIZE;   /* :223-225 */
  outbuf o = {out1, out2, 0, n1 + n2};
  volatile int32_t sres = 0;
  int code = setjmp(A->jb);
  if (code) { *out_len = 0; return code; }
  sres = run_mode(A, mode, s1, n1, s2, n2, sc, a, b, &o);
  *score = sres;
  *out_len = o.len;
  return OR_OK;
}

/* ---------------------------------------------------------------- CPU baseline ------- */

typedef struct {
  int mode; size_t npairs;
  const uint8_t* const* s1; const size_t* n1; const uint8_t* const* s2; const size_t* n2;
  const or_scoring* sc; int32_t a, b; int exact;
  int32_t* scores; int* statuses;
  size_t next; pthread_mutex_t mu;
} batch_ctx;

static void* batch_worker(void* p) {
  batch_ctx* B = (batch_ctx*)p;
  or_aligner* A = B->exact ? or_aligner_new_exact() : or_aligner_new();
  size_t cap = 0;
  uint8_t *o1 = NULL, *o2 = NULL;
  for (;;) {
    pthread_mutex_lock(&B->mu);
    size_t t = B->next++;
    pthread_mutex_unlock(&B->mu);
    if (t >= B->npairs) break;
    size_t need = B->n1[t] + B->n2[t] + 1;
    if (need > cap) {
      free(o1); free(o2);
      cap = need;
      o1 = (uint8_t*)malloc(cap); o2 = (uint8_t*)malloc(cap);
    }
    size_t len;
    int32_t sc;
    int st = or_align(A, B->mode, B->s1[t], B->n1[t], B->s2[t], B->n2[t], B->sc, B->a, B->b, &sc,
                      o1, o2, &len);
    if (B->scores) B->scores[t] = sc;
    if (B->statuses) B->statuses[t] = st;
  }
  free(o1); free(o2);
  or_aligner_free(A);
  return NULL;
}

double or_align_batch(int mode, size_t npairs, const uint8_t* const* s1, const size_t* n1,
                      const uint8_t* const* s2, const size_t* n2, const or_scoring* sc, int32_t a,
                      int32_t b, int nthreads, int exact, int32_t* scores, int* statuses) {
  batch_ctx B = {mode, npairs, s1, n1, s2, n2, sc, a, b, exact, scores, statuses, 0,
                 PTHREAD_MUTEX_INITIALIZER};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &B);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---------------------------------------------------------------------------------------------
 * analysis::seq::edit_distance (src/analysis/seq.rs:105-130): the unit-cost Levenshtein table
 * over raw bytes, memo[i][0] = i, memo[0][j] = j, memo[i][j] = min(memo[i-1][j-1] + (s1[i-1] !=
 * s2[j-1]), min(memo[i][j-1] + 1, memo[i-1][j] + 1)).  The reference's u128 cells never exceed
 * max(n1, n2), so uint64 is exact.  Two rows instead of the full table (same values). */
uint64_t or_edit_distance(const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2) {
  uint64_t* prev = (uint64_t*)malloc((n2 + 1) * sizeof(uint64_t));
  uint64_t* cur = (uint64_t*)malloc((n2 + 1) * sizeof(uint64_t));
  for (size_t j = 0; j <= n2; ++j) prev[j] = j;                    /* :113-115 */
  for (size_t i = 1; i <= n1; ++i) {                               /* :118-127 */
    cur[0] = i;                                                    /* :110-112 */
    for (size_t j = 1; j <= n2; ++j) {
      const uint64_t d = prev[j - 1] + (s1[i - 1] != s2[j - 1]);
      const uint64_t l = cur[j - 1] + 1, u = prev[j] + 1;
      const uint64_t m = l < u ? l : u;
      cur[j] = d < m ? d : m;
    }
    uint64_t* t = prev; prev = cur; cur = t;
  }
  const uint64_t r = prev[n2];
  free(prev); free(cur);
  return r;
}

/* processing::patterns::longest_common_subsequence (src/processing/patterns.rs:82-118): the
 * match table with its tie rules (a match always takes the diagonal; otherwise up only when
 * strictly greater than left, :88-98) and the walk from (n1, n2) while the cell is non-zero,
 * pushing seq1[i-1] on diagonal moves (:104-114).  Writes the subsequence to out (capacity
 * >= min(n1, n2)); returns its length. */
size_t or_lcs(const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2, uint8_t* out) {
  const size_t W = n2 + 1;
  uint32_t* L = (uint32_t*)calloc((n1 + 1) * W, sizeof(uint32_t));
  uint8_t* prev = (uint8_t*)calloc((n1 + 1) * W, 1);    /* 0 diag, 1 up, 2 left */
  for (size_t i = 1; i <= n1; ++i)
    for (size_t j = 1; j <= n2; ++j) {
      if (s1[i - 1] == s2[j - 1]) {
        L[i * W + j] = L[(i - 1) * W + j - 1] + 1; prev[i * W + j] = 0;
      } else if (L[(i - 1) * W + j] > L[i * W + j - 1]) {
        L[i * W + j] = L[(i - 1) * W + j]; prev[i * W + j] = 1;
      } else {
        L[i * W + j] = L[i * W + j - 1]; prev[i * W + j] = 2;
      }
    }
  size_t i = n1, j = n2, len = 0;
  while (L[i * W + j] != 0) {
    const uint8_t p = prev[i * W + j];
    if (p == 0) { out[len++] = s1[i - 1]; --i; --j; }
    else if (p == 1) --i;
    else --j;
  }
  for (size_t x = 0; x < len / 2; ++x) { const uint8_t t = out[x]; out[x] = out[len - 1 - x]; out[len - 1 - x] = t; }
  free(L); free(prev);
  return len;
}
