/*
 * biogarden_gpu.h — C ABI of the MI355X-native aligner (libbiogarden_gpu.so).
 *
 * Drop-in boundary for robsndr/biogarden's alignment hot path.  Each entry point names the
 * reference interface it replaces (paths relative to the reference crate root):
 *
 *   bg_aligner_new / bg_aligner_free   SequenceAligner::new / Default / drop
 *                                      (src/alignment/aligner.rs:44-55, 605-609)
 *   bg_align(mode=BG_GLOBAL)           SequenceAligner::global_alignment      (aligner.rs:84-121)
 *   bg_align(mode=BG_LOCAL)            SequenceAligner::local_alignment       (aligner.rs:150-185)
 *   bg_align(mode=BG_FITTING)          SequenceAligner::fitting_alignment     (aligner.rs:216-260)
 *   bg_align(mode=BG_OVERLAP)          SequenceAligner::overlap_alignment     (aligner.rs:290-321)
 *   bg_align(mode=BG_SEMIGLOBAL)       SequenceAligner::semiglobal_alignment  (aligner.rs:351-435)
 *   bg_align_batch                     the same call over a Tile of pairs (ds/tile.rs:9-11)
 *   bg_scoring_builtin                 score::blosum62 / pam250 / unit        (score.rs:38,78,114)
 *   bg_scoring (struct)                the `&dyn Fn(&u8,&u8)->i32` closure, tabulated as data
 *   status codes                       BioError::{InvalidArgumentRange, InvalidInputSize}
 *                                      (error.rs:8-14) + the reference's panics
 *
 * Semantics: identical integer score and aligned strings to the reference for every input on
 * which the reference returns (including its traceback quirks); see DESIGN.md.  Plain pointers
 * and sizes only; no allocation crosses the boundary; one in-flight call per handle.
 */
#ifndef BIOGARDEN_GPU_H
#define BIOGARDEN_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: bg_stats gained `grouped` / `group_pairs` (a caller built against version 1 has a smaller
 * struct: use bg_get_stats_sized, which writes only the bytes the caller's struct holds). */
#define BG_ABI_VERSION 2

typedef enum bg_mode {
  BG_GLOBAL = 0,
  BG_LOCAL = 1,
  BG_FITTING = 2,
  BG_OVERLAP = 3,
  BG_SEMIGLOBAL = 4
} bg_mode;

/* Per-pair status (bg_pair_result.status, bg_align return value). */
enum {
  BG_OK = 0,
  BG_INVALID_ARGUMENT_RANGE = 1, /* Err(BioError::InvalidArgumentRange): a > 0 || b > 0 (global/local/fitting) */
  BG_INVALID_INPUT_SIZE = 2,     /* Err(BioError::InvalidInputSize): fitting with len1 < len2 */
  BG_UNSCORABLE = 3,             /* the reference panics in the score closure (byte outside its table) */
  BG_REF_DIVERGENT = 4,          /* the reference (fresh SequenceAligner) panics or hangs on this input;
                                    the result of the exactly-sized DP is returned and flagged */
  BG_INTERNAL = 5                /* the traceback's walker waited too long for a recomputed chunk (a
                                    build defect, never expected); the pair's strings are incomplete */
};

/* Call-level errors (negative return values). */
enum {
  BG_E_ARG = -1,        /* bad argument (null pointer, capacity too small, unknown mode) */
  BG_E_HIP = -2,        /* HIP runtime failure */
  BG_E_NOMEM = -3,      /* device or host allocation failed */
  BG_E_SCORE_RANGE = -4,/* no longer returned (kept for ABI stability; LCS beyond the checkpoint keys runs the mask kernel) */
  BG_E_NO_BATCH = -5,   /* bg_batch_execute/fetch without a prepared batch */
  BG_E_ALPHABET = -6,   /* no longer returned (kept for ABI stability; big int32 alphabets keep their profiles in HBM) */
  BG_E_IO = -7,         /* bg_fasta_open: the file cannot be opened */
  BG_E_FORMAT = -8,     /* bg_fasta_next_batch: "Expected > at record start." (fasta.rs:104-109) */
  BG_E_UTF8 = -9        /* bg_fasta_next_batch: a line is not valid UTF-8 (BufRead::read_line's
                           io::ErrorKind::InvalidData, fasta.rs:97, 115) */
};

/* Scoring closure as data: code[byte] in [0, alphabet_size) or 0xFF when the closure would
 * panic on that byte; table[c1 * 32 + c2] = S(byte1, byte2) with c1 from seq1. */
typedef struct bg_scoring {
  int32_t alphabet_size;
  uint8_t code[256];
  int32_t table[32 * 32];
} bg_scoring;

enum { BG_BLOSUM62 = 0, BG_PAM250 = 1, BG_UNIT = 2 };

/* Fills *out with the reference's 26x26 table ('A'..'Z'; other bytes unscorable). */
int bg_scoring_builtin(int which, bg_scoring* out);

typedef struct bg_aligner bg_aligner;

/* device: HIP device ordinal (one process per GPU).  NULL on failure. */
bg_aligner* bg_aligner_new(int device);
/* A second aligner on peer's device that shares peer's HIP streams: several handles holding
 * different batches in flight (the streaming rotation of biogarden_amd/stream.py, one reference
 * SequenceAligner fed batch after batch) then use four streams in all — uploads, DPs,
 * tracebacks, downloads — and so four hardware queues, whatever the number of handles.  The DPs
 * and tracebacks of consecutive batches pipeline as one handle's executes do.  Each handle keeps
 * its own arenas and batch; waits (prepare, fetch, synchronize) wait for the handle's own work
 * only.  The streams live until the last handle sharing them is freed.  NULL on failure. */
bg_aligner* bg_aligner_new_shared(bg_aligner* peer);
void bg_aligner_free(bg_aligner* h);
/* on != 0: every bg_batch_execute also queues the download of its results (scores, both
 * aligned strings) into the handle's pinned host buffers, on a stream of its own right after the
 * traceback; bg_batch_fetch then waits for that download and unpacks it, with no copy of its own.
 * For callers that fetch every execute (the streaming rotation).  Default 0. */
int bg_set_async_fetch(bg_aligner* h, int on);

/* One alignment.  out1/out2 receive the aligned strings ('-' for gaps), both *out_len bytes;
 * cap must be >= n1 + n2.  Returns a BG_* status (>= 0) or a BG_E_* error (< 0). */
int bg_align(bg_aligner* h, int mode, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
             const bg_scoring* scoring, int32_t a, int32_t b, int32_t* score, uint8_t* out1,
             uint8_t* out2, size_t cap, size_t* out_len);

typedef struct bg_pair_result {
  int32_t status;    /* BG_* */
  int32_t score;
  uint64_t offset;   /* pair p's strings are at out1+offset / out2+offset; offset = sum_{q<p} (n1_q+n2_q) */
  uint32_t len;      /* aligned length */
  uint32_t end_i;    /* DP cell the traceback started from */
  uint32_t end_j;
  uint32_t start1;   /* cell (start1, start2) where the traceback walk stopped */
  uint32_t start2;
  uint32_t reserved;
} bg_pair_result;

/* Many independent pairs with one mode / scoring / (a, b) — the batched form of one
 * SequenceAligner::*_alignment call per pair, in order, on one aligner.  out1/out2 capacity
 * >= sum(n1+n2).  Returns 0 or BG_E_*.
 * Sizes: each length <= 2^30 - 1 (BG_E_ARG beyond).  Pairs too long for the checkpoint
 * tracebacks' chunk keys (>= 4096 strips of 64R rows, or len2 >= ~4.19M) run the full-trace
 * kernels instead (BG_E_NOMEM if that trace does not fit the device). */
int bg_align_batch(bg_aligner* h, int mode, size_t npairs, const uint8_t* const* s1,
                   const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                   const bg_scoring* scoring, int32_t a, int32_t b, bg_pair_result* results,
                   uint8_t* out1, uint8_t* out2, size_t out_cap);

/* Split form of bg_align_batch for callers that keep inputs resident on the device:
 * prepare (validate, plan, upload) once, execute (enqueue DP + end cell + traceback on the
 * handle's stream; async) any number of times, fetch (wait, download, unpack). */
int bg_batch_prepare(bg_aligner* h, int mode, size_t npairs, const uint8_t* const* s1,
                     const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                     const bg_scoring* scoring, int32_t a, int32_t b);
/* bg_batch_prepare with a score table of up to 256 codes (the reference's closure over any
 * bytes, score.rs:38-41 / A.8): code[byte] < k selects row / column of table (k x k, row = seq1
 * code), code[byte] >= k marks a byte the closure panics on (status BG_UNSCORABLE).  Batches
 * using more than 32 codes run on the score-only affine-family kernels when their values fit
 * int8 (scores minus the open and extend penalties), otherwise on the mask-trace kernel reading
 * its k x k table from HBM (with the per-wave k x 64 int32 profiles in HBM too when they exceed
 * the CU's LDS: more than ~150 codes with scores beyond int16). */
int bg_batch_prepare_table(bg_aligner* h, int mode, size_t npairs, const uint8_t* const* s1,
                           const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                           const uint16_t* code, int32_t k, const int32_t* table, int32_t a,
                           int32_t b);
int bg_batch_execute(bg_aligner* h);
int bg_batch_fetch(bg_aligner* h, bg_pair_result* results, uint8_t* out1, uint8_t* out2,
                   size_t out_cap);
/* Blocks until the enqueued work is done. */
int bg_synchronize(bg_aligner* h);

typedef struct bg_stats {
  uint64_t cells;          /* sum n1*n2 of the prepared batch */
  uint64_t trace_bytes;    /* trace arena bytes written per execute */
  uint64_t boundary_bytes; /* strip-boundary bytes written per execute */
  uint64_t residue_bytes;  /* seq1+seq2 bytes */
  uint64_t device_bytes;   /* device memory held by the handle */
  int32_t R;               /* rows per lane */
  int32_t waves;           /* waves per workgroup (one workgroup per pair) */
  int32_t affine;          /* 1: affine kernel (open < extend), 0: linear-gap kernel */
  int32_t tagged;          /* 1: tagged linear kernel (tie-break tag in the score's low bits) */
  int32_t dna;             /* 1: register profile (<= 4 symbols), 0: LDS profile */
  int32_t local;
  int32_t npairs;
  int32_t wide;            /* tagged kernel with each pair spread over a group of workgroups:
                              1 of one wave per SIMD (WIDE), 2 of several (SPAN); 0 one per pair */
  int32_t workgroups;      /* DP grid size */
  int32_t checkpoint;      /* 1: score-only DP + traceback recomputing the chunks its path crosses */
  float dp_ms;             /* last execute: DP kernel time (HIP events on the handle's stream) */
  float finish_ms;         /* last execute: end-cell + traceback kernel time */
  int32_t fin_waves;       /* finish workgroup: waves (walker + recomputing helpers) */
  int32_t fin_slots;       /* finish workgroup: recomputed-chunk slots in use (0: all) */
  int32_t split;           /* 1: the traceback is split at strip boundaries (few long pairs) */
  int32_t grouped;         /* pair groups of the grouped DP (four short reads per wave sharing one
                              reference), 0: one wave per pair */
  int32_t group_pairs;     /* pairs per wave of the grouped DP (4 or 2), 0: not grouped */
} bg_stats;

/* Writes the whole bg_stats of this header (ABI version 2). */
int bg_get_stats(bg_aligner* h, bg_stats* out);
/* Writes min(size, sizeof(bg_stats)) bytes of it: a caller built against an older, smaller
 * bg_stats passes its own sizeof and gets the fields it knows, nothing past its struct. */
int bg_get_stats_sized(bg_aligner* h, bg_stats* out, size_t size);

/* Split traceback of the last execute (few long pairs, linear gaps): pairs whose
 * walk was cut at strip boundaries, strips whose walks the stitching took, traceback moves the
 * stitching had to walk itself (0 when every strip walk was used), pairs whose exit pass left its
 * packed range (walked whole), and exit-pass items done beside the DP.  All 0 when the batch is
 * not split.  Waits for the handle's work.  The results never depend on it: a diagnostic. */
int bg_split_stats(bg_aligner* h, uint64_t* pairs_split, uint64_t* strips_taken,
                   uint64_t* tail_moves, uint64_t* pairs_overflow, uint64_t* items_beside_dp);
/* Diagnostics of the last execute's concurrent exit pass (BG_SPLIT_CONC=1), six words: [0] 1 if a
 * worker waited longer than BG_SPLIT_WAIT_MS for an input and abandoned the pass (the pass after
 * the DP then did the remaining items), [1] that item, [2] which input (1 the row above, 2 the
 * segment's checkpoint), [3] the tag it saw, [4] the epoch it waited for, [5] 1 if the workers
 * gave up waiting for the DP's workgroups to become resident.  Not a reference interface. */
int bg_split_conc_diag(bg_aligner* h, uint32_t* out6);

/* The reference aligner's scratch dims this handle models (SequenceAligner::buffer_size,
 * aligner.rs:30): 1024 x 1024 after bg_aligner_new (:44-55); every alignment call of a prepared
 * batch, in caller order, resizes it to (len1+1, len2+1) when len1 > rows || len2 > cols
 * (:92-94, 594-602), as the reference's calls would.  Status BG_REF_DIVERGENT is judged against
 * the dims each call starts from. */
int bg_aligner_buffer_size(bg_aligner* h, size_t* rows, size_t* cols);
/* Sets those dims (takes effect at the next bg_batch_prepare): several handles that together
 * stand for ONE reference aligner — the streaming rotation of biogarden_amd/stream.py — pass
 * the state on in call order. */
int bg_aligner_set_buffer_size(bg_aligner* h, size_t rows, size_t cols);
/* The dims each call of the NEXT prepared batch starts from, given per pair: a shard of a larger
 * batch whose earlier calls ran on other ranks (biogarden_amd/shard.py call_dims replays the
 * resize rule over the whole batch in caller order, so every rank judges status BG_REF_DIVERGENT
 * against the history one reference aligner fed the whole batch would have).  rows / cols hold
 * npairs entries; the next bg_batch_prepare / bg_batch_prepare_table must have exactly npairs
 * pairs (else it returns BG_E_ARG and leaves them pending) and a successful prepare consumes
 * them; afterwards the handle's dims are what the last pair's call leaves.  npairs = 0 or NULL
 * arrays clear a pending set. */
int bg_aligner_set_call_dims(bg_aligner* h, size_t npairs, const uint64_t* rows, const uint64_t* cols);

/* Kernel timing over a region of executes (HIP events recorded on the handle's stream around
 * the DP and the finish kernel of every execute; up to 4096 executes per region).
 * bg_profile_end waits for the work and returns per-execute averages in milliseconds. */
int bg_profile_begin(bg_aligner* h);
int bg_profile_end(bg_aligner* h, float* avg_dp_ms, float* avg_finish_ms, int* executes);

/* Compact export of the last execute's results, the payload of the multi-GPU gather (SURVEY
 * §8(e)): per caller pair a header, then the alignment cores as edit scripts, 2 bits per column
 * (0 = (s1, s2), 1 = (s1, '-'), 2 = ('-', s2)), back to back:
 *   [u64 "BGC1"][u64 npairs][u64 ops bytes][u64 mode][bg_compact_hdr x npairs][ops]
 * A pair's strings are npre prefix columns (semiglobal: s1[0, npre) against gaps when end_i < n1,
 * else s2[0, npre)), the core's columns consuming s1 from start1 and s2 from start2, and ntail
 * tail columns (s1[end_i, ...) against gaps when end_i < n1, else s2[end_j, ...)); len counts all
 * of them.  bg_compact_expand rebuilds bg_batch_fetch's output from it and the input sequences.
 * dst = NULL: computes the record on the device (waits for the execute) and returns its exact
 * size in *bytes; then call again with dst (device memory of the handle's GPU, *bytes >= size). */
/* The record's largest size for the prepared batch (32 + npairs x sizeof(bg_compact_hdr) + every
 * pair's ops at ceil((n1 + n2) / 4)): the capacity bg_batch_export_compact_async needs. */
int bg_batch_export_compact_bound(bg_aligner* h, size_t* bytes);
/* bg_batch_export_compact of the last execute WITHOUT a host wait, for callers that gather every
 * execute's record inside a pipelined step (the strong-scaling form of SURVEY §8(d)): the record
 * is written to dst (device memory of the handle's GPU, cap >= the bound above) on the handle's
 * export stream after that execute's traceback.  The handle's next execute into the same arena
 * slot waits for it.  after (a hipStream_t of the same device; NULL = that device's null stream)
 * is made to wait for the record, so a collective queued on it afterwards sends a finished record.  The record's own size
 * is 32 + npairs x sizeof(bg_compact_hdr) + its header's ops bytes (u64 [2]); the bytes past it
 * are unspecified. */
int bg_batch_export_compact_async(bg_aligner* h, void* dst, size_t cap, void* after);
typedef struct bg_compact_hdr {
  int32_t status, score;
  uint64_t ops_off;  /* into the ops area */
  uint32_t len, end_i, end_j, start1, start2, npre, ntail, reserved;
} bg_compact_hdr;
int bg_batch_export_compact(bg_aligner* h, void* dst, size_t* bytes);
/* Host-only: expands a compact record (rec_bytes bytes in host memory) of npairs pairs into the
 * form bg_batch_fetch returns for the same pairs (results, out1 / out2 at offset sum of n1 + n2 over
 * earlier pairs, out_cap >= that sum).  BG_E_ARG if the record does not match the pairs. */
int bg_compact_expand(const void* rec, size_t rec_bytes, size_t npairs, const uint8_t* const* s1,
                      const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                      bg_pair_result* results, uint8_t* out1, uint8_t* out2, size_t out_cap);

/* ---- Several GPUs from one process: the batched SequenceAligner call over a Tile
 * (aligner.rs:84-435, ds/tile.rs:9-11; as tests/integration.rs:234-312 and
 * examples/from_file.rs:19-32 call it) spread over the node's devices.
 * bg_group_new: one aligner per entry of devices[0..n) (a device may repeat: several shards on one
 * GPU, which then share its streams) and one RCCL communicator over the distinct devices
 * (ncclCommInitAll; librccl is loaded at this call).  NULL on failure (no device, no librccl).
 * bg_group_align_batch: bg_align_batch's contract over the group — the pairs are split over the
 * members by cells (largest first, to the least-loaded member; bg_group_plan), every member aligns
 * its shard and packs the compact record on its device (bg_batch_export_compact), the records are
 * gathered to the first member's device (RCCL send / recv over xGMI; a device copy for members on
 * that device) and downloaded once, and the host expands them into out1 / out2 at the offsets
 * bg_align_batch uses.  The group stands for ONE reference aligner: every pair's status 4 is judged
 * against the scratch dims that aligner would have after the pairs before it in caller order
 * (bg_group_buffer_size; aligner.rs:92-94, 594-602).  Results are identical to bg_align_batch on
 * one aligner fed the same batches. */
typedef struct bg_group bg_group;
bg_group* bg_group_new(const int* devices, int n);
void bg_group_free(bg_group* g);
int bg_group_size(const bg_group* g);
/* member m's aligner (for bg_get_stats and the like), owned by the group */
bg_aligner* bg_group_member(bg_group* g, int m);
int bg_group_align_batch(bg_group* g, int mode, size_t npairs, const uint8_t* const* s1,
                         const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                         const bg_scoring* scoring, int32_t a, int32_t b, bg_pair_result* results,
                         uint8_t* out1, uint8_t* out2, size_t out_cap);
/* The same call in two halves, so that three batches are in flight (SURVEY §8(d)'s wall pipelined):
 * bg_group_submit splits the batch, moves the group's scratch dims on, and has every member
 * prepare and execute its shard, then returns; bg_group_collect finishes the OLDEST submitted
 * batch (the members' compact exports, the gather, the download and the expansion into
 * results / out1 / out2, out_cap >= that batch's sum(n1 + n2)).  The pair arrays are copied at
 * submit; the sequence bytes must stay valid until the batch's collect.  At most 3 batches are
 * submitted and not collected (a fourth submit: BG_E_ARG; a collect with none: BG_E_ARG);
 * bg_group_align_batch needs none pending.  bg_group_pending: how many are. */
int bg_group_submit(bg_group* g, int mode, size_t npairs, const uint8_t* const* s1, const size_t* n1,
                    const uint8_t* const* s2, const size_t* n2, const bg_scoring* scoring, int32_t a,
                    int32_t b);
int bg_group_collect(bg_group* g, bg_pair_result* results, uint8_t* out1, uint8_t* out2, size_t out_cap);
int bg_group_pending(const bg_group* g);
/* Host-only: the group's split of a batch over nshards (shard_of[p] for every pair). */
int bg_group_plan(size_t npairs, const size_t* n1, const size_t* n2, int nshards, int32_t* shard_of);
int bg_group_buffer_size(bg_group* g, size_t* rows, size_t* cols);
/* Accumulated ms per phase of bg_group_align_batch / submit / collect: [0] prepare + execute
 * (submit), [1] the members' waits and exports, [2] the gather, [3] the download, [4] the
 * expansion; *calls the count of collected batches. */
int bg_group_timing(bg_group* g, double* ms, size_t n, uint64_t* calls, int reset);

/* Host-side time of this handle's bg_batch_prepare / bg_batch_fetch calls, accumulated (ms):
 *   ms[0] waiting for the handle's previous work   ms[1] validation + staging (byte pass)
 *   ms[2] planning (history, alphabet, geometry)   ms[3] device allocation
 *   ms[4] upload (queue + wait)                    ms[5] fetch: waiting for the kernels
 *   ms[6] fetch: device-to-host copies             ms[7] fetch: string unpacking (byte pass)
 * Up to n entries are written; calls (3 entries, may be NULL) receives the prepare count, the
 * fetch count and the host threads the byte passes use.  reset != 0 zeroes the totals after
 * reading.  Returns the number of phases (8). */
int bg_host_timing(bg_aligner* h, double* ms, size_t n, uint64_t* calls, int reset);

/* Device-to-device export of the last execute's results for a collective (e.g. an RCCL
 * gather to rank 0): dst (device memory, same GPU) receives the packed record
 *   [u64 npairs][bg_pair_result x npairs][aligned1 bytes][aligned2 bytes]
 * with offsets as in bg_batch_fetch.  Pass dst = NULL to query the size in *bytes. */
int bg_batch_export(bg_aligner* h, void* dst, size_t* bytes);

/* Tuning overrides for tests/benchmarks (0 = automatic). */
int bg_set_tuning(bg_aligner* h, int R, int waves);

/* Pipeline depth 1-4: with 2 to 4 (default 3) slots of per-execute arenas the end-cell/traceback
 * kernel of execute k overlaps the DP kernel of execute k+1 (two HIP streams); 1 serialises.
 * Takes effect at the next bg_batch_prepare. */
int bg_set_pipeline(bg_aligner* h, int depth);

/* Per-handle options of the planner and the traceback (take effect at the next bg_batch_prepare /
 * bg_batch_execute).  -1 restores the automatic choice.  The environment variable BG_OPTIONS
 * ("name=value,...", names as below without the BG_OPT_ prefix, lower case) is read once per
 * handle at bg_aligner_new, for tools that cannot call this. */
enum {
  BG_OPT_GROUPED = 0,            /* grouped DP (short reads sharing a reference): 0 never, 1 at any
                                    fill, -1 when the groups fill (default) */
  BG_OPT_GROUP_PAIRS = 1,        /* pairs per wave of the grouped DP: 2 or 4 (-1: 4 when the reads
                                    fit 16 lanes x 10 rows) */
  BG_OPT_GROUP_WAVES = 2,        /* waves per workgroup of the grouped DP, 1..16 (-1: 4) */
  BG_OPT_WIDE_WAVES = 3,         /* waves per workgroup of a WIDE pair, 1..4 (-1: 4) */
  BG_OPT_FIN_WAVES = 4,          /* traceback workgroup waves (walker + helpers), 1..4 */
  BG_OPT_FIN_SLOTS = 5,          /* recomputed-chunk slots of a traceback workgroup, 0 = all */
  BG_OPT_FIN_SYNC = 6,           /* 1: recomputation at a workgroup barrier (no helper waves) */
  BG_OPT_FIN_SELFSERVE = 7,      /* 1: the walker recomputes every chunk it misses itself */
  BG_OPT_SPLIT = 8,              /* split traceback of few long pairs: 0 never, 1 also for SPAN
                                    batches (-1: WIDE batches) */
  BG_OPT_SPLIT_SEGMENT = 9,      /* chunks per segment of the split traceback's exit pass */
  BG_OPT_SPLIT_CONCURRENT = 10,  /* the exit pass beside the DP: 0 never, 1 always (-1: when no
                                    other execute's DP is in flight) */
  BG_OPT_SPLIT_WAIT_MS = 11,     /* the concurrent exit pass's wait bound per input (-1: 500) */
  BG_OPT_TWO_DP_STREAMS = 12,    /* WIDE batches: consecutive DPs on two streams: 0 never */
  BG_OPT_WAIT_MS = 13,           /* bound of every spin of a traceback on another wave (-1: 2000
                                    ms); past it the pair ends with BG_INTERNAL and
                                    bg_wait_diag records where */
  BG_OPT_SPAN = 14,              /* fewer pairs than CUs: each pair over a group of many-wave
                                    workgroups: 0 never, 1 whenever it applies (-1: when the
                                    planner's estimate gains) */
  BG_OPT_WIDE = 15,              /* 0: never WIDE (few long pairs over lone-wave workgroups).
                                    WIDE and SPAN DPs spin on workgroups of their own grid, so all
                                    of a grid's workgroups must be resident at once: processes
                                    sharing one GPU should turn both off */
  BG_OPT_COUNT = 16
};
int bg_set_option(bg_aligner* h, int key, int value);
int bg_get_option(bg_aligner* h, int key, int* value);
/* The last execute's traceback wait that ran out (status BG_INTERNAL), up to n of its 18 words;
 * all zero when none did.  [0] kind: 1 the walker waited for a recomputed chunk, 2 the walker
 * waited for the slot lock, 3 a helper waited for it, 4 the walker recomputed one chunk over and
 * over; [1] pair (plan order), [2] wave, [3] awaited chunk (strip << 16 | chunk), [4] its map
 * entry, [5] slots being filled (bit per slot), [6] lock word, [7] / [8] the walker's row and
 * column, [9] its recomputations of the chunk, [10..17] the slots' chunks.  Waits for the handle's
 * work.  Not a reference interface: the evidence for a defect. */
int bg_wait_diag(bg_aligner* h, uint32_t* out, size_t n);

/* Kernel selection for tests and benchmarks (default 7).  Bit 0: allow the tagged linear kernel
 * (else the mask-trace kernel); bit 1: with it, run the score-only DP and recompute the chunks
 * the traceback crosses from checkpoints (else the tagged DP writes the full trace); bit 2: the
 * same score-only DP + recomputing traceback for affine gaps, local mode and alphabets of more
 * than four symbols (else the mask-trace kernel).  Takes effect at the next bg_batch_prepare. */
int bg_set_kernel_options(bg_aligner* h, int allow_tagged);

/* analysis::seq::edit_distance (src/analysis/seq.rs:105-130) for a batch of pairs: unit-cost
 * Levenshtein distance over raw bytes, dist[p] = the reference's Ok(usize).  Runs the global DP
 * (byte equality 0 / -1, open = extend = -1) score-only on the GPU, any byte values (up to 256
 * distinct per batch).  Replaces the prepared batch. */
int bg_edit_distance_batch(bg_aligner* h, size_t npairs, const uint8_t* const* s1,
                           const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                           uint64_t* dist);

/* processing::patterns::longest_common_subsequence (src/processing/patterns.rs:82-118) for a
 * batch: the reference's subsequence (its tie rules) of pair p is out[offset[p] .. +len[p]);
 * out_cap >= sum of min(n1, n2).  Global DP (byte equality +1 / -1, open = extend = 0) with the
 * LCS tie rule in the traceback, any byte values.  Replaces the prepared batch.  shortest_common_supersequence (:198-235) is the host-side merge around it. */
int bg_lcs_batch(bg_aligner* h, size_t npairs, const uint8_t* const* s1, const size_t* n1,
                 const uint8_t* const* s2, const size_t* n2, uint8_t* out, size_t out_cap,
                 uint64_t* offset, uint64_t* len);

/* ---- Streaming FASTA ingest (io::fasta::Reader::read / read_all, src/io/fasta.rs:95-135).
 * Records are returned in batches, residues back to back in one reader-owned buffer: record r
 * is seq[seq_off[r] .. seq_off[r+1]), its id the NUL-terminated text + id_off[r], its
 * description text + desc_off[r] or absent (desc_off[r] == UINT64_MAX).  The batch is valid
 * until the next call.  A batch ends after max_records records or once max_residues residues
 * are buffered; reading stops for good at EOF or at the first empty record (read_all's rule).
 * The pointer + length arrays bg_batch_prepare takes are seq + seq_off[r], seq_off[r+1] -
 * seq_off[r]: no per-record copy on the way to the GPU. */
typedef struct bg_fasta bg_fasta;
typedef struct bg_fasta_batch {
  size_t n;                    /* records in this batch (0: the file is exhausted) */
  const uint8_t* seq;          /* NULL allowed when the batch holds no residues */
  const uint64_t* seq_off;     /* n + 1 entries */
  const char* text;
  const uint64_t* id_off;      /* n entries */
  const uint64_t* desc_off;    /* n entries, UINT64_MAX = no description */
} bg_fasta_batch;
bg_fasta* bg_fasta_open(const char* path, int* err);        /* err: 0, BG_E_ARG or BG_E_IO */
long bg_fasta_next_batch(bg_fasta* r, size_t max_records, size_t max_residues,
                         bg_fasta_batch* out);               /* records, or BG_E_* (< 0); both
                                                                maxima must be > 0 (BG_E_ARG) */
void bg_fasta_close(bg_fasta* r);

/* The hipError_t of the last HIP call that failed on this thread (BG_E_HIP), 0 if none; the
 * failing call and the error's name are also printed on stderr. */
int bg_last_hip_error(void);

const char* bg_status_string(int status);
int bg_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BIOGARDEN_GPU_H */
