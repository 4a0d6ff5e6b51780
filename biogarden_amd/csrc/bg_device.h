// Shared host/device layout for the MI355X aligner (gfx950).
//
// One "batch" = many independent pairs (seq1 = rows, seq2 = columns) aligned with one mode,
// one scoring table and one (open, extend) pair — exactly the arguments of one
// SequenceAligner::*_alignment call in the reference (aligner.rs:84,150,216,290,351), applied to
// a list of pairs.  Everything lives in HBM; see DESIGN.md "Data layout in HBM".
#pragma once
#include <stdint.h>

#define BG_WAVE 64
#define BG_CHUNK 64          // steps per chunk == columns per boundary block
#define BG_TRACE_BLK 32      // steps per trace word (one bit per step per lane)

// Modes, numbered like include/biogarden_gpu.h (bg_mode).
enum { BGK_GLOBAL = 0, BGK_LOCAL = 1, BGK_FITTING = 2, BGK_OVERLAP = 3, BGK_SEMIGLOBAL = 4 };

// Per-pair descriptor, built by the host planner (bg_host.cpp) in LPT order.
struct BgPair {
  uint64_t off1;       // byte offset of seq1 in the packed seq1 byte arena
  uint64_t off2;       // byte offset of seq2 in the packed seq2 byte arena
  uint64_t trace_off;  // byte offset of this pair's trace in the trace arena
  uint64_t bnd_off;    // int32 offset of this pair's boundary rows (nstrips rows of NC*64)
  uint64_t aux_off;    // int32 offset of this pair's aux area (lastcol n1+1 | rowbest n1 | rowpos n1)
  uint64_t out_off;    // byte offset of this pair's output slot (capacity n1+n2)
  int32_t n1, n2;
  int32_t nstrips;     // ceil(n1 / (64 R)); 0 when n1 == 0 or n2 == 0 (no DP cells)
  int32_t pad;         // virtual rows above row 1 in strip 0: nstrips*64R - n1
  int32_t nc;          // chunks per strip: n2/64 + 2
  int32_t index;       // plan slot (results array index)
  uint64_t caller_off; // caller's output offset (sum of n1+n2 over earlier caller pairs)
  int32_t caller;      // caller's pair index
  int32_t wg_count;    // tagged kernel, WIDE mode: workgroups working on this pair (else 1)
  uint32_t prog_off;   // WIDE mode: offset of the pair's wg_count*W progress counters in gprog
  int32_t buf_rows;    // the reference aligner's scratch when this pair's call starts (rows, cols)
  int32_t buf_cols;
  uint64_t ops_off;    // byte offset of this pair's packed core ops (ceil((n1+n2)/4) bytes)
  uint64_t split_off;  // split traceback (bg_split.hip): int32 offset of the pair's split area
  int32_t lane0;       // grouped pairs (bg_grp_kernel.hip): the pair's first lane in its wave's
                       // checkpoints (16 g); 0 otherwise
  int32_t lanes;       // lanes per strip: 64, or 16 for grouped pairs
};

// ---- split traceback (WIDE linear checkpoint batches).  The walk of one long
// pair is cut at strip boundaries: an exit pass gives every cell of a strip's bottom row the
// column where its traceback path enters the strip above (its "exit"), a chain over the strips
// turns the start cell into one entry column per strip, and the strips' walks then run as
// independent workgroups that the tail stitches together.
#define BG_SPLIT_EBITS 17                          // exit column field of the packed values
#define BG_SPLIT_SYM(R) ((1 << BG_SPLIT_EBITS) - ((R) + 1) * 64)   // first symbolic exit
#define BG_SPLIT_SEGC 16                           // default chunks per exit-pass segment

// Per (pair, strip) record of a strip walk.
struct BgStripHdr {
  int32_t sk, sl;      // cell the walk started from
  int32_t ek, el;      // cell it stopped at (crossed: the first cell in the strip above)
  int32_t nops;        // ops written to the strip's scratch (backwards from its end)
  int32_t crossed;     // 1: stopped on entering the strip above; 0: the walk ended in this strip
  int32_t status;      // 0, 4 (reference index underflow), 5 (internal)
  int32_t pre;         // tail: ops of the strips stitched before this one
};

// Split area of one pair (int32 offsets from BgPair::split_off; `ops` is a byte offset from the
// area's start).  head: [0] end row, [1] end column, [2] score, [3] column case, [4] raw exit of
// the start cell, [5] its segment, [6] overflow flag, [7] start strip (-1: nothing to split).
struct BgSplitLayout {
  uint64_t head, startcol, hdr, ebot, front, fres, ckg, done, ops, total_ints;
  int32_t G, F, capS;
};
__host__ __device__ inline BgSplitLayout bg_split_layout(int n1, int n2, int nstrips, int nc, int R,
                                                         int segc) {
  BgSplitLayout L;
  const uint64_t S = (uint64_t)nstrips;
  L.G = (nc + segc - 1) / segc;
  L.F = (R + 1) * 64;
  L.capS = 64 * R + n2 + 1;
  (void)n1;
  uint64_t o = 0;
  L.head = o; o += 16;
  L.startcol = o; o += (S + 15) / 16 * 16;
  L.hdr = o; o += S * 8;
  L.ebot = o; o += (S * (uint64_t)(n2 + 1) + 15) / 16 * 16;
  L.front = o; o += S * (uint64_t)L.G * L.F;
  L.fres = o; o += S * (uint64_t)L.G * L.F;
  // concurrent exit pass: the DP's segment-start checkpoints as {value, epoch} granules
  // (8 bytes: two ints), and a done tag per exit-pass item
  L.ckg = o; o += 2 * S * (uint64_t)L.G * L.F;
  L.done = o; o += (S * (uint64_t)L.G + 15) / 16 * 16;
  L.ops = o * 4;
  o += (S * (uint64_t)L.capS + 63) / 64 * 16;
  L.total_ints = o;
  return L;
}

// Exit pass, resolve and chain kernels (bg_split.hip).
struct BgSplitArgs {
  const BgPair* pairs;
  const uint8_t* codes1;
  const uint8_t* codes2;
  const int32_t* ckpt;     // the slot's checkpoint arena (int32 view of the trace arena)
  const int32_t* bndM;     // strip-boundary rows M'(last row of strip, j)
  const int32_t* profile;  // [192 + q]: 4 packed int8 S(q, c) - 2a
  int32_t* split;          // the slot's split arena
  const int32_t* itemBase; // exit pass: first work item of each plan pair (npairs + 1)
  const int32_t* stripBase;// resolve: first workgroup (strips 1 .. nstrips - 1) of each plan pair
  // concurrent exit pass (conc = 1: launched beside the DP, persistent workers taking items in
  // `order` from *counter, inputs from the DP's epoch-tagged granules; conc = 0: the pass after
  // the DP, skipping items whose done tag is this epoch)
  int32_t conc;
  uint32_t epoch;
  const unsigned long long* gran;
  const int32_t* order;
  uint32_t* counter;
  const uint32_t* resident;
  // a worker that waits longer than waitTicks (s_memrealtime, 100 MHz) for one input abandons the
  // concurrent pass (the pass after the DP does the remaining items): diag[0] = 1, [1] the item,
  // [2] which input (1 top row, 2 checkpoint), [3] the tag lane 0 saw, [4] the epoch waited for
  uint32_t* diag;
  int32_t waitTicks;
  int32_t dpWgs;
  int32_t npairs, nitems;
  int32_t open, ext, mode, R, segc;
  int32_t margin;          // headroom below a chunk's smallest input: clampv + max(0, max S - 2a) + 1
  int32_t clampv;          // max(0, -(min S - 2a)): field value of a clamped column-0 value
  int32_t grow;            // 65 * max(0, max S - 2a): growth of a value inside one chunk
  // end-cell keys of the split pairs, folded by many workgroups (bg_endkey_kernel) before the
  // traceback's HEAD phase: [2p] column n2 (bias(M) << 32 | ~i), [2p + 1] row n1 (| j)
  unsigned long long* endKeys;
  const int32_t* aux;      // the slot's aux arena (column n2: M(i, n2) at aux_off + i)
  int2* xcount;            // deferred expansion: per (pair, block) ops consuming s1 / s2
  int32_t xblocks;         // deferred expansion: blocks per pair
};

// Would the reference SequenceAligner, whose scratch is rows x cols when this call starts
// (1024 x 1024 for SequenceAligner::new, aligner.rs:44-55; resize_buffers(len1 + 1, len2 + 1)
// whenever len1 > rows || len2 > cols, :92-94, 594-602), panic, hang or answer from stale scratch
// on this pair?  Exact-size semantics differ from it only when it does not resize and either
// indexes row `rows` / column `cols` (ndarray bounds panic) or its end-cell fold reaches cells
// beyond the pair's region (DESIGN.md "Buffer semantics").  Whether it hangs or
// answers from stale scratch there depends on the call history; both are flagged.
__host__ __device__ inline bool bg_ref_divergent(int mode, long n1, long n2, int score, long rows,
                                                 long cols) {
  if (n1 > rows || n2 > cols) {
    // resized to exactly (n1+1, n2+1); the border writes row0[1] / col0[1] (global, :98-104;
    // fitting, :235) then index a dimension of length 1 when a sequence is empty
    if (mode == BGK_GLOBAL) return n1 == 0 || n2 == 0;
    if (mode == BGK_FITTING) return n2 == 0;
    return false;
  }
  const bool e1 = n1 == rows, e2 = n2 == cols;
  switch (mode) {
    case BGK_GLOBAL: return e1 || e2 || rows < 2 || cols < 2;
    case BGK_LOCAL: return (e1 || e2) && n1 > 0 && n2 > 0;
    case BGK_FITTING: return e2 || cols < 2 || (e1 && n2 > 0) || (score < 0 && n1 + 1 < rows);
    case BGK_OVERLAP: return e1 || e2 || (score <= 0 && n2 + 1 < cols);
    default: return e1 || e2 || (score == 0 && n2 + 1 < cols);
  }
}

// Checkpoint tracebacks key a recomputed chunk by (strip << 20 | chunk << 4 | slot) in 32 bits
// (bg_finish.h ckMap): pairs beyond these limits take the full-trace kernels (bg_host.cpp).
#define BG_CK_MAX_STRIPS 4096
#define BG_CK_MAX_CHUNKS 65536

// Per-pair result written by the finish kernel.
struct BgResult {
  int32_t status;      // 0 ok, 4 reference would panic (traceback underflow)
  int32_t score;
  int32_t end_i, end_j;    // cell the traceback started from
  uint32_t out_start;      // aligned strings occupy [out_start, n1+n2) of the pair's slot
  uint32_t out_len;
  uint32_t start1, start2; // cell (k, l) where the traceback walk stopped
  uint32_t npre, ntail;    // semiglobal prefix / tail gap columns (aligner.rs:389-428); the core's
                           // out_len - npre - ntail ops are packed 2 bits each at F.ops + ops_off
};

struct BgDpArgs {
  const BgPair* pairs;
  const uint8_t* seq1;     // raw bytes of seq1, all pairs
  const uint8_t* seq2;     // raw bytes of seq2, all pairs
  const uint8_t* lut;      // 256 entries: byte -> dense code (DNA path: code*8)
  const uint8_t* codes1;   // lut[seq1] (host-computed), same offsets as seq1
  const uint8_t* codes2;   // lut[seq2]
  uint32_t* trace;         // trace arena
  int32_t* bndM;           // strip-boundary rows: M + open, per strip output
  int32_t* bndX;           // strip-boundary rows: X (affine kernels only)
  int32_t* aux;            // lastcol / rowbest / rowpos
  const int32_t* profile;  // DNA: [q] = 4 packed int8 S(q, c) - open; tagged kernel: [64+q] packed
                           // 4(S-2*open)-2, [128+q] packed 4(S-2*open)-3; LDS path: int16 [32][32]
  int32_t kdim;            // alphabet size (LDS path)
  int32_t open, ext;       // reference `a`, `b`
  int32_t mode;
  int32_t npairs;
  int32_t prog_off;        // byte offset of the 16 per-wave progress counters in dynamic LDS
  int32_t codes_off;       // byte offset of the staged seq2 codes in dynamic LDS
  int32_t codes_in_lds;    // 1 if every pair's seq2 fits there; 2: tagged WIDE, 2-bit packed row
  int32_t aux_lds_off;     // tagged kernel: per-wave area (boundary block, ring, profile, codes)
  const int2* wgmap;       // tagged kernel, WIDE mode: per workgroup (plan index, index in group)
  uint32_t* gprog;         // tagged kernel, WIDE mode: global per-wave progress counters
  int32_t pstride;         // row stride of the int16 profile table (the batch's dense alphabet)
  unsigned long long* dbg; // optional per-wave timestamps of the first strip (env BG_DEBUG=dp):
                           // [gw * 8 + k], k: 0 strip, 1 start, 2 chunk 0 done, 3 end, 4 waited
  int32_t* prof_scratch;   // mask kernel, int32 profiles in HBM: kdim x 64 x R ints per (pair, wave)
  unsigned long long* gran;  // tagged WIDE checkpoint mode: strip-boundary rows as {value, epoch}
                             // granules, indexed like bndM (zeroed when allocated)
  uint32_t epoch;          // this execute's granule tag (never 0, never reused by the handle)
  // split traceback with the exit pass running beside the DP (bg_split.hip): the slot's split
  // arena (segment-start checkpoints as {value, epoch} granules, every strip's output row as
  // granules too), the exit pass's segment length, and the resident-workgroup counter
  int32_t* split;
  int32_t segc;
  uint32_t* resident;
  // grouped single-strip pairs (bg_grp_kernel.hip): per wave four plan indices (-1: padding)
  const int32_t* grp;
  int32_t ngroups;
  // semiglobal / overlap: each grouped pair's last-row end-cell key (BgFinishArgs::keys[2 p + 1])
  unsigned long long* keys;
};

struct BgFinishArgs {
  const unsigned long long* keys;   // split HEAD: bg_endkey_kernel's keys (BgSplitArgs::endKeys);
                                    // grouped: the last-row keys the DP folded; or nullptr
  const BgPair* pairs;
  const uint8_t* seq1;     // raw bytes (the aligned strings are built from them)
  const uint8_t* seq2;
  const uint32_t* trace;
  const int32_t* bndM;
  const int32_t* aux;
  uint8_t* out1;           // aligned seq1, per-pair slot (written backwards)
  uint8_t* out2;
  BgResult* results;
  int32_t open, ext;
  int32_t mode;
  int32_t R;               // rows per lane of the DP kernel that produced the trace
  int32_t affine;          // trace carries x/y bits
  int32_t tag;             // 1: tagged linear kernel (2-bit m_trace codes, boundary rows X forms);
                           // 2: checkpoint traceback (untagged M' boundary rows, no trace)
  int32_t npairs;
  int32_t win_bytes;       // LDS trace window (bg_finish_window_bytes)
  // checkpoint traceback (tag == 2): trace = checkpoint arena; recomputation inputs
  const uint8_t* codes1;
  const uint8_t* codes2;
  const int32_t* profile;
  unsigned long long* dbg;  // optional per-pair cycle counters (env BG_DEBUG=finish)
  // affine / local checkpoint traceback (bg_aff_kernel.hip): X boundary rows, alphabet size
  // (per-lane profile entries) and the ints of one wave's recompute area
  const int32_t* bndX;
  int32_t kdim;
  int32_t area_ints;
  int32_t flags;           // BG_FIN_* below
  int32_t nslots;          // checkpoint modes: recomputed-chunk slots in use (0: all)
  int32_t pstride;         // row stride of the int16 profile table (affine checkpoint path)
  uint8_t* ops;            // packed core ops (2 bits per column, op 0 diagonal, 1 up, 2 left)
  // split traceback (linear checkpoint kernel only): BG_PH_* phase, the slot's split arena, the
  // exit pass's segment length and, for BG_PH_WALK, the (plan index, strip) of each workgroup
  int32_t phase;
  int32_t segc;
  int32_t* split;
  const int2* splitMap;
  // linear checkpoint traceback's helpers: chunks prefetched left of the walker in its strip
  // (0 .. kSpecDepth) and the rows from the strip's top within which the strip above is
  // prefetched (bg_host.cpp: BG_SPEC="depth,rows")
  int32_t specDepth;
  int32_t specAbove;
  // grouped single-strip pairs (bg_grp_kernel.hip): chunks are recomputed as 16-lane jobs, up to
  // four per pass, into 16-lane slots
  int32_t grouped;
  // every spin of the asynchronous traceback on another wave (the walker waiting for a chunk, the
  // LDS slot lock, a helper waiting for the walker) is bounded by waitTicks of s_memrealtime
  // (100 MHz); past it the pair ends with BG_INTERNAL and the first such wait writes wdiag
  // (words below, bg_wait_diag)
  int32_t waitTicks;
  uint32_t* wdiag;
};

// bg_wait_diag's record: the first bounded wait of an execute's traceback that ran out
enum {
  BG_WD_NONE = 0,
  BG_WD_CHUNK = 1,        // the walker waited for a recomputed chunk
  BG_WD_LOCK_WALKER = 2,  // the walker waited for the slot lock
  BG_WD_LOCK_HELPER = 3,  // a helper waited for the slot lock
  BG_WD_THRASH = 4,       // the walker recomputed the same chunk again and again without finding it
  BG_WD_WORDS = 18
};
// words: [0] kind, [1] pair (plan index), [2] wave, [3] key (strip << 16 | chunk), [4] its map
// entry, [5] slot filling flags (bit z), [6] lock word, [7] walker row, [8] walker column,
// [9] the walker's recomputations of the key, [10..17] slot keys

// BgFinishArgs::phase
enum {
  BG_PH_FULL = 0,   // end cell + the whole walk + strings (one workgroup per pair)
  BG_PH_HEAD = 1,   // end cell only, into the split head
  BG_PH_WALK = 2,   // one strip's walk per workgroup, into the strip's scratch
  BG_PH_TAIL = 3    // stitch the strip walks (finish any walk the chain did not cover) + strings
};

// BgFinishArgs::flags
enum {
  BG_FIN_SCORE_ONLY = 2,   // end cell and score only, no traceback (analysis::seq::edit_distance)
  BG_FIN_LCS = 4,          // LCS tie rule in the recomputed trace; out2 receives the op codes
  BG_FIN_SYNC = 8,         // linear checkpoint traceback: recompute at barriers (BG_FIN_SYNC=1, A/B)
  BG_FIN_SELFSERVE = 16,   // asynchronous traceback: the walker recomputes every miss itself at
                           // once (tests the forward-progress path; BG_FIN_SELFSERVE=1)
  BG_FIN_NOPRIO = 32,      // the walker keeps priority 0 (many-pair linear batches)
  BG_FIN_DEFER_EXPAND = 64 // split TAIL: the core's op packing and expansion are left to
                           // bg_expand_count_kernel / bg_expand_kernel (many workgroups per pair)
};

// bg_pair_result of include/biogarden_gpu.h, as the export kernel writes it.
struct BgPairResultDev {
  int32_t status, score;
  uint64_t offset;
  uint32_t len, end_i, end_j, start1, start2, reserved;
};

// Compact export (bg_batch_export_compact): per caller pair a header, then the pairs' packed core
// ops back to back.  The layout is include/biogarden_gpu.h's bg_compact_hdr.
struct BgCompactHdr {
  int32_t status, score;
  uint64_t ops_off;        // byte offset of the packed ops in the record's ops area
  uint32_t len, end_i, end_j, start1, start2, npre, ntail, reserved;
};

struct BgCompactArgs {
  const BgPair* pairs;
  const BgResult* results;
  const BgPairResultDev* recs;   // caller-order template (pre-decided statuses)
  const uint8_t* ops;            // the slot's packed ops (BgPair::ops_off)
  uint64_t* sizes;               // caller order: packed bytes, then (scan) offsets; [n] = total
  uint8_t* dst;                  // the record
  uint64_t npairs_caller;
  int32_t nplan;
  int32_t mode;
};

// bg_download_kernel (bg_io.hip): up to three device -> host-mapped copies
struct BgDownloadSeg {
  const uint8_t* src;      // device
  uint8_t* dst;            // host-mapped pinned memory (hipHostGetDevicePointer)
  uint64_t bytes;
};
struct BgDownloadArgs {
  BgDownloadSeg seg[3];
  int32_t nseg;
};

struct BgExportArgs {
  const BgPair* pairs;
  const BgResult* results;
  const uint8_t* out1;
  const uint8_t* out2;
  uint8_t* dst;            // [u64 n][BgPairResultDev x n][aligned1 bytes][aligned2 bytes]
  uint64_t npairs_caller;
  uint64_t out_bytes;      // sum over caller pairs of n1+n2
  int32_t mode;
};


