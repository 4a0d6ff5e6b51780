// End cell + traceback + string assembly kernel (bg_finish_kernel), shared by bg_kernels.hip
// (full-trace and linear checkpoint instantiations) and bg_aff_finish.hip (the affine / local
// checkpoint instantiations).  Replaces the end-cell folds of the reference's
// *_alignment functions (src/alignment/aligner.rs:112, 173-176, 247-251, 308-312, 369-404),
// backtrack (:511-592) and the semiglobal output assembly (:383-432).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_aff_common.h"
#include "bg_dev_util.h"

// idle recompute helpers of the checkpoint traceback (bg_finish_ck): BG_HELP_FAST polls 512
// cycles apart, then BG_HELP_LONG x 64 cycles apart
#ifndef BG_HELP_FAST
#define BG_HELP_FAST 4
#endif
#ifndef BG_FIN_DEBUG
#define BG_FIN_DEBUG 0     // range checks with printf in the traceback (diagnosis builds)
#endif
#ifndef BG_SEQCHECK
#define BG_SEQCHECK 0      // verification builds: the walker re-checks its decode (reanchor)
#endif
#ifndef BG_HELP_LONG
#define BG_HELP_LONG 8
#endif
// the helpers' pauses (the walker never wakes them: DESIGN §4.4, s_wakeup)
#define help_pause(n) __builtin_amdgcn_s_sleep(n)
#include "bg_device.h"
#include "bg_tag_common.h"

using namespace bgk;

// ------------------------------------------------------------------ finish: end cell + traceback

namespace {

struct Fin {
  const BgFinishArgs* F;
  const BgPair* P;
  int n1, n2, a, b, mode;
  const uint8_t* s1;
  const uint8_t* s2;
  const int32_t* lastrowMa;   // bndM row of the last strip = M(n1, j) + a
  const int32_t* lastcol;     // M(i, n2)
};

// M(n1, j), j >= 1, from the last strip's stored row value v = lastrowMa[j]
__device__ __forceinline__ int lastrow_from(const Fin& f, int v, int j) {
  // the tagged kernel stores X forms 4*(M(n1,j) - a*(n1+j)) + 2
  // checkpoint mode (tag 2) stores M'(n1,j) = M(n1,j) - a*(n1+j) itself
  if (f.F->tag == 2) return wadd(v, wmul(f.a, f.n1 + j));
  // affine checkpoint path, non-local: O(n1,j) = M(n1,j) - b(n1+j) + (a - b)
  if (f.F->tag == 3) return wadd(wadd(v, -wadd(f.a, -f.b)), wmul(f.b, f.n1 + j));
  return f.F->tag ? wadd(v >> 2, wmul(f.a, f.n1 + j)) : wadd(v, -f.a);
}
__device__ __forceinline__ int lastrowM(const Fin& f, int j) {
  if (f.n1 == 0) return row0_M(f.mode, j, f.a, f.b);
  if (j == 0) return col0_M(f.mode, f.n1, f.a, f.b);
  return lastrow_from(f, f.lastrowMa[j], j);
}
// end-cell folds: loads in flight per thread
constexpr int kEndU = 8;
__device__ __forceinline__ int lastcolM(const Fin& f, int i) {
  if (f.n2 == 0) return col0_M(f.mode, i, f.a, f.b);
  if (i == 0) return row0_M(f.mode, f.n2, f.a, f.b);
  return f.lastcol[i];
}

// 64-bit key max over the wave
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned lo = __shfl_xor((unsigned)v, o, 64);
    const unsigned hi = __shfl_xor((unsigned)(v >> 32), o, 64);
    const u64 other = ((u64)hi << 32) | lo;
    v = other > v ? other : v;
  }
  return v;
}
__device__ __forceinline__ unsigned bias(int v) { return (unsigned)v ^ 0x80000000u; }
__device__ __forceinline__ int unbias(unsigned v) { return (int)(v ^ 0x80000000u); }

}  // namespace

// Trace-window geometry of the finish kernel: a window of 32-step trace blocks of one strip
// staged in LDS, plus an 8x8 neighbourhood of decoded cells held one per lane.
constexpr int kWinBytesMax = 57344;  // 56 KiB window + scalars/scan, under the 64 KiB default
constexpr int kCodeMiss = 32, kCodeBorder = 16;
// split traceback (BG_PH_WALK): a cell in the strip above the walked strip ends the strip's walk
constexpr int kCodeSplit = 64;

// ------------------------------------------------------------------ checkpoint traceback
// One wave recomputes chunk c of strip s of a pair from the forward pass's checkpoint with the
// tagged step (tag_chunk<KIND_RECOMP>, the same arithmetic as the tagged forward kernel) and
// leaves the chunk's 2-bit trace in an LDS slot laid out like the HBM trace of two 32-step
// blocks: [h][row k][lane] x uint2.
// resident recomputed chunks: 8, or 6 for tall strips (keeps the finish workgroup's LDS small
// enough to run beside the DP's)
template <int R>
__host__ __device__ constexpr int ck_slots() { return R >= 8 ? 6 : 8; }
template <int R>
__host__ __device__ constexpr int ck_slot_dw() { return 2 * R * BG_WAVE * 2; }
template <int R>
__host__ __device__ constexpr int ck_wave_ints() { return 64 + 4 * 64 * ProfW<R>::v + 96; }

// Grouped pairs (BgFinishArgs::grouped, bg_grp_kernel.hip, P pairs per wave): the pair holds
// L = 64 / P lanes of its wave's checkpoints (from BgPair::lane0), a slot holds one chunk as
// [half][row k][L lanes] x uint2, and one pass recomputes up to P chunks of the pair, one per
// L-lane job.  Per wave (sized for P = 4): four staged top blocks (row 0), the lanes' profile
// entries and four 192-code stages.
template <int R, int P>
__host__ __device__ constexpr int ck_grp_slot_dw() { return 2 * R * (64 / P) * 2; }
template <int R>
__host__ __device__ constexpr int ck_grp_wave_ints() { return 4 * 64 + 4 * 64 * ProfW<R>::v + 4 * 96; }
constexpr int kGrpSlots = 8;

template <int R, int GP>
__device__ void recompute_grp(const BgFinishArgs& F, const BgPair& P, int nj, const int (&chunks)[4],
                              const int (&zs)[4], uint32_t* win, int* area, int lane) {
  constexpr int RW = ProfW<R>::v;
  constexpr int L = 64 / GP;
  const int n1 = P.n1, n2 = P.n2, NC = P.nc;
  const int a = F.open, b = F.ext, mode = F.mode;
  const int j = lane / L, ql = lane % L;
  const int jj = j < nj ? j : 0;
  const int c = jj == 0 ? chunks[0] : (jj == 1 ? chunks[1] : (jj == 2 ? chunks[2] : chunks[3]));
  const int z = jj == 0 ? zs[0] : (jj == 1 ? zs[1] : (jj == 2 ? zs[2] : zs[3]));
  int* bIn = area + j * 64;
  int* profTab = area + 4 * 64;
  uint16_t* stage = reinterpret_cast<uint16_t*>(profTab + 4 * 64 * RW) + j * 192;
  TagCtx C;
  TagStrip<R> S;
  C.a = a; C.b = b; C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = ql;
  C.rowbase = ql * R;
  C.orow = R - 1;
  C.lastcol = nullptr; C.ring = nullptr; C.oLane = nullptr; C.mail = nullptr; C.bndOut = nullptr;
  const uint8_t* c1 = F.codes1 + P.off1;
  const uint8_t* g2 = F.codes2 + P.off2;
  int pk[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    const int qq = (i <= n1) ? c1[i - 1] : 0;
    pk[k] = F.profile[(k == 0 ? 64 : 128) + (qq >> 3)];
  }
#pragma unroll
  for (int cd = 0; cd < 4; ++cd)
#pragma unroll
    for (int wd = 0; wd < RW; ++wd) {
      unsigned v = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
        if (wd * 4 + bb < R) v |= (((unsigned)pk[wd * 4 + bb] >> (8 * cd)) & 0xffu) << (8 * bb);
      profTab[(cd * 64 + lane) * RW + wd] = (int)v;
    }
  // the job's codes of columns c * 64 - 64 .. c * 64 + 127, 192 / L per job lane
#pragma unroll
  for (int m = 0; m < 192 / L; ++m) {
    const int xx = ql + L * m;
    const int x = c * BG_CHUNK - 64 + xx;
    const int v = g2[x < 0 ? 0 : (x >= n2 ? n2 - 1 : x)];
    stage[xx] = (uint16_t)(((unsigned)x < (unsigned)n2) ? v * (32 * RW) : 0);
  }
  // row 0 above the pair's first lane at step u: column c * 64 + u (X form)
#pragma unroll
  for (int m = 0; m < 64 / L; ++m) {
    const int u = ql + L * m;
    const int col = c * BG_CHUNK + u;
    bIn[u] = 4 * wadd(row0_M(mode, col, a, b), -wmul(a, col)) + 2;
  }
  (void)NC;
  const int32_t* ck = reinterpret_cast<const int32_t*>(F.trace + P.trace_off / 4) +
                      (size_t)c * (R + 1) * BG_WAVE + P.lane0 + ql;
#pragma unroll
  for (int k = 0; k < R; ++k) { S.Y[k] = 4 * ck[k * BG_WAVE] + 3; S.tA[k] = 0; S.tB[k] = 0; }
  S.topPrev = 4 * ck[R * BG_WAVE] + 2;
  S.Xlast = S.Y[R - 1] - 1;
  C.bIn = bIn;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);
  C.codeLane = stage + 63 - ql;
  uint32_t* slot = win + (size_t)z * ck_grp_slot_dw<R, GP>();
  const bool edge = ballot(c == 0) != 0;
  if (edge) tag_chunk_jobs<R, true, GP>(S, C, c, slot, ql, j < nj);
  else tag_chunk_jobs<R, false, GP>(S, C, c, slot, ql, j < nj);
}

template <int R>
__device__ void recompute_chunk(const BgFinishArgs& F, const BgPair& P, int s, int c,
                                uint32_t* slot, int* area, int lane) {
  constexpr int RW = ProfW<R>::v;
  const int n1 = P.n1, n2 = P.n2, NC = P.nc;
  const int a = F.open, b = F.ext, mode = F.mode;
  int* bIn = area;
  int* profTab = area + 64;
  uint16_t* stage = reinterpret_cast<uint16_t*>(profTab + 4 * 64 * RW);
  TagCtx C;
  TagStrip<R> S;
  C.a = a; C.b = b; C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = lane;
  C.rowbase = s * BG_WAVE * R + lane * R;
  C.orow = R - 1;
  C.lastcol = nullptr; C.ring = nullptr; C.oLane = nullptr; C.mail = nullptr; C.bndOut = nullptr;
  const uint8_t* c1 = F.codes1 + P.off1;
  const uint8_t* g2 = F.codes2 + P.off2;
  int pk[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    const int q = (i <= n1) ? c1[i - 1] : 0;
    pk[k] = F.profile[(k == 0 ? 64 : 128) + (q >> 3)];
  }
#pragma unroll
  for (int cd = 0; cd < 4; ++cd)
#pragma unroll
    for (int wd = 0; wd < RW; ++wd) {
      unsigned v = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
        if (wd * 4 + bb < R) v |= (((unsigned)pk[wd * 4 + bb] >> (8 * cd)) & 0xffu) << (8 * bb);
      profTab[(cd * 64 + lane) * RW + wd] = (int)v;
    }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int x = c * BG_CHUNK - 64 + lane + 64 * q;
    const int v = g2[x < 0 ? 0 : (x >= n2 ? n2 - 1 : x)];
    stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? v * (32 * RW) : 0);
  }
  const int jb = c * BG_CHUNK + lane;
  if (s == 0) {
    bIn[lane] = 4 * wadd(row0_M(mode, jb, a, b), -wmul(a, jb)) + 2;
  } else {
    bIn[lane] = 4 * F.bndM[P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb] + 2;
  }
  const int32_t* ck = reinterpret_cast<const int32_t*>(F.trace + P.trace_off / 4) +
                      ((size_t)(s * NC + c) * (R + 1)) * BG_WAVE + lane;
#pragma unroll
  for (int k = 0; k < R; ++k) { S.Y[k] = 4 * ck[k * BG_WAVE] + 3; S.tA[k] = 0; S.tB[k] = 0; }
  S.topPrev = 4 * ck[R * BG_WAVE] + 2;
  S.Xlast = S.Y[R - 1] - 1;
  C.bIn = bIn;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);
  C.codeLane = stage + 63 - lane;
  C.trace = slot - (size_t)(2 * c) * (R * 2 * BG_WAVE);    // tag_chunk adds ((t0 >> 5) + h) blocks
  if (c == 0) tag_chunk<R, TV_EDGE, false, KIND_RECOMP>(S, C, c);
  else tag_chunk<R, TV_FAST, false, KIND_RECOMP>(S, C, c);
}

// ---- affine / local checkpoint traceback (bg_aff_kernel.hip): a recomputed chunk holds the
// full 4-bit trace, two 32-step blocks of [row k][lane] x uint4
template <int R>
__host__ __device__ constexpr int ack_slots() { return R >= 8 ? 4 : (R >= 4 ? 5 : 8); }
template <int R, bool LOCAL>
__host__ __device__ constexpr int ack_slot_dw() { return 2 * ack_planes<LOCAL>() * R * BG_WAVE; }
// per-wave recompute area: (M, X) boundary block, 192 u16 codes; the K x 64 x RW profile dwords
// of the strip being recomputed are shared by the workgroup's waves (ack_prof_ints)
constexpr int kAckWaveInts = 128 + 96;
template <int R>
__host__ __device__ constexpr int ack_prof_ints(int K) { return K * 64 * AffW<R>::v; }
// chunk map: direct-mapped (strip & 15, chunk & 15) -> (s << 20 | c << 4 | slot)
constexpr int kCkMapEntries = 256;
// asynchronous recomputation: at most this many chunks ahead of the walker in its strip / in the
// strip above (the depth used, and how close to the strip's top the strip above is prefetched,
// are BgFinishArgs::specDepth / specAbove: tools/r05/spec_ab.sh measured less speculation only
// adding misses — every recomputed chunk is one the walk needs)
#ifndef BG_SPEC_DEPTH
#define BG_SPEC_DEPTH 2
#endif
constexpr int kSpecDepth = BG_SPEC_DEPTH;
// asynchronous recomputation: polls of the chunk map before the walker serves its own request
constexpr int kSelfPolls = 4096;
__device__ __forceinline__ int ck_map_idx(int s, int c) { return ((s & 15) << 4) | (c & 15); }

// Bounded waits of the asynchronous traceback (BgFinishArgs::waitTicks, s_memrealtime at 100 MHz)
__device__ __forceinline__ bool wait_expired(const BgFinishArgs& F, unsigned long long t0) {
  return (long long)(__builtin_amdgcn_s_memrealtime() - t0) > (long long)F.waitTicks;
}
// The slot lock of the asynchronous traceback (sh[36]): lane 0 tries, the wave decides uniformly
// (SGPR loop state, so no register of the loops around it is taken); false when the wait bound
// ran out.  Holders keep it for a slot scan of straight-line code only.
__device__ __forceinline__ bool slot_lock(const BgFinishArgs& F, int* lk, int lane) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int sp = 0;; ++sp) {
    int got = 0;
    if (lane == 0) got = __hip_atomic_exchange(lk, 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
    if (__builtin_amdgcn_readfirstlane(got)) return true;
    __builtin_amdgcn_s_sleep(1);
    if ((sp & 255) == 255 && wait_expired(F, t0)) return false;
  }
}

// The first wait of an execute that ran out writes where it stood (one lane; include/
// biogarden_gpu.h bg_wait_diag): the kind, the pair, the wave, the awaited key, its map entry,
// the slots' filling flags and keys, the lock word, the walker's cell and its recomputations
__device__ __forceinline__ void wait_diag(const BgFinishArgs& F, int kind, int pidx, int wave, int key,
                                       const unsigned* ckMap, int* sh, int nSlots, int k, int l,
                                       int selfN) {
  if (!F.wdiag) return;
  if (atomicCAS(F.wdiag, 0u, (unsigned)kind) != 0u) return;
  uint32_t* d = F.wdiag;
  d[1] = (uint32_t)pidx;
  d[2] = (uint32_t)wave;
  d[3] = (uint32_t)key;
  d[4] = key >= 0 ? ckMap[ck_map_idx(key >> 16, key & 0xffff)] : 0xFFFFFFFFu;
  unsigned fl = 0;
  for (int z = 0; z < nSlots && z < 8; ++z) {
    if (__hip_atomic_load(&sh[48 + z], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) fl |= 1u << z;
    d[10 + z] = (uint32_t)sh[40 + z];
  }
  d[5] = fl;
  d[6] = (uint32_t)__hip_atomic_load(&sh[36], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  d[7] = (uint32_t)k;
  d[8] = (uint32_t)l;
  d[9] = (uint32_t)selfN;
  __threadfence();
}

// this wave-lane's profile entries for strip s, built by the whole workgroup
template <int R>
__device__ void build_prof_aff(const BgFinishArgs& F, const BgPair& P, int s, int* profTab, int tid, int NT) {
  constexpr int RW = AffW<R>::v;
  const int K = F.kdim, n1 = P.n1;
  const uint8_t* c1 = F.codes1 + P.off1;
  const int16_t* tab = reinterpret_cast<const int16_t*>(F.profile);
  for (int x = tid; x < K * 64; x += NT) {
    const int lane = x & 63, cd = x >> 6;
    const int rowbase = s * BG_WAVE * R + lane * R;
#pragma unroll
    for (int wd = 0; wd < RW; ++wd) {
      unsigned v = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int k = wd * 4 + bb, i = rowbase + k + 1;
        if (k < R) v |= ((unsigned)tab[(i <= n1 ? c1[i - 1] : 0) * F.pstride + cd] & 0xffu) << (8 * bb);
      }
      profTab[(cd * 64 + lane) * RW + wd] = (int)v;
    }
  }
}

template <int R, bool LOCAL, bool FIND, bool LCS = false>
__device__ void recompute_chunk_aff(const BgFinishArgs& F, const BgPair& P, int s, int c,
                                    uint32_t* slot, int* area, const int* profTab, int lane,
                                    int fq, int fl, int target, int* foundOut) {
  constexpr int RW = AffW<R>::v;
  const int n1 = P.n1, n2 = P.n2, NC = P.nc;
  const int a = F.open, b = F.ext, mode = F.mode;
  int2* bIn = reinterpret_cast<int2*>(area);
  uint16_t* stage = reinterpret_cast<uint16_t*>(area + 128);
  AffCtx C;
  AffStrip<R, LOCAL> S;
  C.a = a; C.b = b; C.e = wadd(b, -a); C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = lane;
  C.rowbase = s * BG_WAVE * R + lane * R;
  C.orow = R - 1;
  C.lastcol = nullptr; C.ring = nullptr; C.oLane = nullptr; C.mail = nullptr;
  C.bndOutM = nullptr; C.bndOutX = nullptr;
  (void)n1;
  const uint8_t* g2 = F.codes2 + P.off2;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int x = c * BG_CHUNK - 64 + lane + 64 * q;
    const int v = g2[x < 0 ? 0 : (x >= n2 ? n2 - 1 : x)];
    stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? v * (256 * RW) : 0);
  }
  const int jb = c * BG_CHUNK + lane;
  if (s == 0) {
    bIn[lane] = make_int2(aff_row0<LOCAL>(mode, jb, a, b), kAffNeg);
  } else {
    const size_t o = P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb;
    bIn[lane] = make_int2(F.bndM[o], F.bndX[o]);
  }
  const int32_t* ck = reinterpret_cast<const int32_t*>(F.trace + P.trace_off / 4) +
                      ((size_t)(s * NC + c) * (2 * R + 2)) * BG_WAVE + lane;
#pragma unroll
  for (int k = 0; k < R; ++k) { S.M[k] = ck[k * BG_WAVE]; S.Y[k] = ck[(R + k) * BG_WAVE]; }
  S.topPrev = ck[2 * R * BG_WAVE];
  S.Xlast = ck[(2 * R + 1) * BG_WAVE];
  C.bIn = bIn;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);
  C.codeLane = stage + 63 - lane;
  int found = -1;
  if (c == 0) aff_recomp<R, LOCAL, true, FIND, LCS>(S, C, c, slot, fq, fl, target, found);
  else aff_recomp<R, LOCAL, false, FIND, LCS>(S, C, c, slot, fq, fl, target, found);
  if constexpr (FIND) {
    if (lane == fl) *foundOut = found;
  }
}

// GRP: grouped pairs, GRP per wave (BgFinishArgs::grouped; own instantiations, bg_grp_finish.hip,
// so the other checkpoint kernels carry none of its registers); 0 otherwise
template <int R, bool AFFINE, int MODE, bool CK = false, int GRP = 0>
__global__ __launch_bounds__(256) void bg_finish_kernel(BgFinishArgs F) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u64 tK0 = __builtin_readcyclecounter();       // BG_DEBUG=finish: the kernel's phases
  const u64 tR0 = __builtin_amdgcn_s_memrealtime();
  constexpr int NW = AFFINE ? 4 : 2;
  constexpr int ROWS = BG_WAVE * R;
  constexpr int BLK_DW = R * BG_WAVE * NW;             // dwords per 32-step trace block
  const int NBW = F.win_bytes / (BLK_DW * 4);          // blocks per window
  uint32_t* win = reinterpret_cast<uint32_t*>(smem);
  int* sh = reinterpret_cast<int*>(smem + F.win_bytes);  // 64 ints of block-shared scalars
  // 2 x 256 ints: the end-cell keys before the walk and the column scan after it, both while the
  // window holds no trace
  int* scan = reinterpret_cast<int*>(smem);
  // checkpoint mode: the window is ck_slots<R>() recomputed chunks; sh[16+z] / sh[24+z] = strip /
  // chunk held by slot z (-1: empty); per-wave recompute areas follow the scan
  int* ckArea = sh + 64;
  constexpr bool ACK = CK && AFFINE;                  // affine / local checkpoint traceback
  constexpr bool LIN_CK = CK && !AFFINE;              // linear checkpoint traceback
  // grouped pairs (BgFinishArgs::grouped): 16-lane chunks, recomputed up to four per pass
  constexpr bool grpMode = LIN_CK && GRP > 0;
  constexpr int GL = GRP > 0 ? 64 / GRP : 64;          // grouped: lanes per pair
  const int ckAreaInts = ACK ? kAckWaveInts : (grpMode ? ck_grp_wave_ints<R>() : ck_wave_ints<R>());
  int* profShared = ckArea;                           // ACK: the strip's profile entries
  if constexpr (ACK) ckArea += F.area_ints;
  int profS = -1;                                     // ACK: strip whose profile is built
  constexpr int kSlotDw = ACK ? ack_slot_dw<R, MODE == BGK_LOCAL>() : ck_slot_dw<R>();
  const int slotDw = grpMode ? ck_grp_slot_dw<R, (GRP > 0 ? GRP : 4)>() : kSlotDw;   // linear checkpoint slots
  const int NWV = (int)(blockDim.x >> 6);              // waves: walker + recompute helpers
  int* jscr = ckArea + (CK ? NWV * ckAreaInts : 0);
  // checkpoint mode: direct-mapped table (strip & 31, chunk & 31) -> (s << 20 | c << 4 | slot)
  unsigned* ckMap = reinterpret_cast<unsigned*>(jscr);
  if (CK) {
    for (int x = threadIdx.x; x < kCkMapEntries; x += blockDim.x) ckMap[x] = 0xFFFFFFFFu;
    __syncthreads();
  }
  const u64 tK1 = __builtin_readcyclecounter();       // BG_DEBUG=finish

  // split traceback phases (linear checkpoint traceback only, BgFinishArgs::phase): WALK runs one
  // strip of a pair per workgroup (F.splitMap), the others one pair per workgroup
  const int ph = LIN_CK ? F.phase : (int)BG_PH_FULL;
  int pidx = (int)blockIdx.x, wstrip = -1;
  if (ph == BG_PH_WALK) {
    const int2 m = F.splitMap[blockIdx.x];
    pidx = m.x;
    wstrip = m.y;
  }
  const BgPair& P = F.pairs[pidx];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6), NT = blockDim.x;
  int32_t* spl = nullptr;                              // the pair's split area
  BgSplitLayout SL{};
  if (ph != BG_PH_FULL) {
    SL = bg_split_layout(P.n1, P.n2, P.nstrips, P.nc, R, F.segc);
    spl = F.split + P.split_off;
    if (ph == BG_PH_WALK && spl[SL.startcol + wstrip] < 0) return;   // the chain did not reach it
  }
  Fin f;
  f.F = &F; f.P = &P;
  f.n1 = P.n1; f.n2 = P.n2; f.a = F.open; f.b = F.ext; f.mode = F.mode;
  f.s1 = F.seq1 + P.off1;
  f.s2 = F.seq2 + P.off2;
  f.lastrowMa = (P.nstrips > 0) ? F.bndM + P.bnd_off + (size_t)(P.nstrips - 1) * P.nc * BG_CHUNK : nullptr;
  f.lastcol = F.aux + P.aux_off;
  const int n1 = f.n1, n2 = f.n2;
  constexpr int mode = MODE;
  const int cap = n1 + n2;
  uint8_t* ob = F.out1 + P.out_off;                    // op codes, then aligned seq1 (in place)
  uint8_t* ob2 = F.out2 + P.out_off;

  // ---------------- end cell (aligner.rs:112, 173-176, 247-251, 308-312, 369-389): every
  // thread folds a strided share into 64-bit keys (value, then the index rule), the waves'
  // keys meet in LDS.  Keys: row/column folds `>= last` and `> first` become max of
  // (bias(v) << 32 | j) and (bias(v) << 32 | ~i).  The split phases after HEAD read it back.
  if (ph != BG_PH_FULL && ph != BG_PH_HEAD) {
    if (tid == 0) {
      sh[0] = spl[SL.head + 0]; sh[1] = spl[SL.head + 1]; sh[2] = spl[SL.head + 2];
      sh[3] = spl[SL.head + 3]; sh[9] = 0;
    }
  } else {
    u64 ka = 0, kb = 0;
    const int32_t* rowbest = f.lastcol + (n1 + 1);
    // split HEAD: the keys of i, j >= 1 were folded by bg_endkey_kernel; the border cells here
    const bool folded = ph == BG_PH_HEAD && F.keys != nullptr && n1 > 0 && n2 > 0 && P.nstrips > 0 &&
                        (mode == BGK_SEMIGLOBAL || mode == BGK_OVERLAP || mode == BGK_FITTING);
    // grouped pairs (semiglobal / overlap): the DP folded the last row's key (bg_grp_kernel.hip)
    const bool rowFolded = GRP > 0 && !folded && F.keys != nullptr && n1 > 0 && n2 > 0 && P.nstrips > 0 &&
                           (mode == BGK_SEMIGLOBAL || mode == BGK_OVERLAP);
    if (rowFolded && tid == 0) {
      const u64 kb0 = (u64)bias(lastrowM(f, 0)) << 32;
      kb = F.keys[2 * (size_t)pidx + 1];
      kb = kb0 > kb ? kb0 : kb;
    }
    if (folded) {
      if (tid == 0) {
        ka = F.keys[2 * (size_t)pidx];
        kb = F.keys[2 * (size_t)pidx + 1];
        const u64 ka0 = ((u64)bias(lastcolM(f, 0)) << 32) | 0xFFFFFFFFu;
        const u64 kb0 = (u64)bias(lastrowM(f, 0)) << 32;
        ka = ka0 > ka ? ka0 : ka;
        kb = kb0 > kb ? kb0 : kb;
      }
    } else if (mode == BGK_LOCAL) {
      // first row-major cell with the strict maximum; (0,0) with 0 when nothing is positive
      if (n2 > 0) {
#pragma unroll 4
        for (int i = 1 + tid; i <= n1; i += NT) {
          const u64 kk = ((u64)bias(rowbest[i - 1]) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
          ka = kk > ka ? kk : ka;
        }
      }
    } else if (mode == BGK_FITTING || mode == BGK_SEMIGLOBAL) {
      // last column, first strict max (:247, :376); the border cell (i = 0) apart, then kEndU
      // loads in flight per thread (one load per pass serialised C4's 10 k-column row fold:
      // ~105 k cycles per pair before the walk)
      if (tid == 0) ka = ((u64)bias(lastcolM(f, 0)) << 32) | 0xFFFFFFFFu;
      if (n2 == 0) {
        for (int i = 1 + tid; i <= n1; i += NT) {
          const u64 kk = ((u64)bias(lastcolM(f, i)) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
          ka = kk > ka ? kk : ka;
        }
      } else {
        for (int i0 = 1 + tid; i0 <= n1; i0 += NT * kEndU) {
          int v[kEndU];
#pragma unroll
          for (int u = 0; u < kEndU; ++u) v[u] = i0 + u * NT <= n1 ? f.lastcol[i0 + u * NT] : 0;
#pragma unroll
          for (int u = 0; u < kEndU; ++u) {
            const int i = i0 + u * NT;
            const u64 kk = ((u64)bias(v[u]) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
            ka = (i <= n1 && kk > ka) ? kk : ka;
          }
        }
      }
    }
    if (!folded && !rowFolded && (mode == BGK_OVERLAP || mode == BGK_SEMIGLOBAL)) {
      // last row, last max (:308, :369): the border cell (j = 0) apart, kEndU loads in flight
      if (tid == 0) kb = (u64)bias(lastrowM(f, 0)) << 32;
      if (n1 == 0) {
        for (int j = 1 + tid; j <= n2; j += NT) {
          const u64 kk = ((u64)bias(lastrowM(f, j)) << 32) | (unsigned)j;
          kb = kk > kb ? kk : kb;
        }
      } else {
        for (int j0 = 1 + tid; j0 <= n2; j0 += NT * kEndU) {
          int v[kEndU];
#pragma unroll
          for (int u = 0; u < kEndU; ++u) v[u] = j0 + u * NT <= n2 ? f.lastrowMa[j0 + u * NT] : 0;
#pragma unroll
          for (int u = 0; u < kEndU; ++u) {
            const int j = j0 + u * NT;
            const u64 kk = ((u64)bias(lastrow_from(f, v[u], j)) << 32) | (unsigned)j;
            kb = (j <= n2 && kk > kb) ? kk : kb;
          }
        }
      }
    }
    ka = wave_max_u64(ka);
    kb = wave_max_u64(kb);
    u64* wk = reinterpret_cast<u64*>(scan);          // 2 keys per wave
    if (lane == 0) { wk[2 * wid] = ka; wk[2 * wid + 1] = kb; }
    __syncthreads();
    if (tid == 0) {
      for (int x = 1; x < NT / 64; ++x) {
        ka = wk[2 * x] > ka ? wk[2 * x] : ka;
        kb = wk[2 * x + 1] > kb ? wk[2 * x + 1] : kb;
      }
      int ei = n1, ej = n2, score = 0, colcase = 0;
      if (mode == BGK_GLOBAL) {
        score = lastcolM(f, n1);
      } else if (mode == BGK_LOCAL) {
        const int v = unbias((unsigned)(ka >> 32));
        if (ka != 0 && v > 0) {
          ei = (int)(0xFFFFFFFFu - (unsigned)ka);
          ej = rowbest[n1 + ei - 1];                 // rowpos follows rowbest (ACK: its chunk)
          score = v;
        } else {
          ei = 0; ej = 0; score = 0;
        }
      } else if (mode == BGK_FITTING) {
        ei = (int)(0xFFFFFFFFu - (unsigned)ka); ej = n2; score = unbias((unsigned)(ka >> 32));
      } else if (mode == BGK_OVERLAP) {
        ei = n1; ej = (int)(unsigned)kb; score = unbias((unsigned)(kb >> 32));
      } else {
        const int mr = unbias((unsigned)(kb >> 32)), mc = unbias((unsigned)(ka >> 32));
        colcase = mc > mr;                           // (:389)
        if (colcase) { ei = (int)(0xFFFFFFFFu - (unsigned)ka); ej = n2; score = mc; }
        else { ei = n1; ej = (int)(unsigned)kb; score = mr; }
      }
      sh[0] = ei; sh[1] = ej; sh[2] = score; sh[3] = colcase; sh[9] = 0;
    }
  }
  const u64 tR1 = __builtin_amdgcn_s_memrealtime();  // this wave at the end-cell barrier
  __syncthreads();
  const u64 tK2 = __builtin_readcyclecounter();       // BG_DEBUG=finish: end cell known
  if (F.dbg && (threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < 2) {
    u64* d = F.dbg + (size_t)F.pairs[(ph == BG_PH_WALK) ? F.splitMap[blockIdx.x].x : blockIdx.x].index * 16;
    d[11 + 2 * (threadIdx.x >> 6)] = tR0;
    d[12 + 2 * (threadIdx.x >> 6)] = tR1;
  }
  const int ei = uni(sh[0]), score = uni(sh[2]), colcase = uni(sh[3]);
  int ej = uni(sh[1]);
  if (ph == BG_PH_HEAD) {
    // the split head: end cell, score, column case; the start strip for the exit pass and chain
    if (tid == 0) {
      spl[SL.head + 0] = ei; spl[SL.head + 1] = ej; spl[SL.head + 2] = score; spl[SL.head + 3] = colcase;
      spl[SL.head + 4] = -1; spl[SL.head + 5] = 0; spl[SL.head + 6] = 0;
      spl[SL.head + 7] = (P.nstrips > 0 && ei >= 1 && ej >= 1) ? (ei - 1) / ROWS : -1;
    }
    return;
  }

  // ---------------- semiglobal tail gaps (:389-404): the last ntail columns of the slot; the
  // walk's op codes (0 = (s1, s2), 1 = (s1, '-'), 2 = ('-', s2)) go backwards in front of them
  const int ntail = (mode == BGK_SEMIGLOBAL) ? (colcase ? n1 - ei : n2 - ej) : 0;

  // ---------------- traceback walk (aligner.rs:511-592)
  const uint32_t* tr = F.trace + P.trace_off / 4;
  const size_t stripDw = (size_t)P.nc * (BG_CHUNK / BG_TRACE_BLK) * BLK_DW;
  const int stripBlocks = P.nc * (BG_CHUNK / BG_TRACE_BLK);
  int k = ei, l = ej, state = 0, status = 0, ncore = 0;
  int curS = -1, curB0 = 0, curNb = 0;
  // where the walk's ops go (backwards from capw, after ntw columns): the pair's slot, or (WALK)
  // the strip's scratch; a WALK stops at the first cell of the strip above (splitTop)
  uint8_t* obw = ob;
  int capw = cap, ntw = ntail, splitTop = 0, crossed = 0;
  if (ph == BG_PH_WALK) {
    const int sStar = spl[SL.head + 7];
    k = (wstrip == sStar) ? ei : (wstrip + 1) * ROWS;
    l = spl[SL.startcol + wstrip];
    splitTop = wstrip * ROWS;
    obw = reinterpret_cast<uint8_t*>(spl) + SL.ops + (size_t)wstrip * SL.capS;
    capw = SL.capS;
    ntw = 0;
  }
  const int kStart = k, lStart = l;
  // an op index outside the walk's capacity (never expected: every move decrements k or l) is
  // dropped and the pair reported BG_INTERNAL instead of written out of bounds
  bool wild = false;
  auto put_op = [&](int at, int op) {
    const int idx = capw - 1 - at;
    if ((unsigned)idx < (unsigned)capw) obw[idx] = (uint8_t)op;
    else wild = true;
  };
  int k0 = -1000000, l0 = -1000000;                  // neighbourhood anchor (invalid)
  int codes = 0;
  // Transition table of backtrack (aligner.rs:520-586), per state, indexed by the 4-bit cell code
  // (bits 0-1 m_trace: 0 'R', 1 'X', 2 'Y', 3 STOP; bit 2 x_trace=='M'; bit 3 y_trace=='M').
  // Entry = (move << 2) | next state; move 0 none, 1 diag (op 0), 2 up (op 1), 3 left (op 2).
  constexpr u64 kLutM = [] {
    u64 v = 0;
    for (int c = 0; c < 16; ++c) {
      const int mt = c & 3;
      const u64 e = mt == 0 ? (1u << 2) | 0 : mt == 1 ? (2u << 2) | 1 : mt == 2 ? (3u << 2) | 2 : 0;
      v |= e << (4 * c);
    }
    return v;
  }();
  constexpr u64 kLutX = [] {
    u64 v = 0;
    for (int c = 0; c < 16; ++c) v |= (u64)((c & 4) ? 0 : ((2u << 2) | 1)) << (4 * c);
    return v;
  }();
  constexpr u64 kLutY = [] {
    u64 v = 0;
    for (int c = 0; c < 16; ++c) v |= (u64)((c & 8) ? 0 : ((3u << 2) | 2)) << (4 * c);
    return v;
  }();
  constexpr int kCkSlots0 = ACK ? ack_slots<R>() : ck_slots<R>();
  constexpr int kCkSlots = (grpMode && kGrpSlots > kCkSlots0) ? kGrpSlots : kCkSlots0;
  int ckS[kCkSlots], ckC[kCkSlots];                  // checkpoint mode: resident chunks
  // slots in use (the host trades cache for more resident workgroups on many-pair batches)
  const int maxSlots = grpMode ? kGrpSlots : kCkSlots0;
  const int nSlots = (F.nslots > 0 && F.nslots < maxSlots) ? F.nslots : maxSlots;
  int ckNext = 0;                                    // next slot to fill (FIFO)
#pragma unroll
  for (int z = 0; z < kCkSlots; ++z) { ckS[z] = -1; ckC[z] = -1; }
  // decodes the 8x8 neighbourhood anchored at (k, l): lane (dk, dl) holds cell (k - dk, l - dl)
  // 4-bit code of cell (kk, ll) from the resident trace (window or recomputed chunks); the chunk-
  // map entry it used goes to usedIdx / usedE (verification builds, BG_SEQCHECK)
  int usedIdx = -1;
  unsigned usedE = 0;
  auto decode_cell = [&](int kk, int ll) -> int {
    usedIdx = -1;
    if (splitTop > 0 && kk <= splitTop) return kCodeSplit;             // the strip above (WALK)
    if (kk <= 0 || ll <= 0) return kCodeBorder | ((kk == 0) ? 2 : 1);  // column 0 'X', row 0 'Y'
    const int vr = kk - 1;
    const int sidx = vr / ROWS, rem = vr - sidx * ROWS, r = rem / R, q = rem - r * R;
    const int t = ll + r, bl = t >> 5;
    if constexpr (CK) {
      const int cc = t >> 6;
      // (s << 20 | c << 4 | slot); an atomic load: helper waves publish chunks concurrently
      const int mi = ck_map_idx(sidx, cc);
      const unsigned e = __hip_atomic_load(&ckMap[mi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((e >> 4) != (((unsigned)sidx << 16) | (unsigned)cc) || e == 0xFFFFFFFFu) return kCodeMiss;
      const int z = (int)(e & 15);
      if (z >= nSlots) return kCodeMiss;                 // never published (guard)
      usedIdx = mi;
      usedE = e;
      if constexpr (ACK) {
        // bit planes (aff_recomp): not-Y, not-X, x_trace 'I', y_trace 'I' [, local stop]
        constexpr int NP = ack_planes<MODE == BGK_LOCAL>();
        const uint32_t* wp = win + (size_t)z * kSlotDw + ((bl & 1) * NP * R + q) * BG_WAVE + r;
        const int bit = 31 - (t & 31);
        const unsigned nY = (wp[0] >> bit) & 1, nX = (wp[R * BG_WAVE] >> bit) & 1;
        const unsigned xI = (wp[2 * R * BG_WAVE] >> bit) & 1, yI = (wp[3 * R * BG_WAVE] >> bit) & 1;
        int mt = nY ? (nX ? 0 : 1) : 2;
        if constexpr (MODE == BGK_LOCAL) mt = ((wp[4 * R * BG_WAVE] >> bit) & 1) ? 3 : mt;
        return mt | ((xI ^ 1) << 2) | ((yI ^ 1) << 3);
      }
      const uint32_t* wp = grpMode ? win + (size_t)z * slotDw + (((bl & 1) * R + q) * GL + r) * 2
                                   : win + (size_t)z * kSlotDw + (((bl & 1) * R + q) * BG_WAVE + r) * 2;
      const uint2 v = *reinterpret_cast<const uint2*>(wp);
      const int u = t & 31;
      const int tg = (int)((u < 16 ? v.x : v.y) >> (2 * (u & 15))) & 3;
      return ((0x2100 >> (4 * tg)) & 3) | 12;
    } else {
      if (sidx != curS || bl < curB0 || bl >= curB0 + curNb) return kCodeMiss;
      const uint32_t* wp = win + (((bl - curB0) * R + q) * BG_WAVE + r) * NW;
      const int bit = 31 - (t & 31);
      if constexpr (AFFINE) {
        const uint4 v = *reinterpret_cast<const uint4*>(wp);
        return (((v.x >> bit) & 1) << 1) | ((v.y >> bit) & 1) | (((v.z >> bit) & 1) << 2) | (((v.w >> bit) & 1) << 3);
      } else if (F.tag) {
        const uint2 v = *reinterpret_cast<const uint2*>(wp);  // 2-bit codes, 16 steps/word
        const int u = t & 31;
        const int tg = (int)((u < 16 ? v.x : v.y) >> (2 * (u & 15))) & 3;
        return ((0x2100 >> (4 * tg)) & 3) | 12;                // tag 0 'R', 2 'X', 3 'Y'
      } else {
        const uint2 v = *reinterpret_cast<const uint2*>(wp);
        return (((v.x >> bit) & 1) << 1) | ((v.y >> bit) & 1) | 12;
      }
    }
  };
  // decodes the 8x8 neighbourhood anchored at (k, l): lane (dk, dl) holds cell (k - dk, l - dl)
  u64 tDec = 0, nDec = 0;                                // BG_DEBUG=finish: decodes
  bool asyncPos = false;                                 // set below: post the walker's position
  auto reanchor = [&](int ka, int la) {
    k0 = ka; l0 = la;
    if (asyncPos && lane == 0) {
      __hip_atomic_store(&sh[34], ka, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&sh[35], la, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const u64 td0 = F.dbg ? __builtin_readcyclecounter() : 0;
    if (CK && asyncPos && BG_SEQCHECK) {
      // Verification builds (BG_SEQCHECK=1): prove that no slot this decode read was re-assigned
      // meanwhile.  A helper invalidates a slot's map entry before it writes into the slot and
      // one wave's LDS operations complete in order, so every lane re-reads the entry it used
      // after the decode; a changed entry means the codes may be torn: decode again.  The
      // shipped build relies on the eviction rules instead (see the helper loop): for prefetches
      // a helper evicts only empty, dead (right of / below a position the walker has already
      // left) or stale slots, and footprint-unguarded ones only for a pending request, while the
      // walker waits and decodes nothing; a served request is withdrawn at once, so no helper
      // acts on one the walker has moved past.  tools/verify_seqcheck.sh counts the retries.
      for (;;) {
        codes = decode_cell(k0 - (lane >> 3), l0 - (lane & 7));
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const bool same = usedIdx < 0 ||
            __hip_atomic_load(&ckMap[usedIdx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == usedE;
        const u64 bad = ballot(!same);
        if (!bad) break;
#if BG_FIN_DEBUG
        {
          const int bl = (int)__builtin_ctzll(bad);
          const unsigned ue = (unsigned)__shfl((int)usedE, bl, 64);
          const int ui = __shfl(usedIdx, bl, 64);
          const unsigned now = ckMap[ui];
          const int vw = k0 - 1, sw = vw / ROWS, remw = vw - sw * ROWS, ccw = (l0 + remw / R) >> 6;
          if (lane == 0)
            printf("BGDBG pair %d: a slot was re-assigned during the decode at (%d, %d) strip %d chunk %d: "
                   "lane %d read chunk (%u, %u) slot %u, entry now %08x, slots [%d %d %d %d %d %d %d %d] filling [%d%d%d%d%d%d%d%d] req %d\n",
                   P.index, k0, l0, sw, ccw, bl, ue >> 20, (ue >> 4) & 0xffff, ue & 15, now,
                   sh[40], sh[41], sh[42], sh[43], sh[44], sh[45], sh[46], sh[47],
                   sh[48], sh[49], sh[50], sh[51], sh[52], sh[53], sh[54], sh[55], sh[33]);
        }
#endif
      }
    } else {
      codes = decode_cell(k0 - (lane >> 3), l0 - (lane & 7));
    }
    if (F.dbg) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      codes = __builtin_amdgcn_readfirstlane(0) + codes;
      tDec += __builtin_readcyclecounter() - td0;
      ++nDec;
    }
  };
  if constexpr (ACK && MODE == BGK_LOCAL) {
    // the end cell's column: the first j of row ei with M == score lies in the chunk where the
    // row's running maximum last rose (rowpos); recompute that chunk into slot 0 and find it
    if (score > 0) {
      const int vr = ei - 1, s0 = vr / ROWS, rem = vr - s0 * ROWS, cc = ej;
      build_prof_aff<R>(F, P, s0, profShared, tid, NT);
      profS = s0;
      __syncthreads();
      if (wid == 0)
        recompute_chunk_aff<R, true, true>(F, P, s0, cc, win, ckArea, profShared, lane, rem % R, rem / R,
                                           score, sh + 12);
      __syncthreads();
      ej = uni(sh[12]);
      if (ej < 1) { ej = 0; status = 4; }   // unreachable: the forward pass saw the maximum there
      l = ej;
      ckS[0] = s0; ckC[0] = cc; ckNext = 1;
      if (tid == 0) ckMap[ck_map_idx(s0, cc)] = ((unsigned)s0 << 20) | ((unsigned)cc << 4);
      __syncthreads();
      if (status) { k = 0; l = 0; }
    }
  }
  // ---- split traceback, TAIL: stitch the strip walks.  Strip s* (the start cell's) was walked from
  // the start cell, every strip s < s* the chain reached from the cell in its bottom row where the
  // path enters it.  Going up from s*, a strip's walk is taken while it started exactly where the
  // walk below it crossed into it; its ops are copied into the slot in walk order.  The first walk
  // that ended inside its strip ends the traceback; if the chain broke before (an exit-pass
  // overflow, or any inconsistency), the walker below continues from the last crossing, so the
  // result never depends on the exit pass.
  bool preDone = false;
  int ffOps = 0;                                       // ops stitched from the strip walks
  if (ph == BG_PH_TAIL) {
    const int sStar = spl[SL.head + 7];
    const int* scol = spl + SL.startcol;
    const BgStripHdr* hd = reinterpret_cast<const BgStripHdr*>(spl + SL.hdr);
    int* preArr = scan + 512;                         // LDS: the window holds no trace yet
    const bool fits = sStar >= 0 && sStar + 1 + 512 <= F.win_bytes / 4;
    if (tid == 0) { sh[12] = -1; sh[13] = -1; }
    __syncthreads();
    if (fits) {
      for (int s = tid; s <= sStar; s += NT) {
        bool ok = scol[s] >= 0;
        int cr = 1;
        if (ok) {
          const BgStripHdr h = hd[s];
          if (s == sStar) {
            ok = h.sk == ei && h.sl == ej;
          } else {
            const BgStripHdr u = hd[s + 1];
            ok = scol[s + 1] >= 0 && u.crossed && h.sk == u.ek && h.sl == u.el;
          }
          ok = ok && h.status != 5 && h.nops >= 0 && h.nops < SL.capS;
          cr = h.crossed;
        }
        if (!ok) atomicMax(&sh[12], s);
        else if (!cr) atomicMax(&sh[13], s);
      }
    }
    __syncthreads();
    const int sb = fits ? sh[12] : sStar, sd = sh[13];
    // taken strips [lim, sStar]; fin: the walk ended in strip lim
    const bool fin = sd > sb;
    const int lim = fin ? sd : sb + 1;
    const int nt = (fits && lim <= sStar) ? sStar - lim + 1 : 0;
    if (nt > 0) {
      // ops before strip s in walk order: the strips above it in [s, sStar] (reversed index
      // x = sStar - s), one contiguous range per thread, then a scan of the thread sums
      const int per = (nt + NT - 1) / NT;
      const int x0 = tid * per < nt ? tid * per : nt, x1 = x0 + per < nt ? x0 + per : nt;
      int sum = 0;
      for (int x = x0; x < x1; ++x) sum += hd[sStar - x].nops;
      scan[tid] = sum;
      __syncthreads();
      for (int o = 1; o < NT; o <<= 1) {
        const int v = tid >= o ? scan[tid - o] : 0;
        __syncthreads();
        scan[tid] += v;
        __syncthreads();
      }
      int acc = scan[tid] - sum;
      for (int x = x0; x < x1; ++x) { preArr[x] = acc; acc += hd[sStar - x].nops; }
      const int total = scan[NT - 1];
      __syncthreads();
      // copy: one wave per strip; the strip's ops sit at the end of its scratch in the slot's order
      const uint8_t* scr = reinterpret_cast<const uint8_t*>(spl) + SL.ops;
      // (a strip's op count from the LDS prefix sums; its bytes loaded in rounds of CB per lane
      // before any is stored: one HBM round trip per strip rather than per 64 bytes)
      // (two strips per wave and round: both strips' loads go out before either's stores)
      constexpr int CB = 8;
      for (int x = wid; x < nt; x += 2 * NWV) {
        const int xb = x + NWV;
        const int na = (x + 1 < nt ? preArr[x + 1] : total) - preArr[x];
        const int nb = xb < nt ? (xb + 1 < nt ? preArr[xb + 1] : total) - preArr[xb] : 0;
        const uint8_t* srcA = scr + (size_t)(sStar - x) * SL.capS + (SL.capS - na);
        const uint8_t* srcB = scr + (size_t)(sStar - (xb < nt ? xb : x)) * SL.capS + (SL.capS - nb);
        uint8_t* dstA = ob + (cap - ntail - preArr[x] - na);
        uint8_t* dstB = ob + (cap - ntail - (xb < nt ? preArr[xb] : 0) - nb);
        for (int y0 = lane; y0 < na || y0 < nb; y0 += CB * 64) {
          uint8_t va[CB], vb[CB];
#pragma unroll
          for (int u = 0; u < CB; ++u) {
            const int y = y0 + 64 * u;
            va[u] = y < na ? srcA[y] : (uint8_t)0;
            vb[u] = y < nb ? srcB[y] : (uint8_t)0;
          }
#pragma unroll
          for (int u = 0; u < CB; ++u) {
            const int y = y0 + 64 * u;
            if (y < na) dstA[y] = va[u];
            if (y < nb) dstB[y] = vb[u];
          }
        }
      }
      ncore = total;
      ffOps = total;
      const BgStripHdr hl = hd[lim];
      k = hl.ek;
      l = hl.el;
      if (fin) { status = hl.status; preDone = true; }
      __threadfence_block();
      __syncthreads();
    }
    if (tid == 0) { spl[SL.head + 8] = nt; spl[SL.head + 9] = preDone ? 1 : 0; }   // bg_split_stats
  }
  u64 tJump = 0, tMiss = 0, nJump = 0, nMiss = 0, nRec = 0;   // BG_DEBUG=finish instrumentation
  u64 nSelf = 0;                                            // chunks the walker recomputed itself
  int lastReqS = -1, lastReqB = -1, sameReq = 0;            // barrier path: repeated requests
  const u64 tWalk0 = __builtin_readcyclecounter();

  // ---- linear checkpoint traceback, asynchronous recomputation.  The helper waves recompute
  // chunks ahead of the walker instead of all waves meeting at a barrier on every miss: the
  // walker posts its position (sh[34], sh[35]) and, on a miss, the chunk it needs (sh[33]); a
  // helper claims a slot under an LDS lock (sh[36]; per slot: chunk key sh[40+z], filling flag
  // sh[48+z]), recomputes the chunk and publishes it in ckMap; the walker spins on ckMap.  With
  // no request pending the helpers prefetch the chunks the walk heads into: left in its strip
  // down to the predicted exit, then the predicted entry of the strip above.  Eviction: a chunk
  // right of or below the walker is dead (the walk only moves up / left); a request may also
  // evict any slot outside the walker's 2 x 2 chunk footprint (it is waiting, so it reads none).
  const bool async = LIN_CK && NWV >= 2 && nSlots >= 5 && !(F.flags & BG_FIN_SYNC) && !grpMode;
  asyncPos = async;
  if (async) {
    if (tid == 0) {
      sh[32] = preDone ? 1 : 0; sh[33] = -1; sh[34] = k; sh[35] = l; sh[36] = 0; sh[37] = 0; sh[56] = -1;
      sh[59] = 0;                        // a wait that ran out: kind, key, recomputations, row, column
      for (int z = 0; z < 8; ++z) { sh[40 + z] = -1; sh[48 + z] = 0; }
    }
    __syncthreads();
  }
  int helperLost = 0;
  if (async && wid != 0) {
    const int NCp = P.nc, NSp = P.nstrips;
    auto enc = [](int key, int z) { return (unsigned)((key >> 16) << 20) | (unsigned)((key & 0xffff) << 4) | (unsigned)z; };
    auto resident = [&](int key) {
      const unsigned e = __hip_atomic_load(&ckMap[ck_map_idx(key >> 16, key & 0xffff)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return e != 0xFFFFFFFFu && (int)(e >> 4) == key;
    };
    int idle = 0;
    for (;;) {
      if (__hip_atomic_load(&sh[32], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
      int key = -1, zz = -1;
      // past the wait bound this helper stops helping (the walker serves itself) and the diag
      // names the lock's state
      if (!slot_lock(F, &sh[36], lane)) { helperLost = 1; break; }
      if (lane == 0) {
        const int req = __hip_atomic_load(&sh[33], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int kw = __hip_atomic_load(&sh[34], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int lw = __hip_atomic_load(&sh[35], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int vw = kw > 0 ? kw - 1 : 0;
        const int sw = vw / ROWS, remw = vw - sw * ROWS, ccw = (lw + remw / R) >> 6;
        const int xA = (lw + 63) >> 6;                     // the strip above, next to the walker
        // the column where the walk leaves this strip, from its slope since it entered it
        // (sh[56..58] = strip, row, column of the entry; diagonal until 16 rows are walked)
        if (sh[56] != sw) { sh[56] = sw; sh[57] = kw; sh[58] = lw; }
        const int dkIn = sh[57] - kw, dlIn = sh[58] - lw;
        const int lOut = lw - (dkIn >= 16 ? (int)((long)remw * dlIn / dkIn) : remw);
        const int cExit = lOut >> 6;                       // this strip's chunk at its top row
        const int xE = (lOut + 62) >> 6;                   // the strip above's entry chunk
        auto mk = [&](int ss, int cc) {
          return (ss < 0 || ss >= NSp || cc < 0 || cc >= NCp || (wstrip > 0 && ss < wstrip)) ? -1 : (ss << 16) | cc;
        };
        int cand[2 + 2 * kSpecDepth];
        constexpr int NCAND = 2 + 2 * kSpecDepth;
        cand[0] = req;
        cand[1] = mk(sw, ccw);
        // up to kSpecDepth chunks left of the walker in its strip, down to the predicted exit;
        // the strip above only near its boundary (earlier, the entry column is a poor guess)
        for (int d = 1; d <= kSpecDepth; ++d) {
          cand[1 + d] = (d <= F.specDepth && ccw - d >= cExit) ? mk(sw, ccw - d) : -1;
          cand[1 + kSpecDepth + d] = (d <= F.specDepth && remw < F.specAbove) ? mk(sw - 1, xE + 1 - d) : -1;
        }
        auto dead = [&](int kk) { const int ss = kk >> 16, cc = kk & 0xffff; return ss > sw || (ss == sw && cc > ccw); };
        auto guarded = [&](int kk) {
          const int ss = kk >> 16, cc = kk & 0xffff;
          return (ss == sw && (cc == ccw || cc == ccw - 1)) || (ss == sw - 1 && (cc == xA || cc == xA - 1));
        };
        for (int q = 0; q < NCAND && key < 0; ++q) {
          const int kk = cand[q];
          if (kk < 0) continue;
          // a filler publishes the chunk in the map, then clears its slot's filling flag: read
          // the flags first and the map second (acquire), or a chunk published between the two
          // reads looks neither resident nor in flight and is recomputed into a second slot (its
          // first copy then turns stale and may be evicted while the walker decodes from it)
          bool flying = false;
          for (int z = 0; z < nSlots; ++z)
            flying |= (__hip_atomic_load(&sh[48 + z], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0 &&
                       sh[40 + z] == kk);
          if (flying || resident(kk)) continue;
          // a slot: empty, stale (its chunk no longer in the map), dead, or (request) unguarded
          int pick = -1;
          for (int z = 0; z < nSlots && pick < 0; ++z) {
            if (sh[48 + z]) continue;
            const int oz = sh[40 + z];
            const bool stale = oz < 0 || ckMap[ck_map_idx(oz >> 16, oz & 0xffff)] != enc(oz, z);
            if (stale || dead(oz)) pick = z;
          }
          if (pick < 0 && q == 0)
            for (int z = 0; z < nSlots && pick < 0; ++z)
              if (!sh[48 + z] && !guarded(sh[40 + z])) pick = z;
          if (pick < 0) continue;
          const int oz = sh[40 + pick];
          if (oz >= 0) {
            unsigned& oe = ckMap[ck_map_idx(oz >> 16, oz & 0xffff)];
            if (oe == enc(oz, pick)) __hip_atomic_store(&oe, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          sh[40 + pick] = kk;
          sh[48 + pick] = 1;
          key = kk;
          zz = pick;
        }
        __hip_atomic_store(&sh[36], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // the slot's old map entry was invalidated above, before any write into the slot below
      // (one wave's LDS operations complete in order; keep the compiler from hoisting the
      // recomputation's stores): the walker's post-decode check relies on that order
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      key = uni(__shfl(key, 0, 64));
      zz = uni(__shfl(zz, 0, 64));
      // keys come from mk() (range-checked) or the walker's miss, which lies inside the pair's
      // strips and chunks; a key outside them would read beyond the pair's checkpoints
      if (key >= 0 && ((key >> 16) >= NSp || (key & 0xffff) >= NCp || zz < 0 || zz >= nSlots)) {
#if BG_FIN_DEBUG
        if (lane == 0) printf("BGDBG pair %d: helper key (%d, %d) slot %d\n", P.index, key >> 16, key & 0xffff, zz);
#endif
        if (lane == 0 && zz >= 0 && zz < nSlots)
          __hip_atomic_store(&sh[48 + zz], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        key = -1;
      }
      if (key < 0) {
        // idle: nothing to recompute ahead of the walk.  Each poll takes the lock and scans the
        // candidates on a SIMD the next execute's DP waves share; after BG_HELP_FAST idle polls
        // the helper polls BG_HELP_LONG x 64 cycles apart
        if (idle < BG_HELP_FAST) { help_pause(8); ++idle; }
        else help_pause(BG_HELP_LONG);
        continue;
      }
      idle = 0;
      recompute_chunk<R>(F, P, key >> 16, key & 0xffff, win + (size_t)zz * kSlotDw,
                         ckArea + wid * ckAreaInts, lane);
      if (F.dbg && lane == 0) __hip_atomic_fetch_add(&sh[37], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) {
        __hip_atomic_store(&ckMap[ck_map_idx(key >> 16, key & 0xffff)], enc(key, zz), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&sh[48 + zz], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  if (helperLost && lane == 0 &&
      __hip_atomic_compare_exchange_strong(&sh[59], &helperLost, BG_WD_LOCK_HELPER, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
    sh[60] = -1; sh[61] = 0; sh[62] = sh[34]; sh[63] = sh[35];
  }
  for (;;) {
    int reqS = -1, reqB0 = 0, done = preDone ? 1 : 0;
    if (wid == 0) {
      // the walk is one latency-bound wave: first claim on the issue slots it shares with the
      // next execute's DP waves (two-stream pipeline)
      if (!(F.flags & BG_FIN_NOPRIO)) __builtin_amdgcn_s_setprio(3);
      for (; !preDone;) {
        int dk = k0 - k, dl = l0 - l;
        if ((unsigned)dk >= 8u || (unsigned)dl >= 8u) { reanchor(k, l); dk = 0; dl = 0; }
        int c = rdlane(codes, dk * 8 + dl);
        if constexpr (!AFFINE) {
          // Linear gaps: inside the matrix x/y_trace are 'M', so states X/Y fall back to M
          // without moving and the walk is a chain of m_trace moves.  Resolve the chain through
          // the whole neighbourhood at once by pointer jumping (4 rounds of ds_bpermute over the
          // 64 cells); the border, STOP and window-miss cells stay with the scalar walker below.
          const bool jumpable = state == 0 && !(c & (kCodeMiss | kCodeBorder | kCodeSplit)) &&
                                (MODE != BGK_LOCAL || (c & 3) != 3);
          if (jumpable) {
            if ((dk | dl) != 0) { reanchor(k, l); c = rdlane(codes, 0); }
            const int cl = codes;
            const bool term = (cl & (kCodeMiss | kCodeBorder | kCodeSplit)) || (MODE == BGK_LOCAL && (cl & 3) == 3);
            const int mv = (int)(kLutM >> (4 * (cl & 15)) >> 2) & 3;   // 1 diag, 2 up, 3 left
            const int nk = (lane >> 3) + (mv != 3), nl = (lane & 7) + (mv != 2);
            const bool ex = !term && (nk >= 8 || nl >= 8);          // the move leaves the block
            int p = (term || ex) ? lane : nk * 8 + nl;
            int d = (term || ex) ? 0 : 1;
            // p <- p(p), d <- d + d(p) (4 rounds: chains of up to 16 cells), interleaved with
            // lane m finding the m-th cell of the chain from the anchor: round rr of that search
            // needs the pointers after 2^rr hops, i.e. p before jumping round rr, so the two
            // ds_bpermute chains overlap
            int x = 0;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
              const int y = __builtin_amdgcn_ds_bpermute(x * 4, p);
              const int qv = __builtin_amdgcn_ds_bpermute(p * 4, p | (d << 8));
              x = ((lane >> rr) & 1) ? y : x;
              p = qv & 255;
              d += qv >> 8;
            }
            const int opx = __builtin_amdgcn_ds_bpermute(x * 4, mv - 1);
            const int Pn = rdlane(p, 0), Dn = rdlane(d, 0);
            const int infoP = rdlane((ex ? 1 : 0) | (mv << 1), Pn);
            const int exP = infoP & 1, mvP = infoP >> 1;
            const int nops = Dn + exP;
#if BG_FIN_DEBUG
            if (lane == 0 && ntw + ncore + nops > capw)
              printf("BGDBG pair %d: jumper writes op %d of cap %d at (%d, %d)\n", P.index, ntw + ncore + nops, capw, k, l);
#endif
            if (lane < nops) put_op(ntw + ncore + lane, opx);
            ncore += nops;
            k -= Pn >> 3;
            l -= Pn & 7;
            // state on arrival: after an up / left move the reference sits in X / Y, which only
            // matters when the chain stopped on a border or window-miss cell
            const int mvIn = exP ? mvP : (Dn > 0 ? rdlane(opx, Dn - 1) + 1 : 1);
            if (exP) {
              k -= (mvP != 3);
              l -= (mvP != 2);
            }
            state = mvIn == 2 ? 1 : (mvIn == 3 ? 2 : 0);
            ++nJump;
            continue;
          }
        } else {
          // Affine gaps.  Inside the neighbourhood the X / Y runs of the 3-state walk are resolved
          // first: an X node at (dk, dl) moves up until the first cell whose x_trace is 'M'
          // (there it falls back to M without moving, aligner.rs:566-585) or that ends the walk,
          // found by one find-first-set over a 64-bit lane mask; the same for Y along the row.
          // What is left is a chain over the 64 M nodes with weights (ops per hop), resolved by
          // pointer jumping with one ds_bpermute per round; the ops are emitted in parallel.
          const bool termC = (c & (kCodeMiss | kCodeBorder | kCodeSplit)) || (MODE == BGK_LOCAL && (c & 3) == 3);
          if (!termC) {
            if ((dk | dl) != 0) reanchor(k, l);
            const int cl = codes;
            const bool tm = (cl & (kCodeMiss | kCodeBorder | kCodeSplit)) || (MODE == BGK_LOCAL && (cl & 3) == 3);
            const u64 Tm = ballot(tm);
            const u64 TX = Tm | ballot(cl & 4);        // a run up stops here (x_trace 'M' or end)
            const u64 TY = Tm | ballot(cl & 8);
            auto emit = [&](int pos, int n, int op) {  // ops pos .. pos+n-1 of this walk
              for (int q = 0; q < n; ++q) put_op(ntw + pos + q, op);
            };
            // the run the walk is in at the anchor (state X / Y), resolved in scalar
            int s0 = 0;
            if (state != 0) {
              const u64 m = state == 1 ? (TX & 0x0101010101010101ull) : (TY & 0xFFull);
              int run = 8, endRun = 1;
              if (m) {
                s0 = (int)__builtin_ctzll(m);
                run = state == 1 ? (s0 >> 3) : (s0 & 7);
                endRun = (int)((Tm >> s0) & 1);
              }
              if (lane == 0) emit(ncore, run, state);
              ncore += run;
              if (state == 1) k -= run; else l -= run;
              if (endRun) continue;                    // an end cell (scalar path) or the edge
              state = 0;
            }
            // per-lane M node: hop target P (self = chain end), hop weight w and op, and for
            // chain ends the trailing run E, the final cell (fk << 4 | fl) and state
            const int dkl = lane >> 3, dll = lane & 7, mt = cl & 3;
            int P = lane, w = 0, op = 0, E = 0, fin = (dkl << 4) | dll, fst = 0;
            if (!tm) {
              if (mt == 0) {
                if (dkl < 7 && dll < 7) { P = lane + 9; w = 1; }
                else { E = 1; fin = ((dkl + 1) << 4) | (dll + 1); }
              } else {
                const bool up = mt == 1;
                op = up ? 1 : 2;
                const u64 lineMask = up ? (0x0101010101010101ull << dll) : (0xFFull << (dkl * 8));
                const u64 m = (up ? TX : TY) & lineMask & ~((2ull << lane) - 1);   // strictly beyond
                if (!m) {
                  E = up ? 8 - dkl : 8 - dll;
                  fin = up ? ((8 << 4) | dll) : ((dkl << 4) | 8);
                  fst = up ? 1 : 2;
                } else {
                  const int bpos = (int)__builtin_ctzll(m);
                  const int dist = up ? (bpos >> 3) - dkl : (bpos & 7) - dll;
                  if ((Tm >> bpos) & 1) { E = dist; fin = ((bpos >> 3) << 4) | (bpos & 7); fst = up ? 1 : 2; }
                  else { P = bpos; w = dist; }
                }
              }
            }
            // pointer jumping: p <- p(p), d <- d + d(p), h <- h + h(p)  (chains <= 14 hops)
            int PK = P | (w << 8) | ((P != lane ? 1 : 0) << 16);
            // interleaved with lane m finding the m-th node from s0 (see the linear jumper)
            int x = s0;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
              const int y = __builtin_amdgcn_ds_bpermute(x * 4, PK & 255);
              const int qv = __builtin_amdgcn_ds_bpermute((PK & 255) * 4, PK);
              x = ((lane >> rr) & 1) ? y : x;
              PK = (qv & 255) | ((PK & ~255) + (qv & ~255));
            }
            const int Dall = (PK >> 8) & 255;                      // weight to the chain's end
            const int Pn = rdlane(PK & 255, s0), Dn = rdlane(Dall, s0), Hn = rdlane(PK >> 16, s0);
            // lane m (the m-th node from s0) writes its hop's ops
            const int wx = __builtin_amdgcn_ds_bpermute(x * 4, w | (op << 8));
            const int dx = __builtin_amdgcn_ds_bpermute(x * 4, Dall);
            if (lane < Hn) emit(ncore + Dn - dx, wx & 255, wx >> 8);
            const int En = rdlane(E, Pn), finN = rdlane(fin, Pn), fstN = rdlane(fst, Pn);
            if (lane == Hn) emit(ncore + Dn, En, fstN);
            ncore += Dn + En;
            k = k0 - (finN >> 4);
            l = l0 - (finN & 15);
            state = fstN;
            ++nJump;
            continue;
          }
        }
        if (c & kCodeSplit) { crossed = 1; done = 1; break; }   // entered the strip above (WALK)
        if (c & kCodeMiss) {
          const int vr = k - 1;
          reqS = vr / ROWS;
          const int bl = (l + (vr - reqS * ROWS) / R) >> 5;
          reqB0 = CK ? (bl >> 1) : (bl - NBW + 1 > 0 ? bl - NBW + 1 : 0);
          if (async) {
            // post the position and the request, then wait for a helper to publish the chunk
            const u64 tw0 = F.dbg ? __builtin_readcyclecounter() : 0;
            const int key = (reqS << 16) | reqB0;
            if (lane == 0) {
              __hip_atomic_store(&sh[34], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_store(&sh[35], l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_store(&sh[33], key, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const unsigned* me = &ckMap[ck_map_idx(reqS, reqB0)];
            // Forward progress: after kSelfPolls polls without a helper taking the request (all
            // busy prefetching), the walker claims a slot under the same lock and recomputes the
            // chunk itself.  A chunk already being filled is only waited for (its filler always
            // finishes); the bound below is a last-resort guard that no schedule reaches.
            const int selfPolls = (F.flags & BG_FIN_SELFSERVE) ? 0 : kSelfPolls;
            int it = 0, selfN = 0, why = BG_WD_CHUNK;
            bool got = false;
            const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
            for (;; ++it) {
              const unsigned e = __hip_atomic_load(me, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (e != 0xFFFFFFFFu && (int)(e >> 4) == key) {
                // served: withdraw the request, so no helper recomputes it again once it has
                // been evicted (a stale request may land on a map entry the walk is using)
                if (lane == 0) __hip_atomic_store(&sh[33], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                got = true;
                break;
              }
              if (it >= selfPolls && (it - selfPolls) % 64 == 0) {
                int zz = -1;
                if (!slot_lock(F, &sh[36], lane)) { why = BG_WD_LOCK_WALKER; break; }
                if (lane == 0) {
                  // in flight (flags first), then published meanwhile (the map second): see the
                  // helpers' candidate check
                  bool busy = false;
                  for (int z = 0; z < nSlots; ++z)
                    busy |= (__hip_atomic_load(&sh[48 + z], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0 &&
                             sh[40 + z] == key);
                  const unsigned e2 = __hip_atomic_load(me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                  busy |= e2 != 0xFFFFFFFFu && (int)(e2 >> 4) == key;
                  if (!busy) {
                    // the helpers' eviction order: an empty, stale or dead slot first (dead =
                    // right of / below the walker, never read again), then one outside the
                    // walker's 2 x 2 chunk footprint (the neighbourhood decode after the miss
                    // reads those), then any slot not being filled
                    const int vw = k > 0 ? k - 1 : 0;
                    const int sw = vw / ROWS, remw = vw - sw * ROWS, ccw = (l + remw / R) >> 6;
                    const int xA = (l + 63) >> 6;
                    for (int pass = 0; pass < 3 && zz < 0; ++pass)
                      for (int z = 0; z < nSlots && zz < 0; ++z) {
                        if (sh[48 + z]) continue;
                        const int oz = sh[40 + z];
                        const int ss = oz >> 16, cc = oz & 0xffff;
                        bool take;
                        if (pass == 0) {
                          const unsigned e = oz < 0 ? 0xFFFFFFFFu : ckMap[ck_map_idx(ss, cc)];
                          take = oz < 0 || (e & 15) != (unsigned)z || (int)(e >> 4) != oz ||
                                 ss > sw || (ss == sw && cc > ccw);
                        } else if (pass == 1) {
                          take = !((ss == sw && (cc == ccw || cc == ccw - 1)) ||
                                   (ss == sw - 1 && (cc == xA || cc == xA - 1)));
                        } else {
                          take = true;
                        }
                        if (take) zz = z;
                      }
                    if (zz >= 0) {
                      const int oz = sh[40 + zz];
                      if (oz >= 0) {
                        unsigned& oe = ckMap[ck_map_idx(oz >> 16, oz & 0xffff)];
                        if ((oe & 15) == (unsigned)zz && (int)(oe >> 4) == oz)
                          __hip_atomic_store(&oe, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                      }
                      sh[40 + zz] = key;
                      sh[48 + zz] = 1;
                    }
                  }
                  __hip_atomic_store(&sh[36], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                zz = uni(__shfl(zz, 0, 64));
#if BG_FIN_DEBUG
                if (zz >= 0 && (reqS < 0 || reqS >= P.nstrips || reqB0 < 0 || reqB0 >= P.nc || zz >= nSlots) && lane == 0)
                  printf("BGDBG pair %d: self-serve key (%d, %d) slot %d of %d x %d / %d\n", P.index, reqS, reqB0, zz,
                         P.nstrips, P.nc, nSlots);
#endif
                if (zz >= 0) {
                  // a chunk the walker recomputed and published is guarded from every eviction
                  // until the walker reads it: needing it again and again is a defect, not a wait
                  if (++selfN > 16) {
                    if (lane == 0) __hip_atomic_store(&sh[48 + zz], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    why = BG_WD_THRASH;
                    break;
                  }
                  recompute_chunk<R>(F, P, reqS, reqB0, win + (size_t)zz * kSlotDw, ckArea, lane);
                  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                  if (lane == 0) {
                    __hip_atomic_store(&ckMap[ck_map_idx(reqS, reqB0)],
                                       ((unsigned)reqS << 20) | ((unsigned)reqB0 << 4) | (unsigned)zz,
                                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_store(&sh[48 + zz], 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                  }
                  ++nSelf;
                  continue;                                // re-check the map
                }
              }
              if ((it & 63) == 63 && wait_expired(F, tw)) break;
              __builtin_amdgcn_s_sleep(1);
            }
            if (!got) {
              // 5: BG_INTERNAL (no schedule reaches it), with the wait's record in bg_wait_diag
              // the record goes out after the walk (bg_wait_diag), where few registers are live
              if (lane == 0) { sh[59] = why; sh[60] = key; sh[61] = selfN; sh[62] = k; sh[63] = l; }
              status = 5;
              done = 1;
              break;
            }
            k0 = -1000000;                                 // decode the neighbourhood again
            ++nMiss;
            if (F.dbg) tMiss += __builtin_readcyclecounter() - tw0;
            continue;
          }
          break;
        }
        const bool interior = !(c & kCodeBorder);
        bool ok;                                       // trace_valid (:117, :181, :256, :317, :409)
        if constexpr (MODE == BGK_GLOBAL) ok = (k | l) != 0;
        else if constexpr (MODE == BGK_LOCAL) ok = interior && (c & 3) != 3;
        else if constexpr (MODE == BGK_SEMIGLOBAL) ok = interior;
        else ok = l != 0;
        if (!ok) { done = 1; break; }
        const u64 lut = state == 0 ? kLutM : (state == 1 ? kLutX : kLutY);
        const int e = (int)(lut >> (4 * (c & 15))) & 15;
        const int mv = e >> 2;
        if ((mv == 2 && k == 0) || (mv == 3 && l == 0)) { status = 4; done = 1; break; }  // index underflow panic
#if BG_FIN_DEBUG
        if (lane == 0 && mv && ntw + ncore + 1 > capw)
          printf("BGDBG pair %d: scalar walker writes op %d of cap %d at (%d, %d)\n", P.index, ntw + ncore + 1, capw, k, l);
#endif
        k -= (0x6 >> mv) & 1;
        l -= (0xA >> mv) & 1;
        state = e & 3;
        if (mv) {
          if (lane == 0) put_op(ntw + ncore, mv - 1);
          ++ncore;
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (lane == 0) { sh[4] = reqS; sh[5] = reqB0; sh[6] = done; sh[11] = crossed; }
      if (ballot(wild) && lane == 0) sh[9] = 5;                // BG_INTERNAL: see put_op
      if (async && lane == 0) __hip_atomic_store(&sh[32], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    done = sh[6];
    if (done) break;
    const u64 tm0 = __builtin_readcyclecounter();
    ++nMiss;
    reqS = uni(sh[4]);
    reqB0 = uni(sh[5]);
    // the chunk (window) just loaded for this request always holds the requested cell, so a
    // repeated request is a defect: end the walk with BG_INTERNAL rather than loop forever
    sameReq = (reqS == lastReqS && reqB0 == lastReqB) ? sameReq + 1 : 0;
    lastReqS = reqS;
    lastReqB = reqB0;
    if (sameReq > 2) {
      if (tid == 0) sh[9] = 5;
      break;
    }
    if constexpr (CK) {
      // recompute the requested chunk and up to three chunks to its left (the walk heads up and
      // left), one per wave, into the oldest slots
      int list[4], nl = 0;
      for (int d = 0; d < (grpMode ? GRP : NWV) && d < 4; ++d) {
        const int cc = reqB0 - d;
        if (cc < 0) break;
        bool res = false;
#pragma unroll
        for (int z = 0; z < kCkSlots; ++z) res |= (ckS[z] == reqS && ckC[z] == cc);
        if (!res || d == 0) list[nl++] = cc;
      }
      const int myz = (ckNext + wid) % nSlots;
      if (ACK && reqS != profS) {                    // the recomputing waves share the profile
        build_prof_aff<R>(F, P, reqS, profShared, tid, NT);
        profS = reqS;
        __syncthreads();
      }
      if (wid < nl) {
        if constexpr (ACK) {
          uint32_t* slotp = win + (size_t)myz * kSlotDw;
          int* areap = ckArea + wid * ckAreaInts;
          if (MODE == BGK_GLOBAL && (F.flags & BG_FIN_LCS))
            recompute_chunk_aff<R, false, false, true>(F, P, reqS, list[wid], slotp, areap, profShared, lane,
                                                       0, 0, 0, nullptr);
          else
            recompute_chunk_aff<R, MODE == BGK_LOCAL, false>(F, P, reqS, list[wid], slotp, areap, profShared,
                                                             lane, 0, 0, 0, nullptr);
        }
        else if (!grpMode)
          recompute_chunk<R>(F, P, reqS, list[wid], win + (size_t)myz * kSlotDw,
                             ckArea + wid * ckAreaInts, lane);
      }
      if (grpMode && wid == 0) {
        // one wave, up to GRP jobs: the requested chunk and those to its left
        int chs[4], zq[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          chs[x] = x < nl ? list[x] : list[0];
          zq[x] = (ckNext + (x < nl ? x : 0)) % nSlots;
        }
        if constexpr (grpMode) recompute_grp<R, GRP>(F, P, nl, chs, zq, win, ckArea, lane);
      }
      for (int x = 0; x < nl; ++x) {
        const int z = (ckNext + x) % nSlots;
        int oldS = -1, oldC = -1;
#pragma unroll
        for (int zz = 0; zz < kCkSlots; ++zz)
          if (zz == z) { oldS = ckS[zz]; oldC = ckC[zz]; ckS[zz] = reqS; ckC[zz] = list[x]; }
        if (tid == 0) {
          if (oldS >= 0) {
            unsigned& oe = ckMap[ck_map_idx(oldS, oldC)];
            if ((oe & 15) == (unsigned)z) oe = 0xFFFFFFFFu;
          }
          ckMap[ck_map_idx(reqS, list[x])] =
              ((unsigned)reqS << 20) | ((unsigned)list[x] << 4) | (unsigned)z;
        }
      }
      ckNext = (ckNext + nl) % nSlots;
      nRec += nl;
      k0 = -1000000;
    } else {
      const int nb = (stripBlocks - reqB0) < NBW ? (stripBlocks - reqB0) : NBW;
      const uint4* src = reinterpret_cast<const uint4*>(tr + (size_t)reqS * stripDw + (size_t)reqB0 * BLK_DW);
      uint4* dst = reinterpret_cast<uint4*>(win);
      const int n4 = nb * BLK_DW / 4;
      constexpr int UNR = 16;                            // all of a thread's loads in flight at once
      for (int x0 = 0; x0 < n4; x0 += UNR * NT) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int x = x0 + u * NT + tid;
          if (x < n4) v[u] = src[x];
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int x = x0 + u * NT + tid;
          if (x < n4) dst[x] = v[u];
        }
      }
      curS = reqS; curB0 = reqB0; curNb = nb;
      k0 = -1000000;                                   // decode the neighbourhood again
    }
    __syncthreads();
    tMiss += __builtin_readcyclecounter() - tm0;
  }
  if (async && tid == 0 && sh[59])
    wait_diag(F, sh[59], P.index, sh[59] == BG_WD_LOCK_HELPER ? -1 : 0, sh[60], ckMap, sh, nSlots, sh[62], sh[63], sh[61]);
  if (F.dbg && tid == 0) {
    u64* d = F.dbg + (size_t)P.index * 16;
    d[0] = __builtin_readcyclecounter() - tWalk0;
    d[1] = tJump + tDec; d[2] = nJump + nDec; d[3] = tMiss; d[4] = nMiss; d[5] = (u64)ncore;
    d[6] = async ? (u64)sh[37] + nSelf : nRec;
    d[7] = tWalk0 - tK0;                               // end cell, tail gaps, set-up
    d[9] = tK1 - tK0;                                  // chunk map cleared
    d[10] = tK2 - tK0;                                 // end cell known
  }

  // ---------------- semiglobal prefix gaps (:416-428); every wave knows k, l through sh
  if (wid == 0 && lane == 0) { sh[7] = k; sh[8] = l; sh[10] = ncore; if (sh[9] != 5) sh[9] = status; }
  __syncthreads();
  if (ph == BG_PH_TAIL && tid == 0) spl[SL.head + 10] = sh[10] - ffOps;   // moves the tail walked
  if (ph == BG_PH_WALK) {
    // the strip's record for the tail
    if (tid == 0) {
      BgStripHdr hr;
      hr.sk = kStart; hr.sl = lStart; hr.ek = sh[7]; hr.el = sh[8]; hr.nops = sh[10];
      hr.crossed = sh[11]; hr.status = sh[9]; hr.pre = 0;
      reinterpret_cast<BgStripHdr*>(spl + SL.hdr)[wstrip] = hr;
    }
    return;
  }
  const int kstop = sh[7], lstop = sh[8];
  status = sh[9];
  ncore = sh[10];
  int npre = 0;
  if (status == 0 && mode == BGK_SEMIGLOBAL) npre = colcase ? kstop : lstop;
  const int L = ntail + ncore + npre;
  const int base = cap - L;

  // ---------------- semiglobal prefix (:416-428) and tail columns: one residue run against gaps
  // each (prefix: s1[0, kstop) or s2[0, lstop); tail: s1[ei, n1) or s2[ej, n2))
  // 16-byte stores between byte heads and tails (C4: ~10 k columns per pair, which byte stores
  // of 8 loads per round took ~20 latency-bound rounds for); the residues' 16 bytes come from five
  // dword-aligned loads and v_alignbyte.  Loads of GB blocks go before their stores (a load after a
  // store to a buffer that may alias it waits for the store).
  auto gap_run = [&](int dst, const uint8_t* src, int n) {
    if (n <= 0) return;
    uint8_t* os = colcase ? ob + dst : ob2 + dst;      // the residues' side
    uint8_t* og = colcase ? ob2 + dst : ob + dst;      // the gaps' side
    {
      const int hg = min(n, (int)((16u - ((unsigned)(uintptr_t)og & 15u)) & 15u));
      const int bg = (n - hg) >> 4;
      if (tid < hg) og[tid] = (uint8_t)'-';
      uint4* ov = reinterpret_cast<uint4*>(og + hg);
      for (int b = tid; b < bg; b += NT) ov[b] = make_uint4(0x2d2d2d2du, 0x2d2d2d2du, 0x2d2d2d2du, 0x2d2d2d2du);
      for (int x = hg + 16 * bg + tid; x < n; x += NT) og[x] = (uint8_t)'-';
    }
    const int hs = min(n, (int)((16u - ((unsigned)(uintptr_t)os & 15u)) & 15u));
    const int bs = (n - hs) >> 4;
    const uint8_t hv = tid < hs ? src[tid] : (uint8_t)0;
    const uint8_t* s0 = src + hs;
    const unsigned sh = (unsigned)(uintptr_t)s0 & 3u;
    const uint32_t* sa = reinterpret_cast<const uint32_t*>(s0 - sh);   // reads <= 4 bytes past n
    uint4* ov = reinterpret_cast<uint4*>(os + hs);
    constexpr int GB = 4;
    for (int b0 = tid; b0 < bs; b0 += GB * NT) {
      uint32_t w[GB][5];
#pragma unroll
      for (int u = 0; u < GB; ++u)
#pragma unroll
        for (int q = 0; q < 5; ++q) w[u][q] = (b0 + u * NT < bs) ? sa[4 * (b0 + u * NT) + q] : 0u;
#pragma unroll
      for (int u = 0; u < GB; ++u)
        if (b0 + u * NT < bs)
          ov[b0 + u * NT] = make_uint4(__builtin_amdgcn_alignbyte(w[u][1], w[u][0], sh),
                                       __builtin_amdgcn_alignbyte(w[u][2], w[u][1], sh),
                                       __builtin_amdgcn_alignbyte(w[u][3], w[u][2], sh),
                                       __builtin_amdgcn_alignbyte(w[u][4], w[u][3], sh));
    }
    if (tid < hs) os[tid] = hv;
    for (int x = hs + 16 * bs + tid; x < n; x += NT) os[x] = src[x];
  };
  gap_run(base, colcase ? f.s1 : f.s2, npre);
  gap_run(cap - ntail, colcase ? f.s1 + ei : f.s2 + ej, ntail);

  // ---------------- expand the walk's op codes into both strings (parallel scan over columns);
  // a split pair's TAIL leaves this to the many-workgroup expansion (BG_FIN_DEFER_EXPAND)
  if (!(ph == BG_PH_TAIL && (F.flags & BG_FIN_DEFER_EXPAND))) {
  const int i0 = kstop, j0 = lstop;                    // first residues the core consumes
  const int cbase = base + npre;
  const int seg = (ncore + NT - 1) / NT;
  const int cend = cbase + ncore;
  const int lo = cbase + tid * seg < cend ? cbase + tid * seg : cend;
  const int hi = lo + seg < cend ? lo + seg : cend;
  int c1 = 0, c2 = 0;
  for (int x0 = lo; x0 < hi; x0 += 8) {               // 8 loads in flight per round
    int opv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) opv[u] = x0 + u < hi ? (int)ob[x0 + u] : 3;
#pragma unroll
    for (int u = 0; u < 8; ++u) { c1 += opv[u] == 0 || opv[u] == 1; c2 += opv[u] == 0 || opv[u] == 2; }
  }
  // the core's ops, 2 bits per column (the compact export's payload, bg_batch_export_compact),
  // before the expansion below overwrites them with residues
  if (F.ops) {
    uint8_t* po = F.ops + P.ops_off;
    const int ng = (ncore + 3) / 4;
    for (int g0 = tid; g0 < ng; g0 += 4 * NT) {        // 4 packed bytes per thread per round
      unsigned v[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int g = g0 + r * NT;
          if (g < ng && 4 * g + q < ncore) v[r] |= (unsigned)(ob[cbase + 4 * g + q] & 3) << (2 * q);
        }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (g0 + r * NT < ng) po[g0 + r * NT] = (uint8_t)v[r];
    }
  }
  scan[tid] = c1;
  scan[NT + tid] = c2;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {                  // inclusive Hillis-Steele scan
    const int v1 = tid >= o ? scan[tid - o] : 0;
    const int v2 = tid >= o ? scan[NT + tid - o] : 0;
    __syncthreads();
    scan[tid] += v1;
    scan[NT + tid] += v2;
    __syncthreads();
  }
  int p1 = i0 + scan[tid] - c1, p2 = j0 + scan[NT + tid] - c2;
#if BG_FIN_DEBUG
  {
    // the core's ops must consume exactly s1[kstop, kstop + ...) up to ei and s2 up to ej
    const int tot1 = scan[NT - 1], tot2 = scan[2 * NT - 1];
    if (tid == 0 && status != 5 && (i0 + tot1 != (colcase ? ei : (mode == BGK_SEMIGLOBAL ? ei : ei)) ||
                                    j0 + tot2 != ej))
      printf("BGDBG pair %d: ops consume (%d, %d) from (%d, %d), end (%d, %d), ncore %d ntail %d status %d\n",
             P.index, tot1, tot2, i0, j0, ei, ej, ncore, ntail, status);
    bool badop = false;
    for (int x = lo; x < hi; ++x) badop |= ob[x] > 2;
    if (badop) printf("BGDBG pair %d: op code > 2 in the core (tid %d)\n", P.index, tid);
  }
#endif
  // in rounds of EB columns: the ops, then the residues they consume, then the stores (the same
  // aliasing rule as the gap runs: two round trips per round instead of two per column)
  constexpr int EB = 16;
  for (int x0 = lo; x0 < hi; x0 += EB) {
    int opv[EB];
    uint8_t c1v[EB], c2v[EB];
#pragma unroll
    for (int u = 0; u < EB; ++u) opv[u] = x0 + u < hi ? (int)ob[x0 + u] : 3;
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int op = opv[u];
#if BG_FIN_DEBUG
      if (op != 3 && ((op != 2 && (p1 < 0 || p1 >= n1)) || (op != 1 && (p2 < 0 || p2 >= n2))))
        printf("BGDBG pair %d: expansion reads s1[%d] / s2[%d] of %d / %d (op %d)\n", P.index, p1, p2, n1, n2, op);
#endif
      const bool t1 = op == 0 || op == 1, t2 = op == 0 || op == 2;
      c1v[u] = t1 ? f.s1[p1] : (uint8_t)'-';
      c2v[u] = t2 ? f.s2[p2] : (uint8_t)'-';
      p1 += t1;
      p2 += t2;
    }
#pragma unroll
    for (int u = 0; u < EB; ++u)
      if (x0 + u < hi) {
        ob[x0 + u] = c1v[u];
        ob2[x0 + u] = (F.flags & BG_FIN_LCS) ? (uint8_t)opv[u] : c2v[u];   // LCS: the caller keeps op-0 columns
      }
  }
  }
  if (tid == 0) {
    BgResult res;
    res.status = status;
    res.score = score;
    res.end_i = ei;
    res.end_j = ej;
    res.out_start = (uint32_t)base;
    res.out_len = (uint32_t)L;
    res.start1 = (uint32_t)kstop;
    res.start2 = (uint32_t)lstop;
    res.npre = (uint32_t)npre;
    res.ntail = (uint32_t)ntail;
    F.results[P.index] = res;
    if (F.dbg) F.dbg[(size_t)P.index * 16 + 8] = __builtin_readcyclecounter() - tK0;   // whole kernel
  }
}

