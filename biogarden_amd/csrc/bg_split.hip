// Split traceback for few long pairs (WIDE linear checkpoint batches, C3): the exit pass, the
// per-strip resolve and the chain over the strips.  The walks themselves and
// the stitching run in bg_finish_kernel's BG_PH_WALK / BG_PH_TAIL phases.
//
// The reference walks the traceback from the end cell one move at a time (backtrack,
// src/alignment/aligner.rs:511-592; for open >= extend the X / Y states fall back to M at once,
// so the walk is a chain of m_trace moves).  Every cell of the DP has exactly one predecessor,
// so the path from a cell of strip s (rows s*64R+1 .. (s+1)*64R) enters the row above the strip
// at one column: the cell's exit.  With every bottom-row cell's exit known, the start cell's
// entry column into each strip above follows from one lookup per strip, and the strips' walks no
// longer depend on each other.
//
// Exit pass.  Work items are (pair, strip, segment of SEGC chunks).  A wave restarts the strip's
// forward recurrence at the segment's first checkpoint (the same data the checkpoint traceback
// recomputes chunks from) and sweeps the segment with the tagged step of bg_tag_kernel.hip,
// except that a value is packed as
//     (M'(i,j) - base) << 19  |  tag << 17  |  exit
// with tag 0 diagonal / 2 X form / 3 Y form as in the tagged kernel.  The predecessor choice is
// the tag's (v_max3_u32 compares value first, then tag: the reference's Y > X > R priority,
// aligner.rs:455-463), and the three candidates never tie on (value, tag), so the exit bits below
// ride along with the winner for free: the step is the tagged kernel's four VALU operations per
// cell.  `base` is wave-uniform, re-chosen at every chunk start from the chunk's inputs; if a
// chunk's values could leave the 13-bit field the pass sets the pair's overflow flag and the
// tail walks the pair sequentially (the reference semantics never depend on this pass).
// Column 0 (and the never-read cells left of it) is left out of the base: in global mode the
// border a + (i-1)b lies ~i below column 1 (interior gaps cost a, the border b per row), so deep
// strips would overflow on it.  A column-0 value below the base is clamped to the field value
// c = max(0, -(min S - 2a)), and the base keeps c + max(S - 2a) + 1 of headroom below every other
// input, so a candidate derived from a clamped value (left, or diagonal + S - 2a, never below 0)
// stays strictly below the column-1 cell's up candidate, which truly wins there too (M' never
// decreases down a column).
// Exits are columns of the row above (concrete), or, for paths that leave the segment through
// its left edge, symbolic references to the segment's first frontier (the R values and the
// top-left input of every lane at the segment start), resolved strip by strip afterwards.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_dev_util.h"
#include "bg_device.h"

using namespace bgk;

namespace {

constexpr int kEBits = BG_SPLIT_EBITS;
constexpr unsigned kEMask = (1u << kEBits) - 1;
constexpr unsigned kT1 = 1u << kEBits;       // one tag unit
constexpr unsigned kT2 = 2u << kEBits;       // X form
constexpr unsigned kT3 = 3u << kEBits;       // Y form
constexpr int kVShift = kEBits + 2;
constexpr int kVMax = (1 << (32 - kVShift)) - 1;

template <int R>
__host__ __device__ constexpr int exit_wave_ints() {
  return 4 * R * 64 + 64 + 96;               // profile [code][k][lane], top block, 192 u16 codes
}

__device__ __forceinline__ unsigned umax3(unsigned x, unsigned y, unsigned z) {
  return __builtin_elementwise_max(__builtin_elementwise_max(x, y), z);
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
// v_mov_b32_dpp wave_shl:1 — lane r receives lane r+1; lane 63 keeps `old`
__device__ __forceinline__ unsigned dpp_shl1u(unsigned old, unsigned src) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x130, 0xf, 0xf, false);
}
__device__ __forceinline__ unsigned dpp_shr1u(unsigned old, unsigned src) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x138, 0xf, 0xf, false);
}

template <int R>
struct ExitStrip {
  unsigned Y[R];      // Y form of the lane's rows at the previous column
  unsigned topPrev;   // X form of (row above the lane, j - 1)
  unsigned Xlast;     // X form of the lane's last row: handed to lane r + 1 by the DPP
  unsigned Q;         // bottom-row conveyor: lane 63's last row of the chunk's steps
};

// One chunk of the packed tagged step.  EDGE: chunk 0 (column 0 borders, aligner.rs:98-104);
// CAP: the chunk holds the walk's start cell, whose exit is captured at step `ts`.
template <int R, bool EDGE, bool CAP>
__device__ __forceinline__ void exit_chunk(ExitStrip<R>& S, int c, int lane, const int* profLane,
                                           const uint16_t* codeLane, const unsigned* bIn,
                                           const unsigned* col0, int ts, int qs, int rs,
                                           unsigned& cap) {
  const int t0 = c * 64;
  // operand pipeline: the profile entries of step u + 1 and the code of step u + 2 are in flight
  // while step u computes
  unsigned nTop = bIn[0];
  unsigned nP[R];
  {
    const int o = codeLane[0];
#pragma unroll
    for (int k = 0; k < R; ++k) nP[k] = (unsigned)profLane[o + k * 64];
  }
  int nCode = codeLane[1];
#pragma unroll
  for (int u = 0; u < 64; ++u) {
    const int t = t0 + u;
    const unsigned topIn = nTop;
    unsigned P[R];
#pragma unroll
    for (int k = 0; k < R; ++k) { P[k] = nP[k]; nP[k] = (unsigned)profLane[nCode + k * 64]; }
    nCode = codeLane[u + 2];
    if (u + 1 < 64) nTop = bIn[u + 1];
    const unsigned topX = dpp_shr1u(topIn, S.Xlast);       // X form of (row above, j)
    unsigned dIn = S.topPrev;                               // X form of (row above, j - 1)
    unsigned xo = topX;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const unsigned yo = S.Y[k];
      const unsigned d = dIn + P[k];                        // tag 0: (S - 2a) << 19 - tag of dIn
      const unsigned best = umax3(d, xo, yo);
      const unsigned yn = best | kT3;                       // Y form for column j + 1
      dIn = yo;
      xo = yn - kT1;                                        // X form for row i + 1
      S.Y[k] = yn;
    }
    S.topPrev = topX;
    S.Xlast = xo;
    if constexpr (EDGE) {
      if (c == 0 && t == lane) {                            // column 0: border, exit 0
#pragma unroll
        for (int k = 0; k < R; ++k) S.Y[k] = col0[k];
        S.Xlast = col0[R - 1] - kT1;
      }
    }
    S.Q = dpp_shl1u(S.Y[R - 1], S.Q);
    if constexpr (CAP) {
      if (t == ts) {
        unsigned v = S.Y[0];
#pragma unroll
        for (int k = 1; k < R; ++k) v = (k == qs) ? S.Y[k] : v;
        cap = (unsigned)__builtin_amdgcn_readlane((int)v, rs);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

}  // namespace

// One exit-pass item: a wave runs (pair, strip s >= 1, segment g).  Outputs (split area):
//   ebot[s][j]        raw exit of the strip's bottom row at column j
//   front[s][g][x]    raw exits of the segment's last frontier, x = k * 64 + lane (k < R: the
//                     lane's rows; k = R: its top-left input), for segment g + 1's symbols
//   head[4], head[5]  raw exit of the walk's start cell and its segment (start strip, after the DP)
//   head[6]           set when a chunk's values could leave the packed field (head[11] = epoch:
//                     the same, from the concurrent pass)
// CONC: the pass beside the DP.  Its inputs are the DP's {value, epoch} granules (the segment's
// start checkpoint, the output row of the strip above), read agent-coherent and waited for until
// every tag is this execute's epoch; the start strip and cell are not known yet, so every strip's
// bottom row is kept and nothing is captured.  The item's done tag then lets the pass after the
// DP skip it.
template <int R, bool CONC>
__device__ void exit_item(const BgSplitArgs& A, int item, int lane, int* wl) {
  constexpr int ROWS = 64 * R;
  constexpr int F = (R + 1) * 64;
  constexpr unsigned kSym = BG_SPLIT_SYM(R);
  int p = 0;
  while (p + 1 < A.npairs && A.itemBase[p + 1] <= item) ++p;
  p = uni(p);
  const BgPair P = A.pairs[p];
  const int n1 = P.n1, n2 = P.n2, NC = P.nc, NS = P.nstrips;
  const BgSplitLayout L = bg_split_layout(n1, n2, NS, NC, R, A.segc);
  const int rel = item - A.itemBase[p];
  const int s = 1 + rel / L.G, g = rel % L.G;
  int32_t* ar = A.split + P.split_off;
  const int sStar = CONC ? NS - 1 : uni(ar[L.head + 7]);
  if (s > sStar || s >= NS) return;
  const int c0 = g * A.segc;
  const int c1 = min(NC, c0 + A.segc);
  const int a = A.open, b = A.ext, mode = A.mode;
  // the start cell, when it lies in this strip (lane rs, row qs, step ts): after the DP only
  const int ei = CONC ? 0 : ar[L.head + 0], ej = CONC ? 0 : ar[L.head + 1];
  const bool capStrip = !CONC && (s == sStar) && ei >= 1 && ej >= 1;
  const int vs = ei - 1 - s * ROWS;
  const int rs = capStrip ? vs / R : 0, qs = capStrip ? vs % R : 0, ts = capStrip ? ej + rs : -1;
  const bool capItem = capStrip && ts >= c0 * 64 && ts < c1 * 64;
  uint32_t* done = reinterpret_cast<uint32_t*>(ar + L.done);
  if (!CONC && !capItem && done[(size_t)(s - 1) * L.G + g] == A.epoch) return;   // done beside the DP
  // the start strip's items after the capture item feed nothing: the strip's bottom row is not
  // wanted and the chain and resolve stop at the capture segment (head[5])
  if (capStrip && c0 * 64 > ts) return;

  int* prof = wl;                                       // [code][k][lane]
  unsigned* bIn = reinterpret_cast<unsigned*>(wl + 4 * R * 64);
  uint16_t* stage = reinterpret_cast<uint16_t*>(wl + 4 * R * 64 + 64);
  const int rowbase = s * ROWS + lane * R;
  const uint8_t* cr1 = A.codes1 + P.off1;
  const uint8_t* cr2 = A.codes2 + P.off2;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = rowbase + k + 1;
    const int q = (i <= n1) ? cr1[i - 1] : 0;
    const int pk = A.profile[192 + (q >> 3)];
    const unsigned tadj = (k == 0 ? 2u : 3u) << kEBits;  // the tag of the diagonal's form
#pragma unroll
    for (int cd = 0; cd < 4; ++cd) {
      const int v = __builtin_amdgcn_sbfe(pk, 8 * cd, 8);   // S(q, cd) - 2a
      prof[(cd * R + k) * 64 + lane] = (int)(((unsigned)v << kVShift) - tadj);
    }
  }
  const int* profLane = prof + lane;
  const uint16_t* codeLane = stage + 63 - lane;
  const size_t topOff = P.bnd_off + (size_t)(s - 1) * NC * 64;        // M'(s*ROWS, j)
  const int32_t* topRow = A.bndM + topOff;
  const unsigned long long* topGran = A.gran + topOff;
  const int tclamp = n2 < NC * 64 - 1 ? n2 : NC * 64 - 1;
  // CONC: a wait that outlasts A.waitTicks (or finds the pass abandoned by another wave)
  // abandons the item and the pass; the pass after the DP then does what is left
  bool dead = false;
  unsigned long long t0 = 0;
  int np = 0;
  auto waited_out = [&](int which, unsigned long long tagv) {
    if ((++np & 63) == 0) {
      if (__hip_atomic_load(A.diag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return true;
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (t0 == 0) t0 = now;
      if (now - t0 > (unsigned long long)A.waitTicks) {
        if (lane == 0) {
          A.diag[1] = (uint32_t)item;
          A.diag[2] = (uint32_t)which;
          A.diag[3] = (uint32_t)(tagv >> 32);
          A.diag[4] = A.epoch;
          __threadfence();
          __hip_atomic_store(A.diag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return true;
      }
    }
    return false;
  };
  // polls back off (~0.2 us, then ~1.7 us, then ~7 us apart): thousands of waiting waves' loads otherwise
  // compete with the DP's own hand-offs in L2
  auto backoff = [&]() {
    if (np < 16) {
      __builtin_amdgcn_s_sleep(8);
    } else if (np < 64) {
      __builtin_amdgcn_s_sleep(63);
    } else {                                             // a long wait: ~7 us between polls
      __builtin_amdgcn_s_sleep(127);
      __builtin_amdgcn_s_sleep(127);
    }
  };
  // the top block of chunk c (columns c*64 + lane, clamped to n2)
  auto top_abs = [&](int c) {
    const int j = min(c * 64 + lane, tclamp);
    if constexpr (!CONC) {
      return topRow[j];
    } else {
      unsigned long long v = __hip_atomic_load(topGran + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t0 = 0;
      np = 0;
      while (!__all((uint32_t)(v >> 32) == A.epoch)) {
        if (waited_out(1, v)) { dead = true; break; }
        backoff();
        v = __hip_atomic_load(topGran + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return (int)(uint32_t)v;
    }
  };

  // initial state: the segment's first checkpoint (absolute M'), or the strip start
  int Yabs[R], tpAbs;
  unsigned Ye[R], tpE;
  if (c0 == 0) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = rowbase + k + 1;
      Yabs[k] = wadd(col0_M(mode, i, a, b), -wmul(a, i));
      Ye[k] = 0;
    }
    tpAbs = Yabs[0];                                     // never read by a valid cell
    tpE = 0;
  } else {
    if constexpr (!CONC) {
      const int32_t* ck = A.ckpt + P.trace_off / 4 + ((size_t)(s * NC + c0) * (R + 1)) * 64 + lane;
#pragma unroll
      for (int k = 0; k < R; ++k) Yabs[k] = ck[k * 64];
      tpAbs = ck[R * 64];
    } else {
      const unsigned long long* cg =
          reinterpret_cast<const unsigned long long*>(ar + L.ckg) + (((size_t)s * L.G + g) * (R + 1)) * 64 + lane;
      unsigned long long v[R + 1];
      bool ok;
      t0 = 0;
      np = 0;
      do {
        // the checkpoint's last granule (k = R, stored last by the DP's wave) first, then all
        unsigned long long last = __hip_atomic_load(cg + R * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (!__all((uint32_t)(last >> 32) == A.epoch)) {
          if (waited_out(2, last)) return;
          backoff();
          last = __hip_atomic_load(cg + R * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k <= R; ++k) v[k] = __hip_atomic_load(cg + k * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool mine = true;
#pragma unroll
        for (int k = 0; k <= R; ++k) mine = mine && (uint32_t)(v[k] >> 32) == A.epoch;
        ok = __all(mine);
        if (!ok) {
          if (waited_out(2, v[0])) return;
          backoff();
        }
      } while (!ok);
#pragma unroll
      for (int k = 0; k < R; ++k) Yabs[k] = (int)(uint32_t)v[k];
      tpAbs = (int)(uint32_t)v[R];
    }
#pragma unroll
    for (int k = 0; k < R; ++k) Ye[k] = kSym + (unsigned)(k * 64 + lane);
    tpE = lane == 0 ? (unsigned)(c0 * 64 - 1) : kSym + (unsigned)(R * 64 + lane);
  }
  int* overflow = ar + L.head + (CONC ? 11 : 6);
  const int ovVal = CONC ? (int)A.epoch : 1;
  int mt = top_abs(c0);
  if (dead) return;
  ExitStrip<R> S;
  int base = 0;
  // field value of an absolute M' (clampv for a clamped column-0 value)
  auto fld = [&](int x) { return (unsigned)max(x - base, A.clampv) << kVShift; };
  {
    // the lanes' frontier cells sit at column c0 * 64 - 1 - lane, the top block at c0 * 64 + lane
    const bool inF = c0 * 64 - 1 - lane >= 1, inT = c0 * 64 + lane >= 1;
    int lo = inT ? mt : 0x7fffffff, hi = inT ? mt : -0x7fffffff - 1;
    if (inF) {
      lo = min(lo, tpAbs); hi = max(hi, tpAbs);
#pragma unroll
      for (int k = 0; k < R; ++k) { lo = min(lo, Yabs[k]); hi = max(hi, Yabs[k]); }
    }
    lo = uni(wave_min(lo));
    hi = uni(wave_max(hi));
    base = lo - A.margin;
    if ((long)hi - base + A.grow > kVMax) { if (lane == 0) *overflow = ovVal; return; }
#pragma unroll
    for (int k = 0; k < R; ++k) S.Y[k] = fld(Yabs[k]) | kT3 | Ye[k];
    S.topPrev = fld(tpAbs) | kT2 | tpE;
    S.Xlast = S.Y[R - 1] - kT1;
    S.Q = 0;
  }
  unsigned col0[R];
  unsigned cap = 0xFFFFFFFFu;
  int32_t* ebot = ar + L.ebot + (size_t)s * (n2 + 1);
  const bool wantBot = s < sStar;
  for (int c = c0; c < c1; ++c) {
    if (c > c0) {
      // re-base on this chunk's inputs: the lanes' values, their top-left inputs, the top block
      // (column 0 left out: only chunk 1's lane 63 holds it)
      const bool inF = c * 64 - 1 - lane >= 1;
      int lo = mt - base, hi = mt - base;
      if (inF) {
        lo = min(lo, (int)(S.topPrev >> kVShift)); hi = max(hi, (int)(S.topPrev >> kVShift));
#pragma unroll
        for (int k = 0; k < R; ++k) { lo = min(lo, (int)(S.Y[k] >> kVShift)); hi = max(hi, (int)(S.Y[k] >> kVShift)); }
      }
      lo = uni(wave_min(lo));
      hi = uni(wave_max(hi));
      const int d = lo - A.margin;                       // new base - old base
      if ((long)hi - d + A.grow > kVMax) { if (lane == 0) *overflow = ovVal; return; }
      auto reb = [&](unsigned v) {
        return ((unsigned)max((int)(v >> kVShift) - d, A.clampv) << kVShift) | (v & ((1u << kVShift) - 1));
      };
#pragma unroll
      for (int k = 0; k < R; ++k) S.Y[k] = reb(S.Y[k]);
      S.topPrev = reb(S.topPrev);
      S.Xlast = reb(S.Xlast);
      base += d;
    }
    bIn[lane] = fld(mt) | kT2 | (unsigned)(c * 64 + lane);
    if (c + 1 < c1) mt = top_abs(c + 1);                 // in flight while the chunk computes
    if (dead) return;
#pragma unroll
    for (int qq = 0; qq < 3; ++qq) {
      const int x = c * 64 - 64 + lane + 64 * qq;
      const int v = ((unsigned)x < (unsigned)n2) ? cr2[x] >> 3 : 0;
      stage[lane + 64 * qq] = (uint16_t)(v * R * 64);
    }
    if (c == 0) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int i = rowbase + k + 1;
        col0[k] = fld(wadd(col0_M(mode, i, a, b), -wmul(a, i))) | kT3;
      }
    }
    const bool capHere = ts >= c * 64 && ts < c * 64 + 64;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (c == 0) {
      if (capHere) exit_chunk<R, true, true>(S, c, lane, profLane, codeLane, bIn, col0, ts, qs, rs, cap);
      else exit_chunk<R, true, false>(S, c, lane, profLane, codeLane, bIn, col0, ts, qs, rs, cap);
    } else {
      if (capHere) exit_chunk<R, false, true>(S, c, lane, profLane, codeLane, bIn, col0, ts, qs, rs, cap);
      else exit_chunk<R, false, false>(S, c, lane, profLane, codeLane, bIn, col0, ts, qs, rs, cap);
    }
    if (capHere) {
      if (lane == 0) {
        ar[L.head + 4] = (int)(cap & kEMask);
        ar[L.head + 5] = g;
      }
      // the start strip's later chunks feed nothing: its bottom row is not needed (the walk
      // starts inside it) and the chain resolves the capture through the frontier before it
      if (capItem) return;
    }
    // the bottom row (lane 63's last row) of steps t0 .. t0 + 63: columns t0 - 63 + lane
    if (wantBot) {
      const int j = c * 64 - 63 + lane;
      if (j >= 0 && j <= n2) ebot[j] = (int)(S.Q & kEMask);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  // the segment's last frontier: the next segment's symbols point into it
  if (g + 1 < L.G) {
    int32_t* fr = ar + L.front + ((size_t)s * L.G + g) * F + lane;
#pragma unroll
    for (int k = 0; k < R; ++k) fr[k * 64] = (int)(S.Y[k] & kEMask);
    fr[R * 64] = (int)(S.topPrev & kEMask);
  }
  if constexpr (CONC) {
    __threadfence();
    if (lane == 0) done[(size_t)(s - 1) * L.G + g] = A.epoch;
  }
}

// The pass after the DP: one wave per item (4 per workgroup).
template <int R>
__global__ __launch_bounds__(256) void bg_exit_kernel(BgSplitArgs A) {
  extern __shared__ __attribute__((aligned(16))) int esm[];
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  const int item = uni((int)blockIdx.x * 4 + w);
  if (item >= A.nitems) return;
  exit_item<R, false>(A, item, lane, esm + w * exit_wave_ints<R>());
}

// The pass beside the DP: persistent workgroups (more than half a CU's LDS each, so none shares a
// CU with a WIDE DP workgroup), every wave taking items in readiness order.  A worker waits for the
// DP's data only once every DP workgroup is resident (else it leaves the items to the pass after
// the DP): it can then never hold a CU the DP still needs.
template <int R>
__global__ __launch_bounds__(R >= 8 ? 512 : 1024) void bg_exit_conc_kernel(BgSplitArgs A) {
  extern __shared__ __attribute__((aligned(16))) int esm[];
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  int polls = 0;
  while (__hip_atomic_load(A.resident, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)A.dpWgs) {
    if (++polls > 4000) {                                // ~2 ms: the DP has not started
      if (threadIdx.x == 0) A.diag[5] = 1u;
      return;
    }
    __builtin_amdgcn_s_sleep(16);
  }
  int* wl = esm + w * exit_wave_ints<R>();
  for (;;) {
    int idx = 0;
    if (lane == 0) idx = (int)__hip_atomic_fetch_add(A.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    idx = uni(__shfl(idx, 0, 64));
    if (idx >= A.nitems) return;
    exit_item<R, true>(A, A.order[idx], lane, wl);
    if (__hip_atomic_load(A.diag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;   // abandoned
  }
}

// End-cell keys of the split pairs (few long pairs: one traceback workgroup scanning a 100 k row
// and column took 0.2 ms): kEndKeyBlocks workgroups per pair fold strided slices of row n1 (the
// last strip's boundary row, M = M' + a(n1 + j)) and column n2 (M(i, n2)) into the two u64 maxima
// bg_finish_kernel's HEAD phase then reads (i, j >= 1; it adds the border cells itself).
constexpr int kEndKeyBlocks = 64;
__global__ __launch_bounds__(256) void bg_endkey_kernel(BgSplitArgs A) {
  const int p = (int)blockIdx.x / kEndKeyBlocks, part = (int)blockIdx.x % kEndKeyBlocks;
  const BgPair P = A.pairs[p];
  const int n1 = P.n1, n2 = P.n2;
  if (P.nstrips == 0 || n1 <= 0 || n2 <= 0) return;
  const int a = A.open;
  const int stride = kEndKeyBlocks * 256;
  const int t = part * 256 + (int)threadIdx.x;
  const int32_t* row = A.bndM + P.bnd_off + (size_t)(P.nstrips - 1) * P.nc * 64;
  const int32_t* col = A.aux + P.aux_off;
  u64 kr = 0, kc = 0;
#pragma unroll 8
  for (int j = 1 + t; j <= n2; j += stride) {
    const u64 key = ((u64)key_bias(wadd(row[j], wmul(a, n1 + j))) << 32) | (unsigned)j;
    kr = key > kr ? key : kr;
  }
#pragma unroll 8
  for (int i = 1 + t; i <= n1; i += stride) {
    const u64 key = ((u64)key_bias(col[i]) << 32) | (0xFFFFFFFFu - (unsigned)i);
    kc = key > kc ? key : kc;
  }
  kr = wave_umax64(kr);
  kc = wave_umax64(kc);
  if ((threadIdx.x & 63) == 0) {
    if (kc) __hip_atomic_fetch_max(A.endKeys + 2 * (size_t)p, kc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kr) __hip_atomic_fetch_max(A.endKeys + 2 * (size_t)p + 1, kr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
extern "C" void* bg_endkey_kernel_ptr(void) { return (void*)&bg_endkey_kernel; }
extern "C" int bg_endkey_blocks(void) { return kEndKeyBlocks; }

// Deferred expansion of a split pair's core (TAIL ran with BG_FIN_DEFER_EXPAND and wrote the
// result record; the core's ops sit in out1 at out_start + npre, one byte per column): block b of
// a pair covers columns [b * kXCols, (b + 1) * kXCols) of the core, 16 per thread.  The count
// kernel records how many of its ops consume s1 / s2; the expansion kernel adds the counts of the
// blocks before it, scans its threads' counts, packs the ops (2 bits per column, the compact
// export's payload) and writes both strings.  One 256-thread workgroup did this for 124 k columns
// in 0.5 ms, one HBM round trip per batch of columns.
constexpr int kXPer = 16, kXCols = 256 * kXPer;
__device__ __forceinline__ void x_load16(const uint8_t* src, int n, int (&op)[kXPer]) {
#pragma unroll
  for (int u = 0; u < kXPer; ++u) op[u] = u < n ? (int)src[u] : 3;
}
__global__ __launch_bounds__(256) void bg_expand_count_kernel(BgFinishArgs F, BgSplitArgs A) {
  const int p = (int)blockIdx.x / A.xblocks, b = (int)blockIdx.x % A.xblocks;
  const BgPair& P = F.pairs[p];
  const BgResult r = F.results[P.index];
  const int ncore = (int)r.out_len - (int)r.npre - (int)r.ntail;
  const int c0 = b * kXCols + (int)threadIdx.x * kXPer;
  int op[kXPer];
  x_load16(F.out1 + P.out_off + r.out_start + r.npre + c0, ncore - c0, op);
  int n1 = 0, n2 = 0;
#pragma unroll
  for (int u = 0; u < kXPer; ++u) { n1 += op[u] == 0 || op[u] == 1; n2 += op[u] == 0 || op[u] == 2; }
  __shared__ int s1[4], s2[4];
  for (int o = 32; o >= 1; o >>= 1) { n1 += __shfl_xor(n1, o, 64); n2 += __shfl_xor(n2, o, 64); }
  if ((threadIdx.x & 63) == 0) { s1[threadIdx.x >> 6] = n1; s2[threadIdx.x >> 6] = n2; }
  __syncthreads();
  if (threadIdx.x == 0)
    A.xcount[(size_t)p * A.xblocks + b] = make_int2(s1[0] + s1[1] + s1[2] + s1[3], s2[0] + s2[1] + s2[2] + s2[3]);
}
__global__ __launch_bounds__(256) void bg_expand_kernel(BgFinishArgs F, BgSplitArgs A) {
  const int p = (int)blockIdx.x / A.xblocks, b = (int)blockIdx.x % A.xblocks;
  const BgPair& P = F.pairs[p];
  const BgResult r = F.results[P.index];
  const int ncore = (int)r.out_len - (int)r.npre - (int)r.ntail;
  if (b * kXCols >= ncore) return;                     // block-uniform
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // residues consumed before this block: the earlier blocks' counts
  int b1 = 0, b2 = 0;
  for (int q = lane; q < b; q += 64) { const int2 c = A.xcount[(size_t)p * A.xblocks + q]; b1 += c.x; b2 += c.y; }
  for (int o = 32; o >= 1; o >>= 1) { b1 += __shfl_xor(b1, o, 64); b2 += __shfl_xor(b2, o, 64); }
  const int c0 = b * kXCols + tid * kXPer;
  uint8_t* ob = F.out1 + P.out_off + r.out_start + r.npre;
  uint8_t* ob2 = F.out2 + P.out_off + r.out_start + r.npre;
  int op[kXPer];
  x_load16(ob + c0, ncore - c0, op);
  int n1 = 0, n2 = 0;
#pragma unroll
  for (int u = 0; u < kXPer; ++u) { n1 += op[u] == 0 || op[u] == 1; n2 += op[u] == 0 || op[u] == 2; }
  // exclusive scan of the threads' counts: within the wave, then over the 4 waves
  int i1 = n1, i2 = n2;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t1 = __shfl_up(i1, o, 64), t2 = __shfl_up(i2, o, 64);
    if (lane >= o) { i1 += t1; i2 += t2; }
  }
  __shared__ int w1[4], w2[4];
  if (lane == 63) { w1[w] = i1; w2[w] = i2; }
  __syncthreads();
  int q1 = 0, q2 = 0;
  for (int x = 0; x < w; ++x) { q1 += w1[x]; q2 += w2[x]; }
  int p1 = (int)r.start1 + b1 + q1 + i1 - n1, p2 = (int)r.start2 + b2 + q2 + i2 - n2;
  // the packed ops (4 columns per byte; c0 is a multiple of 16)
  if (F.ops) {
    uint8_t* po = F.ops + P.ops_off + c0 / 4;
#pragma unroll
    for (int g = 0; g < kXPer / 4; ++g) {
      if (c0 + 4 * g >= ncore) break;
      unsigned v = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) v |= (unsigned)(op[4 * g + q] == 3 ? 0 : (op[4 * g + q] & 3)) << (2 * q);
      po[g] = (uint8_t)v;
    }
  }
  const uint8_t* s1p = F.seq1 + P.off1;
  const uint8_t* s2p = F.seq2 + P.off2;
  uint8_t a1[kXPer], a2[kXPer];
#pragma unroll
  for (int u = 0; u < kXPer; ++u) {
    const bool t1 = op[u] == 0 || op[u] == 1, t2 = op[u] == 0 || op[u] == 2;
    a1[u] = t1 ? s1p[p1] : (uint8_t)'-';
    a2[u] = t2 ? s2p[p2] : (uint8_t)'-';
    p1 += t1;
    p2 += t2;
  }
#pragma unroll
  for (int u = 0; u < kXPer; ++u)
    if (c0 + u < ncore) { ob[c0 + u] = a1[u]; ob2[c0 + u] = a2[u]; }
}
extern "C" void* bg_expand_kernel_ptr(int which) {
  return which == 0 ? (void*)&bg_expand_count_kernel : (void*)&bg_expand_kernel;
}
extern "C" int bg_expand_cols_per_block(void) { return kXCols; }

// One workgroup per (pair, strip s in [1, start strip]): resolves the strip's frontiers segment
// by segment (segment g's symbols refer to segment g - 1's last frontier).  The bottom row's
// symbolic exits are resolved by the chain, for the one column per strip it reads (resolving
// all n2 + 1 of every strip here took 0.2 ms for C3).
template <int R>
__global__ __launch_bounds__(256) void bg_exit_resolve_kernel(BgSplitArgs A) {
  constexpr int F = (R + 1) * 64;
  constexpr int kSym = BG_SPLIT_SYM(R);
  __shared__ int fa[F], fb[F];
  int p = 0;
  const int item = blockIdx.x;
  while (p + 1 < A.npairs && A.stripBase[p + 1] <= item) ++p;
  const BgPair P = A.pairs[p];
  const int n1 = P.n1, n2 = P.n2, NC = P.nc, NS = P.nstrips;
  const BgSplitLayout L = bg_split_layout(n1, n2, NS, NC, R, A.segc);
  const int s = 1 + (item - A.stripBase[p]);
  int32_t* ar = A.split + P.split_off;
  const int sStar = ar[L.head + 7];
  if (s > sStar || s >= NS || ar[L.head + 6] || (uint32_t)ar[L.head + 11] == A.epoch) return;
  const int tid = threadIdx.x;
  const int32_t* fr = ar + L.front + (size_t)s * L.G * F;
  int32_t* fs = ar + L.fres + (size_t)s * L.G * F;
  // the start strip: the chain reads the resolved frontier of the segment before the capture
  // segment head[5] only, and the exit pass stopped at the capture item (later segments' raw
  // frontiers are stale) — resolve up to that segment
  int GL = L.G;
  if (s == sStar) {
    const int cgs = ar[L.head + 5];
    if (cgs >= 0 && cgs < L.G) GL = cgs + 1;   // (HEAD sets it to 0 before the pass: nothing to read)
  }
  // The segments form a chain (segment g's symbols point into g - 1's resolved frontier), walked
  // by wave 0 alone: a wave's LDS operations complete in order, so a link costs its lookups, not
  // a workgroup barrier.  The raw frontiers do not depend on the chain: each lane keeps the raw
  // values of the next D segments in flight, so a link is not an HBM round trip either.
  if (tid < 64) {
    int* prev = fa;
    int* cur = fb;
    constexpr int D = 8, QW = (F + 63) / 64;
    for (int x = tid; x < F; x += 64) { prev[x] = fr[x]; fs[x] = fr[x]; }
    int raw[D][QW];
    auto fetch = [&](int g, int (&r)[QW]) {
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int x = tid + 64 * q;
        r[q] = (g + 1 < GL && x < F) ? fr[(size_t)g * F + x] : 0;
      }
    };
#pragma unroll
    for (int d = 0; d < D; ++d) fetch(1 + d, raw[d]);
    for (int g0 = 1; g0 + 1 < GL; g0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int g = g0 + d;
        if (g + 1 >= GL) break;                         // wave-uniform
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          const int x = tid + 64 * q;
          if (x < F) {
            const int rv = raw[d][q];
            const int v = rv >= kSym ? prev[rv - kSym] : rv;
            cur[x] = v;
            fs[(size_t)g * F + x] = v;
          }
        }
        fetch(g + D, raw[d]);                            // this slot's next segment
        int* t = prev; prev = cur; cur = t;
      }
    }
  }
}

// One wave per pair: the start cell's exit, then one lookup per strip up to the first strip
// whose walk stops in it; writes every strip's start column (-1: not walked).
template <int R>
__global__ __launch_bounds__(64) void bg_exit_chain_kernel(BgSplitArgs A) {
  constexpr int F = (R + 1) * 64;
  constexpr int kSym = BG_SPLIT_SYM(R);
  const BgPair P = A.pairs[blockIdx.x];
  const int n1 = P.n1, n2 = P.n2, NC = P.nc, NS = P.nstrips;
  if (NS == 0) return;
  const BgSplitLayout L = bg_split_layout(n1, n2, NS, NC, R, A.segc);
  int32_t* ar = A.split + P.split_off;
  const int lane = threadIdx.x;
  int sStar = ar[L.head + 7];
  const bool over = ar[L.head + 6] != 0 || (uint32_t)ar[L.head + 11] == A.epoch;
  int lo = NS;                                           // strips lo .. sStar are walked
  if (sStar >= 0 && !over) {
    lo = sStar;
    if (lane == 0) {
      ar[L.startcol + sStar] = ar[L.head + 1];
      if (sStar >= 1) {
        int c = ar[L.head + 4];
        const int cg = ar[L.head + 5];
        if (c >= kSym) c = (cg >= 1 && cg < L.G) ? ar[L.fres + ((size_t)sStar * L.G + cg - 1) * F + (c - kSym)] : -1;
        for (int s = sStar - 1; s >= 0; --s) {
          if ((c <= 0 && A.mode != BGK_GLOBAL) || c < 0 || c > n2) break;
          ar[L.startcol + s] = c;
          lo = s;
          if (s == 0) break;
          // strip s's bottom-row exit at column c, resolved here when symbolic (the resolve
          // kernel only resolves the frontiers: the chain reads one column per strip)
          int v = ar[L.ebot + (size_t)s * (n2 + 1) + c];
          if (v >= kSym) {
            const int seg = ((c + 63) >> 6) / A.segc;     // lane 63 is at column c at step c + 63
            v = seg >= 1 ? ar[L.fres + ((size_t)s * L.G + seg - 1) * F + (v - kSym)] : -1;
          }
          c = v;
        }
      }
    }
    lo = __shfl(lo, 0, 64);
  } else if (lane == 0) {
    ar[L.head + 7] = -1;
    sStar = -1;
  }
  sStar = __shfl(sStar, 0, 64);
  for (int s = lane; s < NS; s += 64)
    if (s < lo || s > sStar) ar[L.startcol + s] = -1;
}

#define BG_SPLIT_INST(RR)                                                    \
  template __global__ void bg_exit_kernel<RR>(BgSplitArgs);                 \
  template __global__ void bg_exit_conc_kernel<RR>(BgSplitArgs);            \
  template __global__ void bg_exit_resolve_kernel<RR>(BgSplitArgs);         \
  template __global__ void bg_exit_chain_kernel<RR>(BgSplitArgs);
BG_SPLIT_INST(2)
BG_SPLIT_INST(3)
BG_SPLIT_INST(4)
BG_SPLIT_INST(5)
BG_SPLIT_INST(8)
BG_SPLIT_INST(10)

// which: 0 exit pass, 1 resolve, 2 chain, 3 exit pass beside the DP
extern "C" void* bg_split_kernel_ptr(int R, int which) {
  switch (R) {
#define BG_SPLIT_CASE(RR)                                                      \
    case RR:                                                                   \
      return which == 0 ? (void*)&bg_exit_kernel<RR>                           \
           : which == 1 ? (void*)&bg_exit_resolve_kernel<RR>                   \
           : which == 2 ? (void*)&bg_exit_chain_kernel<RR>                     \
                        : (void*)&bg_exit_conc_kernel<RR>;
    BG_SPLIT_CASE(2)
    BG_SPLIT_CASE(3)
    BG_SPLIT_CASE(4)
    BG_SPLIT_CASE(5)
    BG_SPLIT_CASE(8)
    BG_SPLIT_CASE(10)
#undef BG_SPLIT_CASE
    default: return nullptr;
  }
}
// dynamic LDS of one workgroup of the concurrent exit pass (16 waves, 8 from R = 8)
extern "C" int bg_exit_conc_lds_bytes(int R) {
  const int w = R >= 8 ? 8 : 16;
  switch (R) {
    case 2: return w * 4 * exit_wave_ints<2>();
    case 3: return w * 4 * exit_wave_ints<3>();
    case 4: return w * 4 * exit_wave_ints<4>();
    case 5: return w * 4 * exit_wave_ints<5>();
    case 8: return w * 4 * exit_wave_ints<8>();
    case 10: return w * 4 * exit_wave_ints<10>();
    default: return 0;
  }
}
// dynamic LDS of one exit-pass workgroup (4 waves)
extern "C" int bg_exit_lds_bytes(int R) {
  switch (R) {
    case 2: return 4 * 4 * exit_wave_ints<2>();
    case 3: return 4 * 4 * exit_wave_ints<3>();
    case 4: return 4 * 4 * exit_wave_ints<4>();
    case 5: return 4 * 4 * exit_wave_ints<5>();
    case 8: return 4 * 4 * exit_wave_ints<8>();
    case 10: return 4 * 4 * exit_wave_ints<10>();
    default: return 0;
  }
}
