// The score-only affine-gap step (forward DP, bg_aff_kernel.hip) and its trace-producing twin
// (the checkpoint traceback's chunk recomputation, bg_finish.h).  Replaces the cell loops of
// compute_scores_global (src/alignment/aligner.rs:437-469) and compute_scores_local (:471-509)
// for every case the linear tagged kernel does not take: affine gaps (a < b), local mode and
// alphabets of more than four symbols.
//
// Geometry is the tagged kernel's (bg_tag_kernel.hip): strips of 64R rows, lane r owns rows
// [rR, rR+R), anti-diagonal sweep with lane r at column t - r, the row above of the lane's first
// row arriving by DPP wave_shr:1 from lane r-1 (lane 0: the staged boundary block of the strip
// above), per-lane LDS profile entries selected by the column code, an all-lane LDS output ring.
//
// Values.
//   global / fitting / overlap / semiglobal: the frame V~ = V - b(i+j) for M, X and Y, in which
//   both extensions are free and the opening constant c = a - b lands once per cell, on M:
//     O(i,j)  = M~(i,j) + c                               (the "opened" M, what is stored)
//     X~(i,j) = max(O(i-1,j), X~(i-1,j))                  (M(i-1,j)+a vs X(i-1,j)+b, shifted)
//     Y~(i,j) = max(O(i,j-1), Y~(i,j-1))
//     M~(i,j) = max(O(i-1,j-1) + S - a - b, X~, Y~)
//   5 VALU ops per cell (v_add_u32_sdwa with the int8 profile byte S - a - b, v_max, v_max,
//   v_max3, v_add) against 6 in the frame V - a(i+j), where X and Y each paid an extension add.
//   The trace bits compare the same pairs shifted by the same amount (x_trace 'I' iff
//   O(i-1,j) < X~(i-1,j) iff M(i-1,j)+a < X(i-1,j)+b), so they are the reference's.  -inf
//   (X row 0, Y column 0, aligner.rs:49-50) is the finite kAffNeg, which no longer drifts; the
//   host only takes this path when every value stays far from wrapping, so saturating_add
//   (aligner.rs:443,447) never saturates and the frame is exact.
//   local: the frame cannot carry the clamp at 0, so values are kept as MA = M + a:
//     X = max3(MA(i-1,j), X(i-1,j) + b, 0),  Y = max3(MA(i,j-1), Y(i,j-1) + b, 0)
//     M = max3(MA(i-1,j-1) + S - a, X, Y),   best_k = max(best_k, M)
//   8 VALU ops per cell.  The clamp follows the trace bits (aligner.rs:477-486), which only the
//   recomputation produces.
//
// No trace is written by the forward pass.  At each chunk start every lane stores its R M and
// R Y values, the M of the row above at the previous column (diagonal input) and the X of its
// last row: ckpt[((s * NC + c) * (2R + 2) + k) * 64 + lane].  The traceback recomputes the
// chunks its path crosses (aff_recomp) and gets the reference's three trace matrices,
// m_trace (2 bits: R / X / Y, local STOP), x_trace == 'M', y_trace == 'M', in the layout of
// the mask kernel's HBM trace.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_dev_util.h"
#include "bg_tag_common.h"

namespace bgk {

constexpr int kAffNeg = -(1 << 30);

// int8 profile entries (S - 2a, local S - a): R per lane and code, padded to a ds_read width
// of 1, 2 or 4 dwords (ProfW); the host takes this path only when every entry fits
template <int R>
struct AffW { static constexpr int v = ProfW<R>::v; };

template <int R, bool LOCAL>
struct AffStrip {
  int M[R];                   // M'(i_k, j-1)  (local: M(i_k, j-1) + a)
  int Y[R];                   // Y'(i_k, j-1)  (local: Y(i_k, j-1))
  int best[LOCAL ? R : 1];    // local: running row maximum of M
  int bc[LOCAL ? R : 1];      // local: chunk in which it last increased
  int topPrev;                // M of (row above the lane's first row, j-1)
  int Xlast;                  // X of (lane's last row, j-1): handed to lane r+1 by DPP
};

struct AffCtx {
  int a, b, e, mode, n1, n2, rowbase, orow, lane;
  int32_t* lastcol;           // M(i, n2) (non-local)
  const int2* bIn;            // LDS: staged (M, X) of the strip above, one per column
  int2* ring;                 // LDS: this wave's 128-entry output ring
  int2* oLane;                // ring write base of this lane: slot = u + 64 - lane
  const uint16_t* codeLane;   // LDS: scaled codes, + u = column t0 + u - lane
  int2* mail;                 // LDS mailbox slot for the block finished in this chunk, or null
  int32_t* bndOutM;           // HBM boundary row (M) of this strip, 64-column blocks
  int32_t* bndOutX;
  const uint8_t* profLane;    // LDS: this lane's profile entries
};

template <int RW>
__device__ __forceinline__ int prof_word(const ProfV<RW>& P, int k) {
  return P.w[k >> 2];
}

// border M of column 0, row i, in the kernel's representation (aligner.rs:98-104, 163, 233-237):
// local M + a, otherwise O = M - b*i + (a - b)
template <bool LOCAL>
__device__ __forceinline__ int aff_col0(int mode, int i, int a, int b) {
  if constexpr (LOCAL) return a;
  return wadd(wadd(col0_M(mode, i, a, b), -wmul(b, i)), wadd(a, -b));
}
template <bool LOCAL>
__device__ __forceinline__ int aff_row0(int mode, int j, int a, int b) {
  if constexpr (LOCAL) return a;
  return wadd(wadd(row0_M(mode, j, a, b), -wmul(b, j)), wadd(a, -b));
}

// One cell; returns M (local: M itself, S.M gets M + a).  x / y are X / Y of the cell.
template <bool LOCAL>
__device__ __forceinline__ void aff_cell(int dIn, int pw, int sel, int mo, int xo, int ml, int yl,
                                         int a, int g, int& x, int& y, int& m) {
  const int d = add_sbyte(dIn, pw, sel);
  if constexpr (LOCAL) {
    x = imax3(mo, xo + g, 0);
    y = imax3(ml, yl + g, 0);
  } else {
    x = imax(mo, xo + g);
    y = imax(ml, yl + g);
  }
  m = imax3(d, x, y);
}

// Forward score-only chunk (64 steps).  VAR: TV_FAST interior chunks, TV_SEL last strip with
// row n1 not the lane's last row, TV_EDGE column-0 borders / column n2 / local validity.
template <int R, bool LOCAL, int VAR>
__device__ __forceinline__ void aff_chunk(AffStrip<R, LOCAL>& S, const AffCtx& C, int c) {
  const int a = C.a;
  const int g = LOCAL ? C.b : 0;            // extend increment in the kernel's representation
  const int oc = wadd(C.a, -C.b);           // non-local: the opening constant c = a - b
  const int t0 = c * BG_CHUNK;
  const int lane = C.lane;
  constexpr int RW = AffW<R>::v;
  int Lc[R] = {};                           // TV_EDGE, non-local: M at column n2 (see below)
  int2 nTop = C.bIn[0];
  ProfV<RW> nP = load_prof<RW>(C.profLane + C.codeLane[0]);
  int nCode = C.codeLane[1];
  const uint16_t* cl = C.codeLane + 2;
  const int2* bi = C.bIn + 1;
#pragma unroll 1
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK, bi += BG_TRACE_BLK) {
#pragma unroll
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int t = t0 + u;
      const int2 top = nTop;
      const ProfV<RW> P = nP;
      nP = load_prof<RW>(C.profLane + nCode);
      nCode = cl[uu];
      nTop = bi[uu];
      const int topM = dpp_shr1(top.x, S.M[R - 1]);          // M of (row above, j)
      const int topX = dpp_shr1(top.y, S.Xlast);              // X of (row above, j)
      bool valid = true;
      if constexpr (VAR == TV_EDGE && LOCAL) valid = (t - lane >= 1) && (t - lane <= C.n2);
      int dIn = S.topPrev;
      int mo = topM, xo = topX;
      int oX = 0;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        int x, y, m;
        aff_cell<LOCAL>(dIn, prof_word(P, k), k & 3, mo, xo, S.M[k], S.Y[k], a, g, x, y, m);
        dIn = S.M[k];
        if constexpr (LOCAL) {
          // opaque v_max: a plain max chain over the unrolled steps is re-associated by LLVM into
          // a tree that keeps every step's M live (spills)
          asm volatile("v_max_i32 %0, %0, %1" : "+v"(S.best[k]) : "v"(valid ? m : 0));
          m = m + a;
        } else {
          m = m + oc;                           // O(i,j)
        }
        S.M[k] = m;
        S.Y[k] = y;
        mo = m;
        xo = x;
        if constexpr (VAR != TV_FAST) oX = (C.orow == k) ? x : oX;
      }
      S.topPrev = topM;
      S.Xlast = xo;
      if constexpr (VAR == TV_EDGE) {
        if (c == 0) {                                         // column 0 (aligner.rs:98-104)
          const bool rst = (t == lane);
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int i = C.rowbase + k + 1;
            S.M[k] = rst ? aff_col0<LOCAL>(C.mode, i, a, C.b) : S.M[k];
            S.Y[k] = rst ? kAffNeg : S.Y[k];
          }
          S.Xlast = rst ? kAffNeg : S.Xlast;
          oX = rst ? kAffNeg : oX;
        }
        if constexpr (!LOCAL) {
          // column n2: M(i, n2), caught in registers by the lane passing it and stored at the
          // chunk's end (a divergent one-lane store per step made these chunks ~200 cycles a
          // step slower, bg_tag_common.h catch_lastcol)
          if (t >= C.n2 && t - C.n2 < BG_WAVE && C.n2 > 0) {  // wave-uniform
            const bool sel = lane == t - C.n2;
#pragma unroll
            for (int k = 0; k < R; ++k) Lc[k] = sel ? S.M[k] : Lc[k];
          }
        }
      }
      int outM = S.M[R - 1], outX = S.Xlast;
      if constexpr (VAR != TV_FAST) {
#pragma unroll
        for (int k = 0; k < R - 1; ++k) outM = (C.orow == k) ? S.M[k] : outM;
        outX = (C.orow == R - 1) ? S.Xlast : oX;
      }
      C.oLane[u] = make_int2(outM, outX);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (h == 1 && c >= 1) {
      // block c-1 (ring slots 0-63) is final: hand it down, slide the ring by one block
      const int2 v = C.ring[lane];
      const int2 nx = C.ring[64 + lane];
      if (C.mail) C.mail[lane] = v;
      C.bndOutM[(c - 1) * BG_CHUNK + lane] = v.x;
      C.bndOutX[(c - 1) * BG_CHUNK + lane] = v.y;
      C.ring[lane] = nx;
    } else if (h == 1) {
      C.ring[lane] = C.ring[64 + lane];
    }
  }
  if constexpr (VAR == TV_EDGE && !LOCAL) {
    const int tl = C.n2 + lane;                   // the step this lane was at column n2
    if (C.n2 > 0 && tl >= t0 && tl < t0 + BG_CHUNK) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int i = C.rowbase + k + 1;
        if (i <= C.n1) C.lastcol[i] = wadd(wadd(Lc[k], -oc), wmul(C.b, i + C.n2));
      }
    }
  }
}

// Recomputation of one chunk from its checkpoint with the reference's trace bits (aligner.rs:
// 441-467 / 475-507), into an LDS slot of bit planes [h][plane][row k][lane] (two 32-step
// halves, step uu at bit 31 - uu):
//   plane 0  m != Y          (m_trace is not 'Y')
//   plane 1  m != X          (with plane 0: 'X' when only this is clear, 'R' when both are set)
//   plane 2  x_trace == 'I'  (the extension beat the opening: xo < satadd(X(i-1,j), b))
//   plane 3  y_trace == 'I'
//   plane 4  local only: M == 0 (the walk stops, aligner.rs:181)
// Each bit is the sign of one difference, shifted in by v_alignbit (no compare, no SGPR round
// trip); the operands arrive through the same one-step-ahead LDS pipeline as the forward pass.
// FIND (local end cell): the first column j of row `fq` of lane `fl` with M == target is
// returned in `found` (-1 if none in this chunk).
// LCS (processing::patterns::longest_common_subsequence, src/processing/patterns.rs:88-98, run as
// a global alignment with S = +1 / -1 and a = b = 0, whose M is the reference's match table): a
// match takes the diagonal whatever its ties, so both "not Y" and "not X" are also set where the
// diagonal candidate reaches M (m - d - 1 < 0; a mismatch's diagonal is always strictly lower).
template <bool LOCAL>
__host__ __device__ constexpr int ack_planes() { return LOCAL ? 5 : 4; }

__device__ __forceinline__ unsigned sign_in(unsigned acc, int diff) {
  return __builtin_amdgcn_alignbit(acc, (unsigned)diff, 31);   // (acc << 1) | (diff < 0)
}

template <int R, bool LOCAL, bool FIRST, bool FIND, bool LCS = false>
__device__ __forceinline__ void aff_recomp(AffStrip<R, LOCAL>& S, const AffCtx& C, int c,
                                           uint32_t* slot, int fq, int fl, int target, int& found) {
  const int a = C.a;
  const int g = LOCAL ? C.b : 0;
  const int oc = wadd(C.a, -C.b);
  const int t0 = c * BG_CHUNK;
  const int lane = C.lane;
  constexpr int RW = AffW<R>::v;
  constexpr int NP = ack_planes<LOCAL>();
  unsigned tr[NP][R];
  int2 nTop = C.bIn[0];
  ProfV<RW> nP = load_prof<RW>(C.profLane + C.codeLane[0]);
  int nCode = C.codeLane[1];
  const uint16_t* cl = C.codeLane + 2;
  const int2* bi = C.bIn + 1;
  constexpr int UNR = R >= 8 ? 8 : BG_TRACE_BLK;     // full unroll of R = 8 exceeds LLVM's limit
#pragma unroll 1
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK, bi += BG_TRACE_BLK) {
#pragma unroll UNR
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int t = t0 + u;
      const int2 top = nTop;
      const ProfV<RW> P = nP;
      nP = load_prof<RW>(C.profLane + nCode);
      nCode = cl[uu];
      nTop = bi[uu];
      const int topM = dpp_shr1(top.x, S.M[R - 1]);
      const int topX = dpp_shr1(top.y, S.Xlast);
      int dIn = S.topPrev;
      int mo = topM, xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int d = add_sbyte(dIn, prof_word(P, k), k & 3);
        const int xs = xo + g, ys = S.Y[k] + g;
        int x, y;
        if constexpr (LOCAL) { x = imax3(mo, xs, 0); y = imax3(S.M[k], ys, 0); }
        else { x = imax(mo, xs); y = imax(S.M[k], ys); }
        const int m = imax3(d, x, y);
        // the empty asm pins each shift to its step (else LLVM sinks them all to the flush and
        // keeps every step's differences live)
        const int dg = LCS ? m - d - 1 : 0;             // < 0: the diagonal reaches M
        tr[0][k] = sign_in(uu ? tr[0][k] : 0u, (y - m) | dg);
        tr[1][k] = sign_in(uu ? tr[1][k] : 0u, (x - m) | dg);
        tr[2][k] = sign_in(uu ? tr[2][k] : 0u, mo - xs);
        tr[3][k] = sign_in(uu ? tr[3][k] : 0u, S.M[k] - ys);
        asm volatile("" : "+v"(tr[0][k]), "+v"(tr[1][k]), "+v"(tr[2][k]), "+v"(tr[3][k]));
        if constexpr (LOCAL) {
          tr[NP - 1][k] = sign_in(uu ? tr[NP - 1][k] : 0u, m - 1);
          asm volatile("" : "+v"(tr[NP - 1][k]));
        }
        if constexpr (FIND) {
          const int j = t - lane;
          if (k == fq && lane == fl && m == target && found < 0 && j >= 1 && j <= C.n2) found = j;
        }
        dIn = S.M[k];
        const int mv = LOCAL ? m + a : m + oc;
        S.M[k] = mv;
        S.Y[k] = y;
        mo = mv;
        xo = x;
      }
      S.topPrev = topM;
      S.Xlast = xo;
      if constexpr (FIRST) {
        const bool rst = (t == lane);
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int i = C.rowbase + k + 1;
          S.M[k] = rst ? aff_col0<LOCAL>(C.mode, i, a, C.b) : S.M[k];
          S.Y[k] = rst ? kAffNeg : S.Y[k];
        }
        S.Xlast = rst ? kAffNeg : S.Xlast;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t* tb = slot + (size_t)(h * NP) * R * BG_WAVE + lane;
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int k = 0; k < R; ++k) tb[(p * R + k) * BG_WAVE] = tr[p][k];
  }
}

}  // namespace bgk
