// The score-only forward steps of the checkpoint DP (bg_tag_kernel.hip only): score_chunk (one
// workgroup per pair, SPAN, and the last strip of a WIDE pair) and the WIDE conveyor step
// score_chunk_conv.  Kept out of bg_tag_common.h, which the traceback kernels include.
#pragma once
#include "bg_tag_common.h"

// operand pipeline depth of the many-wave score step (A/B builds: -DBG_PF_MANY=2)
#ifndef BG_PF_MANY
#define BG_PF_MANY 1
#endif

namespace bgk {

// Score-only forward step (checkpoint mode): values are the untagged M'(i,j) = M(i,j) - a(i+j),
// where M'(i,j) = max(M'(i-1,j-1) + S - 2a, M'(i-1,j), M'(i,j-1)) — two VALU ops per cell
// (v_add_u32_sdwa, v_max3).  No trace: the traceback recomputes the chunks its path crosses
// from the per-chunk checkpoints with tag_chunk<KIND_RECOMP>.  Every strip's boundary row goes
// to HBM (the recomputation's top input), plus the LDS mailbox for a consumer in the workgroup.
// TOP0 (strip 0, interior chunks): the row above is row 0, M'(0, j) = top0 + (j - t0) topStep
// (aligner.rs:98-104 borders, linear in j for j >= 1), kept in a scalar register instead of one
// broadcast LDS read per step — the read that makes single-strip batches (C4) LDS-bound.
// AGT: the boundary row goes out with agent-scope (sc1) stores, for a consumer in another
// workgroup, possibly on another XCD (WIDE and SPAN); else plain stores (the same workgroup, or
// the traceback after the kernel's end)
template <int R, int VAR, bool WIDE, bool TOP0 = false, bool AGT = WIDE>
__device__ __forceinline__ void score_chunk(TagStrip<R>& S, const TagCtx& C, int c) {
  const int a = C.a;
  const int lane = C.lane;
  constexpr int RW = ProfW<R>::v;
  // operand pipeline depth: the profile entries and row-above inputs of the next PF steps are in
  // flight while a step computes.  One step hides the LDS latency at several waves per SIMD; a
  // lone wave per SIMD (WIDE) issues a step in a few tens of cycles, so it runs 4 steps ahead
  // (rotating registers; 32 % PF == 0 keeps the rotation aligned across the two 32-step halves).
  constexpr int PF = WIDE ? 4 : BG_PF_MANY;
  int c0v[R];                                                // TV_COL0: this lane's M'(i, 0)
  if constexpr (VAR == TV_COL0) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;
      const int ii = (C.repeatN1 && i > C.n1) ? C.n1 : i;       // rows below n1: row n1's
      c0v[k] = wadd(col0_M(C.mode, ii, a, C.b), -wmul(a, ii));
    }
  }
  // (the codes run 2 PF steps ahead: a profile load's address is a code loaded PF steps earlier)
  int nTop = TOP0 ? C.top0 : C.bIn[0];
  int qTop[PF], qCode[PF];
  ProfV<RW> qP[PF];
#pragma unroll
  for (int d = 0; d < PF; ++d) {
    qTop[d] = TOP0 ? 0 : C.bIn[d];
    qP[d] = load_prof<RW>(C.profLane + C.codeLane[d]);
    qCode[d] = C.codeLane[PF + d];
  }
  const uint16_t* cl = C.codeLane + 2 * PF;
  const int* bi = C.bIn + PF;
#pragma unroll
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK, bi += BG_TRACE_BLK) {
#pragma unroll
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int slot = uu % PF;                               // constant after unrolling
      const int topIn = TOP0 ? nTop : qTop[slot];
      const ProfV<RW> P = qP[slot];
      qP[slot] = load_prof<RW>(C.profLane + qCode[slot]);    // step u + PF
      qCode[slot] = cl[uu];                                   // step u + 2 PF
      // row above of step u + PF (past the 64-entry block at the chunk's end: never used)
      if constexpr (!TOP0) qTop[slot] = bi[uu];
      const int topX = dpp_shr1(topIn, S.Xlast);             // M'(row above, j)
      // lane 0 keeps the DPP's old operand, the only lane whose row-0 input matters
      if constexpr (TOP0) nTop = topX + C.topStep;
      int dIn = S.topPrev;                                    // M'(row above, j-1)
      int xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int yo = S.Y[k];
        const int d = add_sbyte(dIn, P.w[k >> 2], k & 3);      // M'(i-1,j-1) + S - 2a
        const int best = imax(imax(d, xo), yo);
        dIn = yo;
        xo = best;
        S.Y[k] = best;
      }
      S.topPrev = topX;
      S.Xlast = xo;
      if constexpr (VAR == TV_COL0) {                         // c == 0: lane u at column 0
        // an opaque lane per step: hoisted, the 64 compares' masks took 128 SGPRs and spilled
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const bool rst = (u == ln);
#pragma unroll
        for (int k = 0; k < R; ++k) S.Y[k] = rst ? c0v[k] : S.Y[k];
        S.Xlast = rst ? c0v[R - 1] : S.Xlast;
      }
      int out = S.Xlast;
      if constexpr (VAR != TV_FAST) {
#pragma unroll
        for (int k = 0; k < R - 1; ++k) out = (C.orow == k) ? S.Y[k] : out;
      }
      C.oLane[u] = out;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (h == 1 && c >= 1) {
      const int v = C.ring[lane];
      const int nx = C.ring[64 + lane];
      if (C.mail) C.mail[lane] = v;
      if constexpr (AGT)
        __hip_atomic_store(C.bndOut + (c - 1) * BG_CHUNK + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        C.bndOut[(c - 1) * BG_CHUNK + lane] = v;
      C.ring[lane] = nx;
    } else if (h == 1) {
      C.ring[lane] = C.ring[64 + lane];
    }
  }
}

// v_mov_b32_dpp wave_shl:1 — lane r receives lane r+1; lane 63 keeps `old`.
__device__ __forceinline__ int dpp_shl1(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false);
}

// Score-only step of a WIDE strip that hands its boundary row to another strip (C3: one wave per
// SIMD, every step a dependent chain, so the LDS instructions per step are the step's latency,
// tools/micro/lone_step.hip).  The row above and the row this strip hands down share ONE register
// Q instead of a broadcast LDS read and a ring write per step:
//   * at the chunk start Q[r] = the row above at column t0 + r (block c);
//   * step u reads Q[0] (the DPP's old operand: lane 0's row above at column t0 + u), then shifts
//     Q down one lane (wave_shl:1) and puts this wave's last-row value of the previous step
//     (lane 63, column t0 + u - 64) into lane 63;
//   * after 64 steps Q[r] = the last row at column t0 - 64 + r: block c - 1, final, ready to go to
//     the consumer.  The caller stores it and loads the next incoming block.
// Only the last strip, whose output row is row n1 (any lane), keeps the ring (score_chunk).
// `mid` runs between the chunk's two halves (the kernel's HBM hand-offs).
// The operand pipeline (codes 2 PF steps ahead, profile entries PF ahead) runs on across chunks:
// a chunk's last steps prefetch the next chunk's first operands from the staged row (which holds
// columns up to t0 + 127), so a chunk starts without a dependent code -> profile LDS round trip.
constexpr int kConvPF = 4;
template <int RW>
struct ConvPipe {
  int qCode[kConvPF];
  ProfV<RW> qP[kConvPF];
};
// the strip's first chunk: operands of steps 0 .. PF - 1 and codes of steps PF .. 2 PF - 1
template <int RW>
__device__ __forceinline__ void conv_pipe_init(ConvPipe<RW>& pp, const TagCtx& C) {
#pragma unroll
  for (int d = 0; d < kConvPF; ++d) {
    pp.qP[d] = load_prof<RW>(C.profLane + C.codeLane[d]);
    pp.qCode[d] = C.codeLane[kConvPF + d];
  }
}
template <int R, int VAR, class Mid>
__device__ __forceinline__ void score_chunk_conv(TagStrip<R>& S, const TagCtx& C, int c, int& Q,
                                                 ConvPipe<ProfW<R>::v>& pp, Mid&& mid) {
  const int a = C.a;
  const int lane = C.lane;
  constexpr int RW = ProfW<R>::v;
  int c0v[R];                                                // TV_COL0: this lane's M'(i, 0)
  if constexpr (VAR == TV_COL0) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;
      c0v[k] = wadd(col0_M(C.mode, i, a, C.b), -wmul(a, i));
    }
  }
  constexpr int PF = kConvPF;
  int (&qCode)[PF] = pp.qCode;
  ProfV<RW> (&qP)[PF] = pp.qP;
  const uint16_t* cl = C.codeLane + 2 * PF;
#pragma unroll
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK) {
#pragma unroll
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int slot = uu % PF;
      const ProfV<RW> P = qP[slot];
      qP[slot] = load_prof<RW>(C.profLane + qCode[slot]);
      qCode[slot] = cl[uu];
      const int topX = dpp_shr1(Q, S.Xlast);                  // M'(row above, j); lane 0: Q[0]
      Q = dpp_shl1(S.Xlast, Q);                               // hand the last row down the conveyor
      int dIn = S.topPrev;
      int xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int yo = S.Y[k];
        const int d = add_sbyte(dIn, P.w[k >> 2], k & 3);
        const int best = imax(imax(d, xo), yo);
        dIn = yo;
        xo = best;
        S.Y[k] = best;
      }
      S.topPrev = topX;
      S.Xlast = xo;
      if constexpr (VAR == TV_COL0) {                         // c == 0: lane u at column 0
        // an opaque lane per step: hoisted, the 64 compares' masks took 128 SGPRs and spilled
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const bool rst = (u == ln);
#pragma unroll
        for (int k = 0; k < R; ++k) S.Y[k] = rst ? c0v[k] : S.Y[k];
        S.Xlast = rst ? c0v[R - 1] : S.Xlast;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (h == 0) {
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

}  // namespace bgk
