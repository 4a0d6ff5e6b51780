// The tagged linear-gap step shared by the forward DP kernel (bg_tag_kernel.hip) and the
// checkpoint traceback's chunk recomputation (bg_ckpt.hip); see bg_tag_kernel.hip for the
// value frame, the tags and the LDS operand routing.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_dev_util.h"

namespace bgk {

template <int R>
struct TagStrip {
  int Y[R];           // Y form of (i_k, j-1): 4*M'(i_k, j-1) + 3
  unsigned tA[R];     // trace codes of steps 0-15 of the current 32-step block (2 bits each)
  unsigned tB[R];     // steps 16-31
  int topPrev;        // X form of (row above, j-1) for the lane's first row
  int Xlast;          // X form of (lane's last row, j): handed down to lane r+1 by DPP
};

struct TagCtx {
  int a, b, mode, n1, n2, rowbase, orow, lane;
  bool repeatN1 = false;    // score_chunk: rows below n1 take row n1's value at column 0
  uint32_t* trace;          // this strip's trace
  int32_t* bndOut;          // this strip's boundary row (X forms), 64-column blocks
  int32_t* lastcol;         // M(i, n2)
  const int* bIn;           // LDS: staged boundary block of the strip above (64 X forms)
  int* ring;                // LDS: this wave's 256-slot output ring
  int* oLane;               // LDS: this lane's ring write base (slot = u + 64 - lane [+128])
  const uint16_t* codeLane; // LDS: this chunk's scaled codes, + u = column t0 + u - lane
  int* mail;                // LDS mailbox slot for the block finished in this chunk (consumer
                            // in this workgroup), or nullptr: the block goes to HBM
  const uint8_t* profLane;  // LDS: this lane's profile entries (+ scaled code = entry address)
  int top0, topStep;        // score_chunk<..., TOP0>: M'(0, t0) and its step along row 0
};

// Column n2 in the score-only steps: the lane at column n2 keeps its R values in chunk-local
// registers (one v_cndmask per row in the steps t in [n2, n2 + 64)) and the lanes that reached it
// in this chunk store them at the chunk's end; a divergent 1-lane store per step there cost the
// strip's last chunks ~200 cycles a step, and in the WIDE chain every strip's tail adds to the
// next one's start.
template <int R>
__device__ __forceinline__ void catch_lastcol(const int (&Y)[R], int (&L)[R], int t, int n2, int lane) {
  if (t >= n2 && t - n2 < BG_WAVE && n2 > 0) {              // wave-uniform
    const bool sel = lane == t - n2;
#pragma unroll
    for (int k = 0; k < R; ++k) L[k] = sel ? Y[k] : L[k];
  }
}
template <int R>
__device__ __forceinline__ void store_lastcol(const int (&L)[R], const TagCtx& C, int t0) {
  const int tl = C.n2 + C.lane;                              // the step this lane was at column n2
  if (C.n2 <= 0 || tl < t0 || tl >= t0 + BG_CHUNK) return;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    if (i <= C.n1) C.lastcol[i] = wadd(L[k], wmul(C.a, i + C.n2));
  }
}

// profile dwords per lane and code: R int8 bytes, padded to an aligned ds_read width
template <int R>
struct ProfW { static constexpr int v = R <= 4 ? 1 : (R <= 8 ? 2 : 4); };

template <int RW>
struct ProfV { int w[RW]; };

template <int RW>
__device__ __forceinline__ ProfV<RW> load_prof(const uint8_t* p) {
  ProfV<RW> r;
  if constexpr (RW == 1) {
    r.w[0] = *reinterpret_cast<const int*>(p);
  } else if constexpr (RW == 2) {
    const int2 v = *reinterpret_cast<const int2*>(p);
    r.w[0] = v.x; r.w[1] = v.y;
  } else {
    const int4 v = *reinterpret_cast<const int4*>(p);
    r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
  }
  return r;
}

// x + sign_extend(byte `sel` of w): written as a constant-offset v_bfe_i32 + v_add, which the
// SDWA peephole folds into one v_add_u32_sdwa ... sext src1_sel:BYTE_sel
__device__ __forceinline__ int add_sbyte(int x, int w, int sel) {
  return x + __builtin_amdgcn_sbfe(w, 8 * sel, 8);
}

// TV_COL0 (score-only steps, bg_score_step.h): chunk 0 when the border values need the column-0
// reset (global mode): straight-line selects.  TV_EDGE's per-step branches (reset and column n2)
// made a strip's first and last chunks ~2x a plain one, and in the WIDE chain both are on the
// critical path; the score-only steps catch column n2 without them (bg_tag_kernel.hip kTagCodes)
enum { TV_FAST = 0, TV_SEL = 1, TV_EDGE = 2, TV_COL0 = 3 };

// Y form of column 0, row i: 4*(M(i,0) - a*i) + 3 (aligner.rs:98-104 borders)
__device__ __forceinline__ int col0_Y(int mode, int i, int a, int b) {
  return 4 * wadd(col0_M(mode, i, a, b), -wmul(a, i)) + 3;
}

// KIND_FWD: the forward tagged DP (trace to HBM, boundary row out, M(i, n2) capture).
// KIND_RECOMP: the traceback's recomputation of one chunk from a checkpoint (bg_ckpt.hip):
// trace to the LDS chunk cache, nothing else written.
enum { KIND_FWD = 0, KIND_RECOMP = 1 };

template <int R, int VAR, bool WIDE, int KIND = KIND_FWD>
__device__ __forceinline__ void tag_chunk(TagStrip<R>& S, const TagCtx& C, int c) {
  const int a = C.a;
  const int t0 = c * BG_CHUNK;
  const int lane = C.lane;
  constexpr int RW = ProfW<R>::v;
  // operand pipeline: the code of step u+2 and the profile entry of step u+1 are in flight
  // while step u computes
  int nTop = C.bIn[0];
  ProfV<RW> nP = load_prof<RW>(C.profLane + C.codeLane[0]);
  int nCode = C.codeLane[1];
  const uint16_t* cl = C.codeLane + 2;   // advanced by 32 per half: immediate offsets inside
  const int* bi = C.bIn + 1;
#pragma unroll 1
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK, bi += BG_TRACE_BLK) {
#pragma unroll
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int t = t0 + u;
      const int topIn = nTop;
      const ProfV<RW> P = nP;
      nP = load_prof<RW>(C.profLane + nCode);
      nCode = cl[uu];
      nTop = bi[uu];
      const int topX = dpp_shr1(topIn, S.Xlast);             // X form of (row above, j)
      int dIn = S.topPrev;                                    // X form of (row above, j-1)
      int xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int yo = S.Y[k];
        const int d = add_sbyte(dIn, P.w[k >> 2], k & 3);      // 4*(M'(i-1,j-1) + S - 2a), tag 0
        const int best = imax(imax(d, xo), yo);
        // append the 2-bit code; the empty asm pins each update to its step (otherwise LLVM
        // sinks all 16 alignbits to the flush and keeps every step's `best` live)
        if (uu < 16) { S.tA[k] = __builtin_amdgcn_alignbit((unsigned)best, S.tA[k], 2); asm volatile("" : "+v"(S.tA[k])); }
        else { S.tB[k] = __builtin_amdgcn_alignbit((unsigned)best, S.tB[k], 2); asm volatile("" : "+v"(S.tB[k])); }
        const int yn = best | 3;                              // Y form for column j+1
        dIn = yo;
        xo = yn - 1;                                          // X form for row i+1
        S.Y[k] = yn;
      }
      S.topPrev = topX;
      S.Xlast = xo;
      if constexpr (VAR == TV_EDGE) {
        if (c == 0) {                                         // column 0 (aligner.rs:98-104)
          const bool rst = (t == lane);
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int i = C.rowbase + k + 1;
            S.Y[k] = rst ? col0_Y(C.mode, i, a, C.b) : S.Y[k];
          }
          S.Xlast = rst ? S.Y[R - 1] - 1 : S.Xlast;
        }
        if (KIND == KIND_FWD && t >= C.n2 && t - C.n2 < BG_WAVE && C.n2 > 0) {   // M(i, n2)
          if (lane == t - C.n2) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
              const int i = C.rowbase + k + 1;
              if (i <= C.n1) C.lastcol[i] = wadd(S.Y[k] >> 2, wmul(a, i + C.n2));
            }
          }
        }
      }
      if constexpr (KIND == KIND_FWD) {
        int out = S.Xlast;
        if constexpr (VAR != TV_FAST) {
#pragma unroll
          for (int k = 0; k < R - 1; ++k) out = (C.orow == k) ? S.Y[k] - 1 : out;
        }
        C.oLane[u] = out;
      }
      // one step per scheduling region: hoisting later steps' profile lookups spills
      __builtin_amdgcn_sched_barrier(0);
    }
    if (KIND == KIND_FWD && h == 1 && c >= 1) {
      // block c-1 (ring slots 0-63) is final: copy it out, slide the ring by one block
      const int v = C.ring[lane];
      const int nx = C.ring[64 + lane];
      if (C.mail)           // the next strip runs on a wave of this workgroup
        C.mail[lane] = v;
      else if constexpr (WIDE)   // read by workgroups on other XCDs: agent-coherent store
        __hip_atomic_store(C.bndOut + (c - 1) * BG_CHUNK + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        C.bndOut[(c - 1) * BG_CHUNK + lane] = v;
      C.ring[lane] = nx;
    } else if (KIND == KIND_FWD && h == 1) {
      C.ring[lane] = C.ring[64 + lane];
    }
    // trace flush every 32 steps: block b, row k, lane r -> dwords [((b*R + k)*64 + r)*2, +2)
    uint32_t* tb = C.trace + (size_t)((t0 >> 5) + h) * (R * 2 * BG_WAVE) + lane * 2;
#pragma unroll
    for (int k = 0; k < R; ++k)
      *reinterpret_cast<uint2*>(tb + k * 2 * BG_WAVE) = make_uint2(S.tA[k], S.tB[k]);
  }
}


// v_mov_b32_dpp row_shr:1 — lane r receives lane r-1 within its 16-lane row; the first lane of
// each row keeps `old` (band recomputation: four independent 16-lane jobs per wave).
__device__ __forceinline__ int dpp_rowshr1(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, 0x111, 0xf, 0xf, false);
}

// The row hand-off of P pairs per wave (64 / P lanes each, bg_grp_kernel.hip): lane r receives
// lane r - 1 and a pair's first lane keeps `old` — row_shr:1 does both for P = 4; for P = 2,
// wave_shr:1 and lane 32 takes `old` by a select.
template <int P>
__device__ __forceinline__ int grp_shr1(int old, int src, bool first) {
  if constexpr (P == 4) {
    (void)first;
    return dpp_rowshr1(old, src);
  } else {
    const int v = dpp_shr1(old, src);
    return first ? old : v;
  }
}

// Recomputation for grouped pairs (BgFinishArgs::grouped): the tagged step of tag_chunk over up
// to P jobs of 64 / P lanes in one wave.  Job j = lane / (64 / P) recomputes one chunk of a pair
// (C.lane = its lane) from its checkpoint; its first lane's row above comes from its own staged
// block (C.bIn, per lane), the others' from the lane above (grp_shr1).  cl0: this lane's job
// chunk (EDGE: column 0 of chunk 0 is reset per lane); the trace goes to `slot` as [half h][row k]
// [job lane ql] x uint2 (64 / P lane stride), when `store`.
template <int R, bool EDGE, int P>
__device__ __forceinline__ void tag_chunk_jobs(TagStrip<R>& S, const TagCtx& C, int cl0, uint32_t* slot, int ql,
                                               bool store) {
  constexpr int L = 64 / P;
  const bool first = C.lane == 0;
  const int a = C.a;
  const int sl = C.lane;
  constexpr int RW = ProfW<R>::v;
  int nTop = C.bIn[0];
  ProfV<RW> nP = load_prof<RW>(C.profLane + C.codeLane[0]);
  int nCode = C.codeLane[1];
  const uint16_t* cl = C.codeLane + 2;
  const int* bi = C.bIn + 1;
#pragma unroll 1
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK, bi += BG_TRACE_BLK) {
#pragma unroll
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int topIn = nTop;
      const ProfV<RW> Pv = nP;
      nP = load_prof<RW>(C.profLane + nCode);
      nCode = cl[uu];
      nTop = bi[uu];
      const int topX = grp_shr1<P>(topIn, S.Xlast, first);    // X form of (row above, j)
      int dIn = S.topPrev;
      int xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int yo = S.Y[k];
        const int d = add_sbyte(dIn, Pv.w[k >> 2], k & 3);
        const int best = imax(imax(d, xo), yo);
        if (uu < 16) { S.tA[k] = __builtin_amdgcn_alignbit((unsigned)best, S.tA[k], 2); asm volatile("" : "+v"(S.tA[k])); }
        else { S.tB[k] = __builtin_amdgcn_alignbit((unsigned)best, S.tB[k], 2); asm volatile("" : "+v"(S.tB[k])); }
        const int yn = best | 3;
        dIn = yo;
        xo = yn - 1;
        S.Y[k] = yn;
      }
      S.topPrev = topX;
      S.Xlast = xo;
      if constexpr (EDGE) {
        const bool rst = (cl0 == 0) && (u == sl);             // column 0 (aligner.rs:98-104)
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int i = C.rowbase + k + 1;
          S.Y[k] = rst ? col0_Y(C.mode, i, a, C.b) : S.Y[k];
        }
        S.Xlast = rst ? S.Y[R - 1] - 1 : S.Xlast;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (store) {
      uint32_t* tb = slot + (size_t)h * (R * 2 * L) + ql * 2;
#pragma unroll
      for (int k = 0; k < R; ++k)
        *reinterpret_cast<uint2*>(tb + k * 2 * L) = make_uint2(S.tA[k], S.tB[k]);
    }
  }
}

}  // namespace bgk
