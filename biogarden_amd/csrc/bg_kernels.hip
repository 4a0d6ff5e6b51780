// MI355X (gfx950) kernels for the affine-gap pairwise aligner.
//
// Replaces the hot loops of the reference aligner (robsndr/biogarden):
//   compute_scores_global  src/alignment/aligner.rs:437-469
//   compute_scores_local   src/alignment/aligner.rs:471-509
//   end-cell selection     aligner.rs:112,173-176,247-251,308-312,369-404
//   backtrack              aligner.rs:511-592 (incl. the one-cell-late X/Y quirk)
//
// Geometry (DESIGN.md "Kernels"):
//   * one workgroup per pair, W waves; a pair's rows are cut into strips of 64*R rows,
//     strip s is owned by wave s % W.  Inside a strip, lane r owns rows [r*R, r*R+R) and the
//     wave sweeps anti-diagonally: at step t lane r computes column j = t - r, so the row above
//     (lane r-1's last row) arrives by one DPP wave_shr:1 per step and everything else stays in
//     VGPRs.  No LDS traffic for scores at all on the DNA path.
//   * strips are pipelined across the waves in phases of 64 steps separated by s_barrier;
//     strip s runs chunk c in phase start(s)+c with start(s) >= start(s-1)+2, so the boundary
//     row block a strip consumes was stored one phase earlier by the strip above.
//   * the trace (2 bits/cell, +2 for the affine kernel) is built with v_cmp -> SGPR masks ->
//     v_addc_co_u32 shift-in into per-lane 32-step words and streamed to HBM as coalesced
//     256-B stores.  Scores never touch HBM except the strip-boundary rows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "bg_device.h"

#include "bg_dev_util.h"
#include "bg_tag_common.h"

using namespace bgk;

namespace {

template <int R, bool AFFINE, bool LOCAL>
struct Strip {
  int Ma[R];               // M(i_k, j-1) + a   (the "left" of the next step)
  int Y[AFFINE ? R : 1];   // Y(i_k, j-1)
  unsigned tA[R];          // trace word: m-trace bit 0  ('Y', or STOP in local mode)
  unsigned tB[R];          // trace word: m-trace bit 1  ('X' and not 'Y', or STOP)
  unsigned tC[AFFINE ? R : 1];  // x_trace == 'M'
  unsigned tD[AFFINE ? R : 1];  // y_trace == 'M'
  int bestv[LOCAL ? R : 1];     // local: running row maximum
  int bpos[LOCAL ? R : 1];      // local: step of the first maximum
  int prof[R];             // DNA path: 4 packed int8 S(q, c) - a
  int topPrev;             // M(row above, j-1) + a  for row 0 of the lane
  int Xlast;               // X of the lane's last row (fed to the lane below)
  int code;                // target residue code of this lane's current column
  int oM, oX;              // boundary-row output accumulators (one 64-column block)
};

struct Ctx {
  int a, b, mode;
  int n1, n2, nc, nst, s;
  int rowbase;             // first 0-based row of this lane: s*64R + lane*R
  int olane, orow;         // which lane / row feeds the boundary output (last strip: row n1)
  uint32_t* trace;         // this strip's trace base
  int32_t* bndOutM;        // this strip's output row (M + a)
  int32_t* bndOutX;
  int32_t* lastcol;        // M(i, n2), i = 0..n1
  const int* ldsProf;      // LDS path: this wave's per-lane table
  int lane;
};

// Chunk code variants: FAST (interior chunks of every strip but the last), SEL (interior chunks
// of the last strip when row n1 is not a lane's last row), EDGE (first chunk: column-0 borders;
// last chunks: column n2 capture / validity; everything general).
enum { VAR_FAST = 0, VAR_SEL = 1, VAR_EDGE = 2 };

// per-lane LDS profile dwords per code: R int16 entries (two per dword), or R int32 entries
// (P32: tables whose S - a leave the int16 range, which the reference's i32 closure allows)
template <int R, bool P32>
struct MaskWPE { static constexpr int v = P32 ? R : (R + 1) / 2; };

// LCS (processing::patterns::longest_common_subsequence, patterns.rs:82-118; global mode, byte
// equality +1 / -1, open = extend = 0): a match always moves diagonally, so its cell's trace bits
// are cleared (a mismatch's diagonal is always strictly below up / left, and left-on-ties is the
// aligner's Y > X priority already).
template <int R, bool AFFINE, bool LOCAL, bool DNA, int VAR, bool P32 = false, bool LCS = false>
__device__ __forceinline__ void run_chunk(Strip<R, AFFINE, LOCAL>& S, const Ctx& C, int c, int bM,
                                          int bX, int cv) {
  const int a = C.a;
  const int b = C.b;
  const int lane = C.lane;
  const int t0 = c * BG_CHUNK;
  constexpr int NW = AFFINE ? 4 : 2;
#pragma unroll 1
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h) {
#pragma unroll
  for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
    const int u = h * BG_TRACE_BLK + uu;
    const int t = t0 + u;
    // ---- inputs from the row above: lane r-1's last row at this column, or the boundary row
    const int topMa = dpp_shr1(rdlane(bM, u), S.Ma[R - 1]);
    int topX = 0;
    if constexpr (AFFINE) topX = dpp_shr1(rdlane(bX, u), S.Xlast);
    S.code = dpp_shr1(rdlane(cv, u), S.code);
    int lp[DNA ? 1 : MaskWPE<R, P32>::v];
    if constexpr (!DNA && P32) {
      static_assert(R == 4, "the int32 profile is built for R = 4");
      const int4 v = *reinterpret_cast<const int4*>(C.ldsProf + (S.code * BG_WAVE + lane) * 4);
      lp[0] = v.x; lp[1] = v.y; lp[2] = v.z; lp[3] = v.w;
    } else if constexpr (!DNA) {
      if constexpr (R == 8) {
        const int4 v = *reinterpret_cast<const int4*>(C.ldsProf + (S.code * BG_WAVE + lane) * 4);
        lp[0] = v.x; lp[1] = v.y; lp[2] = v.z; lp[3] = v.w;
      } else if constexpr (R == 4) {
        const int2 v = *reinterpret_cast<const int2*>(C.ldsProf + (S.code * BG_WAVE + lane) * 2);
        lp[0] = v.x; lp[1] = v.y;
      } else {
#pragma unroll
        for (int q = 0; q < (R + 1) / 2; ++q) lp[q] = C.ldsProf[(S.code * BG_WAVE + lane) * ((R + 1) / 2) + q];
      }
    }
    bool valid = true;
    if constexpr (VAR == VAR_EDGE && LOCAL) valid = (t - lane >= 1) && (t - lane <= C.n2);
    int diag = S.topPrev;
    int xo = topMa;
    int xt = topX;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      int sp;
      if constexpr (DNA) sp = sbfe(S.prof[k], S.code, 8);
      else if constexpr (P32) sp = lp[k];
      else sp = sbfe(lp[k >> 1], (k & 1) * 16, 16);
      const int d = wadd(diag, sp);           // M(i-1,j-1) + S(seq1[i-1], seq2[j-1])
      const int yo = S.Ma[k];                 // M(i,j-1) + a
      int X, Yv;
      u64 mXt = 0, mYt = 0;
      if constexpr (AFFINE) {
        const int xs = sadd(xt, b);           // X(i-1,j).saturating_add(b)
        const int ys = sadd(S.Y[k], b);       // Y(i,j-1).saturating_add(b)
        mXt = ballot(xo >= xs);               // x_trace == 'M'  (aligner.rs:444/478)
        mYt = ballot(yo >= ys);               // y_trace == 'M'  (:448/484)
        if constexpr (LOCAL) { X = imax3(xo, xs, 0); Yv = imax3(yo, ys, 0); }  // clamp after trace
        else { X = imax(xo, xs); Yv = imax(yo, ys); }
        S.Y[k] = Yv;
      } else {
        // a >= b: X == M(i-1,j)+a and Y == M(i,j-1)+a exactly, x/y_trace == 'M' 
        if constexpr (LOCAL) { X = imax(xo, 0); Yv = imax(yo, 0); }
        else { X = xo; Yv = yo; }
      }
      const int best = imax3(d, X, Yv);
      u64 mY = ballot(best == Yv);            // priority Y > X > R (aligner.rs:455-463)
      u64 mX = ballot(best == X) & ~mY;
      if constexpr (LCS) {
        const u64 match = ballot(sp > 0);
        mY &= ~match;
        mX &= ~match;
      }
      if constexpr (LOCAL) {
        const u64 z = ballot(best == 0);      // M == 0: backtrack stops here (:181)
        mY |= z;
        mX |= z;
        const u64 gt = ballot(valid && (best > S.bestv[k]));
        S.bestv[k] = vsel(gt, best, S.bestv[k]);
        S.bpos[k] = vsel(gt, t, S.bpos[k]);
      }
      S.tA[k] = shift_in(S.tA[k], mY);
      S.tB[k] = shift_in(S.tB[k], mX);
      if constexpr (AFFINE) {
        S.tC[k] = shift_in(S.tC[k], mXt);
        S.tD[k] = shift_in(S.tD[k], mYt);
      }
      const int man = wadd(best, a);          // local: best >= 0 already, so M = best
      diag = yo;                              // M(i,j-1)+a = diagonal input of row i+1 (+S-a)
      xo = man;                               // M(i,j)+a   = vertical input of row i+1
      if constexpr (AFFINE) xt = X;
      S.Ma[k] = man;
    }
    S.topPrev = topMa;
    if constexpr (AFFINE) S.Xlast = xt;

    if constexpr (VAR == VAR_EDGE) {
      // column 0: this lane is at j == 0 -> load the border (aligner.rs:98-104 / fill(0))
      if (c == 0) {
        const bool rst = (t == lane);
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int i = C.rowbase + k + 1;
          const int border = wadd(col0_M(C.mode, i, a, b), a);
          S.Ma[k] = rst ? border : S.Ma[k];
          if constexpr (AFFINE) S.Y[k] = rst ? kNegInf : S.Y[k];
        }
      }
      // last column j == n2: M(i, n2) for the end-cell searches
      if (t >= C.n2 && t - C.n2 < BG_WAVE && C.n2 > 0) {
        if (lane == t - C.n2) {
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int i = C.rowbase + k + 1;
            if (i <= C.n1) C.lastcol[i] = wadd(S.Ma[k], -a);
          }
        }
      }
    }

    // ---- boundary output: row `orow` of lane `olane` at column t - olane
    {
      int sel = S.Ma[R - 1];
      if constexpr (VAR != VAR_FAST) {
#pragma unroll
        for (int k = 0; k < R - 1; ++k) sel = (C.orow == k) ? S.Ma[k] : sel;
      }
      const int jo = t - C.olane;
      if (VAR != VAR_EDGE || (jo >= 0 && jo <= C.n2)) {
        S.oM = wrlane(rdlane(sel, C.olane), jo & 63, S.oM);
        if constexpr (AFFINE) S.oX = wrlane(rdlane(S.Xlast, C.olane), jo & 63, S.oX);
        if ((jo & 63) == 63 || (VAR == VAR_EDGE && jo == C.n2)) {
          const int blk = jo & ~63;
          C.bndOutM[blk + lane] = S.oM;
          if constexpr (AFFINE) C.bndOutX[blk + lane] = S.oX;
        }
      }
    }

  }
  // ---- trace flush every 32 steps: R coalesced stores of NW words per lane
  //      layout: block b, row k, lane r -> dwords [((b*R + k)*64 + r)*NW, +NW)
  {
    uint32_t* tb = C.trace + (size_t)((t0 >> 5) + h) * (R * NW * BG_WAVE) + lane * NW;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if constexpr (AFFINE) {
        *reinterpret_cast<uint4*>(tb + k * NW * BG_WAVE) = make_uint4(S.tA[k], S.tB[k], S.tC[k], S.tD[k]);
      } else {
        *reinterpret_cast<uint2*>(tb + k * NW * BG_WAVE) = make_uint2(S.tA[k], S.tB[k]);
      }
    }
  }
  }
}

}  // namespace

// PGLOB (with P32): the per-wave int32 profile tables live in HBM (A.prof_scratch, one
// kdim x 64 x R table per (pair, wave)) instead of LDS — alphabets whose table does not fit the
// CU's LDS (more than ~150 codes with scores beyond int16); the step reads its entry through the
// vector L1.  LCS: see run_chunk.
template <int R, bool AFFINE, bool LOCAL, bool DNA, bool P32 = false, bool PGLOB = false, bool LCS = false>
__global__ __launch_bounds__((AFFINE || LOCAL) ? 512 : 1024) void bg_dp_kernel(BgDpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* sLut = smem;                                        // 256 B
  int16_t* sTab = reinterpret_cast<int16_t*>(smem + 256);      // 32x32 int16 (LDS path)
  int32_t* sTab32 = reinterpret_cast<int32_t*>(smem + 256);    // 32x32 int32 (P32)
  constexpr int TABB = P32 ? 4096 : 2048;
  const int lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  const int w = uni(threadIdx.x >> 6);
  constexpr int NW = AFFINE ? 4 : 2;
  constexpr int ROWS = BG_WAVE * R;

  for (int x = threadIdx.x; x < 256; x += blockDim.x) sLut[x] = A.lut[x];
  if (threadIdx.x < 16) reinterpret_cast<int*>(smem + A.prog_off)[threadIdx.x] = 0;
  // this pair's seq2 codes, staged once in LDS (every strip sweeps all of them)
  uint8_t* sCodes = smem + A.codes_off;
  {
    const BgPair& Pp = A.pairs[blockIdx.x];
    const uint8_t* g = A.codes2 + Pp.off2;
    if (A.codes_in_lds)
      for (int x = threadIdx.x; x < Pp.n2; x += blockDim.x) sCodes[x] = g[x];
  }
  // the batch's dense table: up to 32 codes staged in LDS (row stride 32); a wider alphabet (up
  // to 256 codes, row stride A.pstride) is read from HBM/L2 while the per-lane profiles are built
  const bool wideTab = A.kdim > 32;
  if constexpr (!DNA && P32) {
    if (!wideTab)
      for (int x = threadIdx.x; x < 1024; x += blockDim.x) sTab32[x] = A.profile[x];
  } else if constexpr (!DNA) {
    const int16_t* g = reinterpret_cast<const int16_t*>(A.profile);
    if (!wideTab)
      for (int x = threadIdx.x; x < 1024; x += blockDim.x) sTab[x] = g[x];
  }
  __syncthreads();
  const int16_t* gTab16 = reinterpret_cast<const int16_t*>(A.profile);
  const int tabStride = wideTab ? A.pstride : 32;

  const BgPair P = A.pairs[blockIdx.x];                        // by value: scalar loads, once
  const int n1 = P.n1, n2 = P.n2, nst = P.nstrips, NC = P.nc;
  if (nst == 0) return;
  const int a = A.open;
  const int b = A.ext;
  const int mode = A.mode;
  const size_t stripDw = (size_t)NC * (BG_CHUNK / BG_TRACE_BLK) * R * NW * BG_WAVE;

  int* ldsProf = nullptr;
  if constexpr (PGLOB)
    ldsProf = A.prof_scratch + ((size_t)blockIdx.x * W + w) * A.kdim * BG_WAVE * MaskWPE<R, P32>::v;
  else if constexpr (!DNA)
    ldsProf = reinterpret_cast<int*>(smem + 256 + TABB) + (size_t)w * A.kdim * BG_WAVE * MaskWPE<R, P32>::v;

  Ctx C;
  C.a = a; C.b = b; C.mode = mode;
  C.n1 = n1; C.n2 = n2; C.nc = NC; C.nst = nst;
  C.lane = lane;
  C.lastcol = A.aux + P.aux_off;
  C.ldsProf = ldsProf;

  Strip<R, AFFINE, LOCAL> S;
  const uint8_t* c1 = A.codes1 + P.off1;
  const uint8_t* c2 = A.codes2 + P.off2;
  const int nblk = NC - 1;                                     // boundary blocks per strip
  // Strips are pipelined through per-wave progress counters in LDS (no workgroup barriers):
  // after chunk c of its rho-th strip a wave publishes rho*nblk + (blocks of this strip stored);
  // strip s waits before chunk c until strip s-1 has stored boundary block c.
  int* sProg = reinterpret_cast<int*>(smem + A.prog_off);
  for (int s = w, rho = 0; s < nst; s += W, ++rho) {
    // ---------------- strip begin
    C.s = s;
    C.rowbase = s * ROWS + lane * R;
    const bool lastStrip = (s == nst - 1);
    const int lastRow = n1 - 1 - s * ROWS;                 // row n1, 0-based within the strip
    C.olane = lastStrip ? lastRow / R : BG_WAVE - 1;
    C.orow = lastStrip ? lastRow % R : R - 1;
    const bool selRow = C.orow != R - 1;
    C.trace = A.trace + P.trace_off / 4 + (size_t)s * stripDw;
    C.bndOutM = A.bndM + P.bnd_off + (size_t)s * NC * BG_CHUNK;
    C.bndOutX = AFFINE ? A.bndX + P.bnd_off + (size_t)s * NC * BG_CHUNK : nullptr;
    int qk[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {                              // independent loads, no branches
      const int i = C.rowbase + k + 1;
      qk[k] = c1[(i <= n1 ? i : n1) - 1];
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;                       // 1-based row
      const int q = (i <= n1) ? qk[k] : 0;
      if constexpr (DNA) S.prof[k] = A.profile[q >> 3];
      S.Ma[k] = wadd(col0_M(mode, i, a, b), a);
      if constexpr (AFFINE) { S.Y[k] = kNegInf; S.tC[k] = 0; S.tD[k] = 0; }
      S.tA[k] = 0; S.tB[k] = 0;
      if constexpr (LOCAL) { S.bestv[k] = (i <= n1) ? INT32_MIN : INT32_MAX; S.bpos[k] = 0; }
    }
    if constexpr (!DNA && P32) {
      // per-lane table [code][lane] of R int32 S(q_k, code) - a
      for (int cd = 0; cd < A.kdim; ++cd) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int i = C.rowbase + k + 1;
          const int qq = (i <= n1) ? c1[i - 1] : 0;
          ldsProf[(cd * BG_WAVE + lane) * R + k] =
              wideTab ? A.profile[qq * tabStride + cd] : sTab32[qq * 32 + cd];
        }
      }
    } else if constexpr (!DNA) {
      // per-lane table [code][lane] of R int16 S(q_k, code) - a, 2R bytes per entry
      constexpr int WPE = (R + 1) / 2;
      for (int cd = 0; cd < A.kdim; ++cd) {
#pragma unroll
        for (int q2 = 0; q2 < WPE; ++q2) {
          int v = 0;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int k = q2 * 2 + hh;
            if (k < R) {
              const int i = C.rowbase + k + 1;
              const int qq = (i <= n1) ? c1[i - 1] : 0;
              const int16_t t = wideTab ? gTab16[qq * tabStride + cd] : sTab[qq * 32 + cd];
              v |= ((int)(uint16_t)t) << (16 * hh);
            }
          }
          ldsProf[(cd * BG_WAVE + lane) * WPE + q2] = v;
        }
      }
    }
    S.topPrev = 0; S.Xlast = kNegInf; S.code = 0; S.oM = 0; S.oX = 0;
    // residue codes of seq2, two chunks in flight: column j = c*64 + lane uses seq2[j-1]
    for (int c = 0; c < NC; ++c) {
      int cv;
      {
        const int j = c * BG_CHUNK + lane;
        const int jj = j < 1 ? 1 : (j > n2 ? n2 : j);
        const int v = A.codes_in_lds ? (int)sCodes[jj - 1] : (int)c2[jj - 1];
        cv = (j >= 1 && j <= n2) ? v : 0;
      }
      const int jb = c * BG_CHUNK + lane;
      int bM, bX = kNegInf;
      if (s == 0) {
        bM = wadd(row0_M(mode, jb, a, b), a);
      } else {
        if (c < nblk) {                                        // block c of strip s-1
          const int need = ((s - 1) / W) * nblk + c + 1;
          const int pw = (s - 1) % W;
          int np = 0;
          while (__hip_atomic_load(sProg + pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
            poll_backoff(np);
        }
        const int32_t* src = A.bndM + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb;
        bM = load_agent(src);
        if constexpr (AFFINE) bX = load_agent(A.bndX + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb);
      }
      const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
      if (edge) run_chunk<R, AFFINE, LOCAL, DNA, VAR_EDGE, P32, LCS>(S, C, c, bM, bX, cv);
      else if (lastStrip && selRow) run_chunk<R, AFFINE, LOCAL, DNA, VAR_SEL, P32, LCS>(S, C, c, bM, bX, cv);
      else run_chunk<R, AFFINE, LOCAL, DNA, VAR_FAST, P32, LCS>(S, C, c, bM, bX, cv);
      // publish: the chunk ends with the R trace stores of its second half; everything issued
      // before them (this chunk's boundary-row stores included) has reached L2 at vmcnt(R)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(R) : "memory");
      if (lane == 0)
        __hip_atomic_store(sProg + w, rho * nblk + (c < nblk ? c : nblk), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // ---------------- strip end
    if constexpr (LOCAL) {
      int32_t* rowbest = A.aux + P.aux_off + (n1 + 1);
      int32_t* rowpos = rowbest + n1;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int i = C.rowbase + k + 1;
        if (i <= n1) { rowbest[i - 1] = S.bestv[k]; rowpos[i - 1] = S.bpos[k] - lane; }
      }
    }
  }
}

#include "bg_finish.h"

// ------------------------------------------------------------------ score only (global)
// End cell of global mode without a traceback (aligner.rs:112: M(n1, n2); borders :98-104), for
// the score-only callers (analysis::seq::edit_distance): one thread per pair.
__global__ __launch_bounds__(256) void bg_global_score_kernel(BgFinishArgs F) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= F.npairs) return;
  const BgPair& P = F.pairs[q];
  int score;
  if (P.n1 == 0) score = row0_M(BGK_GLOBAL, P.n2, F.open, F.ext);
  else if (P.n2 == 0) score = col0_M(BGK_GLOBAL, P.n1, F.open, F.ext);
  else score = F.aux[P.aux_off + P.n1];                // lastcol[n1] = M(n1, n2)
  BgResult res;
  res.status = 0; res.score = score; res.end_i = P.n1; res.end_j = P.n2;
  res.out_start = (uint32_t)(P.n1 + P.n2); res.out_len = 0;
  res.start1 = (uint32_t)P.n1; res.start2 = (uint32_t)P.n2;
  res.npre = 0; res.ntail = 0;
  F.results[P.index] = res;
}
extern "C" void* bg_global_score_kernel_ptr() { return (void*)&bg_global_score_kernel; }

// ------------------------------------------------------------------ export (for collectives)

__global__ __launch_bounds__(256) void bg_export_kernel(BgExportArgs E) {
  const BgPair& P = E.pairs[blockIdx.x];
  const BgResult& r = E.results[P.index];
  BgPairResultDev* recs = reinterpret_cast<BgPairResultDev*>(E.dst + 8);
  uint8_t* s1 = E.dst + 8 + E.npairs_caller * sizeof(BgPairResultDev);
  uint8_t* s2 = s1 + E.out_bytes;
  const uint8_t* src1 = E.out1 + P.out_off + r.out_start;
  const uint8_t* src2 = E.out2 + P.out_off + r.out_start;
  for (uint32_t x = threadIdx.x; x < r.out_len; x += blockDim.x) {
    s1[P.caller_off + x] = src1[x];
    s2[P.caller_off + x] = src2[x];
  }
  if (threadIdx.x == 0) {
    BgPairResultDev o;
    o.status = r.status;
    if (o.status == 0 && bg_ref_divergent(E.mode, P.n1, P.n2, r.score, P.buf_rows, P.buf_cols)) o.status = 4;
    o.score = r.score;
    o.offset = P.caller_off;
    o.len = r.out_len;
    o.end_i = (uint32_t)r.end_i;
    o.end_j = (uint32_t)r.end_j;
    o.start1 = r.start1;
    o.start2 = r.start2;
    o.reserved = 0;
    recs[P.caller] = o;
  }
}

extern "C" void* bg_export_kernel_ptr() { return (void*)&bg_export_kernel; }

// ------------------------------------------------------------------ compact export (§8(e) gather)
// Three launches on the handle's stream: per caller pair its header from the template and its
// packed-ops size (plan pairs from their results); one workgroup's exclusive scan of the sizes
// into offsets; per plan pair its header and ops copied into the record.
__global__ __launch_bounds__(256) void bg_compact_size_kernel(BgCompactArgs E) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;   // sizes zeroed by the host
  if (p >= (uint64_t)E.nplan) return;
  const BgPair& P = E.pairs[p];
  const BgResult& r = E.results[P.index];
  const uint32_t ncore = r.out_len - r.npre - r.ntail;
  E.sizes[P.caller] = (ncore + 3) / 4;
}

__global__ __launch_bounds__(256) void bg_compact_write_kernel(BgCompactArgs E) {
  uint64_t* head = reinterpret_cast<uint64_t*>(E.dst);
  BgCompactHdr* hdr = reinterpret_cast<BgCompactHdr*>(E.dst + 32);
  uint8_t* opsArea = E.dst + 32 + E.npairs_caller * sizeof(BgCompactHdr);
  if (blockIdx.x >= (unsigned)E.nplan) {
    // caller pairs never planned (statuses decided on the host): the template's status
    const uint64_t base = (uint64_t)(blockIdx.x - E.nplan) * blockDim.x + threadIdx.x;
    if (base < E.npairs_caller) {
      const BgPairResultDev& t = E.recs[base];
      BgCompactHdr o;
      o.status = t.status; o.score = 0; o.ops_off = E.sizes[base]; o.len = 0; o.end_i = 0; o.end_j = 0;
      o.start1 = 0; o.start2 = 0; o.npre = 0; o.ntail = 0; o.reserved = 0;
      // planned pairs are written by their own workgroups (after this one may have run): only
      // pairs whose template status marks them as decided on the host
      if (t.status != 0) hdr[base] = o;
    }
    if (base == 0) { head[0] = 0x31434742ull;   /* "BGC1" */ head[1] = E.npairs_caller; head[2] = E.sizes[E.npairs_caller]; head[3] = (uint64_t)E.mode; }
    return;
  }
  const BgPair& P = E.pairs[blockIdx.x];
  const BgResult& r = E.results[P.index];
  const uint32_t nb = (r.out_len - r.npre - r.ntail + 3) / 4;
  const uint64_t off = E.sizes[P.caller];
  for (uint32_t x = threadIdx.x; x < nb; x += blockDim.x) opsArea[off + x] = E.ops[P.ops_off + x];
  if (threadIdx.x == 0) {
    BgCompactHdr o;
    o.status = r.status;
    if (o.status == 0 && bg_ref_divergent(E.mode, P.n1, P.n2, r.score, P.buf_rows, P.buf_cols)) o.status = 4;
    o.score = r.score; o.ops_off = off; o.len = r.out_len;
    o.end_i = (uint32_t)r.end_i; o.end_j = (uint32_t)r.end_j; o.start1 = r.start1; o.start2 = r.start2;
    o.npre = r.npre; o.ntail = r.ntail; o.reserved = 0;
    hdr[P.caller] = o;
  }
}

extern "C" void* bg_compact_size_kernel_ptr() { return (void*)&bg_compact_size_kernel; }
extern "C" void* bg_compact_write_kernel_ptr() { return (void*)&bg_compact_write_kernel; }

// Residue coding on the device: codes[x] = lut[raw[x]] over both concatenated sequence sets
// (the host uploads only the raw bytes, which the strings are built from anyway).  16 bytes per
// lane, grid-stride; the 256-byte table is read through the scalar-free vector path from L1.
__global__ __launch_bounds__(256) void bg_code_kernel(const uint8_t* __restrict__ raw1,
                                                      uint8_t* __restrict__ cd1, size_t n1,
                                                      const uint8_t* __restrict__ raw2,
                                                      uint8_t* __restrict__ cd2, size_t n2,
                                                      const uint8_t* __restrict__ lut) {
  __shared__ uint8_t t[256];
  t[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const size_t v1 = (n1 + 15) / 16, v2 = (n2 + 15) / 16;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < v1 + v2; v += stride) {
    const bool first = v < v1;
    const size_t base = (first ? v : v - v1) * 16;
    const uint8_t* in = first ? raw1 : raw2;
    uint8_t* out = first ? cd1 : cd2;
    const size_t n = first ? n1 : n2;
    if (base + 16 <= n) {
      const uint4 w = *reinterpret_cast<const uint4*>(in + base);
      const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = (uint32_t)t[ww[k] & 0xff] | ((uint32_t)t[(ww[k] >> 8) & 0xff] << 8) |
               ((uint32_t)t[(ww[k] >> 16) & 0xff] << 16) | ((uint32_t)t[ww[k] >> 24] << 24);
      *reinterpret_cast<uint4*>(out + base) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
      for (size_t x = base; x < n; ++x) out[x] = t[in[x]];
    }
  }
}

extern "C" void* bg_code_kernel_ptr() { return (void*)&bg_code_kernel; }

// ------------------------------------------------------------------ instantiation table

typedef void (*bg_dp_fn)(BgDpArgs);

#define BG_INST(R, AF, LO, DNA) \
  template __global__ void bg_dp_kernel<R, AF, LO, DNA>(BgDpArgs);

#define BG_INST_R(R)            \
  BG_INST(R, false, false, true) \
  BG_INST(R, false, true, true)  \
  BG_INST(R, true, false, true)  \
  BG_INST(R, true, true, true)   \
  BG_INST(R, false, false, false) \
  BG_INST(R, false, true, false)  \
  BG_INST(R, true, false, false)  \
  BG_INST(R, true, true, false)

BG_INST_R(4)
BG_INST_R(8)
// int32 profile entries (tables whose S - a leave int16): R = 4, every gap model and mode
template __global__ void bg_dp_kernel<4, false, false, false, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, false, true, false, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, true, false, false, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, true, true, false, true>(BgDpArgs);

// ... with the per-wave profile tables in HBM (more than ~150 codes)
template __global__ void bg_dp_kernel<4, false, false, false, true, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, false, true, false, true, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, true, false, false, true, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, true, true, false, true, true>(BgDpArgs);
// LCS tie rule (bg_lcs_batch beyond the checkpoint tracebacks' chunk keys): linear global, R = 4
template __global__ void bg_dp_kernel<4, false, false, true, false, false, true>(BgDpArgs);
template __global__ void bg_dp_kernel<4, false, false, false, false, false, true>(BgDpArgs);

extern "C" void* bg_dp_kernel_p32_ptr(int R, int affine, int local, int global) {
  if (R != 4) return nullptr;
  if (global) {
    if (affine) return local ? (void*)&bg_dp_kernel<4, true, true, false, true, true> : (void*)&bg_dp_kernel<4, true, false, false, true, true>;
    return local ? (void*)&bg_dp_kernel<4, false, true, false, true, true> : (void*)&bg_dp_kernel<4, false, false, false, true, true>;
  }
  if (affine) return local ? (void*)&bg_dp_kernel<4, true, true, false, true> : (void*)&bg_dp_kernel<4, true, false, false, true>;
  return local ? (void*)&bg_dp_kernel<4, false, true, false, true> : (void*)&bg_dp_kernel<4, false, false, false, true>;
}
extern "C" void* bg_dp_kernel_lcs_ptr(int R, int dna) {
  if (R != 4) return nullptr;
  return dna ? (void*)&bg_dp_kernel<4, false, false, true, false, false, true>
             : (void*)&bg_dp_kernel<4, false, false, false, false, false, true>;
}
// metric-path (linear gaps, DNA register profile) kernels at extra strip heights: the planner
// picks R so that a pair's strip count fills the workgroup's waves (DESIGN.md "Geometry")
BG_INST(5, false, false, true)
BG_INST(10, false, false, true)
BG_INST(5, false, true, true)
BG_INST(10, false, true, true)

extern "C" void* bg_dp_kernel_ptr(int R, int affine, int local, int dna) {
#define BG_PICK(RR)                                                                        \
  if (R == RR) {                                                                           \
    if (!affine && !local && dna) return (void*)&bg_dp_kernel<RR, false, false, true>;     \
    if (!affine && local && dna) return (void*)&bg_dp_kernel<RR, false, true, true>;       \
    if (affine && !local && dna) return (void*)&bg_dp_kernel<RR, true, false, true>;       \
    if (affine && local && dna) return (void*)&bg_dp_kernel<RR, true, true, true>;         \
    if (!affine && !local && !dna) return (void*)&bg_dp_kernel<RR, false, false, false>;   \
    if (!affine && local && !dna) return (void*)&bg_dp_kernel<RR, false, true, false>;     \
    if (affine && !local && !dna) return (void*)&bg_dp_kernel<RR, true, false, false>;     \
    if (affine && local && !dna) return (void*)&bg_dp_kernel<RR, true, true, false>;       \
  }
  BG_PICK(4)
  BG_PICK(8)
#undef BG_PICK
  if (!affine && dna && (R == 5 || R == 10)) {
    if (R == 5) return local ? (void*)&bg_dp_kernel<5, false, true, true> : (void*)&bg_dp_kernel<5, false, false, true>;
    return local ? (void*)&bg_dp_kernel<10, false, true, true> : (void*)&bg_dp_kernel<10, false, false, true>;
  }
  return nullptr;
}

template <int R>
static void* finish_ck_ptr(int mode) {
  switch (mode) {
    case BGK_GLOBAL: return (void*)&bg_finish_kernel<R, false, BGK_GLOBAL, true>;
    case BGK_FITTING: return (void*)&bg_finish_kernel<R, false, BGK_FITTING, true>;
    case BGK_OVERLAP: return (void*)&bg_finish_kernel<R, false, BGK_OVERLAP, true>;
    case BGK_SEMIGLOBAL: return (void*)&bg_finish_kernel<R, false, BGK_SEMIGLOBAL, true>;
    default: return nullptr;
  }
}
// checkpoint traceback (linear gaps, non-local): the finish kernel over recomputed chunks
extern "C" void* bg_finish_ck_kernel_ptr(int R, int mode) {
  switch (R) {
    case 2: return finish_ck_ptr<2>(mode);
    case 3: return finish_ck_ptr<3>(mode);
    case 4: return finish_ck_ptr<4>(mode);
    case 5: return finish_ck_ptr<5>(mode);
    case 8: return finish_ck_ptr<8>(mode);
    case 10: return finish_ck_ptr<10>(mode);
    default: return nullptr;
  }
}
// LDS of the checkpoint finish kernel with `nslots` chunk slots (0: the maximum) and `nw` waves:
// chunk slots (the scan aliases them), scalars, nw recompute areas, the chunk map
extern "C" size_t bg_finish_ck_lds_bytes(int R, int nslots, int nw, int* win_bytes) {
  int slot = 0, area = 0, maxs = 8;
  switch (R) {
    case 2: slot = ck_slot_dw<2>(); area = ck_wave_ints<2>(); maxs = ck_slots<2>(); break;
    case 3: slot = ck_slot_dw<3>(); area = ck_wave_ints<3>(); maxs = ck_slots<3>(); break;
    case 4: slot = ck_slot_dw<4>(); area = ck_wave_ints<4>(); maxs = ck_slots<4>(); break;
    case 5: slot = ck_slot_dw<5>(); area = ck_wave_ints<5>(); maxs = ck_slots<5>(); break;
    case 8: slot = ck_slot_dw<8>(); area = ck_wave_ints<8>(); maxs = ck_slots<8>(); break;
    default: slot = ck_slot_dw<10>(); area = ck_wave_ints<10>(); maxs = ck_slots<10>(); break;
  }
  const int ns = (nslots > 0 && nslots < maxs) ? nslots : maxs;
  *win_bytes = std::max(ns * slot * 4, 2 * 256 * 4);
  return (size_t)*win_bytes + 64 * 4 + (size_t)nw * area * 4 + kCkMapEntries * 4;  // + chunk map
}

template <int R, bool AF>
static void* finish_ptr(int mode) {
  switch (mode) {
    case BGK_GLOBAL: return (void*)&bg_finish_kernel<R, AF, BGK_GLOBAL>;
    case BGK_LOCAL: return (void*)&bg_finish_kernel<R, AF, BGK_LOCAL>;
    case BGK_FITTING: return (void*)&bg_finish_kernel<R, AF, BGK_FITTING>;
    case BGK_OVERLAP: return (void*)&bg_finish_kernel<R, AF, BGK_OVERLAP>;
    default: return (void*)&bg_finish_kernel<R, AF, BGK_SEMIGLOBAL>;
  }
}
extern "C" void* bg_finish_kernel_ptr(int R, int affine, int mode) {
  if (R == 4) return affine ? finish_ptr<4, true>(mode) : finish_ptr<4, false>(mode);
  if (R == 8) return affine ? finish_ptr<8, true>(mode) : finish_ptr<8, false>(mode);
  if (R == 2 && !affine) return finish_ptr<2, false>(mode);
  if (R == 3 && !affine) return finish_ptr<3, false>(mode);
  if (R == 5 && !affine) return finish_ptr<5, false>(mode);
  if (R == 10 && !affine) return finish_ptr<10, false>(mode);
  return nullptr;
}

// Which strip heights exist for a kernel family (the planner's candidate set).
extern "C" int bg_dp_has_R(int R, int affine, int local, int dna) {
  return bg_dp_kernel_ptr(R, affine, local, dna) != nullptr;
}
// Trace window of the finish kernel: the full 56 KiB (2 workgroups per CU) for few long pairs;
// for batches of many pairs a smaller window (>= 8 blocks) lets more pairs walk per CU.
extern "C" int bg_finish_window_bytes(int R, int affine, size_t npairs, int cus) {
  const int blk = R * BG_WAVE * (affine ? 4 : 2) * 4;
  if (npairs <= (size_t)cus * 2) return kWinBytesMax / blk * blk;
  int w = std::max(8 * blk, 20480);
  return std::min(w, kWinBytesMax) / blk * blk;
}
extern "C" size_t bg_finish_lds_bytes(int win_bytes) { return (size_t)win_bytes + 64 * 4; }
