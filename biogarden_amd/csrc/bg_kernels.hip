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

template <int R, bool AFFINE, bool LOCAL, bool DNA, int VAR>
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
    int lp[DNA ? 1 : (R + 1) / 2];
    if constexpr (!DNA) {
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

template <int R, bool AFFINE, bool LOCAL, bool DNA>
__global__ __launch_bounds__((AFFINE || LOCAL) ? 512 : 1024) void bg_dp_kernel(BgDpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* sLut = smem;                                        // 256 B
  int16_t* sTab = reinterpret_cast<int16_t*>(smem + 256);      // 32x32 int16 (LDS path)
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
  if constexpr (!DNA) {
    const int16_t* g = reinterpret_cast<const int16_t*>(A.profile);
    for (int x = threadIdx.x; x < 1024; x += blockDim.x) sTab[x] = g[x];
  }
  __syncthreads();

  const BgPair P = A.pairs[blockIdx.x];                        // by value: scalar loads, once
  const int n1 = P.n1, n2 = P.n2, nst = P.nstrips, NC = P.nc;
  if (nst == 0) return;
  const int a = A.open;
  const int b = A.ext;
  const int mode = A.mode;
  const size_t stripDw = (size_t)NC * (BG_CHUNK / BG_TRACE_BLK) * R * NW * BG_WAVE;

  int* ldsProf = nullptr;
  if constexpr (!DNA) ldsProf = reinterpret_cast<int*>(smem + 256 + 2048) + (size_t)w * A.kdim * BG_WAVE * ((R + 1) / 2);

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
    if constexpr (!DNA) {
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
              v |= ((int)(uint16_t)sTab[qq * 32 + cd]) << (16 * hh);
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
          while (__hip_atomic_load(sProg + pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
            __builtin_amdgcn_s_sleep(1);
        }
        const int32_t* src = A.bndM + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb;
        bM = load_agent(src);
        if constexpr (AFFINE) bX = load_agent(A.bndX + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb);
      }
      const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
      if (edge) run_chunk<R, AFFINE, LOCAL, DNA, VAR_EDGE>(S, C, c, bM, bX, cv);
      else if (lastStrip && selRow) run_chunk<R, AFFINE, LOCAL, DNA, VAR_SEL>(S, C, c, bM, bX, cv);
      else run_chunk<R, AFFINE, LOCAL, DNA, VAR_FAST>(S, C, c, bM, bX, cv);
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

__device__ __forceinline__ int lastrowM(const Fin& f, int j) {
  if (f.n1 == 0) return row0_M(f.mode, j, f.a, f.b);
  if (j == 0) return col0_M(f.mode, f.n1, f.a, f.b);
  const int v = f.lastrowMa[j];
  // the tagged kernel stores X forms 4*(M(n1,j) - a*(n1+j)) + 2
  // checkpoint mode (tag 2) stores M'(n1,j) = M(n1,j) - a*(n1+j) itself
  if (f.F->tag == 2) return wadd(v, wmul(f.a, f.n1 + j));
  return f.F->tag ? wadd(v >> 2, wmul(f.a, f.n1 + j)) : wadd(v, -f.a);
}
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

template <int R, bool AFFINE, int MODE, bool CK = false>
__global__ __launch_bounds__(256) void bg_finish_kernel(BgFinishArgs F) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int NW = AFFINE ? 4 : 2;
  constexpr int ROWS = BG_WAVE * R;
  constexpr int BLK_DW = R * BG_WAVE * NW;             // dwords per 32-step trace block
  const int NBW = F.win_bytes / (BLK_DW * 4);          // blocks per window
  uint32_t* win = reinterpret_cast<uint32_t*>(smem);
  int* sh = reinterpret_cast<int*>(smem + F.win_bytes);  // 64 ints of block-shared scalars
  int* scan = sh + 64;                                 // 2 x 256 ints
  // checkpoint mode: the window is ck_slots<R>() recomputed chunks; sh[16+z] / sh[24+z] = strip /
  // chunk held by slot z (-1: empty); per-wave recompute areas follow the scan
  int* ckArea = scan + 2 * 256;
  int* jscr = ckArea + (CK ? 4 * ck_wave_ints<R>() : 0);
  // checkpoint mode: direct-mapped table (strip & 31, chunk & 31) -> (s << 20 | c << 4 | slot)
  unsigned* ckMap = reinterpret_cast<unsigned*>(jscr);
  if (CK) {
    for (int x = threadIdx.x; x < 1024; x += blockDim.x) ckMap[x] = 0xFFFFFFFFu;
    __syncthreads();
  }

  const BgPair& P = F.pairs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6), NT = blockDim.x;
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
  // (bias(v) << 32 | j) and (bias(v) << 32 | ~i).
  {
    u64 ka = 0, kb = 0;
    const int32_t* rowbest = f.lastcol + (n1 + 1);
    if (mode == BGK_LOCAL) {
      // first row-major cell with the strict maximum; (0,0) with 0 when nothing is positive
      if (n2 > 0) {
#pragma unroll 4
        for (int i = 1 + tid; i <= n1; i += NT) {
          const u64 kk = ((u64)bias(rowbest[i - 1]) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
          ka = kk > ka ? kk : ka;
        }
      }
    } else if (mode == BGK_FITTING || mode == BGK_SEMIGLOBAL) {
#pragma unroll 4
      for (int i = tid; i <= n1; i += NT) {          // last column, first strict max (:247, :376)
        const u64 kk = ((u64)bias(lastcolM(f, i)) << 32) | (unsigned)(0xFFFFFFFFu - (unsigned)i);
        ka = kk > ka ? kk : ka;
      }
    }
    if (mode == BGK_OVERLAP || mode == BGK_SEMIGLOBAL) {
#pragma unroll 4
      for (int j = tid; j <= n2; j += NT) {          // last row, last max (:308, :369)
        const u64 kk = ((u64)bias(lastrowM(f, j)) << 32) | (unsigned)j;
        kb = kk > kb ? kk : kb;
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
          ej = rowbest[n1 + ei - 1];                 // rowpos follows rowbest
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
      sh[0] = ei; sh[1] = ej; sh[2] = score; sh[3] = colcase;
    }
  }
  __syncthreads();
  const int ei = uni(sh[0]), ej = uni(sh[1]), score = uni(sh[2]), colcase = uni(sh[3]);

  // ---------------- semiglobal tail gaps (:389-404): the last ntail columns of the slot; the
  // walk's op codes (0 = (s1, s2), 1 = (s1, '-'), 2 = ('-', s2)) go backwards in front of them
  const int ntail = (mode == BGK_SEMIGLOBAL) ? (colcase ? n1 - ei : n2 - ej) : 0;

  // ---------------- traceback walk (aligner.rs:511-592)
  const uint32_t* tr = F.trace + P.trace_off / 4;
  const size_t stripDw = (size_t)P.nc * (BG_CHUNK / BG_TRACE_BLK) * BLK_DW;
  const int stripBlocks = P.nc * (BG_CHUNK / BG_TRACE_BLK);
  int k = ei, l = ej, state = 0, status = 0, ncore = 0;
  int curS = -1, curB0 = 0, curNb = 0;
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
  constexpr int kCkSlots = ck_slots<R>();
  int ckS[kCkSlots], ckC[kCkSlots];                  // checkpoint mode: resident chunks
  int ckNext = 0;                                    // next slot to fill (FIFO)
#pragma unroll
  for (int z = 0; z < kCkSlots; ++z) { ckS[z] = -1; ckC[z] = -1; }
  // decodes the 8x8 neighbourhood anchored at (k, l): lane (dk, dl) holds cell (k - dk, l - dl)
  // 4-bit code of cell (kk, ll) from the resident trace (window or recomputed chunks)
  auto decode_cell = [&](int kk, int ll) -> int {
    if (kk <= 0 || ll <= 0) return kCodeBorder | ((kk == 0) ? 2 : 1);  // column 0 'X', row 0 'Y'
    const int vr = kk - 1;
    const int sidx = vr / ROWS, rem = vr - sidx * ROWS, r = rem / R, q = rem - r * R;
    const int t = ll + r, bl = t >> 5;
    if constexpr (CK) {
      const int cc = t >> 6;
      const unsigned e = ckMap[((sidx & 31) << 5) | (cc & 31)];   // (s << 20 | c << 4 | slot)
      if ((e >> 4) != (((unsigned)sidx << 16) | (unsigned)cc) || e == 0xFFFFFFFFu) return kCodeMiss;
      const int z = (int)(e & 15);
      const uint32_t* wp = win + (size_t)z * ck_slot_dw<R>() + (((bl & 1) * R + q) * BG_WAVE + r) * 2;
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
  auto reanchor = [&](int ka, int la) {
    k0 = ka; l0 = la;
    codes = decode_cell(k0 - (lane >> 3), l0 - (lane & 7));
  };
  u64 tJump = 0, tMiss = 0, nJump = 0, nMiss = 0;        // BG_FINISH_TIMING instrumentation
  const u64 tWalk0 = __builtin_readcyclecounter();
  for (;;) {
    int reqS = -1, reqB0 = 0, done = 0;
    if (wid == 0) {
      // the walk is one latency-bound wave: first claim on the issue slots it shares with the
      // next execute's DP waves (two-stream pipeline)
      __builtin_amdgcn_s_setprio(3);
      for (;;) {
        int dk = k0 - k, dl = l0 - l;
        if ((unsigned)dk >= 8u || (unsigned)dl >= 8u) { reanchor(k, l); dk = 0; dl = 0; }
        int c = rdlane(codes, dk * 8 + dl);
        if constexpr (!AFFINE) {
          // Linear gaps: inside the matrix x/y_trace are 'M', so states X/Y fall back to M
          // without moving and the walk is a chain of m_trace moves.  Resolve the chain through
          // the whole neighbourhood at once by pointer jumping (4 rounds of ds_bpermute over the
          // 64 cells); the border, STOP and window-miss cells stay with the scalar walker below.
          const bool jumpable = state == 0 && !(c & (kCodeMiss | kCodeBorder)) &&
                                (MODE != BGK_LOCAL || (c & 3) != 3);
          if (jumpable) {
            if ((dk | dl) != 0) { reanchor(k, l); c = rdlane(codes, 0); }
            const int cl = codes;
            const bool term = (cl & (kCodeMiss | kCodeBorder)) || (MODE == BGK_LOCAL && (cl & 3) == 3);
            const int mv = (int)(kLutM >> (4 * (cl & 15)) >> 2) & 3;   // 1 diag, 2 up, 3 left
            const int nk = (lane >> 3) + (mv != 3), nl = (lane & 7) + (mv != 2);
            const bool ex = !term && (nk >= 8 || nl >= 8);          // the move leaves the block
            int p = (term || ex) ? lane : nk * 8 + nl;
            int d = (term || ex) ? 0 : 1;
            int J[4];
            J[0] = p;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {                        // p <- p(p), d <- d + d(p)
              const int qv = __builtin_amdgcn_ds_bpermute(p * 4, p | (d << 8));
              p = qv & 255;
              d += qv >> 8;
              if (rr < 3) J[rr + 1] = p;
            }
            // lane m finds the m-th cell of the chain from the anchor, then its move
            int x = 0;
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) {
              const int y = __builtin_amdgcn_ds_bpermute(x * 4, J[bb]);
              x = ((lane >> bb) & 1) ? y : x;
            }
            const int opx = __builtin_amdgcn_ds_bpermute(x * 4, mv - 1);
            const int Pn = rdlane(p, 0), Dn = rdlane(d, 0);
            const int infoP = rdlane((ex ? 1 : 0) | (mv << 1), Pn);
            const int exP = infoP & 1, mvP = infoP >> 1;
            const int nops = Dn + exP;
            if (lane < nops) ob[cap - 1 - (ntail + ncore + lane)] = (uint8_t)opx;
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
          // Affine gaps: the same pointer jumping over (cell, state) nodes — 3 per lane, node id
          // state*64 + lane.  An X (Y) node whose x_trace (y_trace) is 'M' falls back to M
          // without moving (aligner.rs:566-585), so its next pointer is that cell's M node's.
          const bool jumpable = !(c & (kCodeMiss | kCodeBorder)) && (MODE != BGK_LOCAL || (c & 3) != 3);
          if (jumpable) {
            if ((dk | dl) != 0) { reanchor(k, l); }
            const int cl = codes;
            const bool term = (cl & (kCodeMiss | kCodeBorder)) || (MODE == BGK_LOCAL && (cl & 3) == 3);
            const int mvM = (int)(kLutM >> (4 * (cl & 15)) >> 2) & 3;   // 1 diag, 2 up, 3 left
            const int mvX = (cl & 4) ? mvM : 2;
            const int mvY = (cl & 8) ? mvM : 3;
            int P[3], D[3], OP[3], INFO[3];
#pragma unroll
            for (int st = 0; st < 3; ++st) {
              const int mv = st == 0 ? mvM : (st == 1 ? mvX : mvY);
              const int nk = (lane >> 3) + (mv != 3), nl = (lane & 7) + (mv != 2);
              const int ns = mv == 2 ? 1 : (mv == 3 ? 2 : 0);      // state after the move
              const bool ex = !term && (nk >= 8 || nl >= 8);
              const int self = st * 64 + lane;
              P[st] = (term || ex) ? self : ns * 64 + nk * 8 + nl;
              D[st] = (term || ex) ? 0 : 1;
              OP[st] = mv - 1;
              INFO[st] = (ex ? 1 : 0) | (mv << 1) | (ns << 3);
            }
            // node value lookup: value of node `node` from the lane holding it
            auto bperm3 = [&](const int (&v)[3], int node) {
              const int src = (node & 63) * 4;
              const int r0 = __builtin_amdgcn_ds_bpermute(src, v[0]);
              const int r1 = __builtin_amdgcn_ds_bpermute(src, v[1]);
              const int r2 = __builtin_amdgcn_ds_bpermute(src, v[2]);
              const int sl = node >> 6;
              return sl == 0 ? r0 : (sl == 1 ? r1 : r2);
            };
            int J[4][3];
#pragma unroll
            for (int st = 0; st < 3; ++st) J[0][st] = P[st];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {                        // p <- p(p), d <- d + d(p)
              int PK[3];
#pragma unroll
              for (int st = 0; st < 3; ++st) PK[st] = P[st] | (D[st] << 8);
#pragma unroll
              for (int st = 0; st < 3; ++st) {
                const int qv = bperm3(PK, P[st]);
                P[st] = qv & 255;
                D[st] += qv >> 8;
              }
              if (rr < 3) {
#pragma unroll
                for (int st = 0; st < 3; ++st) J[rr + 1][st] = P[st];
              }
            }
            const int entry = state * 64;                           // (anchor cell, state)
            int x = entry;
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) {
              const int y = bperm3(J[bb], x);
              x = ((lane >> bb) & 1) ? y : x;
            }
            const int opx = bperm3(OP, x);
            const int Pn = rdlane(state == 0 ? P[0] : (state == 1 ? P[1] : P[2]), 0);
            const int Dn = rdlane(state == 0 ? D[0] : (state == 1 ? D[1] : D[2]), 0);
            const int sP = Pn >> 6, lP = Pn & 63;
            const int infoP = rdlane(sP == 0 ? INFO[0] : (sP == 1 ? INFO[1] : INFO[2]), lP);
            const int exP = infoP & 1, mvP = (infoP >> 1) & 3, nsP = infoP >> 3;
            const int nops = Dn + exP;
            if (lane < nops) ob[cap - 1 - (ntail + ncore + lane)] = (uint8_t)opx;
            ncore += nops;
            k -= lP >> 3;
            l -= lP & 7;
            if (exP) {
              k -= (mvP != 3);
              l -= (mvP != 2);
              state = nsP;
            } else {
              state = sP;
            }
            continue;
          }
        }
        if (c & kCodeMiss) {
          const int vr = k - 1;
          reqS = vr / ROWS;
          const int bl = (l + (vr - reqS * ROWS) / R) >> 5;
          reqB0 = CK ? (bl >> 1) : (bl - NBW + 1 > 0 ? bl - NBW + 1 : 0);
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
        k -= (0x6 >> mv) & 1;
        l -= (0xA >> mv) & 1;
        state = e & 3;
        if (mv) {
          if (lane == 0) ob[cap - 1 - (ntail + ncore)] = (uint8_t)(mv - 1);
          ++ncore;
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (lane == 0) { sh[4] = reqS; sh[5] = reqB0; sh[6] = done; }
    }
    __syncthreads();
    done = sh[6];
    if (done) break;
    const u64 tm0 = __builtin_readcyclecounter();
    ++nMiss;
    reqS = uni(sh[4]);
    reqB0 = uni(sh[5]);
    if constexpr (CK) {
      // recompute the requested chunk and up to three chunks to its left (the walk heads up and
      // left), one per wave, into the oldest slots
      int list[4], nl = 0;
      for (int d = 0; d < 4; ++d) {
        const int cc = reqB0 - d;
        if (cc < 0) break;
        bool res = false;
#pragma unroll
        for (int z = 0; z < kCkSlots; ++z) res |= (ckS[z] == reqS && ckC[z] == cc);
        if (!res || d == 0) list[nl++] = cc;
      }
      const int myz = (ckNext + wid) % kCkSlots;
      if (wid < nl)
        recompute_chunk<R>(F, P, reqS, list[wid], win + (size_t)myz * ck_slot_dw<R>(),
                           ckArea + wid * ck_wave_ints<R>(), lane);
      for (int x = 0; x < nl; ++x) {
        const int z = (ckNext + x) % kCkSlots;
        int oldS = -1, oldC = -1;
#pragma unroll
        for (int zz = 0; zz < kCkSlots; ++zz)
          if (zz == z) { oldS = ckS[zz]; oldC = ckC[zz]; ckS[zz] = reqS; ckC[zz] = list[x]; }
        if (tid == 0) {
          if (oldS >= 0) {
            unsigned& oe = ckMap[((oldS & 31) << 5) | (oldC & 31)];
            if ((oe & 15) == (unsigned)z) oe = 0xFFFFFFFFu;
          }
          ckMap[((reqS & 31) << 5) | (list[x] & 31)] =
              ((unsigned)reqS << 20) | ((unsigned)list[x] << 4) | (unsigned)z;
        }
      }
      ckNext = (ckNext + nl) % kCkSlots;
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
  if (F.dbg && tid == 0) {
    u64* d = F.dbg + (size_t)P.index * 8;
    d[0] = __builtin_readcyclecounter() - tWalk0;
    d[1] = tJump; d[2] = nJump; d[3] = tMiss; d[4] = nMiss; d[5] = (u64)ncore;
  }

  // ---------------- semiglobal prefix gaps (:416-428); every wave knows k, l through sh
  if (wid == 0 && lane == 0) { sh[7] = k; sh[8] = l; sh[9] = status; sh[10] = ncore; }
  __syncthreads();
  const int kstop = sh[7], lstop = sh[8];
  status = sh[9];
  ncore = sh[10];
  int npre = 0;
  if (status == 0 && mode == BGK_SEMIGLOBAL) npre = colcase ? kstop : lstop;
  const int L = ntail + ncore + npre;
  const int base = cap - L;

  // ---------------- semiglobal prefix (:416-428) and tail columns: one residue run against gaps
  // each (prefix: s1[0, kstop) or s2[0, lstop); tail: s1[ei, n1) or s2[ej, n2))
  for (int x = tid; x < npre; x += NT) {
    ob[base + x] = colcase ? f.s1[x] : (uint8_t)'-';
    ob2[base + x] = colcase ? (uint8_t)'-' : f.s2[x];
  }
  for (int x = tid; x < ntail; x += NT) {
    ob[cap - ntail + x] = colcase ? f.s1[ei + x] : (uint8_t)'-';
    ob2[cap - ntail + x] = colcase ? (uint8_t)'-' : f.s2[ej + x];
  }

  // ---------------- expand the walk's op codes into both strings (parallel scan over columns)
  const int i0 = kstop, j0 = lstop;                    // first residues the core consumes
  const int cbase = base + npre;
  const int seg = (ncore + NT - 1) / NT;
  const int cend = cbase + ncore;
  const int lo = cbase + tid * seg < cend ? cbase + tid * seg : cend;
  const int hi = lo + seg < cend ? lo + seg : cend;
  int c1 = 0, c2 = 0;
  for (int x = lo; x < hi; ++x) { const int op = ob[x]; c1 += op != 2; c2 += op != 1; }
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
  for (int x = lo; x < hi; ++x) {
    const int op = ob[x];
    const uint8_t ch1 = op != 2 ? f.s1[p1++] : (uint8_t)'-';
    const uint8_t ch2 = op != 1 ? f.s2[p2++] : (uint8_t)'-';
    ob[x] = ch1;
    ob2[x] = ch2;
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
    F.results[P.index] = res;
  }
}

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
    if (o.status == 0 && bg_ref_fresh_divergent(E.mode, P.n1, P.n2, r.score)) o.status = 4;
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
// LDS of the checkpoint finish kernel: chunk slots, scalars + scan, 4 recompute areas
extern "C" size_t bg_finish_ck_lds_bytes(int R, int* win_bytes) {
  int slot = 0, area = 0, nslot = 8;
  switch (R) {
    case 2: slot = ck_slot_dw<2>(); area = ck_wave_ints<2>(); nslot = ck_slots<2>(); break;
    case 3: slot = ck_slot_dw<3>(); area = ck_wave_ints<3>(); nslot = ck_slots<3>(); break;
    case 4: slot = ck_slot_dw<4>(); area = ck_wave_ints<4>(); nslot = ck_slots<4>(); break;
    case 5: slot = ck_slot_dw<5>(); area = ck_wave_ints<5>(); nslot = ck_slots<5>(); break;
    case 8: slot = ck_slot_dw<8>(); area = ck_wave_ints<8>(); nslot = ck_slots<8>(); break;
    default: slot = ck_slot_dw<10>(); area = ck_wave_ints<10>(); nslot = ck_slots<10>(); break;
  }
  *win_bytes = nslot * slot * 4;
  return (size_t)*win_bytes + 64 * 4 + 2 * 256 * 4 + 4 * (size_t)area * 4 + 4 * 1024;  // + chunk map
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
extern "C" size_t bg_finish_lds_bytes(int win_bytes) { return (size_t)win_bytes + 64 * 4 + 2 * 256 * 4; }
