// Score-only DP of short single-strip pairs, GP = 4 or 2 pairs per wave (150 bp
// reads against shared 10 kbp references; aligner.rs:351-435 per pair, the DP of :437-469).
//
// The checkpoint kernel (bg_tag_kernel.hip) gives every pair one wave of 64 lanes x R rows; a
// 150-row read at R = 3 leaves 42 of 192 row slots idle and pays the step's per-lane overhead
// (row hand-off, profile address, the code) for three rows.  Here a wave holds GP pairs of
// L = 64 / GP lanes each, at R rows per lane with L R >= n1 (150 bp: GP = 4 at R = 10, 600 of 640
// row slots used; GP = 2 at R = 5, 300 of 320):
//   * the rows hand down lane to lane, and each pair's first lane takes row 0 instead (GP = 4:
//     row_shr:1, whose first lane of every 16-lane row keeps the DPP's old operand; GP = 2:
//     wave_shr:1 and a select at lane 32) — the same for every pair: one mode, one gap pair, one
//     column schedule (lane l computes column t - (l mod L));
//   * the pairs share seq2 (the host groups reads by reference), so one code stage serves them;
//     each lane's profile entries are built from its own pair's rows;
//   * each pair's last row n1 leaves through a ring of its own: the rows below n1 repeat row n1
//     (profile bytes -128, row n1's column-0 value; M'(i, j) >= M'(i, j - 1) in the frame), so the
//     lane holding row n1 is the last writer of its row's ring, and the ring goes to the pair's
//     boundary row at each block — the end cell's last row (aligner.rs:369-389) — and, semiglobal
//     and overlap, into the pair's running end-cell key;
//   * the checkpoints are the tagged kernel's, per wave: [chunk][k][64 lanes], the pair's L lanes
//     at BgPair::lane0; the traceback recomputes a pair's chunks as L-lane jobs (bg_finish.h).
// GP = 4 packs the most rows per step and runs reads up to 160 rows; GP = 2 takes reads up to 320
// (the DP is VALU-bound: C4 at GP = 4 issues 513 M VALU instructions, 72 % of the SIMDs' issue
// over the kernel, against 674 M at GP = 2 — twice the waves do not pay for them).
// Values are the frame M'(i, j) = M(i, j) - a(i + j) of bg_tag_common.h's score_chunk.
#include <hip/hip_runtime.h>

#include "bg_device.h"
#include "bg_dev_util.h"
#include "bg_tag_common.h"

using namespace bgk;

namespace {

constexpr int kGrpStageU16 = 192;

// per wave: row-0 block (64), P rings (P x 128), profile entries (4 codes x 64 lanes x RW), the
// chunk's codes (192 u16)
template <int R, int P>
__host__ __device__ constexpr int grp_wave_ints() {
  return 64 + P * 128 + 4 * 64 * ProfW<R>::v + kGrpStageU16 / 2;
}

// fold of the last row's end-cell key (aligner.rs:308, :369 — the last maximum of row n1, as the
// finish kernel's fold): (biased M(n1, j) << 32 | j), one running maximum per pair and lane
__device__ __forceinline__ void fold_lastrow(u64& kb, int v, int j, int n1, int n2, int a) {
  const u64 kk = ((u64)key_bias(wadd(v, wmul(a, n1 + j))) << 32) | (unsigned)j;
  kb = (j >= 1 && j <= n2 && kk > kb) ? kk : kb;
}

// score_chunk (bg_tag_common.h) with GP pairs' hand-offs (grp_shr1) and GP output rings
template <int R, int GP, bool EDGE, bool TOP0>
__device__ __forceinline__ void grp_chunk(TagStrip<R>& S, TagCtx& C, int c, int* ring4, int32_t* const (&bnd)[GP],
                                          const int (&n1g)[GP], u64 (&kb)[GP], bool fold, int lane) {
  const int a = C.a;
  const int t0 = c * BG_CHUNK;
  const int sl = C.lane;                                      // the pair's lane (0 .. 64 / GP - 1)
  const bool first = sl == 0;
  constexpr int RW = ProfW<R>::v;
  int Lc[R] = {};
  int nTop = TOP0 ? C.top0 : C.bIn[0];
  int qTop = TOP0 ? 0 : C.bIn[0];
  ProfV<RW> qP = load_prof<RW>(C.profLane + C.codeLane[0]);
  int qCode = C.codeLane[1];
  const uint16_t* cl = C.codeLane + 2;
  const int* bi = C.bIn + 1;
#pragma unroll
  for (int h = 0; h < BG_CHUNK / BG_TRACE_BLK; ++h, cl += BG_TRACE_BLK, bi += BG_TRACE_BLK) {
#pragma unroll
    for (int uu = 0; uu < BG_TRACE_BLK; ++uu) {
      const int u = h * BG_TRACE_BLK + uu;
      const int t = t0 + u;
      const int topIn = TOP0 ? nTop : qTop;
      const ProfV<RW> P = qP;
      qP = load_prof<RW>(C.profLane + qCode);
      qCode = cl[uu];
      if constexpr (!TOP0) qTop = bi[uu];
      const int topX = grp_shr1<GP>(topIn, S.Xlast, first);    // M'(row above, j); first lanes: row 0
      if constexpr (TOP0) nTop = topX + C.topStep;
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
      if constexpr (EDGE) {
        if (c == 0) {                                         // column 0 (aligner.rs:98-104)
          const bool rst = (t == sl);
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int i = C.rowbase + k + 1;
            const int ii = i > C.n1 ? C.n1 : i;               // rows below n1 repeat row n1
            S.Y[k] = rst ? wadd(col0_M(C.mode, ii, a, C.b), -wmul(a, ii)) : S.Y[k];
          }
          S.Xlast = rst ? S.Y[R - 1] : S.Xlast;
        }
        catch_lastcol<R>(S.Y, Lc, t, C.n2, sl);              // column n2: M(i, n2)
      }
      C.oLane[u] = S.Xlast;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (h == 1) {
      // block c - 1 (ring slots 0-63) is final in every ring: to each pair's boundary row, then
      // slide the rings by one block
#pragma unroll
      for (int g = 0; g < GP; ++g) {
        int* rg = ring4 + g * 128;
        const int v = rg[lane];
        const int nx = rg[64 + lane];
        if (c >= 1 && bnd[g]) bnd[g][(c - 1) * BG_CHUNK + lane] = v;
        if (fold) fold_lastrow(kb[g], v, (c - 1) * BG_CHUNK + lane, n1g[g], C.n2, a);
        rg[lane] = nx;
      }
    }
  }
  if constexpr (EDGE) store_lastcol<R>(Lc, C, t0);
}

}  // namespace

template <int R, int GP>
__global__ __launch_bounds__(1024) void bg_dp_grp_kernel(BgDpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int RW = ProfW<R>::v;
  constexpr int L = 64 / GP;                                   // lanes per pair
  const int lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  const int w = uni(threadIdx.x >> 6);
  const int g = lane / L, sl = lane % L;
  const int wv = blockIdx.x * W + w;                          // the wave's group of GP pairs
  if (wv >= A.ngroups) return;
  const int* grp = A.grp + GP * wv;
  const int p0 = grp[0];                                      // every group has its first pair
  const int pl = grp[g] >= 0 ? grp[g] : p0;                   // this lane's pair
  const BgPair P0 = A.pairs[p0];
  const BgPair& P = A.pairs[pl];
  const int n1 = P.n1, n2 = P0.n2, NC = P0.nc;
  const int a = A.open, b = A.ext, mode = A.mode;
  int* waveLds = reinterpret_cast<int*>(smem + A.aux_lds_off) + w * grp_wave_ints<R, GP>();
  int* bIn = waveLds;
  int* ring4 = waveLds + 64;
  int* profTab = ring4 + GP * 128;
  uint16_t* stage = reinterpret_cast<uint16_t*>(profTab + 4 * 64 * RW);
  int* dummyRing = reinterpret_cast<int*>(smem + A.prog_off);  // 128 ints, shared garbage

  TagCtx C;
  C.a = a; C.b = b; C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = sl;
  C.rowbase = sl * R;
  C.lastcol = A.aux + P.aux_off;
  C.bIn = bIn;
  C.mail = nullptr;
  C.ring = ring4;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);
  C.codeLane = stage + 63 - sl;                               // (t - sl - 1) - (t0 - 64)
  // row n1 sits in lane olane: lanes up to it write their row's ring (olane last), the lanes
  // below n1 a shared dummy ring
  const int olane = (n1 - 1) / R;
  const bool real = grp[g] >= 0;
  C.oLane = ((sl <= olane && real) ? ring4 + g * 128 : dummyRing) + 64 - sl;
  int32_t* bnd[GP];
  int n1g[GP];
  u64 kb[GP];
  const bool fold = A.keys != nullptr;
#pragma unroll
  for (int x = 0; x < GP; ++x) {
    kb[x] = 0;
    const int px = grp[x];
    bnd[x] = px >= 0 ? A.bndM + A.pairs[px].bnd_off : nullptr;   // nstrips = 1: the last row
    n1g[x] = px >= 0 ? A.pairs[px].n1 : 0;
  }

  const uint8_t* c1 = A.codes1 + P.off1;
  const uint8_t* g2 = A.codes2 + P0.off2;                     // code * 8, shared by the group
  int pk[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    const int q = i <= n1 ? c1[i - 1] : 0;
    pk[k] = i > n1 ? (int)0x80808080 : A.profile[192 + (q >> 3)];   // 4 codes x int8 S - 2a
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
  TagStrip<R> S;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    const int ii = i > n1 ? n1 : i;
    S.Y[k] = wadd(col0_M(mode, ii, a, b), -wmul(a, ii));
  }
  S.topPrev = 0;
  S.Xlast = 0;
  if (!real) C.n1 = 0;                                        // a padding row writes nothing
  // checkpoints of the group: [chunk][k][64 lanes] from the first pair's trace_off
  int32_t* ckBase = reinterpret_cast<int32_t*>(A.trace + P0.trace_off / 4) + lane;
  int cv[3];
  auto fetch_codes = [&](int c) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      cv[q] = g2[x < 0 ? 0 : (x >= n2 ? n2 - 1 : x)];
    }
  };
  fetch_codes(0);
  const bool flat = mode == BGK_SEMIGLOBAL || mode == BGK_LOCAL || mode == BGK_OVERLAP;
  C.topStep = flat ? -a : b - a;
  for (int c = 0; c < NC; ++c) {
    // this chunk's codes into the stage (scaled to profile-entry offsets), the next ones in flight
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? cv[q] * (32 * RW) : 0);
    }
    fetch_codes(c + 1 < NC ? c + 1 : c);
    const int jb = c * BG_CHUNK + lane;
    bIn[lane] = wadd(row0_M(mode, jb, a, b), -wmul(a, jb));  // M'(0, j), the edge chunks' input
    int32_t* ck = ckBase + (size_t)c * (R + 1) * BG_WAVE;
#pragma unroll
    for (int k = 0; k < R; ++k) ck[k * BG_WAVE] = S.Y[k];
    ck[R * BG_WAVE] = S.topPrev;
    const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
    if (edge) {
      grp_chunk<R, GP, true, false>(S, C, c, ring4, bnd, n1g, kb, fold, lane);
    } else {
      C.top0 = wadd(row0_M(mode, c * BG_CHUNK, a, b), -wmul(a, c * BG_CHUNK));
      grp_chunk<R, GP, false, true>(S, C, c, ring4, bnd, n1g, kb, fold, lane);
    }
  }
  if (fold) {
#pragma unroll
    for (int x = 0; x < GP; ++x) {
      const u64 k = wave_umax64(kb[x]);
      if (lane == 0 && grp[x] >= 0) A.keys[2 * (size_t)grp[x] + 1] = k;
    }
  }
}

#define BG_GRP_INST(RR)                                              \
  template __global__ void bg_dp_grp_kernel<RR, 4>(BgDpArgs);        \
  template __global__ void bg_dp_grp_kernel<RR, 2>(BgDpArgs);
BG_GRP_INST(2)
BG_GRP_INST(3)
BG_GRP_INST(4)
BG_GRP_INST(5)
BG_GRP_INST(8)
BG_GRP_INST(10)

template <int P>
static void* grp_ptr(int R) {
  switch (R) {
    case 2: return (void*)&bg_dp_grp_kernel<2, P>;
    case 3: return (void*)&bg_dp_grp_kernel<3, P>;
    case 4: return (void*)&bg_dp_grp_kernel<4, P>;
    case 5: return (void*)&bg_dp_grp_kernel<5, P>;
    case 8: return (void*)&bg_dp_grp_kernel<8, P>;
    case 10: return (void*)&bg_dp_grp_kernel<10, P>;
    default: return nullptr;
  }
}
// P pairs per wave: 4 (16 lanes each) or 2 (32 lanes)
extern "C" void* bg_dp_grp_kernel_ptr(int R, int P) { return P == 2 ? grp_ptr<2>(R) : P == 4 ? grp_ptr<4>(R) : nullptr; }

template <int P>
static int grp_bytes(int R) {
  switch (R) {
    case 2: return grp_wave_ints<2, P>() * 4;
    case 3: return grp_wave_ints<3, P>() * 4;
    case 4: return grp_wave_ints<4, P>() * 4;
    case 5: return grp_wave_ints<5, P>() * 4;
    case 8: return grp_wave_ints<8, P>() * 4;
    default: return grp_wave_ints<10, P>() * 4;
  }
}
extern "C" int bg_dp_grp_wave_lds_bytes(int R, int P) { return P == 2 ? grp_bytes<2>(R) : grp_bytes<4>(R); }
