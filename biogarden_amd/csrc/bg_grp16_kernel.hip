// Score-only DP of short single-strip pairs, EIGHT pairs per wave: bg_grp_kernel.hip's four 16-lane
// DPP rows, each lane carrying two pairs of one reference in the 16-bit halves of its registers
// (150 bp reads against shared 10 kbp references; aligner.rs:351-435 per pair,
// the DP of :437-469).
//
// bg_grp_kernel.hip issues two VALU instructions per cell (v_add_u32_sdwa, v_max3_i32) and is
// VALU-bound.  Two cells per instruction: v_pk_add_u16 of the profile pair and two
// v_pk_max_i16 — three instructions per two cells — and the step's own instructions (row hand-off,
// profile address, row-0 input) serve twice the cells.  The frame values M'(i, j) = M(i, j) -
// a(i + j) must fit int16: the host takes this kernel only when a bound on every cell's value
// (borders, plus (max S - 2a) per diagonal step, plus a margin for the garbage cells before each
// lane's column 0) stays inside it (bg_host.cpp plan_grouped).
//   * group layout: grp[g] is the low-half pair of DPP row g, grp[4 + g] the high-half one; both
//     share the row's lanes, column schedule and row-0 input (one reference per group);
//   * profile entries: per lane and code R dwords, each the two pairs' int16 S - 2a of that row
//     (-128 for rows below a pair's n1: they repeat row n1, bg_tag_kernel.hip);
//   * each pair's last row leaves through a 16-bit ring of its own (ds_write_b16 /
//     ds_write_b16_d16_hi), the lane holding its row n1 the last writer, as in bg_grp_kernel.hip;
//   * checkpoints: the low halves' as a four-pair group's at the group's first trace area, the high
//     halves' at its second — so the traceback (bg_finish.h recompute_grp, GRP = 4) reads each pair
//     as a four-pair group's 16 lanes and needs no change.
#include <hip/hip_runtime.h>

#include "bg_device.h"
#include "bg_dev_util.h"
#include "bg_tag_common.h"

using namespace bgk;

namespace {

typedef short s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int pk_add(int x, int y) {
  return __builtin_bit_cast(int, __builtin_bit_cast(s2, x) + __builtin_bit_cast(s2, y));
}
__device__ __forceinline__ int pk_max(int x, int y) {
  return __builtin_bit_cast(int, __builtin_elementwise_max(__builtin_bit_cast(s2, x), __builtin_bit_cast(s2, y)));
}
__device__ __forceinline__ int pk2(int lo, int hi) { return (int)(((unsigned)lo & 0xffffu) | ((unsigned)hi << 16)); }
__device__ __forceinline__ int lo16(int v) { return (int)(short)(v & 0xffff); }
__device__ __forceinline__ int hi16(int v) { return v >> 16; }

// profile dwords per lane and code, padded to 16-byte loads
template <int R>
struct Pk16W { static constexpr int v = (R + 3) & ~3; };

template <int R>
__host__ __device__ constexpr int grp16_wave_ints() {
  // row-0 block (64), 8 rings of 128 int16 (512 ints), profile entries, the chunk's codes
  return 64 + 512 + 4 * 64 * Pk16W<R>::v + 96;
}

template <int R>
struct PkProf { int w[Pk16W<R>::v]; };

template <int R>
__device__ __forceinline__ PkProf<R> load_pk(const uint8_t* p) {
  PkProf<R> r;
#pragma unroll
  for (int q = 0; q < Pk16W<R>::v / 4; ++q) {
    const int4 v = *reinterpret_cast<const int4*>(p + 16 * q);
    r.w[4 * q] = v.x; r.w[4 * q + 1] = v.y; r.w[4 * q + 2] = v.z; r.w[4 * q + 3] = v.w;
  }
  return r;
}

__device__ __forceinline__ void fold_lastrow(u64& kb, int v, int j, int n1, int n2, int a) {
  const u64 kk = ((u64)key_bias(wadd(v, wmul(a, n1 + j))) << 32) | (unsigned)j;
  kb = (j >= 1 && j <= n2 && kk > kb) ? kk : kb;
}

struct Ctx16 {
  int a, b, mode, n2, lane, rowbase;
  int n1lo, n1hi;
  int32_t* lastLo;             // M(i, n2) of the low / high pair
  int32_t* lastHi;
  const int* bIn;              // row-0 block (packed, both halves equal)
  short* oLo;                  // this lane's ring write bases (slot = u + 64 - lane)
  short* oHi;
  const uint8_t* profLane;
  const uint16_t* codeLane;
  int top0, topStep;           // packed
};

template <int R>
struct Strip16 {
  int Y[R];                    // packed M' of rows k, both pairs
  int topPrev, Xlast;
};

template <int R, bool EDGE, bool TOP0>
__device__ __forceinline__ void grp16_chunk(Strip16<R>& S, Ctx16& C, int c, short* ring8, int32_t* const (&bnd)[8],
                                            const int (&n1g)[8], u64 (&kb)[8], bool fold, const int (&c0)[R],
                                            int lane) {
  const int a = C.a;
  const int t0 = c * BG_CHUNK;
  const int sl = C.lane;
  int Lc[R];
#pragma unroll
  for (int k = 0; k < R; ++k) Lc[k] = 0;
  int nTop = TOP0 ? C.top0 : C.bIn[0];
  int qTop = TOP0 ? 0 : C.bIn[0];
  PkProf<R> qP = load_pk<R>(C.profLane + C.codeLane[0]);
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
      const PkProf<R> P = qP;
      qP = load_pk<R>(C.profLane + qCode);
      qCode = cl[uu];
      if constexpr (!TOP0) qTop = bi[uu];
      const int topX = dpp_rowshr1(topIn, S.Xlast);          // both pairs' row above; first lanes: row 0
      if constexpr (TOP0) nTop = pk_add(topX, C.topStep);
      int dIn = S.topPrev;
      int xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int yo = S.Y[k];
        const int d = pk_add(dIn, P.w[k]);                     // M'(i-1,j-1) + S - 2a, both pairs
        const int best = pk_max(pk_max(d, yo), xo);            // the chain only through xo
        dIn = yo;
        xo = best;
        S.Y[k] = best;
      }
      S.topPrev = topX;
      S.Xlast = xo;
      if constexpr (EDGE) {
        if (c == 0) {                                          // column 0 (aligner.rs:98-104)
          const bool rst = (t == sl);
#pragma unroll
          for (int k = 0; k < R; ++k) S.Y[k] = rst ? c0[k] : S.Y[k];
          S.Xlast = rst ? S.Y[R - 1] : S.Xlast;
        }
        if (t >= C.n2 && t - C.n2 < BG_WAVE && C.n2 > 0) {     // column n2 (wave-uniform)
          const bool sel = sl == t - C.n2;
#pragma unroll
          for (int k = 0; k < R; ++k) Lc[k] = sel ? S.Y[k] : Lc[k];
        }
      }
      C.oLo[u] = (short)S.Xlast;
      C.oHi[u] = (short)(S.Xlast >> 16);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (h == 1) {
      // block c - 1 (ring slots 0-63) is final in every ring: to each pair's boundary row (and
      // end-cell key), then the rings slide by one block
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        short* rg = ring8 + g * 128;
        const int v = rg[lane];
        const short nx = rg[64 + lane];
        const int j = (c - 1) * BG_CHUNK + lane;
        if (c >= 1 && bnd[g]) bnd[g][j] = v;
        if (c >= 1 && fold) fold_lastrow(kb[g], v, j, n1g[g], C.n2, a);
        rg[lane] = nx;
      }
    }
  }
  if constexpr (EDGE) {
    const int tl = C.n2 + sl;                                  // the step this lane was at column n2
    if (C.n2 > 0 && tl >= t0 && tl < t0 + BG_CHUNK) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int i = C.rowbase + k + 1;
        if (i <= C.n1lo) C.lastLo[i] = wadd(lo16(Lc[k]), wmul(a, i + C.n2));
        if (i <= C.n1hi) C.lastHi[i] = wadd(hi16(Lc[k]), wmul(a, i + C.n2));
      }
    }
  }
}

}  // namespace

template <int R>
__global__ __launch_bounds__(256) void bg_dp_grp16_kernel(BgDpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int PW = Pk16W<R>::v;
  const int lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  const int w = uni(threadIdx.x >> 6);
  const int g = lane >> 4, sl = lane & 15;
  const int wv = blockIdx.x * W + w;                          // the wave's group of eight pairs
  if (wv >= A.ngroups) return;
  if (A.prio) __builtin_amdgcn_s_setprio(1);
  const int* grp = A.grp + 8 * wv;
  const int p0 = grp[0];                                      // every group has its first pair
  const int plo = grp[g] >= 0 ? grp[g] : p0;                  // this lane's two pairs
  const int phi = grp[4 + g] >= 0 ? grp[4 + g] : p0;
  const bool realLo = grp[g] >= 0, realHi = grp[4 + g] >= 0;
  const BgPair P0 = A.pairs[p0];
  const BgPair& PL = A.pairs[plo];
  const BgPair& PH = A.pairs[phi];
  const int n1lo = PL.n1, n1hi = PH.n1, n2 = P0.n2, NC = P0.nc;
  const int a = A.open, b = A.ext, mode = A.mode;
  int* waveLds = reinterpret_cast<int*>(smem + A.aux_lds_off) + w * grp16_wave_ints<R>();
  int* bIn = waveLds;
  short* ring8 = reinterpret_cast<short*>(waveLds + 64);
  int* profTab = waveLds + 64 + 512;
  uint16_t* stage = reinterpret_cast<uint16_t*>(profTab + 4 * 64 * PW);
  short* dummyRing = reinterpret_cast<short*>(smem + A.prog_off);   // 128 int16, shared garbage

  Ctx16 C;
  C.a = a; C.b = b; C.mode = mode; C.n2 = n2; C.lane = sl;
  C.rowbase = sl * R;
  C.n1lo = realLo ? n1lo : 0;                                 // a padding half writes nothing
  C.n1hi = realHi ? n1hi : 0;
  C.lastLo = A.aux + PL.aux_off;
  C.lastHi = A.aux + PH.aux_off;
  C.bIn = bIn;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * PW);
  C.codeLane = stage + 63 - sl;
  const int olo = (n1lo - 1) / R, ohi = (n1hi - 1) / R;
  C.oLo = ((sl <= olo && realLo) ? ring8 + g * 128 : dummyRing) + 64 - sl;
  C.oHi = ((sl <= ohi && realHi) ? ring8 + (4 + g) * 128 : dummyRing) + 64 - sl;
  int32_t* bnd[8];
  int n1g[8];
  u64 kb[8];
  const bool fold = A.keys != nullptr;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    kb[x] = 0;
    const int px = grp[x];
    bnd[x] = px >= 0 ? A.bndM + A.pairs[px].bnd_off : nullptr;
    n1g[x] = px >= 0 ? A.pairs[px].n1 : 0;
  }

  const uint8_t* cLo = A.codes1 + PL.off1;
  const uint8_t* cHi = A.codes1 + PH.off1;
  const uint8_t* g2 = A.codes2 + P0.off2;                     // code * 8, shared by the group
  int pkl[R], pkh[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    pkl[k] = i > n1lo ? (int)0x80808080 : A.profile[192 + (cLo[i - 1] >> 3)];   // 4 codes x int8 S - 2a
    pkh[k] = i > n1hi ? (int)0x80808080 : A.profile[192 + (cHi[i - 1] >> 3)];
  }
#pragma unroll
  for (int cd = 0; cd < 4; ++cd)
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      int v = 0;
      if (k < R) v = pk2((int)(int8_t)(pkl[k] >> (8 * cd)), (int)(int8_t)(pkh[k] >> (8 * cd)));
      profTab[(cd * 64 + lane) * PW + k] = v;
    }
  Strip16<R> S;
  int c0[R];                                                  // column 0: M'(i, 0), both pairs
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = C.rowbase + k + 1;
    const int il = i > n1lo ? n1lo : i, ih = i > n1hi ? n1hi : i;   // rows below n1 repeat row n1
    c0[k] = pk2(wadd(col0_M(mode, il, a, b), -wmul(a, il)), wadd(col0_M(mode, ih, a, b), -wmul(a, ih)));
    S.Y[k] = c0[k];
  }
  S.topPrev = 0;
  S.Xlast = 0;
  // checkpoints: low halves at the group's first trace area, high halves at its second (each the
  // layout of a four-pair group: [chunk][R + 1][64 lanes])
  int32_t* ckLo = reinterpret_cast<int32_t*>(A.trace + P0.trace_off / 4) + lane;
  int32_t* ckHi = ckLo + (size_t)NC * (R + 1) * BG_WAVE;
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
  const int ts = flat ? -a : b - a;
  C.topStep = pk2(ts, ts);
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? cv[q] * (32 * PW) : 0);
    }
    fetch_codes(c + 1 < NC ? c + 1 : c);
    const int jb = c * BG_CHUNK + lane;
    const int r0 = wadd(row0_M(mode, jb, a, b), -wmul(a, jb));
    bIn[lane] = pk2(r0, r0);                                  // M'(0, j), the edge chunks' input
    int32_t* kl = ckLo + (size_t)c * (R + 1) * BG_WAVE;
    int32_t* kh = ckHi + (size_t)c * (R + 1) * BG_WAVE;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      kl[k * BG_WAVE] = lo16(S.Y[k]);
      kh[k * BG_WAVE] = hi16(S.Y[k]);
    }
    kl[R * BG_WAVE] = lo16(S.topPrev);
    kh[R * BG_WAVE] = hi16(S.topPrev);
    const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
    if (edge) {
      grp16_chunk<R, true, false>(S, C, c, ring8, bnd, n1g, kb, fold, c0, lane);
    } else {
      const int t0v = wadd(row0_M(mode, c * BG_CHUNK, a, b), -wmul(a, c * BG_CHUNK));
      C.top0 = pk2(t0v, t0v);
      grp16_chunk<R, false, true>(S, C, c, ring8, bnd, n1g, kb, fold, c0, lane);
    }
  }
  if (fold) {
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const u64 k = wave_umax64(kb[x]);
      if (lane == 0 && grp[x] >= 0) A.keys[2 * (size_t)grp[x] + 1] = k;
    }
  }
}

template __global__ void bg_dp_grp16_kernel<2>(BgDpArgs);
template __global__ void bg_dp_grp16_kernel<3>(BgDpArgs);
template __global__ void bg_dp_grp16_kernel<4>(BgDpArgs);
template __global__ void bg_dp_grp16_kernel<5>(BgDpArgs);
template __global__ void bg_dp_grp16_kernel<8>(BgDpArgs);
template __global__ void bg_dp_grp16_kernel<10>(BgDpArgs);

extern "C" void* bg_dp_grp16_kernel_ptr(int R) {
  switch (R) {
    case 2: return (void*)&bg_dp_grp16_kernel<2>;
    case 3: return (void*)&bg_dp_grp16_kernel<3>;
    case 4: return (void*)&bg_dp_grp16_kernel<4>;
    case 5: return (void*)&bg_dp_grp16_kernel<5>;
    case 8: return (void*)&bg_dp_grp16_kernel<8>;
    case 10: return (void*)&bg_dp_grp16_kernel<10>;
    default: return nullptr;
  }
}

extern "C" int bg_dp_grp16_wave_lds_bytes(int R) {
  switch (R) {
    case 2: return grp16_wave_ints<2>() * 4;
    case 3: return grp16_wave_ints<3>() * 4;
    case 4: return grp16_wave_ints<4>() * 4;
    case 5: return grp16_wave_ints<5>() * 4;
    case 8: return grp16_wave_ints<8>() * 4;
    default: return grp16_wave_ints<10>() * 4;
  }
}
