// Tagged linear-gap DP kernel: the metric path (semiglobal / global / fitting / overlap,
// a >= b, DNA-sized alphabets).  Replaces compute_scores_global (src/alignment/aligner.rs:437-469)
// for the case where the x/y gap matrices provably collapse onto M.
//
// Same strip geometry and trace layout as bg_dp_kernel (one workgroup per pair, W waves, strips
// of 64*R rows, lane r owns rows [rR, rR+R), anti-diagonal sweep with lane r at column t - r),
// but everything per step that is not cell arithmetic is moved off the VALU:
//
//   * values live in the frame M'(i,j) = M(i,j) - a*(i+j), where both gap candidates carry no
//     constant (M(i-1,j) + a and M(i,j-1) + a become M'(i-1,j) and M'(i,j-1)) and the diagonal
//     one adds S - 2a (folded into the profile).  They are kept as 4*M' + tag with tag 0 for the
//     diagonal form, 2 for the X form (from the row above) and 3 for the Y form (from the left),
//     so one v_max3 yields M' and the m_trace code with the reference's tie priority
//     Y > X > R (aligner.rs:455-463), the Y form of the result is `best | 3` and its X form
//     `(best | 3) - 1`;
//   * the column code is read by every lane from the pair's code row in LDS at (t - lane - 1)
//     with a compile-time immediate offset per step (ds_read_u16 of a pre-scaled code); it
//     selects the lane's R profile bytes S'(q_k, code) from a per-wave LDS table (one ds_read
//     per step) and each cell adds its byte with an SDWA operand select (v_add_u32_sdwa ...
//     sext src1_sel:BYTE_k), so the profile lookup costs no VALU op of its own;
//   * the row above of lane 0 (the boundary row of the strip above) is staged per 64-column
//     block in LDS and read as a broadcast per step, feeding the `old` operand of the one DPP
//     wave_shr:1 that moves each lane's last row down to the next lane;
//   * the boundary row this strip hands to the strip below is written by EVERY lane into an LDS
//     ring at slot (u + 64 - lane): position p = t - lane receives its final value from the
//     last lane that writes it — lane 63 (or the lane holding row n1 in the last strip; lanes
//     below it write to a dummy half of the ring) — and each finished 64-column block is
//     copied to HBM once per chunk.  No v_readlane / v_writelane in the loop.
//
// Per cell: v_add_sdwa (diagonal + profile byte), v_max3, v_alignbit (2-bit trace code), v_or,
// v_add.  Per step: one DPP, one v_add (profile address).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_dev_util.h"

using namespace bgk;

namespace {

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
  uint32_t* trace;          // this strip's trace
  int32_t* bndOut;          // this strip's boundary row (X forms), 64-column blocks
  int32_t* lastcol;         // M(i, n2)
  const int* bIn;           // LDS: staged boundary block of the strip above (64 X forms)
  int* ring;                // LDS: this wave's 256-slot output ring
  int* oLane;               // LDS: this lane's ring write base (slot = u + 64 - lane [+128])
  const uint16_t* codeLane; // LDS: scaled code row + t0 - lane - 1 (this chunk)
  const uint8_t* profLane;  // LDS: this lane's profile entries (+ scaled code = entry address)
};

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

enum { TV_FAST = 0, TV_SEL = 1, TV_EDGE = 2 };

// Y form of column 0, row i: 4*(M(i,0) - a*i) + 3 (aligner.rs:98-104 borders)
__device__ __forceinline__ int col0_Y(int mode, int i, int a, int b) {
  return 4 * wadd(col0_M(mode, i, a, b), -wmul(a, i)) + 3;
}

template <int R, int VAR>
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
        if (t >= C.n2 && t - C.n2 < BG_WAVE && C.n2 > 0) {    // column n2: M(i, n2)
          if (lane == t - C.n2) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
              const int i = C.rowbase + k + 1;
              if (i <= C.n1) C.lastcol[i] = wadd(S.Y[k] >> 2, wmul(a, i + C.n2));
            }
          }
        }
      }
      int out = S.Xlast;
      if constexpr (VAR != TV_FAST) {
#pragma unroll
        for (int k = 0; k < R - 1; ++k) out = (C.orow == k) ? S.Y[k] - 1 : out;
      }
      C.oLane[u] = out;
      // one step per scheduling region: hoisting later steps' profile lookups spills
      __builtin_amdgcn_sched_barrier(0);
    }
    if (h == 1 && c >= 1) {
      // block c-1 (ring slots 0-63) is final: copy it out, slide the ring by one block
      const int v = C.ring[lane];
      const int nx = C.ring[64 + lane];
      C.bndOut[(c - 1) * BG_CHUNK + lane] = v;
      C.ring[lane] = nx;
    } else if (h == 1) {
      C.ring[lane] = C.ring[64 + lane];
    }
    // trace flush every 32 steps: block b, row k, lane r -> dwords [((b*R + k)*64 + r)*2, +2)
    uint32_t* tb = C.trace + (size_t)((t0 >> 5) + h) * (R * 2 * BG_WAVE) + lane * 2;
#pragma unroll
    for (int k = 0; k < R; ++k)
      *reinterpret_cast<uint2*>(tb + k * 2 * BG_WAVE) = make_uint2(S.tA[k], S.tB[k]);
  }
}

}  // namespace

// LDS layout (bytes from the dynamic base, offsets from the host, bg_tag_lds_bytes()):
//   progress counters 64 B @prog_off | scaled code row @codes_off: u16, 64 zero entries, then
//   (NC + 2) * 64 entries (code * 256 * RW, zero past n2) | per wave @aux_lds_off: 64-int
//   boundary block, 256-int output ring, 4 codes x 64 lanes x RW-dword profile entries.
constexpr int kTagWaveInts = 64 + 256;
template <int R>
__global__ __launch_bounds__(1024) void bg_dp_tag_kernel(BgDpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  const int w = uni(threadIdx.x >> 6);
  constexpr int ROWS = BG_WAVE * R;

  constexpr int RW = ProfW<R>::v;
  if (threadIdx.x < 16) reinterpret_cast<int*>(smem + A.prog_off)[threadIdx.x] = 0;
  uint16_t* sCodes = reinterpret_cast<uint16_t*>(smem + A.codes_off) + 64;
  {
    const BgPair& Pp = A.pairs[blockIdx.x];
    const uint8_t* g = A.codes2 + Pp.off2;   // code * 8 (DNA path)
    const int n = (Pp.nc + 2) * BG_CHUNK;
    for (int x = (int)threadIdx.x - 64; x < n; x += blockDim.x)
      sCodes[x] = (x >= 0 && x < Pp.n2) ? (uint16_t)(g[x] * (32 * RW)) : (uint16_t)0;
  }
  __syncthreads();

  const BgPair P = A.pairs[blockIdx.x];
  const int n1 = P.n1, n2 = P.n2, nst = P.nstrips, NC = P.nc;
  if (nst == 0) return;
  const int a = A.open;
  const int b = A.ext;
  const int mode = A.mode;
  const size_t stripDw = (size_t)NC * (BG_CHUNK / BG_TRACE_BLK) * R * 2 * BG_WAVE;
  int* waveLds = reinterpret_cast<int*>(smem + A.aux_lds_off) + w * (kTagWaveInts + 4 * 64 * RW);
  int* profTab = waveLds + kTagWaveInts;

  TagCtx C;
  C.a = a; C.b = b; C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = lane;
  C.lastcol = A.aux + P.aux_off;
  C.bIn = waveLds;
  C.ring = waveLds + 64;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);

  TagStrip<R> S;
  const uint8_t* c1 = A.codes1 + P.off1;
  const int nblk = NC - 1;
  int* sProg = reinterpret_cast<int*>(smem + A.prog_off);
  for (int s = w, rho = 0; s < nst; s += W, ++rho) {
    C.rowbase = s * ROWS + lane * R;
    const bool lastStrip = (s == nst - 1);
    const int lastRow = n1 - 1 - s * ROWS;
    const int olane = lastStrip ? lastRow / R : BG_WAVE - 1;
    C.orow = lastStrip ? lastRow % R : R - 1;
    const bool selRow = C.orow != R - 1;
    C.oLane = C.ring + (lane <= olane ? 64 : 192) - lane;
    C.trace = A.trace + P.trace_off / 4 + (size_t)s * stripDw;
    C.bndOut = A.bndM + P.bnd_off + (size_t)s * NC * BG_CHUNK;
    int qk[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;
      qk[k] = c1[(i <= n1 ? i : n1) - 1];
    }
    int pk[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;
      const int q = (i <= n1) ? qk[k] : 0;
      pk[k] = A.profile[(k == 0 ? 64 : 128) + (q >> 3)];   // 4 codes x int8
      S.Y[k] = col0_Y(mode, i, a, b);
      S.tA[k] = 0; S.tB[k] = 0;
    }
    // this lane's profile entries: for code cd, dword wd holds rows 4wd..4wd+3
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
    S.topPrev = 0; S.Xlast = 2;
    for (int c = 0; c < NC; ++c) {
      // stage block c of the row above (X forms) for this wave
      const int jb = c * BG_CHUNK + lane;
      int bv;
      if (s == 0) {
        bv = 4 * wadd(row0_M(mode, jb, a, b), -wmul(a, jb)) + 2;   // X form of row 0
      } else {
        if (c < nblk) {
          const int need = ((s - 1) / W) * nblk + c + 1;
          const int pw = (s - 1) % W;
          while (__hip_atomic_load(sProg + pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
            __builtin_amdgcn_s_sleep(1);
        }
        bv = load_agent(A.bndM + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb);
      }
      waveLds[lane] = bv;
      C.codeLane = sCodes + c * BG_CHUNK - lane - 1;
      const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
      if (edge) tag_chunk<R, TV_EDGE>(S, C, c);
      else if (lastStrip && selRow) tag_chunk<R, TV_SEL>(S, C, c);
      else tag_chunk<R, TV_FAST>(S, C, c);
      // publish: the chunk ends with the block copy-out store and R trace stores; at vmcnt(R)
      // the copy-out has reached L2
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(R) : "memory");
      if (lane == 0)
        __hip_atomic_store(sProg + w, rho * nblk + (c < nblk ? c : nblk), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

template __global__ void bg_dp_tag_kernel<4>(BgDpArgs);
template __global__ void bg_dp_tag_kernel<5>(BgDpArgs);
template __global__ void bg_dp_tag_kernel<8>(BgDpArgs);
template __global__ void bg_dp_tag_kernel<10>(BgDpArgs);

extern "C" void* bg_dp_kernel_tag_ptr(int R) {
  switch (R) {
    case 4: return (void*)&bg_dp_tag_kernel<4>;
    case 5: return (void*)&bg_dp_tag_kernel<5>;
    case 8: return (void*)&bg_dp_tag_kernel<8>;
    case 10: return (void*)&bg_dp_tag_kernel<10>;
    default: return nullptr;
  }
}
