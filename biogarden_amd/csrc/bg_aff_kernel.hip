// Score-only affine / local DP kernel: every case the linear tagged kernel does not take —
// affine gaps (a < b), local mode, alphabets of more than four symbols.  Replaces
// compute_scores_global (src/alignment/aligner.rs:437-469) and compute_scores_local (:471-509);
// the step and the value frames are in bg_aff_common.h.
//
// Same workgroup organisation as bg_dp_tag_kernel: one workgroup of W waves per pair, strip s on
// wave s mod W, per-wave progress counters in LDS, boundary blocks handed between the waves of a
// workgroup through LDS mailboxes (HBM only for round wraps and the last strip), per-chunk
// staging of the column codes.  The boundary rows carry (M, X) pairs: the strip below needs the
// vertical gap state as well as M.  Every strip's rows also go to HBM (the recomputation's top
// input), and at each chunk start the lanes store their checkpoints.
//
// Local mode also keeps, per row, the running maximum of M and the chunk in which it last
// increased (aux: rowbest[i-1], rowpos[i-1]); the traceback kernel finds the reference's end cell
// (the first row-major maximum, aligner.rs:173-176) from them and recomputes that one chunk to
// find its column.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_aff_common.h"
#include "bg_dev_util.h"

using namespace bgk;

// LDS layout (bytes from the dynamic base; sized by bg_dp_aff_lds_bytes):
//   @prog_off: 16 produced + 16 consumed counters, a 128-entry int2 dummy ring (1152 B)
//   @aux_lds_off, per wave: 64-entry int2 boundary block, 128-entry int2 output ring, K codes x
//   64 lanes x RW-dword profile entries, 192 u16 scaled codes of the current chunk (columns
//   t0-64 .. t0+127), 4 x 64-entry int2 mailbox
constexpr int kAffMailSlots = 4;
constexpr int kAffHeadInts = 32 + 256;

template <int R>
__host__ __device__ constexpr int aff_wave_ints(int K) {
  return 128 + 256 + K * 64 * AffW<R>::v + 96 + kAffMailSlots * 128;
}

template <int R, bool LOCAL>
__global__ __launch_bounds__(1024) void bg_dp_aff_kernel(BgDpArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int RW = AffW<R>::v;
  const int lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  const int w = uni(threadIdx.x >> 6);
  constexpr int ROWS = BG_WAVE * R;
  const int K = A.kdim;
  const int waveInts = aff_wave_ints<R>(K);

  int* sProg = reinterpret_cast<int*>(smem + A.prog_off);   // blocks produced (per wave)
  int* sCons = sProg + 16;                                   // chunks consumed (per wave)
  int2* dummyRing = reinterpret_cast<int2*>(sProg + 32);     // 128 entries, shared garbage
  if (threadIdx.x < 32) sProg[threadIdx.x] = 0;
  __syncthreads();

  const BgPair P = A.pairs[blockIdx.x];
  const int n1 = P.n1, n2 = P.n2, nst = P.nstrips, NC = P.nc;
  if (nst == 0) return;
  const int a = A.open;
  const int b = A.ext;
  const int mode = A.mode;
  int* waveLds = reinterpret_cast<int*>(smem + A.aux_lds_off) + w * waveInts;
  int2* bBlk = reinterpret_cast<int2*>(waveLds);
  int2* ring = reinterpret_cast<int2*>(waveLds + 128);
  int* profTab = waveLds + 384;
  uint16_t* stage = reinterpret_cast<uint16_t*>(profTab + K * 64 * RW);
  int2* mailbox = reinterpret_cast<int2*>(profTab + K * 64 * RW + 96);
  const int prevW = (w + W - 1) % W;
  int2* prevMail = reinterpret_cast<int2*>(reinterpret_cast<int*>(smem + A.aux_lds_off) +
                                           prevW * waveInts + 384 + K * 64 * RW + 96);
  const int codeScale = 256 * RW;       // byte offset of code cd's entries: cd * 64 lanes * RW * 4

  AffCtx C;
  C.a = a; C.b = b; C.e = wadd(b, -a); C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = lane;
  C.lastcol = A.aux + P.aux_off;
  C.bIn = bBlk;
  C.mail = nullptr;
  C.ring = ring;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);
  C.codeLane = stage + 63 - lane;       // (t - lane - 1) - (t0 - 64) = u + 63 - lane

  const uint8_t* c1 = A.codes1 + P.off1;
  const uint8_t* g2 = A.codes2 + P.off2;
  const int16_t* tab = reinterpret_cast<const int16_t*>(A.profile);   // [q * pstride + cd]
  auto fetch_codes = [&](int c, int (&v)[3]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      v[q] = g2[x < 0 ? 0 : (x >= n2 ? n2 - 1 : x)];
    }
  };
  auto stage_codes = [&](int c, const int (&v)[3]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? v[q] * codeScale : 0);
    }
  };

  AffStrip<R, LOCAL> S;
  const int nblk = NC - 1;
  for (int s = w, rho = 0; s < nst; s += W, ++rho) {
    C.rowbase = s * ROWS + lane * R;
    const bool lastStrip = (s == nst - 1);
    const int lastRow = n1 - 1 - s * ROWS;
    const int olane = lastStrip ? lastRow / R : BG_WAVE - 1;
    C.orow = lastStrip ? lastRow % R : R - 1;
    const bool selRow = C.orow != R - 1;
    C.oLane = (lane <= olane ? ring : dummyRing) + 64 - lane;
    C.bndOutM = A.bndM + P.bnd_off + (size_t)s * NC * BG_CHUNK;
    C.bndOutX = A.bndX + P.bnd_off + (size_t)s * NC * BG_CHUNK;
    const bool mailOut = (s + 1 < nst) && (w + 1 < W);
    const bool mailIn = (s > 0) && (w > 0);
    int qk[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;
      qk[k] = (i <= n1) ? c1[i - 1] : 0;
    }
    // this lane's profile entries: for code cd, dword wd holds rows 4wd..4wd+3
    for (int cd = 0; cd < K; ++cd) {
#pragma unroll
      for (int wd = 0; wd < RW; ++wd) {
        unsigned v = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
          if (wd * 4 + bb < R) v |= ((unsigned)tab[qk[wd * 4 + bb] * A.pstride + cd] & 0xffu) << (8 * bb);
        profTab[(cd * 64 + lane) * RW + wd] = (int)v;
      }
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int i = C.rowbase + k + 1;
      S.M[k] = aff_col0<LOCAL>(mode, i, a, b);
      S.Y[k] = kAffNeg;
      if constexpr (LOCAL) { S.best[k] = 0; S.bc[k] = 0; }
    }
    S.topPrev = 0;
    S.Xlast = kAffNeg;
    int32_t* ckBase = reinterpret_cast<int32_t*>(A.trace + P.trace_off / 4) +
                      (size_t)s * NC * (2 * R + 2) * BG_WAVE + lane;
    int cv[3];
    fetch_codes(0, cv);
    for (int c = 0; c < NC; ++c) {
      stage_codes(c, cv);
      fetch_codes(c + 1 < NC ? c + 1 : c, cv);
      // the row above, block c: row 0, the producer's LDS mailbox, or HBM
      const int seq = rho * NC + c;
      const int jb = c * BG_CHUNK + lane;
      if (s == 0) {
        bBlk[lane] = make_int2(aff_row0<LOCAL>(mode, jb, a, b), kAffNeg);
        C.bIn = bBlk;
      } else {
        if (c < nblk) {
          const int need = ((s - 1) / W) * nblk + c + 1;
          const int pw = (s - 1) % W;
          int np = 0;
          while (__hip_atomic_load(sProg + pw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
            poll_backoff(np);
        }
        if (mailIn) {
          C.bIn = prevMail + (seq % kAffMailSlots) * 64;
        } else {
          const size_t o = P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb;
          bBlk[lane] = make_int2(load_agent(A.bndM + o), load_agent(A.bndX + o));
          C.bIn = bBlk;
        }
      }
      C.mail = nullptr;
      if (mailOut && c >= 1 && c - 1 < nblk) {
        const int needC = seq - kAffMailSlots;
        int np = 0;
        while (__hip_atomic_load(sCons + w + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < needC)
          poll_backoff(np);
        C.mail = mailbox + ((seq - 1) % kAffMailSlots) * 64;
      }
      // checkpoint: the lane's state before this chunk
      {
        int32_t* ck = ckBase + (size_t)c * (2 * R + 2) * BG_WAVE;
#pragma unroll
        for (int k = 0; k < R; ++k) { ck[k * BG_WAVE] = S.M[k]; ck[(R + k) * BG_WAVE] = S.Y[k]; }
        ck[2 * R * BG_WAVE] = S.topPrev;
        ck[(2 * R + 1) * BG_WAVE] = S.Xlast;
      }
      int b0[LOCAL ? R : 1];
      if constexpr (LOCAL) {
#pragma unroll
        for (int k = 0; k < R; ++k) b0[k] = S.best[k];
      }
      const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
      if (edge) aff_chunk<R, LOCAL, TV_EDGE>(S, C, c);
      else if (lastStrip && selRow) aff_chunk<R, LOCAL, TV_SEL>(S, C, c);
      else aff_chunk<R, LOCAL, TV_FAST>(S, C, c);
      if constexpr (LOCAL) {
#pragma unroll
        for (int k = 0; k < R; ++k) S.bc[k] = (S.best[k] != b0[k]) ? c : S.bc[k];
      }
      const int done = rho * nblk + (c < nblk ? c : nblk);
      if (mailOut) {
        if (lane == 0) __hip_atomic_store(sProg + w, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(sProg + w, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (mailIn && lane == 0)
        __hip_atomic_store(sCons + w, seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if constexpr (LOCAL) {
      int32_t* rowbest = A.aux + P.aux_off + (n1 + 1);
      int32_t* rowpos = rowbest + n1;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int i = C.rowbase + k + 1;
        if (i <= n1) { rowbest[i - 1] = S.best[k]; rowpos[i - 1] = S.bc[k]; }
      }
    }
  }
}

#define BG_AFF_INST(RR)                                                 \
  template __global__ void bg_dp_aff_kernel<RR, false>(BgDpArgs);       \
  template __global__ void bg_dp_aff_kernel<RR, true>(BgDpArgs);
BG_AFF_INST(2)
BG_AFF_INST(4)
BG_AFF_INST(8)

extern "C" void* bg_dp_aff_kernel_ptr(int R, int local) {
  switch (R) {
    case 2: return local ? (void*)&bg_dp_aff_kernel<2, true> : (void*)&bg_dp_aff_kernel<2, false>;
    case 4: return local ? (void*)&bg_dp_aff_kernel<4, true> : (void*)&bg_dp_aff_kernel<4, false>;
    case 8: return local ? (void*)&bg_dp_aff_kernel<8, true> : (void*)&bg_dp_aff_kernel<8, false>;
    default: return nullptr;
  }
}

// LDS of the affine kernel: header + W waves (prog_off = 0, aux_lds_off = header)
extern "C" int bg_dp_aff_head_bytes(void) { return kAffHeadInts * 4; }
extern "C" int bg_dp_aff_wave_lds_bytes(int R, int K) {
  switch (R) {
    case 2: return aff_wave_ints<2>(K) * 4;
    case 4: return aff_wave_ints<4>(K) * 4;
    case 8: return aff_wave_ints<8>(K) * 4;
    default: return 0;
  }
}
