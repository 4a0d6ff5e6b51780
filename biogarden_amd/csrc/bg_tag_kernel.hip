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

#include <type_traits>

#include "bg_dev_util.h"
#include "bg_tag_common.h"
#include "bg_score_step.h"

using namespace bgk;

// LDS layout (bytes from the dynamic base; the host sizes it in bg_host.cpp):
//   16 produced + 16 consumed counters + a 128-int shared dummy ring (640 B, @prog_off) | the
//   pair's scaled code row when it
//   fits (@codes_off, u16, 64 zeros before it, NC + 2 chunks) | per wave @aux_lds_off: 64-int
//   boundary block, 256-int output ring, 4 codes x 64 lanes x RW-dword profile entries, 192 u16
//   scaled codes of the current chunk (columns t0-64 .. t0+127), 4 x 64-int mailbox.
//
// Boundary rows between strips on two waves of the same workgroup go through the producer's
// LDS mailbox (slot = block sequence number mod 4, flow-controlled by the consumer's counter),
// never through HBM; only a strip whose successor starts a new round (or sits in another
// workgroup, or is the finish kernel) writes its row to HBM.
//
// WIDE: the strips of one pair are spread over the pair's group of P.wg_count workgroups
// (A.wgmap[blockIdx] = (pair, index in group)); strip s runs on the group's wave s mod (G*W)
// and the progress counters live in global memory (A.gprog + P.prog_off), written and polled
// with agent-scope atomics like the boundary rows, so the group may span XCDs.  All workgroups
// of a group are resident together (the host caps the group at the CU count).
constexpr int kTagWaveInts = 64 + 128;   // boundary block + output ring (last-strip lanes below
                                         // row n1 write a workgroup-shared dummy ring)
constexpr int kTagStageU16 = 192;
#ifndef BG_MAIL_SLOTS
#define BG_MAIL_SLOTS 4
#endif
constexpr int kMailSlots = BG_MAIL_SLOTS;   // boundary blocks in flight between two waves of a workgroup

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kSC1 = 16;                     // buffer op cache policy: sc1 (agent-coherent)
// a raw buffer descriptor over [p, p + bytes) built from wave-uniform (readfirstlane) words, so
// that the buffer ops need no waterfall loop
__device__ __forceinline__ rsrc_t uniform_rsrc(const void* p, unsigned bytes) {
  const unsigned long long x = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Polling pauses.  WIDE runs one wave per SIMD: nothing else wants the issue slots, and every
// poll's wake-up latency adds to the strip's pace whenever it has caught up with its producer
// (the downstream strips of a chain of caught-up consumers slow down by that much per chunk), so
// it spins; the many-wave path sleeps to leave the slots to the other waves.
#ifndef BG_WIDE_SLEEP
#define BG_WIDE_SLEEP 0
#endif
// BG_WIDE_LONG > 0: a wait that outlasts BG_WIDE_FAST spinning polls (the strip pipeline's fill,
// where the wave of strip s waits ~5s chunks) sleeps BG_WIDE_LONG x 64 cycles between polls, so
// hundreds of parked waves stop loading progress counters through L2 beside the working strips
#ifndef BG_WIDE_LONG
#define BG_WIDE_LONG 0
#endif
#ifndef BG_WIDE_FAST
#define BG_WIDE_FAST 256
#endif
__device__ __forceinline__ void wide_poll_pause(int& n) {
  if constexpr (BG_WIDE_LONG > 0) {
    if (n < BG_WIDE_FAST) ++n;
    else __builtin_amdgcn_s_sleep(BG_WIDE_LONG);
  }
  if constexpr (BG_WIDE_SLEEP > 0) __builtin_amdgcn_s_sleep(BG_WIDE_SLEEP);
}
template <bool WIDE>
__device__ __forceinline__ void poll_pause(int& n) {
  if constexpr (WIDE) wide_poll_pause(n);
  else poll_backoff(n);
}

// profile entries per wave: the four DNA codes and (checkpoint mode) the border code, every byte
// -128, that the code row holds outside seq2 (columns j <= 0 and j > n2): there the diagonal
// candidate never wins, so
//   * beyond n2 every cell repeats its row's column n2: M'(i, j) = max(M'(i-1, j), M'(i, j-1)) and
//     M'(i, n2) >= M'(i-1, n2) in the frame.  A strip's registers end holding M(i, n2), stored
//     once, instead of a per-step catch in its last chunks;
//   * before column 0, with the border values M'(i, 0) non-decreasing from 0 (every mode but
//     global, a <= 0; global with a == b), the lanes' column-0 values loaded at the strip's start
//     survive the steps before each lane reaches column 0: chunk 0 needs no per-step reset.
// The row above of strip 0 is row 0 clamped at column n2, so that it freezes too.
// The last chunk's row above (block NC - 1, beyond n2 for lane 0) is never handed down: the strip
// above finishes before it is final.  Stale there, it would break the freeze, so a consumer takes
// kRowAboveNone for it (the row above then never wins past n2 either).
constexpr int kTagCodes = 5;
constexpr int kRowAboveNone = -(1 << 29);
template <int R>
__host__ __device__ constexpr int tag_wave_ints() {
  return kTagWaveInts + kTagCodes * 64 * ProfW<R>::v + kTagStageU16 / 2 + kMailSlots * 64;
}

// CKPT: the score-only forward pass of the checkpoint traceback (score_chunk, untagged M'
// values); at every chunk start each lane stores its R values and topPrev to the checkpoint
// arena: ckpt[((s * NC + c) * (R + 1) + k) * 64 + lane] (k = R: topPrev).
// WIDE: one workgroup of 4 waves per CU (one per SIMD), so a wave may hold up to 512 VGPRs: the
// six conveyor-loop instantiations then run without spills (at 1024 threads they spilled 48 B/lane)
// WM (the pair's width): 0 one workgroup per pair; 1 WIDE, a group of lone-wave workgroups per pair
// (few long pairs: the strip chain's latency); 2 SPAN, a group of many-wave workgroups per pair
// (fewer pairs than CUs: throughput).  SPAN hands rows between workgroups as WIDE does (boundary
// rows in HBM, agent-scope progress counters, at every W-th strip) and computes, polls and
// stages codes as the one-workgroup path does (several waves per SIMD).
template <int R, int WM, bool CKPT>
__global__ __launch_bounds__(WM == 1 ? 256 : 1024) void bg_dp_tag_kernel(BgDpArgs A) {
  constexpr bool WIDE = WM != 0;          // a group of workgroups per pair
  constexpr bool LONE = WM == 1;          // ... of one wave per SIMD
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int RW = ProfW<R>::v;
  const int lane = threadIdx.x & 63;
  const int W = blockDim.x >> 6;
  const int w = uni(threadIdx.x >> 6);
  constexpr int ROWS = BG_WAVE * R;

  int pairIdx = blockIdx.x, gi = 0;
  if constexpr (WIDE) {
    const int2 m = A.wgmap[blockIdx.x];
    pairIdx = m.x;
    gi = m.y;
  }
  int* sProg = reinterpret_cast<int*>(smem + A.prog_off);   // blocks produced (per wave)
  int* sCons = sProg + 16;                                   // chunks consumed (per wave)
  int* dummyRing = sProg + 32;                               // 128 ints, shared garbage
  if (threadIdx.x < 32) sProg[threadIdx.x] = 0;
  // the pair's whole scaled code row, when it fits (A.codes_in_lds): 64 zero entries before it
  // and zeros past n2 up to (NC + 2) chunks; else codes are staged per wave and chunk
  uint16_t* sRow = reinterpret_cast<uint16_t*>(smem + A.codes_off) + 64;
  // WIDE pairs too long for that: 2-bit codes, byte p = columns 4p - 64 .. 4p - 61 (0 outside
  // the row), unpacked into the wave's stage once per chunk
  uint8_t* sPk = smem + A.codes_off;
  if (A.codes_in_lds == 1) {
    const BgPair& Pp = A.pairs[pairIdx];
    const uint8_t* g = A.codes2 + Pp.off2;
    const int n = (Pp.nc + 2) * BG_CHUNK;
    for (int x = (int)threadIdx.x - 64; x < n; x += blockDim.x)
      sRow[x] = (x >= 0 && x < Pp.n2) ? (uint16_t)(g[x] * (32 * RW)) : (uint16_t)(CKPT ? 4 * 256 * RW : 0);
  } else if (WIDE && A.codes_in_lds == 2) {
    const BgPair& Pp = A.pairs[pairIdx];
    const uint8_t* g = A.codes2 + Pp.off2;   // code * 8
    const int nb = (Pp.nc + 3) * 16;
    for (int p = threadIdx.x; p < nb; p += blockDim.x) {
      unsigned v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int x = 4 * p - 64 + k;
        if (x >= 0 && x < Pp.n2) v |= ((unsigned)g[x] >> 3) << (2 * k);
      }
      sPk[p] = (uint8_t)v;
    }
  }
  __syncthreads();

  const BgPair P = A.pairs[pairIdx];
  const int n1 = P.n1, n2 = P.n2, nst = P.nstrips, NC = P.nc;
  // concurrent exit pass (bg_split.hip): it waits for this DP's data only once every workgroup of
  // the DP is resident, so its workers can never hold the CUs this DP still needs
  const bool ckgOn = WIDE && CKPT && A.split != nullptr;
  if (ckgOn && threadIdx.x == 0) __hip_atomic_fetch_add(A.resident, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nst == 0) return;
  // its inputs: every segc-th checkpoint of each strip as {value, epoch} granules
  unsigned long long* ckgPair = nullptr;
  int ckgG = 1;
  if (ckgOn) {
    const BgSplitLayout SLy = bg_split_layout(n1, n2, nst, NC, R, A.segc);
    ckgPair = reinterpret_cast<unsigned long long*>(A.split + P.split_off + SLy.ckg);
    ckgG = SLy.G;
  }
  const int GW = (WIDE ? P.wg_count : 1) * W;                  // waves working on this pair
  const int gw = gi * W + w;
  uint32_t* gProg = WIDE ? A.gprog + P.prog_off : nullptr;
  const int a = A.open;
  const int b = A.ext;
  const int mode = A.mode;
  const size_t stripDw = (size_t)NC * (BG_CHUNK / BG_TRACE_BLK) * R * 2 * BG_WAVE;
  int* waveLds = reinterpret_cast<int*>(smem + A.aux_lds_off) + w * tag_wave_ints<R>();
  int* profTab = waveLds + kTagWaveInts;
  uint16_t* stage = reinterpret_cast<uint16_t*>(profTab + kTagCodes * 64 * RW);
  int* mailbox = profTab + kTagCodes * 64 * RW + kTagStageU16 / 2;   // this wave's outgoing blocks
  const int prevW = (w + W - 1) % W;                         // producer wave of the strip above
  int* prevMail = reinterpret_cast<int*>(smem + A.aux_lds_off) + prevW * tag_wave_ints<R>() +
                  (kTagWaveInts + kTagCodes * 64 * RW + kTagStageU16 / 2);

  TagCtx C;
  C.a = a; C.b = b; C.mode = mode; C.n1 = n1; C.n2 = n2; C.lane = lane;
  C.lastcol = A.aux + P.aux_off;
  C.bIn = waveLds;
  C.mail = nullptr;
  C.ring = waveLds + 64;
  C.profLane = reinterpret_cast<const uint8_t*>(profTab + lane * RW);
  const bool rowInLds = A.codes_in_lds == 1;
  const bool rowPacked = WIDE && A.codes_in_lds == 2;
  C.codeLane = stage + 63 - lane;       // (t - lane - 1) - (t0 - 64) = u + 63 - lane

  const uint8_t* c1 = A.codes1 + P.off1;
  const uint8_t* g2 = A.codes2 + P.off2;  // code * 8 (DNA path)
  // the staged code of a column outside seq2: the border entry (checkpoint mode), else code 0
  constexpr uint16_t kBorder = CKPT ? 4 * 256 * RW : 0;
  // checkpoint mode: chunk 0 without a column-0 reset (see kTagCodes)
  const bool colMono = CKPT && a <= 0 && (mode != BGK_GLOBAL || a == b);
  // raw codes of columns t0-64+lane+64q, q = 0..2 (clamped, unconditional loads: they are only
  // consumed at the next chunk's start, so their latency hides behind a whole chunk)
  auto fetch_codes = [&](int c, int (&v)[3]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      v[q] = g2[x < 0 ? 0 : (x >= n2 ? n2 - 1 : x)];
    }
  };
  // ... scaled to profile-entry byte offsets (0 outside the row) when staged
  auto stage_codes = [&](int c, const int (&v)[3]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? v[q] * (32 * RW) : kBorder);
    }
  };
  // ... or from the packed row in LDS (columns t0 - 64 + lane + 64q: byte 16(c + q) + lane / 4)
  auto stage_packed = [&](int c) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const unsigned v = sPk[16 * (c + q) + (lane >> 2)];
      const int x = c * BG_CHUNK - 64 + lane + 64 * q;
      stage[lane + 64 * q] = (uint16_t)(((unsigned)x < (unsigned)n2) ? ((v >> (2 * (lane & 3))) & 3u) * (256 * RW) : kBorder);
    }
  };

  TagStrip<R> S;
  const int nblk = NC - 1;
  for (int s = gw, rho = 0; s < nst; s += GW, ++rho) {
    C.rowbase = s * ROWS + lane * R;
    const bool lastStrip = (s == nst - 1);
    const int lastRow = n1 - 1 - s * ROWS;
    const int olane = lastStrip ? lastRow / R : BG_WAVE - 1;
    C.orow = lastStrip ? lastRow % R : R - 1;
    // score-only strips (not WIDE): the rows below row n1 of the last strip are made to repeat row
    // n1 — profile bytes -128 and row n1's column-0 value there, so max3 always takes the row above
    // (M'(i, j) >= M'(i, j - 1) in the frame) — and the lane holding row n1 hands it down as its
    // last row: the last strip runs the plain step instead of a select per row and step (1.8 % of
    // the metric DP's VALU).  Nothing reads those rows: the traceback never walks below row n1.
    const bool repeatN1 = CKPT && !LONE && lastStrip && C.orow != R - 1;
    if (repeatN1) C.orow = R - 1;
    C.repeatN1 = repeatN1;
    const bool selRow = C.orow != R - 1;
    C.oLane = (lane <= olane ? C.ring : dummyRing) + 64 - lane;
    C.trace = A.trace + P.trace_off / 4 + (size_t)s * stripDw;
    C.bndOut = A.bndM + P.bnd_off + (size_t)s * NC * BG_CHUNK;
    // strip s+1 on the next wave of this workgroup in this round: hand blocks over in LDS
    const bool mailOut = (s + 1 < nst) && (w + 1 < W);
    // strip s-1 on the previous wave of this workgroup in this round: read its mailbox
    const bool mailIn = (s > 0) && (w > 0);
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
      if constexpr (CKPT) {
        pk[k] = (repeatN1 && i > n1) ? (int)0x80808080 : A.profile[192 + (q >> 3)];   // 4 codes x int8 S - 2a
        const int ii = (repeatN1 && i > n1) ? n1 : i;
        S.Y[k] = wadd(col0_M(mode, ii, a, b), -wmul(a, ii));
      } else {
        pk[k] = A.profile[(k == 0 ? 64 : 128) + (q >> 3)];   // 4 codes x int8
        S.Y[k] = col0_Y(mode, i, a, b);
      }
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
    if constexpr (CKPT) {
#pragma unroll
      for (int wd = 0; wd < RW; ++wd) profTab[(4 * 64 + lane) * RW + wd] = (int)0x80808080;   // border
    }
    S.topPrev = 0; S.Xlast = CKPT ? 0 : 2;
    int32_t* ckBase = CKPT ? reinterpret_cast<int32_t*>(A.trace + P.trace_off / 4) +
                                 (size_t)s * NC * (R + 1) * BG_WAVE + lane
                           : nullptr;
    int cv[3] = {0, 0, 0};
    if (!rowInLds && !rowPacked) fetch_codes(0, cv);
    const bool hbmAhead = WIDE && s > 0 && !mailIn;
    const int pwH = (s - 1) % GW;
    const int needBase = ((s - 1) / GW) * nblk;
    const int32_t* bndAbove = A.bndM + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + lane;
    const bool dbgOn = A.dbg != nullptr && rho == 0 && pairIdx == 0 && gw < 4096;
    unsigned long long tWait = 0, tStart = dbgOn ? __builtin_amdgcn_s_memrealtime() : 0;
    const unsigned long long cStart = dbgOn ? __builtin_amdgcn_s_memtime() : 0;
    // CONV mode (WIDE, checkpoint): every strip but the last runs the one-register conveyor step
    // (score_chunk_conv) and hands its last row down in HALF blocks of 32 columns, as soon as
    // each half leaves the conveyor: a consumer then trails its producer by 64 + 32 steps (the
    // lanes' anti-diagonal skew plus one half) instead of two whole chunks.
    //  * same workgroup: 32-int half slots of the producer's LDS mailbox (2 kMailSlots of them),
    //    counters in halves, one sequence per wave across its rounds (seq = rho * nh + half);
    //  * another workgroup: 8-byte {value, epoch} granules (A.gran, the MI355X guide's data-tagged
    //    hand-off: one aligned `sc1` store each, read with `sc1` loads until every tag equals
    //    this launch's epoch) — no counter, no store drain before a publication, and the reader's
    //    only loads are issued a half ahead, so no wait of this loop waits on a fresh store.
    // The last strip reads whole blocks (two adjacent half slots, or 64 granules) and keeps the
    // ring path for its output row (row n1 may sit in any lane).
    constexpr bool CONVMODE = LONE && CKPT;
    constexpr int KH = 2 * kMailSlots;                          // half slots per mailbox
    const int nh = 2 * nblk;                                     // halves handed down per strip
    const uint32_t ep = A.epoch;
    unsigned long long* gOut = A.gran + P.bnd_off + (size_t)s * NC * BG_CHUNK;
    const unsigned long long* gIn = A.gran + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK;
    if (CONVMODE && !lastStrip) {
      // one loop per (incoming, outgoing) kind, so that no register of one kind's loads is
      // reused by another kind's code (the compiler then waits vmcnt(0) on every such reuse)
      auto conv_loop = [&](auto inK, auto outK) {
      constexpr int IN = decltype(inK)::value;                   // 0 row 0, 1 mailbox, 2 granules
      constexpr bool MOUT = decltype(outK)::value;               // consumer in this workgroup
      const bool lo = lane < 32;
      const int l32 = lane & 31;
      const int hb = rho * nh;                                   // this round's half sequence base
      // Global memory through buffer descriptors (wave-uniform SGPRs) and lane offsets computed
      // once: the compiler waits vmcnt before it overwrites ANY register a pending memory op reads
      // (address or data), so per-boundary 64-bit addresses in temporaries made every boundary
      // wait for its own stores.  The data registers of this boundary's stores are kept live
      // (kv, kg, ckv) until the next boundary, by when the stores have completed.
      const rsrc_t rCk = uniform_rsrc(ckBase - lane, NC * (R + 1) * BG_WAVE * 4);
      const rsrc_t rBnd = uniform_rsrc(C.bndOut, NC * BG_CHUNK * 4);
      const rsrc_t rGo = uniform_rsrc(gOut, NC * BG_CHUNK * 8);
      const int vL4 = lane * 4, vH4 = l32 * 4, vH8 = l32 * 8;
      const rsrc_t rGi = uniform_rsrc(s > 0 ? gIn : gOut, NC * BG_CHUNK * 8);
      // concurrent exit pass: segment-start checkpoints of this strip ({value, epoch}, [g][k][lane])
      const rsrc_t rCkg = uniform_rsrc(ckgOn ? ckgPair + (size_t)s * ckgG * (R + 1) * BG_WAVE : gOut,
                                       ckgOn ? ckgG * (R + 1) * BG_WAVE * 8 : 8);
      // two halves in flight: even halves in gvA, odd halves in gvB (the two boundary call sites
      // of a chunk), so a load has two halves' time to land and is never copied while pending
      u32x2 gvA = {0u, 0u}, gvB = {0u, 0u};
      if (IN == 2 && 0 < nh) gvA = __builtin_amdgcn_raw_buffer_load_b64(rGi, vH8, 0, kSC1);
      if (IN == 2 && 1 < nh) gvB = __builtin_amdgcn_raw_buffer_load_b64(rGi, vH8, 256, kSC1);
      int kv = 0;
      u32x2 kg = {0u, 0u};
      int ckv[R + 1];
      u32x2 ckgv[R + 1];                                         // concurrent exit pass granules
#pragma unroll
      for (int k = 0; k <= R; ++k) { ckv[k] = 0; ckgv[k] = u32x2{0u, 0u}; }
      int Q = 0;
      ConvPipe<RW> pipe;                                         // operands across chunks
      unsigned long long tData = 0, tFlow = 0;                   // BG_DEBUG=dp: spin cycles
      // LDS words read a boundary ahead (their latency hides behind the half's compute; the
      // words are monotonic, so a stale read only sends the wave down the polling path):
      // pc = the producer's half count, pv = the half after this boundary's (valid when pc says
      // so: the count is read before the data, in this wave's LDS order, and the producer wrote
      // the data before the count), fc = the consumer's release count
      int pc = -1, pv = 0, fc = -(1 << 30);
      // half og of this strip's last row, in lanes 32-63 of v: to the consumer and to bndOut
      auto emit = [&](int og, int v) {
        const int col = 32 * og + l32;
        if constexpr (MOUT) {
          const int sq = hb + og;
          if (fc < sq + 1 - KH) {
            int np = 0;
            const unsigned long long tf0 = dbgOn ? __builtin_amdgcn_s_memtime() : 0;
            while ((fc = __hip_atomic_load(sCons + w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < sq + 1 - KH)
              wide_poll_pause(np);
            if (dbgOn) tFlow += __builtin_amdgcn_s_memtime() - tf0;
          }
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          if (!lo) mailbox[(sq % KH) * 32 + l32] = v;
          __atomic_signal_fence(__ATOMIC_SEQ_CST);              // LDS: the counter after the data
          if (lane == 0) __hip_atomic_store(sProg + w, sq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          fc = __hip_atomic_load(sCons + w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          kg = u32x2{(unsigned)v, ep};
          if (!lo) __builtin_amdgcn_raw_buffer_store_b64(kg, rGo, vH8, og * 256, kSC1);
        }
        if constexpr (MOUT) {
          // the concurrent exit pass reads every strip's row from the granules
          if (ckgOn) {
            kg = u32x2{(unsigned)v, ep};
            if (!lo) __builtin_amdgcn_raw_buffer_store_b64(kg, rGo, vH8, og * 256, kSC1);
          }
        }
        kv = v;
        if (!lo) __builtin_amdgcn_raw_buffer_store_b32(kv, rBnd, vH4, og * 128, 0);
        (void)col;
      };
      // before half g: the row above's half g into lanes 0-31 (lane 0 reads it at the next step),
      // the finished half g - 3 (lanes 32-63) out
      auto boundary = [&](int g, u32x2& gv) {
        // the previous boundary's store data stays allocated until here
        asm volatile("" ::"v"(kv), "v"(kg.x), "v"(kg.y));
        const unsigned long long tw0 = dbgOn ? __builtin_amdgcn_s_memtime() : 0;
        const unsigned long long tw0r =
            (dbgOn && (g < 12 || g == 1000 || g == 1003)) ? __builtin_amdgcn_s_memrealtime() : 0;
        int inV;
        if constexpr (IN == 0) {
          const int j = min(32 * g + l32, n2);                             // frozen past n2
          inV = wadd(row0_M(mode, j, a, b), -wmul(a, j));                    // M'(0, j)
        } else if constexpr (IN == 1) {
          const int sq = hb + g;
          if (g < nh && pc < sq + 1) {
            int np = 0;
            const unsigned long long td0 = dbgOn ? __builtin_amdgcn_s_memtime() : 0;
            while (__hip_atomic_load(sProg + prevW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < sq + 1)
              wide_poll_pause(np);
            if (dbgOn) tData += __builtin_amdgcn_s_memtime() - td0;
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            pv = prevMail[(sq % KH) * 32 + l32];
          }
          inV = g < nh ? pv : kRowAboveNone;                             // past the last block: frozen
          __atomic_signal_fence(__ATOMIC_SEQ_CST);              // LDS: the release after the read
          if (lane == 0) __hip_atomic_store(sCons + w, sq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          pc = __hip_atomic_load(sProg + prevW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          pv = prevMail[((sq + 1) % KH) * 32 + l32];
        } else {
          if (g < nh) {
            int np = 0;
            const unsigned long long td0 = dbgOn ? __builtin_amdgcn_s_memtime() : 0;
            while (!__all(!lo || gv.y == ep)) {
              wide_poll_pause(np);
              gv = __builtin_amdgcn_raw_buffer_load_b64(rGi, vH8, g * 256, kSC1);
            }
            if (dbgOn) tData += __builtin_amdgcn_s_memtime() - td0;
          }
          inV = g < nh ? (int)gv.x : kRowAboveNone;                       // past the last block: frozen
          if (g + 2 < nh) gv = __builtin_amdgcn_raw_buffer_load_b64(rGi, vH8, (g + 2) * 256, kSC1);
        }
        const int Qo = Q;
        Q = lo ? inV : Q;
        if (g >= 3) emit(g - 3, Qo);
        if (dbgOn) {
          tWait += __builtin_amdgcn_s_memtime() - tw0;
          // BG_DEBUG=dp: the first boundaries' and two steady ones' (1000, 1003) arrival / departure
          // (s_memrealtime), [g][arrive, depart] after the 8-word records
          const int gs = g < 12 ? g : (g == 1000 ? 12 : (g == 1003 ? 13 : -1));
          if (gs >= 0 && lane == 0) {
            A.dbg[8 * 4096 + gw * 32 + 2 * gs] = tw0r;
            A.dbg[8 * 4096 + gw * 32 + 2 * gs + 1] = __builtin_amdgcn_s_memrealtime();
          }
        }
      };
      for (int c = 0; c < NC; ++c) {
        if (dbgOn && c == 1 && lane == 0) A.dbg[gw * 8 + 2] = __builtin_amdgcn_s_memrealtime();
        if (rowInLds) {
          C.codeLane = sRow + c * BG_CHUNK - lane - 1;
        } else if (rowPacked) {
          stage_packed(c);
        } else {
          stage_codes(c, cv);
          fetch_codes(c + 1 < NC ? c + 1 : c, cv);
        }
        // the checkpoint stores go first: a boundary's own stores are then the youngest memory
        // operations when the compute starts, and nothing waits on them before the next boundary
#pragma unroll
        for (int k = 0; k <= R; ++k) {
          ckv[k] = k < R ? S.Y[k] : S.topPrev;
          asm volatile("" : "+v"(ckv[k]));                    // a register of its own
          __builtin_amdgcn_raw_buffer_store_b32(ckv[k], rCk, vL4, (c * (R + 1) + k) * BG_WAVE * 4, 0);
        }
        if (ckgOn && c % A.segc == 0) {
          const int gseg = c / A.segc;
#pragma unroll
          for (int k = 0; k <= R; ++k) {
            ckgv[k] = u32x2{(unsigned)ckv[k], ep};
            asm volatile("" : "+v"(ckgv[k]));               // registers of their own (see ckv)
            __builtin_amdgcn_raw_buffer_store_b64(ckgv[k], rCkg, vL4 * 2, ((gseg * (R + 1) + k) * BG_WAVE) * 8, kSC1);
          }
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        boundary(2 * c, gvA);
        auto mid = [&]() {
#pragma unroll
          for (int k = 0; k <= R; ++k) asm volatile("" ::"v"(ckv[k]), "v"(ckgv[k].x), "v"(ckgv[k].y));
          boundary(2 * c + 1, gvB);
        };
        if (c == 0) conv_pipe_init(pipe, C);
        if (c == 0 && !colMono) score_chunk_conv<R, TV_COL0>(S, C, c, Q, pipe, mid);
        else score_chunk_conv<R, TV_FAST>(S, C, c, Q, pipe, mid);
      }
      if (nh >= 1) emit(nh - 1, Q);                              // the last half: 2 NC - 3
      if (dbgOn && lane == 0) {
        A.dbg[gw * 8 + 6] = tData;
        A.dbg[gw * 8 + 7] = tFlow;
      }
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      using I2 = std::integral_constant<int, 2>;
      using BT = std::integral_constant<bool, true>;
      using BF = std::integral_constant<bool, false>;
      if (s == 0) {
        if (mailOut) conv_loop(I0{}, BT{}); else conv_loop(I0{}, BF{});
      } else if (mailIn) {
        if (mailOut) conv_loop(I1{}, BT{}); else conv_loop(I1{}, BF{});
      } else {
        if (mailOut) conv_loop(I2{}, BT{}); else conv_loop(I2{}, BF{});
      }
    } else {
    // the last strip of a CONV-mode pair reads whole blocks of 64 granules, one block ahead
    unsigned long long gL = 0;
    if (CONVMODE && hbmAhead && 0 < nblk) gL = __hip_atomic_load(gIn + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // WIDE, strip above on another workgroup: its blocks come through HBM one chunk ahead of
    // use — block c + 1 (and the producer's counter for the check at chunk c + 1) is loaded
    // while chunk c computes, so neither the counter poll nor the block load (each a cross-XCD
    // L2 / MALL round trip of ~1-2 us) sits between two chunks of the strip pipeline
    // Cross-workgroup hand-off (the MI355X guide's measured-valid form without an acquire
    // fence: sc1 stores, a flag behind their completion, an sc1 poll, then sc1 loads by the wave
    // that polled): the producer stores the block `sc1` (relaxed agent-scope store), waits for
    // its completion (vmcnt: vector memory operations of a wave complete in issue order) and
    // only then stores its progress counter `sc1`; this wave polls the counter with `sc1` loads
    // and issues the block's `sc1` load only after a poll has returned a sufficient value (the
    // compare consumes it).  The signal fences keep the compiler from moving the block load
    // above the poll; an agent acquire fence (vmcnt(0) + buffer_inv sc1, ~1.7 us) per chunk
    // would cost more than the chunk.
    int nbV = 0, pollV = 0;
    if (hbmAhead && !CONVMODE) {
      int np0 = 0;
      if (0 < nblk)
        while ((int)__hip_atomic_load(gProg + pwH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < needBase + 1)
          poll_pause<LONE>(np0);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      nbV = load_agent(bndAbove);
      pollV = (int)__hip_atomic_load(gProg + pwH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int c = 0; c < NC; ++c) {
      if (dbgOn && c == 1 && lane == 0) A.dbg[gw * 8 + 2] = __builtin_amdgcn_s_memrealtime();
      const unsigned long long tw0 = dbgOn ? __builtin_amdgcn_s_memtime() : 0;
      if (rowInLds) {
        C.codeLane = sRow + c * BG_CHUNK - lane - 1;
      } else if (rowPacked) {
        stage_packed(c);
      } else {
        // this chunk's codes into LDS, the next chunk's in flight
        stage_codes(c, cv);
        fetch_codes(c + 1 < NC ? c + 1 : c, cv);
      }
      // the row above, block c: row 0, the producer's LDS mailbox, or HBM
      const int seq = rho * NC + c;                              // block sequence number
      const int hseq = rho * nh + 2 * c;                         // CONV mode: its first half
      const int jb = c * BG_CHUNK + lane;
      if (s == 0) {
        const int jr = CKPT ? min(jb, n2) : jb;                            // frozen past n2
        const int m0 = wadd(row0_M(mode, jr, a, b), -wmul(a, jr));          // M'(0, j)
        waveLds[lane] = CKPT ? m0 : 4 * m0 + 2;                             // (X form)
        C.bIn = waveLds;
      } else if (hbmAhead && CONVMODE) {
        if (c < nblk) {
          int np = 0;
          while (!__all((uint32_t)(gL >> 32) == ep)) {
            wide_poll_pause(np);
            gL = __hip_atomic_load(gIn + (size_t)c * BG_CHUNK + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        waveLds[lane] = (int)(uint32_t)gL;
        C.bIn = waveLds;
        if (c + 1 < nblk)
          gL = __hip_atomic_load(gIn + (size_t)(c + 1) * BG_CHUNK + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (hbmAhead) {
        waveLds[lane] = nbV;
        C.bIn = waveLds;
        if (c + 1 < NC) {
          if (c + 1 < nblk) {
            int np1 = 0;
            while (pollV < needBase + c + 2) {
              poll_pause<LONE>(np1);
              pollV = (int)__hip_atomic_load(gProg + pwH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          __atomic_signal_fence(__ATOMIC_SEQ_CST);
          nbV = load_agent(bndAbove + (size_t)(c + 1) * BG_CHUNK);         // block c + 1
          pollV = (int)__hip_atomic_load(gProg + pwH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        if (c < nblk) {
          const int need = CONVMODE ? hseq + 2 : ((s - 1) / GW) * nblk + c + 1;
          const int pw = mailIn ? prevW : (s - 1) % GW;
          if (WIDE && !mailIn) {
            int np2 = 0;
            while ((int)__hip_atomic_load(gProg + pw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need)
              poll_pause<LONE>(np2);
          } else {
            int np = 0;
            while (__hip_atomic_load(sProg + pw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
              poll_pause<LONE>(np);
          }
        }
        if (mailIn) {
          // CONV mode: halves hseq, hseq + 1 sit in adjacent half slots (hseq is even)
          C.bIn = CONVMODE ? prevMail + (hseq % KH) * 32 : prevMail + (seq % kMailSlots) * 64;
        } else {
          __atomic_signal_fence(__ATOMIC_SEQ_CST);                          // after the poll
          waveLds[lane] = load_agent(A.bndM + P.bnd_off + (size_t)(s - 1) * NC * BG_CHUNK + jb);
          C.bIn = waveLds;
        }
      }
      if (CKPT && s > 0 && c >= nblk) {                            // never handed down: frozen
        waveLds[lane] = kRowAboveNone;
        C.bIn = waveLds;
      }
      // the block this chunk finishes (c-1) goes to mailbox slot (seq-1) mod 4 once the
      // consumer has finished the chunk that read that slot last (sequence seq-1-4)
      C.mail = nullptr;
      if (mailOut && c >= 1 && c - 1 < nblk) {
        const int needC = seq - kMailSlots;                      // consumer chunks finished
        int np = 0;
        while (__hip_atomic_load(sCons + w + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < needC)
          poll_pause<LONE>(np);
        C.mail = mailbox + ((seq - 1) % kMailSlots) * 64;
      }
      if (dbgOn) tWait += __builtin_amdgcn_s_memtime() - tw0;
      const bool edge = (c == 0) || (c * BG_CHUNK + BG_CHUNK - 1 >= n2);
      if constexpr (CKPT) {
        int32_t* ck = ckBase + (size_t)c * (R + 1) * BG_WAVE;
#pragma unroll
        for (int k = 0; k < R; ++k) ck[k * BG_WAVE] = S.Y[k];
        ck[R * BG_WAVE] = S.topPrev;
        if (ckgOn && c % A.segc == 0) {
          unsigned long long* cg = ckgPair + (((size_t)s * ckgG + c / A.segc) * (R + 1)) * BG_WAVE + lane;
#pragma unroll
          for (int k = 0; k <= R; ++k)
            __hip_atomic_store(cg + k * BG_WAVE,
                               ((unsigned long long)A.epoch << 32) | (uint32_t)(k < R ? S.Y[k] : S.topPrev),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (c == 0 && !colMono) score_chunk<R, TV_COL0, LONE, false, WIDE>(S, C, c);
        else if (lastStrip && selRow) score_chunk<R, TV_SEL, LONE, false, WIDE>(S, C, c);
        else if (R <= 4 && s == 0 && !edge) {
          // row 0 above: M'(0, j) for j >= 1 is linear (semiglobal / local / overlap: M = 0;
          // global / fitting: a + (j - 1) b)
          const bool flat = mode == BGK_SEMIGLOBAL || mode == BGK_LOCAL || mode == BGK_OVERLAP;
          C.topStep = flat ? -a : b - a;
          C.top0 = wadd(row0_M(mode, c * BG_CHUNK, a, b), -wmul(a, c * BG_CHUNK));
          score_chunk<R, TV_FAST, LONE, true, WIDE>(S, C, c);
        } else score_chunk<R, TV_FAST, LONE, false, WIDE>(S, C, c);
      } else {
        if (edge) tag_chunk<R, TV_EDGE, LONE>(S, C, c);
        else if (lastStrip && selRow) tag_chunk<R, TV_SEL, LONE>(S, C, c);
        else tag_chunk<R, TV_FAST, LONE>(S, C, c);
      }
      // publish.  LDS mailbox: the block's ds_writes precede the counter's in this wave's LDS
      // queue.  HBM: the chunk ends with the block store and R trace stores; at vmcnt(R) the
      // block store has completed (vector memory operations complete in order).
      int done = rho * nblk + (c < nblk ? c : nblk);
      if (mailOut) {
        if (lane == 0) __hip_atomic_store(sProg + w, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else if (s + 1 < nst) {                                    // a consumer reads HBM
        if constexpr (CKPT) {
          // interior chunks publish one block late instead of draining the stores: a chunk's
          // vector memory operations are its R + 1 checkpoint stores, then the block store, so
          // at vmcnt(R + 2) the previous chunk's block has completed (in-order completion); a
          // drain per chunk stalled this wave (the last of a round, or of a WIDE workgroup) for
          // the store round trip, and the strip pipeline behind it with it
          if (!edge && c >= 2) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(R + 2) : "memory");
            done -= 1;
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(R) : "memory");
        }
        if constexpr (WIDE) {
          if (lane == 0) __hip_atomic_store(gProg + gw, (uint32_t)done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          if (lane == 0) __hip_atomic_store(sProg + w, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      if (mailIn && lane == 0)   // release: this chunk's reads of the slot(s) are done
        __hip_atomic_store(sCons + w, CONVMODE ? hseq + 2 : seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    }
    if constexpr (CKPT) {
      // M(i, n2): past column n2 every cell repeats it (the border code), so the strip's registers
      // end holding the lane's column n2 (every lane passes it: NC = n2 / 64 + 2 chunks)
      if (n2 > 0) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int i = C.rowbase + k + 1;
          if (i <= n1) C.lastcol[i] = wadd(S.Y[k], wmul(a, i + n2));
        }
      }
    }
    if (dbgOn && lane == 0) {
      A.dbg[gw * 8 + 0] = (unsigned long long)s;
      A.dbg[gw * 8 + 1] = tStart;
      A.dbg[gw * 8 + 3] = __builtin_amdgcn_s_memrealtime();
      A.dbg[gw * 8 + 4] = tWait;
      A.dbg[gw * 8 + 5] = __builtin_amdgcn_s_memtime() - cStart;
    }
  }
}

#define BG_TAG_INST(RR)                                                   \
  template __global__ void bg_dp_tag_kernel<RR, 0, false>(BgDpArgs);      \
  template __global__ void bg_dp_tag_kernel<RR, 1, false>(BgDpArgs);      \
  template __global__ void bg_dp_tag_kernel<RR, 0, true>(BgDpArgs);       \
  template __global__ void bg_dp_tag_kernel<RR, 1, true>(BgDpArgs);       \
  template __global__ void bg_dp_tag_kernel<RR, 2, true>(BgDpArgs);
BG_TAG_INST(2)
BG_TAG_INST(3)
BG_TAG_INST(4)
BG_TAG_INST(5)
BG_TAG_INST(8)
BG_TAG_INST(10)

// wide: 0 one workgroup per pair, 1 WIDE (lone waves), 2 SPAN (checkpoint only)
extern "C" void* bg_dp_kernel_tag_ptr(int R, int wide, int ckpt) {
  switch (R) {
#define BG_TAG_CASE(RR)                                                                   \
    case RR:                                                                              \
      if (ckpt) return wide == 2 ? (void*)&bg_dp_tag_kernel<RR, 2, true>                  \
                     : wide ? (void*)&bg_dp_tag_kernel<RR, 1, true> : (void*)&bg_dp_tag_kernel<RR, 0, true>; \
      if (wide == 2) return nullptr;                                                      \
      return wide ? (void*)&bg_dp_tag_kernel<RR, 1, false> : (void*)&bg_dp_tag_kernel<RR, 0, false>;
    BG_TAG_CASE(2)
    BG_TAG_CASE(3)
    BG_TAG_CASE(4)
    BG_TAG_CASE(5)
    BG_TAG_CASE(8)
    BG_TAG_CASE(10)
#undef BG_TAG_CASE
    default: return nullptr;
  }
}

// LDS bytes per wave of the tagged kernel (host sizing)
extern "C" int bg_dp_tag_wave_lds_bytes(int R) {
  switch (R) {
    case 2: return tag_wave_ints<2>() * 4;
    case 3: return tag_wave_ints<3>() * 4;
    case 4: return tag_wave_ints<4>() * 4;
    case 5: return tag_wave_ints<5>() * 4;
    case 8: return tag_wave_ints<8>() * 4;
    case 10: return tag_wave_ints<10>() * 4;
    default: return 0;
  }
}
