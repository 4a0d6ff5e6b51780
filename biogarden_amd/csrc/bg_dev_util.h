// Device helpers shared by the DP and finish kernels (gfx950 wave64 primitives).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bg_device.h"

typedef unsigned long long u64;

extern "C" __device__ int bg_writelane_i32(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace bgk {

constexpr int kNegInf = INT32_MIN;  // i32::MIN: x/y buffers' initial value (aligner.rs:49-50)

// Polling an LDS progress counter on the many-wave paths.  The first BG_POLL_FAST polls of a
// wait sleep 64 cycles (a steady-state wait ends within a few); later ones BG_POLL_LONG x 64, so
// a wave parked for a long wait (the strip pipeline's fill: the wave of strip s starts ~2s
// chunks after strip 0) stops taking issue slots from the computing waves of its SIMD.
// tools/poll_ab.sh, same box: LONG = 1 (every poll 64 cycles) metric 10 100-10 190 / MA 4 630-4 650
// GCUPS; 8: 10 350 / 4 776; 32: 10 375-10 405 / 4 777-4 783; 127: 10 287 / 4 766; FAST 2-32 alike.
#ifndef BG_POLL_LONG
#define BG_POLL_LONG 32
#endif
#ifndef BG_POLL_FAST
#define BG_POLL_FAST 8
#endif
__device__ __forceinline__ void poll_backoff(int& n) {
  if constexpr (BG_POLL_LONG > 1) {
    if (n < BG_POLL_FAST) { __builtin_amdgcn_s_sleep(1); ++n; }
    else __builtin_amdgcn_s_sleep(BG_POLL_LONG);
  } else {
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ int dpp_shr1(int old, int src) {
  // v_mov_b32_dpp wave_shr:1 — lane r receives lane r-1; lane 0 keeps `old`.
  return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int wrlane(int val, int l, int old) { return bg_writelane_i32(val, l, old); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// release-mode i32 `+` wraps; `saturating_add` is v_add_i32 ... clamp
__device__ __forceinline__ int wadd(int x, int y) { return (int)((unsigned)x + (unsigned)y); }
__device__ __forceinline__ int wmul(int x, int y) { return (int)((unsigned)x * (unsigned)y); }
__device__ __forceinline__ int sadd(int x, int y) { return __builtin_elementwise_add_sat(x, y); }
__device__ __forceinline__ int imax(int x, int y) { return __builtin_elementwise_max(x, y); }
// v_max3_i32 kept opaque so the compiler cannot turn `best == y` into a max+compare pair.
__device__ __forceinline__ int imax3(int x, int y, int z) {
  int r;
  asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
__device__ __forceinline__ u64 ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ int sbfe(int v, int off, int w) { return __builtin_amdgcn_sbfe(v, off, w); }

// acc = 2*acc + (this lane's bit of mask): one VALU op per trace bit.
__device__ __forceinline__ unsigned shift_in(unsigned acc, u64 mask) {
  unsigned r;
  u64 co;
  asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(acc), "s"(mask));
  return r;
}

// v_cndmask_b32 kept opaque: a plain `gt ? best : old` chain over the unrolled steps is
// re-associated by LLVM into a max-tree that keeps every step's value live (register spills).
__device__ __forceinline__ int vsel(u64 mask, int if_set, int if_clear) {
  int r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(mask));
  return r;
}

__device__ __forceinline__ int load_agent(const int32_t* p) {
  // L1-bypassing load (global_load_dword sc1): boundary rows written by another wave.
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// End-cell keys (the reference's first / last and > / >= rules as one u64 max): the value biased
// to unsigned in the high word, the index rule in the low word
__device__ __forceinline__ unsigned key_bias(int v) { return (unsigned)v ^ 0x80000000u; }
__device__ __forceinline__ u64 wave_umax64(u64 v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned lo = __shfl_xor((unsigned)v, o, 64);
    const unsigned hi = __shfl_xor((unsigned)(v >> 32), o, 64);
    const u64 other = ((u64)hi << 32) | lo;
    v = other > v ? other : v;
  }
  return v;
}

// Row 0 / column 0 initialisation per mode (aligner.rs:96-104, 163, 233-237, 299, 360).
__device__ __forceinline__ int row0_M(int mode, int j, int a, int b) {
  if (j == 0) return 0;
  return (mode == BGK_GLOBAL || mode == BGK_FITTING) ? wadd(a, wmul(j - 1, b)) : 0;
}
__device__ __forceinline__ int col0_M(int mode, int i, int a, int b) {
  if (i == 0) return 0;
  return (mode == BGK_GLOBAL) ? wadd(a, wmul(i - 1, b)) : 0;
}

}  // namespace bgk
