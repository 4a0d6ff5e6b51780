// Microbenchmark: the packed two-strip score-only step (16-bit halves, v_pk_*) against the
// current 32-bit score-only step, both with their LDS operand reads (code row, profile entry,
// row-above broadcast) and the per-step output ring write, at several waves per CU.
//
// Packed step (lo half = strip 2m, hi half = strip 2m+1 running 64 steps behind it):
//   rot = wave_ror:1(Xlast); topX = v_perm(rot, topIn, sel)    (lane 0: lo <- topIn, hi <- lane 63's lo)
//   per row pair k: d = v_pk_add_u16(dIn, P[k]); m = v_pk_max_i16(d, Y[k]); best = v_pk_max_i16(m, xo)
// P[k] comes from a per-lane table indexed by the (lo column code, hi column code) combination.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int pk_add(int x, int y) { int r; asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y)); return r; }
__device__ __forceinline__ int pk_max(int x, int y) { int r; asm volatile("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y)); return r; }
__device__ __forceinline__ int vperm(int s0, int s1, int sel) { int r; asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(s0), "v"(s1), "v"(sel)); return r; }
__device__ __forceinline__ int ror1(int src) { return __builtin_amdgcn_update_dpp(0, src, 0x13c, 0xf, 0xf, false); }
__device__ __forceinline__ int shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }

template <int R> struct PV { int w[R]; };
template <int R>
__device__ __forceinline__ PV<R> ldp(const int* p) {
  PV<R> v;
  if constexpr (R == 4) { const int4 q = *reinterpret_cast<const int4*>(p); v.w[0] = q.x; v.w[1] = q.y; v.w[2] = q.z; v.w[3] = q.w; }
  else if constexpr (R == 2) { const int2 q = *reinterpret_cast<const int2*>(p); v.w[0] = q.x; v.w[1] = q.y; }
  else { for (int k = 0; k < R; ++k) v.w[k] = p[k]; }
  return v;
}

constexpr int kSteps = 4096;   // code row length per wave iteration

// LDS: code row (u16, shared), per wave: table 16 x 64 x R dwords, top row 64 ints, ring 256 ints
template <int R, int PF>
__global__ __launch_bounds__(1024) void pk_step(int* out, int iters) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
  uint16_t* codes = reinterpret_cast<uint16_t*>(smem);                   // kSteps + 64
  int* wl = smem + (kSteps + 64) / 2 + w * (16 * 64 * R + 64 + 256);
  int* tab = wl;
  int* top = wl + 16 * 64 * R;
  int* ring = top + 64;
  for (int x = threadIdx.x; x < kSteps + 64; x += blockDim.x) codes[x] = (uint16_t)(((x * 2654435761u) >> 13) & 15) * (64 * R * 4);
  for (int x = lane; x < 16 * 64 * R; x += 64) tab[x] = (int)((x * 0x9E3779B9u) & 0x00070007u);
  top[lane] = lane * 3;
  __syncthreads();
  (void)W;
  int Y[R];
#pragma unroll
  for (int k = 0; k < R; ++k) Y[k] = lane * (k + 1);
  int Xlast = 0, topPrev = 0;
  const int sel = lane == 0 ? 0x05040100 : 0x07060504;
  const char* tabLane = reinterpret_cast<const char*>(tab + lane * R);
  int* oLane = ring + 64 - lane;
  for (int it = 0; it < iters; ++it) {
    const uint16_t* cl = codes + 64 - lane;
    PV<R> qP[PF];
    int qC[PF], qT[PF];
#pragma unroll
    for (int d = 0; d < PF; ++d) { qP[d] = ldp<R>(reinterpret_cast<const int*>(tabLane + cl[d])); qC[d] = cl[PF + d]; qT[d] = top[d]; }
    for (int c = 0; c < kSteps / 64; ++c, cl += 64) {
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        const int s = u % PF;
        const PV<R> P = qP[s];
        const int topIn = qT[s];
        qP[s] = ldp<R>(reinterpret_cast<const int*>(tabLane + qC[s]));
        qC[s] = cl[u + 2 * PF];
        qT[s] = top[(u + PF) & 63];
        const int topX = vperm(ror1(Xlast), topIn, sel);
        int dIn = topPrev, xo = topX;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int yo = Y[k];
          const int best = pk_max(pk_max(pk_add(dIn, P.w[k]), yo), xo);
          dIn = yo; xo = best; Y[k] = best;
        }
        topPrev = topX;
        Xlast = xo;
        oLane[u & 127] = Xlast;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  int s = Xlast;
#pragma unroll
  for (int k = 0; k < R; ++k) s += Y[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the current 32-bit score-only step: R int8 profile bytes per lane (SDWA add), v_max3
template <int R>
__global__ __launch_bounds__(1024) void i32_step(int* out, int iters) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  constexpr int RW = R <= 4 ? 1 : 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint16_t* codes = reinterpret_cast<uint16_t*>(smem);
  int* wl = smem + (kSteps + 64) / 2 + w * (4 * 64 * RW + 64 + 256);
  int* tab = wl;
  int* top = wl + 4 * 64 * RW;
  int* ring = top + 64;
  for (int x = threadIdx.x; x < kSteps + 64; x += blockDim.x) codes[x] = (uint16_t)(((x * 2654435761u) >> 13) & 3) * (64 * RW * 4);
  for (int x = lane; x < 4 * 64 * RW; x += 64) tab[x] = (int)((x * 0x9E3779B9u) & 0x07070707u);
  top[lane] = lane * 3;
  __syncthreads();
  int Y[R];
#pragma unroll
  for (int k = 0; k < R; ++k) Y[k] = lane * (k + 1);
  int Xlast = 0, topPrev = 0;
  const char* tabLane = reinterpret_cast<const char*>(tab + lane * RW);
  int* oLane = ring + 64 - lane;
  for (int it = 0; it < iters; ++it) {
    const uint16_t* cl = codes + 64 - lane;
    int nP[RW], nC = cl[1], nT = top[0];
    for (int x = 0; x < RW; ++x) nP[x] = reinterpret_cast<const int*>(tabLane + cl[0])[x];
    for (int c = 0; c < kSteps / 64; ++c, cl += 64) {
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        int P[RW];
#pragma unroll
        for (int x = 0; x < RW; ++x) P[x] = nP[x];
        const int topIn = nT;
        if constexpr (RW == 2) { const int2 q = *reinterpret_cast<const int2*>(tabLane + nC); nP[0] = q.x; nP[1] = q.y; }
        else nP[0] = *reinterpret_cast<const int*>(tabLane + nC);
        nC = cl[u + 2];
        nT = top[(u + 1) & 63];
        const int topX = shr1(topIn, Xlast);
        int dIn = topPrev, xo = topX;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int yo = Y[k];
          const int d = dIn + __builtin_amdgcn_sbfe(P[k >> 2], 8 * (k & 3), 8);
          const int best = __builtin_elementwise_max(__builtin_elementwise_max(d, xo), yo);
          dIn = yo; xo = best; Y[k] = best;
        }
        topPrev = topX;
        Xlast = xo;
        oLane[u & 127] = Xlast;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  int s = Xlast;
#pragma unroll
  for (int k = 0; k < R; ++k) s += Y[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int wavesPerCU, int ldsPerWave, double cellsPerStepLane, int iters) {
  int* d;
  hipMalloc(&d, 256 * 1024 * 4 * 4);
  const int lds = (kSteps + 64) * 2 + wavesPerCU * ldsPerWave;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  kern<<<256, 64 * wavesPerCU, lds>>>(d, 1);
  if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed (lds %d)\n", name, lds); return; }
  hipEventRecord(e0);
  kern<<<256, 64 * wavesPerCU, lds>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double steps = (double)iters * kSteps;           // per wave
  const double cells = steps * 64 * cellsPerStepLane * wavesPerCU * 256;
  const double cyc = ms * 1e-3 * 2.1e9;                  // at the DP's ~2.1 GHz under load
  printf("%-14s waves/CU=%2d lds=%6d B  %.3f ms  %.0f Gcell/s  %.2f cycles/step/wave-per-SIMD  %.2f cycles per cell-lane\n",
         name, wavesPerCU, lds, ms, cells / (ms * 1e-3) / 1e9, cyc / (steps * wavesPerCU / 4.0),
         cyc / (steps * wavesPerCU / 4.0) / cellsPerStepLane);
  hipFree(d);
}

int main() {
  const int it = 40;
  run("i32 R=8", i32_step<8>, 16, (4 * 64 * 2 + 64 + 256) * 4, 8, it);
  run("i32 R=4", i32_step<4>, 16, (4 * 64 * 1 + 64 + 256) * 4, 4, it);
  run("pk R=4 PF1", pk_step<4, 1>, 8, (16 * 64 * 4 + 64 + 256) * 4, 8, it);
  run("pk R=4 PF2", pk_step<4, 2>, 8, (16 * 64 * 4 + 64 + 256) * 4, 8, it);
  run("pk R=4 PF2", pk_step<4, 2>, 4, (16 * 64 * 4 + 64 + 256) * 4, 8, it);
  run("pk R=3 PF2", pk_step<3, 2>, 12, (16 * 64 * 3 + 64 + 256) * 4, 6, it);
  run("pk R=3 PF1", pk_step<3, 1>, 12, (16 * 64 * 3 + 64 + 256) * 4, 6, it);
  run("pk R=2 PF2", pk_step<2, 2>, 16, (16 * 64 * 2 + 64 + 256) * 4, 4, it);
  run("pk R=2 PF1", pk_step<2, 1>, 16, (16 * 64 * 2 + 64 + 256) * 4, 4, it);
  return 0;
}
