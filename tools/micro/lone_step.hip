// Microbenchmark: step latency of ONE wave per SIMD running the score-only step (score_chunk in
// bg_tag_common.h) — the regime of C3's WIDE pipeline, where each strip is a lone wave and the
// DP's critical path is (2 n1 / R + n2) steps of this latency.  Variants: operands from LDS with
// a prefetch depth PF (as the kernel), and registers only (no LDS at all).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int add_sbyte(int x, int w, int sel) { return x + __builtin_amdgcn_sbfe(w, 8 * sel, 8); }

constexpr int kSteps = 4096;

template <int R, int PF, bool LDS>
__global__ __launch_bounds__(256) void lone(int* out, int iters) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint16_t* codes = reinterpret_cast<uint16_t*>(smem);
  int* wl = smem + (kSteps + 128) / 2 + w * (4 * 64 + 64 + 256);
  int* tab = wl;
  int* top = wl + 4 * 64;
  int* ring = top + 64;
  for (int x = threadIdx.x; x < kSteps + 128; x += blockDim.x) codes[x] = (uint16_t)(((x * 2654435761u) >> 13) & 3) * 256;
  for (int x = lane; x < 4 * 64; x += 64) tab[x] = (int)((x * 0x9E3779B9u) & 0x07070707u);
  top[lane] = lane * 3;
  __syncthreads();
  int Y[R];
#pragma unroll
  for (int k = 0; k < R; ++k) Y[k] = lane * (k + 1);
  int Xlast = 0, topPrev = 0;
  const char* tabLane = reinterpret_cast<const char*>(tab + lane);
  int* oLane = ring + 64 - lane;
  int regP = (int)(lane * 0x01020304u), regT = lane;
  for (int it = 0; it < iters; ++it) {
    const uint16_t* cl = codes + 64 - lane;
    int qP[PF], qC[PF], qT[PF];
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      qP[d] = LDS ? *reinterpret_cast<const int*>(tabLane + cl[d]) : regP + d;
      qC[d] = LDS ? cl[PF + d] : d * 256;
      qT[d] = LDS ? top[d] : regT + d;
    }
    for (int c = 0; c < kSteps / 64; ++c, cl += 64) {
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        const int s = u % PF;
        const int P = qP[s];
        const int topIn = qT[s];
        if constexpr (LDS) {
          qP[s] = *reinterpret_cast<const int*>(tabLane + qC[s]);
          qC[s] = cl[u + 2 * PF];
          qT[s] = top[(u + PF) & 63];
        } else {
          qP[s] = P ^ qC[s];
          qT[s] = topIn + 1;
        }
        const int topX = shr1(topIn, Xlast);
        int dIn = topPrev, xo = topX;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int yo = Y[k];
          const int d = add_sbyte(dIn, P, k & 3);
          const int best = __builtin_elementwise_max(__builtin_elementwise_max(d, xo), yo);
          dIn = yo; xo = best; Y[k] = best;
        }
        topPrev = topX;
        Xlast = xo;
        if constexpr (LDS) oLane[u & 127] = Xlast;
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
void run(const char* name, K kern, int iters) {
  int* d;
  (void)hipMalloc(&d, 256 * 256 * 4);
  const int lds = (kSteps + 128) * 2 + 4 * (4 * 64 + 64 + 256) * 4;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  kern<<<256, 256, lds>>>(d, 1);
  if (hipDeviceSynchronize() != hipSuccess) { printf("%s failed\n", name); return; }
  (void)hipEventRecord(e0);
  kern<<<256, 256, lds>>>(d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double steps = (double)iters * kSteps;
  printf("%-22s %.3f ms  %.1f cycles per step at 2.4 GHz (one wave per SIMD)\n", name, ms, ms * 1e-3 * 2.4e9 / steps);
  (void)hipFree(d);
}

int main() {
  const int it = 100;
  run("R=2 regs", lone<2, 1, false>, it);
  run("R=2 LDS PF=1", lone<2, 1, true>, it);
  run("R=2 LDS PF=2", lone<2, 2, true>, it);
  run("R=2 LDS PF=4", lone<2, 4, true>, it);
  run("R=2 LDS PF=8", lone<2, 8, true>, it);
  run("R=4 regs", lone<4, 1, false>, it);
  run("R=4 LDS PF=4", lone<4, 4, true>, it);
  run("R=1 regs", lone<1, 1, false>, it);
  run("R=1 LDS PF=4", lone<1, 4, true>, it);
  run("R=1 LDS PF=8", lone<1, 8, true>, it);
  return 0;
}
