// Microbenchmark: the tagged DP step (bg_tag_kernel.hip) on registers only — no LDS, no HBM,
// no strip pipeline — to separate the cell arithmetic's own issue rate from everything else.
// Per cell: v_add_u32_sdwa (diagonal + profile byte), v_max3, v_alignbit, v_or, v_add; per step
// one DPP and one v_add per profile dword (stands in for the kernel's per-step ds_read).
// ILP=2 interleaves two independent half-height strips in one wave.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int dpp_shr1(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);
}

template <int R, int ILP>
__global__ __launch_bounds__(1024) void tag_step(int* out, int iters, int a4x) {
  constexpr int RW = (R + 3) / 4;
  int Y[ILP][R], prof[ILP][RW];
  unsigned tA[ILP][R];
  int topPrev[ILP], Xlast[ILP];
#pragma unroll
  for (int g = 0; g < ILP; ++g) {
#pragma unroll
    for (int k = 0; k < R; ++k) {
      Y[g][k] = threadIdx.x * (k + 1) + g;
      tA[g][k] = 0;
    }
#pragma unroll
    for (int w = 0; w < RW; ++w) prof[g][w] = (int)(threadIdx.x * 0x01030507u) ^ (a4x * (w + 1 + g));
    topPrev[g] = 0;
    Xlast[g] = 1;
  }
  int code = (threadIdx.x & 3) * 8;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int g = 0; g < ILP; ++g) {
        int P[RW];
#pragma unroll
        for (int w = 0; w < RW; ++w) P[w] = prof[g][w] + code + u;
        const int topX = dpp_shr1(topPrev[g] + u, Xlast[g]);
        int dIn = topPrev[g];
        int xo = topX;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int yo = Y[g][k];
          const int d = dIn + __builtin_amdgcn_sbfe(P[k >> 2], 8 * (k & 3), 8);
          const int best = __builtin_elementwise_max(__builtin_elementwise_max(d, xo), yo);
          tA[g][k] = __builtin_amdgcn_alignbit((unsigned)best, tA[g][k], 2);
          asm volatile("" : "+v"(tA[g][k]));
          const int yn = best | 3;
          dIn = yo;
          xo = yn - 1;
          Y[g][k] = yn;
        }
        topPrev[g] = topX;
        Xlast[g] = xo;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    code = (code + 8) & 24;
  }
  int s = 0;
#pragma unroll
  for (int g = 0; g < ILP; ++g)
#pragma unroll
    for (int k = 0; k < R; ++k) s += Y[g][k] + (int)tA[g][k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + a4x;
}

template <int R, int ILP>
void run(int wavesPerCU) {
  int* d;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  const int iters = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  tag_step<R, ILP><<<256, 64 * wavesPerCU>>>(d, 4, 5);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  tag_step<R, ILP><<<256, 64 * wavesPerCU>>>(d, iters, 5);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double steps = (double)iters * 16 * ILP;             // per wave
  const double instr = (double)iters * 16 * ILP * (5.0 * R + 1 + (R + 3) / 4);  // per wave
  const double perSimd = instr * wavesPerCU / 4.0;
  const double cells = steps * R * 64 * wavesPerCU * 256.0;
  printf("R=%2d ILP=%d waves/CU=%2d  %.2f cycles per wave-instr per SIMD @2.4GHz   %.2f Tcells/s\n", R, ILP,
         wavesPerCU, ms * 1e-3 * 2.4e9 / perSimd, cells / (ms * 1e-3) / 1e12);
  (void)hipFree(d);
}

int main() {
  for (int w : {4, 8, 12, 16}) run<4, 1>(w);
  for (int w : {4, 8, 12, 16}) run<5, 1>(w);
  for (int w : {4, 8, 12, 16}) run<8, 1>(w);
  for (int w : {4, 8, 12}) run<10, 1>(w);
  return 0;
}
