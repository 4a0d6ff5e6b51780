// Microbenchmark: how fast ONE wave runs a dependent scalar (SALU) chain on gfx950, with and
// without a v_readlane feeding it — the cost model of a scalar traceback walk (one move = a
// handful of dependent s_ ops plus a readlane of the decoded trace word).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void salu(int* out, int iters, int seed) {
  int a = seed, b = seed * 3 + 1;
  const int v = threadIdx.x * 7 + seed;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (KIND == 0) {          // 8 dependent s_add / s_xor
        asm volatile(
            "s_add_u32 %0, %0, %1\n s_xor_b32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_xor_b32 %0, %0, %1\n"
            "s_add_u32 %0, %0, %1\n s_xor_b32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_xor_b32 %0, %0, %1\n"
            : "+s"(a) : "s"(b) : "scc");
      } else if constexpr (KIND == 1) {   // 8 independent s_ ops (2 chains interleaved)
        asm volatile(
            "s_add_u32 %0, %0, %2\n s_add_u32 %1, %1, %2\n s_xor_b32 %0, %0, %2\n s_xor_b32 %1, %1, %2\n"
            "s_add_u32 %0, %0, %2\n s_add_u32 %1, %1, %2\n s_xor_b32 %0, %0, %2\n s_xor_b32 %1, %1, %2\n"
            : "+s"(a), "+s"(b) : "s"(seed) : "scc");
      } else if constexpr (KIND == 2) {   // readlane (index from the chain) + 7 dependent s_ ops
        asm volatile(
            "s_and_b32 %0, %0, 63\n s_nop 3\n v_readlane_b32 %0, %2, %0\n s_lshr_b32 %0, %0, 1\n s_and_b32 %0, %0, 0xffff\n"
            "s_flbit_i32_b32 %0, %0\n s_add_u32 %0, %0, %1\n s_xor_b32 %0, %0, %1\n"
            : "+s"(a) : "s"(b), "v"(v) : "scc");
      } else {                            // 8 dependent s_ ops with 64-bit shifts / bfm / flbit
        asm volatile(
            "s_bfm_b32 %0, %0, 0\n s_and_b32 %0, %0, %1\n s_flbit_i32_b32 %0, %0\n s_and_b32 %0, %0, 31\n"
            "s_lshr_b32 %0, %1, %0\n s_and_b32 %0, %0, 31\n s_add_u32 %0, %0, 1\n s_and_b32 %0, %0, 31\n"
            : "+s"(a) : "s"(b) : "scc");
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b;
}

template <int KIND>
void run(const char* name, int wavesPerSimd) {
  int* d;
  (void)hipMalloc(&d, 1024 * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int iters = 2000;
  salu<KIND><<<256, 256 * wavesPerSimd>>>(d, 10, 1);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  salu<KIND><<<256, 256 * wavesPerSimd>>>(d, iters, 1);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double instr = (double)iters * 16 * 8;     // per wave
  printf("%-28s waves/SIMD=%d  %.2f cycles per instruction per wave (2.4 GHz)\n", name, wavesPerSimd,
         ms * 1e-3 * 2.4e9 / instr);
  fflush(stdout);
  (void)hipFree(d);
}

int main() {
  printf("start\n"); fflush(stdout);
  run<0>("dependent s_add/s_xor", 1);
  run<1>("two interleaved chains", 1);
  run<2>("readlane + 7 dependent s_", 1);
  run<3>("bfm/flbit/lshr chain", 1);
  run<0>("dependent s_add/s_xor", 4);
  return 0;
}
