// Microbenchmark: throughput of dependent VALU chains on gfx950 vs independent chains per wave
// and waves per SIMD.  Each "cell" is the tagged-kernel chain max3 -> add -> and -> or.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int CH>
__global__ void chain(int* out, int iters, int c0) {
  int x[CH], y = threadIdx.x, z = threadIdx.x * 3;
#pragma unroll
  for (int i = 0; i < CH; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        int m = __builtin_elementwise_max(__builtin_elementwise_max(x[i], y), z);
        m = m + c0;
        x[i] = (m & ~3) | 1;
      }
    }
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < CH; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
void run(int wavesPerCU) {
  int* d;
  hipMalloc(&d, 256 * 1024 * 4 * 4);
  const int iters = 4000 / CH;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  chain<CH><<<256, 64 * wavesPerCU>>>(d, 10, 1);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  chain<CH><<<256, 64 * wavesPerCU>>>(d, iters, 1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // VALU ops per wave: iters * 8 * CH * 3 (max3, add, and-or -> compiled as 3 or 4)
  double waveInstr = (double)iters * 8 * CH * 4;
  double perSimd = waveInstr * wavesPerCU / 4.0;
  double cycles = ms * 1e-3 * 2.4e9;
  printf("chains/wave=%d waves/CU=%2d  ms=%7.3f  cycles per wave-instr per SIMD=%.2f  (2.0 = VALU peak)\n",
         CH, wavesPerCU, ms, cycles / perSimd);
  hipFree(d);
}

int main() {
  for (int w : {4, 8, 16, 32}) run<1>(w);
  for (int w : {4, 8, 16}) run<2>(w);
  for (int w : {4, 8, 16}) run<4>(w);
  return 0;
}
