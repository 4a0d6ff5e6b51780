// Issue rate of the metric DP's step mix at the shader clock the GPU actually runs (round 6).
// profiles/r01/micro_valu_rates.txt converted kernel time to cycles at 2.4 GHz; the DP runs near
// 2.1 GHz under load (GRBM_GUI_ACTIVE), so its "4.4 cycles per instruction" ceiling was never
// measured in real cycles.  Here every wave stamps s_memtime (shader clock) and s_memrealtime
// (100 MHz) around its loop, so the table gives both the clock and the cycles per instruction.
// The mix is the tagged score-only step at R = 8: per row one v_add_u32_sdwa (diagonal + profile
// byte) and one v_max3_i32, per step one DPP (8 rows + 1 = 17 instructions), R rows chained as in
// the DP (the max3 of row k feeds row k + 1).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/issue_clock.hip -o tools/micro/issue_clock
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int R>
__global__ void k_step(int* out, unsigned long long* stamps, int iters) {
  int Y[R];
  for (int k = 0; k < R; ++k) Y[k] = threadIdx.x * (k + 1);
  int xl = threadIdx.x, top = threadIdx.x ^ 3, dIn0 = 5;
  const int prof0 = threadIdx.x * 0x01010101, prof1 = threadIdx.x * 0x02020202;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      int topX;
      asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(topX) : "v"(xl), "0"(top));
      int dIn = dIn0, xo = topX;
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int w = k < 4 ? prof0 : prof1;
        int d;
        asm volatile("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
                     : "=v"(d) : "v"(dIn), "v"(w));
        int best;
        asm volatile("v_max3_i32 %0, %1, %2, %3" : "=v"(best) : "v"(d), "v"(xo), "v"(Y[k]));
        dIn = Y[k];
        xo = best;
        Y[k] = best;
      }
      dIn0 = topX;
      xl = xo;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  int acc = xl;
  for (int k = 0; k < R; ++k) acc += Y[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) {
    const int wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    stamps[2 * wv] = t1 - t0;
    stamps[2 * wv + 1] = r1 - r0;
  }
}

template <int R>
static void run(int wavesPerSimd) {
  const int cus = 256, wpc = 4 * wavesPerSimd, iters = 4000;
  int* d;
  unsigned long long* st;
  (void)hipMalloc(&d, (size_t)cus * wpc * 64 * 4);
  (void)hipMalloc(&st, (size_t)cus * wpc * 16);
  hipLaunchKernelGGL(k_step<R>, dim3(cus), dim3(64 * wpc), 0, 0, d, st, 10);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_step<R>, dim3(cus), dim3(64 * wpc), 0, 0, d, st, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)cus * wpc * 2);
  (void)hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int w = 0; w < cus * wpc; ++w) { cyc += (double)h[2 * w]; rt += (double)h[2 * w + 1]; }
  cyc /= cus * wpc;
  rt /= cus * wpc;
  const double instr = (double)iters * 16 * (2 * R + 1);     // per wave
  const double ghz = cyc / (rt * 10.0);                      // s_memrealtime ticks at 100 MHz
  // the waves of one SIMD share its issue over the same interval
  std::printf("R=%2d waves/SIMD=%d  clock %.3f GHz  %.2f cycles per wave-instr per SIMD (shader clock)"
              "  %.2f at 2.4 GHz from the event time  (%.3f ms)\n",
              R, wavesPerSimd, ghz, cyc / (instr * wavesPerSimd), ms * 1e-3 * 2.4e9 / (instr * wavesPerSimd), ms);
  (void)hipFree(d);
  (void)hipFree(st);
}

int main() {
  for (int w : {1, 2, 4}) run<8>(w);
  for (int w : {1, 4}) run<5>(w);
  for (int w : {1, 4}) run<2>(w);
  return 0;
}
