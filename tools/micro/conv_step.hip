// Microbenchmark: the WIDE conveyor step (score_chunk_conv in bg_tag_common.h) for ONE wave per
// SIMD, with its per-step operands from LDS (profile entry by scaled code + the code itself, as
// the kernel) versus from registers (a lane's 16 upcoming column codes in one 2-bit packed word
// refilled every 16 steps from a packed LDS row; the R profile bytes picked by v_perm_b32 from
// per-row dwords holding the four codes' bytes, two rows per v_perm).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int shl1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false); }
__device__ __forceinline__ int add_sbyte(int x, int w, int sel) { return x + __builtin_amdgcn_sbfe(w, 8 * sel, 8); }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

constexpr int kSteps = 4096;

template <int R, bool PERM>
__global__ __launch_bounds__(256) void conv(int* out, int iters) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int RW = R <= 4 ? 1 : 2;
  uint16_t* codes = reinterpret_cast<uint16_t*>(smem);                    // kSteps + 192 u16
  uint32_t* packed = reinterpret_cast<uint32_t*>(smem) + (kSteps + 192) / 2;   // (kSteps + 192) / 16
  int* tab = reinterpret_cast<int*>(packed + (kSteps + 192) / 16) + w * 4 * 64 * RW;
  for (int x = threadIdx.x; x < kSteps + 192; x += blockDim.x)
    codes[x] = (uint16_t)((((x * 2654435761u) >> 13) & 3) * 32 * RW);
  __syncthreads();
  for (int x = threadIdx.x; x < (kSteps + 192) / 16; x += blockDim.x) {
    uint32_t v = 0;
    for (int j = 0; j < 16; ++j) v |= (uint32_t)(codes[16 * x + j] / (32 * RW)) << (2 * j);
    packed[x] = v;
  }
  for (int x = lane; x < 4 * 64 * RW; x += 64) tab[x] = (int)((x * 0x9E3779B9u) & 0x07070707u);
  __syncthreads();
  int B[R];
#pragma unroll
  for (int k = 0; k < R; ++k) B[k] = (int)(((lane + k) * 0x9E3779B9u) & 0x07070707u);
  int Y[R];
#pragma unroll
  for (int k = 0; k < R; ++k) Y[k] = lane * (k + 1);
  int Xlast = 0, topPrev = 0, Q = lane;
  const uint8_t* profLane = reinterpret_cast<const uint8_t*>(tab + lane * RW);
  for (int it = 0; it < iters; ++it) {
    for (int c = 0; c < kSteps / 64; ++c) {
      const uint16_t* cl = codes + 64 * c + 63 - lane;
      constexpr int PF = 4;
      int qCode[PF];
      int qP[PF][RW];
      uint32_t cw = 0, nlo = 0, nhi = 0;
      int col = 64 * c + 63 - lane;                                        // + u: this lane's column
      if constexpr (!PERM) {
#pragma unroll
        for (int d = 0; d < PF; ++d) {
          const uint8_t* p = profLane + cl[d];
          qP[d][0] = *reinterpret_cast<const int*>(p);
          if constexpr (RW == 2) qP[d][1] = *reinterpret_cast<const int*>(p + 4);
          qCode[d] = cl[PF + d];
        }
        cl += 2 * PF;
      } else {
        const int wd = col >> 4;
        nlo = packed[wd]; nhi = packed[wd + 1];
      }
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        int P0 = 0, P1 = 0;
        int PP[(R + 1) / 2];
        if constexpr (!PERM) {
          const int s = u % PF;
          P0 = qP[s][0];
          if constexpr (RW == 2) P1 = qP[s][1];
          const uint8_t* p = profLane + qCode[s];
          qP[s][0] = *reinterpret_cast<const int*>(p);
          if constexpr (RW == 2) qP[s][1] = *reinterpret_cast<const int*>(p + 4);
          qCode[s] = cl[u];
        } else {
          if (u % 16 == 0) {
            cw = __builtin_amdgcn_alignbit(nhi, nlo, (uint32_t)(2 * (col + u)));   // 16 codes from column col + u
            if (u + 16 < 64 + 16) {
              const int wd = (col + u + 16) >> 4;
              nlo = packed[wd]; nhi = packed[wd + 1];
            }
          }
          const uint32_t code = __builtin_amdgcn_ubfe(cw, 2 * (u % 16), 2);
          const uint32_t sel = code * 0x0101u + 0x0400u;
#pragma unroll
          for (int m = 0; m < (R + 1) / 2; ++m)
            PP[m] = (int)__builtin_amdgcn_perm((uint32_t)B[2 * m + 1 < R ? 2 * m + 1 : 2 * m], (uint32_t)B[2 * m], sel);
        }
        const int topX = shr1(Q, Xlast);
        Q = shl1(Xlast, Q);
        int dIn = topPrev, xo = topX;
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const int yo = Y[k];
          int d;
          if constexpr (PERM) d = add_sbyte(dIn, PP[k >> 1], k & 1);
          else d = add_sbyte(dIn, k < 4 ? P0 : P1, k & 3);
          const int best = imax(imax(d, xo), yo);
          dIn = yo; xo = best; Y[k] = best;
        }
        topPrev = topX;
        Xlast = xo;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  int s = Xlast + Q;
#pragma unroll
  for (int k = 0; k < R; ++k) s += Y[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int iters) {
  int* d;
  (void)hipMalloc(&d, 256 * 256 * 4);
  const int lds = (kSteps + 192) * 2 + (kSteps + 192) / 16 * 4 + 4 * 4 * 64 * 2 * 4;
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
  fflush(stdout);
  (void)hipFree(d);
}

int main() {
  const int it = 100;
  run("R=5 conv LDS", conv<5, false>, it);
  run("R=5 conv perm", conv<5, true>, it);
  run("R=4 conv LDS", conv<4, false>, it);
  run("R=4 conv perm", conv<4, true>, it);
  run("R=8 conv LDS", conv<8, false>, it);
  run("R=8 conv perm", conv<8, true>, it);
  run("R=2 conv LDS", conv<2, false>, it);
  run("R=2 conv perm", conv<2, true>, it);
  return 0;
}
