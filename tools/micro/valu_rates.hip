// Issue-rate table for the VALU ops the DP kernel uses (gfx950): cycles per wave64 instruction
// per SIMD with 8 independent chains per wave and 4 waves per SIMD (16 waves per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define OPS(name, expr)                                                                      \
  __global__ void k_##name(int* out, int iters) {                                             \
    int x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,    \
        x6 = x0 + 6, x7 = x0 + 7;                                                              \
    const int y = threadIdx.x ^ 5, z = threadIdx.x * 7;                                        \
    for (int it = 0; it < iters; ++it) {                                                       \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                         \
        asm volatile(expr : "+v"(x0) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x1) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x2) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x3) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x4) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x5) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x6) : "v"(y), "v"(z));                                        \
        asm volatile(expr : "+v"(x7) : "v"(y), "v"(z));                                        \
      }                                                                                        \
    }                                                                                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;        \
  }

OPS(add_u32, "v_add_u32 %0, %0, %1")
OPS(and_b32, "v_and_b32 %0, %0, %1")
OPS(or_b32, "v_or_b32 %0, %0, %1")
OPS(sub_u32, "v_sub_u32 %0, %0, %1")
OPS(lshlrev, "v_lshlrev_b32 %0, %1, %0")
OPS(max_i32, "v_max_i32 %0, %0, %1")
OPS(max_u32, "v_max_u32 %0, %0, %1")
OPS(max_f32, "v_max_f32 %0, %0, %1")
OPS(max3_i32, "v_max3_i32 %0, %0, %1, %2")
OPS(med3_i32, "v_med3_i32 %0, %0, %1, %2")
OPS(bfe_u32, "v_bfe_u32 %0, %1, %0, 8")
OPS(perm_b32, "v_perm_b32 %0, %1, %2, %0")
OPS(mad_u24, "v_mad_u32_u24 %0, %0, 4, %1")
OPS(lshl_add, "v_lshl_add_u32 %0, %0, 2, %1")
OPS(cmp_e32, "v_cmp_eq_u32 vcc, %0, %1\n v_add_u32 %0, %0, %2")
OPS(cmp_e64, "v_cmp_eq_u32_e64 s[40:41], %0, %1\n v_add_u32 %0, %0, %2")
OPS(addc_e32, "v_addc_co_u32 %0, vcc, %0, %0, vcc")
OPS(addc_e64, "v_addc_co_u32_e64 %0, s[42:43], %0, %0, s[40:41]")
OPS(cnd_e64, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]")
OPS(mov_dpp, "v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf")
OPS(add_dpp, "v_add_u32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf")
OPS(readlane, "v_readlane_b32 s44, %0, 5\n v_add_u32 %0, s44, %0")
OPS(max3_f32, "v_max3_f32 %0, %0, %1, %2")
OPS(pk_max_i16, "v_pk_max_i16 %0, %0, %1")
OPS(pk_add_u16, "v_pk_add_u16 %0, %0, %1")

OPS(add_sdwa, "v_add_u32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")
OPS(add_sdwa_w, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1")
OPS(max_sdwa, "v_max_i32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
OPS(mov_sdwa_pres, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD")
OPS(add3_u32, "v_add3_u32 %0, %0, %1, %2")
OPS(xor_b32, "v_xor_b32 %0, %0, %1")
OPS(mov_b32, "v_mov_b32 %0, %1\n v_add_u32 %0, %0, %2")
OPS(lshrrev, "v_lshrrev_b32 %0, %1, %0")
OPS(ashrrev, "v_ashrrev_i32 %0, 2, %0")
OPS(alignbit, "v_alignbit_b32 %0, %1, %0, 2")
OPS(or3_b32, "v_or3_b32 %0, %0, %1, %2")
OPS(and_or, "v_and_or_b32 %0, %0, %1, %2")
OPS(cnd_e32, "v_cndmask_b32 %0, %0, %1, vcc")
OPS(add_co, "v_add_co_u32 %0, vcc, %0, %1")
OPS(sub_co, "v_sub_co_u32 %0, vcc, %0, %1")
OPS(max_i16, "v_max_i16 %0, %0, %1")
OPS(add_u16, "v_add_u16 %0, %0, %1")
OPS(min_i32, "v_min_i32 %0, %0, %1")
OPS(bfe_i32, "v_bfe_i32 %0, %1, %0, 8")
OPS(add_k, "v_add_u32 %0, 0x1234, %0")
OPS(and_k, "v_and_b32 %0, -4, %0")
OPS(max_k, "v_max_i32 %0, 7, %0")
OPS(sad_u8, "v_sad_u8 %0, %0, %1, %2")
OPS(pk_max_i16x, "v_pk_max_i16 %0, %0, %1 op_sel_hi:[1,1]")
OPS(mul_lo_u16, "v_mul_lo_u16 %0, %0, %1")
OPS(max_f16, "v_max_f16 %0, %0, %1")
OPS(add_f32, "v_add_f32 %0, %0, %1")


// round 2: 16-bit forms and encodings for a half-width DP
OPS(max3_i16, "v_max3_i16 %0, %0, %1, %2")
OPS(add_u16_sdwa, "v_add_u16_sdwa %0, %0, sext(%1) dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:BYTE_1")
OPS(max_i16_e64, "v_max_i16_e64 %0, %0, %1")
OPS(max_i32_e64, "v_max_i32_e64 %0, %0, %1")
OPS(add_u32_e64, "v_add_u32_e64 %0, %0, %1")
OPS(max_i16_dpp, "v_max_i16_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf")
OPS(sub_u16, "v_sub_u16 %0, %0, %1")
OPS(max_u16, "v_max_u16 %0, %0, %1")
OPS(max_i32_sw, "v_max_i32 %0, %1, %0")
OPS(pk_add_i16, "v_pk_add_i16 %0, %0, %1")
OPS(max_i16_sdwa, "v_max_i16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1")
OPS(add_u16_k, "v_add_u16 %0, 7, %0")
OPS(min_i16, "v_min_i16 %0, %0, %1")
OPS(med3_i16, "v_med3_i16 %0, %0, %1, %2")
OPS(max3_u32, "v_max3_u32 %0, %0, %1, %2")
OPS(subrev_u32, "v_subrev_u32 %0, %1, %0")
OPS(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
OPS(max_f32_sw, "v_max_f32 %0, %1, %0")
OPS(min_f32, "v_min_f32 %0, %0, %1")
OPS(pk_max_f16, "v_pk_max_f16 %0, %0, %1")
OPS(max_i16_mix, "v_max_i16 %0, %0, %1\n v_max_i32 %0, %0, %2")

// op_sel (VOP3 16-bit half selects)
OPS(add_u16_opsel, "v_add_i16 %0, %0, %1 op_sel:[0,1,0]")
OPS(max_i16_opsel, "v_add_i16 %0, %0, %1")
OPS(max_i16_opsel_d, "v_mad_u16 %0, %0, %1, %2 op_sel:[0,1,0,0]")
OPS(add_u16_e64, "v_add_u16_e64 %0, %0, %1")
OPS(add_i16_clamp, "v_add_i16 %0, %0, %1 clamp")
OPS(sub_i16_clamp, "v_sub_i16 %0, %0, %1 clamp")
OPS(max_i16_k, "v_max_i16 %0, -5, %0")

typedef void (*kfn)(int*, int);
static void run(const char* name, kfn f, int wavesPerCU) {
  int* d;
  (void)hipMalloc(&d, 256 * 1024 * 4);
  const int iters = 2000;
  hipLaunchKernelGGL(f, dim3(256), dim3(64 * wavesPerCU), 0, 0, d, 10);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(f, dim3(256), dim3(64 * wavesPerCU), 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double perSimd = (double)iters * 16 * 8 * wavesPerCU / 4.0;
  printf("%-12s waves/SIMD=%d  %.2f cycles per wave-instr per SIMD (at 2.4 GHz)\n", name, wavesPerCU / 4,
         ms * 1e-3 * 2.4e9 / perSimd);
  (void)hipFree(d);
}

int main() {
#define R(n) run(#n, k_##n, 16);
  R(add_u32) R(and_b32) R(or_b32) R(sub_u32) R(lshlrev) R(max_i32) R(max_u32) R(max_f32) R(max3_i32)
  R(med3_i32) R(bfe_u32) R(perm_b32) R(mad_u24) R(lshl_add) R(cmp_e32) R(cmp_e64) R(addc_e32)
  R(addc_e64) R(cnd_e64) R(mov_dpp) R(add_dpp) R(readlane) R(max3_f32) R(pk_max_i16) R(pk_add_u16)
  R(add_sdwa) R(add_sdwa_w) R(max_sdwa) R(mov_sdwa_pres) R(add3_u32) R(xor_b32) R(mov_b32) R(lshrrev)
  R(ashrrev) R(alignbit) R(or3_b32) R(and_or) R(cnd_e32) R(add_co) R(sub_co) R(max_i16) R(add_u16)
  R(min_i32) R(bfe_i32) R(add_k) R(and_k) R(max_k) R(sad_u8) R(pk_max_i16x) R(mul_lo_u16) R(max_f16) R(add_f32)
  if (getenv("R2ONLY")) {}
  R(max3_i16) R(add_u16_sdwa) R(max_i16_e64) R(max_i32_e64) R(add_u32_e64) R(max_i16_dpp) R(sub_u16)
  R(max_u16) R(max_i32_sw) R(pk_add_i16) R(max_i16_sdwa) R(add_u16_k) R(min_i16) R(med3_i16)
  R(max3_u32) R(subrev_u32) R(mul_u32_u24) R(max_f32_sw) R(min_f32) R(pk_max_f16) R(max_i16_mix)
  R(add_u16_opsel) R(max_i16_opsel) R(max_i16_opsel_d) R(add_u16_e64) R(add_i16_clamp) R(sub_i16_clamp) R(max_i16_k)
  return 0;
}
