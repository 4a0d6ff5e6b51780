// Finish kernel instantiations for grouped pairs (bg_grp_kernel.hip), BG_GRP_P pairs per wave (the
// Makefile builds this file once for 4 and once for 2): the end cell (semiglobal / overlap: the
// DP folded the last row's key), the traceback over chunks recomputed as 64 / P-lane jobs
// (bg_finish.h recompute_grp) and the string assembly.  Own translation units: their registers
// stay out of the other checkpoint kernels, and the library's kernel objects build in parallel.
#include <algorithm>

#include "bg_finish.h"

#ifndef BG_GRP_P
#define BG_GRP_P 4
#endif
#define BG_CAT2(a, b, c) a##b##c
#define BG_CAT(a, b, c) BG_CAT2(a, b, c)

template <int R>
static void* finish_grp_ptr(int mode) {
  switch (mode) {
    case BGK_GLOBAL: return (void*)&bg_finish_kernel<R, false, BGK_GLOBAL, true, BG_GRP_P>;
    case BGK_FITTING: return (void*)&bg_finish_kernel<R, false, BGK_FITTING, true, BG_GRP_P>;
    case BGK_OVERLAP: return (void*)&bg_finish_kernel<R, false, BGK_OVERLAP, true, BG_GRP_P>;
    case BGK_SEMIGLOBAL: return (void*)&bg_finish_kernel<R, false, BGK_SEMIGLOBAL, true, BG_GRP_P>;
    default: return nullptr;
  }
}

// bg_finish_grp4_kernel_ptr / bg_finish_grp2_kernel_ptr
extern "C" void* BG_CAT(bg_finish_grp, BG_GRP_P, _kernel_ptr)(int R, int mode) {
  switch (R) {
    case 2: return finish_grp_ptr<2>(mode);
    case 3: return finish_grp_ptr<3>(mode);
    case 4: return finish_grp_ptr<4>(mode);
    case 5: return finish_grp_ptr<5>(mode);
    case 8: return finish_grp_ptr<8>(mode);
    case 10: return finish_grp_ptr<10>(mode);
    default: return nullptr;
  }
}

template <int R>
static int grp_slot_dw(int P) { return P == 2 ? ck_grp_slot_dw<R, 2>() : ck_grp_slot_dw<R, 4>(); }

// LDS of the grouped finish (P pairs per wave) with `nslots` chunk slots (0: kGrpSlots) and `nw`
// waves: chunk slots (the scan aliases them), scalars, nw recompute areas, the chunk map
extern "C" size_t BG_CAT(bg_finish_grp, BG_GRP_P, _lds_bytes)(int R, int nslots, int nw, int* win_bytes) {
  int slot = 0, area = 0;
  switch (R) {
    case 2: slot = grp_slot_dw<2>(BG_GRP_P); area = ck_grp_wave_ints<2>(); break;
    case 3: slot = grp_slot_dw<3>(BG_GRP_P); area = ck_grp_wave_ints<3>(); break;
    case 4: slot = grp_slot_dw<4>(BG_GRP_P); area = ck_grp_wave_ints<4>(); break;
    case 5: slot = grp_slot_dw<5>(BG_GRP_P); area = ck_grp_wave_ints<5>(); break;
    case 8: slot = grp_slot_dw<8>(BG_GRP_P); area = ck_grp_wave_ints<8>(); break;
    default: slot = grp_slot_dw<10>(BG_GRP_P); area = ck_grp_wave_ints<10>(); break;
  }
  const int ns = (nslots > 0 && nslots < kGrpSlots) ? nslots : kGrpSlots;
  *win_bytes = std::max(ns * slot * 4, 2 * 256 * 4);
  return (size_t)*win_bytes + 64 * 4 + (size_t)nw * area * 4 + kCkMapEntries * 4;
}
