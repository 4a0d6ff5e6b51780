// Finish kernel instantiations for grouped pairs (bg_grp_kernel.hip): the end cell (the DP folded
// the last row's key), the traceback over chunks recomputed as 16-lane jobs (bg_finish.h
// recompute_grp) and the string assembly.  Own translation unit: its registers stay out of the
// other checkpoint kernels, and the library's kernel objects build in parallel.
#include <algorithm>

#include "bg_finish.h"

template <int R>
static void* finish_grp_ptr(int mode) {
  switch (mode) {
    case BGK_GLOBAL: return (void*)&bg_finish_kernel<R, false, BGK_GLOBAL, true, true>;
    case BGK_FITTING: return (void*)&bg_finish_kernel<R, false, BGK_FITTING, true, true>;
    case BGK_OVERLAP: return (void*)&bg_finish_kernel<R, false, BGK_OVERLAP, true, true>;
    case BGK_SEMIGLOBAL: return (void*)&bg_finish_kernel<R, false, BGK_SEMIGLOBAL, true, true>;
    default: return nullptr;
  }
}

extern "C" void* bg_finish_grp_kernel_ptr(int R, int mode) {
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

// the same for grouped pairs (BgFinishArgs::grouped): kGrpSlots 16-lane chunk slots
extern "C" size_t bg_finish_grp_lds_bytes(int R, int nslots, int nw, int* win_bytes) {
  int slot = 0, area = 0;
  switch (R) {
    case 2: slot = ck_grp_slot_dw<2>(); area = ck_grp_wave_ints<2>(); break;
    case 3: slot = ck_grp_slot_dw<3>(); area = ck_grp_wave_ints<3>(); break;
    case 4: slot = ck_grp_slot_dw<4>(); area = ck_grp_wave_ints<4>(); break;
    case 5: slot = ck_grp_slot_dw<5>(); area = ck_grp_wave_ints<5>(); break;
    case 8: slot = ck_grp_slot_dw<8>(); area = ck_grp_wave_ints<8>(); break;
    default: slot = ck_grp_slot_dw<10>(); area = ck_grp_wave_ints<10>(); break;
  }
  const int ns = (nslots > 0 && nslots < kGrpSlots) ? nslots : kGrpSlots;
  *win_bytes = std::max(ns * slot * 4, 2 * 256 * 4);
  return (size_t)*win_bytes + 64 * 4 + (size_t)nw * area * 4 + kCkMapEntries * 4;
}

