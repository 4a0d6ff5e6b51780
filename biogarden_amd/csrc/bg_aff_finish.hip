// Finish kernel instantiations for the affine / local checkpoint path (bg_aff_kernel.hip): the
// end cell, the traceback over chunks recomputed with the reference's full trace (x_trace and
// y_trace included, aligner.rs:441-507) and the string assembly.  Own translation unit so the
// library's kernel objects build in parallel.
#include <algorithm>

#include "bg_finish.h"

template <int R>
static void* finish_ack_ptr(int mode) {
  switch (mode) {
    case BGK_GLOBAL: return (void*)&bg_finish_kernel<R, true, BGK_GLOBAL, true>;
    case BGK_LOCAL: return (void*)&bg_finish_kernel<R, true, BGK_LOCAL, true>;
    case BGK_FITTING: return (void*)&bg_finish_kernel<R, true, BGK_FITTING, true>;
    case BGK_OVERLAP: return (void*)&bg_finish_kernel<R, true, BGK_OVERLAP, true>;
    default: return (void*)&bg_finish_kernel<R, true, BGK_SEMIGLOBAL, true>;
  }
}

extern "C" void* bg_finish_ack_kernel_ptr(int R, int mode) {
  switch (R) {
    case 2: return finish_ack_ptr<2>(mode);
    case 4: return finish_ack_ptr<4>(mode);
    case 8: return finish_ack_ptr<8>(mode);
    default: return nullptr;
  }
}

// LDS of the affine checkpoint finish kernel for alphabet size K, `nslots` chunk slots (0: the
// kernel's maximum) and `nw` waves: chunk slots (four bit planes, five in local mode), 64
// scalars, the shared profile entries, nw per-wave recompute areas, the chunk map.
// *area_ints = the profile entries' ints (BgFinishArgs::area_ints).
extern "C" size_t bg_finish_ack_lds_bytes(int R, int K, int local, int nslots, int nw, int* win_bytes,
                                          int* area_ints) {
  int slot = 0, prof = 0, maxs = 0;
  switch (R) {
    case 2: slot = local ? ack_slot_dw<2, true>() : ack_slot_dw<2, false>(); prof = ack_prof_ints<2>(K); maxs = ack_slots<2>(); break;
    case 4: slot = local ? ack_slot_dw<4, true>() : ack_slot_dw<4, false>(); prof = ack_prof_ints<4>(K); maxs = ack_slots<4>(); break;
    default: slot = local ? ack_slot_dw<8, true>() : ack_slot_dw<8, false>(); prof = ack_prof_ints<8>(K); maxs = ack_slots<8>(); break;
  }
  const int ns = (nslots > 0 && nslots < maxs) ? nslots : maxs;
  *win_bytes = std::max(ns * slot * 4, 2 * 256 * 4);     // the end-cell / column scan aliases it
  *area_ints = prof;
  return (size_t)*win_bytes + 64 * 4 + (size_t)prof * 4 + (size_t)nw * kAckWaveInts * 4 + kCkMapEntries * 4;
}
