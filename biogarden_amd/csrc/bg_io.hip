// Result download as a kernel: the aligned strings and result records of an execute, written from
// HBM straight into the handle's pinned host buffers (bg_set_async_fetch).
//
// The host holds the batch's strings after bg_batch_fetch (aligner.rs:84-435 returns them as
// owned Strings); the streaming path (AlignStream) queues their download behind each traceback.
// Done with hipMemcpyAsync, the download is a copy-engine command, and the HIP runtime that ships
// with PyTorch blocks the host inside hipMemcpyAsync for ~7 ms at a time once several such copies
// wait on tracebacks.  A kernel on the download stream has no such limit: each lane
// moves 16-byte vectors from HBM to the host-mapped buffer over PCIe, so the copy costs a few CUs
// for as long as PCIe takes (10.2 MB per metric batch) and no copy-engine queue.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bg_device.h"

// grid-stride over every segment; 16-byte vectors where source and destination agree in
// alignment (hipMalloc / hipHostMalloc bases are page aligned), bytes for the rest
__global__ __launch_bounds__(256) void bg_download_kernel(BgDownloadArgs A) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
  for (int s = 0; s < A.nseg; ++s) {
    const BgDownloadSeg g = A.seg[s];
    const bool vec = (((uintptr_t)g.src | (uintptr_t)g.dst) & 15) == 0;
    const uint64_t nv = vec ? g.bytes / 16 : 0;
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u* sv = reinterpret_cast<const v4u*>(g.src);
    v4u* dv = reinterpret_cast<v4u*>(g.dst);
    for (uint64_t i = tid; i < nv; i += nth) dv[i] = __builtin_nontemporal_load(sv + i);
    for (uint64_t i = nv * 16 + tid; i < g.bytes; i += nth) g.dst[i] = g.src[i];
  }
}

extern "C" void* bg_download_kernel_ptr() { return (void*)&bg_download_kernel; }

// Exclusive scan of the compact record's caller-order sizes (bg_batch_export_compact): ONE wave,
// a chunk per lane, then a shuffle scan; sizes[n] = the total.  One wave fits on a CU beside the
// next execute's DP workgroup and its tracebacks.  (The first form was one 1024-thread workgroup
// scanning its partial sums in one thread: it found no CU until the DP beside it ended, and on the
// pipelined group's path every third DP then waited ~1 ms for the collect behind it.)
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int o) {
  const unsigned lo = __shfl_up((unsigned)v, o, 64), hi = __shfl_up((unsigned)(v >> 32), o, 64);
  return ((uint64_t)hi << 32) | lo;
}
__global__ __launch_bounds__(64) void bg_compact_scan_kernel(BgCompactArgs E) {
  const uint64_t n = E.npairs_caller;
  const unsigned lane = threadIdx.x;
  const uint64_t per = (n + 63) / 64;
  const uint64_t lo = lane * per, hi = lo + per < n ? lo + per : n;
  uint64_t s = 0;
  for (uint64_t p = lo; p < hi; ++p) s += E.sizes[p];
  uint64_t x = s;                                         // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = shfl_up_u64(x, o);
    if ((int)lane >= o) x += y;
  }
  if (lane == 63) E.sizes[n] = x;
  uint64_t acc = x - s;                                   // this lane's chunk starts here
  for (uint64_t p = lo; p < hi; ++p) { const uint64_t v = E.sizes[p]; E.sizes[p] = acc; acc += v; }
}

extern "C" void* bg_compact_scan_kernel_ptr() { return (void*)&bg_compact_scan_kernel; }
