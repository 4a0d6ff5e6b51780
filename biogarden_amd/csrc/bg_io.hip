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
