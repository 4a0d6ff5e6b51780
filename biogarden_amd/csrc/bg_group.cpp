// Multi-device batches behind the C ABI (include/biogarden_gpu.h, bg_group_*): one process drives
// several GPUs — the node's 8 MI355X — with one bg_aligner per member, and gathers the results to
// the first member's device over RCCL.
//
// A batch of independent pairs (the reference's one SequenceAligner call per pair,
// src/alignment/aligner.rs:84-435, over a Tile, src/ds/tile.rs:9-11; its caller
// tests/integration.rs:234-312 / examples/from_file.rs:19-32) is
//   1. split over the members by cells, largest pair first, to the least-loaded member
//      (bgh::lpt_plan, the rule of biogarden_amd/shard.py);
//   2. given, per pair, the scratch dims ONE reference aligner running the whole batch in caller
//      order would start that call from (bgh::batch_call_dims, aligner.rs:92-94, 594-602), so every
//      member judges status 4 exactly as that aligner would;
//   3. prepared, executed and packed into a compact record on each member's device, one host
//      thread per member (bg_batch_export_compact: headers + 2-bit edit scripts);
//   4. gathered into one buffer on the root device: RCCL send / recv over xGMI for members on other
//      devices (one communicator over the distinct devices, ncclCommInitAll), a device copy for
//      members on the root device;
//   5. downloaded once and expanded on the host into the caller's buffers at the caller's
//      offsets (bgh::compact_expand), exactly the layout bg_align_batch returns.
// Members on one device share that device's HIP streams (bg_aligner_new_shared), so their DPs and
// tracebacks pipeline as consecutive executes of one handle do.
// bg_group_submit / bg_group_collect split a call in two so that kGSlots batches are in flight:
// every member has kGSlots aligners (pipeline slots), a submit runs steps 1-3 (each member's
// compact export queued on its traceback's stream right behind it) and returns, a collect runs 4
// and 5 of the oldest batch on the download streams, which wait for that batch's exports only.  Three: while the host
// collects batch k (its traceback, then ~1 ms of expansion), k + 1 and k + 2 keep the device's
// DP stream busy (two left it idle for the expansion: M 6 500 GCUPS against 4 608 synchronous).  While one batch's DPs and
// tracebacks run on the devices, the host prepares the next and expands the previous, and the
// devices overlap one batch's tracebacks with the next one's DPs.
//
// librccl is opened at bg_group_new (dlopen), not linked: a process that never groups devices
// does not load it, and one that already holds torch's copy reuses it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include "bg_device.h"
#include "bg_host_passes.h"
#include "biogarden_gpu.h"

extern "C" void* bg_aligner_aux_stream(bg_aligner* h);   // bg_host.cpp
extern "C" int bg_batch_export_compact_behind_traceback(bg_aligner* h, void* dst, size_t cap,
                                                         void* first, void* done);   // bg_host.cpp
extern "C" void* bg_download_kernel_ptr();                // bg_io.hip

namespace {

struct Rccl {
  bool ok = false;
  ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*groupStart)() = nullptr;
  ncclResult_t (*groupEnd)() = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*errorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!so) so = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!so) {
      std::fprintf(stderr, "biogarden_gpu: bg_group needs librccl: %s\n", dlerror());
      return;
    }
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(so, name));
      return f != nullptr;
    };
    R.ok = sym(R.commInitAll, "ncclCommInitAll") && sym(R.commDestroy, "ncclCommDestroy") &&
           sym(R.groupStart, "ncclGroupStart") && sym(R.groupEnd, "ncclGroupEnd") &&
           sym(R.send, "ncclSend") && sym(R.recv, "ncclRecv") && sym(R.errorString, "ncclGetErrorString");
    if (!R.ok) std::fprintf(stderr, "biogarden_gpu: librccl lacks a symbol bg_group needs\n");
  });
  return R;
}

double ms_since(std::chrono::steady_clock::time_point& t) {
  const auto now = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(now - t).count();
  t = now;
  return ms;
}

}  // namespace

enum { kGPrepExec, kGExport, kGGather, kGDownload, kGExpand, kGN };
constexpr int kGSlots = 3;       // batches in flight (submitted, not collected)

// one submitted batch: the caller's pair arrays (copied; the sequence bytes stay the caller's
// until the collect), the shards, and the slot its members' aligners run it on
struct GBatch {
  int slot = 0;
  size_t npairs = 0;
  std::vector<const uint8_t*> s1, s2;
  std::vector<size_t> n1, n2;
  std::vector<uint64_t> coff;
  uint64_t need = 0;
  std::vector<std::vector<size_t>> idx;   // member -> its pairs (caller indices)
  std::vector<size_t> size;               // member -> its compact record's bound (bytes)
};

struct bg_group {
  std::vector<int> dev;            // member -> HIP device
  std::vector<bg_aligner*> h;      // (member, slot) -> aligner, at kGSlots m + slot
  std::vector<int> rankDev;        // communicator rank -> device (rank 0: member 0's device)
  std::vector<int> rankOf;         // member -> rank
  std::vector<ncclComm_t> comm;    // per rank
  std::vector<hipStream_t> cs;     // per rank: the gather's stream (its device's shared download
                                   // stream, owned by the members' aligners)
  std::vector<void*> ebuf;         // (member, slot) -> its compact record (on its device)
  std::vector<size_t> ecap;
  std::vector<hipEvent_t> xev;     // (member, slot) -> its record written (traceback stream)
  std::vector<hipEvent_t> sev;     // (member, slot) -> its record read by the gather (on cs)
  std::deque<GBatch> pending;      // submitted, not yet collected (at most kGSlots)
  int nextSlot = 0;
  void* gbuf = nullptr;            // the gathered records, on the root device
  size_t gcap = 0;
  void* hbuf = nullptr;            // ... downloaded (pinned, host-mapped: a kernel writes it)
  void* hdev = nullptr;            // hbuf's device address
  size_t hcap = 0;
  long rows = 1024, cols = 1024;   // the reference aligner's scratch dims (the group is ONE aligner)
  int rcclSelf = 0;                // BG_GROUP_RCCL_SELF=1: root-device members go through RCCL too
  double ms[kGN] = {0, 0, 0, 0, 0};
  uint64_t calls = 0;
};

static int hip_fail(hipError_t e, const char* what) {
  std::fprintf(stderr, "biogarden_gpu: bg_group: %s: %s (%d)\n", what, hipGetErrorName(e), (int)e);
  return BG_E_HIP;
}

static int nccl_fail(ncclResult_t r, const char* what) {
  std::fprintf(stderr, "biogarden_gpu: bg_group: %s: %s (%d)\n", what,
               rccl().errorString ? rccl().errorString(r) : "?", (int)r);
  return BG_E_HIP;
}

extern "C" void bg_group_free(bg_group* g) {
  if (!g) return;
  for (size_t r = 0; r < g->comm.size(); ++r)
    if (g->comm[r]) (void)rccl().commDestroy(g->comm[r]);
  for (size_t x = 0; x < g->ebuf.size(); ++x)
    if (g->ebuf[x]) { (void)hipSetDevice(g->dev[x / kGSlots]); (void)hipFree(g->ebuf[x]); }
  for (size_t x = 0; x < g->xev.size(); ++x) {
    (void)hipSetDevice(g->dev[x / kGSlots]);
    if (g->xev[x]) (void)hipEventDestroy(g->xev[x]);
    if (g->sev[x]) (void)hipEventDestroy(g->sev[x]);
  }
  if (g->gbuf) { (void)hipSetDevice(g->rankDev[0]); (void)hipFree(g->gbuf); }
  if (g->hbuf) (void)hipHostFree(g->hbuf);
  // members sharing a device's streams: the stream owner (the first on its device) goes last
  for (size_t m = g->h.size(); m-- > 0;)
    if (g->h[m]) bg_aligner_free(g->h[m]);
  delete g;
}

extern "C" bg_group* bg_group_new(const int* devices, int n) {
  if (!devices || n < 1 || n > 4096) return nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return nullptr;
  for (int m = 0; m < n; ++m)
    if (devices[m] < 0 || devices[m] >= ndev) return nullptr;
  if (!rccl().ok) return nullptr;
  bg_group* g = new bg_group();
  g->dev.assign(devices, devices + n);
  g->h.assign(kGSlots * n, nullptr);
  g->rankOf.assign(n, -1);
  for (int m = 0; m < n; ++m) {
    int r = 0;
    while (r < (int)g->rankDev.size() && g->rankDev[r] != devices[m]) ++r;
    if (r == (int)g->rankDev.size()) g->rankDev.push_back(devices[m]);
    g->rankOf[m] = r;
    // the first member on a device owns its streams (its slot-0 aligner); every other aligner on
    // the device shares them
    int first = 0;
    while (g->dev[first] != devices[m]) ++first;
    for (int sl = 0; sl < kGSlots; ++sl) {
      bg_aligner*& hh = g->h[kGSlots * m + sl];
      hh = (first == m && sl == 0) ? bg_aligner_new(devices[m]) : bg_aligner_new_shared(g->h[kGSlots * first]);
      if (!hh || bg_set_pipeline(hh, 2) != BG_OK) { bg_group_free(g); return nullptr; }
      // the device's whole stream set now, before RCCL creates streams of its own (see
      // bg_aligner_aux_stream)
      if (first == m && sl == 0 && !bg_aligner_aux_stream(hh)) { bg_group_free(g); return nullptr; }
    }
  }
  const int nr = (int)g->rankDev.size();
  g->comm.assign(nr, nullptr);
  g->cs.assign(nr, nullptr);
  for (int r = 0; r < nr; ++r) {
    int first = 0;
    while (g->dev[first] != g->rankDev[r]) ++first;
    g->cs[r] = static_cast<hipStream_t>(bg_aligner_aux_stream(g->h[kGSlots * first]));
    if (!g->cs[r]) { bg_group_free(g); return nullptr; }
  }
  g->xev.assign(kGSlots * n, nullptr);
  g->sev.assign(kGSlots * n, nullptr);
  for (int x = 0; x < kGSlots * n; ++x)
    if (hipSetDevice(g->dev[x / kGSlots]) != hipSuccess ||
        hipEventCreateWithFlags(&g->xev[x], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->sev[x], hipEventDisableTiming) != hipSuccess) {
      bg_group_free(g);
      return nullptr;
    }
  const ncclResult_t rc = rccl().commInitAll(g->comm.data(), nr, g->rankDev.data());
  if (rc != ncclSuccess) {
    nccl_fail(rc, "ncclCommInitAll");
    g->comm.assign(nr, nullptr);
    bg_group_free(g);
    return nullptr;
  }
  g->ebuf.assign(kGSlots * n, nullptr);
  g->ecap.assign(kGSlots * n, 0);
  const char* e = std::getenv("BG_GROUP_RCCL_SELF");
  g->rcclSelf = e && e[0] == '1';
  return g;
}

extern "C" int bg_group_size(const bg_group* g) { return g ? (int)g->dev.size() : BG_E_ARG; }

extern "C" bg_aligner* bg_group_member(bg_group* g, int m) {
  return (g && m >= 0 && m < (int)g->dev.size()) ? g->h[kGSlots * m] : nullptr;
}

extern "C" int bg_group_plan(size_t npairs, const size_t* n1, const size_t* n2, int nshards,
                             int32_t* shard_of) {
  if (nshards < 1 || (npairs && (!n1 || !n2 || !shard_of))) return BG_E_ARG;
  bgh::lpt_plan(npairs, n1, n2, nshards, shard_of);
  return BG_OK;
}

extern "C" int bg_group_buffer_size(bg_group* g, size_t* rows, size_t* cols) {
  if (!g || !rows || !cols) return BG_E_ARG;
  *rows = (size_t)g->rows;
  *cols = (size_t)g->cols;
  return BG_OK;
}

extern "C" int bg_group_timing(bg_group* g, double* ms, size_t n, uint64_t* calls, int reset) {
  if (!g || (n && !ms)) return BG_E_ARG;
  for (size_t i = 0; i < n && i < (size_t)kGN; ++i) ms[i] = g->ms[i];
  if (calls) *calls = g->calls;
  if (reset) {
    for (double& x : g->ms) x = 0.0;
    g->calls = 0;
  }
  return kGN;
}

extern "C" int bg_group_submit(bg_group* g, int mode, size_t npairs, const uint8_t* const* s1,
                               const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                               const bg_scoring* sc, int32_t a, int32_t b) {
  if (!g || !sc || mode < BG_GLOBAL || mode > BG_SEMIGLOBAL || g->pending.size() >= (size_t)kGSlots) return BG_E_ARG;
  if (npairs && (!s1 || !n1 || !s2 || !n2)) return BG_E_ARG;
  auto t = std::chrono::steady_clock::now();
  const int M = (int)g->dev.size();
  GBatch B;
  B.slot = g->nextSlot;
  B.npairs = npairs;
  B.s1.assign(s1, s1 + npairs);
  B.s2.assign(s2, s2 + npairs);
  B.n1.assign(n1, n1 + npairs);
  B.n2.assign(n2, n2 + npairs);
  B.coff.resize(npairs);
  for (size_t p = 0; p < npairs; ++p) {
    B.coff[p] = B.need;
    B.need += (uint64_t)n1[p] + n2[p];
  }
  // 1-2: the shards and every call's scratch dims (the group's dims move on with each submit)
  std::vector<int32_t> shardOf(npairs);
  bgh::lpt_plan(npairs, n1, n2, M, shardOf.data());
  long rows = g->rows, cols = g->cols;
  std::vector<std::pair<long, long>> dims;
  bgh::batch_call_dims(mode, npairs, n1, n2, a, b, rows, cols, dims);
  B.idx.assign(M, {});
  for (size_t p = 0; p < npairs; ++p) B.idx[shardOf[p]].push_back(p);
  // 3 (first half): every member prepares and executes its shard (one host thread each)
  std::vector<int> rc(M, BG_OK);
  auto member = [&](int m) {
    const std::vector<size_t>& I = B.idx[m];
    const size_t k = I.size();
    if (!k) return;
    bg_aligner* h = g->h[kGSlots * m + B.slot];
    std::vector<const uint8_t*> p1(k), p2(k);
    std::vector<size_t> l1(k), l2(k);
    std::vector<uint64_t> r(k), c(k);
    for (size_t q = 0; q < k; ++q) {
      p1[q] = s1[I[q]]; l1[q] = n1[I[q]];
      p2[q] = s2[I[q]]; l2[q] = n2[I[q]];
      r[q] = (uint64_t)dims[I[q]].first; c[q] = (uint64_t)dims[I[q]].second;
    }
    int e = bg_aligner_set_call_dims(h, k, r.data(), c.data());
    if (!e) e = bg_batch_prepare(h, mode, k, p1.data(), l1.data(), p2.data(), l2.data(), sc, a, b);
    if (!e) e = bg_batch_execute(h);
    rc[m] = e;
  };
  {
    std::vector<std::thread> th;
    for (int m = 1; m < M; ++m) th.emplace_back(member, m);
    member(0);
    for (auto& x : th) x.join();
  }
  for (int m = 0; m < M; ++m)
    if (rc[m]) return rc[m];
  g->ms[kGPrepExec] += ms_since(t);
  // 3 (second half): every member's compact export, queued without a host wait on its traceback's
  // stream right behind it, into its slot's buffer (sized by the record's bound) once the gather of
  // the slot's previous batch has read it (sev); xev marks it written
  B.size.assign(M, 0);
  for (int m = 0; m < M; ++m) {
    if (B.idx[m].empty()) continue;
    const int x = kGSlots * m + B.slot;
    bg_aligner* h = g->h[x];
    size_t sz = 0;
    int e = bg_batch_export_compact_bound(h, &sz);
    hipError_t he = hipSetDevice(g->dev[m]);
    if (!e && he != hipSuccess) e = hip_fail(he, "hipSetDevice");
    if (!e && g->ecap[x] < sz) {
      if (g->ebuf[x]) (void)hipFree(g->ebuf[x]);
      g->ebuf[x] = nullptr;
      g->ecap[x] = 0;
      if (hipMalloc(&g->ebuf[x], sz + sz / 4) != hipSuccess) { g->ebuf[x] = nullptr; e = BG_E_NOMEM; }
      else g->ecap[x] = sz + sz / 4;
    }
    if (!e) e = bg_batch_export_compact_behind_traceback(h, g->ebuf[x], sz, g->sev[x], g->xev[x]);
    if (e) return e;
    B.size[m] = sz;
  }
  g->rows = rows;
  g->cols = cols;
  g->nextSlot = (g->nextSlot + 1) % kGSlots;
  g->pending.push_back(std::move(B));
  g->ms[kGExport] += ms_since(t);
  return BG_OK;
}

extern "C" int bg_group_collect(bg_group* g, bg_pair_result* res, uint8_t* out1, uint8_t* out2,
                                size_t out_cap) {
  if (!g || g->pending.empty()) return BG_E_ARG;
  const GBatch& B = g->pending.front();
  if (B.npairs && !res) return BG_E_ARG;
  if (B.need && (!out1 || !out2 || out_cap < B.need)) return BG_E_ARG;
  auto t = std::chrono::steady_clock::now();
  ++g->calls;
  const int M = (int)g->dev.size();
  const std::vector<size_t>& size = B.size;
  auto finish = [&](int e) {
    g->pending.pop_front();
    return e;
  };
  // 4: the gather into one buffer on the root device
  std::vector<uint64_t> goff(M + 1, 0);
  for (int m = 0; m < M; ++m) goff[m + 1] = goff[m] + size[m];
  const int root = g->rankDev[0];
  hipError_t he;
  if (goff[M] > g->gcap) {
    if ((he = hipSetDevice(root)) != hipSuccess) return finish(hip_fail(he, "hipSetDevice"));
    if (g->gbuf) (void)hipFree(g->gbuf);
    g->gbuf = nullptr;
    g->gcap = 0;
    if (hipMalloc(&g->gbuf, goff[M] + goff[M] / 4) != hipSuccess) { g->gbuf = nullptr; return finish(BG_E_NOMEM); }
    g->gcap = goff[M] + goff[M] / 4;
  }
  uint8_t* gb = static_cast<uint8_t*>(g->gbuf);
  bool viaRccl = false;
  for (int m = 0; m < M; ++m)
    if (size[m] && (g->rankOf[m] != 0 || g->rcclSelf)) viaRccl = true;
  // every gather stream waits for the records it reads (this batch's exports, xev)
  for (int m = 0; m < M; ++m) {
    if (!size[m]) continue;
    const int r = g->rankOf[m];
    if ((he = hipSetDevice(g->rankDev[r])) != hipSuccess) return finish(hip_fail(he, "hipSetDevice"));
    if ((he = hipStreamWaitEvent(g->cs[r], g->xev[kGSlots * m + B.slot], 0)) != hipSuccess)
      return finish(hip_fail(he, "wait export"));
  }
  for (int m = 0; m < M; ++m)
    if (size[m] && g->rankOf[m] == 0 && !g->rcclSelf) {
      if ((he = hipSetDevice(root)) != hipSuccess) return finish(hip_fail(he, "hipSetDevice"));
      if ((he = hipMemcpyAsync(gb + goff[m], g->ebuf[kGSlots * m + B.slot], size[m], hipMemcpyDeviceToDevice,
                               g->cs[0])) != hipSuccess ||
          (he = hipEventRecord(g->sev[kGSlots * m + B.slot], g->cs[0])) != hipSuccess)
        return finish(hip_fail(he, "gather copy"));
    }
  if (viaRccl) {
    const Rccl& R = rccl();
    ncclResult_t nr = R.groupStart();
    if (nr != ncclSuccess) return finish(nccl_fail(nr, "ncclGroupStart"));
    // per member in member order: its rank sends, the root receives (NCCL matches each pair of
    // ranks' sends and receives in issue order)
    for (int m = 0; m < M && nr == ncclSuccess; ++m) {
      if (!size[m] || (g->rankOf[m] == 0 && !g->rcclSelf)) continue;
      const int r = g->rankOf[m];
      nr = R.send(g->ebuf[kGSlots * m + B.slot], size[m], ncclUint8, 0, g->comm[r], g->cs[r]);
      if (nr == ncclSuccess) nr = R.recv(gb + goff[m], size[m], ncclUint8, r, g->comm[0], g->cs[0]);
    }
    const ncclResult_t ne = R.groupEnd();
    if (nr != ncclSuccess) return finish(nccl_fail(nr, "ncclSend / ncclRecv"));
    if (ne != ncclSuccess) return finish(nccl_fail(ne, "ncclGroupEnd"));
    // the slot's next export waits for the send that reads its buffer (sev)
    for (int m = 0; m < M; ++m) {
      if (!size[m] || (g->rankOf[m] == 0 && !g->rcclSelf)) continue;
      const int r = g->rankOf[m];
      if ((he = hipSetDevice(g->rankDev[r])) != hipSuccess ||
          (he = hipEventRecord(g->sev[kGSlots * m + B.slot], g->cs[r])) != hipSuccess)
        return finish(hip_fail(he, "record send"));
    }
  }
  // (no host wait: the download below is queued behind the receives on the root's stream)
  if ((he = hipSetDevice(root)) != hipSuccess) return finish(hip_fail(he, "hipSetDevice"));
  g->ms[kGGather] += ms_since(t);
  // 5: one download, then the expansion into the caller's buffers at the caller's offsets.  The
  // download is a kernel writing host-mapped pinned memory (bg_download_kernel), as the handles'
  // asynchronous fetch: a hipMemcpyAsync device-to-host under the HIP runtime torch loads waits
  // for the device's other queued work (1.7 ms of a 3.8 ms pipelined M batch)
  if (goff[M] > g->hcap) {
    if (g->hbuf) (void)hipHostFree(g->hbuf);
    g->hbuf = nullptr;
    g->hdev = nullptr;
    g->hcap = 0;
    if (hipHostMalloc(&g->hbuf, goff[M] + goff[M] / 4, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess ||
        hipHostGetDevicePointer(&g->hdev, g->hbuf, 0) != hipSuccess) {
      if (g->hbuf) (void)hipHostFree(g->hbuf);
      g->hbuf = nullptr;
      g->hdev = nullptr;
      return finish(BG_E_NOMEM);
    }
    g->hcap = goff[M] + goff[M] / 4;
  }
  if (goff[M]) {
    BgDownloadArgs D;
    std::memset(&D, 0, sizeof(D));
    D.seg[0] = {static_cast<const uint8_t*>(g->gbuf), static_cast<uint8_t*>(g->hdev), goff[M]};
    D.nseg = 1;
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(64, (goff[M] / 16 + 255) / 256));
    void* dargs[] = {&D};
    if ((he = hipLaunchKernel(bg_download_kernel_ptr(), dim3(blocks), dim3(256), dargs, 0, g->cs[0])) != hipSuccess ||
        (he = hipStreamSynchronize(g->cs[0])) != hipSuccess)
      return finish(hip_fail(he, "download"));
  }
  g->ms[kGDownload] += ms_since(t);
  // every member's record in one pass over the host pool (bgh::compact_expand_multi): the
  // members' pairs are the work items, written at the caller's offsets
  const uint8_t* hb = static_cast<const uint8_t*>(g->hbuf);
  {
    std::vector<bgh::CompactRec> recs;
    std::vector<size_t> idx;
    std::vector<uint64_t> dst;
    idx.reserve(B.npairs);
    dst.reserve(B.npairs);
    for (int m = 0; m < M; ++m) {
      const std::vector<size_t>& I = B.idx[m];
      if (I.empty()) continue;
      recs.push_back({hb + goff[m], size[m], I.size()});
      for (size_t q : I) { idx.push_back(q); dst.push_back(B.coff[q]); }
    }
    const int e = bgh::compact_expand_multi(recs.data(), recs.size(), B.s1.data(), B.n1.data(), B.s2.data(),
                                            B.n2.data(), idx.data(), res, out1, out2, out_cap, dst.data());
    if (e) return finish(e);
  }
  g->ms[kGExpand] += ms_since(t);
  return finish(BG_OK);
}

extern "C" int bg_group_pending(const bg_group* g) { return g ? (int)g->pending.size() : BG_E_ARG; }

extern "C" int bg_group_align_batch(bg_group* g, int mode, size_t npairs, const uint8_t* const* s1,
                                    const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                                    const bg_scoring* sc, int32_t a, int32_t b, bg_pair_result* res,
                                    uint8_t* out1, uint8_t* out2, size_t out_cap) {
  if (!g || !g->pending.empty()) return BG_E_ARG;
  if (npairs && (!s1 || !n1 || !s2 || !n2 || !res)) return BG_E_ARG;
  uint64_t need = 0;
  for (size_t p = 0; p < npairs; ++p) need += (uint64_t)n1[p] + n2[p];
  if (need && (!out1 || !out2 || out_cap < need)) return BG_E_ARG;
  // the dims move on only if the batch runs: a failed collect restores them
  const long rows = g->rows, cols = g->cols;
  int e = bg_group_submit(g, mode, npairs, s1, n1, s2, n2, sc, a, b);
  if (e) return e;
  e = bg_group_collect(g, res, out1, out2, out_cap);
  if (e) { g->rows = rows; g->cols = cols; }
  return e;
}
