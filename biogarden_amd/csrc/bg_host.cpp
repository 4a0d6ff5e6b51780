// Host runtime behind the C ABI (include/biogarden_gpu.h): validation in the reference's order,
// batch planning (strips, LPT order, arenas in HBM), kernel launches on the handle's HIP
// stream, download and unpacking of the aligned strings.
//
// Reference call sites mirrored here:
//   argument checks      aligner.rs:87-89, 153-155, 219-225
//   score closure        score.rs:38-41 (+ A.8 tabulation: bg_scoring)
//   buffer semantics     aligner.rs:92-94, 594-602 (exact-size here; divergences are flagged)
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bg_device.h"
#include "bg_host_passes.h"
#include "biogarden_gpu.h"

extern "C" void* bg_dp_kernel_ptr(int R, int affine, int local, int dna);
extern "C" int bg_dp_has_R(int R, int affine, int local, int dna);
extern "C" void* bg_dp_kernel_p32_ptr(int R, int affine, int local, int global);
extern "C" void* bg_dp_kernel_lcs_ptr(int R, int dna);
extern "C" void* bg_dp_kernel_tag_ptr(int R, int wide, int ckpt);
extern "C" void* bg_finish_ck_kernel_ptr(int R, int mode);
extern "C" void* bg_split_kernel_ptr(int R, int which);
extern "C" void* bg_endkey_kernel_ptr(void);
extern "C" void* bg_expand_kernel_ptr(int which);
extern "C" int bg_expand_cols_per_block(void);
extern "C" int bg_endkey_blocks(void);
extern "C" int bg_exit_lds_bytes(int R);
extern "C" int bg_exit_conc_lds_bytes(int R);
extern "C" size_t bg_finish_ck_lds_bytes(int R, int nslots, int nw, int* win_bytes);
extern "C" size_t bg_finish_grp4_lds_bytes(int R, int nslots, int nw, int* win_bytes);
extern "C" size_t bg_finish_grp2_lds_bytes(int R, int nslots, int nw, int* win_bytes);
extern "C" void* bg_finish_grp4_kernel_ptr(int R, int mode);
extern "C" void* bg_finish_grp2_kernel_ptr(int R, int mode);
extern "C" void* bg_dp_grp_kernel_ptr(int R, int P);
extern "C" int bg_dp_grp_wave_lds_bytes(int R, int P);
// grouped pairs, P per wave (bg_grp_kernel.hip, bg_grp_finish.hip)
static size_t bg_finish_grp_lds_bytes(int P, int R, int nslots, int nw, int* win) {
  return P == 2 ? bg_finish_grp2_lds_bytes(R, nslots, nw, win) : bg_finish_grp4_lds_bytes(R, nslots, nw, win);
}
static void* bg_finish_grp_kernel_ptr(int P, int R, int mode) {
  return P == 2 ? bg_finish_grp2_kernel_ptr(R, mode) : bg_finish_grp4_kernel_ptr(R, mode);
}
extern "C" int bg_dp_tag_wave_lds_bytes(int R);
extern "C" void* bg_finish_kernel_ptr(int R, int affine, int mode);
extern "C" size_t bg_finish_lds_bytes(int win_bytes);
extern "C" int bg_finish_window_bytes(int R, int affine, size_t npairs, int cus);
extern "C" void* bg_export_kernel_ptr();
extern "C" void* bg_compact_size_kernel_ptr();
extern "C" void* bg_compact_scan_kernel_ptr();
extern "C" void* bg_compact_write_kernel_ptr();
extern "C" void* bg_code_kernel_ptr();
extern "C" void* bg_download_kernel_ptr();
extern "C" void* bg_global_score_kernel_ptr();
extern "C" void* bg_dp_aff_kernel_ptr(int R, int local);
extern "C" int bg_dp_aff_head_bytes(void);
extern "C" int bg_dp_aff_wave_lds_bytes(int R, int K);
extern "C" void* bg_finish_ack_kernel_ptr(int R, int mode);
extern "C" size_t bg_finish_ack_lds_bytes(int R, int K, int local, int nslots, int nw, int* win_bytes,
                                          int* area_ints);

#include "bg_tables.inc"

namespace {

using bgh::HScore;
using bgh::host_threads;
using bgh::par_ranges;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; return false; }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// Pinned host staging (hipHostMalloc): uploads and downloads DMA straight from / into it, with
// no runtime bounce copy; grown and kept by the handle like its device arenas.
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    if (hipHostMalloc(&p, want, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) { p = nullptr; return false; }
    cap = want;
    dev = nullptr;
    return true;
  }
  // the address kernels write through (bg_download_kernel)
  void* dev = nullptr;
  void* device_ptr() {
    if (!dev && p && hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) dev = nullptr;
    return dev;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

inline size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

// bg_download_kernel's grid: enough 256-thread blocks to keep PCIe busy, few enough to sit
// beside the next DP (no LDS, a handful of VGPRs)
static constexpr unsigned kDownloadBlocks = 64u;

// Diagnostics on stderr, chosen once per process by BG_DEBUG (comma-separated): prepare (host
// phases per prepare / fetch), exec (host time of each execute's steps), dp (WIDE strip timeline
// of the first pair), finish (traceback phase cycles), plan (the geometry candidates).  They
// never change results.
struct BgDebug {
  bool prepare = false, exec = false, dp = false, finish = false, plan = false;
};
static const BgDebug& dbg_flags() {
  static const BgDebug d = [] {
    BgDebug x;
    const char* e = std::getenv("BG_DEBUG");
    if (!e) return x;
    std::string v(e);
    auto has = [&](const char* k) {
      const size_t n = std::strlen(k);
      for (size_t at = v.find(k); at != std::string::npos; at = v.find(k, at + 1))
        if ((at == 0 || v[at - 1] == ',') && (at + n == v.size() || v[at + n] == ',')) return true;
      return false;
    };
    x.prepare = has("prepare");
    x.exec = has("exec");
    x.dp = has("dp");
    x.finish = has("finish");
    x.plan = has("plan");
    return x;
  }();
  return d;
}

// bg_set_option names, for BG_OPTIONS ("name=value,...")
static const char* const kOptNames[BG_OPT_COUNT] = {
    "grouped", "group_pairs", "group_waves", "wide_waves", "fin_waves", "fin_slots", "fin_sync",
    "fin_selfserve", "split", "split_segment", "split_concurrent", "split_wait_ms",
    "two_dp_streams", "wait_ms", "span", "wide"};

// Host-side phases of prepare / fetch, accumulated per handle (bg_host_timing) and, with
// BG_DEBUG=prepare, printed per call on stderr
enum { kPhSync, kPhStage, kPhPlan, kPhAlloc, kPhUpload, kPhFetchWait, kPhFetchCopy, kPhFetchUnpack, kPhN };
struct PhaseTimer {
  double* acc;
  bool on = dbg_flags().prepare;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  char buf[512];
  int n = 0;
  explicit PhaseTimer(double* a) : acc(a) { buf[0] = 0; }
  void mark(int ph, const char* what) {
    const auto now = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
    acc[ph] += ms;
    if (on)
      n += std::snprintf(buf + n, sizeof(buf) - n > 0 ? sizeof(buf) - n : 0, " %s %.3f", what, ms);
  }
  ~PhaseTimer() { if (on && n) std::fprintf(stderr, "host ms:%s\n", buf); }
};

}  // namespace

// Per-execute arenas.  Two slots let the finish kernel of execute k (stream2) run while the
// DP kernel of execute k+1 (stream) fills the other slot's trace.
struct Slot {
  DevBuf trace, bndM, bndX, aux, out1, out2, results, ops, gran, split, gprog;
  DevBuf keys;                      // split pairs: bg_endkey_kernel's end-cell keys (2 u64 per pair)
  DevBuf wdiag;                     // the traceback's bounded-wait record (bg_wait_diag)
  DevBuf xcnt;                      // split pairs: the deferred expansion's per-block counts
  hipEvent_t dpDone = nullptr, finDone = nullptr;
  hipEvent_t resetDone = nullptr;   // the DP's progress words zeroed (the concurrent exit pass waits)
  // a reader of the slot's results queued on another stream (the asynchronous download or
  // compact export): the next execute into this slot waits for it before its kernels write
  hipEvent_t readDone = nullptr;
  bool inflight = false, readPending = false;
  bool dpPending = false;           // a DP queued by an execute that failed before its finDone
};

// The HIP streams of one handle, or of several handles on one device that share them
// (bg_aligner_new_shared).  HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues
// (4 on the MI355X boxes); a stream sharing a queue with another stream's kernels waits behind
// them.  Handles in rotation (biogarden_amd/stream.py) therefore share ONE set: uploads, DPs,
// tracebacks and downloads each get their own stream and queue however many batches are in
// flight, and the DPs / tracebacks of consecutive batches pipeline exactly as the executes of one
// handle do.  Streams beyond the first two are created on first use.
enum { kSDp, kSFin, kSFin2, kSFin3, kSDps, kSUp, kSDl, kSN };
struct StreamGroup {
  int device = 0;
  hipStream_t s[kSN] = {};
  std::mutex mu;
  ~StreamGroup() {
    (void)hipSetDevice(device);
    for (hipStream_t x : s)
      if (x) { (void)hipStreamSynchronize(x); (void)hipStreamDestroy(x); }
  }
};

struct bg_aligner {
  int device = 0;
  int cus = 256;
  std::shared_ptr<StreamGroup> sg; // the stream set (shared with other handles, or this one's)
  hipStream_t stream = nullptr;    // DP kernels (and, unshared, uploads and downloads)
  hipStream_t stream2 = nullptr;   // end cell + traceback kernels
  hipStream_t stream3 = nullptr;   // WIDE batches: every other execute's traceback (see execute)
  hipStream_t stream4 = nullptr;   // WIDE batches at pipeline depth 4: every third one
  // WIDE batches: every other execute's DP.  A WIDE DP holds one CU per group workgroup (C3: 79 of
  // 256), so two executes' DPs run side by side on disjoint CUs (each waits for its own slot's
  // previous traceback); created on first use (BG_TWO_DP_STREAMS=1)
  hipStream_t dps = nullptr;
  hipStream_t upS = nullptr;       // shared handles: uploads (a queue of their own)
  hipStream_t dlS = nullptr;       // downloads of the asynchronous fetch (bg_set_async_fetch)
  hipStream_t lastFs = nullptr;    // the stream the last execute's traceback ran on
  // bg_set_async_fetch: every execute queues its results' download (into ho1 / ho2 / hresPin)
  // right after its traceback; bg_batch_fetch then only waits for it and unpacks
  int asyncFetch = 0;
  int dlExec = -1;                 // the execute (execCount) whose download was queued last
  hipEvent_t dlDone = nullptr;
  uint64_t planOut = 0;            // prepared batch: sum of n1 + n2 over the plan's pairs
  hipEvent_t upDone = nullptr;     // shared handles: the prepared batch's upload (not waited for
  bool upPending = false;          // on the host; the DPs wait for it)
  std::vector<int32_t> profHost;   // the prepared batch's profile table and result templates,
  std::vector<BgPairResultDev> tmplHost;   // kept until the upload has read them
  bool shared() const { return sg && sg.use_count() > 1; }
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // last execute: dp start/end, fin start/end
  DevBuf seq1, seq2, codes1, codes2, lut, prof, pairs, recs;
  Slot slot[4];
  int depth = 3;                   // pipeline depth: arena slots in flight (1..4; 3 lets the
                                   // traceback of step k overlap the DPs of k+1 and k+2)
  int execCount = 0;
  uint32_t epoch = 0;              // WIDE granule tag of the last execute (never reset)
  int lastSlot = 0;

  // profiling ring (bg_profile_begin/end)
  std::vector<hipEvent_t> ring;
  bool profiling = false;
  int ringUsed = 0;

  // prepared batch
  bool prepared = false;
  bool executed = false;
  int mode = 0;
  int32_t a = 0, b = 0;
  size_t npairs = 0;
  std::vector<size_t> n1v, n2v;
  std::vector<int> prestatus;        // 1/2/3 = decided on the host; -1 = computed on the GPU
  std::vector<uint64_t> outoff;      // caller output offsets
  std::vector<BgPair> plan;          // GPU pairs in launch (LPT) order
  std::vector<size_t> order_;        // plan slot -> caller index
  int R = 8, W = 1, affine = 0, local = 0, dna = 1, kdim = 0, tag = 0;
  int allowTag = 1;
  int allowCkpt = 1;
  int allowAck = 1;
  int ckpt = 0;                    // tagged path: score-only DP + checkpoint traceback
  int p32 = 0;                     // mask kernel with int32 profile entries (S - a beyond int16)
  int pglob = 0;                   // ... with the per-wave profile tables in HBM (too big for LDS)
  int pstride = 32;                // int16 profile table row stride (the batch's dense alphabet, >= 32)
  std::vector<uint64_t> pmaskW;    // prepare: 256-bit code sets per pair (alphabets beyond 32)
  int finFlags = 0;                // BG_FIN_* for the finish kernel (edit distance, LCS)
  int ack = 0;                     // affine / local path: score-only DP (bg_aff_kernel.hip) +
                                   // traceback over recomputed full-trace chunks
  size_t lds = 0;
  int progOff = 256;
  int codesOff = 320;
  int codesInLds = 0;
  int auxLdsOff = 0;
  int wide = 0;                    // tagged kernel: pairs spread over groups of workgroups
  int span = 0;                    // ... of many-wave workgroups (fewer pairs than CUs, SPAN)
  // grouped DP (bg_grp_kernel.hip): short reads sharing a reference, `grouped` (P = 4 or 2) per
  // wave, 0 off; grpHost holds P plan indices per group (-1: an empty row)
  int grouped = 0, ngroups = 0;
  std::vector<int32_t> grpHost;
  DevBuf grpBuf;
  // split traceback (bg_split.hip): WIDE linear checkpoint batches walk their pairs
  // strip by strip in parallel; BG_SPLIT=0 walks them whole (one workgroup per pair)
  int split = 0, segc = BG_SPLIT_SEGC, splitMargin = 0, splitClamp = 0, splitGrow = 0;
  int splitItems = 0, splitResolve = 0;
  uint64_t splitInts = 0;
  std::vector<int2> splitMap;
  std::vector<int32_t> splitBases;  // exit-pass item bases (np + 1), then resolve bases (np + 1),
                                    // then the items in estimated readiness order (concurrent pass)
  int splitXBlocks = 1;             // deferred expansion: blocks per split pair (max n1 + n2 / 4096)
  int splitConc = 0;                // the exit pass beside the DP: 1 always (BG_SPLIT_CONC=1), 0 never
                                    // (=0), 2 (unset) when no other execute's DP is in flight
  DevBuf splitMapBuf, splitBaseBuf;
  int tagRow = 0;                  // tagged kernel: the code row staged whole in LDS
  std::vector<int> groupOf;        // caller pair -> workgroups (WIDE)
  std::vector<int2> wgmap;
  int gridWgs = 0;
  uint32_t progWords = 0;
  DevBuf wgmapBuf, gprogBuf, dbgBuf, dpDbg, profScratch, compactSizes;
  int compactExec = -1;            // bg_batch_export_compact: the execute its sizes were made for
  uint64_t compactOps = 0;
  uint64_t opsBytes = 0;           // packed core ops per slot (sum of ceil((n1+n2)/4))
  uint64_t cells = 0, traceBytes = 0, bndBytes = 0, resBytes = 0, outBytes = 0;
  int tuneR = 0, tuneW = 0;
  int opt[BG_OPT_COUNT];            // bg_set_option, -1 = automatic
  int o(int key, int dflt) const { return opt[key] < 0 ? dflt : opt[key]; }
  float dp_ms = 0.f, fin_ms = 0.f;
  hipEvent_t last[4] = {nullptr, nullptr, nullptr, nullptr};

  std::vector<BgResult> hres;
  PinBuf ho1, ho2;                 // fetch: the slot's aligned strings, downloaded
  PinBuf hresPin;                  // asynchronous fetch: the results, downloaded
  PinBuf up;                       // prepare: raw residues + codes of the batch, uploaded
  std::vector<uint32_t> pmask;     // prepare: per pair, the score codes its residues use
  std::vector<uint64_t> coff1, coff2;   // prepare: caller-order offsets of the staged residues

  // The reference aligner's scratch dims (aligner.rs:30 buffer_size): 1024 x 1024 at
  // SequenceAligner::new (:44-55), reset to (len1+1, len2+1) by a call with len1 > rows ||
  // len2 > cols (:92-94, 594-602).  A prepared batch is that many calls in caller order;
  // bufAt[p] is the state pair p's call starts from (what bg_ref_divergent judges it against).
  long bufRows = 1024, bufCols = 1024;
  std::vector<std::pair<long, long>> bufAt;
  std::vector<std::pair<long, long>> callDims;   // bg_aligner_set_call_dims: pending per-pair dims
  int finWaves = 0, finSlots = 0;   // last prepared batch: finish workgroup geometry
  double hostMs[kPhN] = {0, 0, 0, 0, 0, 0, 0, 0};   // bg_host_timing: host phases, accumulated
  uint64_t nPrepare = 0, nFetch = 0;

  size_t device_bytes() const {
    size_t t = seq1.cap + seq2.cap + codes1.cap + codes2.cap + lut.cap + prof.cap + pairs.cap + recs.cap +
               profScratch.cap;
    for (const Slot& S : slot)
      t += S.trace.cap + S.bndM.cap + S.bndX.cap + S.aux.cap + S.out1.cap + S.out2.cap + S.results.cap +
           S.ops.cap + S.gran.cap + S.split.cap + S.gprog.cap;
    return t;
  }
};

static const char kDig[] = "0123456789ABCDEFGHIJKLMNOPQRSTUV";

extern "C" int bg_scoring_builtin(int which, bg_scoring* out) {
  if (!out) return BG_E_ARG;
  const char* enc = which == BG_BLOSUM62 ? kBlosum62Enc : which == BG_PAM250 ? kPam250Enc
                  : which == BG_UNIT ? kUnitEnc : nullptr;
  if (!enc) return BG_E_ARG;
  std::memset(out, 0, sizeof(*out));
  out->alphabet_size = 26;
  std::memset(out->code, 0xFF, sizeof(out->code));
  for (int c = 0; c < 26; ++c) out->code['A' + c] = (uint8_t)c;  // score.rs:40 `(*a as usize) - 65`
  for (int r = 0; r < 26; ++r)
    for (int c = 0; c < 26; ++c) {
      const char ch = enc[r * 26 + c];
      const int v = (int)(std::strchr(kDig, ch) - kDig) - 8;
      out->table[r * 32 + c] = v;
    }
  return BG_OK;
}

extern "C" const char* bg_status_string(int s) {
  switch (s) {
    case BG_OK: return "ok";
    case BG_INVALID_ARGUMENT_RANGE: return "InvalidArgumentRange";
    case BG_INVALID_INPUT_SIZE: return "InvalidInputSize";
    case BG_UNSCORABLE: return "unscorable byte (reference panics)";
    case BG_REF_DIVERGENT: return "reference would panic/hang (exact-size result returned)";
    case BG_INTERNAL: return "internal error (traceback recomputation timed out)";
    case BG_E_ARG: return "bad argument";
    case BG_E_HIP: return "HIP error";
    case BG_E_NOMEM: return "out of memory";
    case BG_E_SCORE_RANGE: return "lengths beyond the LCS value frame";
    case BG_E_IO: return "cannot open file";
    case BG_E_FORMAT: return "Expected > at record start.";
    case BG_E_UTF8: return "stream did not contain valid UTF-8";
    case BG_E_NO_BATCH: return "no prepared batch";
    case BG_E_ALPHABET: return "more than ~150 symbols with scores beyond int16";
    default: return "unknown";
  }
}

extern "C" int bg_abi_version(void) { return BG_ABI_VERSION; }

// The group's stream `which`, created on first use (nullptr if HIP cannot create it)
static hipStream_t group_stream(bg_aligner* h, int which) {
  StreamGroup& G = *h->sg;
  std::lock_guard<std::mutex> lk(G.mu);
  if (!G.s[which] && hipStreamCreateWithFlags(&G.s[which], hipStreamNonBlocking) != hipSuccess)
    G.s[which] = nullptr;
  return G.s[which];
}

// Waits for this handle's own work.  A handle alone on its streams waits for the streams; a handle
// sharing them waits for its own events only (every execute ends in its slot's finDone, recorded
// after its DP and traceback; a queued download in dlDone), so other handles' batches keep flowing.
static hipError_t drain(bg_aligner* h) {
  hipError_t e = hipSetDevice(h->device);
  if (e != hipSuccess) return e;
  if (!h->shared()) {
    for (hipStream_t s : {h->stream, h->stream2, h->stream3, h->stream4, h->dps, h->upS, h->dlS})
      if (s && (e = hipStreamSynchronize(s)) != hipSuccess) return e;
    return hipSuccess;
  }
  for (const Slot& S : h->slot) {
    if (S.inflight && (e = hipEventSynchronize(S.finDone)) != hipSuccess) return e;
    if (S.readPending && (e = hipEventSynchronize(S.readDone)) != hipSuccess) return e;
    if (S.dpPending && (e = hipEventSynchronize(S.dpDone)) != hipSuccess) return e;
  }
  if (h->dlExec >= 0 && (e = hipEventSynchronize(h->dlDone)) != hipSuccess) return e;
  if (h->upPending && (e = hipEventSynchronize(h->upDone)) != hipSuccess) return e;
  return hipSuccess;
}

static bg_aligner* aligner_init(int device, const std::shared_ptr<StreamGroup>& share) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  bg_aligner* h = new bg_aligner();
  h->device = device;
  for (int& v : h->opt) v = -1;
  if (const char* e = std::getenv("BG_OPTIONS")) {
    // "name=value,...": the tools' way to set bg_set_option (read once, here)
    std::string all(e);
    for (size_t at = 0; at <= all.size();) {
      size_t end = all.find(',', at);
      if (end == std::string::npos) end = all.size();
      const std::string kv = all.substr(at, end - at);
      const size_t eq = kv.find('=');
      if (eq != std::string::npos)
        for (int k = 0; k < BG_OPT_COUNT; ++k)
          if (kv.compare(0, eq, kOptNames[k]) == 0 && std::strlen(kOptNames[k]) == eq)
            h->opt[k] = std::atoi(kv.c_str() + eq + 1);
      at = end + 1;
    }
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    h->cus = prop.multiProcessorCount;
  if (share) {
    h->sg = share;
  } else {
    h->sg = std::make_shared<StreamGroup>();
    h->sg->device = device;
  }
  h->stream = group_stream(h, kSDp);
  h->stream2 = group_stream(h, kSFin);
  if (!h->stream || !h->stream2) {
    bg_aligner_free(h);
    return nullptr;
  }
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) { bg_aligner_free(h); return nullptr; }
  if (hipEventCreateWithFlags(&h->dlDone, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->upDone, hipEventDisableTiming) != hipSuccess) {
    bg_aligner_free(h);
    return nullptr;
  }
  for (Slot& S : h->slot)
    if (hipEventCreateWithFlags(&S.dpDone, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.finDone, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.readDone, hipEventDisableTiming) != hipSuccess) {
      bg_aligner_free(h);
      return nullptr;
    }
  return h;
}

extern "C" bg_aligner* bg_aligner_new(int device) { return aligner_init(device, nullptr); }

extern "C" bg_aligner* bg_aligner_new_shared(bg_aligner* peer) {
  if (!peer || !peer->sg) return nullptr;
  return aligner_init(peer->device, peer->sg);
}

extern "C" void bg_aligner_free(bg_aligner* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->sg) (void)drain(h);
  for (DevBuf* d : {&h->seq1, &h->seq2, &h->codes1, &h->codes2, &h->lut, &h->prof, &h->pairs, &h->recs,
                    &h->wgmapBuf, &h->gprogBuf, &h->dbgBuf, &h->dpDbg, &h->profScratch, &h->compactSizes})
    d->release();
  for (PinBuf* q : {&h->ho1, &h->ho2, &h->up, &h->hresPin}) q->release();
  for (Slot& S : h->slot) {
    for (DevBuf* d : {&S.trace, &S.bndM, &S.bndX, &S.aux, &S.out1, &S.out2, &S.results, &S.ops, &S.gran, &S.split,
                      &S.gprog, &S.keys, &S.xcnt})
      d->release();
    S.wdiag.release();
    if (S.dpDone) (void)hipEventDestroy(S.dpDone);
    if (S.finDone) (void)hipEventDestroy(S.finDone);
    if (S.resetDone) (void)hipEventDestroy(S.resetDone);
    if (S.readDone) (void)hipEventDestroy(S.readDone);
  }
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : h->ring)
    if (e) (void)hipEventDestroy(e);
  if (h->dlDone) (void)hipEventDestroy(h->dlDone);
  if (h->upDone) (void)hipEventDestroy(h->upDone);
  h->sg.reset();                   // the last handle of a group destroys its streams
  delete h;
}

extern "C" int bg_set_tuning(bg_aligner* h, int R, int waves) {
  if (!h || (R != 0 && R != 2 && R != 3 && R != 4 && R != 5 && R != 8 && R != 10) || waves < 0 || waves > 16)
    return BG_E_ARG;
  h->tuneR = R;
  h->tuneW = waves;
  return BG_OK;
}

extern "C" int bg_set_option(bg_aligner* h, int key, int value) {
  if (!h || key < 0 || key >= BG_OPT_COUNT || value < -1) return BG_E_ARG;
  h->opt[key] = value;
  return BG_OK;
}

extern "C" int bg_get_option(bg_aligner* h, int key, int* value) {
  if (!h || !value || key < 0 || key >= BG_OPT_COUNT) return BG_E_ARG;
  *value = h->opt[key];
  return BG_OK;
}

extern "C" int bg_set_kernel_options(bg_aligner* h, int allow_tagged) {
  if (!h) return BG_E_ARG;
  h->allowTag = (allow_tagged & 1) ? 1 : 0;
  h->allowCkpt = (allow_tagged & 2) ? 1 : 0;
  h->allowAck = (allow_tagged & 4) ? 1 : 0;
  h->prepared = false;
  h->executed = false;
  return BG_OK;
}

extern "C" int bg_set_pipeline(bg_aligner* h, int depth) {
  if (!h || depth < 1 || depth > 4) return BG_E_ARG;
  if (drain(h) != hipSuccess) return BG_E_HIP;
  h->depth = depth;
  h->prepared = false;   // arenas are sized at prepare time
  h->executed = false;
  return BG_OK;
}

// A failing HIP call returns BG_E_HIP; its error name goes to stderr (the ABI's status codes have
// no room for it) and to bg_last_hip_error().
static thread_local int g_lastHip = 0;
static void note_hip(hipError_t e, const char* what, int line) {
  g_lastHip = (int)e;
  std::fprintf(stderr, "biogarden_gpu: %s failed at bg_host.cpp:%d: %s (%d)\n", what, line,
               hipGetErrorName(e), (int)e);
}
#define BG_HIP(x)                                              \
  do {                                                         \
    const hipError_t bg_e_ = (x);                              \
    if (bg_e_ != hipSuccess) {                                 \
      note_hip(bg_e_, #x, __LINE__);                           \
      return BG_E_HIP;                                         \
    }                                                          \
  } while (0)

extern "C" int bg_last_hip_error(void) { return g_lastHip; }

// bg_group (bg_group.cpp, not a public entry point): the stream a handle's device shares for
// downloads and exports, so the group's gather queues there instead of on a stream of its own (a
// fifth stream shares a hardware queue with the DP stream at the box's 4 queues, and its copies
// wait behind the DPs queued there)
// It also creates the shared upload stream, so that a caller creating other streams afterwards
// (bg_group: RCCL's communicator) cannot put one of them between the device's DP, traceback,
// upload and download streams in the round-robin of hardware queues: an upload stream on the
// traceback's queue queued each batch's upload behind the previous batch's traceback, and so the
// next DP (measured: DPs 1.5 ms apart, the traceback in between, tools/r05/group_trace.sh).
extern "C" void* bg_aligner_aux_stream(bg_aligner* h) {
  if (!h || hipSetDevice(h->device) != hipSuccess) return nullptr;
  if (!h->upS) h->upS = group_stream(h, kSUp);
  if (!h->dlS) h->dlS = group_stream(h, kSDl);
  return (void*)h->dlS;
}

extern "C" int bg_set_async_fetch(bg_aligner* h, int on) {
  if (!h) return BG_E_ARG;
  BG_HIP(drain(h));
  h->asyncFetch = on ? 1 : 0;
  h->dlExec = -1;
  return BG_OK;
}

// Strip pipeline of one pair on `gw` waves: phases (64-step chunks) until its last strip ends.
static int pipeline_phases(int S, int gw, int NC, int lag = 2) {
  std::vector<int> start(S), end(S);
  int P = 0;
  for (int s = 0; s < S; ++s) {
    int st = s ? start[s - 1] + lag : 0;
    if (s >= gw) st = std::max(st, end[s - gw]);
    start[s] = st;
    end[s] = st + NC;
    P = std::max(P, end[s]);
  }
  return P;
}

// WIDE planner (tagged kernel, few large pairs): each pair gets a group of workgroups of 4 waves
// (one wave per SIMD, a lone wave issues fastest) in proportion to its cells, at most one wave
// per strip and at most the CU count in all, so every group is resident at once.  R minimises
// the slowest pair's pipeline: phases * 64 steps * the lone-wave step latency.  Measured on C3
// (BG_DEBUG=dp, conveyor step): ~48 + 10R cycles per step (the R-long v_max3 chain of a step
// plus its DPP and two LDS reads), and an effective ~5 chunks per strip: a strip starts ~3.3
// chunks after the one above (two for the anti-diagonal skew and the block, the rest hand-off),
// and every caught-up consumer adds its hand-off latency to the pace of the strips below it.
// Fitted on C3's DP at R = 2 / 4 / 5 / 8 (12.3 / 10.1 / 9.8 / 10.3 ms): R = 5.
// grouped semiglobal / overlap batches: the DP folds each pair's last-row end-cell key, so the
// traceback's one wave does not fold 10 k-column rows
static bool grp_fold(const bg_aligner* h) {
  return h->grouped && (h->mode == BG_SEMIGLOBAL || h->mode == BG_OVERLAP);
}

// Grouped planner (bg_grp_kernel.hip): every computed pair's read at most 320
// rows and its reference shared by others (the same caller buffer, or equal bytes), so that P
// pairs of one reference fill a wave, 64 / P lanes each; R is the least with (64 / P) R >= the
// longest read.  P = 4 (16-lane DPP rows) for reads up to 160, else P = 2 (a select per step).
// P = 4 wins even at 2 waves per SIMD: C4's 8 192 pairs run their DP in 1.16 ms at P = 4 (R = 10,
// 2 048 waves, 513 M VALU instructions) against 1.34 ms at P = 2 (R = 5, 4 096 waves, 674 M) —
// the DP is VALU-bound (72 % of the SIMDs' quad-cycle issue), so fewer instructions per cell beat
// more waves (profiles/r05/grouped/pmc_c4_p*.json).  Off when the groups would average under
// 0.6 P pairs.  BG_OPT_GROUPED 0 never, 1 at any fill; BG_OPT_GROUP_PAIRS 2 / 4 forces P.
// Returns P, or 0.
static int plan_grouped(bg_aligner* h, size_t npairs, const size_t* n1, const size_t* n2,
                        const uint8_t* const* s2, int64_t dmax, int* Rout, int* Wout, std::vector<int>& refOf) {
  const int og = h->o(BG_OPT_GROUPED, -1);
  if (og == 0) return 0;
  const bool force = og == 1;
  size_t maxn1 = 0, ndp = 0;
  for (size_t p = 0; p < npairs; ++p) {
    if (h->prestatus[p] >= 0 || n1[p] == 0 || n2[p] == 0) continue;
    if (n1[p] > 320) return 0;
    maxn1 = std::max(maxn1, n1[p]);
    ++ndp;
  }
  if (ndp == 0 || (ndp < 64 && !force)) return 0;
  refOf.assign(npairs, -1);
  std::map<std::pair<const uint8_t*, size_t>, int> byPtr;
  std::unordered_map<uint64_t, std::vector<int>> bySig;
  std::vector<size_t> repOf, count;
  for (size_t p = 0; p < npairs; ++p) {
    if (h->prestatus[p] >= 0 || n1[p] == 0 || n2[p] == 0) continue;
    const auto key = std::make_pair(s2[p], n2[p]);
    auto it = byPtr.find(key);
    int cls = -1;
    if (it != byPtr.end()) {
      cls = it->second;
    } else {
      // a sampled signature, then the bytes against the class representatives that share it
      uint64_t sig = 1469598103934665603ULL ^ n2[p];
      const size_t step = std::max<size_t>(1, n2[p] / 64);
      for (size_t x = 0; x < n2[p]; x += step) sig = (sig ^ s2[p][x]) * 1099511628211ULL;
      std::vector<int>& cand = bySig[sig];
      for (int c : cand)
        if (std::memcmp(s2[repOf[c]], s2[p], n2[p]) == 0) { cls = c; break; }
      if (cls < 0) {
        cls = (int)repOf.size();
        repOf.push_back(p);
        count.push_back(0);
        cand.push_back(cls);
      }
      byPtr.emplace(key, cls);
    }
    refOf[p] = cls;
    ++count[cls];
  }
  size_t g4 = 0, g2 = 0;
  for (size_t c : count) { g4 += (c + 3) / 4; g2 += (c + 1) / 2; }
  int P = maxn1 <= 160 ? 4 : 2;
  const int op = h->o(BG_OPT_GROUP_PAIRS, 0);
  if (op == 2 || (op == 4 && maxn1 <= 160)) P = op;
  (void)dmax;
  const size_t groups = P == 4 ? g4 : g2;
  if (!force && 10 * ndp < 6 * (size_t)P * groups) return 0;
  const int L = 64 / P;                                 // lanes per pair
  int R = 10;
  for (int r : {2, 3, 4, 5, 8, 10})
    if ((size_t)L * r >= maxn1) { R = r; break; }
  const int W = std::min(16, std::max(1, h->o(BG_OPT_GROUP_WAVES, 4)));
  *Rout = R;
  *Wout = W;
  h->tagRow = 0;
  return P;
}

static bool plan_wide(bg_aligner* h, const size_t* n1, const size_t* n2, size_t npairs, int* Rout,
                      int* Wout) {
  std::vector<size_t> comp;
  uint64_t cells = 0;
  for (size_t p = 0; p < npairs; ++p)
    if (h->prestatus[p] < 0 && n1[p] > 0 && n2[p] > 0) {
      comp.push_back(p);
      cells += (uint64_t)n1[p] * n2[p];
    }
  if (comp.empty() || comp.size() * 4 > (size_t)h->cus || h->tuneW || h->o(BG_OPT_WIDE, -1) == 0) return false;
  // more than cus / 8 pairs (M's 64- and 128-pair shares at 4 and 2 GPUs): the DP's throughput
  // over the strip chain's latency (plan_span), unless the SPAN kernel is switched off.  At 32
  // pairs the WIDE DP (0.97 ms) and SPAN's (1.07) are alike and WIDE's split traceback decides:
  // 3 103 GCUPS against 2 843 (SPAN, split) and 1 969 (SPAN, one walker per pair;
  // profiles/r06/shares)
  if ((comp.size() * 8 > (size_t)h->cus && h->o(BG_OPT_SPAN, -1) != 0) || h->o(BG_OPT_SPAN, -1) == 1) return false;
  size_t maxn1 = 0;
  for (size_t p : comp) maxn1 = std::max(maxn1, n1[p]);
  if (maxn1 < 64 * 4 * 16) return false;                   // one workgroup's 16 waves suffice
  // (the WIDE kernel is built for at most 4 waves per workgroup, bg_tag_kernel.hip)
  const int W = std::max(1, std::min(4, h->o(BG_OPT_WIDE_WAVES, 4)));
  const int cand[] = {2, 3, 4, 5, 8, 10};
  double best = 1e300;
  int bestR = 0;
  std::vector<int> groups(npairs, 0), bestGroups;
  for (int Rc : cand) {
    if (h->tuneR && Rc != h->tuneR) continue;
    double T = 0.0;
    for (size_t p : comp) {
      const int S = (int)((n1[p] + 64 * Rc - 1) / (64 * Rc));
      const double share = (double)h->cus * ((double)n1[p] * n2[p]) / (double)cells;
      int G = std::max(1, std::min((int)share, (S + W - 1) / W));
      groups[p] = G;
      const int NC = (int)(n2[p] / 64 + 2);
      T = std::max(T, (double)pipeline_phases(S, G * W, NC, 5) * 64.0 * (48.0 + 10.0 * Rc));
    }
    if (T < best) { best = T; bestR = Rc; bestGroups = groups; }
  }
  if (!bestR) return false;
  *Rout = bestR;
  *Wout = W;
  h->groupOf = bestGroups;
  h->tagRow = 1;                   // kept when it fits (the LDS is padded to one group per CU)
  return true;
}

// Geometry planner (DESIGN.md "Geometry").  For each strip height R and wave count W the strip
// pipeline of the largest pair is simulated phase by phase (a phase = 64 anti-diagonal steps;
// strip s starts two phases after strip s-1 and after its wave finished strip s-W).  A phase
// with a active waves per SIMD costs 64 * ops_per_step * a * (4.0 + 3.0 / a) cycles: ~4 cycles
// per VALU instruction when enough waves share the SIMD (tools/micro/tag_step.hip), and the
// measured ~5.6 at two waves per SIMD (PMC, profiles/r01/pmc_summary_ckptR10W8.json), where the
// per-step LDS and memory latencies are no longer hidden.  Workgroups per CU are bounded by
// waves (32 per CU), VGPRs and LDS; with the two-slot pipeline a finish workgroup must still fit
// beside them.  Ties within 1 % go to more waves per SIMD.
static int vgprs_of(const void* fn) {
  hipFuncAttributes at;
  if (!fn || hipFuncGetAttributes(&at, fn) != hipSuccess || at.numRegs <= 0) return 128;
  return (at.numRegs + 7) / 8 * 8;
}

// DP and finish kernels of the prepared family at strip height R (nullptr: R not built)
static void* dp_fn(const bg_aligner* h, int R) {
  if (h->tag) return bg_dp_kernel_tag_ptr(R, 0, h->ckpt);
  if (h->ack) return bg_dp_aff_kernel_ptr(R, h->local);
  if (h->p32) return bg_dp_kernel_p32_ptr(R, h->affine, h->local, h->pglob);
  if (h->finFlags & BG_FIN_LCS) return bg_dp_kernel_lcs_ptr(R, h->dna);
  return bg_dp_kernel_ptr(R, h->affine, h->local, h->dna);
}
static void* fin_fn(const bg_aligner* h, int R) {
  if (h->ack) return bg_finish_ack_kernel_ptr(R, h->mode);
  if (h->ckpt) return bg_finish_ck_kernel_ptr(R, h->mode);
  return bg_finish_kernel_ptr(R, h->affine, h->mode);
}
// Finish workgroup of the checkpoint modes: waves (the walker + recompute helpers) and
// recomputed-chunk slots.  Few pairs: 4 waves and every slot (the walk's latency is the step's
// tail).  Many pairs: fewer waves and slots, so more pairs walk per CU at once (the walks are
// latency-bound).  BG_OPT_FIN_WAVES / BG_OPT_FIN_SLOTS override.
static void fin_geom(const bg_aligner* h, size_t np, int* nw, int* nslots) {
  *nw = 4;
  *nslots = 0;
  // many pairs: two waves (walker + one recomputing helper at each miss) and three slots
  // (tools/fin_geom_sweep.sh: one wave / two slots C2 1 266, C4 5 630, C5 2 274 GCUPS; two waves /
  // three slots 1 269, 6 017, 2 396; four waves 1 298, 6 039, 2 123)
  if ((h->ack || h->ckpt) && np > (size_t)h->cus * 2) { *nw = 2; *nslots = 3; }
  // local (affine checkpoint) batches: one wave and two slots, the walker recomputing its own
  // misses — more walks per CU beside the DP (tools/fin_geom_np.py at three pipeline slots: C2
  // shape 1 548 -> 1 656 / 1 767 -> 1 854 GCUPS at 1 024 / 4 096 pairs; the C5 shape, global
  // protein, loses with it: 2 576 -> 2 490)
  if (h->ack && h->local && np > (size_t)h->cus * 2) { *nw = 1; *nslots = 2; }
  // grouped pairs: the walker recomputes up to four 16-lane chunks in one pass itself (one wave)
  // into small slots (bg_finish.h recompute_grp)
  if (h->grouped) { *nw = 1; *nslots = 6; }
  if (h->opt[BG_OPT_FIN_WAVES] >= 0) *nw = std::min(4, std::max(1, h->opt[BG_OPT_FIN_WAVES]));
  if (h->opt[BG_OPT_FIN_SLOTS] >= 0) *nslots = h->opt[BG_OPT_FIN_SLOTS];
  if (*nslots && *nslots < *nw + 1) *nslots = *nw + 1;
  if (h->grouped && *nslots && *nslots < 4) *nslots = 4;
}

// LDS of one finish workgroup (and the window / recompute-area sizes it launches with)
static size_t fin_lds(const bg_aligner* h, int R, size_t np, int* win, int* area) {
  *area = 0;
  int nw = 4, ns = 0;
  fin_geom(h, np, &nw, &ns);
  if (h->ack) return bg_finish_ack_lds_bytes(R, h->kdim, h->local, ns, nw, win, area);
  if (h->ckpt && h->grouped) return bg_finish_grp_lds_bytes(h->grouped, R, ns, nw, win);
  if (h->ckpt) return bg_finish_ck_lds_bytes(R, ns, nw, win);
  *win = bg_finish_window_bytes(R, h->affine, np, h->cus);
  return bg_finish_lds_bytes(*win);
}

// affine / local checkpoint traceback: per-row cost R^2 coefficient.  Fitted on the step, not on
// the finish kernel alone (C5 at R = 4 / R = 2: finish 1.22x at the same wave count, but the
// step pays the R = 4 recomputation again as interference with the next DP): 24 picks R = 2 for
// C5 (tools/c5_sweep.sh, tools/cfg_lib_ab.sh) and keeps C2's R = 2.
#ifndef BG_FIN_R2
#define BG_FIN_R2 24.0
#endif
static constexpr double kFinR2 = BG_FIN_R2;

// SPAN planner (linear checkpoint path, fewer pairs than CUs: one batch strong-scaled over
// several GPUs, SURVEY §8(d) M at G = 2, 4, 8): each pair's strips are dealt over a group of
// many-wave workgroups, W consecutive strips per workgroup and round, the boundary row handed to
// the next workgroup through HBM (bg_dp_tag_kernel<R, 2, true>).  One pair per CU (the
// one-workgroup plan) leaves cus - npairs CUs idle; the group spreads a pair over
// cus * cells_p / cells CUs.  Per (R, W) the strip pipeline of every distinct pair shape is
// simulated phase by phase as in plan_geometry (a strip starts two phases after the one above in
// its workgroup, three across workgroups, and after its wave's previous strip ended; a phase with
// a active waves per SIMD on the busiest workgroup of the group costs 64 * (2R + 2) * a *
// (4 + 3 / a) cycles); the slowest pair's estimate decides, and the group plan is kept only when
// it beats the same simulation at one workgroup per pair.  BG_OPT_SPAN: 0 never, 1 whenever the
// batch qualifies.
static double span_estimate(int S, int G, int W, int NC, int ops) {
  const int GW = G * W;
  std::vector<int> start(S), end(S), wg(S);
  int P = 0;
  for (int s = 0; s < S; ++s) {
    wg[s] = (s % GW) / W;
    int st = 0;
    if (s) st = start[s - 1] + (wg[s] == wg[s - 1] ? 2 : 3);
    if (s >= GW) st = std::max(st, end[s - GW]);
    start[s] = st;
    end[s] = st + NC;
    P = std::max(P, end[s]);
  }
  std::vector<int> act((size_t)P * G, 0);
  for (int s = 0; s < S; ++s)
    for (int q = start[s]; q < end[s]; ++q) ++act[(size_t)q * G + wg[s]];
  double T = 0.0;
  for (int q = 0; q < P; ++q) {
    int A = 0;
    for (int g = 0; g < G; ++g) A = std::max(A, act[(size_t)q * G + g]);
    const int a = std::max(1, (A + 3) / 4);
    T += 64.0 * ops * a * (4.0 + 3.0 / a);
  }
  return T;
}

static bool plan_span(bg_aligner* h, const size_t* n1, const size_t* n2, size_t npairs, int* Rout,
                      int* Wout) {
  const int os = h->o(BG_OPT_SPAN, -1);
  if (os == 0 || (h->tuneW && os != 1)) return false;
  std::vector<size_t> comp;
  uint64_t cells = 0;
  for (size_t p = 0; p < npairs; ++p)
    if (h->prestatus[p] < 0 && n1[p] > 0 && n2[p] > 0) {
      comp.push_back(p);
      cells += (uint64_t)n1[p] * n2[p];
    }
  if (comp.empty() || comp.size() * 2 > (size_t)h->cus) return false;
  size_t maxn1 = 0, maxn2 = 0;
  for (size_t p : comp) { maxn1 = std::max(maxn1, n1[p]); maxn2 = std::max(maxn2, n2[p]); }
  const int cand[] = {2, 3, 4, 5, 8, 10};
  double best = 1e300, best1 = 1e300;
  int bestR = 0, bestW = 0;
  std::vector<int> groups(npairs, 0), bestGroups;
  std::map<std::pair<std::pair<size_t, size_t>, int>, double> memo;
  // relax: no candidate leaves a traceback wave's VGPRs beside the DP's on each SIMD
  for (int relax = 0; relax < 2 && !bestR; ++relax)
  for (int Rc : cand) {
    if (h->tuneR && Rc != h->tuneR) continue;
    const void* fn = bg_dp_kernel_tag_ptr(Rc, 2, 1);
    if (!fn) continue;
    const int vg = vgprs_of(fn);
    const int fin = (h->depth > 1 && !relax) ? vgprs_of(fin_fn(h, Rc)) : 0;
    const int ops = 2 * Rc + 2;
    for (int Wc : {4, 8, 12, 16}) {
      if (h->tuneW && Wc != h->tuneW) continue;
      const int wps = (Wc + 3) / 4;
      if (wps * vg + fin > 512 && !h->tuneW) continue;
      if (640 + (size_t)Wc * bg_dp_tag_wave_lds_bytes(Rc) > 160 * 1024) continue;
      double T = 0.0, T1 = 0.0;
      int total = 0;
      memo.clear();
      for (size_t p : comp) {
        const int S = (int)((n1[p] + 64 * Rc - 1) / (64 * Rc));
        const double share = (double)h->cus * ((double)n1[p] * n2[p]) / (double)cells;
        const int G = std::max(1, std::min((int)share, (S + Wc - 1) / Wc));
        groups[p] = G;
        total += G;
        const int NC = (int)(n2[p] / 64 + 2);
        auto key = std::make_pair(std::make_pair(n1[p], n2[p]), G);
        auto it = memo.find(key);
        const double t = it != memo.end() ? it->second : (memo[key] = span_estimate(S, G, Wc, NC, ops));
        T = std::max(T, t);
        T1 = std::max(T1, span_estimate(S, 1, Wc, NC, ops));
      }
      if (total > h->cus) continue;
      // within 5 % the taller strips win: fewer instructions per cell than the model charges them
      // (64 pairs: R = 10 / W = 4 ran 5 111 GCUPS against 4 788 for the estimate's R = 5 / W = 8,
      // 2.7 % apart in the model; profiles/r06/span_sweep/)
      if (T < best * 0.95 || (T < best * 1.05 && Rc > bestR)) {
        best = T; bestR = Rc; bestW = Wc; bestGroups = groups;
      }
      best1 = std::min(best1, T1);
    }
  }
  if (!bestR) return false;
  bool multi = false;
  for (size_t p : comp) multi |= bestGroups[p] > 1;
  if (!multi || (os < 0 && best > 0.9 * best1)) return false;
  if (dbg_flags().plan)
    std::fprintf(stderr, "plan span R %d W %d T %.4g (one workgroup per pair %.4g)\n", bestR, bestW, best, best1);
  *Rout = bestR;
  *Wout = bestW;
  h->groupOf = bestGroups;
  h->tagRow = 1;
  return true;
}

static void plan_geometry(bg_aligner* h, size_t maxn1, size_t maxn2, size_t ncomp, int* Rout,
                          int* Wout) {
  const int cand[] = {2, 3, 4, 5, 8, 10};
  const size_t np = std::max<size_t>(ncomp, 1);
  const int NC = (int)(maxn2 / 64 + 2);
  double best = 1e300;
  struct Cand { double T; int R, W, wps, row, wavesCu; };
  std::vector<Cand> cands;
  std::vector<int> start, end, diff;
  // relax: no candidate leaves room for a finish workgroup beside the DP's (big alphabets: both
  // hold a K x 64 profile table) — plan the DP alone; the finish then waits for LDS
  for (int relax = 0; relax < 2 && cands.empty(); ++relax)
  for (int Rc : cand) {
    if (h->tuneR && Rc != h->tuneR) continue;
    const void* fn = dp_fn(h, Rc);
    if (!fn) continue;
    // the affine-family kernels stage codes pre-scaled by 256 * RW bytes in u16: RW = 2 (R = 8)
    // holds codes < 128 only
    if (h->ack && h->kdim > 128 && Rc > 4) continue;
    const int vg = vgprs_of(fn);
    const int fin = (h->depth > 1 && !relax) ? vgprs_of(fin_fn(h, Rc)) : 0;
    // LDS of one finish workgroup that must fit beside the DP's when pipelining
    size_t finLds = 0;
    if (h->depth > 1 || h->ack) {
      int win = 0, area = 0;
      finLds = fin_lds(h, Rc, np, &win, &area);
    }
    const size_t finLdsRes = (h->depth > 1 && !relax) ? finLds : 0;   // must fit beside the DP's
    const int opsPerStep = h->ack ? (h->local ? 8 * Rc + 4 : 6 * Rc + 4)
                         : h->ckpt ? 2 * Rc + 2 : (h->tag ? 5 * Rc + 2 : (h->affine ? 18 * Rc + 16 : 8 * Rc + 12));
    const int S = maxn1 ? (int)((maxn1 + 64 * Rc - 1) / (64 * Rc)) : 1;
    // many pairs on the affine / local checkpoint path: at most 4 waves per pair (C5: R = 2 runs
    // W = 4 at 2 232 GCUPS, W = 8 at 2 077; every CU holds several pairs anyway).  With fewer
    // than two pairs per CU a 4-wave workgroup leaves one wave per SIMD and the step's dependent
    // chain unhidden (MA, 256 x 10k x 10k -11/-1: R = 2 / W = 4 DP 13.3 ms, R = 8 / W = 8 5.9 ms)
    const bool manyAck = h->ack && np >= 2 * (size_t)h->cus;
    const int wmax = (!h->ack && (h->affine || h->local)) ? 8 : ((manyAck && !h->tuneW) ? 4 : 16);
    for (int Wc = 1; Wc <= wmax; ++Wc) {
      if (h->tuneW && Wc != h->tuneW) continue;
      if (Wc > S && !h->tuneW) continue;
      // many pairs on the affine / local path: wave counts that divide over the 4 SIMDs (W = 3
      // estimates best for C5 and measures worst: 2 089 GCUPS against 2 232 at R = 2 / W = 4)
      if (manyAck && !h->tuneW && (Wc & (Wc - 1))) continue;
      const int wps = (Wc + 3) / 4;                      // waves per SIMD per workgroup
      const int want = (int)((np + h->cus - 1) / h->cus);
      int wg = std::min(want, 32 / Wc);
      // VGPRs: a workgroup's waves spread over the 4 SIMDs; each SIMD keeps room for one
      // traceback wave when pipelining
      if (Wc >= 4) wg = std::min(wg, (512 - fin) / (wps * vg));
      else wg = std::min(wg, 4 * ((512 - fin) / vg) / Wc);
      bool rowc = false;
      if (h->tag) {
        // the code row in LDS saves per-chunk staging, unless it costs co-resident workgroups
        const size_t waves = (size_t)Wc * bg_dp_tag_wave_lds_bytes(Rc);
        const size_t row = round_up(2 * (64 + (maxn2 / 64 + 4) * 64), 16);
        const size_t ldsCu = 160 * 1024 > finLdsRes ? 160 * 1024 - finLdsRes : 0;
        const int wgNoRow = (int)(ldsCu / (640 + waves));
        const int wgRow = (int)(ldsCu / (640 + waves + row));
        rowc = wgRow >= std::min(wg, wgNoRow) && wgRow >= 1;
        wg = std::min(wg, rowc ? wgRow : wgNoRow);
        if (wg < 1) {
          if (!(h->tuneR && h->tuneW)) continue;
          wg = 1;
        }
      }
      if (!h->tag && !h->ack && !h->dna) {
        // mask kernel, LDS profiles: lut, the 32 x 32 table, then per wave K x 64 lanes x WPE
        const size_t wpe = h->p32 ? (size_t)Rc : (size_t)(Rc + 1) / 2;
        if (!h->pglob && 256 + (h->p32 ? 4096 : 2048) + (size_t)h->kdim * 64 * wpe * 4 + 64 > 160 * 1024) continue;
      }
      if (h->ack) {
        const size_t ldsCu = 160 * 1024 > finLdsRes ? 160 * 1024 - finLdsRes : 0;
        const size_t one = bg_dp_aff_head_bytes() + (size_t)Wc * bg_dp_aff_wave_lds_bytes(Rc, h->kdim);
        if (one > 160 * 1024) continue;
        wg = std::min(wg, (int)(ldsCu / one));
      }
      if (wg < 1) {
        if (!(h->tuneR && h->tuneW)) continue;
        wg = 1;
      }
      start.assign(S, 0);
      end.assign(S, 0);
      for (int s = 0; s < S; ++s) {
        int st = s ? start[s - 1] + 2 : 0;
        if (s >= Wc) st = std::max(st, end[s - Wc]);
        start[s] = st;
        end[s] = st + NC;
      }
      const int P = end[S - 1] > 0 ? *std::max_element(end.begin(), end.end()) : 0;
      diff.assign(P + 1, 0);
      for (int s = 0; s < S; ++s) { ++diff[start[s]]; --diff[end[s]]; }
      double T = 0.0;
      int A = 0;
      for (int p = 0; p < P; ++p) {
        A += diff[p];
        const int a = std::max(1, (A * wg + 3) / 4);
        T += 64.0 * opsPerStep * a * (4.0 + 3.0 / a);
      }
      // workgroups are dealt dynamically, so a partial last round costs its share, not a full
      // round (C4, 32 pairs per CU: R = 3 at 28 resident runs 1.14 rounds, 1.80 ms, against
      // R = 5 at 16 resident, 2 rounds, 2.32 ms; a whole-round count picked R = 5)
      const double rounds = std::max(1.0, (double)np / ((double)h->cus * wg));
      T *= rounds;
      if (h->ack) {
        // the traceback recomputes the chunks its path crosses: per pair ~ (600 + 8R^2) cycles
        // per row of walk and recomputation (BG_DEBUG=finish, C2 / C5), with as many pairs in
        // flight per CU as the finish workgroup's LDS allows
        const double fwg = std::max(1.0, std::floor(160.0 * 1024 / (double)std::max<size_t>(finLds, 1)));
        const double frounds = std::ceil((double)np / ((double)h->cus * fwg));
        const double Tf = frounds * (600.0 + kFinR2 * Rc * Rc) * (double)(maxn1 + maxn2) * 0.5;
        // pipelined (depth > 1): the traceback of step k runs beside the DP of step k + 1; the
        // step is the longer of the two plus ~0.2 of the shorter (interference), as measured
        // on MA across R = 2..8, W = 4..16 (tools/aff_sweep.sh)
        T = (h->depth > 1 && !manyAck) ? std::max(T, Tf) + 0.2 * std::min(T, Tf) : T + Tf;
      }
      const int wpsAll = wps * wg;
      cands.push_back({T, Rc, Wc, wpsAll, rowc ? 1 : 0, wg * Wc});
      best = std::min(best, T);
    }
  }
  // within 5 % of the best estimate: taller strips (fewer per-step overhead ops per cell; the
  // pipeline tail the model charges for is filled by the overlapped traceback), then more waves
  // per SIMD, then the estimate
  const Cand* pick = nullptr;
  const bool manyAckPlan = h->ack && !h->tuneW && np >= 2 * (size_t)h->cus;
  if (dbg_flags().plan)
    for (const Cand& c : cands)
      std::fprintf(stderr, "plan R %d W %d wps %d T %.4g\n", c.R, c.W, c.wps, c.T);
  // (the affine / local checkpoint path pays taller strips again in the traceback's
  // recomputation: lowest estimate)
  for (const Cand& c : cands) {
    if (h->ack) {
      // many pairs: within 8 % of the best estimate, the most DP waves resident per CU (the
      // model undervalues occupancy there: C5, R = 2, W = 2 keeps 14 waves per CU against 12 for
      // W = 4 and runs 2 753 against 2 576 GCUPS at an estimate 7 % higher; C2's W = 4 holds the
      // most waves and the lowest estimate); otherwise the lowest estimate
      // (W = 1 excluded: one wave per pair hands every strip's row through HBM and rebuilds the
      // strip prologue alone, which the phase model does not see: C5 at R = 2, W = 1 runs its DP in
      // 8.7 ms against 5.9 for W = 2)
      if (manyAckPlan && c.W >= 2 && c.T <= best * 1.08) {
        if (!pick || c.wavesCu > pick->wavesCu || (c.wavesCu == pick->wavesCu && c.T < pick->T)) pick = &c;
        continue;
      }
      if (c.T > best * 1.05) continue;
      if (!pick || c.T < pick->T) pick = &c;
      continue;
    }
    if (c.T > best * 1.05) continue;
    if (!pick || c.R > pick->R || (c.R == pick->R && (c.wps > pick->wps || (c.wps == pick->wps && c.T < pick->T))))
      pick = &c;
  }
  if (pick) {
    *Rout = pick->R;
    *Wout = pick->W;
    h->tagRow = pick->row;
  } else if (h->ack && h->kdim > 128 && dp_fn(h, 4)) {
    *Rout = 4;                           // one wave, the R the 8-bit codes allow
    *Wout = 1;
  }
}

static int prepare_impl(bg_aligner* h, int mode, size_t npairs, const uint8_t* const* s1,
                        const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                        const HScore& S, int32_t a, int32_t b) {
  if (!h || mode < BG_GLOBAL || mode > BG_SEMIGLOBAL || S.K < 1 || S.K > 256) return BG_E_ARG;
  if (npairs && (!s1 || !n1 || !s2 || !n2)) return BG_E_ARG;
  // the pending per-pair dims (aligner calls only): copied, and consumed only when this prepare
  // succeeds, so a prepare that fails early (argument, HIP or memory error) leaves them for a retry
  std::vector<std::pair<long, long>> callDims;
  if (!h->finFlags) callDims = h->callDims;
  PhaseTimer tm(h->hostMs);
  ++h->nPrepare;
  BG_HIP(drain(h));
  tm.mark(kPhSync, "sync");
  for (Slot& S : h->slot) S.inflight = S.readPending = S.dpPending = false;
  h->dlExec = -1;
  h->execCount = 0;
  h->prepared = false;
  h->executed = false;
  h->mode = mode;
  h->a = a;
  h->b = b;
  h->npairs = npairs;
  h->n1v.assign(n1, n1 + npairs);
  h->n2v.assign(n2, n2 + npairs);
  h->outoff.resize(npairs);
  uint64_t off = 0;
  for (size_t p = 0; p < npairs; ++p) {
    h->outoff[p] = off;
    off += n1[p] + n2[p];
  }
  h->outBytes = off;

  // ---- per-pair validation, in the reference's order, and the staging pass (bg_host_passes.h):
  // the raw residues go to pinned staging in caller order (the plan's LPT order only permutes
  // BgPair records, never the bytes), with each pair's score-code set, in one read of the
  // caller's buffers
  if (bgh::stage_validate(mode, npairs, s1, n1, s2, n2, a, b, h->prestatus, h->coff1, h->coff2))
    return BG_E_ARG;
  const uint64_t o1 = h->coff1[npairs], o2 = h->coff2[npairs];
  if (!h->up.ensure(o1 + o2 + 512)) return BG_E_NOMEM;
  uint8_t* st1 = h->up.as<uint8_t>();
  uint8_t* st2 = st1 + o1 + 16;
  std::vector<char> present;
  bgh::stage_copy(npairs, s1, n1, s2, n2, S, h->prestatus, h->coff1, h->coff2, st1, st2, h->pmask,
                  h->pmaskW, present);

  tm.mark(kPhStage, "validate+stage");
  // ---- the reference's scratch history over the batch's calls (aligner.rs:92-94): the
  // argument errors return before the resize, everything else (the score panic included)
  // resizes first.  Edit distance and LCS do not use a SequenceAligner.
  // A shard's calls may start from dims given per pair (bg_aligner_set_call_dims): the history
  // of the whole batch, replayed by the caller; the dims after the shard follow its last call.
  if (!callDims.empty() && callDims.size() != npairs) return BG_E_ARG;
  long bufR = h->bufRows, bufC = h->bufCols;
  bgh::call_history(npairs, n1, n2, h->prestatus, callDims, h->finFlags != 0, bufR, bufC, h->bufAt);

  // ---- dense alphabet, profile, kernel family
  const int KS = S.K;
  std::vector<int> dense(KS);
  int K = 0;
  for (int c = 0; c < KS; ++c) dense[c] = present[c] ? K++ : -1;
  int32_t maxAbsS = 0;
  for (int q = 0; q < KS; ++q)
    for (int c = 0; c < KS; ++c)
      if (present[q] && present[c]) maxAbsS = std::max<int32_t>(maxAbsS, std::abs(S.at(q, c)));
  bool dnaOK = K <= 4;
  bool i16OK = true;
  for (int q = 0; q < KS; ++q)
    for (int c = 0; c < KS; ++c) {
      if (!present[q] || !present[c]) continue;
      const int64_t v = (int64_t)S.at(q, c) - (int64_t)a;
      if (v < -128 || v > 127) dnaOK = false;
      if (v < -32768 || v > 32767) i16OK = false;
    }
  // S - a beyond int16 (the reference's closure is any i32): the mask kernel with int32 profile
  // entries (bg_dp_kernel<4, ..., P32>), which keeps the reference's wrapping i32 arithmetic
  h->p32 = (!dnaOK && !i16OK) ? 1 : 0;
  // one wave's K x 64 x R int32 profile (R = 4) beyond the CU's LDS: the tables go to HBM
  h->pglob = (h->p32 && 256 + 4096 + (size_t)std::max(K, 1) * 64 * 4 * 4 + 64 > 160 * 1024) ? 1 : 0;
  h->dna = dnaOK ? 1 : 0;
  h->kdim = std::max(K, 1);
  h->pstride = std::max(K, 32);         // row stride of the int16 profile table in HBM
  h->local = mode == BG_LOCAL;

  size_t maxn1 = 0, maxn2 = 0, ncomp = 0;
  for (size_t p = 0; p < npairs; ++p)
    if (h->prestatus[p] < 0) {
      maxn1 = std::max(maxn1, n1[p]);
      maxn2 = std::max(maxn2, n2[p]);
      ++ncomp;
    }
  // linear-gap kernel iff a >= b (x/y traces provably 'M') and no intermediate can wrap
  const double bound = ((double)maxAbsS + std::abs((double)a) + std::abs((double)b)) *
                       ((double)maxn1 + (double)maxn2 + 2.0);
  h->affine = (a >= b && bound < 1073741824.0) ? 0 : 1;
  // tagged linear kernel: values 4(M - a(i+j)) + tag must stay far from overflow and the
  // profile bytes 4(S-2a)-2 / -3 must fit int8
  bool tagOK = h->allowTag && !h->affine && mode != BG_LOCAL && dnaOK && bound < 134217728.0;
  for (int q = 0; q < KS && tagOK; ++q)
    for (int c = 0; c < KS && tagOK; ++c)
      if (present[q] && present[c]) {
        const int64_t v = 4 * ((int64_t)S.at(q, c) - 2 * (int64_t)a);
        if (v - 3 < -128 || v - 2 > 127) tagOK = false;
      }
  h->tag = tagOK ? 1 : 0;
  int64_t dmaxS2a = -((int64_t)1 << 40);       // max S - 2a over the batch's codes (grouped DP's int16 bound)
  for (int q = 0; q < KS; ++q)
    for (int c = 0; c < KS; ++c)
      if (present[q] && present[c]) dmaxS2a = std::max<int64_t>(dmaxS2a, (int64_t)S.at(q, c) - 2 * (int64_t)a);
  bool ckLimit = false;   // a pair beyond the checkpoint tracebacks' chunk keys (BG_CK_MAX_*)
plan_again:
  h->ckpt = (h->tag && h->allowCkpt && !ckLimit) ? 1 : 0;
  // affine / local score-only kernel (bg_aff_common.h): int8 profile entries S - 2a (local
  // S - a); values, and the finite -inf drifting by e = b - a per step, far from wrapping
  bool ackOK = !h->tag && h->allowAck && bound < 268435456.0 &&
               std::abs((double)b - (double)a) * ((double)maxn1 + (double)maxn2 + 2.0) < 268435456.0;
  for (int q = 0; q < KS && ackOK; ++q)
    for (int c = 0; c < KS && ackOK; ++c)
      if (present[q] && present[c]) {
        // profile bytes: local S - a; otherwise S - a - b (the opened frame, bg_aff_common.h)
        const int64_t v = (int64_t)S.at(q, c) - (int64_t)a - (mode == BG_LOCAL ? 0 : (int64_t)b);
        if (v < -128 || v > 127) ackOK = false;
      }
  h->ack = (ackOK && !ckLimit) ? 1 : 0;
  // more than 32 symbols in the batch off the score-only affine family: the mask-trace kernel
  // reads its K x K table (row stride pstride) from HBM while it builds the per-lane profiles,
  // and the planner keeps one wave's K x 64 profile within the CU's LDS (R <= 2 at K = 256)

  // ---- geometry: rows per lane R, waves per workgroup W (one workgroup per pair, or a group
  // of workgroups per pair in the tagged kernel's WIDE mode)
  int R = 8, W = 1;
  h->wide = 0;
  h->span = 0;
  h->grouped = 0;
  std::vector<int> refOf;     // grouped DP: caller pair -> reference class (-1: not grouped)
  if (h->tag && h->ckpt && !h->finFlags) h->grouped = plan_grouped(h, npairs, n1, n2, s2, dmaxS2a, &R, &W, refOf);
  if (h->grouped) {
  } else if (h->tag && plan_wide(h, n1, n2, npairs, &R, &W)) h->wide = 1;
  else if (h->tag && h->ckpt && !h->finFlags && plan_span(h, n1, n2, npairs, &R, &W)) h->span = 1;
  else plan_geometry(h, maxn1, maxn2, ncomp, &R, &W);
  if ((h->ckpt || h->ack) && ncomp &&
      ((maxn1 + 64 * R - 1) / (64 * R) >= BG_CK_MAX_STRIPS || maxn2 / 64 + 2 >= BG_CK_MAX_CHUNKS)) {
    ckLimit = true;
    goto plan_again;
  }
  tm.mark(kPhPlan, "plan");
  size_t lds = 0;
  if (h->grouped) {
    // grouped DP (bg_grp_kernel.hip): the shared dummy ring (512 B), then per wave the row-0
    // block, four output rings, profile entries and the chunk's codes
    h->progOff = 0;
    h->codesOff = 0;
    h->codesInLds = 0;
    h->auxLdsOff = 512;
    lds = 512 + (size_t)W * bg_dp_grp_wave_lds_bytes(R, h->grouped);
  } else if (h->tag) {
    // tagged kernel (bg_tag_kernel.hip): 16 produced + 16 consumed counters, then per wave the
    // boundary block, output ring, profile entries, the current chunk's codes and the mailbox
    h->progOff = 0;                  // counters + shared dummy ring: 640 B
    h->codesOff = 640;
    const size_t waves = (size_t)W * bg_dp_tag_wave_lds_bytes(R);
    const size_t row = round_up(2 * (64 + (maxn2 / 64 + 4) * 64), 16);
    h->codesInLds = (h->tagRow && 640 + row + waves <= 160 * 1024) ? 1 : 0;
    // WIDE pairs whose u16 row does not fit: the row as 2-bit codes (4 columns per byte), so
    // no chunk of the strip pipeline loads its codes from HBM (a per-chunk load made the
    // compiler drain the previous chunk's stores at every chunk start)
    const size_t packed = round_up((size_t)(maxn2 / 64 + 5) * 16, 16);
    if (!h->codesInLds && h->wide && 640 + packed + waves <= 160 * 1024) h->codesInLds = 2;
    h->auxLdsOff = (int)(640 + (h->codesInLds == 1 ? row : (h->codesInLds == 2 ? packed : 0)));
    lds = h->auxLdsOff + waves;
    // WIDE: one workgroup (one wave per SIMD) per CU — claim over half of the CU's LDS so the
    // dispatcher cannot stack a group's workgroups on one CU
    if (h->wide) lds = std::max<size_t>(lds, 80 * 1024 + 64);
  } else if (h->ack) {
    // affine kernel (bg_aff_kernel.hip): counters + dummy ring, then per wave the (M, X)
    // boundary block, output ring, profile entries, chunk codes and mailbox
    h->progOff = 0;
    h->codesOff = 0;
    h->codesInLds = 0;
    h->auxLdsOff = bg_dp_aff_head_bytes();
    for (;;) {
      lds = h->auxLdsOff + (size_t)W * bg_dp_aff_wave_lds_bytes(R, h->kdim);
      if (lds <= 160 * 1024 || W == 1) break;
      --W;
    }
  } else {
    lds = 256;               // lut (+ int16 / int32 table and per-wave profiles on the LDS path)
    if (h->pglob) {
      lds = 256 + 4096;      // lut + the 32 x 32 int32 table slot; the profiles live in HBM
    } else if (!h->dna) {
      const int WPE = h->p32 ? R : (R + 1) / 2;
      for (;;) {
        lds = 256 + (h->p32 ? 4096 : 2048) + (size_t)W * h->kdim * 64 * WPE * 4;
        if (lds + 64 <= 160 * 1024 || W == 1) break;
        --W;
      }
      if (lds + 64 > 160 * 1024) return BG_E_ALPHABET;   // unreachable: pglob covers it
    }
    h->progOff = (int)lds;   // 16 per-wave progress counters follow
    lds += 64;
    h->codesOff = (int)lds;
    // seq2 codes staged in LDS when they fit next to the rest (160 KiB per CU)
    const size_t need = round_up(maxn2 + 16, 16);
    h->codesInLds = (lds + need <= 160 * 1024) ? 1 : 0;
    if (h->codesInLds) lds += need;
    h->auxLdsOff = (int)lds;
  }
  h->R = R;
  h->W = W;
  h->lds = lds;

  // ---- plan: LPT order, arenas
  const int NW = h->affine ? 4 : 2;
  std::vector<size_t> order;
  for (size_t p = 0; p < npairs; ++p)
    if (h->prestatus[p] < 0) order.push_back(p);
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
    return (uint64_t)n1[x] * n2[x] > (uint64_t)n1[y] * n2[y];
  });
  h->plan.clear();
  h->plan.reserve(order.size());
  h->wgmap.clear();
  h->progWords = 0;
  uint64_t tro = 0, bo = 0, ao = 0, oo = 0, po = 0;
  h->cells = 0;
  for (size_t p : order) {
    BgPair P;
    std::memset(&P, 0, sizeof(P));
    P.n1 = (int32_t)n1[p];
    P.n2 = (int32_t)n2[p];
    P.index = (int32_t)h->plan.size();
    P.caller = (int32_t)p;
    P.caller_off = h->outoff[p];
    P.off1 = h->coff1[p];
    P.off2 = h->coff2[p];
    const bool dp = n1[p] > 0 && n2[p] > 0;
    P.nstrips = dp ? (int32_t)((n1[p] + 64 * R - 1) / (64 * R)) : 0;
    P.pad = P.nstrips * 64 * R - P.n1;
    P.nc = (int32_t)(n2[p] / 64 + 2);
    P.trace_off = tro;
    if (h->ckpt)   // checkpoints: R + 1 ints per lane per chunk
      tro += round_up((uint64_t)P.nstrips * P.nc * (R + 1) * BG_WAVE * 4, 256);
    else if (h->ack)   // checkpoints: 2R + 2 ints per lane per chunk
      tro += round_up((uint64_t)P.nstrips * P.nc * (2 * R + 2) * BG_WAVE * 4, 256);
    else
      tro += round_up((uint64_t)P.nstrips * P.nc * (BG_CHUNK / BG_TRACE_BLK) * R * NW * BG_WAVE * 4, 256);
    P.bnd_off = bo;
    bo += (uint64_t)P.nstrips * P.nc * BG_CHUNK;
    P.aux_off = ao;
    ao += round_up((uint64_t)(n1[p] + 1) + (h->local ? 2 * n1[p] : 0), 64);
    P.out_off = oo;
    oo += n1[p] + n2[p];
    P.ops_off = po;
    po += (n1[p] + n2[p] + 3) / 4;
    P.wg_count = (h->wide || h->span) ? std::max(1, h->groupOf[p]) : 1;
    P.prog_off = (h->wide || h->span) ? h->progWords : 0;
    P.buf_rows = (int32_t)std::min<long>(h->bufAt[p].first, 0x7FFFFFFF);
    P.buf_cols = (int32_t)std::min<long>(h->bufAt[p].second, 0x7FFFFFFF);
    if (h->wide || h->span) {
      // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8
      // share one, MI355X_MICROARCH.md), so consecutive indices in the group (consecutive strips:
      // a boundary row handed through HBM) go to blocks of one XCD class, and the hand-offs stay
      // inside one XCD's L2 except at the seven class boundaries.
      const int b0 = (int)h->wgmap.size(), G = P.wg_count;
      int cls[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int g = 0; g < G; ++g) ++cls[(b0 + g) & 7];
      int first[8], seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int x = 0, acc = 0; x < 8; ++x) { first[(b0 + x) & 7] = acc; acc += cls[(b0 + x) & 7]; }
      for (int g = 0; g < G; ++g) {
        const int x = (b0 + g) & 7;
        h->wgmap.push_back(make_int2((int)h->plan.size(), first[x] + seen[x]++));
      }
      h->progWords += (uint32_t)(P.wg_count * W);
    }
    h->cells += (uint64_t)n1[p] * n2[p];
    h->plan.push_back(P);
  }
  // split traceback: WIDE linear checkpoint batches (few long pairs), exits within the packed
  // field (n2 below the symbolic range), some pair with more than one strip
  h->split = 0;
  h->splitMap.clear();
  h->splitBases.clear();
  h->splitItems = h->splitResolve = 0;
  h->splitInts = 0;
  {
    h->segc = std::max(1, h->o(BG_OPT_SPLIT_SEGMENT, BG_SPLIT_SEGC));
    // SPAN batches only on request (BG_OPT_SPLIT = 1): at 64 and 128 pairs the split traceback's
    // phases take longer than the one walker per pair they replace (128: 2.89 against 1.71 ms,
    // 4 293 against 7 119 GCUPS; profiles/r06/shares)
    const int osp = h->o(BG_OPT_SPLIT, -1);
    bool ok = (h->wide || (h->span && osp == 1)) && h->ckpt && !h->affine && !h->finFlags && mode != BG_LOCAL &&
              osp != 0;
    bool multi = false;
    for (const BgPair& P : h->plan) {
      if (P.n2 + 1 >= BG_SPLIT_SYM(R)) ok = false;
      if (P.nstrips >= 2) multi = true;
    }
    if (ok && multi) {
      int dmin = 1 << 30, dmax = -(1 << 30);
      for (int q = 0; q < KS; ++q)
        for (int c = 0; c < KS; ++c)
          if (present[q] && present[c]) {
            const int d = S.at(q, c) - 2 * a;
            dmin = std::min(dmin, d);
            dmax = std::max(dmax, d);
          }
      h->splitClamp = std::max(0, -dmin);
      h->splitMargin = h->splitClamp + std::max(0, dmax) + 1;
      h->splitGrow = 65 * std::max(0, dmax);
      h->split = 1;
      const size_t np = h->plan.size();
      h->splitBases.assign(2 * (np + 1), 0);
      for (size_t q = 0; q < np; ++q) {
        BgPair& P = h->plan[q];
        const BgSplitLayout L = bg_split_layout(P.n1, P.n2, P.nstrips, P.nc, R, h->segc);
        P.split_off = h->splitInts;
        h->splitInts += (L.total_ints + 63) / 64 * 64;
        const int ns1 = P.nstrips > 1 ? P.nstrips - 1 : 0;
        h->splitBases[q + 1] = h->splitBases[q] + ns1 * L.G;
        h->splitBases[np + 1 + q + 1] = h->splitBases[np + 1 + q] + ns1;
        for (int s2 = 0; s2 < P.nstrips; ++s2) h->splitMap.push_back(make_int2((int)q, s2));
      }
      h->splitItems = h->splitBases[np];
      {
        long capMax = 1;
        for (const BgPair& P : h->plan) capMax = std::max(capMax, (long)P.n1 + P.n2);
        const long cols = bg_expand_cols_per_block();
        h->splitXBlocks = (int)((capMax + cols - 1) / cols);
      }
      h->splitResolve = h->splitBases[2 * np + 1];
      // the concurrent pass takes items in the order the DP makes them ready: strip s reaches
      // chunk c at about (3 s + c) chunk times (a strip starts ~3 chunks after the one above)
      {
        const int oc = h->o(BG_OPT_SPLIT_CONCURRENT, -1);
        h->splitConc = oc < 0 ? 2 : oc == 1 ? 1 : 0;
      }
      std::vector<std::pair<int64_t, int32_t>> keyed;
      keyed.reserve(h->splitItems);
      for (size_t q = 0; q < np; ++q) {
        const BgPair& P = h->plan[q];
        const BgSplitLayout L = bg_split_layout(P.n1, P.n2, P.nstrips, P.nc, R, h->segc);
        for (int s2 = 1; s2 < P.nstrips; ++s2)
          for (int g = 0; g < L.G; ++g)
            keyed.emplace_back(3LL * s2 + (int64_t)g * h->segc,
                               h->splitBases[q] + (s2 - 1) * L.G + g);
      }
      std::stable_sort(keyed.begin(), keyed.end());
      for (const auto& kv : keyed) h->splitBases.push_back(kv.second);
    }
  }
  if (h->grouped) {
    // groups of P plan pairs of one reference class (plan order within a class: longest first),
    // the largest groups first; a group's pairs share one wave's checkpoints
    const int GP = h->grouped;
    std::vector<std::vector<int>> byRef;
    for (size_t q = 0; q < h->plan.size(); ++q) {
      const int rc = refOf[h->plan[q].caller];
      if (rc < 0) continue;
      if ((size_t)rc >= byRef.size()) byRef.resize(rc + 1);
      byRef[rc].push_back((int)q);
    }
    std::vector<std::array<int32_t, 8>> groups;
    for (const auto& v : byRef)
      for (size_t x = 0; x < v.size(); x += GP) {
        std::array<int32_t, 8> gq = {-1, -1, -1, -1, -1, -1, -1, -1};
        for (size_t y = 0; y < (size_t)GP && x + y < v.size(); ++y) gq[y] = v[x + y];
        groups.push_back(gq);
      }
    std::stable_sort(groups.begin(), groups.end(), [&](const std::array<int32_t, 8>& x, const std::array<int32_t, 8>& y) {
      return (uint64_t)h->plan[x[0]].n1 * h->plan[x[0]].n2 > (uint64_t)h->plan[y[0]].n1 * h->plan[y[0]].n2;
    });
    tro = 0;
    h->grpHost.clear();
    for (const auto& gq : groups) {
      const BgPair& P0 = h->plan[gq[0]];
      // P = 8: the low halves (y < 4) as a four-pair group at tro, the high ones right after
      const uint64_t area = (uint64_t)P0.nc * (R + 1) * BG_WAVE * 4;
      for (int y = 0; y < GP; ++y) {
        h->grpHost.push_back(gq[y]);
        if (gq[y] < 0) continue;
        BgPair& P = h->plan[gq[y]];
        P.trace_off = tro + (GP == 8 && y >= 4 ? area : 0);
        P.lane0 = GP == 8 ? 16 * (y & 3) : (64 / GP) * y;
        P.lanes = GP == 8 ? 16 : 64 / GP;
      }
      tro += round_up((GP == 8 ? 2 : 1) * area, 256);
    }
    h->ngroups = (int)groups.size();
  }
  h->traceBytes = tro;
  h->opsBytes = po;
  h->compactExec = -1;
  h->bndBytes = bo * 4 * ((h->affine || h->ack) ? 2 : 1);
  h->resBytes = o1 + o2;

  tm.mark(kPhPlan, "layout");
  // ---- device memory
  if (!h->seq1.ensure(o1 + 16) || !h->seq2.ensure(o2 + 16) || !h->codes1.ensure(o1 + 16) ||
      !h->codes2.ensure(o2 + 16) || !h->lut.ensure(256) ||
      !h->prof.ensure(std::max<size_t>(4096, (size_t)h->pstride * h->pstride * 4 + 64)) || !h->pairs.ensure(sizeof(BgPair) * (h->plan.size() + 1)) ||
      !h->wgmapBuf.ensure(sizeof(int2) * (h->wgmap.size() + 1)) ||
      (h->grouped && !h->grpBuf.ensure(4 * (h->grpHost.size() + 4))) ||
      !h->gprogBuf.ensure(4 * ((size_t)h->progWords + 1)) ||
      (h->split && (!h->splitMapBuf.ensure(sizeof(int2) * (h->splitMap.size() + 1)) ||
                    !h->splitBaseBuf.ensure(4 * (h->splitBases.size() + 1)))) ||
      (h->pglob && !h->profScratch.ensure((h->plan.size() + 1) * (size_t)h->W * h->kdim * 64 * 4 * 4)))
    return BG_E_NOMEM;
  h->gridWgs = (h->wide || h->span) ? (int)h->wgmap.size() : h->grouped ? (h->ngroups + W - 1) / W : (int)h->plan.size();
  for (int z = 0; z < h->depth; ++z) {
    Slot& S = h->slot[z];
    if (!S.trace.ensure(tro + 256) || !S.bndM.ensure(bo * 4 + 256) ||
        !S.bndX.ensure((h->affine || h->ack) ? bo * 4 + 256 : 256) || !S.aux.ensure(ao * 4 + 256) ||
        !S.out1.ensure(oo + 16) || !S.out2.ensure(oo + 16) || !S.ops.ensure(po + 16) ||
        !S.results.ensure(sizeof(BgResult) * (h->plan.size() + 1)) ||
        ((h->split || h->grouped) && !S.keys.ensure(16 * (h->plan.size() + 1))) ||
        (h->split && !S.xcnt.ensure(8 * ((size_t)h->plan.size() * h->splitXBlocks + 1))) ||
        (h->split && !S.split.ensure(h->splitInts * 4 + 256)) ||
        ((h->wide || h->span) && !S.gprog.ensure(4 * ((size_t)h->progWords + 8))))
      return BG_E_NOMEM;
    // WIDE checkpoint batches hand strip rows between workgroups as epoch-tagged granules: a
    // fresh arena is zeroed so that no stale tag (of another handle) can match an epoch
    if (h->wide && h->tag && h->ckpt) {
      const size_t gb = bo * 8 + 256;
      if (S.gran.cap < gb) {
        if (!S.gran.ensure(gb)) return BG_E_NOMEM;
        BG_HIP(hipMemset(S.gran.p, 0, S.gran.cap));
      }
    }
  }

  tm.mark(kPhAlloc, "alloc");
  // uploads go on the DP stream of a handle alone, on the group's upload stream otherwise (the DP
  // stream then holds other handles' DPs, which the upload must not queue behind)
  hipStream_t us = h->stream;
  if (h->shared()) {
    if (!h->upS) h->upS = group_stream(h, kSUp);
    if (!h->upS) return BG_E_HIP;
    us = h->upS;
  }
  // the split arena holds epoch-tagged words (done tags, checkpoint granules, the head's overflow
  // tag) beside plain column numbers; a batch with another layout would read the previous batch's
  // columns where its tags live, and a small column can equal an epoch — zeroed at every prepare
  if (h->split)
    for (int z = 0; z < h->depth; ++z)
      BG_HIP(hipMemsetAsync(h->slot[z].split.p, 0, h->splitInts * 4 + 256, us));
  // asynchronous fetch: the pinned download buffers sized now, while nothing is in flight
  h->planOut = oo;
  if (h->asyncFetch && (!h->ho1.ensure(oo + 1) || !h->ho2.ensure(oo + 1) ||
                        !h->hresPin.ensure(sizeof(BgResult) * (h->plan.size() + 1))))
    return BG_E_NOMEM;
  // ---- uploads: the raw residues staged above (one DMA each), the tables; the codes are
  // made on the device (bg_code_kernel)
  uint8_t lut[256];
  for (int x = 0; x < 256; ++x) {
    const uint16_t c = S.code[x];
    const int d = (c < KS && dense[c] >= 0) ? dense[c] : 0;
    lut[x] = (uint8_t)((h->dna && !h->ack) ? d * 8 : d);
  }
  // (a handle member: a shared handle's upload is still in flight when prepare returns)
  std::vector<int32_t>& prof = h->profHost;
  prof.assign(std::max<size_t>(1024, (size_t)h->pstride * h->pstride), 0);
  if (h->ack) {
    int16_t* t16 = reinterpret_cast<int16_t*>(prof.data());
    const int sub = mode == BG_LOCAL ? a : a + b;
    for (int q = 0; q < KS; ++q)
      for (int c = 0; c < KS; ++c)
        if (dense[q] >= 0 && dense[c] >= 0)
          t16[dense[q] * h->pstride + dense[c]] = (int16_t)(S.at(q, c) - sub);
  } else if (h->dna) {
    for (int q = 0; q < KS; ++q) {
      if (dense[q] < 0) continue;
      uint32_t packed = 0;
      for (int c = 0; c < KS; ++c) {
        if (dense[c] < 0) continue;
        const int v = S.at(q, c) - a;
        packed |= (uint32_t)(uint8_t)(int8_t)v << (8 * dense[c]);
      }
      prof[dense[q]] = (int32_t)packed;
      if (h->tag) {
        uint32_t px = 0, py = 0;
        for (int c = 0; c < KS; ++c) {
          if (dense[c] < 0) continue;
          const int v = 4 * (S.at(q, c) - 2 * a);   // frame M - a*(i+j)
          px |= (uint32_t)(uint8_t)(int8_t)(v - 2) << (8 * dense[c]);
          py |= (uint32_t)(uint8_t)(int8_t)(v - 3) << (8 * dense[c]);
        }
        prof[64 + dense[q]] = (int32_t)px;
        prof[128 + dense[q]] = (int32_t)py;
        uint32_t pz = 0;                       // score-only pass: S - 2a, untagged
        for (int c = 0; c < KS; ++c)
          if (dense[c] >= 0)
            pz |= (uint32_t)(uint8_t)(int8_t)(S.at(q, c) - 2 * a) << (8 * dense[c]);
        prof[192 + dense[q]] = (int32_t)pz;
      }
    }
  } else if (h->p32) {
    for (int q = 0; q < KS; ++q)
      for (int c = 0; c < KS; ++c)
        if (dense[q] >= 0 && dense[c] >= 0)
          prof[dense[q] * h->pstride + dense[c]] = (int32_t)((uint32_t)S.at(q, c) - (uint32_t)a);
  } else {
    int16_t* t16 = reinterpret_cast<int16_t*>(prof.data());
    for (int q = 0; q < KS; ++q)
      for (int c = 0; c < KS; ++c)
        if (dense[q] >= 0 && dense[c] >= 0) t16[dense[q] * h->pstride + dense[c]] = (int16_t)(S.at(q, c) - a);
  }
  st1[o1] = st2[o2] = 0;
  std::memcpy(st2 + o2 + 16, lut, 256);
  BG_HIP(hipMemcpyAsync(h->seq1.p, st1, o1 + 1, hipMemcpyHostToDevice, us));
  BG_HIP(hipMemcpyAsync(h->seq2.p, st2, o2 + 1, hipMemcpyHostToDevice, us));
  BG_HIP(hipMemcpyAsync(h->lut.p, st2 + o2 + 16, 256, hipMemcpyHostToDevice, us));
  {
    const uint8_t* r1 = h->seq1.as<uint8_t>();
    uint8_t* c1 = h->codes1.as<uint8_t>();
    size_t m1 = o1 + 1;
    const uint8_t* r2 = h->seq2.as<uint8_t>();
    uint8_t* c2 = h->codes2.as<uint8_t>();
    size_t m2 = o2 + 1;
    const uint8_t* lt = h->lut.as<uint8_t>();
    void* args[] = {&r1, &c1, &m1, &r2, &c2, &m2, &lt};
    const int blocks = (int)std::min<uint64_t>(4096, std::max<uint64_t>(1, (m1 + m2) / (16 * 256) + 2));
    BG_HIP(hipLaunchKernel(bg_code_kernel_ptr(), dim3(blocks), dim3(256), args, 0, us));
  }
  BG_HIP(hipMemcpyAsync(h->prof.p, prof.data(), prof.size() * 4, hipMemcpyHostToDevice, us));
  if (!h->plan.empty())
    if (h->wide || h->span)
    BG_HIP(hipMemcpyAsync(h->wgmapBuf.p, h->wgmap.data(), sizeof(int2) * h->wgmap.size(),
                          hipMemcpyHostToDevice, us));
  BG_HIP(hipMemcpyAsync(h->pairs.p, h->plan.data(), sizeof(BgPair) * h->plan.size(),
                          hipMemcpyHostToDevice, us));
  if (h->grouped)
    BG_HIP(hipMemcpyAsync(h->grpBuf.p, h->grpHost.data(), 4 * h->grpHost.size(), hipMemcpyHostToDevice, us));
  if (h->split) {
    BG_HIP(hipMemcpyAsync(h->splitMapBuf.p, h->splitMap.data(), sizeof(int2) * h->splitMap.size(),
                          hipMemcpyHostToDevice, us));
    BG_HIP(hipMemcpyAsync(h->splitBaseBuf.p, h->splitBases.data(), 4 * h->splitBases.size(),
                          hipMemcpyHostToDevice, us));
  }
  {
    std::vector<BgPairResultDev>& tmpl = h->tmplHost;
    tmpl.resize(npairs);
    for (size_t p = 0; p < npairs; ++p) {
      std::memset(&tmpl[p], 0, sizeof(tmpl[p]));
      tmpl[p].status = h->prestatus[p] < 0 ? 0 : h->prestatus[p];
      tmpl[p].offset = h->outoff[p];
    }
    if (!h->recs.ensure(sizeof(BgPairResultDev) * (npairs + 1))) return BG_E_NOMEM;
    if (npairs)
      BG_HIP(hipMemcpyAsync(h->recs.p, tmpl.data(), sizeof(BgPairResultDev) * npairs,
                            hipMemcpyHostToDevice, us));
  }
  tm.mark(kPhUpload, "queue");
  // a handle alone waits for its upload here; a shared handle does not (the code kernel on the
  // upload stream needs CUs, which the DP of the batch before holds): its executes' DPs wait for
  // the upload on the device, and its next prepare drains it (every source stays untouched until
  // then: the pinned staging and handle-owned vectors)
  if (h->shared()) {
    BG_HIP(hipEventRecord(h->upDone, us));
    h->upPending = true;
  } else {
    BG_HIP(hipStreamSynchronize(us));
  }
  tm.mark(kPhUpload, "upload");
  h->order_ = order;
  h->bufRows = bufR;
  h->bufCols = bufC;
  fin_geom(h, h->plan.size(), &h->finWaves, &h->finSlots);
  tm.mark(kPhPlan, "fin_geom");
  if (!h->finFlags) h->callDims.clear();
  h->prepared = true;
  return BG_OK;
}

extern "C" int bg_batch_prepare(bg_aligner* h, int mode, size_t npairs, const uint8_t* const* s1,
                                const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                                const bg_scoring* sc, int32_t a, int32_t b) {
  if (!h || !sc || sc->alphabet_size < 0 || sc->alphabet_size > 32) return BG_E_ARG;
  HScore S;
  S.K = 32;
  for (int x = 0; x < 256; ++x) S.code[x] = sc->code[x] < 32 ? sc->code[x] : 0xFFFF;
  S.tab.assign(sc->table, sc->table + 1024);
  return prepare_impl(h, mode, npairs, s1, n1, s2, n2, S, a, b);
}

extern "C" int bg_batch_prepare_table(bg_aligner* h, int mode, size_t npairs,
                                      const uint8_t* const* s1, const size_t* n1,
                                      const uint8_t* const* s2, const size_t* n2,
                                      const uint16_t* code, int32_t k, const int32_t* table,
                                      int32_t a, int32_t b) {
  if (!h || !code || !table || k < 1 || k > 256) return BG_E_ARG;
  HScore S;
  S.K = k;
  for (int x = 0; x < 256; ++x) S.code[x] = code[x] < k ? code[x] : 0xFFFF;
  S.tab.assign(table, table + (size_t)k * k);
  return prepare_impl(h, mode, npairs, s1, n1, s2, n2, S, a, b);
}

namespace {
// BG_DEBUG=dp: 8 words per wave, then 32 words of conveyor boundary times per wave
constexpr size_t kDpDbgBytes = 8 * 4096 * (8 + 32);
// BG_DEBUG=exec: the whole call, entry to return (stderr)
struct CallClock {
  const char* what;
  bool on;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  CallClock(const char* w, bool o) : what(w), on(o) {}
  ~CallClock() {
    if (on)
      std::fprintf(stderr, "%s total %.3f ms\n", what,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
};
}  // namespace

extern "C" int bg_batch_execute(bg_aligner* h) {
  const bool callTiming = dbg_flags().exec;
  CallClock clk("execute", callTiming);
  if (!h) return BG_E_ARG;
  if (!h->prepared) return BG_E_NO_BATCH;
  // BG_DEBUG=exec: host time of this call's steps on stderr (which HIP call blocks)
  const bool exTiming = dbg_flags().exec;
  auto exT = std::chrono::steady_clock::now();
  char exBuf[256];
  int exN = 0;
  auto exMark = [&](const char* what) {
    if (!exTiming) return;
    const auto now = std::chrono::steady_clock::now();
    exN += std::snprintf(exBuf + exN, sizeof(exBuf) - exN > 0 ? sizeof(exBuf) - exN : 0, " %s %.3f", what,
                         std::chrono::duration<double, std::milli>(now - exT).count());
    exT = now;
  };
  BG_HIP(hipSetDevice(h->device));
  exMark("setdev");
  const unsigned np = (unsigned)h->plan.size();
  const int z = h->execCount % h->depth;
  Slot& S = h->slot[z];
  // the DP's stream: WIDE batches alternate two (see bg_aligner::dps)
  // (C3, pipeline 3: 8.35 -> 4.82 ms per execute; BG_OPT_TWO_DP_STREAMS 0 keeps one).  Two WIDE DPs
  // need 2 x gridWgs <= CU count workgroups resident (their strips spin on each other), and
  // nothing else running waits for a DP, so they cannot hold each other's CUs.
  hipStream_t ds = h->stream;
  if (h->wide && h->depth >= 2 && (h->execCount & 1) && h->o(BG_OPT_TWO_DP_STREAMS, 1) != 0 &&
      2 * h->gridWgs <= h->cus && !dbg_flags().dp) {
    if (!h->dps) h->dps = group_stream(h, kSDps);
    if (h->dps) ds = h->dps;
  }
  // the exit pass beside the DP needs the CUs this DP leaves idle: in the automatic mode it runs
  // only when no other execute's DP is still in flight (a lone alignment's wall, not a pipeline's
  // throughput: a second DP wants those CUs) — on either DP stream, so every slot's last DP is
  // asked; and only when the DP leaves a CU free
  // (the concurrent pass reads WIDE's epoch-tagged granules: not SPAN)
  bool conc = h->split && h->splitConc == 1 && h->wide;
  if (h->split && h->splitConc == 2 && h->wide) {
    conc = h->shared() ? false : true;       // other handles' DPs are not visible here
    for (int x = 0; x < h->depth && conc; ++x) {
      if (!h->slot[x].inflight) continue;
      const hipError_t q = hipEventQuery(h->slot[x].dpDone);
      if (q == hipErrorNotReady) conc = false;
      else BG_HIP(q);
    }
  }
  if (h->cus - h->gridWgs <= 0) conc = false;
  // the previous user of this slot must have finished reading its trace, and a download or
  // export queued behind it reading its results
  if (S.inflight) BG_HIP(hipStreamWaitEvent(ds, S.finDone, 0));
  if (S.readPending) BG_HIP(hipStreamWaitEvent(ds, S.readDone, 0));
  S.readPending = false;
  // a shared handle's upload, not waited for by prepare
  if (h->upPending) BG_HIP(hipStreamWaitEvent(ds, h->upDone, 0));
  exMark("waits");
  hipEvent_t e[4] = {h->ev[0], h->ev[1], h->ev[2], h->ev[3]};
  if (h->profiling && h->ringUsed + 4 <= (int)h->ring.size()) {
    for (int x = 0; x < 4; ++x) e[x] = h->ring[h->ringUsed + x];
    h->ringUsed += 4;
  }
  BG_HIP(hipEventRecord(e[0], ds));
  if (np) {
    void* fn = h->grouped ? bg_dp_grp_kernel_ptr(h->R, h->grouped)
             : h->tag ? bg_dp_kernel_tag_ptr(h->R, h->wide ? 1 : h->span ? 2 : 0, h->ckpt) : dp_fn(h, h->R);
    if (!fn) return BG_E_ARG;
    BgDpArgs A;
    A.pairs = h->pairs.as<BgPair>();
    A.seq1 = h->seq1.as<uint8_t>();
    A.seq2 = h->seq2.as<uint8_t>();
    A.lut = h->lut.as<uint8_t>();
    A.codes1 = h->codes1.as<uint8_t>();
    A.codes2 = h->codes2.as<uint8_t>();
    A.prog_off = h->progOff;
    A.codes_off = h->codesOff;
    A.codes_in_lds = h->codesInLds;
    A.aux_lds_off = h->auxLdsOff;
    A.wgmap = h->wgmapBuf.as<int2>();
    A.gprog = (h->wide || h->span) ? S.gprog.as<uint32_t>() : h->gprogBuf.as<uint32_t>();
    A.dbg = nullptr;
    if (dbg_flags().dp && h->tag && h->dpDbg.ensure(kDpDbgBytes)) {
      A.dbg = h->dpDbg.as<unsigned long long>();
      BG_HIP(hipMemsetAsync(h->dpDbg.p, 0, kDpDbgBytes, ds));
    }
    if (h->wide || h->span) BG_HIP(hipMemsetAsync(S.gprog.p, 0, 4 * ((size_t)h->progWords + 8), ds));
    if (conc) {
      if (!S.resetDone) BG_HIP(hipEventCreateWithFlags(&S.resetDone, hipEventDisableTiming));
      BG_HIP(hipEventRecord(S.resetDone, ds));
    }
    A.prof_scratch = h->pglob ? h->profScratch.as<int32_t>() : nullptr;
    if (++h->epoch == 0) h->epoch = 1;
    A.epoch = h->epoch;
    A.gran = S.gran.as<unsigned long long>();
    A.split = conc ? S.split.as<int32_t>() : nullptr;
    A.segc = h->segc;
    A.resident = h->wide ? S.gprog.as<uint32_t>() + h->progWords : nullptr;
    A.trace = S.trace.as<uint32_t>();
    A.bndM = S.bndM.as<int32_t>();
    A.bndX = S.bndX.as<int32_t>();
    A.aux = S.aux.as<int32_t>();
    A.profile = h->prof.as<int32_t>();
    A.kdim = h->kdim;
    A.pstride = h->pstride;
    A.open = h->a;
    A.ext = h->b;
    A.mode = h->mode;
    A.npairs = (int32_t)np;
    A.grp = h->grouped ? h->grpBuf.as<int32_t>() : nullptr;
    A.ngroups = h->grouped ? h->ngroups : 0;
    // semiglobal / overlap: the grouped DP folds each pair's last-row end-cell key
    A.keys = grp_fold(h) ? S.keys.as<unsigned long long>() : nullptr;
    void* args[] = {&A};
    if (h->lds > 65536)
      BG_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds));
    exMark("dp-attr");
    BG_HIP(hipLaunchKernel(fn, dim3(h->gridWgs), dim3(64 * h->W), args, h->lds, ds));
  }
  exMark("dp");
  BG_HIP(hipEventRecord(e[1], ds));
  BG_HIP(hipEventRecord(S.dpDone, ds));
  S.dpPending = true;              // until the finish is queued behind it (finDone covers it)
  exMark("dp-events");
  // The traceback stream.  A WIDE batch (a few long pairs: C3) is traceback-bound and its walks
  // occupy a handful of CUs, so consecutive executes' tracebacks alternate between two streams
  // and run side by side (each still waits for its own DP; the slot it reads is not reused before
  // its finDone); the step then follows the DP.  Many-pair batches keep one stream: their finish
  // workgroups fill the CUs beside the next DP as it is.
  // At pipeline depth 4 a WIDE batch's tracebacks rotate over three streams: a C3 walk (one
  // latency-bound workgroup, ~13 ms) then hides behind three DPs instead of two.
  // SPAN batches (fewer pairs than CUs) alternate two: one walk of a 10 k x 10 k pair (~1.6 ms)
  // is longer than their DP (1.1 ms at 64 pairs), and the walks of two executes fit side by side.
  int nfs = 1;
  if ((h->wide || h->span) && !dbg_flags().finish)
    nfs = h->wide ? std::min(3, std::max(2, h->depth - 1)) : 2;
  // the third stream is created on first use: HIP maps a process's streams onto 4 hardware
  // queues round-robin, and an extra stream per handle moves other handles' copies behind
  // kernels in a shared queue (host_to_host runs four handles)
  if (nfs >= 2 && !h->stream3) h->stream3 = group_stream(h, kSFin2);
  if (nfs >= 2 && !h->stream3) nfs = 1;
  if (nfs == 3 && !h->stream4) h->stream4 = group_stream(h, kSFin3);
  if (nfs == 3 && !h->stream4) nfs = 2;
  const hipStream_t fss[3] = {h->stream2, h->stream3, h->stream4};
  hipStream_t fs = fss[h->execCount % nfs];
  // split traceback: its arguments, and the exit pass beside the DP (it waits for the DP's
  // progress words to be zeroed, then takes items as the DP makes them ready)
  BgSplitArgs X;
  std::memset(&X, 0, sizeof(X));
  if (np && h->split) {
    X.pairs = h->pairs.as<BgPair>();
    X.codes1 = h->codes1.as<uint8_t>();
    X.codes2 = h->codes2.as<uint8_t>();
    X.ckpt = S.trace.as<int32_t>();
    X.bndM = S.bndM.as<int32_t>();
    X.profile = h->prof.as<int32_t>();
    X.split = S.split.as<int32_t>();
    X.itemBase = h->splitBaseBuf.as<int32_t>();
    X.stripBase = h->splitBaseBuf.as<int32_t>() + (np + 1);
    X.order = h->splitBaseBuf.as<int32_t>() + 2 * (np + 1);
    X.npairs = (int32_t)np;
    X.nitems = h->splitItems;
    X.open = h->a;
    X.ext = h->b;
    X.mode = h->mode;
    X.R = h->R;
    X.segc = h->segc;
    X.margin = h->splitMargin;
    X.clampv = h->splitClamp;
    X.grow = h->splitGrow;
    X.epoch = h->epoch;
    X.gran = S.gran.as<unsigned long long>();
    X.resident = S.gprog.as<uint32_t>() + h->progWords;
    X.counter = S.gprog.as<uint32_t>() + h->progWords + 1;
    X.dpWgs = h->gridWgs;
    X.endKeys = S.keys.as<unsigned long long>();
    X.aux = S.aux.as<int32_t>();
    X.xcount = S.xcnt.as<int2>();
    X.xblocks = h->splitXBlocks;
    X.diag = S.gprog.as<uint32_t>() + h->progWords + 2;
    {
      const long ms = h->o(BG_OPT_SPLIT_WAIT_MS, 500);
      X.waitTicks = (int32_t)std::min<long>(std::max<long>(ms, 1) * 100000L, 0x7FFFFFFFL);
    }
    if (conc && h->splitItems > 0) {
      X.conc = 1;
      void* cargs[] = {&X};
      void* cfn = bg_split_kernel_ptr(h->R, 3);
      // more than half a CU's LDS: never beside a WIDE DP workgroup (which claims over half too)
      const size_t clds = std::max<size_t>((size_t)bg_exit_conc_lds_bytes(h->R), 80 * 1024 + 64);
      BG_HIP(hipFuncSetAttribute(cfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)clds));
      BG_HIP(hipStreamWaitEvent(fs, S.resetDone, 0));
      // one workgroup per CU the DP leaves free: even dispatched first, they leave the DP its CUs
      // (conc is off when the DP holds every CU)
      const int cg = h->cus - h->gridWgs;
      BG_HIP(hipLaunchKernel(cfn, dim3(cg), dim3(h->R >= 8 ? 512 : 1024), cargs, clds, fs));
      X.conc = 0;
    }
  }
  BG_HIP(hipStreamWaitEvent(fs, S.dpDone, 0));
  BG_HIP(hipEventRecord(e[2], fs));
  if (np) {
    BgFinishArgs F;
    F.keys = grp_fold(h) ? S.keys.as<unsigned long long>() : nullptr;
    F.pairs = h->pairs.as<BgPair>();
    F.seq1 = h->seq1.as<uint8_t>();
    F.seq2 = h->seq2.as<uint8_t>();
    F.trace = S.trace.as<uint32_t>();
    F.bndM = S.bndM.as<int32_t>();
    F.aux = S.aux.as<int32_t>();
    F.out1 = S.out1.as<uint8_t>();
    F.out2 = S.out2.as<uint8_t>();
    F.results = S.results.as<BgResult>();
    F.open = h->a;
    F.ext = h->b;
    F.mode = h->mode;
    F.R = h->R;
    F.affine = h->affine;
    F.tag = h->ckpt ? 2 : h->tag;
    F.npairs = (int32_t)np;
    F.codes1 = h->codes1.as<uint8_t>();
    F.codes2 = h->codes2.as<uint8_t>();
    F.profile = h->prof.as<int32_t>();
    F.dbg = nullptr;
    F.bndX = S.bndX.as<int32_t>();
    F.kdim = h->kdim;
    F.pstride = h->pstride;
    F.ops = S.ops.as<uint8_t>();
    F.area_ints = 0;
    F.flags = h->finFlags;
    F.grouped = h->grouped;
    F.phase = BG_PH_FULL;
    F.segc = h->segc;
    F.specDepth = 2;
    F.specAbove = 128;
    if (!S.wdiag.ensure(4 * BG_WD_WORDS)) return BG_E_NOMEM;
    BG_HIP(hipMemsetAsync(S.wdiag.p, 0, 4 * BG_WD_WORDS, fs));
    F.wdiag = S.wdiag.as<uint32_t>();
    F.waitTicks = (int32_t)std::min<long>(std::max<long>(h->o(BG_OPT_WAIT_MS, 2000), 1) * 100000L, 0x7FFFFFFFL);
    F.split = S.split.as<int32_t>();
    F.splitMap = h->splitMapBuf.as<int2>();
    if (h->o(BG_OPT_FIN_SYNC, 0) == 1) F.flags |= BG_FIN_SYNC;
    if (h->o(BG_OPT_FIN_SELFSERVE, 0) == 1) F.flags |= BG_FIN_SELFSERVE;
    // the walker's priority 3 costs a many-pair linear batch's DP (the metric: 10 390 -> 10 530
    // GCUPS without it, tools/r04/prio_ab.sh); a WIDE batch's walks are its latency, and the
    // affine walks (recomputing with barriers) gain from it: MA 4 587 -> 4 714 GCUPS, C5 +0.9 %,
    // C2 even (tools/r05/prio_ab.sh).
    if (!h->wide && !h->span && !h->ack) F.flags |= BG_FIN_NOPRIO;
    if (dbg_flags().finish && h->dbgBuf.ensure(128 * (np + 1))) {
      F.dbg = h->dbgBuf.as<unsigned long long>();
      BG_HIP(hipMemsetAsync(h->dbgBuf.p, 0, 128 * np, fs));
    }
    void* args[] = {&F};
    int fnw = 4, fns = 0;
    fin_geom(h, np, &fnw, &fns);
    F.nslots = fns;
    if (h->finFlags & BG_FIN_SCORE_ONLY) {
      BG_HIP(hipLaunchKernel(bg_global_score_kernel_ptr(), dim3((np + 255) / 256), dim3(256), args, 0,
                             fs));
    } else if (h->ack) {
      int win = 0, area = 0;
      const size_t lds = bg_finish_ack_lds_bytes(h->R, h->kdim, h->local, fns, fnw, &win, &area);
      F.win_bytes = win;
      F.area_ints = area;
      F.tag = h->local ? 2 : 3;          // 3: the opened frame's boundary rows (bg_aff_common.h)
      F.affine = 1;
      void* ffn = bg_finish_ack_kernel_ptr(h->R, h->mode);
      if (lds > 65536) BG_HIP(hipFuncSetAttribute(ffn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      BG_HIP(hipLaunchKernel(ffn, dim3(np), dim3(64 * fnw), args, lds, fs));
    } else if (h->ckpt) {
      int win = 0;
      const int fgp = h->grouped;
      const size_t lds = h->grouped ? bg_finish_grp_lds_bytes(fgp, h->R, fns, fnw, &win)
                                    : bg_finish_ck_lds_bytes(h->R, fns, fnw, &win);
      F.win_bytes = win;
      void* ffn = h->grouped ? bg_finish_grp_kernel_ptr(fgp, h->R, h->mode) : bg_finish_ck_kernel_ptr(h->R, h->mode);
      if (lds > 65536) BG_HIP(hipFuncSetAttribute(ffn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      if (!h->split) {
        BG_HIP(hipLaunchKernel(ffn, dim3(np), dim3(64 * fnw), args, lds, fs));
      } else {
        // split traceback: end cell -> exit pass (the items the pass beside the DP
        // did not do) -> per-strip resolve -> chain -> the strips' walks in parallel -> stitch
        void* xargs[] = {&X};
        // the end-cell keys folded by many workgroups per pair, then HEAD reads them
        BG_HIP(hipMemsetAsync(S.keys.p, 0, 16 * (size_t)np, fs));
        BG_HIP(hipLaunchKernel(bg_endkey_kernel_ptr(), dim3(np * (unsigned)bg_endkey_blocks()), dim3(256), xargs, 0, fs));
        F.keys = S.keys.as<unsigned long long>();
        F.phase = BG_PH_HEAD;
        BG_HIP(hipLaunchKernel(ffn, dim3(np), dim3(64 * fnw), args, lds, fs));
        if (h->splitItems > 0)
          BG_HIP(hipLaunchKernel(bg_split_kernel_ptr(h->R, 0), dim3((h->splitItems + 3) / 4), dim3(256), xargs,
                                 bg_exit_lds_bytes(h->R), fs));
        if (h->splitResolve > 0)
          BG_HIP(hipLaunchKernel(bg_split_kernel_ptr(h->R, 1), dim3(h->splitResolve), dim3(64), xargs, 0, fs));
        BG_HIP(hipLaunchKernel(bg_split_kernel_ptr(h->R, 2), dim3(np), dim3(64), xargs, 0, fs));
        F.phase = BG_PH_WALK;
        BG_HIP(hipLaunchKernel(ffn, dim3((unsigned)h->splitMap.size()), dim3(64 * fnw), args, lds, fs));
        F.phase = BG_PH_TAIL;
        // the core's packing and expansion by many workgroups per pair (bg_split.hip)
        const bool defer = true;
        F.flags |= BG_FIN_DEFER_EXPAND;
        BG_HIP(hipLaunchKernel(ffn, dim3(np), dim3(64 * fnw), args, lds, fs));
        if (defer) {
          F.flags &= ~BG_FIN_DEFER_EXPAND;
          void* eargs[] = {&F, &X};
          const unsigned nb = (unsigned)X.xblocks;
          BG_HIP(hipLaunchKernel(bg_expand_kernel_ptr(0), dim3(np * nb), dim3(256), eargs, 0, fs));
          BG_HIP(hipLaunchKernel(bg_expand_kernel_ptr(1), dim3(np * nb), dim3(256), eargs, 0, fs));
        }
      }
    } else {
      F.win_bytes = bg_finish_window_bytes(h->R, h->affine, np, h->cus);
      BG_HIP(hipLaunchKernel(bg_finish_kernel_ptr(h->R, h->affine, h->mode), dim3(np), dim3(256), args,
                             bg_finish_lds_bytes(F.win_bytes), fs));
    }
  }
  exMark("finish");
  BG_HIP(hipEventRecord(e[3], fs));
  BG_HIP(hipEventRecord(S.finDone, fs));
  h->lastFs = fs;
  S.inflight = true;
  S.dpPending = false;
  exMark("fin-events");
  // asynchronous fetch: the results' download queued behind the traceback, on a stream (and
  // hardware queue) of its own, so it neither waits behind the next DPs nor delays the next
  // tracebacks; bg_batch_fetch then finds the strings on the host
  if (h->asyncFetch && np) {
    if (!h->dlS) h->dlS = group_stream(h, kSDl);
    if (!h->dlS) return BG_E_HIP;
    if (!h->ho1.ensure(h->planOut + 1) || !h->ho2.ensure(h->planOut + 1) ||
        !h->hresPin.ensure(sizeof(BgResult) * (np + 1)))
      return BG_E_NOMEM;
    exMark("dl-ensure");
    BG_HIP(hipStreamWaitEvent(h->dlS, S.finDone, 0));
    exMark("dl-wait");
    // the download as a kernel writing the host-mapped buffers (bg_io.hip): the copy-engine form
    // (BG_DL_COPY=1) can block this call for several ms in PyTorch's HIP runtime
    const bool dlCopy = false;
    void* dres = h->hresPin.device_ptr();
    void* d1 = h->ho1.device_ptr();
    void* d2 = h->ho2.device_ptr();
    if (!dlCopy && dres && d1 && d2) {
      BgDownloadArgs D;
      std::memset(&D, 0, sizeof(D));
      D.seg[0] = {S.results.as<uint8_t>(), static_cast<uint8_t*>(dres), sizeof(BgResult) * np};
      D.seg[1] = {S.out1.as<uint8_t>(), static_cast<uint8_t*>(d1), (uint64_t)h->planOut};
      D.seg[2] = {S.out2.as<uint8_t>(), static_cast<uint8_t*>(d2), (uint64_t)h->planOut};
      D.nseg = 3;
      const uint64_t vec = (2 * (uint64_t)h->planOut + sizeof(BgResult) * np) / 16;
      const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(kDownloadBlocks, (vec + 255) / 256));
      void* dargs[] = {&D};
      BG_HIP(hipLaunchKernel(bg_download_kernel_ptr(), dim3(blocks), dim3(256), dargs, 0, h->dlS));
    } else {
      BG_HIP(hipMemcpyAsync(h->hresPin.p, S.results.p, sizeof(BgResult) * np, hipMemcpyDeviceToHost, h->dlS));
      if (h->planOut) {
        BG_HIP(hipMemcpyAsync(h->ho1.p, S.out1.p, h->planOut, hipMemcpyDeviceToHost, h->dlS));
        BG_HIP(hipMemcpyAsync(h->ho2.p, S.out2.p, h->planOut, hipMemcpyDeviceToHost, h->dlS));
      }
    }
    BG_HIP(hipEventRecord(h->dlDone, h->dlS));
    BG_HIP(hipEventRecord(S.readDone, h->dlS));
    S.readPending = true;
    h->dlExec = h->execCount;
    exMark("download");
  }
  if (exTiming && exN) std::fprintf(stderr, "execute ms:%s\n", exBuf);
  if (e[0] != h->ev[0]) {  // keep the last execute's events for bg_get_stats
    h->last[0] = e[0]; h->last[1] = e[1]; h->last[2] = e[2]; h->last[3] = e[3];
  } else {
    for (int x = 0; x < 4; ++x) h->last[x] = h->ev[x];
  }
  h->lastSlot = z;
  ++h->execCount;
  h->executed = true;
  return BG_OK;
}

extern "C" int bg_synchronize(bg_aligner* h) {
  if (!h) return BG_E_ARG;
  BG_HIP(drain(h));
  if (h->executed) {
    (void)hipEventElapsedTime(&h->dp_ms, h->last[0], h->last[1]);
    (void)hipEventElapsedTime(&h->fin_ms, h->last[2], h->last[3]);
  }
  return BG_OK;
}

extern "C" int bg_batch_fetch(bg_aligner* h, bg_pair_result* res, uint8_t* out1, uint8_t* out2,
                              size_t out_cap) {
  if (!h || (h->npairs && !res)) return BG_E_ARG;
  if (!h->prepared || !h->executed) return BG_E_NO_BATCH;
  if (h->outBytes && (!out1 || !out2 || out_cap < h->outBytes)) return BG_E_ARG;
  PhaseTimer tm(h->hostMs);
  ++h->nFetch;
  int rc = bg_synchronize(h);
  if (rc) return rc;
  tm.mark(kPhFetchWait, "fetch-wait");
  const size_t np = h->plan.size();
  if (dbg_flags().dp && h->dpDbg.p && np) {
    // first pair's waves: strip start / chunk-0 end / strip end relative to the earliest start
    // (s_memrealtime, 100 MHz, one clock for every XCD), and the shader cycles each wave spent
    // polling for the strip above out of its whole strip (s_memtime)
    std::vector<unsigned long long> d(kDpDbgBytes / 8);
    BG_HIP(hipMemcpy(d.data(), h->dpDbg.p, kDpDbgBytes, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, tend = 0;
    int nrec = 0;
    for (int g = 0; g < 4096; ++g)
      if (d[8 * g + 1]) { t0 = std::min(t0, d[8 * g + 1]); tend = std::max(tend, d[8 * g + 3]); ++nrec; }
    std::fprintf(stderr, "dp timing: span %.1f us\n", (tend - t0) * 0.01);
    for (int g = 0; g < 4096; ++g) {
      if (!d[8 * g + 1]) continue;
      // every wave of a small group, else waves 64k .. 64k+7 + the last
      if (nrec > 64 && g % 64 >= 8 && g + 1 < 4096 && d[8 * (g + 1) + 1]) continue;
      std::fprintf(stderr, "  wave %4d strip %4llu start %8.1f c0done %8.1f end %8.1f us  waited %10.0f of %10.0f cycles  data %10.0f flow %10.0f\n", g,
                   d[8 * g], (d[8 * g + 1] - t0) * 0.01, (d[8 * g + 2] - t0) * 0.01,
                   (d[8 * g + 3] - t0) * 0.01, (double)d[8 * g + 4], (double)d[8 * g + 5],
                   (double)d[8 * g + 6], (double)d[8 * g + 7]);
    }
    // conveyor strips: the first twelve half boundaries and two steady ones (g = 1000, 1003),
    // arrival / departure in us from t0, and the departure behind the producer's at g + 3
    const unsigned long long* bt = d.data() + 8 * 4096;
    for (int g = 0; g < 4096; ++g) {
      const unsigned long long* q = bt + 32 * g;
      if (!q[1]) continue;
      if (!(g < 10 || (g >= 64 && g < 68) || (g >= 128 && g < 132) || (g >= 256 && g < 260))) continue;
      std::fprintf(stderr, "  bnd wave %4d:", g);
      for (int x = 0; x < 14; ++x) {
        if (!q[2 * x + 1]) { std::fprintf(stderr, "     -     "); continue; }
        std::fprintf(stderr, " %6.2f/%6.2f", (q[2 * x] - t0) * 0.01, (q[2 * x + 1] - t0) * 0.01);
      }
      std::fprintf(stderr, "\n");
      if (g > 0 && bt[32 * (g - 1) + 1]) {
        const unsigned long long* p = bt + 32 * (g - 1);
        std::fprintf(stderr, "  lag  wave %4d:", g);
        for (int x = 0; x + 3 < 12; ++x)
          std::fprintf(stderr, " %6.2f", q[2 * x + 1] && p[2 * (x + 3) + 1] ? ((double)q[2 * x + 1] - (double)p[2 * (x + 3) + 1]) * 0.01 : 0.0);
        std::fprintf(stderr, "  steady %6.2f\n", q[25] && p[27] ? ((double)q[25] - (double)p[27]) * 0.01 : 0.0);
      }
    }
  }
  if (dbg_flags().finish && h->dbgBuf.p && np) {
    std::vector<unsigned long long> d(16 * np);
    BG_HIP(hipMemcpy(d.data(), h->dbgBuf.p, 128 * np, hipMemcpyDeviceToHost));
    double s[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (size_t p = 0; p < np; ++p)
      for (int x = 0; x < 11; ++x) s[x] += (double)d[16 * p + x];
    std::fprintf(stderr, "finish timing: before walk: map cleared at %.0f, end cell at %.0f\n", s[9] / np, s[10] / np);
    double w0 = 0, w1 = 0, l01 = 0;
    for (size_t p = 0; p < np; ++p) {
      const auto* q = &d[16 * p];
      w0 += (double)(q[12] - q[11]);
      if (q[13]) { w1 += (double)(q[14] - q[13]); l01 += (double)q[13] - (double)q[11]; }
    }
    std::fprintf(stderr, "finish timing (us): wave 0 entry -> end-cell barrier %.2f, wave 1 %.2f, wave 1 entry after wave 0 by %.2f\n",
                 w0 / np * 0.01, w1 / np * 0.01, l01 / np * 0.01);
    std::fprintf(stderr, "finish timing (per pair avg, cycles): kernel %.0f = before walk %.0f + walk %.0f + after %.0f;"
                 "  walk: jump %.0f (n %.1f)  miss %.0f (n %.1f)  ops %.0f  chunks recomputed %.1f\n",
                 s[8] / np, s[7] / np, s[0] / np, (s[8] - s[7] - s[0]) / np,
                 s[1] / np, s[2] / np, s[3] / np, s[4] / np, s[5] / np, s[6] / np);
  }
  h->hres.resize(np);
  uint64_t ob = 0;
  for (const BgPair& P : h->plan) ob += (uint64_t)P.n1 + P.n2;
  if (h->asyncFetch && np && h->dlExec == h->execCount - 1) {
    // downloaded behind the traceback (bg_set_async_fetch); the wait above covered it
    std::memcpy(h->hres.data(), h->hresPin.p, sizeof(BgResult) * np);
  } else {
    if (!h->ho1.ensure(ob + 1) || !h->ho2.ensure(ob + 1)) return BG_E_NOMEM;
    if (np) {
      const Slot& S = h->slot[h->lastSlot];
      // a handle sharing its streams downloads on the group's download stream (the DP stream
      // holds other handles' DPs)
      hipStream_t cs = h->stream;
      if (h->shared()) {
        if (!h->dlS) h->dlS = group_stream(h, kSDl);
        if (!h->dlS) return BG_E_HIP;
        cs = h->dlS;
      }
      BG_HIP(hipMemcpyAsync(h->hres.data(), S.results.p, sizeof(BgResult) * np, hipMemcpyDeviceToHost, cs));
      BG_HIP(hipMemcpyAsync(h->ho1.p, S.out1.p, ob, hipMemcpyDeviceToHost, cs));
      BG_HIP(hipMemcpyAsync(h->ho2.p, S.out2.p, ob, hipMemcpyDeviceToHost, cs));
      BG_HIP(hipStreamSynchronize(cs));
    }
  }
  tm.mark(kPhFetchCopy, "fetch-d2h");
  for (size_t p = 0; p < h->npairs; ++p) {
    std::memset(&res[p], 0, sizeof(res[p]));
    res[p].status = h->prestatus[p] < 0 ? 0 : h->prestatus[p];
    res[p].offset = h->outoff[p];
  }
  for (size_t q = 0; q < np; ++q) {
    const BgPair& P = h->plan[q];
    const BgResult& r = h->hres[q];
    if (r.out_len > (uint32_t)(P.n1 + P.n2) || r.out_start + r.out_len > (uint32_t)(P.n1 + P.n2)) return BG_E_HIP;
  }
  std::vector<bgh::UnpackJob> jobs(np);
  for (size_t q = 0; q < np; ++q) {
    const BgPair& P = h->plan[q];
    const BgResult& r = h->hres[q];
    const size_t p = h->order_[q];
    bg_pair_result& o = res[p];
    o.status = r.status;
    o.score = r.score;
    o.len = r.out_len;
    o.end_i = (uint32_t)r.end_i;
    o.end_j = (uint32_t)r.end_j;
    o.start1 = r.start1;
    o.start2 = r.start2;
    if (o.status == BG_OK && bg_ref_divergent(h->mode, (long)h->n1v[p], (long)h->n2v[p], r.score,
                                              h->bufAt[p].first, h->bufAt[p].second))
      o.status = BG_REF_DIVERGENT;
    jobs[q] = bgh::UnpackJob{P.out_off + r.out_start, h->outoff[p], r.out_len};
  }
  bgh::unpack_strings(jobs, h->ho1.as<uint8_t>(), h->ho2.as<uint8_t>(), out1, out2);
  tm.mark(kPhFetchUnpack, "fetch-unpack");
  return BG_OK;
}

extern "C" int bg_host_timing(bg_aligner* h, double* ms, size_t n, uint64_t* calls, int reset) {
  if (!h || (n && !ms)) return BG_E_ARG;
  for (size_t i = 0; i < n && i < (size_t)kPhN; ++i) ms[i] = h->hostMs[i];
  if (calls) { calls[0] = h->nPrepare; calls[1] = h->nFetch; calls[2] = (uint64_t)host_threads(~0ull); }
  if (reset) {
    for (double& x : h->hostMs) x = 0.0;
    h->nPrepare = h->nFetch = 0;
  }
  return kPhN;
}

extern "C" int bg_align_batch(bg_aligner* h, int mode, size_t npairs, const uint8_t* const* s1,
                              const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                              const bg_scoring* sc, int32_t a, int32_t b, bg_pair_result* res,
                              uint8_t* out1, uint8_t* out2, size_t out_cap) {
  int rc = bg_batch_prepare(h, mode, npairs, s1, n1, s2, n2, sc, a, b);
  if (rc) return rc;
  rc = bg_batch_execute(h);
  if (rc) return rc;
  return bg_batch_fetch(h, res, out1, out2, out_cap);
}

extern "C" int bg_align(bg_aligner* h, int mode, const uint8_t* s1, size_t n1, const uint8_t* s2,
                        size_t n2, const bg_scoring* sc, int32_t a, int32_t b, int32_t* score,
                        uint8_t* out1, uint8_t* out2, size_t cap, size_t* out_len) {
  if (!h || !score || !out_len || cap < n1 + n2 || ((n1 + n2) && (!out1 || !out2))) return BG_E_ARG;
  bg_pair_result r;
  const uint8_t* p1 = s1;
  const uint8_t* p2 = s2;
  int rc = bg_align_batch(h, mode, 1, &p1, &n1, &p2, &n2, sc, a, b, &r, out1, out2, cap);
  if (rc) return rc;
  *score = r.score;
  *out_len = r.len;
  return r.status;
}

extern "C" int bg_get_stats(bg_aligner* h, bg_stats* o) {
  if (!h || !o) return BG_E_ARG;
  std::memset(o, 0, sizeof(*o));
  o->cells = h->cells;
  o->trace_bytes = h->traceBytes;
  o->boundary_bytes = h->bndBytes;
  o->residue_bytes = h->resBytes;
  o->device_bytes = h->device_bytes();
  o->R = h->R;
  o->waves = h->W;
  o->affine = h->affine;
  o->wide = h->wide ? 1 : h->span ? 2 : 0;
  o->workgroups = h->gridWgs;
  o->tagged = h->tag;
  o->checkpoint = h->ckpt || h->ack;
  o->dna = h->dna;
  o->local = h->local;
  o->npairs = (int32_t)h->npairs;
  o->dp_ms = h->dp_ms;
  o->finish_ms = h->fin_ms;
  o->fin_waves = h->finWaves;
  o->fin_slots = h->finSlots;
  o->split = h->split;
  o->grouped = h->grouped ? h->ngroups : 0;
  o->group_pairs = h->grouped;
  return BG_OK;
}

extern "C" int bg_get_stats_sized(bg_aligner* h, bg_stats* o, size_t size) {
  if (!h || !o) return BG_E_ARG;
  bg_stats full;
  const int rc = bg_get_stats(h, &full);
  if (rc) return rc;
  std::memcpy(o, &full, std::min(size, sizeof(full)));
  return BG_OK;
}

extern "C" int bg_wait_diag(bg_aligner* h, uint32_t* out, size_t n) {
  if (!h || (!out && n)) return BG_E_ARG;
  for (size_t x = 0; x < n; ++x) out[x] = 0;
  if (!h->executed) return BG_OK;
  const int rc = bg_synchronize(h);
  if (rc) return rc;
  const Slot& S = h->slot[h->lastSlot];
  if (!S.wdiag.p) return BG_OK;
  uint32_t w[BG_WD_WORDS];
  BG_HIP(hipMemcpy(w, S.wdiag.p, sizeof(w), hipMemcpyDeviceToHost));
  for (size_t x = 0; x < n && x < (size_t)BG_WD_WORDS; ++x) out[x] = w[x];
  return BG_OK;
}

extern "C" int bg_split_stats(bg_aligner* h, uint64_t* pairs_split, uint64_t* strips_taken,
                              uint64_t* tail_moves, uint64_t* pairs_overflow, uint64_t* items_beside_dp) {
  if (!h || !pairs_split || !strips_taken || !tail_moves || !pairs_overflow || !items_beside_dp) return BG_E_ARG;
  *pairs_split = *strips_taken = *tail_moves = *pairs_overflow = *items_beside_dp = 0;
  if (!h->split || !h->executed) return BG_OK;
  const int rc = bg_synchronize(h);
  if (rc) return rc;
  const Slot& S = h->slot[h->lastSlot];
  for (const BgPair& P : h->plan) {
    int32_t head[16];
    BG_HIP(hipMemcpy(head, S.split.as<int32_t>() + P.split_off, sizeof(head), hipMemcpyDeviceToHost));
    if (head[6] || (uint32_t)head[11] == h->epoch) ++*pairs_overflow;
    const BgSplitLayout L = bg_split_layout(P.n1, P.n2, P.nstrips, P.nc, h->R, h->segc);
    if (P.nstrips > 1) {
      std::vector<uint32_t> dn((size_t)(P.nstrips - 1) * L.G);
      BG_HIP(hipMemcpy(dn.data(), S.split.as<int32_t>() + P.split_off + L.done, dn.size() * 4, hipMemcpyDeviceToHost));
      for (uint32_t v : dn) *items_beside_dp += v == h->epoch;
    }
    if (head[7] >= 0) ++*pairs_split;
    if (head[7] >= 0 && head[8] > 0) *strips_taken += (uint64_t)head[8];
    if (head[7] >= 0 && head[10] > 0) *tail_moves += (uint64_t)head[10];
  }
  return BG_OK;
}

extern "C" int bg_split_conc_diag(bg_aligner* h, uint32_t* out6) {
  if (!h || !out6) return BG_E_ARG;
  for (int x = 0; x < 6; ++x) out6[x] = 0;
  if (!h->split || !h->executed || !h->wide) return BG_OK;
  const int rc = bg_synchronize(h);
  if (rc) return rc;
  const Slot& S = h->slot[h->lastSlot];
  BG_HIP(hipMemcpy(out6, S.gprog.as<uint32_t>() + h->progWords + 2, 6 * 4, hipMemcpyDeviceToHost));
  return BG_OK;
}

extern "C" int bg_aligner_set_buffer_size(bg_aligner* h, size_t rows, size_t cols) {
  if (!h || rows > 0x7FFFFFFF || cols > 0x7FFFFFFF) return BG_E_ARG;
  h->bufRows = (long)rows;
  h->bufCols = (long)cols;
  return BG_OK;
}

extern "C" int bg_aligner_set_call_dims(bg_aligner* h, size_t npairs, const uint64_t* rows,
                                        const uint64_t* cols) {
  if (!h) return BG_E_ARG;
  h->callDims.clear();
  if (!npairs || !rows || !cols) return BG_OK;
  for (size_t p = 0; p < npairs; ++p)
    if (rows[p] > 0x7FFFFFFF || cols[p] > 0x7FFFFFFF) return BG_E_ARG;
  h->callDims.resize(npairs);
  for (size_t p = 0; p < npairs; ++p) h->callDims[p] = std::make_pair((long)rows[p], (long)cols[p]);
  return BG_OK;
}

extern "C" int bg_aligner_buffer_size(bg_aligner* h, size_t* rows, size_t* cols) {
  if (!h || !rows || !cols) return BG_E_ARG;
  *rows = (size_t)h->bufRows;
  *cols = (size_t)h->bufCols;
  return BG_OK;
}

extern "C" int bg_profile_begin(bg_aligner* h) {
  if (!h) return BG_E_ARG;
  BG_HIP(hipSetDevice(h->device));
  if (h->ring.empty()) {
    h->ring.resize(4 * 4096, nullptr);
    for (auto& e : h->ring) BG_HIP(hipEventCreate(&e));
  }
  h->profiling = true;
  h->ringUsed = 0;
  return BG_OK;
}

extern "C" int bg_profile_end(bg_aligner* h, float* avg_dp, float* avg_fin, int* n) {
  if (!h) return BG_E_ARG;
  BG_HIP(hipSetDevice(h->device));
  BG_HIP(drain(h));
  double dp = 0, fin = 0;
  const int cnt = h->ringUsed / 4;
  for (int i = 0; i < cnt; ++i) {
    float x = 0, y = 0;
    BG_HIP(hipEventElapsedTime(&x, h->ring[4 * i], h->ring[4 * i + 1]));
    BG_HIP(hipEventElapsedTime(&y, h->ring[4 * i + 2], h->ring[4 * i + 3]));
    dp += x;
    fin += y;
  }
  h->profiling = false;
  if (avg_dp) *avg_dp = cnt ? (float)(dp / cnt) : 0.f;
  if (avg_fin) *avg_fin = cnt ? (float)(fin / cnt) : 0.f;
  if (n) *n = cnt;
  return BG_OK;
}

extern "C" int bg_batch_export(bg_aligner* h, void* dst, size_t* bytes) {
  if (!h || !bytes) return BG_E_ARG;
  if (!h->prepared) return BG_E_NO_BATCH;
  const size_t need = 8 + sizeof(BgPairResultDev) * h->npairs + 2 * h->outBytes;
  if (!dst) { *bytes = need; return BG_OK; }
  if (*bytes < need) return BG_E_ARG;
  if (!h->executed) return BG_E_NO_BATCH;
  BG_HIP(hipSetDevice(h->device));
  BG_HIP(drain(h));
  const Slot& S = h->slot[h->lastSlot];
  const uint64_t n = h->npairs;
  BG_HIP(hipMemcpyAsync(dst, &n, 8, hipMemcpyHostToDevice, h->stream));
  if (n)
    BG_HIP(hipMemcpyAsync((uint8_t*)dst + 8, h->recs.p, sizeof(BgPairResultDev) * n,
                          hipMemcpyDeviceToDevice, h->stream));
  if (!h->plan.empty()) {
    BgExportArgs E;
    E.pairs = h->pairs.as<BgPair>();
    E.results = S.results.as<BgResult>();
    E.out1 = S.out1.as<uint8_t>();
    E.out2 = S.out2.as<uint8_t>();
    E.dst = (uint8_t*)dst;
    E.npairs_caller = n;
    E.out_bytes = h->outBytes;
    E.mode = h->mode;
    void* args[] = {&E};
    BG_HIP(hipLaunchKernel(bg_export_kernel_ptr(), dim3((unsigned)h->plan.size()), dim3(256), args, 0, h->stream));
  }
  BG_HIP(hipStreamSynchronize(h->stream));
  *bytes = need;
  return BG_OK;
}

extern "C" int bg_batch_export_compact(bg_aligner* h, void* dst, size_t* bytes) {
  if (!h || !bytes) return BG_E_ARG;
  if (!h->prepared || !h->executed) return BG_E_NO_BATCH;
  BG_HIP(hipSetDevice(h->device));
  const uint64_t n = h->npairs;
  const Slot& S = h->slot[h->lastSlot];
  BgCompactArgs E;
  E.pairs = h->pairs.as<BgPair>();
  E.results = S.results.as<BgResult>();
  E.recs = h->recs.as<BgPairResultDev>();
  E.ops = S.ops.as<uint8_t>();
  E.npairs_caller = n;
  E.nplan = (int32_t)h->plan.size();
  E.mode = h->mode;
  void* args[] = {&E};
  // a handle sharing its device's streams exports on the shared download stream: on the DP stream
  // the export would queue behind the DPs other handles queued after this batch's (bg_group with
  // three batches in flight waited for two more DPs per collect)
  hipStream_t xs = h->stream;
  if (h->shared()) {
    if (!h->dlS) h->dlS = group_stream(h, kSDl);
    if (!h->dlS) return BG_E_HIP;
    xs = h->dlS;
  }
  if (h->compactExec != h->execCount) {
    // sizes and their scan for this execute (after its traceback), then the total to the host
    if (!h->compactSizes.ensure(8 * (n + 1))) return BG_E_NOMEM;
    E.sizes = h->compactSizes.as<uint64_t>();
    E.dst = nullptr;
    BG_HIP(drain(h));
    BG_HIP(hipMemsetAsync(E.sizes, 0, 8 * (n + 1), xs));
    const unsigned g = (unsigned)(((uint64_t)E.nplan + 255) / 256);
    if (g) BG_HIP(hipLaunchKernel(bg_compact_size_kernel_ptr(), dim3(g), dim3(256), args, 0, xs));
    BG_HIP(hipLaunchKernel(bg_compact_scan_kernel_ptr(), dim3(1), dim3(64), args, 0, xs));
    BG_HIP(hipMemcpyAsync(&h->compactOps, E.sizes + n, 8, hipMemcpyDeviceToHost, xs));
    BG_HIP(hipStreamSynchronize(xs));
    h->compactExec = h->execCount;
  }
  const size_t need = 32 + n * sizeof(bg_compact_hdr) + h->compactOps;
  if (!dst) { *bytes = need; return BG_OK; }
  if (*bytes < need) return BG_E_ARG;
  E.sizes = h->compactSizes.as<uint64_t>();
  E.dst = (uint8_t*)dst;
  // plan pairs, then enough workgroups for the caller pairs decided on the host (and the head)
  const unsigned g = (unsigned)E.nplan + (unsigned)((n + 255) / 256) + 1;
  BG_HIP(hipLaunchKernel(bg_compact_write_kernel_ptr(), dim3(g), dim3(256), args, 0, xs));
  BG_HIP(hipStreamSynchronize(xs));
  *bytes = need;
  return BG_OK;
}

// Upper bound of the compact record of the prepared batch: the header, every caller pair's
// bg_compact_hdr and every planned pair's packed ops at their largest, ceil((n1 + n2) / 4).
extern "C" int bg_batch_export_compact_bound(bg_aligner* h, size_t* bytes) {
  if (!h || !bytes) return BG_E_ARG;
  if (!h->prepared) return BG_E_NO_BATCH;
  *bytes = 32 + h->npairs * sizeof(bg_compact_hdr) + h->opsBytes;
  return BG_OK;
}

// bg_batch_export_compact without a host wait (the record of EVERY execute gathered inside a
// pipelined step): the size, scan and write kernels go on the handle's export stream behind the
// last execute's traceback; the slot's next execute waits for them (readDone), and `after` (a
// stream of the handle's device; null = its null stream) waits for them too, so a collective
// queued there reads a finished record.
// the size, scan and write kernels of the last execute's compact record, queued on xs behind its
// traceback; the slot's next execute waits for them (readDone)
static int export_compact_queue(bg_aligner* h, void* dst, size_t cap, hipStream_t xs) {
  const uint64_t n = h->npairs;
  if (cap < 32 + n * sizeof(bg_compact_hdr) + h->opsBytes) return BG_E_ARG;
  Slot& S = h->slot[h->lastSlot];
  if (!h->compactSizes.ensure(8 * (n + 1))) return BG_E_NOMEM;
  BgCompactArgs E;
  E.pairs = h->pairs.as<BgPair>();
  E.results = S.results.as<BgResult>();
  E.recs = h->recs.as<BgPairResultDev>();
  E.ops = S.ops.as<uint8_t>();
  E.sizes = h->compactSizes.as<uint64_t>();
  E.dst = static_cast<uint8_t*>(dst);
  E.npairs_caller = n;
  E.nplan = (int32_t)h->plan.size();
  E.mode = h->mode;
  void* args[] = {&E};
  if (S.inflight) BG_HIP(hipStreamWaitEvent(xs, S.finDone, 0));
  BG_HIP(hipMemsetAsync(E.sizes, 0, 8 * (n + 1), xs));
  const unsigned gs = (unsigned)(((uint64_t)E.nplan + 255) / 256);
  if (gs) BG_HIP(hipLaunchKernel(bg_compact_size_kernel_ptr(), dim3(gs), dim3(256), args, 0, xs));
  BG_HIP(hipLaunchKernel(bg_compact_scan_kernel_ptr(), dim3(1), dim3(64), args, 0, xs));
  const unsigned gw = (unsigned)E.nplan + (unsigned)((n + 255) / 256) + 1;
  BG_HIP(hipLaunchKernel(bg_compact_write_kernel_ptr(), dim3(gw), dim3(256), args, 0, xs));
  BG_HIP(hipEventRecord(S.readDone, xs));
  S.readPending = true;
  h->compactExec = -1;             // the sizes now belong to this record
  return BG_OK;
}

extern "C" int bg_batch_export_compact_async(bg_aligner* h, void* dst, size_t cap, void* after) {
  if (!h || !dst) return BG_E_ARG;
  if (!h->prepared || !h->executed) return BG_E_NO_BATCH;
  BG_HIP(hipSetDevice(h->device));
  if (!h->dlS) h->dlS = group_stream(h, kSDl);
  if (!h->dlS) return BG_E_HIP;
  const int e = export_compact_queue(h, dst, cap, h->dlS);
  if (e) return e;
  // NULL is the device's null stream (torch's default current stream): a valid stream to order
  BG_HIP(hipStreamWaitEvent(static_cast<hipStream_t>(after), h->slot[h->lastSlot].readDone, 0));
  return BG_OK;
}

// bg_group's form (not in the C ABI): the record is queued on the traceback's own stream right
// after the execute, once `first` (the previous reader of dst) has fired, and `done` marks it
// written.  On the download stream the exports of the batches in flight would sit ahead of the
// oldest batch's gather and download, and each waits for its own traceback.
extern "C" int bg_batch_export_compact_behind_traceback(bg_aligner* h, void* dst, size_t cap,
                                                         void* first, void* done) {
  if (!h || !dst || !done) return BG_E_ARG;
  if (!h->prepared || !h->executed) return BG_E_NO_BATCH;
  BG_HIP(hipSetDevice(h->device));
  hipStream_t xs = h->lastFs ? h->lastFs : h->stream2;
  if (first) BG_HIP(hipStreamWaitEvent(xs, static_cast<hipEvent_t>(first), 0));
  const int e = export_compact_queue(h, dst, cap, xs);
  if (e) return e;
  BG_HIP(hipEventRecord(static_cast<hipEvent_t>(done), xs));
  return BG_OK;
}

extern "C" int bg_compact_expand(const void* rec, size_t rec_bytes, size_t npairs,
                                 const uint8_t* const* s1, const size_t* n1, const uint8_t* const* s2,
                                 const size_t* n2, bg_pair_result* results, uint8_t* out1,
                                 uint8_t* out2, size_t out_cap) {
  return bgh::compact_expand(static_cast<const uint8_t*>(rec), rec_bytes, npairs, s1, n1, s2, n2,
                             results, out1, out2, out_cap);
}

// ------------------------------------------------------------------ edit distance, LCS
// Both run on the aligner's hot path with a byte-equality scoring over the bytes the batch holds
// (any of the 256):
//   analysis::seq::edit_distance (src/analysis/seq.rs:105-130) = -(global score) with S = 0 / -1
//     and a = b = -1 (the Levenshtein recurrence is the linear-gap global DP), score only;
//   processing::patterns::longest_common_subsequence (src/processing/patterns.rs:82-118) = the
//     diagonal columns of the global traceback with S = +1 / -1, a = b = 0 (M is the match
//     table), under the LCS tie rule (BG_FIN_LCS), on the score-only kernel family that
//     recomputes full-trace chunks.
static int equality_scoring(size_t npairs, const uint8_t* const* s1, const size_t* n1,
                            const uint8_t* const* s2, const size_t* n2, int32_t match,
                            int32_t mismatch, HScore* sc) {
  bool seen[256] = {false};
  for (size_t p = 0; p < npairs; ++p) {
    if ((n1[p] && !s1[p]) || (n2[p] && !s2[p])) return BG_E_ARG;
    for (size_t i = 0; i < n1[p]; ++i) seen[s1[p][i]] = true;
    for (size_t j = 0; j < n2[p]; ++j) seen[s2[p][j]] = true;
  }
  int k = 0;
  for (int x = 0; x < 256; ++x) sc->code[x] = seen[x] ? (uint16_t)k++ : (uint16_t)0xFFFF;
  sc->K = std::max(k, 1);
  sc->tab.assign((size_t)sc->K * sc->K, mismatch);
  for (int r = 0; r < sc->K; ++r) sc->tab[(size_t)r * sc->K + r] = match;
  return BG_OK;
}

// results of the last execute in caller order (no strings)
static int fetch_scores(bg_aligner* h, std::vector<BgResult>& out) {
  int rc = bg_synchronize(h);
  if (rc) return rc;
  const size_t np = h->plan.size();
  h->hres.resize(np);
  if (np)
    BG_HIP(hipMemcpy(h->hres.data(), h->slot[h->lastSlot].results.p, sizeof(BgResult) * np,
                     hipMemcpyDeviceToHost));
  out.assign(h->npairs, BgResult{});
  for (size_t q = 0; q < np; ++q) out[h->order_[q]] = h->hres[q];
  return BG_OK;
}

extern "C" int bg_edit_distance_batch(bg_aligner* h, size_t npairs, const uint8_t* const* s1,
                                      const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                                      uint64_t* dist) {
  if (!h || (npairs && (!s1 || !n1 || !s2 || !n2 || !dist))) return BG_E_ARG;
  HScore sc;
  int rc = equality_scoring(npairs, s1, n1, s2, n2, 0, -1, &sc);
  if (rc) return rc;
  h->finFlags = BG_FIN_SCORE_ONLY;
  rc = prepare_impl(h, BG_GLOBAL, npairs, s1, n1, s2, n2, sc, -1, -1);
  if (!rc) rc = bg_batch_execute(h);
  std::vector<BgResult> res;
  if (!rc) rc = fetch_scores(h, res);
  h->finFlags = 0;
  h->prepared = false;       // the flags belong to this call's batch
  if (rc) return rc;
  for (size_t p = 0; p < npairs; ++p) {
    if (h->prestatus[p] >= 0) return BG_E_ARG;        // unreachable: equality scores every byte
    dist[p] = (uint64_t)(-(int64_t)res[p].score);
  }
  return BG_OK;
}

extern "C" int bg_lcs_batch(bg_aligner* h, size_t npairs, const uint8_t* const* s1,
                            const size_t* n1, const uint8_t* const* s2, const size_t* n2,
                            uint8_t* out, size_t out_cap, uint64_t* offset, uint64_t* len) {
  if (!h || (npairs && (!s1 || !n1 || !s2 || !n2 || !offset || !len))) return BG_E_ARG;
  size_t need = 0;
  for (size_t p = 0; p < npairs; ++p) need += std::min(n1[p], n2[p]);
  if (need && (!out || out_cap < need)) return BG_E_ARG;
  HScore sc;
  int rc = equality_scoring(npairs, s1, n1, s2, n2, 1, -1, &sc);
  if (rc) return rc;
  const int allowTag = h->allowTag, allowAck = h->allowAck;
  h->allowTag = 0;           // the LCS tie rule lives in the recomputing affine-family traceback
  h->allowAck = 1;
  h->finFlags = BG_FIN_LCS;
  rc = prepare_impl(h, BG_GLOBAL, npairs, s1, n1, s2, n2, sc, 0, 0);
  // (pairs beyond the checkpoint tracebacks' chunk keys run the full-trace mask kernel with the
  // LCS rule in its trace bits, bg_dp_kernel<4, ..., LCS>)
  if (!rc) rc = bg_batch_execute(h);
  std::vector<bg_pair_result> res(npairs);
  std::vector<uint8_t> a1(h->outBytes + 1), ops(h->outBytes + 1);
  if (!rc) rc = bg_batch_fetch(h, res.data(), a1.data(), ops.data(), h->outBytes + 1);
  h->allowTag = allowTag;
  h->allowAck = allowAck;
  h->finFlags = 0;
  h->prepared = false;
  if (rc) return rc;
  size_t o = 0;
  for (size_t p = 0; p < npairs; ++p) {
    offset[p] = o;
    const size_t base = res[p].offset;
    for (uint32_t x = 0; x < res[p].len; ++x)
      if (ops[base + x] == 0) out[o++] = a1[base + x];       // diagonal column = a match
    len[p] = o - offset[p];
  }
  return BG_OK;
}
