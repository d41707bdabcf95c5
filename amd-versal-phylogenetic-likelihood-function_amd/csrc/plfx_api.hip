// plfx_api.hip -- the C ABI of include/plfx.h over the HIP kernels.
//
// Replaces the reference host's XRT layer (app/src/host_mem.cpp:108-157
// kernel/bo/run setup, :283-394 run loop) and its CPU entry point plf()
// (app/src/plf.h:1-5).  No C++ exception crosses this boundary; every entry
// point returns a plfx_status.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <deque>
#include <new>
#include <string>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/plfx.h"
#include "plf_kernels.hpp"
#include "testbench.hpp"

constexpr int kHostChunksMax = 16;

// Scaler-sum / lnL reduction workspace of one stream (plf_dna.hpp
// block_ticket_sum, plf_lnl.hpp): zero at rest, restored to zero by the last
// arriving block of every launch.  One per stream, so sum-producing launches
// on different streams of one context may overlap (plfx.h, "Streams and the
// scaler-sum workspace").  hipStreamPerThread is one handle value that names a
// different stream in every host thread, so its workspaces are keyed by
// (handle, thread).  Entries come from a pool allocated and zeroed with the
// context (no allocation on a call path for the first kWsPool streams, so a
// stream's first use may be inside a graph capture); plfx_ctx_release_stream
// returns an entry to the pool -- unless a graph was captured through it: the
// graph's replays keep using the entry's words, so it is retired (never handed
// to another stream) and the context waits for the device when destroyed.
// plfx_ctx_destroy never touches a caller's stream handle (the stream may be
// gone by then): an entry still held by a stream other than the context's is
// waited for device-wide.  (An event recorded after each call cannot stand
// in: HIP rejects waiting on an event whose stream was destroyed -- an exited
// thread's hipStreamPerThread gave hipErrorCapturedEvent (907) on the box.)
struct StreamWs {
  hipStream_t stream = nullptr;
  std::thread::id tid;               // owning thread for hipStreamPerThread, else none
  bool in_use = false;
  bool captured = false;             // used while its stream was capturing
  bool retired = false;              // released after a capture, or its thread exited
  bool cap_now = false;              // the current call's stream is capturing
  unsigned long long *ws = nullptr;  // kWsRegions x kWsWords u64
  double *lnl_partials = nullptr;    // kLnlMaxGrid doubles
  unsigned long long *lnl_ticket = nullptr;
  // tip/tip protein combination tables (kTtEntryBytes): allocated with the
  // entry, or on first use with PLFX_CTX_LAZY_TABLES (nullptr until then)
  char *tt = nullptr;
};
constexpr int kWsPool = PLFX_WS_POOL;

struct plfx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_blocks = 0;               // grid cap for the grid-stride kernels (0 = resident blocks)
  int node_segments = -1;           // node kernels' XCD-segmented mapping: -1 by size, 0 off, 1 on
                                    // (PLFX_NODE_SEGMENTS; plf_kernels.hip use_segments)
  int streams = 1;                  // one-node calls kept in flight (plfx_ctx_set_streams, PLFX_STREAMS)
  int fuse = 3;  // traverse: 3 six-level subtrees before 2's, 2 three-level subtrees +
                 // level pairs, 1 level pairs, 0 none (PLFX_FUSE)
  bool lazy_tables = false;         // PLFX_CTX_LAZY_TABLES
  std::deque<StreamWs> wss;         // per-stream workspaces (stable addresses)
  std::vector<void *> ws_blocks;    // their allocations (the pool's, then one per extra entry)
  uint8_t *tt_codes = nullptr;      // the tip/tip tables' two constant 576-code arrays (kTtCodeBytes)
  int sched[PLFX_SCHED_COUNTS] = {};  // schedule of the last traverse
  // grow-only staging for the synchronous host entry points
  void *d_buf = nullptr;
  size_t d_cap = 0;
  // host entry pipelining: D2H of chunk i on its own stream while chunk i+1 uploads
  hipStream_t d2h_stream = nullptr;
  hipEvent_t chunk_done[kHostChunksMax] = {};
  std::string err;
  // calls on one context from several host threads are serialised (recursive:
  // entry points call each other, e.g. instance_run_host -> instance_run)
  mutable std::recursive_mutex mu;
};

namespace {

// Every entry point runs with the context's device current and gives the
// caller's current device back (hipSetDevice is per host thread).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
    else prev = -1;  // nothing to restore
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard &) = delete;
  DeviceGuard &operator=(const DeviceGuard &) = delete;
};

#define PLFX_BIND(ctx)                                              \
  if (!(ctx)) return PLFX_ERR_INVALID;                              \
  std::lock_guard<std::recursive_mutex> plfx_lock_((ctx)->mu);      \
  DeviceGuard plfx_guard_((ctx)->device)

constexpr size_t kWsRegions = std::max({(size_t)plfx::kMaxBatch, (size_t)7 * plfx::kMaxSeptets,
                                        (size_t)plfx::kDeepNodes, (size_t)plfx::kDeepQueueRegion + 1});
constexpr size_t kWsBytes = kWsRegions * plfx::kWsWords * sizeof(unsigned long long);
constexpr size_t kLnlPartialBytes = plfx::kLnlMaxGrid * sizeof(double);
constexpr size_t kLnlTicketBytes = plfx::kWsWords * sizeof(unsigned long long);

int fail(plfx_ctx *ctx, int code, const char *fmt, ...) {
  if (ctx) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    ctx->err = buf;
  }
  return code;
}

int hip_fail(plfx_ctx *ctx, hipError_t e, const char *what) {
  return fail(ctx, PLFX_ERR_HIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

#define PLFX_HIP(ctx, call)                          \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
  } while (0)

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// NULL is the HIP null stream, as in every HIP API; pass plfx_ctx_stream(ctx)
// to run on the context's own stream.
hipStream_t pick(plfx_ctx *, void *stream) { return reinterpret_cast<hipStream_t>(stream); }

constexpr size_t kWsEntryBytes = kWsBytes + kLnlPartialBytes + kLnlTicketBytes;

// Tip/tip protein combination tables (plf_prot.hpp prot_tiptip_gather_kernel):
// per node of a launch group, a 576 x 80 table of the node's dtype and 576
// scaler bytes, in every workspace entry (written by the table kernel before
// each use, so never zeroed), and the two constant 576-code arrays (combo
// k = code1 * 24 + code2) once per context.  Allocated with the entries, so
// a stream's first tip/tip call -- also inside a capture -- takes the tables;
// under PLFX_CTX_LAZY_TABLES they are allocated on an entry's first tip/tip
// call instead, and that first call is refused (PLFX_ERR_INVALID) inside a
// capture.
constexpr size_t kTtCodeBytes = 2048;
constexpr size_t kTtTabBytes = (size_t)plfx::kProtCombos * 80 * sizeof(double);
constexpr size_t kTtScBytes = 1024;
constexpr size_t kTtEntryBytes = (size_t)plfx::kMaxBatch * (kTtTabBytes + kTtScBytes);

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  return s && hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
}

// Threads that took a hipStreamPerThread workspace of a live context: when
// such a thread exits without releasing it, its entry is retired (its stream
// is gone with the thread, so nothing may wait on it) and reclaimed, after a
// device synchronisation, when the context runs out of entries.
std::mutex g_live_mu;
std::vector<plfx_ctx *> g_live;  // contexts not yet destroyed

void orphan_thread_entries(plfx_ctx *ctx, std::thread::id tid);

struct PerThreadEntries {
  std::vector<plfx_ctx *> ctxs;
  ~PerThreadEntries() {
    std::lock_guard<std::mutex> l(g_live_mu);
    for (plfx_ctx *c : ctxs)
      if (std::find(g_live.begin(), g_live.end(), c) != g_live.end())
        orphan_thread_entries(c, std::this_thread::get_id());
  }
};
thread_local PerThreadEntries t_entries;

// the key thread of a stream handle: the calling thread for hipStreamPerThread
std::thread::id ws_thread(hipStream_t s) {
  return s == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id();
}

StreamWs *ws_find(plfx_ctx *ctx, hipStream_t s) {
  const std::thread::id tid = ws_thread(s);
  for (StreamWs &w : ctx->wss)
    if (w.in_use && !w.retired && w.stream == s && w.tid == tid) return &w;
  return nullptr;
}

void orphan_thread_entries(plfx_ctx *ctx, std::thread::id tid) {
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  for (StreamWs &w : ctx->wss)
    if (w.in_use && !w.retired && w.stream == hipStreamPerThread && w.tid == tid) {
      w.retired = true;
      w.stream = nullptr;
      w.tid = std::thread::id();
    }
}

void ws_carve(StreamWs &w, void *base, void *tt) {
  char *b = static_cast<char *>(base);
  w.ws = reinterpret_cast<unsigned long long *>(b);
  w.lnl_partials = reinterpret_cast<double *>(b + kWsBytes);
  w.lnl_ticket = reinterpret_cast<unsigned long long *>(b + kWsBytes + kLnlPartialBytes);
  w.tt = static_cast<char *>(tt);
}

// An entry taken by stream s: keyed to it, marked if s is capturing, and for
// hipStreamPerThread remembered by the calling thread (retired at its exit).
StreamWs *ws_take(plfx_ctx *ctx, StreamWs &w, hipStream_t s) {
  w.in_use = true;
  w.retired = false;
  w.captured = false;
  w.stream = s;
  w.tid = ws_thread(s);
  if (s == hipStreamPerThread &&
      std::find(t_entries.ctxs.begin(), t_entries.ctxs.end(), ctx) == t_entries.ctxs.end())
    t_entries.ctxs.push_back(ctx);
  return &w;
}

// The workspace of stream s: its own, else a free pool entry (zero at rest),
// else a retired per-thread entry reclaimed after a device synchronisation,
// else a new allocation (zeroed in order on s) -- neither of the last two
// inside a stream capture.  An entry used while s is capturing is marked: the
// graph keeps using it after the capture.
StreamWs *ws_for(plfx_ctx *ctx, hipStream_t s, int *rc) {
  *rc = PLFX_OK;
  const bool cap = capturing(s);
  StreamWs *got = ws_find(ctx, s);
  if (!got)
    for (StreamWs &w : ctx->wss)
      if (!w.in_use) {
        got = ws_take(ctx, w, s);
        break;
      }
  if (!got && !cap) {
    // entries of exited threads' per-thread streams (not captured: those
    // stay retired): their last launches must be done before reuse, and the
    // thread's stream is gone -- so the device is waited for
    bool any = false;
    for (StreamWs &w : ctx->wss) any |= w.in_use && w.retired && !w.captured;
    if (any) {
      hipError_t e = hipDeviceSynchronize();
      if (e != hipSuccess) {
        *rc = hip_fail(ctx, e, "reclaiming workspaces of exited threads");
        return nullptr;
      }
      for (StreamWs &w : ctx->wss)
        if (w.in_use && w.retired && !w.captured) w.in_use = false;
      for (StreamWs &w : ctx->wss)
        if (!w.in_use) {
          got = ws_take(ctx, w, s);
          break;
        }
    }
  }
  if (got) {
    got->captured = got->captured || cap;
    got->cap_now = cap;
    return got;
  }
  if ((int)ctx->wss.size() >= PLFX_MAX_STREAMS) {
    *rc = fail(ctx, PLFX_ERR_INVALID,
               "more than %d streams in use with one context (release idle ones with "
               "plfx_ctx_release_stream)", PLFX_MAX_STREAMS);
    return nullptr;
  }
  if (cap) {
    *rc = fail(ctx, PLFX_ERR_INVALID,
               "more than %d streams in use and this one is being captured: issue one call on "
               "the stream before capturing (its reduction workspace is allocated then)", kWsPool);
    return nullptr;
  }
  // stream-ordered on s: usable by s's next launch with no host wait (and
  // freed stream-ordered at destroy, which a plain hipFree would turn into a
  // wait for the whole device)
  void *block = nullptr;
  const size_t bytes = kWsEntryBytes + (ctx->lazy_tables ? 0 : kTtEntryBytes);
  hipError_t e = hipMallocAsync(&block, bytes, s);
  if (e != hipSuccess) {
    *rc = fail(ctx, PLFX_ERR_NOMEM, "workspace hipMallocAsync(%zu): %s", bytes, hipGetErrorString(e));
    return nullptr;
  }
  e = hipMemsetAsync(block, 0, kWsEntryBytes, s);
  if (e != hipSuccess) {
    (void)hipFreeAsync(block, s);
    *rc = hip_fail(ctx, e, "workspace memset");
    return nullptr;
  }
  ctx->ws_blocks.push_back(block);
  StreamWs w;
  ws_carve(w, block, ctx->lazy_tables ? nullptr : static_cast<char *>(block) + kWsEntryBytes);
  ctx->wss.push_back(w);
  return ws_take(ctx, ctx->wss.back(), s);
}

// the workspace of stream s as `out`; returns from the caller on failure
#define PLFX_WS(ctx, s, out)                      \
  StreamWs *out = nullptr;                        \
  do {                                            \
    int wrc_ = PLFX_OK;                           \
    out = ws_for((ctx), (s), &wrc_);              \
    if (!out) return wrc_;                        \
  } while (0)

// [a, a + na) and [b, b + nb) share a byte
bool overlap(const void *a, size_t na, const void *b, size_t nb) {
  const uintptr_t pa = reinterpret_cast<uintptr_t>(a), pb = reinterpret_cast<uintptr_t>(b);
  return na > 0 && nb > 0 && pa < pb + nb && pb < pa + na;
}

// clv_bytes: bytes of one CLV of the call (n * 4 categories * states * element
// size); a tip child is n code bytes.  The parent may not share a byte with
// either child: every site's children are read by other blocks than the one
// writing that site's parent.
int check_dev_args(plfx_ctx *ctx, const void *x1, const void *x2, const void *x3, const void *EV,
                   int64_t n, const void *left, const void *right, size_t clv_bytes) {
  if (!ctx) return PLFX_ERR_INVALID;
  if (n < 0) return fail(ctx, PLFX_ERR_INVALID, "n < 0 (%lld)", (long long)n);
  if (n == 0) return PLFX_OK;
  if (!x1 || !x2 || !x3 || !EV || !left || !right)
    return fail(ctx, PLFX_ERR_INVALID, "null CLV/matrix pointer");
  if (!aligned16(x1) || !aligned16(x2) || !aligned16(x3))
    return fail(ctx, PLFX_ERR_INVALID, "CLV pointers must be 16-byte aligned");
  if (overlap(x3, clv_bytes, x1, clv_bytes) || overlap(x3, clv_bytes, x2, clv_bytes))
    return fail(ctx, PLFX_ERR_INVALID, "x3 may not overlap x1/x2");
  return PLFX_OK;
}

template <typename T>
int plf_dev(plfx_ctx *ctx, const T *x1, const T *x2, T *x3, const T *EV, int64_t n, const T *left,
            const T *right, const int32_t *wgt, uint8_t *scaler, int64_t *scaler_sum,
            void *stream) {
  int rc = check_dev_args(ctx, x1, x2, x3, EV, n, left, right, (size_t)n * 16 * sizeof(T));
  if (rc != PLFX_OK) return rc;
  hipStream_t s = pick(ctx, stream);
  if (n == 0) {
    if (scaler_sum) PLFX_HIP(ctx, hipMemsetAsync(scaler_sum, 0, sizeof(int64_t), s));
    return PLFX_OK;
  }
  PLFX_WS(ctx, s, w);
  plfx::DnaArgs a{x1, x2, x3, EV, left, right, wgt, scaler, scaler_sum, w->ws, n, ctx->node_segments};
  a.streams = ctx->streams;
  hipError_t e = sizeof(T) == 4 ? plfx::launch_plf_dna_f32(a, ctx->max_blocks, s)
                                : plfx::launch_plf_dna_f64(a, ctx->max_blocks, s);
  if (e != hipSuccess) return hip_fail(ctx, e, "plf_dna launch");
  return PLFX_OK;
}

int ensure_dbuf(plfx_ctx *ctx, size_t bytes) {
  if (bytes <= ctx->d_cap) return PLFX_OK;
  if (ctx->d_buf) {
    // the last call's downloads (d2h_stream) and launches (stream) read it
    if (ctx->d2h_stream) PLFX_HIP(ctx, hipStreamSynchronize(ctx->d2h_stream));
    PLFX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PLFX_HIP(ctx, hipFreeAsync(ctx->d_buf, ctx->stream));
    ctx->d_buf = nullptr;
    ctx->d_cap = 0;
  }
  hipError_t e = hipMallocAsync(&ctx->d_buf, bytes, ctx->stream);
  if (e != hipSuccess) return fail(ctx, PLFX_ERR_NOMEM, "hipMallocAsync(%zu): %s", bytes, hipGetErrorString(e));
  ctx->d_cap = bytes;
  return PLFX_OK;
}

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// plf()-shaped synchronous host entry (the reference's hm / msm / mh regions,
// host_mem.cpp:293-318): H2D -> fused kernel -> D2H, pipelined over up to
// kHostChunksMax site chunks -- chunk i's results go back on a second stream
// while chunk i+1 uploads, so the two PCIe directions overlap (the reference
// overlaps its two uploads and its two downloads, host_mem.cpp:297-314).  The
// chunks are independent sites; the scaler sum is the sum of the chunk sums.
template <typename T>
int plf_host(plfx_ctx *ctx, const T *x1, const T *x2, T *x3, const T *EV, int n, const T *left,
             const T *right, const int *wgt, int *scalerIncrement) {
  if (!ctx) return PLFX_ERR_INVALID;
  if (n < 0) return fail(ctx, PLFX_ERR_INVALID, "n < 0 (%d)", n);
  if (n > 0 && (!x1 || !x2 || !x3 || !EV || !left || !right))
    return fail(ctx, PLFX_ERR_INVALID, "null argument");
  if (wgt && n >= 512) {  // the reduction's bound (plfx.h): sum |wgt| < 2^40
    int64_t tot = 0;
    for (int i = 0; i < n; i++) tot += wgt[i] < 0 ? -(int64_t)wgt[i] : (int64_t)wgt[i];
    if (tot >= (int64_t(1) << 40)) return fail(ctx, PLFX_ERR_INVALID, "sum |wgt| >= 2^40");
  }
  constexpr int64_t kMinChunk = 1 << 17;  // sites; smaller chunks pay per-copy overheads
  const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(kHostChunksMax, n / kMinChunk));
  const int64_t chunk = ((int64_t)n + nch - 1) / nch;
  const size_t clv = (size_t)n * 16 * sizeof(T);
  const size_t o_x1 = 0, o_x2 = round_up(clv, 256), o_x3 = o_x2 + round_up(clv, 256);
  const size_t o_mat = o_x3 + round_up(clv, 256);  // EV 16 | left 64 | right 64
  const size_t o_wgt = o_mat + round_up(144 * sizeof(T), 256);
  const size_t o_sum = o_wgt + round_up((size_t)n * sizeof(int32_t), 256);  // int64 per chunk
  const size_t total = o_sum + round_up(kHostChunksMax * sizeof(int64_t), 256);
  int rc = ensure_dbuf(ctx, total);
  if (rc != PLFX_OK) return rc;
  if (!ctx->d2h_stream) {
    PLFX_HIP(ctx, hipStreamCreateWithFlags(&ctx->d2h_stream, hipStreamNonBlocking));
    for (hipEvent_t &e : ctx->chunk_done) PLFX_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  char *d = static_cast<char *>(ctx->d_buf);
  hipStream_t s = ctx->stream, s2 = ctx->d2h_stream;
  const T *dm = reinterpret_cast<const T *>(d + o_mat);
  int64_t *dsum = reinterpret_cast<int64_t *>(d + o_sum);
  if (n > 0) {
    PLFX_HIP(ctx, hipMemcpyAsync(d + o_mat, EV, 16 * sizeof(T), hipMemcpyHostToDevice, s));
    PLFX_HIP(ctx, hipMemcpyAsync(d + o_mat + 16 * sizeof(T), left, 64 * sizeof(T), hipMemcpyHostToDevice, s));
    PLFX_HIP(ctx, hipMemcpyAsync(d + o_mat + 80 * sizeof(T), right, 64 * sizeof(T), hipMemcpyHostToDevice, s));
  }
  int used = 0;
  for (int64_t lo = 0; lo < n || (n == 0 && used == 0); lo += chunk, used++) {
    const int64_t m = std::min<int64_t>(chunk, n - lo);
    const size_t off = (size_t)lo * 16 * sizeof(T), bytes = (size_t)m * 16 * sizeof(T);
    if (m > 0) {
      PLFX_HIP(ctx, hipMemcpyAsync(d + o_x1 + off, x1 + lo * 16, bytes, hipMemcpyHostToDevice, s));
      PLFX_HIP(ctx, hipMemcpyAsync(d + o_x2 + off, x2 + lo * 16, bytes, hipMemcpyHostToDevice, s));
      if (wgt)
        PLFX_HIP(ctx, hipMemcpyAsync(d + o_wgt + lo * 4, wgt + lo, (size_t)m * 4, hipMemcpyHostToDevice, s));
    }
    rc = plf_dev<T>(ctx, reinterpret_cast<const T *>(d + o_x1 + off),
                    reinterpret_cast<const T *>(d + o_x2 + off), reinterpret_cast<T *>(d + o_x3 + off),
                    dm, std::max<int64_t>(m, 0), dm + 16, dm + 80,
                    wgt ? reinterpret_cast<const int32_t *>(d + o_wgt + lo * 4) : nullptr, nullptr,
                    dsum + used, s);
    if (rc != PLFX_OK) return rc;
    if (m > 0) {
      PLFX_HIP(ctx, hipEventRecord(ctx->chunk_done[used], s));
      PLFX_HIP(ctx, hipStreamWaitEvent(s2, ctx->chunk_done[used], 0));
      PLFX_HIP(ctx, hipMemcpyAsync(x3 + lo * 16, d + o_x3 + off, bytes, hipMemcpyDeviceToHost, s2));
    }
    if (n == 0) break;
  }
  int64_t sums[kHostChunksMax] = {};
  PLFX_HIP(ctx, hipMemcpyAsync(sums, dsum, (size_t)used * sizeof(int64_t), hipMemcpyDeviceToHost, s));
  PLFX_HIP(ctx, hipStreamSynchronize(s));
  PLFX_HIP(ctx, hipStreamSynchronize(s2));
  int64_t sum = 0;
  for (int i = 0; i < used; i++) sum += sums[i];
  if (scalerIncrement) *scalerIncrement = (int)sum;
  return PLFX_OK;
}

// One node of a kind (tips = number of tip children, tip child first); i
// names it in the message (the op index in a traversal); clv_bytes as
// check_dev_args.
int check_node(plfx_ctx *ctx, const plfx_node &d, int tips, int64_t n, int i, size_t clv_bytes) {
  if (n <= 0) return PLFX_OK;
  if (!d.x1 || !d.x2 || !d.x3 || !d.left || !d.right)
    return fail(ctx, PLFX_ERR_INVALID, "node %d: null CLV/tip/matrix pointer", i);
  if ((tips < 1 && !aligned16(d.x1)) || (tips < 2 && !aligned16(d.x2)) || !aligned16(d.x3))
    return fail(ctx, PLFX_ERR_INVALID, "node %d: CLV pointers must be 16-byte aligned", i);
  const size_t b1 = tips >= 1 ? (size_t)n : clv_bytes, b2 = tips >= 2 ? (size_t)n : clv_bytes;
  if (overlap(d.x3, clv_bytes, d.x1, b1) || overlap(d.x3, clv_bytes, d.x2, b2))
    return fail(ctx, PLFX_ERR_INVALID, "node %d: x3 may not overlap a child", i);
  return PLFX_OK;
}

size_t clv_bytes_of(int dtype, int states, int64_t n) {
  return (size_t)(n > 0 ? n : 0) * 4 * states * (dtype == PLFX_F32 ? 4 : 8);
}

// A tip/tip protein node whose values sit in its stream's combination tables
// after batch_impl: its CLV (x3), its table and its two tip-code arrays.
struct TabRef {
  const void *x3;
  const void *tab;
  const uint8_t *ca, *cb;
};

// Nodes of one kind (tips = number of tip children, tip child first) in
// launches of kMaxBatch.  A tip child is a uint8 code array (no alignment rule).
// *launches counts the kernel launches issued (may be NULL).  *tabs (may be
// NULL) receives the tip/tip protein nodes whose tables are still in the
// stream's workspace afterwards (the last launch group's).
int batch_impl(plfx_ctx *ctx, int dtype, const plfx_node *nodes, int count, const void *EV,
               int64_t n, const int32_t *wgt, hipStream_t s, int tips,
               const void *tipvec = nullptr, int states = 4, int flags = PLFX_EXACT,
               int *launches = nullptr, std::vector<TabRef> *tabs = nullptr,
               const int *ids = nullptr, int streams = 1) {
  if (tabs) tabs->clear();
  if (count < 0 || n < 0 || (count > 0 && (!nodes || !EV)))
    return fail(ctx, PLFX_ERR_INVALID, "bad batch arguments");
  for (int i = 0; i < count; i++) {
    const plfx_node &d = nodes[i];
    int rc = check_node(ctx, d, tips, n, ids ? ids[i] : i, clv_bytes_of(dtype, states, n));
    if (rc != PLFX_OK) return rc;
    if (n == 0 && d.scaler_sum) PLFX_HIP(ctx, hipMemsetAsync(d.scaler_sum, 0, sizeof(int64_t), s));
  }
  if (n == 0 || count == 0) return PLFX_OK;
  PLFX_WS(ctx, s, w);
  if (states == 20 && tips == 2) {
    // both children coded tips: the node's 576 code pairs through its own
    // kernel, then x3 / scaler / sum gathered by code pair (a write stream;
    // the direct kernel is compute-bound: 77 us f64, 95 us f32 per 2^18 sites)
    {
      if (!w->tt) {  // PLFX_CTX_LAZY_TABLES: this entry's tables on its first tip/tip use
        if (w->cap_now)
          return fail(ctx, PLFX_ERR_INVALID,
                      "protein tip/tip tables: the context was created with PLFX_CTX_LAZY_TABLES and "
                      "this stream has not made a tip/tip call outside a capture yet");
        void *t = nullptr;
        hipError_t e = hipMallocAsync(&t, kTtEntryBytes, s);
        if (e != hipSuccess)
          return fail(ctx, PLFX_ERR_NOMEM, "tip/tip tables hipMallocAsync(%zu): %s", kTtEntryBytes,
                      hipGetErrorString(e));
        ctx->ws_blocks.push_back(t);
        w->tt = static_cast<char *>(t);
      }
      char *tt = w->tt;
      const uint8_t *cc1 = ctx->tt_codes, *cc2 = cc1 + 1024;
      for (int j = 0; j < count; j += plfx::kMaxBatch) {
        const int c = std::min(count - j, plfx::kMaxBatch);
        plfx::NodeDescH comb[plfx::kMaxBatch];
        plfx::ProtGatherDescH g[plfx::kMaxBatch];
        for (int i = 0; i < c; i++) {
          const plfx_node &d = nodes[j + i];
          char *tab = tt + (size_t)i * (kTtTabBytes + kTtScBytes);
          uint8_t *tsc = reinterpret_cast<uint8_t *>(tab + kTtTabBytes);
          comb[i] = plfx::NodeDescH{cc1, cc2, tab, d.left, d.right, tsc, nullptr};
          g[i] = plfx::ProtGatherDescH{static_cast<const uint8_t *>(d.x1), static_cast<const uint8_t *>(d.x2),
                                       d.x3, d.scaler, d.scaler_sum, tab, tsc};
        }
        hipError_t e = plfx::launch_plf_prot_batch(dtype, (flags & PLFX_FMA) != 0, comb, c, EV, nullptr,
                                                   plfx::kProtCombos, w->ws, ctx->max_blocks, s, 2, tipvec);
        if (e != hipSuccess) return hip_fail(ctx, e, "plf_prot combination tables");
        e = plfx::launch_prot_tiptip_gather(dtype, g, c, wgt, n, w->ws, ctx->max_blocks, s);
        if (e != hipSuccess) return hip_fail(ctx, e, "plf_prot tip/tip gather");
        if (launches) *launches += 2;
        if (tabs) {  // this group's tables stay until the next group overwrites them
          tabs->clear();
          for (int i = 0; i < c; i++)
            tabs->push_back(TabRef{nodes[j + i].x3, comb[i].x3, static_cast<const uint8_t *>(nodes[j + i].x1),
                                   static_cast<const uint8_t *>(nodes[j + i].x2)});
        }
      }
      return PLFX_OK;
    }
  }
  if (states == 20 && count > 1) {
    // protein: up to kMaxBatch nodes per launch, node = blockIdx.y, each node
    // with the full resident grid so the nodes' blocks follow each other
    // through the co-resident slots (the next node's blocks fill the CUs the
    // previous node's last trips leave idle).  64-taxon tree at 2^18 sites per
    // sweep vs one launch per node: f64 FMA 5.67 -> 5.38 ms, f64 exact 8.45 ->
    // 8.02 ms, f32 FMA 2.94 -> 2.66 ms; splitting the resident grid over the
    // nodes (the DNA batches' rule) gains only 1-3 % (tools/prot_batch_ab.py@f9b3af3,
    // profiles/r03_protein_batch_ab.log).
    const plfx::NodeDescH *all = reinterpret_cast<const plfx::NodeDescH *>(nodes);
    for (int j = 0; j < count; j += plfx::kMaxBatch) {
      const int c = std::min(count - j, plfx::kMaxBatch);
      hipError_t e = plfx::launch_plf_prot_batch(dtype, (flags & PLFX_FMA) != 0, all + j, c, EV, wgt, n,
                                                 w->ws, ctx->max_blocks, s, tips, tipvec);
      if (e != hipSuccess) return hip_fail(ctx, e, "plf_prot batch launch");
      if (launches) ++*launches;
    }
    return PLFX_OK;
  }
  if (states == 20) {  // protein, one node: one full-GPU launch (plf_prot.hpp)
    const plfx_node &d = nodes[0];
    plfx::DnaArgs a{d.x1, d.x2, d.x3, EV, d.left, d.right, wgt, d.scaler, d.scaler_sum, w->ws, n};
    hipError_t e = plfx::launch_plf_prot(dtype, (flags & PLFX_FMA) != 0, a, ctx->max_blocks, s, tips,
                                         tipvec);
    if (e != hipSuccess) return hip_fail(ctx, e, "plf_prot launch");
    if (launches) ++*launches;
    return PLFX_OK;
  }
  // More than kMaxBatch nodes: launch j takes nodes j, j + L, j + 2L, ... (L
  // launches), so every launch mixes nodes from across the caller's list.
  // Consecutive nodes are usually consecutive allocations, and a launch made of
  // 32 neighbouring allocations of 128 MiB ran up to 15 % slower than a mixed
  // one while each of its nodes alone ran at the same speed (nodes512 at N = 1:
  // launches of 2.09-2.48 ms consecutive, 2.10-2.12 ms interleaved;
  // tools/probes/nodes_groups.py, nodes_sched.py, HISTORY.md section 5).
  const int L = (count + plfx::kMaxBatch - 1) / plfx::kMaxBatch;
  const plfx::NodeDescH *all = reinterpret_cast<const plfx::NodeDescH *>(nodes);
  for (int j = 0; j < L; j++) {
    plfx::NodeDescH sel[plfx::kMaxBatch];
    int c = 0;
    for (int i = j; i < count; i += L) sel[c++] = all[i];
    hipError_t e = plfx::launch_plf_dna_batch(dtype, L == 1 ? all : sel, c, EV, wgt, n, w->ws,
                                              ctx->max_blocks, s, tips, tipvec, streams);
    if (e != hipSuccess) return hip_fail(ctx, e, "plf batch launch");
    if (launches) ++*launches;
  }
  return PLFX_OK;
}

}  // namespace

extern "C" {

int plfx_get_version(void) { return PLFX_VERSION; }

int plfx_ctx_create(int device, plfx_ctx **out) { return plfx_ctx_create_ex(device, 0u, out); }

int plfx_ctx_create_ex(int device, unsigned flags, plfx_ctx **out) {
  if (!out) return PLFX_ERR_INVALID;
  if (flags & ~(unsigned)PLFX_CTX_LAZY_TABLES) return PLFX_ERR_INVALID;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return PLFX_ERR_NODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return PLFX_ERR_NODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return PLFX_ERR_NODEV;
  plfx_ctx *ctx = new (std::nothrow) plfx_ctx();
  if (!ctx) return PLFX_ERR_NOMEM;
  ctx->device = device;
  ctx->lazy_tables = (flags & PLFX_CTX_LAZY_TABLES) != 0;
  DeviceGuard guard(device);  // the caller's current device is restored on return
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return PLFX_ERR_HIP;
  }
  // Grid cap: 0 = as many blocks as are co-resident (occupancy x CUs);
  // PLFX_MAX_BLOCKS overrides it for experiments.
  if (const char *env = std::getenv("PLFX_MAX_BLOCKS")) {
    int v = std::atoi(env);
    if (v > 0) ctx->max_blocks = v;
  }
  if (const char *env = std::getenv("PLFX_FUSE")) ctx->fuse = std::atoi(env);
  // PLFX_NODE_SEGMENTS: "1" on, "0" off, "-1" / "auto" / unset by size; any
  // other value is refused (a typo must not silently switch the mapping)
  if (const char *env = std::getenv("PLFX_NODE_SEGMENTS")) {
    if (!std::strcmp(env, "1")) ctx->node_segments = 1;
    else if (!std::strcmp(env, "0")) ctx->node_segments = 0;
    else if (!std::strcmp(env, "-1") || !std::strcmp(env, "auto") || !*env) ctx->node_segments = -1;
    else {
      (void)hipStreamDestroy(ctx->stream);
      delete ctx;
      return PLFX_ERR_INVALID;
    }
  }
  // PLFX_STREAMS: one-node calls kept in flight, "1".."8" (PLFX_STREAMS_MAX), empty
  // = 1; anything else is refused like PLFX_NODE_SEGMENTS
  const char *streams_env = std::getenv("PLFX_STREAMS");
  if (streams_env && *streams_env) {
    const char *env = streams_env;
    static_assert(PLFX_STREAMS_MAX <= 9, "PLFX_STREAMS is parsed as one digit");
    const int v = (env[0] >= '1' && env[0] <= '0' + PLFX_STREAMS_MAX && !env[1]) ? env[0] - '0' : 0;
    if (!v) {
      (void)hipStreamDestroy(ctx->stream);
      delete ctx;
      return PLFX_ERR_INVALID;
    }
    ctx->streams = v;
  }
  // the workspace pool: kWsPool entries (reduction words zeroed before return,
  // tip/tip tables), and the tables' constant code arrays
  auto undo = [&](int code) {
    for (void *b : ctx->ws_blocks) (void)hipFreeAsync(b, ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return code;
  };
  void *pool = nullptr, *tabs = nullptr, *codes = nullptr;
  if (hipMallocAsync(&pool, kWsPool * kWsEntryBytes, ctx->stream) != hipSuccess) return undo(PLFX_ERR_NOMEM);
  ctx->ws_blocks.push_back(pool);
  if (!ctx->lazy_tables) {
    if (hipMallocAsync(&tabs, kWsPool * kTtEntryBytes, ctx->stream) != hipSuccess) return undo(PLFX_ERR_NOMEM);
    ctx->ws_blocks.push_back(tabs);
  }
  if (hipMallocAsync(&codes, kTtCodeBytes, ctx->stream) != hipSuccess) return undo(PLFX_ERR_NOMEM);
  ctx->ws_blocks.push_back(codes);
  uint8_t cc[kTtCodeBytes] = {};
  for (int k = 0; k < plfx::kProtCombos; k++) {
    cc[k] = (uint8_t)(k / 24);
    cc[1024 + k] = (uint8_t)(k % 24);
  }
  if (hipMemsetAsync(pool, 0, kWsPool * kWsEntryBytes, ctx->stream) != hipSuccess ||
      hipMemcpyAsync(codes, cc, kTtCodeBytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return undo(PLFX_ERR_HIP);
  ctx->tt_codes = static_cast<uint8_t *>(codes);
  for (int i = 0; i < kWsPool; i++) {
    StreamWs w;
    ws_carve(w, static_cast<char *>(pool) + i * kWsEntryBytes,
             tabs ? static_cast<char *>(tabs) + i * kTtEntryBytes : nullptr);
    ctx->wss.push_back(w);
  }
  {
    std::lock_guard<std::mutex> l(g_live_mu);
    g_live.push_back(ctx);
  }
  *out = ctx;
  return PLFX_OK;
}

int plfx_ctx_destroy(plfx_ctx *ctx) {
  if (!ctx) return PLFX_OK;
  {
    // no exiting thread may retire entries of this context from here on
    std::lock_guard<std::mutex> l(g_live_mu);
    g_live.erase(std::remove(g_live.begin(), g_live.end(), ctx), g_live.end());
  }
  {
    DeviceGuard guard(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    // the staging buffer's last downloads run on d2h_stream: done before the
    // free.  All device memory of the context is stream-ordered
    // (hipMallocAsync): freed on its stream below, since hipFree would wait for
    // the whole device
    if (ctx->d2h_stream) {
      (void)hipStreamSynchronize(ctx->d2h_stream);
      (void)hipStreamDestroy(ctx->d2h_stream);
    }
    if (ctx->d_buf) (void)hipFreeAsync(ctx->d_buf, ctx->stream);
    for (hipEvent_t e : ctx->chunk_done)
      if (e) (void)hipEventDestroy(e);
    // Workspace entries still held by a stream other than the context's:
    // their last launches must be done before the free.  The caller's stream
    // handle is never used here -- the stream may already be destroyed (e.g.
    // a context collected after its user's streams) -- so the device is
    // waited for; releasing streams (plfx_ctx_release_stream) before destroy
    // avoids that wait.  An entry used under a capture needs it anyway (its
    // graph may still be replaying on any stream).
    bool device_wide = false;
    for (StreamWs &w : ctx->wss)
      if (w.in_use && (w.captured || w.retired || w.stream != ctx->stream)) device_wide = true;
    if (device_wide) (void)hipDeviceSynchronize();
    for (void *b : ctx->ws_blocks) (void)hipFreeAsync(b, ctx->stream);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
  return PLFX_OK;
}

// A copy taken under the context's lock, so another thread's failure cannot
// free the string under the caller; valid until this thread's next call.
const char *plfx_last_error(const plfx_ctx *ctx) {
  if (!ctx) return "null context";
  thread_local std::string copy;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  copy = ctx->err;
  return copy.c_str();
}

void *plfx_ctx_stream(plfx_ctx *ctx) { return ctx ? reinterpret_cast<void *>(ctx->stream) : nullptr; }

int plfx_ctx_device(const plfx_ctx *ctx) { return ctx ? ctx->device : -1; }

int plfx_ctx_synchronize(plfx_ctx *ctx) {
  PLFX_BIND(ctx);
  PLFX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return PLFX_OK;
}

int plfx_ctx_release_stream(plfx_ctx *ctx, void *stream) {
  PLFX_BIND(ctx);
  hipStream_t s = pick(ctx, stream);
  StreamWs *w = ws_find(ctx, s);
  if (!w) return PLFX_OK;  // no workspace held: nothing to release
  if (capturing(s))  // a wait on a capturing stream would invalidate the capture
    return fail(ctx, PLFX_ERR_INVALID, "stream is being captured: release it after the capture ends");
  // the stream's last sum-producing launch must be done before another stream
  // may take the entry (it is zero again once that launch has finished)
  PLFX_HIP(ctx, hipStreamSynchronize(s));
  // a graph captured through the entry keeps using its words (sum tickets,
  // queue heads, tip/tip tables): retired, never handed to another stream
  if (w->captured) w->retired = true;
  else w->in_use = false;
  w->stream = nullptr;
  w->tid = std::thread::id();
  return PLFX_OK;
}

int plfx_ctx_set_streams(plfx_ctx *ctx, int streams) {
  if (!ctx) return PLFX_ERR_INVALID;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  if (streams < 1 || streams > PLFX_STREAMS_MAX)
    return fail(ctx, PLFX_ERR_INVALID, "streams %d not in 1..%d", streams, PLFX_STREAMS_MAX);
  ctx->streams = streams;
  return PLFX_OK;
}

int plfx_ctx_streams(const plfx_ctx *ctx) {
  if (!ctx) return PLFX_ERR_INVALID;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  return ctx->streams;
}

int plfx_plf_f32(plfx_ctx *ctx, const float *x1, const float *x2, float *x3, const float *EV, int n,
                 const float *left, const float *right, const int *wgt, int *scalerIncrement) {
  PLFX_BIND(ctx);
  return plf_host<float>(ctx, x1, x2, x3, EV, n, left, right, wgt, scalerIncrement);
}

int plfx_plf_f64(plfx_ctx *ctx, const double *x1, const double *x2, double *x3, const double *EV,
                 int n, const double *left, const double *right, const int *wgt,
                 int *scalerIncrement) {
  PLFX_BIND(ctx);
  return plf_host<double>(ctx, x1, x2, x3, EV, n, left, right, wgt, scalerIncrement);
}

int plfx_plf_dev_f32(plfx_ctx *ctx, const float *x1, const float *x2, float *x3, const float *EV,
                     int64_t n, const float *left, const float *right, const int32_t *wgt,
                     uint8_t *scaler, int64_t *scaler_sum, void *stream) {
  PLFX_BIND(ctx);
  return plf_dev<float>(ctx, x1, x2, x3, EV, n, left, right, wgt, scaler, scaler_sum, stream);
}

int plfx_plf_dev_f64(plfx_ctx *ctx, const double *x1, const double *x2, double *x3,
                     const double *EV, int64_t n, const double *left, const double *right,
                     const int32_t *wgt, uint8_t *scaler, int64_t *scaler_sum, void *stream) {
  PLFX_BIND(ctx);
  return plf_dev<double>(ctx, x1, x2, x3, EV, n, left, right, wgt, scaler, scaler_sum, stream);
}

int plfx_plf_dev_gen(plfx_ctx *ctx, int dtype, int states, int flags, const void *x1,
                     const void *x2, void *x3, const void *EV, int64_t n, const void *left,
                     const void *right, const int32_t *wgt, uint8_t *scaler,
                     int64_t *scaler_sum, void *stream) {
  PLFX_BIND(ctx);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (flags & ~(PLFX_FMA | PLFX_VALU)) return fail(ctx, PLFX_ERR_INVALID, "bad flags %d", flags);
  const bool valu = (flags & PLFX_VALU) != 0;
  if (valu && (states != 20 || dtype != PLFX_F64))
    return fail(ctx, PLFX_ERR_INVALID, "PLFX_VALU: protein (states 20), f64 only");
  if (states == 4) {
    return dtype == PLFX_F32
               ? plf_dev<float>(ctx, (const float *)x1, (const float *)x2, (float *)x3,
                                (const float *)EV, n, (const float *)left, (const float *)right,
                                wgt, scaler, scaler_sum, stream)
               : plf_dev<double>(ctx, (const double *)x1, (const double *)x2, (double *)x3,
                                 (const double *)EV, n, (const double *)left,
                                 (const double *)right, wgt, scaler, scaler_sum, stream);
  }
  if (states != 20) return fail(ctx, PLFX_ERR_UNSUPPORTED, "states=%d not built (4, 20)", states);
  int rc = check_dev_args(ctx, x1, x2, x3, EV, n, left, right,
                          (size_t)n * 80 * (dtype == PLFX_F32 ? 4 : 8));
  if (rc != PLFX_OK) return rc;
  hipStream_t s = pick(ctx, stream);
  if (n == 0) {
    if (scaler_sum) PLFX_HIP(ctx, hipMemsetAsync(scaler_sum, 0, sizeof(int64_t), s));
    return PLFX_OK;
  }
  PLFX_WS(ctx, s, w);
  plfx::DnaArgs a{x1, x2, x3, EV, left, right, wgt, scaler, scaler_sum, w->ws, n};
  a.streams = ctx->streams;
  // f64 exact: the scalar-operand kernel (plf_prot_valu_exact.hip, 3 waves per
  // SIMD; +10 % over the LDS-matrix kernel, same bits) with or without PLFX_VALU
  const bool fma = (flags & PLFX_FMA) != 0;
  hipError_t e = dtype == PLFX_F64 && !fma ? plfx::launch_plf_prot_valu_exact_f64(a, ctx->max_blocks, s)
                 : valu                    ? plfx::launch_plf_prot_valu_f64(a, ctx->max_blocks, s)
                                           : plfx::launch_plf_prot(dtype, fma, a, ctx->max_blocks, s);
  if (e != hipSuccess) return hip_fail(ctx, e, valu ? "plf_prot_valu launch" : "plf_prot launch");
  return PLFX_OK;
}

int plfx_instance_run(plfx_ctx *ctx, const void *in_left, const void *in_right, void *out_clv,
                      uint8_t *out_scaler, uint32_t alignment_sites, uint32_t window_size,
                      int layout, int dtype, void *stream) {
  PLFX_BIND(ctx);
  if (layout != PLFX_LAYOUT_COMBINED && layout != PLFX_LAYOUT_SEPARATE)
    return fail(ctx, PLFX_ERR_INVALID, "bad layout %d", layout);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (window_size % 16 != 0) return fail(ctx, PLFX_ERR_INVALID, "window_size %u not a multiple of 16", window_size);
  if (!in_left || !in_right) return fail(ctx, PLFX_ERR_INVALID, "null instance buffer");
  // Header words: in_left = [EV | P_L] (mm2sleft reads mem[0], mem[1..4]);
  // in_right = [EV | P_R] (COMBINED, mem[1..4]) or [P_R] (SEPARATE, mem[0..3]).
  const size_t es = dtype == PLFX_F32 ? 4 : 8;
  const char *L = static_cast<const char *>(in_left);
  const char *R = static_cast<const char *>(in_right);
  const size_t rhdr = layout == PLFX_LAYOUT_COMBINED ? 80 : 64;
  const void *EV = L;
  const void *left = L + 16 * es;
  const void *x1 = L + 80 * es;
  const void *right = R + (rhdr - 64) * es;
  const void *x2 = R + rhdr * es;
  if (dtype == PLFX_F32)
    return plf_dev<float>(ctx, (const float *)x1, (const float *)x2, (float *)out_clv,
                          (const float *)EV, alignment_sites, (const float *)left,
                          (const float *)right, nullptr, out_scaler, nullptr, stream);
  return plf_dev<double>(ctx, (const double *)x1, (const double *)x2, (double *)out_clv,
                         (const double *)EV, alignment_sites, (const double *)left,
                         (const double *)right, nullptr, out_scaler, nullptr, stream);
}

int plfx_instance_run_host(plfx_ctx *ctx, const void *in_left, const void *in_right,
                           void *out_clv, uint8_t *out_scaler, uint32_t alignment_sites,
                           uint32_t window_size, int layout, int dtype) {
  PLFX_BIND(ctx);
  if (layout != PLFX_LAYOUT_COMBINED && layout != PLFX_LAYOUT_SEPARATE)
    return fail(ctx, PLFX_ERR_INVALID, "bad layout %d", layout);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (!in_left || !in_right || (alignment_sites > 0 && !out_clv))
    return fail(ctx, PLFX_ERR_INVALID, "null instance buffer");
  const size_t es = dtype == PLFX_F32 ? 4 : 8, n = alignment_sites;
  const size_t lbytes = (80 + 16 * n) * es;                                        // active prefix of in_left
  const size_t rbytes = ((layout == PLFX_LAYOUT_COMBINED ? 80 : 64) + 16 * n) * es;  // and of in_right
  const size_t obytes = 16 * n * es;
  const size_t o_l = 0, o_r = round_up(lbytes, 256), o_o = o_r + round_up(rbytes, 256);
  const size_t o_s = o_o + round_up(obytes, 256);
  int rc = ensure_dbuf(ctx, o_s + round_up(std::max<size_t>(n, 1), 256));
  if (rc != PLFX_OK) return rc;
  char *d = static_cast<char *>(ctx->d_buf);
  hipStream_t s = ctx->stream;
  PLFX_HIP(ctx, hipMemcpyAsync(d + o_l, in_left, lbytes, hipMemcpyHostToDevice, s));
  PLFX_HIP(ctx, hipMemcpyAsync(d + o_r, in_right, rbytes, hipMemcpyHostToDevice, s));
  rc = plfx_instance_run(ctx, d + o_l, d + o_r, d + o_o, out_scaler ? (uint8_t *)(d + o_s) : nullptr,
                         alignment_sites, window_size, layout, dtype, s);
  if (rc != PLFX_OK) return rc;
  if (n > 0) {
    PLFX_HIP(ctx, hipMemcpyAsync(out_clv, d + o_o, obytes, hipMemcpyDeviceToHost, s));
    if (out_scaler) PLFX_HIP(ctx, hipMemcpyAsync(out_scaler, d + o_s, n, hipMemcpyDeviceToHost, s));
  }
  PLFX_HIP(ctx, hipStreamSynchronize(s));
  return PLFX_OK;
}

int plfx_plf_batch_dev(plfx_ctx *ctx, int dtype, int states, const plfx_node *nodes, int count,
                       const void *EV, int64_t n, const int32_t *wgt, void *stream) {
  PLFX_BIND(ctx);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (states != 4 && states != 20)
    return fail(ctx, PLFX_ERR_UNSUPPORTED, "batched nodes: states=%d not built (4, 20)", states);
  // DNA batches share the resident grid with the batches of the other
  // streams in flight (plfx_ctx_set_streams)
  return batch_impl(ctx, dtype, nodes, count, EV, n, wgt, pick(ctx, stream), 0, nullptr, states,
                    PLFX_EXACT, nullptr, nullptr, nullptr, ctx->streams);
}

int plfx_plf_tips_dev_gen(plfx_ctx *ctx, int dtype, int states, int flags, const uint8_t *tip1,
                          const void *x1, const uint8_t *tip2, const void *x2, void *x3,
                          const void *EV, int64_t n, const void *left, const void *right,
                          const int32_t *wgt, uint8_t *scaler, int64_t *scaler_sum,
                          const void *tipvec, void *stream) {
  PLFX_BIND(ctx);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (states != 4 && states != 20)
    return fail(ctx, PLFX_ERR_UNSUPPORTED, "states=%d not built (4, 20)", states);
  if (flags & ~PLFX_FMA) return fail(ctx, PLFX_ERR_INVALID, "bad flags %d", flags);
  if ((tip1 != nullptr) == (x1 != nullptr) || (tip2 != nullptr) == (x2 != nullptr))
    return fail(ctx, PLFX_ERR_INVALID, "each child needs exactly one of tip / CLV");
  plfx_node nd{tip1 ? (const void *)tip1 : x1, tip2 ? (const void *)tip2 : x2, x3, left, right,
               scaler, scaler_sum};
  int tips = (tip1 ? 1 : 0) + (tip2 ? 1 : 0);
  if (!tip1 && tip2) {  // dense/tip runs as tip/dense: u1*u2 == u2*u1 exactly
    std::swap(nd.x1, nd.x2);
    std::swap(nd.left, nd.right);
  }
  return batch_impl(ctx, dtype, &nd, 1, EV, n, wgt, pick(ctx, stream), tips, tipvec, states, flags);
}

int plfx_plf_tips_dev(plfx_ctx *ctx, int dtype, const uint8_t *tip1, const void *x1,
                      const uint8_t *tip2, const void *x2, void *x3, const void *EV, int64_t n,
                      const void *left, const void *right, const int32_t *wgt, uint8_t *scaler,
                      int64_t *scaler_sum, const void *tipvec, void *stream) {
  return plfx_plf_tips_dev_gen(ctx, dtype, 4, PLFX_EXACT, tip1, x1, tip2, x2, x3, EV, n, left,
                               right, wgt, scaler, scaler_sum, tipvec, stream);
}

int plfx_traverse(plfx_ctx *ctx, int dtype, int states, const plfx_trav_op *ops, int nops,
                  void *const *clv, int nslots, const void *pmats, int npmats, const void *EV,
                  int64_t n, const int32_t *wgt, uint8_t *const *scalers, int64_t *scaler_sums,
                  void *stream) {
  return plfx_traverse_tips(ctx, dtype, states, PLFX_EXACT, ops, nops, clv, nullptr, nslots, pmats,
                            npmats, EV, n, wgt, scalers, scaler_sums, nullptr, stream);
}

int plfx_traverse_tips(plfx_ctx *ctx, int dtype, int states, int flags, const plfx_trav_op *ops,
                       int nops,
                       void *const *clv, const uint8_t *const *tips, int nslots, const void *pmats,
                       int npmats, const void *EV, int64_t n, const int32_t *wgt,
                       uint8_t *const *scalers, int64_t *scaler_sums, const void *tipvec,
                       void *stream) {
  PLFX_BIND(ctx);
  for (int &c : ctx->sched) c = 0;
  if (states != 4 && states != 20)
    return fail(ctx, PLFX_ERR_UNSUPPORTED, "traverse: states=%d not built (4, 20)", states);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (flags & ~PLFX_FMA) return fail(ctx, PLFX_ERR_INVALID, "bad flags %d", flags);
  if (nops < 0 || (nops > 0 && (!ops || !clv || !pmats || !EV)))
    return fail(ctx, PLFX_ERR_INVALID, "bad traverse arguments");
  const size_t es = dtype == PLFX_F32 ? 4 : 8;
  const size_t mat = (size_t)states * states * 4;  // C*S*S values per matrix
  const size_t cb = clv_bytes_of(dtype, states, n);
  auto is_tip = [&](int sl) { return tips && tips[sl]; };
  // dependency levels: RAW on children (cdep), WAR/WAW on the parent slot (pdep)
  std::vector<int> level(nops, 0), pdep(nops, 0), w1(nops, -1), w2(nops, -1);
  std::vector<int> slot_write(nslots, -1), slot_read(nslots, -1), last_writer(nslots, -1);
  int nlev = 0;
  for (int j = 0; j < nops; j++) {
    const plfx_trav_op &o = ops[j];
    if (o.parent < 0 || o.parent >= nslots || o.child1 < 0 || o.child1 >= nslots || o.child2 < 0 ||
        o.child2 >= nslots || o.pmat < 0 || o.pmat >= npmats)
      return fail(ctx, PLFX_ERR_INVALID, "op %d: slot/pmat index out of range", j);
    if (o.parent == o.child1 || o.parent == o.child2)
      return fail(ctx, PLFX_ERR_INVALID, "op %d: parent slot aliases a child", j);
    if (is_tip(o.parent)) return fail(ctx, PLFX_ERR_INVALID, "op %d: parent slot is a tip", j);
    int cdep = 0, pd = 0;
    for (int sl : {o.child1, o.child2})
      if (slot_write[sl] >= 0) cdep = std::max(cdep, slot_write[sl] + 1);
    if (slot_write[o.parent] >= 0) pd = std::max(pd, slot_write[o.parent] + 1);
    if (slot_read[o.parent] >= 0) pd = std::max(pd, slot_read[o.parent] + 1);
    const int lv = std::max(cdep, pd);
    level[j] = lv;
    pdep[j] = pd;
    w1[j] = last_writer[o.child1];
    w2[j] = last_writer[o.child2];
    slot_write[o.parent] = lv;
    last_writer[o.parent] = j;
    for (int sl : {o.child1, o.child2}) slot_read[sl] = std::max(slot_read[sl], lv);
    nlev = std::max(nlev, lv + 1);
  }
  hipStream_t s = pick(ctx, stream);
  unsigned long long *ws = nullptr;
  if (nops > 0 && n > 0) {
    PLFX_WS(ctx, s, w);
    ws = w->ws;
  }
  const char *pm = static_cast<const char *>(pmats);
  // the node descriptor of op j, tip child first (dense/tip runs as tip/dense:
  // the product u1*u2 commutes exactly); *kind = number of tip children
  auto node_of = [&](int j, int *kind) {
    const plfx_trav_op &o = ops[j];
    const bool t1 = is_tip(o.child1), t2 = is_tip(o.child2);
    plfx_node nd{t1 ? (const void *)tips[o.child1] : clv[o.child1],
                 t2 ? (const void *)tips[o.child2] : clv[o.child2], clv[o.parent],
                 pm + (size_t)(2 * o.pmat) * mat * es, pm + (size_t)(2 * o.pmat + 1) * mat * es,
                 scalers ? scalers[j] : nullptr, scaler_sums ? scaler_sums + j : nullptr};
    if (!t1 && t2) {
      std::swap(nd.x1, nd.x2);
      std::swap(nd.left, nd.right);
    }
    *kind = (t1 ? 1 : 0) + (t2 ? 1 : 0);
    return nd;
  };
  // Fused level pairs (DNA): op P whose two children were last written by
  // ops A, B of the level just below it, with the same tip kind, and whose own
  // slot is free by then (pdep <= level of A), runs with A and B in one pass
  // (plf_dna.hpp TripleDesc): A's and B's CLVs are written but not read back.
  struct Triple {
    int a, b, p, kind;
  };
  std::vector<Triple> triples;
  std::vector<char> used(nops, 0);
  // Fused three-level subtrees (DNA, plf_dna.hpp SeptetDesc): root R two
  // levels above four ops A of one tip kind, through the two ops B that R's
  // children were last written by; R's and the B's slots free by level L.
  // Ordered so that a[2i], a[2i+1] are b[i]'s child1, child2 and b[0], b[1]
  // are R's.  Tried first; the remaining ops form triples.
  struct Septet {
    int a[4], b[2], r, kind;
  };
  std::vector<Septet> septets;
  auto fusible_pair = [&](int p, int L, int &x, int &y) {  // p's writers at level L
    x = w1[p];
    y = w2[p];
    return x >= 0 && y >= 0 && x != y && !used[x] && !used[y] && !used[p] && level[x] == L &&
           level[y] == L && level[p] == L + 1;
  };
  // Fused deep subtrees (DNA, plf_dna.hpp DeepDesc): a complete binary
  // subtree of depth D = 6, 5 or 4 (2^D - 1 ops on consecutive levels
  // L..L+D-1), every op's own slot free by L (pdep <= L), all leaves dense
  // or all leaves tips.  Collected per level in heap
  // order (children left to right before parents): the ops of level k are
  // lv[k], and lv[k][i]'s children were written by lv[k-1][2i], lv[k-1][2i+1].
  // Tried before the three-level subtrees.
  struct Deep {
    std::vector<int> ops;  // the 2^D - 1 ops in DeepDesc node order
    int L, D, tips;        // tips: 0 dense leaves, 2 every leaf a tip
  };
  std::vector<Deep> deeps;
  std::function<bool(int, int, int, std::vector<int> *)> complete =
      [&](int r, int D, int L, std::vector<int> *lv) {
        if (r < 0 || used[r] || level[r] != L + D - 1 || pdep[r] > L) return false;
        if (D > 1 && (w1[r] < 0 || w2[r] < 0 || w1[r] == w2[r] ||
                      !complete(w1[r], D - 1, L, lv) || !complete(w2[r], D - 1, L, lv)))
          return false;
        lv[D - 1].push_back(r);
        return true;
      };
  if (ctx->fuse >= 3 && states == 4) {
    for (int D = 6; D >= 4; D--) {  // deepest first
      for (int r = 0; r < nops; r++) {
        if (level[r] < D - 1 || used[r]) continue;
        std::vector<int> lv[6];
        if (!complete(r, D, level[r] - (D - 1), lv)) continue;
        // every leaf dense, or every leaf a tip (the coded-leaf pass's
        // tables); mixed leaves stay with the three-level passes
        bool dense = true, coded = true;
        for (int j : lv[0]) {
          const bool t1 = is_tip(ops[j].child1), t2 = is_tip(ops[j].child2);
          dense = dense && !t1 && !t2;
          coded = coded && t1 && t2;
        }
        // nor may a deep pass take the top of a subtree whose lower levels are
        // still unfused (over coded leaves: the septets below it would become
        // level pairs and move more bytes in all)
        for (int j : lv[0])
          for (int wr : {w1[j], w2[j]})
            if (wr >= 0 && !used[wr] && level[wr] == level[r] - D) dense = coded = false;
        if (!dense && !coded) continue;
        Deep t{{}, level[r] - (D - 1), D, coded ? 2 : 0};
        for (int k = 0; k < D; k++) t.ops.insert(t.ops.end(), lv[k].begin(), lv[k].end());
        for (int j : t.ops) used[j] = 1;
        deeps.push_back(std::move(t));
      }
    }
  }
  if (ctx->fuse >= 2 && states == 4) {
    for (int r = 0; r < nops; r++) {
      Septet t{};
      t.r = r;
      const int L = level[r] - 2;
      if (L < 0 || used[r] || pdep[r] > L) continue;
      if (!fusible_pair(r, L + 1, t.b[0], t.b[1])) continue;
      if (pdep[t.b[0]] > L || pdep[t.b[1]] > L) continue;
      if (!fusible_pair(t.b[0], L, t.a[0], t.a[1]) || !fusible_pair(t.b[1], L, t.a[2], t.a[3]))
        continue;
      int k[4];
      for (int i = 0; i < 4; i++) node_of(t.a[i], &k[i]);
      if (k[1] != k[0] || k[2] != k[0] || k[3] != k[0]) continue;
      t.kind = k[0];
      for (int j : {t.a[0], t.a[1], t.a[2], t.a[3], t.b[0], t.b[1], r}) used[j] = 1;
      septets.push_back(t);
    }
  }
  if (ctx->fuse >= 1 && states == 4) {
    for (int p = 0; p < nops; p++) {
      const int a = w1[p], b = w2[p];
      if (a < 0 || b < 0 || a == b || used[a] || used[b] || used[p]) continue;
      const int L = level[a];
      if (level[b] != L || level[p] != L + 1 || pdep[p] > L) continue;
      int ka, kb;
      node_of(a, &ka);
      node_of(b, &kb);
      if (ka != kb) continue;
      used[a] = used[b] = used[p] = 1;
      triples.push_back({a, b, p, ka});
    }
  }
  // the schedule, as plfx_traverse_schedule reports it
  int sched[PLFX_SCHED_COUNTS] = {};
  for (const Deep &t : deeps) sched[6 - t.D]++;
  sched[3] = (int)septets.size();
  sched[4] = (int)triples.size();
  for (int j = 0; j < nops; j++) sched[5] += used[j] ? 0 : 1;
  std::vector<plfx_node> batch[3];  // by number of tip children
  std::vector<int> bop[3];           // the op index of each batch entry
  std::vector<plfx::TripleDescH> tb[3];
  std::vector<plfx::SeptetDescH> sb[3];
  // protein: the previous level's tip/tip nodes still in their
  // combination tables; a node of this level whose two children are among them
  // stages its child tiles from the tables (plf_prot.hpp kTab) instead of
  // reading the children's CLVs back from HBM.  Only for the next level: later
  // levels may overwrite the tables or the children's slots.
  std::vector<TabRef> prev_tabs, cur_tabs;
  const bool tab_mode = states == 20 && n > 0;
  for (int lv = 0; lv < nlev; lv++) {
    for (int k = 0; k < 3; k++) {
      batch[k].clear();
      bop[k].clear();
      tb[k].clear();
      sb[k].clear();
    }
    for (const Deep &t : deeps) {
      if (t.L != lv) continue;
      plfx::DeepDescH d{};
      const int nodes = (1 << t.D) - 1, leaf_ops = 1 << (t.D - 1);
      for (int q = 0; q < nodes; q++) {
        const int j = t.ops[q];
        const plfx_trav_op &o = ops[j];
        int kq;
        const int rc = check_node(ctx, node_of(j, &kq), kq, n, j, cb);
        if (rc != PLFX_OK) return rc;
        if (q < leaf_ops) {  // level 1: the leaves (CLVs or tip codes), child1 then child2
          d.g[2 * q] = t.tips ? (const void *)tips[o.child1] : clv[o.child1];
          d.g[2 * q + 1] = t.tips ? (const void *)tips[o.child2] : clv[o.child2];
        }
        d.x[q] = clv[o.parent];
        d.mat[2 * q] = pm + (size_t)(2 * o.pmat) * mat * es;
        d.mat[2 * q + 1] = pm + (size_t)(2 * o.pmat + 1) * mat * es;
        d.sc[q] = scalers ? scalers[j] : nullptr;
        d.ss[q] = scaler_sums ? scaler_sums + j : nullptr;
      }
      if (n == 0) {
        for (int64_t *ss : d.ss)
          if (ss) PLFX_HIP(ctx, hipMemsetAsync(ss, 0, sizeof(int64_t), s));
        continue;
      }
      hipError_t e = plfx::launch_plf_dna_deep(dtype, t.D, &d, EV, wgt, n, ws, ctx->max_blocks, s,
                                               t.tips, tipvec);
      if (e != hipSuccess) return hip_fail(ctx, e, "fused deep-subtree launch");
      sched[6]++;
    }
    for (const Septet &t : septets) {
      if (level[t.a[0]] != lv) continue;
      const int id[7] = {t.a[0], t.a[1], t.a[2], t.a[3], t.b[0], t.b[1], t.r};
      plfx::SeptetDescH d{};
      for (int q = 0; q < 7; q++) {
        int kq;
        const plfx_node nd = node_of(id[q], &kq);
        const int rc = check_node(ctx, nd, kq, n, id[q], cb);
        if (rc != PLFX_OK) return rc;
        if (q < 4) {
          d.g[2 * q] = nd.x1;
          d.g[2 * q + 1] = nd.x2;
        }
        d.x[q] = nd.x3;
        d.mat[2 * q] = nd.left;
        d.mat[2 * q + 1] = nd.right;
        d.sc[q] = nd.scaler;
        d.ss[q] = nd.scaler_sum;
      }
      sb[t.kind].push_back(d);
    }
    for (const Triple &t : triples) {
      if (level[t.a] != lv) continue;
      int ka, kb, kp;
      const plfx_node A = node_of(t.a, &ka), B = node_of(t.b, &kb), P = node_of(t.p, &kp);
      for (int rc : {check_node(ctx, A, ka, n, t.a, cb), check_node(ctx, B, kb, n, t.b, cb),
                     check_node(ctx, P, kp, n, t.p, cb)})
        if (rc != PLFX_OK) return rc;
      // P's children as op P names them: child1 = A's slot or B's slot
      const bool a_first = ops[t.p].child1 == ops[t.a].parent;
      const plfx_node &F = a_first ? A : B, &G = a_first ? B : A;
      tb[t.kind].push_back(plfx::TripleDescH{
          F.x1, F.x2, G.x1, G.x2, F.x3, G.x3, P.x3, (const double *)F.left,
          (const double *)F.right, (const double *)G.left, (const double *)G.right,
          (const double *)P.left, (const double *)P.right, F.scaler, G.scaler, P.scaler,
          F.scaler_sum, G.scaler_sum, P.scaler_sum});
    }
    for (int j = 0; j < nops; j++) {
      if (level[j] != lv || used[j]) continue;
      int kind;
      const plfx_node nd = node_of(j, &kind);
      batch[kind].push_back(nd);
      bop[kind].push_back(j);
    }
    for (int k = 0; k < 3; k++) {
      for (size_t i = 0; i < sb[k].size(); i += plfx::kMaxSeptets) {
        const int c = (int)std::min<size_t>(plfx::kMaxSeptets, sb[k].size() - i);
        if (n == 0) {
          for (int q = 0; q < c; q++)
            for (int64_t *ss : sb[k][i + q].ss)
              if (ss) PLFX_HIP(ctx, hipMemsetAsync(ss, 0, sizeof(int64_t), s));
          continue;
        }
        hipError_t e = plfx::launch_plf_dna_septets(dtype, sb[k].data() + i, c, EV, wgt, n,
                                                    ws, ctx->max_blocks, s, k, tipvec);
        if (e != hipSuccess) return hip_fail(ctx, e, "fused three-level launch");
        sched[6]++;
      }
      for (size_t i = 0; i < tb[k].size(); i += plfx::kMaxTriples) {
        const int c = (int)std::min<size_t>(plfx::kMaxTriples, tb[k].size() - i);
        if (n == 0) {
          for (int q = 0; q < c; q++)
            for (int64_t *ss : {tb[k][i + q].ssa, tb[k][i + q].ssb, tb[k][i + q].ssp})
              if (ss) PLFX_HIP(ctx, hipMemsetAsync(ss, 0, sizeof(int64_t), s));
          continue;
        }
        hipError_t e = plfx::launch_plf_dna_triples(dtype, tb[k].data() + i, c, EV, wgt, n, ws,
                                                    ctx->max_blocks, s, k, tipvec);
        if (e != hipSuccess) return hip_fail(ctx, e, "fused level-pair launch");
        sched[6]++;
      }
      if (k == 0 && tab_mode && !prev_tabs.empty() && !batch[0].empty()) {
        auto find = [&](const void *x) -> const TabRef * {
          for (const TabRef &t : prev_tabs)
            if (t.x3 == x) return &t;
          return nullptr;
        };
        std::vector<plfx::ProtTabDescH> tab;
        std::vector<plfx_node> rest;
        std::vector<int> rest_op;
        for (size_t q = 0; q < batch[0].size(); q++) {
          const plfx_node &nd = batch[0][q];
          const TabRef *a = find(nd.x1), *b = find(nd.x2);
          if (!a || !b) {
            rest.push_back(nd);
            rest_op.push_back(bop[0][q]);
            continue;
          }
          // these nodes do not go through batch_impl's checks: checked here
          const int rc = check_node(ctx, nd, 0, n, bop[0][q], cb);
          if (rc != PLFX_OK) return rc;
          tab.push_back(plfx::ProtTabDescH{a->tab, b->tab, a->ca, a->cb, b->ca, b->cb, nd.x3, nd.left,
                                           nd.right, nd.scaler, nd.scaler_sum});
        }
        for (size_t i = 0; i < tab.size(); i += plfx::kMaxBatch) {
          const int c = (int)std::min<size_t>(plfx::kMaxBatch, tab.size() - i);
          hipError_t e = plfx::launch_prot_tab_batch(dtype, (flags & PLFX_FMA) != 0, tab.data() + i, c, EV,
                                                     wgt, n, ws, ctx->max_blocks, s);
          if (e != hipSuccess) return hip_fail(ctx, e, "plf_prot table-children launch");
          sched[6]++;
        }
        batch[0].swap(rest);
        bop[0].swap(rest_op);
      }
      if (batch[k].empty()) continue;
      int rc = batch_impl(ctx, dtype, batch[k].data(), (int)batch[k].size(), EV, n, wgt, s, k,
                          tipvec, states, flags, &sched[6], k == 2 && tab_mode ? &cur_tabs : nullptr,
                          bop[k].data());
      if (rc != PLFX_OK) return rc;
    }
    prev_tabs.swap(cur_tabs);
    cur_tabs.clear();
  }
  for (int i = 0; i < PLFX_SCHED_COUNTS; i++) ctx->sched[i] = sched[i];
  return PLFX_OK;
}

int plfx_traverse_schedule(const plfx_ctx *ctx, int *counts, int ncounts) {
  if (!ctx || (ncounts > 0 && !counts)) return 0;
  std::lock_guard<std::recursive_mutex> lock(ctx->mu);
  const int m = std::min(ncounts, PLFX_SCHED_COUNTS);
  for (int i = 0; i < m; i++) counts[i] = ctx->sched[i];
  return m < 0 ? 0 : m;
}

int plfx_root_lnl(plfx_ctx *ctx, int dtype, int states, const void *x, int64_t n,
                  const double *catw, const double *freq, const int32_t *wgt,
                  const int64_t *scaler_sums, int nsums, double *out_lnl, double *site_lnl,
                  void *stream) {
  PLFX_BIND(ctx);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (states != 4 && states != 20) return fail(ctx, PLFX_ERR_UNSUPPORTED, "lnl: states=%d", states);
  if (!out_lnl || n < 0 || (n > 0 && !x) || nsums < 0 || (nsums > 0 && !scaler_sums))
    return fail(ctx, PLFX_ERR_INVALID, "bad root_lnl arguments");
  hipStream_t s = pick(ctx, stream);
  if (n == 0) {
    PLFX_HIP(ctx, hipMemsetAsync(out_lnl, 0, sizeof(double), s));
    if (nsums == 0) return PLFX_OK;
  }
  PLFX_WS(ctx, s, w);
  hipError_t e = plfx::launch_root_lnl(dtype, states, x, n, catw, freq, wgt, scaler_sums, nsums,
                                       w->lnl_partials, w->lnl_ticket, out_lnl, site_lnl, s);
  if (e != hipSuccess) return hip_fail(ctx, e, "root_lnl launch");
  return PLFX_OK;
}

int plfx_scaler_sum(plfx_ctx *ctx, const uint8_t *scaler, const int32_t *wgt, int64_t n,
                    int64_t *out_sum, void *stream) {
  PLFX_BIND(ctx);
  if (!out_sum || n < 0 || (n > 0 && !scaler)) return fail(ctx, PLFX_ERR_INVALID, "bad scaler_sum args");
  hipStream_t s = pick(ctx, stream);
  if (n == 0) {
    PLFX_HIP(ctx, hipMemsetAsync(out_sum, 0, sizeof(int64_t), s));
    return PLFX_OK;
  }
  PLFX_WS(ctx, s, w);
  hipError_t e = plfx::launch_scaler_sum(scaler, wgt, n, out_sum, w->ws, ctx->max_blocks, s);
  if (e != hipSuccess) return hip_fail(ctx, e, "scaler_sum launch");
  return PLFX_OK;
}

int plfx_pmatrix(plfx_ctx *ctx, int dtype, int states, int convention, const double *eigen,
                 const double *rates, int ncat, const double *blen, int64_t nbranch, void *pmats,
                 void *stream) {
  PLFX_BIND(ctx);
  if (dtype != PLFX_F32 && dtype != PLFX_F64) return fail(ctx, PLFX_ERR_INVALID, "bad dtype %d", dtype);
  if (convention != PLFX_PMAT_STATE && convention != PLFX_PMAT_EIGEN)
    return fail(ctx, PLFX_ERR_INVALID, "bad convention %d", convention);
  if (states < 2 || states > 64 || ncat < 1 || nbranch < 0)
    return fail(ctx, PLFX_ERR_INVALID, "bad pmatrix sizes (states %d, ncat %d)", states, ncat);
  if (nbranch == 0) return PLFX_OK;
  if (!eigen || !rates || !blen || !pmats) return fail(ctx, PLFX_ERR_INVALID, "null pmatrix pointer");
  hipError_t e = plfx::launch_pmatrix(dtype, convention == PLFX_PMAT_EIGEN, eigen, states, rates,
                                      ncat, blen, nbranch, pmats, pick(ctx, stream));
  if (e != hipSuccess) return hip_fail(ctx, e, "pmatrix launch");
  return PLFX_OK;
}

}  // extern "C"
