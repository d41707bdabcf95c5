/*
 * plfx.h -- C ABI of the MI355X-native PLF engine (libplfx.so).
 *
 * This is the drop-in boundary.  It replaces the two interfaces through which
 * the reference drives its PLF hot path:
 *
 *   (1) the CPU entry point  void plf(float* x1_start, float* x2_start,
 *       float* x3_start, float* EV, const int n, float* left, float* right,
 *       int* wgt, int& scalerIncrement)
 *       -- /root/reference/app/src/plf.h:1-5, defined app/src/plf.cpp:8-68,
 *       called from app/src/host_mem.cpp:418;
 *   (2) the XRT accelerator contract of app/src/host_mem.cpp:108-157,283-394:
 *       per instance an `in_left` bo = [EV16 | P_L64 | CLV_L], an `in_right`
 *       bo = [EV16 | P_R64 | CLV_R] (COMBINED) or [P_R64 | CLV_R] (SEPARATE),
 *       an `out` bo (CLV) and an `out_scaler` bo (char per site), with kernel
 *       arguments mm2sleft/mm2sright(mem, alignment_sites, window_size)
 *       (hls/src/mm2sleft_memDNAwindowComb.cpp:16) and
 *       s2mm(mem, scalerIncrement, alignment_sites, window_size)
 *       (hls/src/s2mm_memDNAwindowComb.cpp:20), and the host-side scaler
 *       reduction sum_j scaler[j]*wgt[j] (host_mem.cpp:384-388).
 *
 * Data layout (identical to the reference): a site is S*C values stored
 * site-major as x[site*16 + cat*4 + state] for DNA (4 Gamma categories x 4
 * states, plf.cpp:21-23); P matrices are left[cat*16 + k*4 + l] (row-major
 * P_c, plf.cpp:37-38); EV is EV[k*4 + l] (plf.cpp:47).
 *
 * Semantics (plf.cpp:19-65): for every site and category
 *   ump_L[k] = sum_l x1[c*4+l]*left[c*16+k*4+l]   (same for right/x2)
 *   x3[c*4+l] = sum_k (ump_L[k]*ump_R[k]) * EV[4k+l]
 * then if every |x3| of the site is < 2^-32 (strict; NaN never scales), all
 * values of the site are multiplied by 2^32, the per-site scaler byte is 1
 * and wgt[site] is added to the scaler increment.  Arithmetic is IEEE with
 * no FMA contraction and the reference's accumulation order, so the f32
 * entry points reproduce the reference bit-for-bit and f64 reproduces the
 * double instantiation of the same loop bit-for-bit.
 *
 * All functions return PLFX_OK (0) or a negative plfx_status; they never
 * throw.  plfx_last_error() gives a message for the last failure on a
 * context.  `stream` arguments are hipStream_t values passed as void* (NULL =
 * the HIP null stream, as everywhere in HIP; plfx_ctx_stream() gives the
 * context's own non-blocking stream).  Device pointers must come from the same HIP
 * device as the context; CLV pointers must be 16-byte aligned.  Every entry
 * point binds the context's device for its duration and restores the
 * caller's current device on return.  Calls on one context from several host
 * threads are serialised by the context (one lock per context, held for the
 * call: host entry points block other threads' calls for their duration;
 * device entry points only for the launch); distinct contexts are independent.
 * plfx_last_error() reports the last failure on the context, whichever thread
 * made it; the string is the calling thread's copy, valid until that thread
 * calls plfx_last_error() again.
 *
 * Streams and the scaler-sum workspace.  Sum-producing launches (scaler_sum
 * outputs, plfx_scaler_sum, plfx_root_lnl) reduce across thread blocks through
 * a small self-resetting device workspace.  The context keeps ONE workspace
 * PER STREAM in use (up to PLFX_MAX_STREAMS at a time), so launches on
 * different streams may run concurrently; launches on one stream are ordered
 * by the stream.  hipStreamPerThread names a different stream in every host
 * thread and gets a workspace per thread.  The first PLFX_WS_POOL streams take
 * workspaces allocated with the context, so their first use may be inside a
 * graph capture; a further stream's first sum-producing use allocates (not
 * inside hipStreamBeginCapture: issue one call on it before capturing).
 * plfx_ctx_release_stream() waits for a stream and returns its workspace to
 * the pool -- call it before destroying a stream used with the context, or
 * when rotating through many streams (not while the stream is being captured:
 * PLFX_ERR_INVALID).  A captured graph keeps the workspace of the stream it
 * was captured on, so its replays must not overlap other work on that
 * workspace, and must not outlive the context; releasing such a stream retires
 * its workspace (no other stream is ever given it) instead of returning it to
 * the pool.  A hipStreamPerThread workspace whose thread exits without
 * releasing it is retired too, and reclaimed (after a device-wide wait, not
 * inside a capture) when the context runs out of workspaces.
 * plfx_ctx_destroy() waits for the context's stream; if a stream other than
 * the context's still holds a workspace, or one was used under a capture, it
 * waits for the whole device (hipDeviceSynchronize, which must not overlap a
 * global-mode capture in another thread) -- it never uses a caller's stream
 * handle, which may already be destroyed.  Release streams before destroy
 * (plfx_ctx_release_stream) to keep destroy off the device-wide wait.  Graph
 * replays still in flight must finish before destroy.
 * The same workspace also holds the tile/chunk queues of the protein f64 FMA
 * kernel (from 2^20 sites) and of the fused six-level tree passes: blocks or
 * waves that run ahead take more of the alignment instead of a fixed share
 * (every site is computed the same way, so results do not change); the queue
 * words, like the sums, reset themselves at the end of each launch.
 * The reduction encodes arrival counts next to the sums and needs
 * sum_j |wgt[j]| < 2^40 per launch (the reference's own scalerIncrement is a
 * 32-bit int); the host entry points check this, the device entry points
 * cannot check it cheaply and leave it to the caller.
 *
 * No allocation happens per call after warm-up (the host entry points keep
 * grow-only staging buffers in the context).  Each workspace also holds the
 * protein tip/tip combination tables (about 11.8 MB; the pool's
 * PLFX_WS_POOL of them, ~95 MB, are allocated with the context).  A context
 * created with PLFX_CTX_LAZY_TABLES (DNA-only users) allocates a workspace's
 * tables on its first protein tip/tip call instead; that first call may then
 * not be inside a capture (PLFX_ERR_INVALID).
 * Every entry point rejects a parent CLV x3 that shares any byte with a child
 * it reads (PLFX_ERR_INVALID).
 *
 * Timing note: after an idle gap of ~0.3 s or more the MI355X lowers its
 * shader clock to ~1.8-2.0 GHz for the first ~10-15 ms of renewed load
 * (DVFS; measured in-kernel, HISTORY.md section 3.3).  HBM-bound calls (DNA)
 * run <= 4 % slower through it, the protein matrix-core kernels ~10 %.  It
 * is a property of the device's power management, not of a context or a
 * process, so no library-side warm-up can absorb it.
 */
#ifndef PLFX_H
#define PLFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLFX_VERSION 10300 /* 1.3.0 */
#define PLFX_MAX_STREAMS 64 /* streams holding a workspace at a time, per context */
#define PLFX_WS_POOL 8      /* workspaces allocated with the context */
#define PLFX_STREAMS_MAX 8  /* plfx_ctx_set_streams */

typedef enum {
  PLFX_OK = 0,
  PLFX_ERR_INVALID = -1,     /* bad argument (null pointer, size, alignment) */
  PLFX_ERR_HIP = -2,         /* HIP runtime failure; see plfx_last_error()   */
  PLFX_ERR_NOMEM = -3,       /* device allocation failed                      */
  PLFX_ERR_NODEV = -4,       /* no such HIP device / not a gfx950 device      */
  PLFX_ERR_UNSUPPORTED = -5  /* states/categories combination not built       */
} plfx_status;

/* Instance-buffer header layout: app/src/include.h:20 (COMBINED, SEPARATE). */
typedef enum { PLFX_LAYOUT_COMBINED = 0, PLFX_LAYOUT_SEPARATE = 1 } plfx_layout;
/* AIE transport of the reference: app/src/include.h:21 (STREAM, WINDOW).
 * Only affects buffer sizing (padding); the GPU needs neither. */
typedef enum { PLFX_AIE_STREAM = 0, PLFX_AIE_WINDOW = 1 } plfx_aie;
typedef enum { PLFX_F32 = 0, PLFX_F64 = 1 } plfx_dtype;

typedef struct plfx_ctx plfx_ctx;

/* ---- context ----------------------------------------------------------- */
/* Replaces acap_info (app/src/include.h:28-147): binds a HIP device and owns
 * a non-blocking stream, the scaler-sum workspace and host staging buffers. */
int plfx_ctx_create(int device, plfx_ctx **ctx);
/* flags: 0 (= plfx_ctx_create) or PLFX_CTX_LAZY_TABLES (see "Streams and the
 * scaler-sum workspace"); other bits are PLFX_ERR_INVALID. */
#define PLFX_CTX_LAZY_TABLES 1u
int plfx_ctx_create_ex(int device, unsigned flags, plfx_ctx **ctx);
int plfx_ctx_destroy(plfx_ctx *ctx);
const char *plfx_last_error(const plfx_ctx *ctx);
int plfx_get_version(void);
/* The context's stream (hipStream_t) and device ordinal. */
void *plfx_ctx_stream(plfx_ctx *ctx);
int plfx_ctx_device(const plfx_ctx *ctx);
/* Synchronise the context's stream. */
int plfx_ctx_synchronize(plfx_ctx *ctx);
/* Wait for `stream` (hipStream_t; NULL = the null stream; hipStreamPerThread =
 * the calling thread's) and return its scaler-sum workspace to the context's
 * pool.  PLFX_OK also when the stream holds none.  (Extension: the reference's
 * XRT queues are fixed per instance, host_mem.cpp:123-127.) */
int plfx_ctx_release_stream(plfx_ctx *ctx, void *stream);
/* One-node calls the caller keeps in flight at once, each on its own stream
 * (default 1; PLFX_STREAMS=1..8 in the environment at context creation,
 * empty = 1, anything else fails plfx_ctx_create with PLFX_ERR_INVALID).  The dense
 * one-node DNA kernels (plfx_plf_dev_f32 / _f64, plfx_plf_dev_gen with 4
 * states, and the host entries' chunks) and the protein FMA kernels
 * (plfx_plf_dev_gen, 20 states, PLFX_FMA; f32 rounds up to whole blocks per
 * CU) then launch the co-resident blocks / streams, and a DNA batch (plfx_plf_batch_dev) the share of them its
 * nodes would take / streams, so the calls in flight fill the GPU together and one call's
 * drain overlaps the others' work: 2^20-site f64 nodes alternating over two
 * streams run 0.80 of the HBM peak instead of 0.78 (0.75 one at a time),
 * f32 0.81 instead of 0.77.  Same bits for any value.
 * A call issued alone with streams > 1 runs on the smaller grid (0.64 for
 * the f64 node at 2): set it to what is actually in flight.  Other entry
 * points ignore it.  For many large nodes, one call per node over two streams
 * beats batches (512 nodes of 2^20 f64 sites: 0.793 vs 0.775 for 32-node
 * batches on two streams, 0.766 on one).  (Extension: the reference's instances run side by side,
 * app/src/include.h:181-195.)  set: PLFX_ERR_INVALID outside 1..8; get: the
 * value, or PLFX_ERR_INVALID for a null context. */
int plfx_ctx_set_streams(plfx_ctx *ctx, int streams);
int plfx_ctx_streams(const plfx_ctx *ctx);

/* ---- (1) drop-in for plf(): host arrays, synchronous -------------------- */
/* Same argument order and meaning as plf() (app/src/plf.h:1-5); `int&` is
 * `int*`.  Copies to the device, runs the fused kernel, copies back.
 * wgt may be NULL (= all ones). */
int plfx_plf_f32(plfx_ctx *ctx, const float *x1_start, const float *x2_start,
                 float *x3_start, const float *EV, int n, const float *left,
                 const float *right, const int *wgt, int *scalerIncrement);
int plfx_plf_f64(plfx_ctx *ctx, const double *x1_start, const double *x2_start,
                 double *x3_start, const double *EV, int n, const double *left,
                 const double *right, const int *wgt, int *scalerIncrement);

/* ---- (2) the hot path on device-resident CLVs, asynchronous ------------- */
/* All pointers are device pointers.  wgt, scaler (uint8 per site, the s2mm
 * char output) and scaler_sum (int64, = sum scaler*wgt, wgt NULL => 1) are
 * each optional (NULL = not produced / not read).  n may be 0.  From 2^25
 * sites (f32 and f64) the kernel deals the sites to the 8 XCDs as eight
 * contiguous segments instead of one grid-wide stride -- same bits, +1-29 %
 * HBM rate on long CLVs; env PLFX_NODE_SEGMENTS,
 * read at context creation: "1" forces the segments, "0" the one window,
 * "-1" / "auto" / "" keep the choice by size; any other value makes context
 * creation fail with PLFX_ERR_INVALID.  Segments need 8 blocks: under a grid
 * cap below 8 (PLFX_MAX_BLOCKS) the one window runs. */
int plfx_plf_dev_f32(plfx_ctx *ctx, const float *x1, const float *x2, float *x3,
                     const float *EV, int64_t n, const float *left,
                     const float *right, const int32_t *wgt, uint8_t *scaler,
                     int64_t *scaler_sum, void *stream);
int plfx_plf_dev_f64(plfx_ctx *ctx, const double *x1, const double *x2, double *x3,
                     const double *EV, int64_t n, const double *left,
                     const double *right, const int32_t *wgt, uint8_t *scaler,
                     int64_t *scaler_sum, void *stream);

/* ---- (2b) any state count (extension: BASELINE configs[4], protein) ------ */
/* states = 4 (DNA, the kernels above) or 20 (protein); 4 Gamma categories.
 * Layout generalises plf(): x[site*4S + cat*S + state], left/right
 * [cat][k][l] (S*S per category), EV[k][l] (S*S).  flags: PLFX_EXACT keeps
 * plf()'s separate multiply/add and operation order (bit-identical to the
 * double/float instantiation of the reference loop); PLFX_FMA fuses each
 * multiply-add (one rounding per term, within 1e-12 relative in f64; protein
 * only, on the matrix cores -- v_mfma_f64_16x16x4 / v_mfma_f32_16x16x4 are
 * k-ordered fma chains, so the result is bit-identical to a fused VALU loop;
 * DNA is always exact).  PLFX_FMA | PLFX_VALU (protein f64, plfx_plf_dev_gen
 * only): the same fused chains on the VALU, the P matrices as scalar operands
 * -- BASELINE configs[4]'s "matvec, not MFMA" -- bit-identical to PLFX_FMA.
 * Exact mode is always on the VALU (PLFX_VALU accepted, no effect). */
#define PLFX_EXACT 0
#define PLFX_FMA 1
#define PLFX_VALU 2
int plfx_plf_dev_gen(plfx_ctx *ctx, int dtype, int states, int flags, const void *x1,
                     const void *x2, void *x3, const void *EV, int64_t n, const void *left,
                     const void *right, const int32_t *wgt, uint8_t *scaler,
                     int64_t *scaler_sum, void *stream);

/* ---- (3) the accelerator instance-buffer contract ----------------------- */
/* in_left/in_right/out_clv/out_scaler: device buffers exactly as the
 * reference packs them (host_mem.cpp:221-243): in_left = [EV 16 | P_L 64 |
 * CLV_L], in_right = [EV 16 | P_R 64 | CLV_R] (COMBINED) or [P_R 64 | CLV_R]
 * (SEPARATE); element type `dtype`.  Writes alignment_sites CLVs to out_clv
 * and alignment_sites scaler bytes to out_scaler (never the window padding,
 * SURVEY Q4/Q5).  window_size (bytes of an AIE window, a multiple of 16; 0
 * for stream configs) is validated for sizing parity but not needed by the
 * kernel. */
int plfx_instance_run(plfx_ctx *ctx, const void *in_left, const void *in_right,
                      void *out_clv, uint8_t *out_scaler, uint32_t alignment_sites,
                      uint32_t window_size, int layout, int dtype, void *stream);

/* The same contract on HOST buffers, synchronous -- one accelerator instance
 * run as host_mem.cpp:293-318 drives it: write the active prefix of the two
 * input bos (bo.write(..., active bytes), :297-298), run the movers and the
 * graph (:305), read back alignment_sites CLVs and scaler bytes (:313-314).
 * The copies go through the context's device staging and stream; out_scaler
 * may be NULL.  Host buffers may be pageable or page-locked. */
int plfx_instance_run_host(plfx_ctx *ctx, const void *in_left, const void *in_right,
                           void *out_clv, uint8_t *out_scaler, uint32_t alignment_sites,
                           uint32_t window_size, int layout, int dtype);

/* ---- (4) scaler reduction (host_mem.cpp:384-388) on the device ---------- */
/* out_sum (device int64) = sum_j scaler[j] * (wgt ? wgt[j] : 1). */
int plfx_scaler_sum(plfx_ctx *ctx, const uint8_t *scaler, const int32_t *wgt,
                    int64_t n, int64_t *out_sum, void *stream);

/* ---- (6) many inner nodes per launch (extension: the reference evaluates
 * one node per call; BASELINE configs 3 and 4) -------------------------- */
/* One inner-node update: parent x3 from children x1, x2 with this node's P
 * matrices (left/right: C*S*S values, layout of plf.cpp:37-38).  scaler
 * (uint8 per site) and scaler_sum (int64) are optional per node. */
typedef struct {
  const void *x1, *x2;
  void *x3;
  const void *left, *right;
  uint8_t *scaler;
  int64_t *scaler_sum;
} plfx_node;

/* `count` independent nodes sharing EV, n and wgt; all device pointers, the
 * `nodes` array itself is host memory (it travels in the kernel arguments, 32
 * nodes per launch: graph-capture safe).  states 4 (DNA) or 20 (protein,
 * exact mode; up to 32 nodes per launch, node = blockIdx.y, each node with
 * its own scaler-sum workspace region). */
int plfx_plf_batch_dev(plfx_ctx *ctx, int dtype, int states, const plfx_node *nodes, int count,
                       const void *EV, int64_t n, const int32_t *wgt, void *stream);

/* A traversal descriptor (RAxML-style post-order list).  Op j computes CLV
 * slot `parent` from slots `child1`, `child2` with the P-matrix pair `pmat`:
 * left = pmats + (2*pmat)*C*S*S, right = pmats + (2*pmat+1)*C*S*S. */
typedef struct {
  int32_t parent, child1, child2, pmat;
} plfx_trav_op;

/* Executes `ops` in an order equivalent to the sequential one: ops are grouped
 * into dependency levels (an op waits for the ops that write its children and
 * for earlier readers/writers of its parent slot) and each level is issued as
 * batched launches.  clv: host array of `nslots` device CLV pointers;
 * scalers: host array of nops device uint8 pointers (or NULL / NULL entries);
 * scaler_sums: device int64[nops] (or NULL): entry j = op j's scalerIncrement. */
int plfx_traverse(plfx_ctx *ctx, int dtype, int states, const plfx_trav_op *ops, int nops,
                  void *const *clv, int nslots, const void *pmats, int npmats, const void *EV,
                  int64_t n, const int32_t *wgt, uint8_t *const *scalers, int64_t *scaler_sums,
                  void *stream);

/* ---- (8) tip children (extension) ---------------
 * A tip (leaf) is stored as one state code per site -- uint8, bit s set =
 * state s possible (A=1 C=2 G=4 T=8, ambiguity codes are unions, 15 = gap /
 * unknown; the upper nibble is ignored), the RAxML/PLL encoding -- instead of
 * a dense CLV of 16 values per site (16x/32x less traffic for that child).
 * Results are bit-identical to plf() on the expanded dense CLV
 * x[i][c][s] = (code_i >> s) & 1 for every category c.
 *
 * Protein (states = 20, plfx_plf_tips_dev_gen / plfx_traverse_tips): a code is
 * an index into a table of 24 dense rows of 20 values (codes >= 24 read row
 * 23); the default table (tipvec NULL), states in ARNDCQEGHILKMFPSTWYV order:
 * 0..19 one state, 20 = B (N|D), 21 = Z (Q|E), 22 = X, 23 = gap (all states);
 * tipvec = a device table of 24 x 20 values of dtype replaces it.  Exact and
 * FMA modes as plfx_plf_dev_gen, bit-identical to the dense computation on
 * x[i][c][s] = tv[code_i][s] in that mode. */

/* tipvec: NULL, or a device table of 16 x 4 values of dtype -- the dense
 * per-category CLV entry of each code, tipvec[code*4 + s] (the default is the
 * 0/1 state indicator; plfx_model_tip_vectors gives the eigen-convention
 * table).  Results are bit-identical to plf() on x[i][c][s] = tipvec[code_i][s].
 *
 * One node: exactly one of (tip1, x1) and one of (tip2, x2) is non-NULL;
 * the other arguments are those of plfx_plf_dev_f32/f64 (device pointers). */
int plfx_plf_tips_dev(plfx_ctx *ctx, int dtype, const uint8_t *tip1, const void *x1,
                      const uint8_t *tip2, const void *x2, void *x3, const void *EV, int64_t n,
                      const void *left, const void *right, const int32_t *wgt, uint8_t *scaler,
                      int64_t *scaler_sum, const void *tipvec, void *stream);

/* plfx_plf_tips_dev for states 4 or 20 and flags as plfx_plf_dev_gen
 * (PLFX_FMA: protein nodes on the f64 / f32 matrix cores; DNA is always exact). */
int plfx_plf_tips_dev_gen(plfx_ctx *ctx, int dtype, int states, int flags, const uint8_t *tip1,
                          const void *x1, const uint8_t *tip2, const void *x2, void *x3,
                          const void *EV, int64_t n, const void *left, const void *right,
                          const int32_t *wgt, uint8_t *scaler, int64_t *scaler_sum,
                          const void *tipvec, void *stream);

/* plfx_traverse with tip slots and flags: tips is a host array of nslots device
 * pointers (or NULL = no tips); a slot with tips[s] != NULL is a tip (clv[s] is
 * not read) and may not be an op's parent (codes and tipvec as above for the
 * states).  Each level is
 * issued as up to three batched launches (tip/tip, tip/inner, inner/inner),
 * six-level subtrees over dense leaves, three-level subtrees and level pairs
 * fused where possible (bit-identical results; env PLFX_FUSE=2 no six-level
 * passes, 1 pairs only, 0 none).  states 4 or 20; flags as
 * plfx_plf_dev_gen (PLFX_FMA: protein nodes on the f64 / f32 matrix cores;
 * DNA is always exact).  plfx_traverse == flags PLFX_EXACT, no tips, no tipvec.
 * Protein tip/tip nodes (here and in plfx_plf_tips_dev_gen) are evaluated once
 * per code pair (24 x 24) into tables of the stream's workspace (allocated
 * with the workspace, so also a stream's first call inside a capture uses
 * them) and gathered per site: the same values as the direct computation.  In
 * a traversal (exact and FMA modes, f64 and f32), a node whose two children
 * are such nodes of the level before stages its children from their tables
 * instead of reading their CLVs back (the CLVs are still written; the results
 * are the same). */
int plfx_traverse_tips(plfx_ctx *ctx, int dtype, int states, int flags, const plfx_trav_op *ops,
                       int nops, void *const *clv, const uint8_t *const *tips, int nslots,
                       const void *pmats,
                       int npmats, const void *EV, int64_t n, const int32_t *wgt,
                       uint8_t *const *scalers, int64_t *scaler_sums, const void *tipvec,
                       void *stream);

/* The schedule the last plfx_traverse(_tips) call on this context chose:
 * counts[i] for i < ncounts (extra entries are not written) of
 *   0: fused six-level passes (63 ops)   1: five-level (31)   2: four-level (15)
 *   3: three-level passes (7 ops)        4: level pairs (3 ops)
 *   5: ops run unfused                   6: kernel launches issued
 * Returns the number of entries written. */
#define PLFX_SCHED_COUNTS 7
int plfx_traverse_schedule(const plfx_ctx *ctx, int *counts, int ncounts);

/* ---- (7) root log-likelihood (extension) -- */
/* lnL = sum_i wgt_i * log( sum_c catw[c] * sum_s freq[s] * x[i][c][s] )
 *       + (sum_{j<nsums} scaler_sums[j]) * log(2^-32)
 * x: device CLV of the root (n sites, states S in {4, 20}, 4 categories);
 * catw (4), freq (S): device f64 arrays or NULL (uniform); wgt NULL = 1;
 * scaler_sums: device int64[nsums] (the inner nodes' scalerIncrements).
 * out_lnl: device double; site_lnl: optional device double[n] (log L_i
 * without the scaling correction).  Deterministic (fixed reduction order). */
int plfx_root_lnl(plfx_ctx *ctx, int dtype, int states, const void *x, int64_t n,
                  const double *catw, const double *freq, const int32_t *wgt,
                  const int64_t *scaler_sums, int nsums, double *out_lnl, double *site_lnl,
                  void *stream);

/* ---- (5) instance sizing: testbench_info (app/src/include.h:150-266) ---- */
/* 64-bit throughout.  `instance` < 0 means "no instance" where the
 * reference has an overload without one. */
typedef struct {
  uint64_t alignment_sites;
  uint32_t parallel_instances;
  uint32_t window_size;  /* bytes, AIE window (include.h:155) */
  int32_t layout;        /* plfx_layout */
  int32_t aie_type;      /* plfx_aie */
} plfx_testbench;

uint64_t plfx_tb_alignments_per_instance(const plfx_testbench *tb, int instance);
uint64_t plfx_tb_alignments_padding(const plfx_testbench *tb);
uint64_t plfx_tb_instance_site_offset(const plfx_testbench *tb, int instance);
uint64_t plfx_tb_elements_per_instance(const plfx_testbench *tb);
uint64_t plfx_tb_instance_elements_left(const plfx_testbench *tb);
uint64_t plfx_tb_instance_elements_right(const plfx_testbench *tb);
uint64_t plfx_tb_instance_elements_out(const plfx_testbench *tb);
uint64_t plfx_tb_instance_active_elements_left(const plfx_testbench *tb, int instance);
uint64_t plfx_tb_instance_active_elements_right(const plfx_testbench *tb, int instance);
uint64_t plfx_tb_num_windows_per_instance(const plfx_testbench *tb);

/* Host packing of one instance's input buffers (host_mem.cpp:221-243) into
 * caller-provided host arrays of instance_elements_{left,right} elements of
 * `dtype`; padding is zero-filled. */
int plfx_pack_instance(const plfx_testbench *tb, int instance, int dtype,
                       const void *EV, const void *left, const void *right,
                       const void *x1_all, const void *x2_all, void *out_left,
                       void *out_right);

/* The reference's partition of `total` items over `parts` (include.h:181-189,
 * offsets host_mem.cpp:229,290-291): n0 = ceil(total/parts), part k covers
 * [k*n0, k*n0 + count), the last part short by n0*parts - total.  Used for
 * sites over instances and for independent inner nodes over ranks (BASELINE
 * configs[3]).  PLFX_ERR_INVALID where the reference's arithmetic underflows
 * (the padding reaches a whole share, e.g. 10 items over 8 parts). */
int plfx_shard(uint64_t total, uint32_t parts, uint32_t k, uint64_t *offset, uint64_t *count);

/* The host_mem.cpp:179-209 input protocol with a fixed seed (the reference
 * uses std::random_device): std::mt19937(seed) + uniform_real_distribution
 * <double>(0,1): EV[16], then left[64]/right[64] interleaved, then x1/x2
 * (16*n each) interleaved, x1 x 1e-12 on every 4th site; wgt (may be NULL)
 * = 1.  Host arrays of `dtype`. */
int plfx_gen_hostmem(int dtype, uint32_t seed, uint64_t n, void *EV, void *left, void *right,
                     void *x1, void *x2, int32_t *wgt);

/* ---- (5b) sw_emu: the accelerator instance emulated on the CPU ----------
 * The reference's software-emulation target (make run TARGET=sw_emu,
 * Makefile:199-220; host_mem.cpp:160-164; BASELINE configs[0]): one instance
 * run as its dataflow on the host, window by window -- mm2sleft/mm2sright
 * (hls/src/mm2s{left,right}_memDNAwindow{Comb,Sep}.cpp, stream:
 * mm2sleft_memDNAstreamComb.cpp) split each 512-bit site word into 4 lane
 * beats and prepend the EV half and the transposed P_c (transpose.cpp:6-24)
 * to every window, each lane runs mmul_branch x2 -> combine -> ev
 * (aie/src/128x9DNAwindow8192Comb/kernels/), and s2mm
 * (hls/src/s2mm_memDNAwindowComb.cpp:45-99) reassembles the 16 values, tests
 * and rescales them with the padding mask.  Host buffers only, no GPU, no
 * context; in_left/in_right must hold the whole padded instance
 * (plfx_tb_instance_elements_left/right).  Writes alignment_sites CLVs and
 * scaler bytes (never the padding, as plfx_instance_run).  Arithmetic in
 * plf()'s order: results are bit-identical to plfx_instance_run.  An explicit
 * target like the reference's, never a fallback of the GPU entry points.
 * aie_type: PLFX_AIE_WINDOW (window_size bytes, a multiple of 32) or
 * PLFX_AIE_STREAM (COMBINED only; window_size ignored). */
int plfx_swemu_instance_run(const void *in_left, const void *in_right, void *out_clv,
                            uint8_t *out_scaler, uint32_t alignment_sites, uint32_t window_size,
                            int layout, int aie_type, int dtype);

/* ---- (9) model setup: P matrices and EV from branch lengths (extension,
 * SURVEY section 8f row 3; the reference's inputs are random or precomputed,
 * host_mem.cpp:189-197, aie/data/inputbranch*) ---------------------------- */
typedef enum { PLFX_PMAT_STATE = 0, PLFX_PMAT_EIGEN = 1 } plfx_pmat_convention;

/* Eigensystem of the time-reversible rate matrix Q_ij = r_ij pi_j (i != j),
 * normalised to one expected substitution per unit time.  exch: S(S-1)/2
 * exchangeabilities, upper triangle row-major (DNA: AC AG AT CG CT GT);
 * freqs: S positive frequencies (normalised here).  eigen (host, S+2S^2
 * doubles) = lambda[S] (descending, lambda_0 = 0) | V[S*S] | Vinv[S*S],
 * row-major, Q = V diag(lambda) Vinv.  Host-only; 2 <= S <= 64. */
int plfx_model_eigen(int states, const double *exch, const double *freqs, double *eigen);

/* Yang (1994) discrete Gamma: ncat equal-probability categories of a
 * Gamma(alpha, alpha) (mean 1); rate = category mean (median = 0) or the
 * median rescaled to mean 1 (median != 0).  Host-only. */
int plfx_gamma_rates(double alpha, int ncat, int median, double *rates);

/* EV (S*S, host) for a convention: STATE -> identity; EIGEN -> EV[k][l] =
 * Vinv[l][k] (CLVs in eigen coordinates, the RAxML form of plf()). */
int plfx_model_ev(int states, int convention, const double *eigen, double *EV);

/* Root weights w (S, host) for plfx_root_lnl's `freq`: STATE -> freqs;
 * EIGEN -> w[k] = sum_s pi_s V[s][k] (the root CLV is in eigen coordinates). */
int plfx_model_root_weights(int states, int convention, const double *eigen, const double *freqs,
                            double *w);

/* Tip vectors (host, 16 x S doubles; DNA: S = 4) for plfx_plf_tips_dev /
 * plfx_traverse_tips: STATE -> tv[code][s] = bit s of code; EIGEN -> tv[code]
 * = Vinv . bits(code) (tips in eigen coordinates). */
int plfx_model_tip_vectors(int states, int convention, const double *eigen, double *tv);

/* Device: pmats[b][c][k][l] (nbranch * ncat * S * S values of dtype) from the
 * eigensystem (device, S+2S^2 doubles, as plfx_model_eigen), category rates
 * (device, ncat doubles) and branch lengths (device, nbranch doubles):
 *   STATE: P_c(t_b) = V diag(exp(lambda r_c t_b)) Vinv;
 *   EIGEN: V[k][l] exp(lambda_l r_c t_b).
 * Branch 2j / 2j+1 are P-matrix pair j's left / right (the traverse layout).
 * f64 arithmetic (device exp, within a few ulp of the host libm). */
int plfx_pmatrix(plfx_ctx *ctx, int dtype, int states, int convention, const double *eigen,
                 const double *rates, int ncat, const double *blen, int64_t nbranch, void *pmats,
                 void *stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* PLFX_H */
