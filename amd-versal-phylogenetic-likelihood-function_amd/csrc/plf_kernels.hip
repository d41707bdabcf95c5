// plf_kernels.hip -- launchers of the fused PLF kernels for CDNA4 (gfx950).
//
// One kernel replaces the reference's whole accelerator pipeline for one PLF
// call: the PL input movers (hls/src/mm2sleft_memDNAwindowComb.cpp:16-100,
// mm2sright_*, transpose.cpp:6-24), the AIE lane chain mmul_branch x2 ->
// combine -> ev (aie/src/128x9DNAwindow8192Comb/kernels/*.cpp) and the PL
// output mover with the underflow test/rescale and the char scaler
// (hls/src/s2mm_memDNAwindowComb.cpp:45-99), plus the host's weighted scaler
// reduction (app/src/host_mem.cpp:384-388).  Arithmetic follows the CPU
// definition plf() (app/src/plf.cpp:19-65) operation for operation.  The
// device code and its mapping are documented in plf_dna.hpp / DESIGN.md.
//
// Grids: grid-stride kernels launch at most the co-resident block count
// (occupancy x CUs) times a tuned multiplier; batched launches spread those
// blocks over the batch's nodes (blockIdx.y = node).
#include <hip/hip_runtime.h>


#include <algorithm>
#include <cstdint>

#include "plf_dna.hpp"
#include "plf_kernels.hpp"
#include "plf_lnl.hpp"
#include "plf_pmat.hpp"
#include "plf_prot.hpp"

namespace plfx {
namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
static_assert(kWsWords == dev::kWsWords, "workspace size mismatch");
static_assert(kMaxBatch == dev::kMaxBatch, "batch size mismatch");
static_assert(sizeof(NodeDescH) == sizeof(dev::NodeDesc), "node descriptor mismatch");
static_assert(sizeof(TripleDescH) == sizeof(dev::TripleDesc), "triple descriptor mismatch");
static_assert(kMaxTriples == dev::kMaxTriples && 3 * kMaxTriples <= kMaxBatch, "triple batch size");
static_assert(sizeof(SeptetDescH) == sizeof(dev::SeptetDesc), "septet descriptor mismatch");
static_assert(kMaxSeptets == dev::kMaxSeptets, "septet batch size");
static_assert(kDeepQueueRegion == dev::kDeepQueueRegion, "deep queue region");
static_assert(sizeof(DeepDescH) == sizeof(dev::DeepDesc), "deep descriptor mismatch");

// Tuned on MI355X (tools/tune_plf.hip@f9b3af3, profiles/r01_tune.log):
// f64 lane-pair kernel, 2 x 16-site steps per trip, non-temporal CLV loads
// and stores, grid = resident blocks.
constexpr int kU64 = 2, kU32 = 4;
constexpr int kGridMul64 = 1, kGridMul32 = 1;
constexpr bool kNt = true;   // f32: NT CLV loads (74.8% vs 70.2% of HBM peak, r01_tune_f32.log)
constexpr bool kNtl64 = true;
constexpr int kMinWaves = 1;
constexpr int kBlocksPerCu32 = 2;  // f32 node kernel grid (launch_cat)
constexpr int kTripleU = 1;  // fused level pairs: 16 sites per trip (tools/tune_triple.hip@f9b3af3)
constexpr int kTripleUTips = 2;  // with coded tips: 32 sites per trip (+13-19 % for 2 tip
                                 // children, equal for 1; profiles/r01_ab_fused_tips.log)
constexpr int kTripleU32 = 2;
// fused three-level subtrees: 2 x 8-site blocks per trip, matrices re-read from
// LDS, next trip's loads in flight (tools/tune_septet.hip@f9b3af3, r01_tune_septet.log)
constexpr int kSeptetU = 2;
constexpr int kSeptetU32 = 2;  // f32 (lane = category): 2 x 16-site blocks per trip
constexpr int kDeepU32 = 2;    // f32 six-level pass: 2 x 16-site blocks per trip

// Co-resident 256-thread blocks of `kernel` on the current device (cached per
// kernel instantiation by the caller).
int resident_blocks(const void *kernel, int &cache) {
  if (!cache) {
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    (void)hipGetDevice(&dev);
    (void)hipGetDeviceProperties(&prop, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 2;
    cache = per_cu * prop.multiProcessorCount;
  }
  return cache;
}

// blocks along x for `count` nodes of n sites each
int64_t grid_x(const void *kernel, int &cache, int grid_mul, int64_t n, int sites_per_block,
               int count, int max_blocks) {
  int64_t blocks = (n + sites_per_block - 1) / sites_per_block;
  const int64_t resident = (int64_t)grid_mul * resident_blocks(kernel, cache);
  // floor: count x cap blocks must fit in one wave of resident blocks (a ceil
  // would leave a few blocks for a second, nearly empty wave: +30% on a
  // 10-node batch)
  const int64_t cap = max_blocks > 0 ? max_blocks : std::max<int64_t>(1, resident / count);
  if (blocks > cap) blocks = cap;
  return blocks < 1 ? 1 : blocks;
}

int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus < 1) cus = 256;
  }
  return cus;
}

// Node kernels switch to the XCD-segmented site mapping (plf_dna.hpp
// wave_sites, kSegL2 = 3) from min_sites up, or always / never with
// DnaArgs::segments.  The thresholds are measured, segmented vs not on the same
// buffers, calls alternating (tools/max_sites.py --ab, three boxes,
// profiles/r05_node_segments_ab.log): f32 +3-4 % at 2^25 sites, +9-29 % from
// 5e7 up; f64 -2 to +1 % at 2^25, +1 % at 2^26, +5-12 % from 1e8 up -- and both
// 6-8 % SLOWER at 2^24, equal below.  Round 6 (tools/node_placement.py, three
// fresh buffer sets per size in one process, profiles/r06_node_placement*.log):
// f64 at 5e7 sites +8-9 % with segments (0.74-0.77 vs 0.68-0.71), so f64 now
// switches from 2^25 as f32 does.  Returns the segmented launch's grid -- the capped grid
// gx rounded down to a multiple of 8 (blocks b and b + 8 share an XCD) -- or
// 0: not segmented.  Never more blocks than gx: below 8 (a small node, or a
// PLFX_MAX_BLOCKS cap < 8) the one-window mapping runs instead.
constexpr int64_t kSegMinSites32 = int64_t(1) << 25, kSegMinSites64 = int64_t(1) << 25;
int64_t segment_grid(const DnaArgs &a, int64_t gx, int64_t min_sites) {
  if (a.segments == 0 || (a.segments < 0 && a.n < min_sites) || gx < 8) return 0;
  return gx - gx % 8;
}

template <typename T, bool kSum>
hipError_t launch_cat(const DnaArgs &a, int max_blocks, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_kernel<T, kU32, kSum, kNt, kMinWaves>;
  // 2 blocks per CU rather than the 3 co-resident ones: at 2^20 sites U = 4
  // leaves 5.33 trips per wave at 3/CU (a sixth trip for a third of the waves)
  // and exactly 8 at 2/CU -- 35.4 vs 35.8 us, and 68.4 vs 69.2 us at 2^21
  // (tools/ab_defer.hip@f9b3af3, tools/tune_f32.hip@f9b3af3; profiles/r02_tune_f32.log)
  // With `streams` calls in flight each takes 1/streams of it: two f32 nodes
  // on two streams at 256 blocks each run 0.773 of the HBM peak in 20-step
  // regions vs 0.746 at 512 (tools/probes/node_grid_lanes_f32.sh,
  // profiles/r06_probe_node_grid_lanes.log)
  const int64_t gx = grid_x((const void *)kernel, cache, kGridMul32, a.n, kWavesPerBlock * 16 * kU32,
                            1, max_blocks > 0 ? max_blocks
                                              : std::max(1, kBlocksPerCu32 * cu_count() / std::max(1, a.streams)));
  const int64_t gs = segment_grid(a, gx, kSegMinSites32);
  if (gs) kernel = &dev::plf_dna_kernel<T, kU32, kSum, kNt, kMinWaves, 3>;
  hipLaunchKernelGGL(kernel, dim3((unsigned)(gs ? gs : gx)), dim3(kBlock), 0, s, (const T *)a.x1,
                     (const T *)a.x2, (T *)a.x3, (const T *)a.EV, (const T *)a.left,
                     (const T *)a.right, a.wgt, a.scaler, a.n, a.ws, a.scaler_sum);
  return hipGetLastError();
}

template <bool kSum>
hipError_t launch_pair(const DnaArgs &a, int max_blocks, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_f64_pair_kernel<kU64, kSum, kMinWaves, kNtl64>;
  // resident blocks / streams: two 2^20-site nodes in flight on two streams at
  // 512 blocks each (16 trips per block) run 0.775 in 20-step regions and 0.80
  // in 200-step ones, vs 0.750 / 0.778 at 1024 (8 trips); one node alone at
  // 512 runs 0.64 (tools/probes/node_grid_lanes.sh, profiles/r06_probe_node_grid_lanes.log)
  const int64_t gx = grid_x((const void *)kernel, cache, kGridMul64, a.n, kWavesPerBlock * 16 * kU64,
                            std::max(1, a.streams), max_blocks);
  const int64_t gs = segment_grid(a, gx, kSegMinSites64);
  if (gs) kernel = &dev::plf_dna_f64_pair_kernel<kU64, kSum, kMinWaves, kNtl64, 3>;
  hipLaunchKernelGGL(kernel, dim3((unsigned)(gs ? gs : gx)), dim3(kBlock), 0, s, (const double *)a.x1,
                     (const double *)a.x2, (double *)a.x3, (const double *)a.EV,
                     (const double *)a.left, (const double *)a.right, a.wgt, a.scaler, a.n, a.ws,
                     a.scaler_sum);
  return hipGetLastError();
}

template <bool kSum, int kTips>
hipError_t launch_pair_batch(const dev::NodeBatch &b, int count, const double *EV,
                             const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                             hipStream_t s, const double *tipvec, int share = 1) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_f64_pair_batch_kernel<kU64, kSum, kMinWaves, kNtl64, kTips>;
  // share: batches the caller keeps in flight on as many streams (plfx_ctx_set_streams)
  const int64_t gx = grid_x((const void *)kernel, cache, kGridMul64, n, kWavesPerBlock * 16 * kU64,
                            count * std::max(1, share), max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt, n,
                     ws, tipvec);
  return hipGetLastError();
}

template <typename T, bool kSum, int kTips>
hipError_t launch_cat_batch(const dev::NodeBatch &b, int count, const T *EV, const int32_t *wgt,
                            int64_t n, unsigned long long *ws, int max_blocks, hipStream_t s,
                            const T *tipvec, int share = 1) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_batch_kernel<T, kU32, kSum, kNt, kMinWaves, kTips>;
  const int64_t gx = grid_x((const void *)kernel, cache, kGridMul32, n, kWavesPerBlock * 16 * kU32,
                            count * std::max(1, share), max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt, n,
                     ws, tipvec);
  return hipGetLastError();
}

template <typename T, int S, int C>
hipError_t launch_lnl_t(const T *x, int64_t n, const double *catw, const double *freq,
                        const int32_t *wgt, const int64_t *sums, int nsums, double *partials,
                        unsigned long long *ticket, double *out, double *site_lnl, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::root_lnl_kernel<T, S, C>;
  // C steps of 64/C sites per wave trip; 2 blocks per CU (more trips per wave: the
  // kernel is short and its ramp and final reduction weigh; tools/ab_lnl.hip@f9b3af3)
  int64_t gx = grid_x((const void *)kernel, cache, 1, n, kWavesPerBlock * 64, 1, 0);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  if (cus > 0 && gx > 2 * (int64_t)cus) gx = 2 * (int64_t)cus;
  if (gx > kLnlMaxGrid) gx = kLnlMaxGrid;
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(kBlock), 0, s, x, n, catw, freq, wgt, sums,
                     nsums, partials, ticket, out, site_lnl);
  return hipGetLastError();
}

// protein root lnL: 64-site LDS tiles, the co-resident grid (plf_lnl.hpp
// root_lnl_prot_kernel; the C-lanes form took 94 us for 2^18 f64 sites)
template <typename T>
hipError_t launch_lnl_prot_t(const T *x, int64_t n, const double *catw, const double *freq,
                             const int32_t *wgt, const int64_t *sums, int nsums, double *partials,
                             unsigned long long *ticket, double *out, double *site_lnl, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::root_lnl_prot_kernel<T>;
  int64_t gx = grid_x((const void *)kernel, cache, 1, n, 64, 1, 0);
  if (gx > kLnlMaxGrid) gx = kLnlMaxGrid;
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(kBlock), 0, s, x, n, catw, freq, wgt, sums, nsums,
                     partials, ticket, out, site_lnl);
  return hipGetLastError();
}

template <typename T, bool kFma, bool kSum, int kTips>
hipError_t launch_prot_t(const DnaArgs &a, int max_blocks, hipStream_t s, const T *tipvec) {
  static_assert(sizeof(T) == 4, "f32 protein; f64 runs launch_prot_mfma_t / launch_prot_exact64_t");
  // f32: FMA mode on the matrix cores (v_mfma_f32_16x16x4_f32 = fmaf chain;
  // rows 16..19 of the products and the back-transform on 4x4x1_16b, kQ = 2:
  // 52.4 -> 46.5 us at 2^18, profiles/r02_tune_protein_f32_q.log), exact mode
  // on the LDS-matrix kernel (4-row groups, tile prefetch)
  // (tools/tune_prot32.hip@f9b3af3, profiles/r02_tune_protein_f32.log)
  if constexpr (kFma) {
    static int cache = 0;
    auto kernel = &dev::plf_prot_mfma32_kernel<kSum, 3, kTips>;
    // with `streams` calls in flight: the resident blocks per CU / streams,
    // rounded UP to whole blocks per CU (3 per CU -> 2 at two streams: 0.743-
    // 0.746 vs 0.728-0.730 at the full grid and 0.737 at 1.5 per CU;
    // profiles/r06_probe_prot_grid_lanes.log)
    int cap = max_blocks;
    if (cap <= 0 && a.streams > 1) {
      const int cus = cu_count(), per_cu = std::max(1, resident_blocks((const void *)kernel, cache) / cus);
      cap = cus * ((per_cu + a.streams - 1) / a.streams);
    }
    const int64_t gx = grid_x((const void *)kernel, cache, 1, a.n, 64, 1, cap);
    hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(kBlock), 0, s, (const T *)a.x1,
                       (const T *)a.x2, (T *)a.x3, (const T *)a.EV, (const T *)a.left,
                       (const T *)a.right, a.wgt, a.scaler, a.n, a.ws, a.scaler_sum, tipvec);
  } else {
    static int cache = 0;
    auto kernel = &dev::plf_prot_lds_kernel<T, kSum, 2, kTips, 4, false>;
    const int64_t gx = grid_x((const void *)kernel, cache, 1, a.n, 64, 1, max_blocks);
    hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(kBlock), 0, s, (const T *)a.x1,
                       (const T *)a.x2, (T *)a.x3, (const T *)a.EV, (const T *)a.left,
                       (const T *)a.right, a.wgt, a.scaler, a.n, a.ws, a.scaler_sum, tipvec);
  }
  return hipGetLastError();
}

template <bool kSum, int kTips>
hipError_t launch_prot_mfma_t(const DnaArgs &a, int max_blocks, hipStream_t s,
                              const double *tipvec) {
  static int cache = 0;
  // X3 to LDS through permuted back-transform rows (kX3 = 2: conflict-free
  // b128 writes; 90.2 vs 91.2 us at 2^18, 342 vs 345 at 2^20, tools/tune_prot.hip@f9b3af3,
  // profiles/r02_tune_protein_v3.log); first tile's loads before the matrix fragments.
  // From 32 tiles per block (2^20 sites at 512 blocks) on, tiles come from the
  // device-wide queue (kDyn, plf_prot.hpp ProtQueue): 2^20 -3..-5 %, 2^22 -10 %
  // dense, tip/inner -8 / -14 %; below that, and for tip/tip nodes at any size,
  // the fixed stride is as fast or faster (tools/tune_prot64d.hip@f9b3af3,
  // profiles/r03_tune_protein_dyn.log)
  auto kernel = &dev::plf_prot_mfma_kernel<kSum, 2, kTips, false>;
  // resident blocks / streams (two 2^18-site nodes in flight: 256 blocks each,
  // +1-2 %; the VALU protein kernels keep their full grid, which measured best
  // with two in flight too -- tools/probes/prot_grid_lanes.sh,
  // profiles/r06_probe_prot_grid_lanes.log)
  const int64_t gx = grid_x((const void *)kernel, cache, 1, a.n, 64, std::max(1, a.streams), max_blocks);
  auto launch = [&](auto k) {
    hipLaunchKernelGGL(k, dim3((unsigned)gx), dim3(kBlock), 0, s, (const double *)a.x1,
                       (const double *)a.x2, (double *)a.x3, (const double *)a.EV,
                       (const double *)a.left, (const double *)a.right, a.wgt, a.scaler, a.n, a.ws,
                       a.scaler_sum, tipvec);
    return hipGetLastError();
  };
  if constexpr (kTips < 2)  // the queue form exists for dense and tip/inner nodes only
    if (a.ws && (a.n + 63) / 64 >= 32 * gx) return launch(&dev::plf_prot_mfma_kernel<kSum, 2, kTips, true>);
  return launch(kernel);
}

template <bool kSum, int kTips>
hipError_t launch_prot_exact64_t(const DnaArgs &a, int max_blocks, hipStream_t s,
                                 const double *tipvec) {
  static int cache = 0;
  // 10-row groups + tile prefetch (tools/tune_prot.hip@f9b3af3, profiles/r02_tune_protein_exact_rows.log)
  auto kernel = &dev::plf_prot_lds_kernel<double, kSum, 2, kTips, 10, true>;
  const int64_t gx = grid_x((const void *)kernel, cache, 1, a.n, 64, 1, max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(kBlock), 0, s, (const double *)a.x1,
                     (const double *)a.x2, (double *)a.x3, (const double *)a.EV,
                     (const double *)a.left, (const double *)a.right, a.wgt, a.scaler, a.n, a.ws,
                     a.scaler_sum, tipvec);
  return hipGetLastError();
}

// dtype x mode x scaler-sum x tips dispatch of the protein kernels
template <int kTips>
hipError_t launch_prot_tips(int dtype, bool fma, const DnaArgs &a, int max_blocks, hipStream_t s,
                            const void *tipvec) {
  const bool sum = a.scaler_sum != nullptr;
  const double *V64 = (const double *)tipvec;
  const float *V32 = (const float *)tipvec;
  if (dtype == 1) {
    if (fma)  // matrix cores: bit-identical to the fused VALU chain (plf_prot.hpp)
      return sum ? launch_prot_mfma_t<true, kTips>(a, max_blocks, s, V64)
                 : launch_prot_mfma_t<false, kTips>(a, max_blocks, s, V64);
    // exact: matrices broadcast from LDS (plf_prot.hpp)
    return sum ? launch_prot_exact64_t<true, kTips>(a, max_blocks, s, V64)
               : launch_prot_exact64_t<false, kTips>(a, max_blocks, s, V64);
  }
  if (fma)
    return sum ? launch_prot_t<float, true, true, kTips>(a, max_blocks, s, V32)
               : launch_prot_t<float, true, false, kTips>(a, max_blocks, s, V32);
  return sum ? launch_prot_t<float, false, true, kTips>(a, max_blocks, s, V32)
             : launch_prot_t<float, false, false, kTips>(a, max_blocks, s, V32);
}

template <bool kSum, int kTips>
hipError_t launch_triples_t(const dev::TripleBatch &b, int count, const double *EV,
                            const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                            hipStream_t s, const double *tipvec) {
  static int cache = 0;
  constexpr int U = kTips ? kTripleUTips : kTripleU;
  auto kernel = &dev::plf_dna_f64_triple_kernel<kSum, 1, kNtl64, kTips, U>;
  const int64_t gx = grid_x((const void *)kernel, cache, 1, n, kWavesPerBlock * 16 * U, count,
                            max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt,
                     n, ws, tipvec);
  return hipGetLastError();
}

template <bool kSum, int kTips>
hipError_t launch_triples32_t(const dev::TripleBatch &b, int count, const float *EV,
                              const int32_t *wgt, int64_t n, unsigned long long *ws,
                              int max_blocks, hipStream_t s, const float *tipvec) {
  static int cache = 0;
  constexpr int U = kTripleU32;
  auto kernel = &dev::plf_dna_cat_triple_kernel<float, kSum, 1, kNt, kTips, U>;
  const int64_t gx = grid_x((const void *)kernel, cache, 1, n, kWavesPerBlock * 16 * U, count,
                            max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt,
                     n, ws, tipvec);
  return hipGetLastError();
}

template <bool kSum, int kTips>
hipError_t launch_septets_t(const dev::SeptetBatch &b, int count, const double *EV,
                            const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                            hipStream_t s, const double *tipvec) {
  static int cache = 0;
  // next-trip prefetch for dense leaves only: with coded leaves the pass is
  // write-bound and the prefetch registers cost 4-4.5 % (r01_ab_fused_tips.log)
  auto kernel = &dev::plf_dna_f64_septet_kernel<kSum, 1, kNtl64, kTips, kSeptetU, kTips == 0>;
  const int64_t gx = grid_x((const void *)kernel, cache, 1, n, kWavesPerBlock * 8 * kSeptetU, count,
                            max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt,
                     n, ws, tipvec);
  return hipGetLastError();
}

template <bool kSum, int kTips>
hipError_t launch_septets32_t(const dev::SeptetBatch &b, int count, const float *EV,
                              const int32_t *wgt, int64_t n, unsigned long long *ws,
                              int max_blocks, hipStream_t s, const float *tipvec) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_cat_septet_kernel<float, kSum, 1, kNt, kTips, kSeptetU32>;
  const int64_t gx = grid_x((const void *)kernel, cache, 1, n, kWavesPerBlock * 16 * kSeptetU32,
                            count, max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt,
                     n, ws, tipvec);
  return hipGetLastError();
}

// fused six-level subtrees: 512-thread blocks (one LDS copy of the 63 nodes'
// matrices per 8 waves), 2 x 8-site blocks per trip, grid = co-resident blocks
// (tools/gpu_deep.sh@f9b3af3, profiles/r01_deep.log)
template <int D, typename T, bool kSum, int U, int kThreads, int kTips, bool kDyn>
hipError_t launch_deep_k(const dev::DeepDesc &d, const T *EV, const int32_t *wgt, int64_t n,
                         unsigned long long *ws, int max_blocks, hipStream_t s, const T *tipvec) {
  static int resident = 0;
  // f64: lane pairs, 8 sites per wave instruction; f32: lane = category, 16
  auto kernel = [] {
    if constexpr (sizeof(T) == 8) return &dev::plf_dna_f64_deep_kernel<D, kSum, kNtl64, U, kThreads, kTips, kDyn>;
    else return &dev::plf_dna_cat_deep_kernel<D, T, kSum, kNt, U, kThreads, kTips, kDyn>;
  }();
  constexpr int kSitesPerWave = sizeof(T) == 8 ? 8 : 16;
  if (!resident) {
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    (void)hipGetDevice(&dev);
    (void)hipGetDeviceProperties(&prop, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kernel, kThreads, 0) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    resident = per_cu * prop.multiProcessorCount;
  }
  const int64_t per_block = (int64_t)(kThreads / 64) * kSitesPerWave * U;
  int64_t gx = (n + per_block - 1) / per_block;
  gx = std::max<int64_t>(1, std::min<int64_t>(gx, max_blocks > 0 ? max_blocks : resident));
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(kThreads), 0, s, d, EV, wgt, n, ws, tipvec);
  return hipGetLastError();
}

template <int D, typename T, bool kSum, int U, int kThreads, int kTips = 0>
hipError_t launch_deep_t(const dev::DeepDesc &d, const T *EV, const int32_t *wgt, int64_t n,
                         unsigned long long *ws, int max_blocks, hipStream_t s,
                         const T *tipvec = nullptr) {
  // chunks from the wave-level queue (plf_dna.hpp WaveQueue) whenever there is
  // a workspace: the fixed stride left wave exits spread over 2.61-3.36 ms of a
  // 2^20-site f64 pass (same process: 3358 -> 3116 us,
  // profiles/r03_tune_deep_dyn.log; bench tree64 f64 --tips 1688 -> 1643 us,
  // f32 --tips 875 -> 861, f32 dense equal, profiles/r03_ab_deep_dyn.log)
  // (the traversal always has a stream workspace when it launches a pass)
  if (!ws) return hipErrorInvalidValue;
  return launch_deep_k<D, T, kSum, U, kThreads, kTips, true>(d, EV, wgt, n, ws, max_blocks, s, tipvec);
}

}  // namespace

template <int D>
hipError_t launch_deep_d(int dtype, bool any_sum, const dev::DeepDesc &d, const void *EV,
                         const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                         hipStream_t s, int tips, const void *tipvec) {
  const double *E64 = (const double *)EV;
  const float *E32 = (const float *)EV;
  if (tips == 2 && dtype != 1) {  // coded leaves, f32
    const float *V = (const float *)tipvec;
    // 4 x 16-site blocks per trip, as f64: tree64 f32 --tips 0.664 (U = 2) ->
    // 0.707 same box, U = 1 0.673; three-level passes 0.633
    // (profiles/r03_ab_deep_tips_u_f32.log)
    return any_sum ? launch_deep_t<D, float, true, 4, 512, 2>(d, E32, wgt, n, ws, max_blocks, s, V)
                   : launch_deep_t<D, float, false, 4, 512, 2>(d, E32, wgt, n, ws, max_blocks, s, V);
  }
  if (tips == 2) {
    const double *V = (const double *)tipvec;
    // coded leaves: 4 x 8-site blocks per trip (every output stream gets 4 KiB
    // runs per wave and trip; the pass is write-bound): 0.693 -> 0.727 of
    // peak on tree64 --tips same box, U = 1 0.637; U = 6/8 spill
    // (profiles/r03_ab_deep_tips_u.log)
    return any_sum ? launch_deep_t<D, double, true, 4, 512, 2>(d, E64, wgt, n, ws, max_blocks, s, V)
                   : launch_deep_t<D, double, false, 4, 512, 2>(d, E64, wgt, n, ws, max_blocks, s, V);
  }
  if (tips != 0) return hipErrorInvalidValue;
  if (dtype == 1)
    return any_sum ? launch_deep_t<D, double, true, 2, 512>(d, E64, wgt, n, ws, max_blocks, s)
                   : launch_deep_t<D, double, false, 2, 512>(d, E64, wgt, n, ws, max_blocks, s);
  return any_sum ? launch_deep_t<D, float, true, kDeepU32, 512>(d, E32, wgt, n, ws, max_blocks, s)
                 : launch_deep_t<D, float, false, kDeepU32, 512>(d, E32, wgt, n, ws, max_blocks, s);
}

hipError_t launch_plf_dna_deep(int dtype, int depth, const DeepDescH *t, const void *EV,
                               const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                               hipStream_t s, int tips, const void *tipvec) {
  if (depth < 4 || depth > 6) return hipErrorInvalidValue;
  dev::DeepDesc d;
  __builtin_memcpy(&d, t, sizeof(d));
  bool any_sum = false;
  for (int q = 0; q < (1 << depth) - 1; q++) any_sum |= t->ss[q] != nullptr;
  switch (depth) {
    case 4: return launch_deep_d<4>(dtype, any_sum, d, EV, wgt, n, ws, max_blocks, s, tips, tipvec);
    case 5: return launch_deep_d<5>(dtype, any_sum, d, EV, wgt, n, ws, max_blocks, s, tips, tipvec);
    default: return launch_deep_d<6>(dtype, any_sum, d, EV, wgt, n, ws, max_blocks, s, tips, tipvec);
  }
}

hipError_t launch_plf_dna_septets(int dtype, const SeptetDescH *t, int count, const void *EV,
                                  const int32_t *wgt, int64_t n, unsigned long long *ws,
                                  int max_blocks, hipStream_t s, int tips, const void *tipvec) {
  if (count < 1 || count > kMaxSeptets || tips < 0 || tips > 2) return hipErrorInvalidValue;
  dev::SeptetBatch b{};
  bool any_sum = false;
  for (int i = 0; i < count; i++) {
    __builtin_memcpy(&b.d[i], &t[i], sizeof(t[i]));
    for (int q = 0; q < 7; q++) any_sum |= t[i].ss[q] != nullptr;
  }
  const double *E64 = (const double *)EV, *V64 = (const double *)tipvec;
  const float *E32 = (const float *)EV, *V32 = (const float *)tipvec;
  switch ((dtype == 1 ? 6 : 0) + (any_sum ? 3 : 0) + tips) {
    case 0: return launch_septets32_t<false, 0>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 1: return launch_septets32_t<false, 1>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 2: return launch_septets32_t<false, 2>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 3: return launch_septets32_t<true, 0>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 4: return launch_septets32_t<true, 1>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 5: return launch_septets32_t<true, 2>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 6: return launch_septets_t<false, 0>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 7: return launch_septets_t<false, 1>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 8: return launch_septets_t<false, 2>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 9: return launch_septets_t<true, 0>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 10: return launch_septets_t<true, 1>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    default: return launch_septets_t<true, 2>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
  }
}

hipError_t launch_plf_dna_triples(int dtype, const TripleDescH *t, int count, const void *EV,
                                  const int32_t *wgt, int64_t n, unsigned long long *ws,
                                  int max_blocks, hipStream_t s, int tips, const void *tipvec) {
  if (count < 1 || count > kMaxTriples || tips < 0 || tips > 2) return hipErrorInvalidValue;
  dev::TripleBatch b{};
  bool any_sum = false;
  for (int i = 0; i < count; i++) {
    static_assert(sizeof(b.d[0]) == sizeof(t[0]), "layout");
    __builtin_memcpy(&b.d[i], &t[i], sizeof(t[i]));
    any_sum |= t[i].ssa || t[i].ssb || t[i].ssp;
  }
  const double *E64 = (const double *)EV, *V64 = (const double *)tipvec;
  const float *E32 = (const float *)EV, *V32 = (const float *)tipvec;
  switch ((dtype == 1 ? 6 : 0) + (any_sum ? 3 : 0) + tips) {
    case 0: return launch_triples32_t<false, 0>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 1: return launch_triples32_t<false, 1>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 2: return launch_triples32_t<false, 2>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 3: return launch_triples32_t<true, 0>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 4: return launch_triples32_t<true, 1>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 5: return launch_triples32_t<true, 2>(b, count, E32, wgt, n, ws, max_blocks, s, V32);
    case 6: return launch_triples_t<false, 0>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 7: return launch_triples_t<false, 1>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 8: return launch_triples_t<false, 2>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 9: return launch_triples_t<true, 0>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    case 10: return launch_triples_t<true, 1>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
    default: return launch_triples_t<true, 2>(b, count, E64, wgt, n, ws, max_blocks, s, V64);
  }
}

// Protein batches: grid (resident blocks, count) -- every node gets the grid a
// one-node launch would (the kernels keep their one-node grid stride) and the
// nodes' blocks follow each other through the co-resident slots.
template <typename K, typename TT>
hipError_t launch_prot_batch_k(K kernel, int &cache, const dev::NodeBatch &b, int count, const TT *EV,
                               const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                               hipStream_t s, const TT *tipvec) {
  const int64_t gx = grid_x((const void *)kernel, cache, 1, n, 64, 1, max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, EV, wgt, n, ws,
                     tipvec);
  return hipGetLastError();
}

template <int kTips, bool kSum>
hipError_t launch_prot_batch_t(int dtype, bool fma, const dev::NodeBatch &b, int count, const void *EV,
                               const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                               hipStream_t s, const void *tipvec) {
  const double *E64 = (const double *)EV, *V64 = (const double *)tipvec;
  const float *E32 = (const float *)EV, *V32 = (const float *)tipvec;
  if (dtype == 1 && fma) {
    static int cache = 0;
    return launch_prot_batch_k(&dev::plf_prot_mfma_batch_kernel<kSum, 2, kTips>, cache, b, count, E64, wgt,
                               n, ws, max_blocks, s, V64);
  }
  if (dtype == 1) {
    static int cache = 0;
    return launch_prot_batch_k(&dev::plf_prot_lds_batch_kernel<double, kSum, 2, kTips, 10, true>, cache, b,
                               count, E64, wgt, n, ws, max_blocks, s, V64);
  }
  if (fma) {
    static int cache = 0;
    return launch_prot_batch_k(&dev::plf_prot_mfma32_batch_kernel<kSum, 3, kTips>, cache, b, count, E32,
                               wgt, n, ws, max_blocks, s, V32);
  }
  static int cache = 0;
  return launch_prot_batch_k(&dev::plf_prot_lds_batch_kernel<float, kSum, 2, kTips, 4, false>, cache, b,
                             count, E32, wgt, n, ws, max_blocks, s, V32);
}

hipError_t launch_plf_prot_batch(int dtype, bool fma, const NodeDescH *nodes, int count, const void *EV,
                                 const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                                 hipStream_t s, int tips, const void *tipvec) {
  if (count < 1 || count > kMaxBatch || tips < 0 || tips > 2) return hipErrorInvalidValue;
  dev::NodeBatch b{};
  bool any_sum = false;
  for (int i = 0; i < count; i++) {
    b.d[i] = dev::NodeDesc{nodes[i].x1, nodes[i].x2, nodes[i].x3, nodes[i].left, nodes[i].right,
                           nodes[i].scaler, nodes[i].scaler_sum};
    any_sum |= nodes[i].scaler_sum != nullptr;
  }
  switch (tips * 2 + (any_sum ? 1 : 0)) {
    case 0: return launch_prot_batch_t<0, false>(dtype, fma, b, count, EV, wgt, n, ws, max_blocks, s, tipvec);
    case 1: return launch_prot_batch_t<0, true>(dtype, fma, b, count, EV, wgt, n, ws, max_blocks, s, tipvec);
    case 2: return launch_prot_batch_t<1, false>(dtype, fma, b, count, EV, wgt, n, ws, max_blocks, s, tipvec);
    case 3: return launch_prot_batch_t<1, true>(dtype, fma, b, count, EV, wgt, n, ws, max_blocks, s, tipvec);
    case 4: return launch_prot_batch_t<2, false>(dtype, fma, b, count, EV, wgt, n, ws, max_blocks, s, tipvec);
    // tips == 2 runs only as the combination tables of tip/tip nodes (plfx_api
    // batch_impl), which carry no sum: a tip/tip node's sum comes from the
    // gather, so the summing tip/tip forms are not built
    default: return hipErrorInvalidValue;
  }
}

template <typename T, bool kSum>
hipError_t launch_gather_t(const dev::ProtGatherBatch &b, int count, const int32_t *wgt, int64_t n,
                           unsigned long long *ws, int max_blocks, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::prot_tiptip_gather_kernel<T, kSum>;
  const int64_t gx = grid_x((const void *)kernel, cache, 1, n, 64, 1, max_blocks);
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, wgt, n, ws);
  return hipGetLastError();
}

hipError_t launch_prot_tiptip_gather(int dtype, const ProtGatherDescH *d, int count, const int32_t *wgt,
                                     int64_t n, unsigned long long *ws, int max_blocks, hipStream_t s) {
  if (count < 1 || count > kMaxBatch) return hipErrorInvalidValue;
  static_assert(kProtCombos == dev::kProtCombos, "combination count");
  dev::ProtGatherBatch b{};
  bool any_sum = false;
  for (int i = 0; i < count; i++) {
    static_assert(sizeof(b.d[0]) == sizeof(d[0]), "layout");
    __builtin_memcpy(&b.d[i], &d[i], sizeof(d[i]));
    any_sum |= d[i].scaler_sum != nullptr;
  }
  if (dtype == 1)
    return any_sum ? launch_gather_t<double, true>(b, count, wgt, n, ws, max_blocks, s)
                   : launch_gather_t<double, false>(b, count, wgt, n, ws, max_blocks, s);
  return any_sum ? launch_gather_t<float, true>(b, count, wgt, n, ws, max_blocks, s)
                 : launch_gather_t<float, false>(b, count, wgt, n, ws, max_blocks, s);
}

hipError_t launch_prot_tab_batch(int dtype, bool fma, const ProtTabDescH *d, int count, const void *EV,
                                 const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                                 hipStream_t s) {
  if (count < 1 || count > kMaxBatch) return hipErrorInvalidValue;
  dev::ProtTabBatch b{};
  bool any_sum = false;
  for (int i = 0; i < count; i++) {
    static_assert(sizeof(b.d[0]) == sizeof(d[0]), "layout");
    __builtin_memcpy(&b.d[i], &d[i], sizeof(d[i]));
    any_sum |= d[i].scaler_sum != nullptr;
  }
  auto launch = [&](auto kernel, int &cache, auto ev) {
    const int64_t gx = grid_x((const void *)kernel, cache, 1, n, 64, 1, max_blocks);  // full grid per node
    hipLaunchKernelGGL(kernel, dim3((unsigned)gx, (unsigned)count), dim3(kBlock), 0, s, b, ev, wgt, n, ws);
    return hipGetLastError();
  };
  static int c64 = 0, c64n = 0, c32 = 0, c32n = 0, x64 = 0, x64n = 0, x32 = 0, x32n = 0;
  const double *E64 = static_cast<const double *>(EV);
  const float *E32 = static_cast<const float *>(EV);
  if (!fma) {  // the exact bodies' shapes (launch_prot_t / launch_prot_exact64_t)
    if (dtype == 1)
      return any_sum ? launch(&dev::plf_prot_lds_tab_batch_kernel<double, true, 10, true>, x64, E64)
                     : launch(&dev::plf_prot_lds_tab_batch_kernel<double, false, 10, true>, x64n, E64);
    return any_sum ? launch(&dev::plf_prot_lds_tab_batch_kernel<float, true, 4, false>, x32, E32)
                   : launch(&dev::plf_prot_lds_tab_batch_kernel<float, false, 4, false>, x32n, E32);
  }
  if (dtype == 1)
    return any_sum ? launch(&dev::plf_prot_mfma_tab_batch_kernel<true>, c64, E64)
                   : launch(&dev::plf_prot_mfma_tab_batch_kernel<false>, c64n, E64);
  return any_sum ? launch(&dev::plf_prot_mfma32_tab_batch_kernel<true>, c32, E32)
                 : launch(&dev::plf_prot_mfma32_tab_batch_kernel<false>, c32n, E32);
}

hipError_t launch_plf_prot(int dtype, bool fma, const DnaArgs &a, int max_blocks, hipStream_t s,
                           int tips, const void *tipvec) {
  // tip/tip nodes (tips == 2) always go through the combination tables of the
  // stream's workspace (launch_plf_prot_batch over the 576 code pairs, then
  // launch_prot_tiptip_gather), never a one-node kernel
  switch (tips) {
    case 0: return launch_prot_tips<0>(dtype, fma, a, max_blocks, s, tipvec);
    case 1: return launch_prot_tips<1>(dtype, fma, a, max_blocks, s, tipvec);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_plf_dna_f32(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_cat<float, true>(a, max_blocks, s)
                      : launch_cat<float, false>(a, max_blocks, s);
}

hipError_t launch_plf_dna_f64(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_pair<true>(a, max_blocks, s) : launch_pair<false>(a, max_blocks, s);
}

hipError_t launch_plf_dna_batch(int dtype, const NodeDescH *nodes, int count, const void *EV,
                                const int32_t *wgt, int64_t n, unsigned long long *ws,
                                int max_blocks, hipStream_t s, int tips, const void *tipvec,
                                int share) {
  if (count < 1 || count > kMaxBatch || tips < 0 || tips > 2) return hipErrorInvalidValue;
  dev::NodeBatch b{};
  bool any_sum = false;
  for (int i = 0; i < count; i++) {
    b.d[i] = dev::NodeDesc{nodes[i].x1, nodes[i].x2, nodes[i].x3, nodes[i].left, nodes[i].right,
                           nodes[i].scaler, nodes[i].scaler_sum};
    any_sum |= nodes[i].scaler_sum != nullptr;
  }
  const int key = (dtype == 1 ? 6 : 0) + (any_sum ? 3 : 0) + tips;
  const double *E64 = (const double *)EV;
  const float *E32 = (const float *)EV;
  const double *TV64 = (const double *)tipvec;
  const float *TV32 = (const float *)tipvec;
  switch (key) {
    case 0: return launch_cat_batch<float, false, 0>(b, count, E32, wgt, n, ws, max_blocks, s, TV32, share);
    case 1: return launch_cat_batch<float, false, 1>(b, count, E32, wgt, n, ws, max_blocks, s, TV32, share);
    case 2: return launch_cat_batch<float, false, 2>(b, count, E32, wgt, n, ws, max_blocks, s, TV32, share);
    case 3: return launch_cat_batch<float, true, 0>(b, count, E32, wgt, n, ws, max_blocks, s, TV32, share);
    case 4: return launch_cat_batch<float, true, 1>(b, count, E32, wgt, n, ws, max_blocks, s, TV32, share);
    case 5: return launch_cat_batch<float, true, 2>(b, count, E32, wgt, n, ws, max_blocks, s, TV32, share);
    case 6: return launch_pair_batch<false, 0>(b, count, E64, wgt, n, ws, max_blocks, s, TV64, share);
    case 7: return launch_pair_batch<false, 1>(b, count, E64, wgt, n, ws, max_blocks, s, TV64, share);
    case 8: return launch_pair_batch<false, 2>(b, count, E64, wgt, n, ws, max_blocks, s, TV64, share);
    case 9: return launch_pair_batch<true, 0>(b, count, E64, wgt, n, ws, max_blocks, s, TV64, share);
    case 10: return launch_pair_batch<true, 1>(b, count, E64, wgt, n, ws, max_blocks, s, TV64, share);
    default: return launch_pair_batch<true, 2>(b, count, E64, wgt, n, ws, max_blocks, s, TV64, share);
  }
}

hipError_t launch_root_lnl(int dtype, int states, const void *x, int64_t n, const double *catw,
                           const double *freq, const int32_t *wgt, const int64_t *scaler_sums,
                           int nsums, double *partials, unsigned long long *ticket, double *out,
                           double *site_lnl, hipStream_t s) {
  if (states == 4 && dtype == 1)
    return launch_lnl_t<double, 4, 4>((const double *)x, n, catw, freq, wgt, scaler_sums, nsums,
                                      partials, ticket, out, site_lnl, s);
  if (states == 4 && dtype == 0)
    return launch_lnl_t<float, 4, 4>((const float *)x, n, catw, freq, wgt, scaler_sums, nsums,
                                     partials, ticket, out, site_lnl, s);
  if (states == 20 && dtype == 1)
    return launch_lnl_prot_t<double>((const double *)x, n, catw, freq, wgt, scaler_sums, nsums,
                                     partials, ticket, out, site_lnl, s);
  if (states == 20 && dtype == 0)
    return launch_lnl_prot_t<float>((const float *)x, n, catw, freq, wgt, scaler_sums, nsums,
                                    partials, ticket, out, site_lnl, s);
  return hipErrorInvalidValue;
}

hipError_t launch_scaler_sum(const uint8_t *scaler, const int32_t *wgt, int64_t n, int64_t *out,
                             unsigned long long *ws, int max_blocks, hipStream_t s) {
  int64_t blocks = (n + kBlock - 1) / kBlock;
  const int64_t cap = max_blocks > 0 ? max_blocks : 2048;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dev::scaler_sum_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, scaler,
                     wgt, n, ws, out);
  return hipGetLastError();
}

hipError_t launch_pmatrix(int dtype, bool eigen_conv, const double *eigen, int S,
                          const double *rates, int ncat, const double *blen, int64_t nbranch,
                          void *out, hipStream_t s) {
  const int64_t total = nbranch * ncat * S * S;
  int64_t blocks = (total + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  const dim3 g((unsigned)blocks), b(kBlock);
  if (dtype == 1) {
    if (eigen_conv)
      hipLaunchKernelGGL((dev::pmatrix_kernel<double, true>), g, b, 0, s, eigen, S, rates, ncat,
                         blen, nbranch, (double *)out);
    else
      hipLaunchKernelGGL((dev::pmatrix_kernel<double, false>), g, b, 0, s, eigen, S, rates, ncat,
                         blen, nbranch, (double *)out);
  } else {
    if (eigen_conv)
      hipLaunchKernelGGL((dev::pmatrix_kernel<float, true>), g, b, 0, s, eigen, S, rates, ncat,
                         blen, nbranch, (float *)out);
    else
      hipLaunchKernelGGL((dev::pmatrix_kernel<float, false>), g, b, 0, s, eigen, S, rates, ncat,
                         blen, nbranch, (float *)out);
  }
  return hipGetLastError();
}

}  // namespace plfx
