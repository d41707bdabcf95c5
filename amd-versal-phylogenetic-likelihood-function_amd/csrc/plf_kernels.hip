// plf_kernels.hip -- fused PLF inner-node update for CDNA4 (gfx950).
//
// One kernel replaces the reference's whole accelerator pipeline for one PLF
// call: the PL input movers (hls/src/mm2sleft_memDNAwindowComb.cpp:16-100,
// mm2sright_*, transpose.cpp:6-24), the AIE lane chain mmul_branch x2 ->
// combine -> ev (aie/src/128x9DNAwindow8192Comb/kernels/*.cpp) and the PL
// output mover with the underflow test/rescale and the char scaler
// (hls/src/s2mm_memDNAwindowComb.cpp:45-99), plus the host's weighted scaler
// reduction (app/src/host_mem.cpp:384-388).  Arithmetic follows the CPU
// definition plf() (app/src/plf.cpp:19-65) operation for operation.
//
// Mapping (DNA, S=4 states, C=4 Gamma categories, V=16 values per site):
//   * 4 consecutive lanes own one site, lane c = category c (the reference's
//     4 AIE lanes, aie/src/128x9DNAwindow8192Comb/graph.h:34-46); a wave covers
//     16 sites per step and issues U steps of loads before computing.
//   * lane c streams its 4 states of x1 and x2 with 16-byte loads (the 4 lanes
//     of a site read one contiguous 64/128-byte site record, the wave one
//     contiguous 1/2 KiB block) and writes its 4 results with non-temporal
//     16-byte stores.
//   * P_L[c], P_R[c] (16 values each) live in VGPRs for the whole grid-stride
//     loop; EV is wave-uniform and sits in SGPRs (scalar loads).
//   * per-site scale test: each lane tests its 4 values, a wave ballot gives a
//     64-bit mask, and the site's nibble == 0xF decides; the rescale is a
//     select (no divergent branch).  Lane c==0 writes the site's scaler byte
//     and accumulates wgt into a register; one 64-bit atomic per block feeds a
//     self-resetting ticket reduction, so no memset launch is needed per call.
//   * no FMA contraction (-ffp-contract=off) and the reference's ascending
//     accumulation order from +0.0: bit-exact against plf() in f32 and against
//     its double instantiation in f64.
//   * grid = resident blocks (occupancy x CUs) x kGridWaves, grid-stride loop.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "plf_dna.hpp"
#include "plf_kernels.hpp"

namespace plfx {
namespace {

using dev::kBlock;
using dev::kWavesPerBlock;
static_assert(kWsWords == dev::kWsWords, "workspace size mismatch");

// Tuned on MI355X (tools/tune_plf.hip, profiles/r01_tune.log):
// f64 lane-pair kernel, 2 x 16-site steps per trip, non-temporal CLV loads
// and stores, grid = resident blocks.
constexpr int kU64 = 2, kU32 = 4;
constexpr int kGridMul64 = 1, kGridMul32 = 1;
constexpr bool kNt = false;
constexpr bool kNtl64 = true;
constexpr int kMinWaves = 1;

// Co-resident 256-thread blocks of `kernel` on the current device (cached per
// kernel; the grid-stride kernels launch at most this many).
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

template <typename T, int U, bool kSum>
hipError_t launch_dna_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_kernel<T, U, kSum, kNt, kMinWaves>;
  const int64_t sites_per_block = (int64_t)kWavesPerBlock * 16 * U;
  int64_t blocks = (a.n + sites_per_block - 1) / sites_per_block;
  const int64_t cap =
      max_blocks > 0 ? max_blocks : (int64_t)kGridMul32 * resident_blocks((const void *)kernel, cache);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, (const T *)a.x1,
                     (const T *)a.x2, (T *)a.x3, (const T *)a.EV, (const T *)a.left,
                     (const T *)a.right, a.wgt, a.scaler, a.n, a.ws, a.scaler_sum);
  return hipGetLastError();
}

template <int U, bool kSum>
hipError_t launch_pair_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
  static int cache = 0;
  auto kernel = &dev::plf_dna_f64_pair_kernel<U, kSum, kMinWaves, kNtl64>;
  const int64_t sites_per_block = (int64_t)kWavesPerBlock * 16 * U;
  int64_t blocks = (a.n + sites_per_block - 1) / sites_per_block;
  const int64_t cap =
      max_blocks > 0 ? max_blocks : (int64_t)kGridMul64 * resident_blocks((const void *)kernel, cache);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, (const double *)a.x1,
                     (const double *)a.x2, (double *)a.x3, (const double *)a.EV,
                     (const double *)a.left, (const double *)a.right, a.wgt, a.scaler, a.n, a.ws,
                     a.scaler_sum);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_plf_dna_f32(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_dna_t<float, kU32, true>(a, max_blocks, s)
                      : launch_dna_t<float, kU32, false>(a, max_blocks, s);
}
hipError_t launch_plf_dna_f64(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_pair_t<kU64, true>(a, max_blocks, s)
                      : launch_pair_t<kU64, false>(a, max_blocks, s);
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

}  // namespace plfx
