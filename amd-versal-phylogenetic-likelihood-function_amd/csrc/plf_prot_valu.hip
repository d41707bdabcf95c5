// plf_prot_valu.hip -- BASELINE configs[4] as its config line words it: a
// protein (S = 20) inner node, f64, the matvecs on the VALU, not the matrix
// cores, in FMA mode (PLFX_FMA | PLFX_VALU): plf()'s loop
// (app/src/plf.cpp:19-65 with 4 -> 20) with every multiply-add fused in the
// same order, u = fma(x[l], P[k][l], u) and x3 = fma(U[k], EV[k][l], x3) from
// +0.0.  That is the oracle's fma restatement and, bit for bit, what the
// matrix-core kernels compute (their v_mfma_f64 tiles are k-ordered fma
// chains), at half the VALU instructions of the exact mode's separate
// roundings.  Its own translation unit, so the other kernels' code objects
// (and the PMC records stamped with them) stay as they are.
//
// Wave = category c, lane = site of a 64-site tile; each child tile is staged
// through LDS with coalesced non-temporal loads (plf_prot.hpp tile_fetch /
// tile_put / row_read, the exact kernel's padded layout) and the next one is
// in flight in registers during the current phase.  The matrices are NOT in
// LDS: P_c and EV rows are wave-uniform, so they are scalar loads straight
// from global memory used as SGPR operands.  With the matrices broadcast from
// LDS (the exact kernel's form with fused chains) each ds_read_b128 fed only
// two fma and the LDS, shared by the CU's four SIMDs, bound it at 0.55 of
// 8 TB/s; with scalar operands LDS holds only the 41-KB tile and three blocks
// (3 waves per SIMD) share a CU: 0.60-0.62 (profiles/r06_protein_valu_forms.log:
// twelve forms A/B'd on two boxes -- row groups of 4/5/10, column chunks
// loaded after the previous one or double-buffered, 2 vs 3 waves per SIMD,
// phase 3 straight to the tile, the device-wide tile queue; the forms are in
// plf_prot_valu.hip@68b50fc).
// Phases: U[k] = fma-chain_l x1[l] P_L[k][l] (kRows rows k at a time: kRows
// independent chains per wave; the columns in chunks of kCols, the next
// chunk's scalar loads issued before this chunk's fma), U[k] *= the same over
// x2 and P_R, x3[l] = fma-chain_k U[k] EV[k][l] (10 states at a time); then
// plf()'s scale test as a wave ballot per category, combined over the block's
// four waves in LDS, and the rescale as one exact v_ldexp per value.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "plf_kernels.hpp"
#include "plf_prot_valu.hpp"

namespace plfx {
namespace dev {

template <bool kSum, int kRows, int kCols, int kMinW>
__global__ void __launch_bounds__(kBlock, kMinW)
plf_prot_valu_fma_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                         double *__restrict__ x3, const double *__restrict__ EV,
                         const double *__restrict__ left, const double *__restrict__ right,
                         const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                         unsigned long long *ws, int64_t *scaler_sum) {
  prot_valu_body<kSum, false, kRows, kCols>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum);
}

}  // namespace dev

namespace {

// 5 rows per chain group, 2-column double-buffered chunks, 3 waves per SIMD
// (profiles/r06_protein_valu_forms.log, form 2)
constexpr int kValuRows = 5, kValuCols = 2, kValuMinW = 3;

template <bool kSum>
hipError_t launch_valu_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
  // the next child tile stays in flight in registers during the phases (168
  // VGPRs, 21 spilled): fetching it right before use instead (no spill) is
  // +0.5 % with two streams in flight but -3 % alone
  // (plf_prot_valu.hip@95468ac), and reading the child's row from the LDS
  // tile per column chunk (2 spilled) -2 % / -6 % (plf_prot_valu.hpp@d4b0f72;
  // profiles/r06_probe_valu_nopf.log)
  auto kernel = &dev::plf_prot_valu_fma_kernel<kSum, kValuRows, kValuCols, kValuMinW>;
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)kernel, dev::kBlock, 0) !=
            hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    resident = per_cu * std::max(cus, 1);
  }
  int64_t gx = (a.n + 63) / 64;  // one 64-site tile per block trip
  gx = std::max<int64_t>(1, std::min<int64_t>(gx, max_blocks > 0 ? max_blocks : resident));
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(dev::kBlock), 0, s, (const double *)a.x1,
                     (const double *)a.x2, (double *)a.x3, (const double *)a.EV, (const double *)a.left,
                     (const double *)a.right, a.wgt, a.scaler, a.n, a.ws, a.scaler_sum);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_plf_prot_valu_f64(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_valu_t<true>(a, max_blocks, s) : launch_valu_t<false>(a, max_blocks, s);
}

}  // namespace plfx
