// plf_prot_valu_exact.hip -- BASELINE configs[4] in exact mode (plf()'s
// separate multiply and add, app/src/plf.cpp:19-65 with 4 -> 20, f64) with the
// P matrices and EV rows as wave-uniform scalar loads (SGPR operands) instead
// of LDS broadcasts: LDS holds only the staged child tile, so three blocks
// share a CU (3 waves per SIMD, where the LDS-matrix kernel's 70.8 KB allow
// two).  Same operations in the same order as plf_prot_lds_kernel, so the
// results are bit-identical to it and to plf()'s double loop.  The body is
// plf_prot_valu.hpp's; its own translation unit, so no other kernel's code
// object (nor the PMC records stamped with them) moves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "plf_kernels.hpp"
#include "plf_prot_valu.hpp"

namespace plfx {
namespace dev {

template <bool kSum, int kRows, int kCols, int kMinW>
__global__ void __launch_bounds__(kBlock, kMinW)
plf_prot_valu_exact_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                           double *__restrict__ x3, const double *__restrict__ EV,
                           const double *__restrict__ left, const double *__restrict__ right,
                           const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                           unsigned long long *ws, int64_t *scaler_sum) {
  // kPrefetch = false: each child tile fetched right before its phase, none
  // held in registers across a phase -- 149 VGPRs and no spill instead of
  // 168 with 23 spilled: +1-2 % alone and with two streams in flight
  // (profiles/r06_probe_valu_nopf.log, plf_prot_valu_exact.hip@95468ac)
  prot_valu_body<kSum, true, kRows, kCols, false>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws,
                                                  scaler_sum);
}

}  // namespace dev

namespace {

template <bool kSum, int kRows, int kCols, int kMinW>
hipError_t launch_k(const DnaArgs &a, int max_blocks, hipStream_t s) {
  auto kernel = &dev::plf_prot_valu_exact_kernel<kSum, kRows, kCols, kMinW>;
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
  int64_t gx = (a.n + 63) / 64;
  gx = std::max<int64_t>(1, std::min<int64_t>(gx, max_blocks > 0 ? max_blocks : resident));
  hipLaunchKernelGGL(kernel, dim3((unsigned)gx), dim3(dev::kBlock), 0, s, (const double *)a.x1,
                     (const double *)a.x2, (double *)a.x3, (const double *)a.EV, (const double *)a.left,
                     (const double *)a.right, a.wgt, a.scaler, a.n, a.ws, a.scaler_sum);
  return hipGetLastError();
}

// 4 rows per chain group, 2-column double-buffered scalar chunks, 3 waves per
// SIMD: 130.0-130.5 us at 2^18 sites against the LDS-matrix kernel's 143.6-143.9
// on the same box (profiles/r06_protein_exact_forms.log, form 3; five forms
// A/B'd, plf_prot_valu_exact.hip@5ad7aa8)
template <bool kSum>
hipError_t launch_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return launch_k<kSum, 4, 2, 3>(a, max_blocks, s);
}

}  // namespace

hipError_t launch_plf_prot_valu_exact_f64(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_t<true>(a, max_blocks, s) : launch_t<false>(a, max_blocks, s);
}

}  // namespace plfx
