// plf_prot_valu.hip -- BASELINE configs[4] as its config line words it: a
// protein (S = 20) inner node with the 20x20 P matrices tiled in LDS and the
// matvecs on the VALU, not the matrix cores, in FMA mode (PLFX_FMA |
// PLFX_VALU): plf()'s loop (app/src/plf.cpp:19-65 with 4 -> 20) with every
// multiply-add fused in the same order, u = fma(x[l], P[k][l], u) and
// x3 = fma(U[k], EV[k][l], x3) from +0.0.  That is the oracle's fma
// restatement and, bit for bit, what the matrix-core kernels compute (their
// v_mfma_f64 tiles are k-ordered fma chains), at half the VALU instructions
// of the exact mode's separate roundings.  The body is the exact kernel's
// (plf_prot.hpp prot_lds_body: wave = category, lane = site, child tiles
// staged through LDS, matrices broadcast from LDS, EV rows as SGPR operands,
// ballot rescale) with kFma set.  Its own translation unit, so the other
// kernels' code objects (and the PMC records stamped with them) stay as they
// are.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#define PLFX_SECONDARY_TU  // plf_dna.hpp's non-template kernel lives in plf_kernels.hip
#include "plf_kernels.hpp"
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

template <bool kSum, int kRows>
__global__ void __launch_bounds__(kBlock, 2)
plf_prot_valu_fma_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                         double *__restrict__ x3, const double *__restrict__ EV,
                         const double *__restrict__ left, const double *__restrict__ right,
                         const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                         unsigned long long *ws, int64_t *scaler_sum) {
  prot_lds_body<double, kSum, 0, kRows, true, false, true>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws,
                                                           scaler_sum, nullptr);
}

}  // namespace dev

namespace {

// rows per chain group (phases 1 and 2): kRows independent fma chains per wave
constexpr int kValuRows = 10;

template <bool kSum>
hipError_t launch_valu_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
  auto kernel = &dev::plf_prot_valu_fma_kernel<kSum, kValuRows>;
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
