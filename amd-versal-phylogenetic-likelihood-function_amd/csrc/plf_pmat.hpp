// plf_pmat.hpp -- P-matrix generation on the device.
//
// For branch b (length t_b) and rate category c (rate r_c), with the model's
// eigensystem Q = V diag(lambda) V^-1 (model.cpp plfx_model_eigen):
//   STATE convention: out[b][c][k][l] = P_c(t_b)[k][l]
//                                     = sum_m V[k][m] exp(lambda_m r_c t_b) Vi[m][l]
//     (with EV = I, plf() is then Felsenstein's pruning step on state-space CLVs)
//   EIGEN convention: out[b][c][k][l] = V[k][l] exp(lambda_l r_c t_b)
//     (with EV[k][l] = Vi[l][k], plf() runs on CLVs stored in eigen coordinates
//     -- the RAxML formulation the reference's EV/left/right argument names
//     come from: ump = P x in state space, x3 = V^-1 (umpL * umpR).)
// The layout [b][c][k][l] is the traverse pmats layout (plfx.h section 6):
// branch 2j / 2j+1 = left / right of P-matrix pair j.  Computed in f64, stored
// as T.  One thread per output value; tiny next to the PLF (C*S*S values per
// branch), so it is latency- not bandwidth-bound.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace plfx {
namespace dev {

template <typename T, bool kEigen>
__global__ void __launch_bounds__(256)
pmatrix_kernel(const double *__restrict__ eigen, int S, const double *__restrict__ rates, int ncat,
               const double *__restrict__ blen, int64_t nbranch, T *__restrict__ out) {
  const int64_t per_branch = (int64_t)ncat * S * S;
  const int64_t total = nbranch * per_branch;
  const double *lam = eigen, *V = eigen + S, *Vi = eigen + S + S * S;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / per_branch;
    const int r = (int)(e - b * per_branch);
    const int c = r / (S * S), k = (r / S) % S, l = r % S;
    const double rt = rates[c] * blen[b];
    double v;
    if constexpr (kEigen) {
      v = V[k * S + l] * exp(lam[l] * rt);
    } else {
      v = 0.0;
      for (int m = 0; m < S; m++) v += V[k * S + m] * exp(lam[m] * rt) * Vi[m * S + l];
    }
    out[e] = (T)v;
  }
}

}  // namespace dev
}  // namespace plfx
