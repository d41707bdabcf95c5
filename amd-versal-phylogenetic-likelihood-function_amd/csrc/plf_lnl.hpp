// plf_lnl.hpp -- root log-likelihood of a CLV (extension: the reference has no
// evaluate step; modelled on RAxML's evaluate over the GTR+Gamma
// CLVs that plf() produces, app/src/plf.cpp being RAxML's newview inner-inner
// case).
//
//   L_i   = sum_c catw[c] * sum_s freq[s] * x[i][c][s]     (ascending s, then c)
//   lnL   = sum_i wgt_i * log(L_i) + (sum of the inner nodes' scalerIncrements)
//                                    * log(2^-32)
// The scaling correction is exact with per-node totals: every rescale of site
// i multiplied L_i by 2^32, and sum_i wgt_i * count_i = sum_nodes
// scalerIncrement_node (plf.cpp:58-64).
//
// Deterministic: per-block partial sums land in fixed slots (sc1 stores,
// drained), a ticket elects the last block, which sums the slots in index
// order (sc1 loads) -- the result does not depend on block arrival order.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "plf_dna.hpp"

namespace plfx {
namespace dev {

constexpr double kLogMinLik = -22.18070977791824990137;  // log(2^-32) = -32 ln 2

// C lanes per site (lane = category); S states per lane.
template <typename T, int S, int C>
__global__ void __launch_bounds__(kBlock)
root_lnl_kernel(const T *__restrict__ x, int64_t n, const double *__restrict__ catw,
                const double *__restrict__ freq, const int32_t *__restrict__ wgt,
                const int64_t *__restrict__ scaler_sums, int nsums, double *partials,
                unsigned long long *ticket, double *out, double *__restrict__ site_lnl) {
  static_assert(64 % C == 0, "categories must divide the wave");
  constexpr int V = S * C;
  constexpr int SPW = 64 / C;  // sites per wave step
  const int lane = threadIdx.x & 63;
  const int c = lane % C;
  const int q = lane / C;
  double fr[S];
#pragma unroll
  for (int s = 0; s < S; s++) fr[s] = freq ? freq[s] : 1.0 / S;
  double cw[C];
#pragma unroll
  for (int k = 0; k < C; k++) cw[k] = catw ? catw[k] : 1.0 / C;

  double acc = 0.0;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * SPW;
  for (int64_t base = wave * SPW; base < n; base += stride) {
    const int64_t site = base + q;
    const bool valid = site < n;
    double t = 0.0;
    if (valid) {
      const T *xs = x + site * V + c * S;
#pragma unroll
      for (int s = 0; s < S; s++) t += fr[s] * (double)xs[s];
    }
    double L = 0.0;
#pragma unroll
    for (int k = 0; k < C; k++) L += cw[k] * __shfl(t, (lane / C) * C + k);
    if (valid && c == 0) {
      const double l = log(L);
      if (site_lnl) site_lnl[site] = l;
      acc += (wgt ? (double)wgt[site] : 1.0) * l;
    }
  }
  // fixed-order block reduction
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  __shared__ double part[kWavesPerBlock];
  __shared__ int last;
  if (lane == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double b = 0.0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; i++) b += part[i];
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(partials) + blockIdx.x,
                       __builtin_bit_cast(unsigned long long, b), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t =
        __hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!last) return;
  double v = 0.0;
  for (unsigned i = threadIdx.x; i < gridDim.x; i += kBlock)
    v += __builtin_bit_cast(double, __hip_atomic_load(
                                        reinterpret_cast<unsigned long long *>(partials) + i,
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if (lane == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; i++) tot += part[i];
    long long nsc = 0;
    for (int i = 0; i < nsums; i++) nsc += scaler_sums[i];
    *out = tot + (double)nsc * kLogMinLik;
    __hip_atomic_store(ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace dev
}  // namespace plfx
