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
// drained), a two-level ticket (kWsWords words, zero at rest) elects the last
// block, which sums the slots in index order (sc1 loads) -- the result does
// not depend on block arrival order.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "plf_dna.hpp"
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

constexpr double kLogMinLik = -22.18070977791824990137;  // log(2^-32) = -32 ln 2

// The fixed-order cross-block part of the root lnL (both kernels): the block's
// lanes' acc into a fixed slot, the last block (two-level election) sums the
// slots in index order and adds the scaler correction.
__device__ __forceinline__ void lnl_finish(double acc, double *partials, unsigned long long *ticket, double *out,
                                  const int64_t *__restrict__ scaler_sums, int nsums) {
  const int lane = threadIdx.x & 63;
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
    // two-level election (a single counter serialises ~12 ns per arrival:
    // 20 us for 1800 blocks): slot counters 128 B apart, then a top counter;
    // both return to zero
    const unsigned long long G = gridDim.x, slot = blockIdx.x % kSlots;
    const unsigned long long nslots = G < kSlots ? G : kSlots;
    const unsigned long long arrivals = (G - slot + kSlots - 1) / kSlots;
    int is_last = 0;
    if (__hip_atomic_fetch_add(ticket + slot * 16, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) == arrivals - 1) {
      __hip_atomic_store(ticket + slot * 16, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      is_last = __hip_atomic_fetch_add(ticket + kSlots * 16, 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) == nslots - 1;
    }
    last = is_last;
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
    __hip_atomic_store(ticket + kSlots * 16, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// C lanes per site (lane = category); S states per lane.  A loop trip covers C
// wave steps (C x 64/C sites): all loads first, then each site's L is built in
// its C lanes (ascending s, then c, as the oracle) and lane c takes the log of
// step c's site -- every lane evaluates one log per trip instead of one lane
// in C (the log, not HBM, bounded the one-step form: 51 us for 2^20 DNA sites).
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
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * SPW * C;
  const int64_t nlast = n - 1;
  for (int64_t base = wave * SPW * C; base < n; base += stride) {
    // every load of the trip first and unconditionally (clamped to the last site,
    // results unused past n), the weight of this lane's log site with them: one
    // memory latency per trip (a conditional weight load after the math was a
    // second one, and the kernel runs only a few trips per wave)
    T v[C][S];
#pragma unroll
    for (int u = 0; u < C; u++) {
      const int64_t site = base + u * SPW + q;
      const T *xs = x + (site < n ? site : nlast) * V + c * S;  // 16-B aligned: S*sizeof(T) % 16 == 0
      if constexpr (sizeof(T) == 8) {
#pragma unroll
        for (int s = 0; s < S; s += 2) {
          const f64x2 w = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(xs + s));
          v[u][s] = w.x;
          v[u][s + 1] = w.y;
        }
      } else {
#pragma unroll
        for (int s = 0; s < S; s += 4) {
          const f32x4 w = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(xs + s));
          v[u][s] = w.x; v[u][s + 1] = w.y; v[u][s + 2] = w.z; v[u][s + 3] = w.w;
        }
      }
    }
    const int64_t site = base + c * SPW + q;  // this lane's log site (step c)
    const bool valid = site < n;
    const int wv = wgt_at(wgt, valid ? site : nlast, partials);
    __builtin_amdgcn_sched_barrier(0);  // keeps the weight load with the CLV loads
    double mine = 1.0;  // L of step c's site
#pragma unroll
    for (int u = 0; u < C; u++) {
      double t = 0.0;
#pragma unroll
      for (int s = 0; s < S; s++) t += fr[s] * (double)v[u][s];
      double L = 0.0;
#pragma unroll
      for (int k = 0; k < C; k++) L += cw[k] * __shfl(t, (lane / C) * C + k);
      if (u == c) mine = L;
    }
    if (valid) {
      const double l = log(mine);
      if (site_lnl) site_lnl[site] = l;
      acc += (double)wv * l;
    }
  }
  lnl_finish(acc, partials, ticket, out, scaler_sums, nsums);
}

// S = 20 (protein), C = 4: the per-lane 160-B rows of the C-lanes-per-site
// form are 16-B loads 160 B apart across the wave (64 cache lines per load
// instruction: 94 us for 2^18 f64 sites, 22 % of peak).  Here a 256-thread
// block stages 64-site tiles through LDS with coalesced loads (the protein
// kernels' ProtTile, the next tile in flight in registers), wave w = category
// w takes its 20 values per site from the tile (lane = site), the four
// category sums meet in LDS and wave 0 forms L (the same operations in the
// same order as root_lnl_kernel: ascending s from +0.0, then ascending c) and
// its log.  Per-site values are bit-identical to the C-lanes form; the lnL
// total sums them in another (fixed) order.
template <typename T>
__global__ void __launch_bounds__(kBlock)
root_lnl_prot_kernel(const T *__restrict__ x, int64_t n, const double *__restrict__ catw,
                     const double *__restrict__ freq, const int32_t *__restrict__ wgt,
                     const int64_t *scaler_sums, int nsums, double *partials,
                     unsigned long long *ticket, double *out, double *__restrict__ site_lnl) {
  constexpr int S = 20, C = 4;
  using PT = ProtTile<T>;
  constexpr int K = PT::kChunks / kBlock;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  double fr[S];
#pragma unroll
  for (int s = 0; s < S; s++) fr[s] = freq ? freq[s] : 1.0 / S;
  double cw[C];
#pragma unroll
  for (int k = 0; k < C; k++) cw[k] = catw ? catw[k] : 1.0 / C;
  __shared__ typename PT::V tile[64 * PT::kStride];
  __shared__ double tc[C][64];
  const int64_t stride = (int64_t)gridDim.x * 64;
  typename PT::V pf[K];
  if ((int64_t)blockIdx.x * 64 < n) tile_fetch<T>(x, (int64_t)blockIdx.x * 64, n, pf);
  double acc = 0.0;
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    const int64_t site = base + lane;
    const bool valid = site < n;
    const int wv = wgt_at(wgt, valid ? site : n - 1, partials);
    tile_put<T>(tile, pf);
    __syncthreads();
    if (base + stride < n) tile_fetch<T>(x, base + stride, n, pf);
    T v[S];
    row_read<T>(tile, lane, c, v);
    double t = 0.0;
#pragma unroll
    for (int s = 0; s < S; s++) t += fr[s] * (double)v[s];
    tc[c][lane] = t;
    __syncthreads();  // also: every wave is done reading the tile
    if (c == 0 && valid) {
      double L = 0.0;
#pragma unroll
      for (int k = 0; k < C; k++) L += cw[k] * tc[k][lane];
      const double l = log(L);
      if (site_lnl) site_lnl[site] = l;
      acc += (double)wv * l;
    }
    __syncthreads();  // tc is rewritten by the next trip
  }
  lnl_finish(acc, partials, ticket, out, scaler_sums, nsums);
}

}  // namespace dev
}  // namespace plfx
