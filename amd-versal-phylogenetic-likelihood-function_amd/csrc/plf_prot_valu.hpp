// plf_prot_valu.hpp -- the body of the VALU protein kernels (f64, S = 20)
// whose P matrices and EV rows are wave-uniform scalar loads used as SGPR
// operands, LDS holding only the staged child tile: FMA mode
// (plf_prot_valu.hip) and exact mode (plf_prot_valu_exact.hip), each
// kernel in its own translation unit.  See plf_prot_valu.hip for the design
// and the measurements.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#define PLFX_SECONDARY_TU  // plf_dna.hpp's non-template kernel lives in plf_kernels.hip
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

// kExact: plf()'s separate multiply and add in its order (bit-identical to
// the exact LDS kernel and to plf()'s double loop); else every multiply-add
// fused (bit-identical to the matrix-core kernels and the fma restatement).
template <bool kSum, bool kExact, int kRows, int kCols, bool kPrefetch = true>
__device__ __forceinline__ void prot_valu_body(const double *__restrict__ x1, const double *__restrict__ x2,
                                               double *__restrict__ x3, const double *__restrict__ EV,
                                               const double *__restrict__ left,
                                               const double *__restrict__ right,
                                               const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                               int64_t n, unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20, kPh3 = 10;
  static_assert(S % kRows == 0 && S % kCols == 0, "row groups and column chunks divide 20");
  using PT = ProtTile<double>;
  using V = typename PT::V;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const double m = Num<double>::minlik();
  __shared__ V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  // fn(k, sum_l x[l] * P[k][l]) for every row k, fused, from +0.0; P = this
  // wave's category's matrix (wave-uniform: scalar loads, SGPR operands)
  auto dot = [&](const double *P, const double (&x)[S], auto &&fn) {
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const double *G = P + gk * kRows * S;
      double u[kRows], cur[kRows][kCols], nxt[kRows][kCols];
#pragma unroll
      for (int j = 0; j < kRows; j++)
#pragma unroll
        for (int q = 0; q < kCols; q++) cur[j][q] = G[j * S + q];
#pragma unroll
      for (int lc = 0; lc < S; lc += kCols) {
        if (lc + kCols < S) {
#pragma unroll
          for (int j = 0; j < kRows; j++)
#pragma unroll
            for (int q = 0; q < kCols; q++) nxt[j][q] = G[j * S + lc + kCols + q];
        }
#pragma unroll
        for (int q = 0; q < kCols; q++) {
          if constexpr (kExact) {
            // plf()'s separate roundings: all kRows products, then all kRows
            // adds (chains start at the first product, as the exact kernel's)
            double pr[kRows];
#pragma unroll
            for (int j = 0; j < kRows; j++) pr[j] = x[lc + q] * cur[j][q];
            pin_chains(pr);
#pragma unroll
            for (int j = 0; j < kRows; j++) u[j] = lc + q == 0 ? pr[j] : u[j] + pr[j];
          } else {
#pragma unroll
            for (int j = 0; j < kRows; j++)
              u[j] = __builtin_fma(x[lc + q], cur[j][q], lc + q == 0 ? 0.0 : u[j]);
          }
        }
        pin_chains(u);
#pragma unroll
        for (int j = 0; j < kRows; j++)
#pragma unroll
          for (int q = 0; q < kCols; q++) cur[j][q] = nxt[j][q];
      }
#pragma unroll
      for (int j = 0; j < kRows; j++) fn(gk * kRows + j, u[j]);
    }
  };
  const double *PL = left + c * S * S, *PR = right + c * S * S;
  const int64_t stride = (int64_t)gridDim.x * 64;
  constexpr int K = PT::kChunks / kBlock;
  V pf[K];  // the next child tile in flight (kPrefetch)
  if (kPrefetch && (int64_t)blockIdx.x * 64 < n) tile_fetch<double>(x1, (int64_t)blockIdx.x * 64, n, pf);
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    double U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int wsite = kSum ? wgt_at(wgt, sq, ws) : 0;
    {
      double a[S];
      if constexpr (!kPrefetch) tile_fetch<double>(x1, base, n, pf);
      tile_put<double>(tile, pf);
      __syncthreads();
      if constexpr (kPrefetch) tile_fetch<double>(x2, base, n, pf);  // this trip's x2 while phase 1 runs
      row_read<double>(tile, lane, c, a);
      __syncthreads();
      dot(PL, a, [&](int k, double u) { U[k] = u; });
    }
    {
      double b[S];
      if constexpr (!kPrefetch) tile_fetch<double>(x2, base, n, pf);
      tile_put<double>(tile, pf);
      __syncthreads();
      if (kPrefetch && base + stride < n) tile_fetch<double>(x1, base + stride, n, pf);  // the next trip's x1
      row_read<double>(tile, lane, c, b);
      __syncthreads();
      dot(PR, b, [&](int k, double u) { U[k] = U[k] * u; });  // prod[k] = umpL[k] * umpR[k]
    }
    // phase 3: O[l] = sum_k U[k] * EV[k][l], fused, from +0.0
    double O[S];
    {
      double tok = 0.0;
#pragma unroll
      for (int h = 0; h < S / kPh3; h++) {
        double v[kPh3];
#pragma unroll
        for (int j = 0; j < kPh3; j++) v[j] = 0.0;
#pragma unroll
        for (int k = 0; k < S; k++) {
          int so = 0;
          asm volatile("" : "+s"(so) : "v"(tok));  // EV row k after the previous row's chains
          const double *er = EV + so + k * S + h * kPh3;
          if constexpr (kExact) {
            double pr[kPh3];
#pragma unroll
            for (int j = 0; j < kPh3; j++) pr[j] = U[k] * er[j];
            pin_chains(pr);
#pragma unroll
            for (int j = 0; j < kPh3; j++) v[j] += pr[j];
          } else {
#pragma unroll
            for (int j = 0; j < kPh3; j++) v[j] = __builtin_fma(U[k], er[j], v[j]);
          }
          pin_chains(v);
          tok = v[kPh3 - 1];
        }
#pragma unroll
        for (int j = 0; j < kPh3; j++) O[h * kPh3 + j] = v[j];
      }
    }
    bool small = base + lane < n;
#pragma unroll
    for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[l]) < m);
    const unsigned long long mk = __ballot(small);
    if (lane == 0) small_mask[c] = mk;
    __syncthreads();  // also: every wave is done reading x2 from the tile
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    const bool sc = (all >> lane) & 1ull;
    int e = sc ? 32 : 0;  // x 2^32 as one exact v_ldexp per value (plf_prot.hpp)
    asm volatile("" : "+v"(e));
#pragma unroll
    for (int l = 0; l < S; l++) O[l] = ldexp(O[l], e);
    row_write<double>(tile, lane, c, O);
    const int64_t site = base + lane;
    if (site < n && c == 0) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wsite;
    }
    __syncthreads();
    tile_store<double>(x3, base, n, tile);
    __syncthreads();  // tile and small_mask are reused by the next trip
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
