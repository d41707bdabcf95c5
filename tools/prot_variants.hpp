// prot_variants.hpp -- experimental protein (S=20) exact-mode kernels for the
// tuning harness tools/tune_prot.hip (not product code).
//
// Phased variant of plf_prot_kernel (csrc/plf_prot.hpp): each lane owns NS
// sites (sites base + s*64 + lane) of one category (wave = category) and runs
//   phase 1: U[s][k]  = sum_l x1[s][l] * PL[k][l]        (ascending l)
//   phase 2: U[s][k] *= sum_l x2[s][l] * PR[k][l]        (prod = umpL * umpR)
//   phase 3: O[s][l]  = sum_k U[s][k] * EV[k][l]         (ascending k)
// -- every value with plf()'s operation order, so the results are bit-identical
// to the product kernel.  One broadcast matrix value serves NS sites.
// kScalar: matrix values come from scalar loads (s_load through the scalar
// cache) instead of v_readlane broadcasts of lane-distributed registers.
#pragma once
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

template <bool kScalar, int NS, int kMinBlocks = 2>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
prot_phased_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                   double *__restrict__ x3, const double *__restrict__ EV,
                   const double *__restrict__ left, const double *__restrict__ right,
                   const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                   unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  constexpr int R = (S * S + 63) / 64;
  double ML[R], MR[R], ME[R];
  const double *gL = left + c * S * S, *gR = right + c * S * S, *gE = EV;
  if constexpr (!kScalar) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int e = r * 64 + lane;
      ML[r] = e < S * S ? gL[e] : 0.0;
      MR[r] = e < S * S ? gR[e] : 0.0;
      ME[r] = e < S * S ? EV[e] : 0.0;
    }
  }
  auto mL = [&](int e) { if constexpr (kScalar) return gL[e]; else return bcast<double>(ML, e); };
  auto mR = [&](int e) { if constexpr (kScalar) return gR[e]; else return bcast<double>(MR, e); };
  auto mE = [&](int e) { if constexpr (kScalar) return gE[e]; else return bcast<double>(ME, e); };
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock][NS];
  long long acc = 0;
  for (int64_t base = (int64_t)blockIdx.x * 64 * NS; base < n; base += (int64_t)gridDim.x * 64 * NS) {
    // opaque per trip: keeps the 3 x 400 broadcasts / scalar loads inside the
    // loop instead of hoisted (and spilled) as loop invariants
    if constexpr (kScalar) {
      asm volatile("" : "+s"(gL), "+s"(gR), "+s"(gE));
    } else {
#pragma unroll
      for (int r = 0; r < R; r++) asm volatile("" : "+v"(ML[r]), "+v"(MR[r]), "+v"(ME[r]));
    }
    double U[NS][S];
    {
      double a[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x1, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, a[s]);
        __syncthreads();
      }
#pragma unroll
      for (int k = 0; k < S; k++) {
        double u[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) u[s] = 0.0;
#pragma unroll
        for (int l = 0; l < S; l++) {
          const double p = mL(k * S + l);
#pragma unroll
          for (int s = 0; s < NS; s++) u[s] += a[s][l] * p;
        }
#pragma unroll
        for (int s = 0; s < NS; s++) U[s][k] = u[s];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    {
      double b[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x2, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, b[s]);
        __syncthreads();
      }
#pragma unroll
      for (int k = 0; k < S; k++) {
        double u[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) u[s] = 0.0;
#pragma unroll
        for (int l = 0; l < S; l++) {
          const double p = mR(k * S + l);
#pragma unroll
          for (int s = 0; s < NS; s++) u[s] += b[s][l] * p;
        }
#pragma unroll
        for (int s = 0; s < NS; s++) U[s][k] = U[s][k] * u[s];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    double O[NS][S];
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int l = 0; l < S; l++) O[s][l] = 0.0;
#pragma unroll
    for (int k = 0; k < S; k++) {
#pragma unroll
      for (int l = 0; l < S; l++) {
        const double e = mE(k * S + l);
#pragma unroll
        for (int s = 0; s < NS; s++) O[s][l] += U[s][k] * e;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
      bool small = base + 64 * s + lane < n;
#pragma unroll
      for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[s][l]) < m);
      const unsigned long long mk = __ballot(small);
      if (lane == 0) small_mask[c][s] = mk;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const unsigned long long all =
          small_mask[0][s] & small_mask[1][s] & small_mask[2][s] & small_mask[3][s];
      const bool sc = (all >> lane) & 1ull;
#pragma unroll
      for (int l = 0; l < S; l++) {
        const double sv = O[s][l] * Num<double>::two32();
        O[s][l] = sc ? sv : O[s][l];
      }
      row_write<double>(tile, lane, c, O[s]);
      const int64_t site = base + 64 * s + lane;
      if (site < n && c == 0) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
      __syncthreads();
      tile_store<double>(x3, base + 64 * s, n, tile);
      __syncthreads();
    }
  }
  block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
