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

#define PLFX_SECONDARY_TU  // plf_dna.hpp's non-template kernel lives in plf_kernels.hip
#include "plf_kernels.hpp"
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

template <bool kSum, int kRows, int kCols, int kMinW>
__global__ void __launch_bounds__(kBlock, kMinW)
plf_prot_valu_fma_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                         double *__restrict__ x3, const double *__restrict__ EV,
                         const double *__restrict__ left, const double *__restrict__ right,
                         const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                         unsigned long long *ws, int64_t *scaler_sum) {
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
        for (int q = 0; q < kCols; q++)
#pragma unroll
          for (int j = 0; j < kRows; j++)
            u[j] = __builtin_fma(x[lc + q], cur[j][q], lc + q == 0 ? 0.0 : u[j]);
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
  V pf[K];  // the next child tile in flight
  if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(x1, (int64_t)blockIdx.x * 64, n, pf);
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    double U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int wsite = kSum ? wgt_at(wgt, sq, ws) : 0;
    {
      double a[S];
      tile_put<double>(tile, pf);
      __syncthreads();
      tile_fetch<double>(x2, base, n, pf);  // this trip's x2 while phase 1 runs
      row_read<double>(tile, lane, c, a);
      __syncthreads();
      dot(PL, a, [&](int k, double u) { U[k] = u; });
    }
    {
      double b[S];
      tile_put<double>(tile, pf);
      __syncthreads();
      if (base + stride < n) tile_fetch<double>(x1, base + stride, n, pf);  // the next trip's x1
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
#pragma unroll
          for (int j = 0; j < kPh3; j++) v[j] = __builtin_fma(U[k], er[j], v[j]);
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

namespace {

// 5 rows per chain group, 2-column double-buffered chunks, 3 waves per SIMD
// (profiles/r06_protein_valu_forms.log, form 2)
constexpr int kValuRows = 5, kValuCols = 2, kValuMinW = 3;

template <bool kSum>
hipError_t launch_valu_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
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
