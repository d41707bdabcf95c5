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
#include <cstdlib>

#define PLFX_SECONDARY_TU  // plf_dna.hpp's non-template kernel lives in plf_kernels.hip
#include "plf_kernels.hpp"
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

// Wave = category c, lane = site of a 64-site tile (as the exact kernel), but
// the P matrices are read as SGPR operands -- wave-uniform scalar loads of
// P_c rows straight from global memory (the scalar cache holds the 25.6 KB of
// P_L / P_R) -- instead of LDS broadcasts: in FMA mode each LDS read fed only
// two fma, and the LDS, shared by the CU's four SIMDs, became the binding unit
// (the LDS-matrix form ran 0.55 of 8 TB/s, profiles/r06_protein_valu_*.log).
// EV rows come the same way (phase 3).  LDS then holds only the staged child
// tile (41 KB), so kMinW = 3 blocks of 4 waves can share a CU.
// Phases: U[k] = fma-chain_l x1[l] P_L[k][l] from +0.0 (kRows rows k at a
// time, kRows independent chains per wave, the columns in chunks of 4 so each
// row's four values are one scalar load), U[k] *= the same over x2 and P_R,
// x3[l] = fma-chain_k U[k] EV[k][l] from +0.0 (10 states at a time).
// the child tile's store with plf()'s rescale applied on the way out: chunk j
// of site s = j / 40 times 2^32 (one exact v_ldexp by 32 or 0 per value) when
// bit s of `scaled` is set (kOT: phase 3 writes its values unscaled)
__device__ __forceinline__ void tile_store_scaled(double *__restrict__ g, int64_t base, int64_t n,
                                                  const f64x2 *lds, unsigned long long scaled) {
  using PT = ProtTile<double>;
  constexpr int K = PT::kChunks / kBlock;
  f64x2 *dst = reinterpret_cast<f64x2 *>(g + base * 80);
  f64x2 v[K];
#pragma unroll
  for (int i = 0; i < K; i++) {
    const int j = threadIdx.x + i * kBlock;
    const int st = j / PT::kChunksPerSite, q = j - st * PT::kChunksPerSite;
    v[i] = lds[st * PT::kStride + q];
    int e = ((scaled >> st) & 1ull) ? 32 : 0;
    asm volatile("" : "+v"(e));
    v[i].x = ldexp(v[i].x, e);
    v[i].y = ldexp(v[i].y, e);
  }
  if (base + 64 <= n) {
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_nontemporal_store(v[i], dst + threadIdx.x + i * kBlock);
  } else {
    const int64_t lim = (n - base) * PT::kChunksPerSite;
#pragma unroll
    for (int i = 0; i < K; i++) {
      const int j = threadIdx.x + i * kBlock;
      if (j < lim) __builtin_nontemporal_store(v[i], dst + j);
    }
  }
}

template <bool kSum, int kRows, int kMinW, int kCols, bool kOT = false, bool kDyn = false>
__global__ void __launch_bounds__(kBlock, kMinW)
plf_prot_valu_fma_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                         double *__restrict__ x3, const double *__restrict__ EV,
                         const double *__restrict__ left, const double *__restrict__ right,
                         const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                         unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20, kPh3 = 10;
  static_assert(S % kRows == 0, "kRows divides 20");
  using PT = ProtTile<double>;
  using V = typename PT::V;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const double m = Num<double>::minlik();
  __shared__ V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  // sum_l x[l] * P[k][l] for the kRows rows of each group, fused, from +0.0;
  // P = this wave's category's matrix (wave-uniform: scalar loads)
  auto dot = [&](const double *P, const double (&x)[S], auto &&fn) {
    double tok = 0.0;
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const double *G = P + gk * kRows * S;
      double u[kRows];
      if constexpr (kCols == 0) {
        // chunks of 4 columns, each chunk's loads after the previous chunk's chains
#pragma unroll
        for (int lc = 0; lc < S; lc += 4) {
          int so = 0;
          asm volatile("" : "+s"(so) : "v"(tok));
          const double *pr = G + so + lc;
#pragma unroll
          for (int l = 0; l < 4; l++)
#pragma unroll
            for (int j = 0; j < kRows; j++)
              u[j] = __builtin_fma(x[lc + l], pr[j * S + l], lc + l == 0 ? 0.0 : u[j]);
          pin_chains(u);
          tok = u[kRows - 1];
        }
      } else {
        // chunks of kCols columns, the next chunk's scalar loads issued before
        // this chunk's fused multiply-adds
        double cur[kRows][kCols], nxt[kRows][kCols];
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
      }
#pragma unroll
      for (int j = 0; j < kRows; j++) fn(gk * kRows + j, u[j]);
    }
  };
  const double *PL = left + c * S * S, *PR = right + c * S * S;
  const int64_t stride = (int64_t)gridDim.x * 64;
  constexpr int K = PT::kChunks / kBlock;
  V pf[K];
  if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(x1, (int64_t)blockIdx.x * 64, n, pf);
  // kDyn: tiles after each block's first two come from the device-wide queue
  // of the matrix-core kernel (plf_prot.hpp ProtQueue: thread 0 publishes the
  // next trip's tile in qslot before the trip's first barrier and dequeues the
  // one after it during the trip), so the blocks' trip counts even out
  ProtQueue pq(ws, n, kDyn);
  __shared__ long long qslot;
  auto trip = [&](const int64_t base) -> int64_t {
    int64_t next = base + stride;
    double U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int wsite = kSum ? wgt_at(wgt, sq, ws) : 0;
    {
      double a[S];
      tile_put<double>(tile, pf);
      __syncthreads();
      if constexpr (kDyn) next = qslot;
      tile_fetch<double>(x2, base, n, pf);  // this trip's x2 while phase 1 runs
      row_read<double>(tile, lane, c, a);
      __syncthreads();
      dot(PL, a, [&](int k, double u) { U[k] = u; });
    }
    {
      double b[S];
      tile_put<double>(tile, pf);
      __syncthreads();
      if (next < n) tile_fetch<double>(x1, next, n, pf);  // the next trip's x1
      if constexpr (kDyn) pq.dequeue();
      row_read<double>(tile, lane, c, b);
      __syncthreads();
      dot(PR, b, [&](int k, double u) { U[k] = U[k] * u; });
    }
    // phase 3: O[l] = sum_k U[k] * EV[k][l], fused, from +0.0 (kOT: each pass's
    // values straight to the tile, unscaled, and into the site's small test)
    double O[kOT ? 1 : S];
    bool small = base + lane < n;
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
          asm volatile("" : "+s"(so) : "v"(tok));
          const double *er = EV + so + k * S + h * kPh3;
#pragma unroll
          for (int j = 0; j < kPh3; j++) v[j] = __builtin_fma(U[k], er[j], v[j]);
          pin_chains(v);
          tok = v[kPh3 - 1];
        }
        if constexpr (kOT) {
          V *xw = tile + lane * PT::kStride + c * (PT::kChunksPerSite / 4) + h * (kPh3 / 2);
#pragma unroll
          for (int j = 0; j < kPh3; j++) small = small && (__builtin_fabs(v[j]) < m);
#pragma unroll
          for (int j = 0; j < kPh3; j += 2) xw[j / 2] = V{v[j], v[j + 1]};
        } else {
#pragma unroll
          for (int j = 0; j < kPh3; j++) O[h * kPh3 + j] = v[j];
        }
      }
    }
    if constexpr (!kOT) {
#pragma unroll
      for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[l]) < m);
    }
    const unsigned long long mk = __ballot(small);
    if (lane == 0) small_mask[c] = mk;
    __syncthreads();  // also: every wave is done reading x2 from the tile
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    const bool sc = (all >> lane) & 1ull;
    const int64_t site = base + lane;
    if (site < n && c == 0) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wsite;
    }
    if constexpr (kOT) {
      tile_store_scaled(x3, base, n, tile, all);
    } else {
      int e = sc ? 32 : 0;  // x 2^32 as one exact v_ldexp per value (plf_prot.hpp)
      asm volatile("" : "+v"(e));
#pragma unroll
      for (int l = 0; l < S; l++) O[l] = ldexp(O[l], e);
      row_write<double>(tile, lane, c, O);
      __syncthreads();
      tile_store<double>(x3, base, n, tile);
    }
    __syncthreads();  // tile and small_mask are reused by the next trip
    return next;
  };
  if constexpr (kDyn) {
    int64_t base = (int64_t)blockIdx.x * 64;
    for (int i = 0; base < n; i++) {
      if (threadIdx.x == 0) qslot = pq.next_base(i);
      base = trip(base);
    }
    pq.finish();
  } else {
    for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) trip(base);
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev

namespace {

// rows per chain group (phases 1 and 2): kRows independent fma chains per
// wave; blocks per CU (launch bounds: kMinW waves per SIMD); kCols: 0 = chunks
// of 4 columns loaded after the previous chunk, else double-buffered chunks
// of kCols columns.  PLFX_VALU_FORM (A/B only) picks a form at first use.
template <bool kSum, int kRows, int kMinW, int kCols, bool kOT = false, bool kDyn = false>
hipError_t launch_valu_k(const DnaArgs &a, int max_blocks, hipStream_t s) {
  if (kDyn && !a.ws) return hipErrorInvalidValue;
  auto kernel = &dev::plf_prot_valu_fma_kernel<kSum, kRows, kMinW, kCols, kOT, kDyn>;
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

template <bool kSum>
hipError_t launch_valu_t(const DnaArgs &a, int max_blocks, hipStream_t s) {
  static int form = -1;
  if (form < 0) {
    const char *e = std::getenv("PLFX_VALU_FORM");
    form = e ? std::atoi(e) : 0;
  }
  switch (form) {
    case 1: return launch_valu_k<kSum, 5, 3, 1>(a, max_blocks, s);
    case 2: return launch_valu_k<kSum, 5, 3, 2>(a, max_blocks, s);
    case 3: return launch_valu_k<kSum, 4, 3, 1>(a, max_blocks, s);
    case 4: return launch_valu_k<kSum, 10, 3, 1>(a, max_blocks, s);
    case 5: return launch_valu_k<kSum, 5, 2, 0>(a, max_blocks, s);
    case 6: return launch_valu_k<kSum, 10, 2, 0>(a, max_blocks, s);
    case 7: return launch_valu_k<kSum, 5, 3, 0, true>(a, max_blocks, s);
    case 8: return launch_valu_k<kSum, 5, 3, 1, true>(a, max_blocks, s);
    case 9: return launch_valu_k<kSum, 5, 3, 2, false, true>(a, max_blocks, s);
    case 10: return launch_valu_k<kSum, 5, 3, 0, false, true>(a, max_blocks, s);
    case 11: return launch_valu_k<kSum, 4, 3, 2, false, true>(a, max_blocks, s);
    default: return launch_valu_k<kSum, 5, 3, 0>(a, max_blocks, s);
  }
}

}  // namespace

hipError_t launch_plf_prot_valu_f64(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return a.scaler_sum ? launch_valu_t<true>(a, max_blocks, s) : launch_valu_t<false>(a, max_blocks, s);
}

}  // namespace plfx
