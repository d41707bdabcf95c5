// prot_prio.hpp -- tuning copy (not product code): the f64 FMA protein
// kernel (plf_prot_mfma_kernel, fixed grid stride) with wave priorities set per
// trip by s_setprio.  Question: at 2 blocks per CU the first-dispatched block's
// waves win the SIMD's oldest-first issue arbitration and finish their 8 trips
// ~8 us before the second block's (tools/probes/prot_timeline.hip,
// profiles/r03_probe_prot_timeline.log); does raising the younger block's
// priority for part of its trips balance the two without the one-trip
// granularity of a tile queue?
#pragma once
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

// kMode 5: the first trip's x1 tile by LDS-DMA straight into the padded tile
// (slot j of the 64 x 41 layout <- chunk (j / 41, min(j % 41, 39)): the pad
// slots get a harmless copy), issued at kernel start together with the
// register fetch of the first x2 tile, so the first trip waits for one load
// latency instead of two in series.
__device__ __forceinline__ void glds16_prio(const void *src, unsigned lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ void tile_dma_padded64(const double *__restrict__ g, int64_t base, int64_t n,
                                                  unsigned tile_byte) {
  using PT = ProtTile<double>;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int kSlots = 64 * PT::kStride;  // 2624
#pragma unroll
  for (int i = 0; i < (kSlots + kBlock - 1) / kBlock; i++) {
    const int j0 = i * kBlock + wv * 64;  // the wave's first slot (wave-uniform)
    if (j0 >= kSlots) break;
    const int j = j0 + (threadIdx.x & 63);
    const int jj = j < kSlots ? j : kSlots - 1;
    const int s = jj / PT::kStride, q0 = jj - s * PT::kStride;
    const int q = q0 < PT::kChunksPerSite ? q0 : PT::kChunksPerSite - 1;
    const int64_t site = base + s < n ? base + s : n - 1;
    glds16_prio(reinterpret_cast<const f64x2 *>(g + site * 80) + q, tile_byte + (unsigned)j0 * 16u);
  }
}

template <bool kSum, int kMinWaves, int kTips, int kMode, int kH>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_prio_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum,
                     const double *__restrict__ tipvec = nullptr) {
  constexpr int S = 20;
  // tips (kTips 1: x1, 2: both): the child's U^T comes from its LDS table in the
  // accumulator layout (lane: rows g + 4r and 16 + g of site lo16), no MFMA, no tile
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  using PT = ProtTile<double>;
  constexpr int kRow = 2 * PT::kStride;  // doubles per site in the LDS tile (82)
  constexpr int K = PT::kChunks / kBlock;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lo16 = lane & 15, g = lane >> 4;
  f64x2 pf[K];
  const int64_t stride = (int64_t)gridDim.x * 64;
  __shared__ f64x2 tile[64 * ProtTile<double>::kStride];
  if constexpr (kMode == 5 && kTips == 0) {
    if ((int64_t)blockIdx.x * 64 < n) {
      tile_dma_padded64(x1, (int64_t)blockIdx.x * 64, n, (unsigned)(uintptr_t)tile);
      tile_fetch<double>(x2, (int64_t)blockIdx.x * 64, n, pf);
    }
  } else if constexpr (!T2)  // the first dense child's first tile, before the matrix fragments
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  // A fragments: [0][s] -> lane holds M[row = lo16][col = 4s + g];
  // [1][s] -> M[row = 16 + lane%4][col = 4s + g] (the 4x4x4_4b form)
  double AL[2][5], AR[2][5], AE[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; mt++)
#pragma unroll
    for (int st = 0; st < 5; st++) {
      const int row = mt == 1 ? 16 + (lane & 3) : lo16, col = 4 * st + g;
      AL[mt][st] = row < S ? left[c * S * S + row * S + col] : 0.0;   // P_L[k=row][l=col]
      AR[mt][st] = row < S ? right[c * S * S + row * S + col] : 0.0;
      // EV^T[l=row][k=col]; A row i of the first tile computes state 4*(i%4) + i/4
      const int erow = mt == 0 ? 4 * (lo16 & 3) + (lo16 >> 2) : row;
      AE[mt][st] = erow < S ? EV[col * S + erow] : 0.0;
    }
  const double m = Num<double>::minlik();
  __shared__ double tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<double, true>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<double, true>(right, tipvec, tabs[1]);
  if constexpr (T1) __syncthreads();
  // U^T of a tip child for sub-tile t, in the MFMA accumulator layout
  auto tip_u = [&](const double *tab, int code_lane, int t, f64x4 &u0, f64x4 &u1) {
    const double *r = tab + c * kProtCodes * 20 + __shfl(code_lane, 16 * t + lo16) * 20;
    u0 = f64x4{r[g], r[g + 4], r[g + 8], r[g + 12]};
    u1 = f64x4{r[16 + g], 0.0, 0.0, 0.0};
  };
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const double *td = reinterpret_cast<const double *>(tile);
  double *tw = reinterpret_cast<double *>(tile);
  long long acc = 0;
  // the five B-fragment values of sub-tile row xr
  auto bfrag = [&](const double *xr, double (&bv)[5]) {
#pragma unroll
    for (int st = 0; st < 5; st++) bv[st] = xr[4 * st];
  };
  auto trip = [&](const int64_t base, const int64_t nb, bool first) -> int64_t {
    int64_t next = nb;
    f64x4 P[4][2];  // per sub-tile: U_L^T, then p = U_L^T * U_R^T
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
    } else {
      if (kMode == 5 && first) {  // x1 landed in the tile by DMA, x2 in flight in pf
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      } else {
        tile_put<double>(tile, pf);
        __syncthreads();
        tile_fetch<double>(x2, base, n, pf);
      }
#pragma unroll
      for (int t = 0; t < 4; t++) {
        double bv[5];
        bfrag(td + (16 * t + lo16) * kRow + c * S + g, bv);
#pragma unroll
        for (int mt = 0; mt < 2; mt++) {
          f64x4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int st = 0; st < 5; st++) {
            if (mt == 1) u[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AL[1][st], bv[st], u[0], 0, 0, 0);
            else u = __builtin_amdgcn_mfma_f64_16x16x4f64(AL[mt][st], bv[st], u, 0, 0, 0);
          }
          P[t][mt] = u;
        }
      }
      __syncthreads();
    }
    if constexpr (T2) {
#pragma unroll
      for (int t = 0; t < 4; t++) {
        f64x4 u0, u1;
        tip_u(tabs[1], code2, t, u0, u1);
        P[t][0] = P[t][0] * u0;  // prod[k] = umpL[k] * umpR[k]
        P[t][1] = P[t][1] * u1;
      }
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      // next trip's first dense child: x1, or x2 when x1 is a tip
      if (next < n) tile_fetch<double>(T1 ? x2 : x1, next, n, pf);
#pragma unroll
      for (int t = 0; t < 4; t++) {
        double bv[5];
        bfrag(td + (16 * t + lo16) * kRow + c * S + g, bv);
#pragma unroll
        for (int mt = 0; mt < 2; mt++) {
          f64x4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int st = 0; st < 5; st++) {
            if (mt == 1) u[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AR[1][st], bv[st], u[0], 0, 0, 0);
            else u = __builtin_amdgcn_mfma_f64_16x16x4f64(AR[mt][st], bv[st], u, 0, 0, 0);
          }
          P[t][mt] = P[t][mt] * u;  // prod[k] = umpL[k] * umpR[k]
        }
      }
      __syncthreads();  // every wave is done reading x2: the tile takes X3 now
    }
    // back-transform: lane holds X3[site 16t+lo16][l = 4g + r] (tile 0) and
    // [l = 16 + g] (tile 1); written unscaled into the tile, the x2^32 rescale
    // happens in the store pass
    unsigned long long mine = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      f64x4 X0 = {0.0, 0.0, 0.0, 0.0}, X1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        X0 = __builtin_amdgcn_mfma_f64_16x16x4f64(AE[0][st], P[t][st >> 2][st & 3], X0, 0, 0, 0);
        X1[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AE[1][st], P[t][st >> 2][st & 3], X1[0], 0, 0, 0);
      }
      const bool small = (__builtin_fabs(X0[0]) < m) && (__builtin_fabs(X0[1]) < m) &&
                         (__builtin_fabs(X0[2]) < m) && (__builtin_fabs(X0[3]) < m) &&
                         (__builtin_fabs(X1[0]) < m);
      const unsigned long long b = __ballot(small);
      // site lo16 of sub-tile t is small in category c iff its 4 lanes agree
      mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
      double *w = tw + (16 * t + lo16) * kRow + c * S;
      *reinterpret_cast<f64x2 *>(w + 4 * g) = f64x2{X0[0], X0[1]};
      *reinterpret_cast<f64x2 *>(w + 4 * g + 2) = f64x2{X0[2], X0[3]};
      w[16 + g] = X1[0];
    }
    if (lane == 0) small_mask[c] = mine;
    __syncthreads();
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    if (c == 0) {
      const int64_t site = base + lane;
      const bool sc = (all >> lane) & 1ull;
      if (site < n) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
    }
    // kMode 4: every wave waits for its loads in flight (the next tile) before
    // its share of the store pass (the product: wave 0 only, through the wait
    // of its weight load)
    if constexpr (kMode == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // coalesced store with the rescale of the scaled sites (exact: x 2^32)
    {
      f64x2 *dst = reinterpret_cast<f64x2 *>(x3 + base * 80);
      f64x2 v[K];
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        const int sl = j / PT::kChunksPerSite, q = j - sl * PT::kChunksPerSite;
        v[i] = tile[sl * PT::kStride + q];
        if ((all >> sl) & 1ull) v[i] = v[i] * Num<double>::two32();
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
    __syncthreads();
    return next;
  };
  {
    // wave priority (s_setprio) by trip: the SIMD's arbiter favours the older
    // waves, i.e. the first-dispatched block of each CU (blockIdx < G/2);
    // kMode 1: the younger block at priority 1 for its first kH trips;
    // 2: the younger block at 1 throughout; 3: leadership alternating by trip;
    // 4: no priorities, every wave drains its loads before the store pass;
    // 5: the first trip's x1 by LDS-DMA beside the first x2 fetch (above)
    const bool young = blockIdx.x >= (gridDim.x + 1) / 2;
    int i = 0;
    for (int64_t b = (int64_t)blockIdx.x * 64; b < n; b += stride, i++) {
      bool hi = false;
      if constexpr (kMode == 1) hi = young && i < kH;
      if constexpr (kMode == 2) hi = young;
      if constexpr (kMode == 3) hi = young == ((i & 1) == 0);
      if constexpr (kMode >= 1 && kMode <= 3) {
        if (hi) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      trip(b, b + stride < n ? b + stride : n, i == 0);
    }
    if constexpr (kMode >= 1 && kMode <= 3) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
