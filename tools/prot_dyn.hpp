// prot_dyn.hpp -- tuning copy (not product code): the f64 FMA protein kernel
// (plf_prot_mfma_kernel, csrc/plf_prot.hpp) with tiles handed out by a
// device-wide dequeue instead of a fixed grid stride.  Why: a per-block
// timeline of the product at 2^18 sites (tools/probes/prot_timeline.hip)
// shows the first block on each CU finishing at ~75 us and the second at
// ~83 us (the older waves win the SIMD's issue arbitration) while both do 8
// trips, so the launch ends at ~89 us with half the CUs idle for its last
// 8 us.  With a queue the faster block takes more tiles.
#pragma once
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

template <bool kSum, int kMinWaves, int kTips, bool kXcd = false>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_dyn_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum,
                     const double *__restrict__ tipvec = nullptr, uint64_t *stamps = nullptr) {
  // stamps (probe only): per block [entry | xcc << 56, trips, trip ends..., exit] (40 words)
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
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
  if constexpr (!T2)  // the first dense child's first tile, before the matrix fragments
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  // Tiles: trip 0 takes blockIdx.x, trip 1 G + blockIdx.x, trip i >= 2 2G + d,
  // d from a dequeue on the head word that thread 0 issued in the middle of trip
  // i - 2 (right after the wave's next-tile loads, so nothing waits for it
  // before the next trip's start) and publishes in LDS at the start of trip
  // i - 1 (the value is used nowhere else: any use makes the wave wait for the
  // atomic there).  kXcd: one head per XCD (tile 2G + 8d + xcd) -- contention
  // of 64 instead of 512 pullers.  The last block out (exit counter) zeroes
  // the words for the next launch; a block's dequeue has returned before its
  // exit add (the add depends on the returned value).
  unsigned long long *q = ws + kWsWords;
  const int64_t G = gridDim.x, ntiles = (n + 63) / 64;
  const bool dyn = ntiles > 2 * G;
  const int xq = kXcd ? (int)(__builtin_amdgcn_s_getreg(20 | (3 << 11)) & 7) : 0;
  unsigned long long *head = q + 16 * xq;
  __shared__ long long qslot;
  long long pend = 0;  // thread 0: the dequeued value for the tile of trip i+2
  auto dequeue = [&](int) {
    if (dyn && threadIdx.x == 0)
      pend = (long long)__hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto tile_of = [&](long long d) -> int64_t { return kXcd ? 2 * G + 8 * d + xq : 2 * G + d; };
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
  __shared__ f64x2 tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const double *td = reinterpret_cast<const double *>(tile);
  double *tw = reinterpret_cast<double *>(tile);
  long long acc = 0;
  // the five B-fragment values of sub-tile row xr
  auto bfrag = [&](const double *xr, double (&bv)[5]) {
#pragma unroll
    for (int st = 0; st < 5; st++) bv[st] = xr[4 * st];
  };
  auto trip = [&](const int64_t base, const int i) -> int64_t {
    int64_t next = n;
    f64x4 P[4][2];  // per sub-tile: U_L^T, then p = U_L^T * U_R^T
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      next = qslot;
      tile_fetch<double>(x2, base, n, pf);
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
      next = qslot;  // published before the trip's barrier
      dequeue(i);
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      if constexpr (T1) next = qslot;
      // next trip's first dense child: x1, or x2 when x1 is a tip
      if (next < ntiles) tile_fetch<double>(T1 ? x2 : x1, next * 64, n, pf);
      dequeue(i);
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
  int64_t cur = blockIdx.x;
  for (int i = 0; cur < ntiles; i++) {
    if (threadIdx.x == 0) {
      int64_t nx = ntiles;
      if (i == 0) nx = G + blockIdx.x;
      else if (dyn) nx = tile_of(pend);
      qslot = nx < ntiles ? nx : ntiles;
    }
    if constexpr (T1 && T2) __syncthreads();
    cur = trip(cur * 64, i);
    if (stamps && threadIdx.x == 0 && i < 37) stamps[(size_t)blockIdx.x * 40 + 2 + i] = __builtin_amdgcn_s_memrealtime();
    if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * 40 + 1] = (uint64_t)(i + 1);
  }
  if (threadIdx.x == 0) {
    const unsigned long long after = (unsigned long long)(pend >> 62);  // 0, once it returned
    const unsigned long long d =
        __hip_atomic_fetch_add(q + 8 * 16, 1ull + after, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned long long)G - 1) {
      for (int x = 0; x < 9; x++) __hip_atomic_store(q + 16 * x, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
  if (stamps && threadIdx.x == 0) {
    stamps[(size_t)blockIdx.x * 40] = t_entry | ((uint64_t)(__builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15) << 56);
    stamps[(size_t)blockIdx.x * 40 + 39] = __builtin_amdgcn_s_memrealtime();
  }
}


template <bool kSum, int kMinWaves, int kTips, int kNH = 8, int kQ = 16>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_items_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum,
                     const double *__restrict__ tipvec = nullptr, uint64_t *stamps = nullptr) {
  // stamps (probe only): per block [entry | xcc << 56, trips, trip ends..., exit] (40 words)
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
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
  if constexpr (!T2)  // the first dense child's first tile, before the matrix fragments
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  // Work items: trip 0 takes tile blockIdx.x, trip 1 tile G + blockIdx.x (64
  // sites each); then dynamic items j = 0..M-1: 64-site tiles, and for the last
  // G tiles' sites kQ-site items (a fine tail: a block that runs out of work
  // waits at most one short item for the others).  Heads: NH words (NH = kNH
  // when G >= kNH, else 1), block b pulls from head b % NH, whose k-th dequeue
  // is item NH k + b % NH -- every head has pullers, no item is left over.
  // Thread 0 issues a trip's dequeue right after the wave's next-item loads and
  // publishes its item (base, length) in LDS at the next trip's start (its
  // only use: any use makes the wave wait for the atomic there).  The last
  // block out (exit counter) zeroes the words for the next launch.
  unsigned long long *q = ws + kWsWords;
  const int64_t G = gridDim.x, ntiles = (n + 63) / 64;
  const bool dyn = ntiles > 2 * G;
  const int NH = G >= kNH ? kNH : 1;
  const int home = (int)(blockIdx.x % NH);
  unsigned long long *head = q + 16 * home;
  const int64_t Tq = kQ < 64 ? (ntiles - 2 * G < G ? ntiles - 2 * G : G) : 0;  // tiles split into items
  const int64_t Bt = ntiles - 2 * G - Tq, S_tail = (ntiles - Tq) * 64;           // bulk tiles, tail start
  const int64_t M = dyn ? Bt + (n - S_tail + kQ - 1) / kQ : 0;
  __shared__ long long qslot;
  __shared__ int qlen;
  long long pend = 0;  // thread 0: the dequeued value for the item of trip i+2
  auto dequeue = [&](int) {
    if (dyn && threadIdx.x == 0)
      pend = (long long)__hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
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
  __shared__ f64x2 tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const double *td = reinterpret_cast<const double *>(tile);
  double *tw = reinterpret_cast<double *>(tile);
  long long acc = 0;
  // the five B-fragment values of sub-tile row xr
  auto bfrag = [&](const double *xr, double (&bv)[5]) {
#pragma unroll
    for (int st = 0; st < 5; st++) bv[st] = xr[4 * st];
  };
  int nlen = 64;  // the next item's length, read with its base after a trip's first barrier
  auto trip = [&](auto NS, const int64_t base, const int len, const int i) -> int64_t {
    constexpr int nsub = decltype(NS)::value;  // sub-tiles of the item: 4, or kQ / 16
    const int64_t ne = base + len < n ? base + len : n;
    int64_t next = n;
    nlen = 64;
    f64x4 P[4][2];  // per sub-tile: U_L^T, then p = U_L^T * U_R^T
    const int64_t sq = base + lane < ne ? base + lane : ne - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      next = qslot;
      nlen = qlen;
      tile_fetch<double>(x2, base, ne, pf);
#pragma unroll
      for (int t = 0; t < nsub; t++) {
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
      next = qslot;  // published before the trip's barrier
      nlen = qlen;
      dequeue(i);
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      if constexpr (T1) { next = qslot; nlen = qlen; }
      // next trip's first dense child: x1, or x2 when x1 is a tip
      if (next < n) tile_fetch<double>(T1 ? x2 : x1, next, next + nlen < n ? next + nlen : n, pf);
      dequeue(i);
#pragma unroll
      for (int t = 0; t < nsub; t++) {
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
    for (int t = 0; t < nsub; t++) {
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
      if (site < ne) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
    }
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
      if (base + 64 <= ne) {
#pragma unroll
        for (int i = 0; i < K; i++) __builtin_nontemporal_store(v[i], dst + threadIdx.x + i * kBlock);
      } else {
        const int64_t lim = (ne - base) * PT::kChunksPerSite;
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
  int64_t cur = (int64_t)blockIdx.x * 64;
  int clen = 64;
  for (int i = 0; cur < n; i++) {
    if (threadIdx.x == 0) {
      int64_t nb = n;
      int nl = 64;
      if (i == 0) {
        nb = (G + blockIdx.x) * 64;
      } else if (dyn) {
        const int64_t j = (int64_t)NH * pend + home;
        if (j < Bt) nb = (2 * G + j) * 64;
        else if (j < M) { nb = S_tail + (j - Bt) * kQ; nl = kQ; }
      }
      qslot = nb < n ? nb : n;
      qlen = nl;
    }
    if constexpr (T1 && T2) __syncthreads();
    int64_t nxt;
    if (kQ == 64 || clen == 64) nxt = trip(std::integral_constant<int, 4>{}, cur, clen, i);
    else nxt = trip(std::integral_constant<int, (kQ + 15) / 16>{}, cur, clen, i);
    clen = nlen;
    cur = nxt;
    if (stamps && threadIdx.x == 0 && i < 37) stamps[(size_t)blockIdx.x * 40 + 2 + i] = __builtin_amdgcn_s_memrealtime();
    if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * 40 + 1] = (uint64_t)(i + 1);
  }
  if (threadIdx.x == 0) {
    const unsigned long long after = (unsigned long long)(pend >> 62);  // 0, once it returned
    const unsigned long long d =
        __hip_atomic_fetch_add(q + 8 * 16, 1ull + after, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned long long)G - 1) {
      for (int x = 0; x < 9; x++) __hip_atomic_store(q + 16 * x, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
  if (stamps && threadIdx.x == 0) {
    stamps[(size_t)blockIdx.x * 40] = t_entry | ((uint64_t)(__builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15) << 56);
    stamps[(size_t)blockIdx.x * 40 + 39] = __builtin_amdgcn_s_memrealtime();
  }
}


template <bool kSum, int kMinWaves, int kTips, int kNum, int kDen>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_split_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
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
  if constexpr (!T2)  // the first dense child's first tile, before the matrix fragments
    {
      const int64_t G = gridDim.x, GA = (G + 1) / 2, GB = G - GA, ntiles = (n + 63) / 64;
      const int64_t TA = GB > 0 ? ntiles * kNum / kDen : ntiles;
      const int64_t t0 = blockIdx.x < GA ? blockIdx.x : TA + (blockIdx.x - GA);
      if (t0 < (blockIdx.x < GA ? TA : ntiles)) tile_fetch<double>(T1 ? x2 : x1, t0 * 64, n, pf);
    }
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
  // kDyn: tiles handed out by a device-wide dequeue (prot_queue below)
  __shared__ f64x2 tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const double *td = reinterpret_cast<const double *>(tile);
  double *tw = reinterpret_cast<double *>(tile);
  long long acc = 0;
  // the five B-fragment values of sub-tile row xr
  auto bfrag = [&](const double *xr, double (&bv)[5]) {
#pragma unroll
    for (int st = 0; st < 5; st++) bv[st] = xr[4 * st];
  };
  auto trip = [&](const int64_t base, const int64_t nb) -> int64_t {
    int64_t next = nb;
    f64x4 P[4][2];  // per sub-tile: U_L^T, then p = U_L^T * U_R^T
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      tile_fetch<double>(x2, base, n, pf);
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
    // the first-dispatched block of each CU (blockIdx < G/2) runs ahead of the
    // second: give the first half kNum/kDen of the tiles
    const int64_t G = gridDim.x, GA = (G + 1) / 2, GB = G - GA, ntiles = (n + 63) / 64;
    const int64_t TA = GB > 0 ? ntiles * kNum / kDen : ntiles;
    const bool first = blockIdx.x < GA;
    const int64_t t0 = first ? blockIdx.x : TA + (blockIdx.x - GA);
    const int64_t tend = first ? TA : ntiles, st = first ? GA : GB;
    for (int64_t t = t0; t < tend; t += st) trip(t * 64, t + st < tend ? (t + st) * 64 : n);
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}


}  // namespace dev
}  // namespace plfx
