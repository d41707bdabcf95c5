// prot_v8.hpp -- tuning variant (not product code yet) of the protein FMA
// kernel: one 512-thread block per CU (8 waves, 2 per SIMD), three LDS tiles
// per block (x1, x2, X3; 3 x 41 KiB), BOTH next child tiles fetched into
// registers at the start of a trip and consumed at its end, so two tiles'
// loads are in flight across the whole trip's matrix-core work; two barriers
// per trip.  Wave w: category c = w & 3, sub-tiles 2h, 2h+1 (h = w >> 2) of
// the 64-site tile.  kPerm: the back-transform's A rows are permuted (row
// g + 4r <-> state 4g + r) so a lane's four results are four consecutive
// states of its site: X3 goes to LDS as two ds_write_b128 (conflict-free)
// instead of four 2-way-conflicted ds_write_b64.  Arithmetic and k order
// as plf_prot_mfma_kernel (bit-identical results).
#pragma once
#include "plf_prot_tune.hpp"

namespace plfx {
namespace dev {

constexpr int kV8Threads = 512;

// kTS = sites per tile: 64 (8 waves, one block per CU by LDS) or 32 (4 waves,
// 3 x 20.5 KiB of LDS, two blocks per CU that drift apart).
template <bool kSum, bool kPerm = true, bool kEarly = true, int kTS = 64>
__global__ void __launch_bounds__(kTS * 8)
plf_prot_mfma8_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                      double *__restrict__ x3, const double *__restrict__ EV,
                      const double *__restrict__ left, const double *__restrict__ right,
                      const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                      unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  constexpr int kStride = PT::kStride;           // 41 chunks per site
  constexpr int kCps = PT::kChunksPerSite;       // 40
  constexpr int kRow = 2 * kStride;              // 82 doubles per site
  constexpr int kThreads = kTS * 8, kWaves = kThreads / 64;
  constexpr int K = kTS * kCps / kThreads;       // 5 chunks per thread per tile
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = wv & 3, h = wv >> 2;
  const int lane = threadIdx.x & 63, lo16 = lane & 15, g = lane >> 4;
  const int64_t stride = (int64_t)gridDim.x * kTS;

  __shared__ f64x2 tA[kTS * kStride], tB[kTS * kStride], tC[kTS * kStride];
  __shared__ unsigned long long small_mask[kWaves];
  const double *dA = reinterpret_cast<const double *>(tA);
  const double *dB = reinterpret_cast<const double *>(tB);
  double *wC = reinterpret_cast<double *>(tC);

  f64x2 p1[K], p2[K];
  auto fetch = [&](const double *src, int64_t b, f64x2 (&v)[K]) {
    const f64x2 *s = reinterpret_cast<const f64x2 *>(src + b * 80);
    if (b + kTS <= n) {
#pragma unroll
      for (int i = 0; i < K; i++) v[i] = __builtin_nontemporal_load(s + threadIdx.x + i * kThreads);
    } else {
      const int64_t lim = (n - b) * kCps;
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kThreads;
        v[i] = f64x2{0.0, 0.0};
        if (j < lim) v[i] = __builtin_nontemporal_load(s + j);
      }
    }
  };
  auto put = [&](f64x2 *t, const f64x2 (&v)[K]) {
#pragma unroll
    for (int i = 0; i < K; i++) {
      const int j = threadIdx.x + i * kThreads;
      const int s = j / kCps, q = j - s * kCps;
      t[s * kStride + q] = v[i];
    }
  };

  int64_t base = (int64_t)blockIdx.x * kTS;
  if constexpr (kEarly) {
    if (base < n) { fetch(x1, base, p1); fetch(x2, base, p2); }
  }
  double AL[2][5], AR[2][5], AE[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; mt++)
#pragma unroll
    for (int st = 0; st < 5; st++) {
      const int row = mt == 1 ? 16 + (lane & 3) : lo16, col = 4 * st + g;
      // kPerm: back-transform row i = lo16 computes state 4*(i%4) + i/4
      const int erow = (kPerm && mt == 0) ? 4 * (lo16 & 3) + (lo16 >> 2) : row;
      AL[mt][st] = row < S ? left[c * S * S + row * S + col] : 0.0;
      AR[mt][st] = row < S ? right[c * S * S + row * S + col] : 0.0;
      AE[mt][st] = erow < S ? EV[col * S + erow] : 0.0;
    }
  const double m = Num<double>::minlik();
  long long acc = 0;
  if constexpr (!kEarly) {
    if (base < n) { fetch(x1, base, p1); fetch(x2, base, p2); }
  }
  if (base < n) { put(tA, p1); put(tB, p2); }
  __syncthreads();

  for (; base < n; base += stride) {
    const int64_t nb = base + stride;
    if (nb < n) { fetch(x1, nb, p1); fetch(x2, nb, p2); }
    f64x4 P[2][2];
#pragma unroll
    for (int tl = 0; tl < 2; tl++) {
      const int t = 2 * h + tl;
      const double *xa = dA + (16 * t + lo16) * kRow + c * S + g;
      const double *xb = dB + (16 * t + lo16) * kRow + c * S + g;
      f64x4 u0 = {0.0, 0.0, 0.0, 0.0}, u1 = {0.0, 0.0, 0.0, 0.0};
      f64x4 v0 = {0.0, 0.0, 0.0, 0.0}, v1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const double a = xa[4 * st];
        u0 = __builtin_amdgcn_mfma_f64_16x16x4f64(AL[0][st], a, u0, 0, 0, 0);
        u1[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AL[1][st], a, u1[0], 0, 0, 0);
      }
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const double b = xb[4 * st];
        v0 = __builtin_amdgcn_mfma_f64_16x16x4f64(AR[0][st], b, v0, 0, 0, 0);
        v1[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AR[1][st], b, v1[0], 0, 0, 0);
      }
      P[tl][0] = u0 * v0;  // prod[k] = umpL[k] * umpR[k]
      P[tl][1] = u1 * v1;
    }
    // back-transform into tile C (free since the previous trip's store pass)
    unsigned long long mine = 0;
#pragma unroll
    for (int tl = 0; tl < 2; tl++) {
      const int t = 2 * h + tl;
      f64x4 X0 = {0.0, 0.0, 0.0, 0.0}, X1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        X0 = __builtin_amdgcn_mfma_f64_16x16x4f64(AE[0][st], P[tl][st >> 2][st & 3], X0, 0, 0, 0);
        X1[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AE[1][st], P[tl][st >> 2][st & 3], X1[0], 0, 0, 0);
      }
      const bool small = (__builtin_fabs(X0[0]) < m) && (__builtin_fabs(X0[1]) < m) &&
                         (__builtin_fabs(X0[2]) < m) && (__builtin_fabs(X0[3]) < m) &&
                         (__builtin_fabs(X1[0]) < m);
      const unsigned long long b = __ballot(small);
      mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
      double *w = wC + (16 * t + lo16) * kRow + c * S;
      if constexpr (kPerm) {
        *reinterpret_cast<f64x2 *>(w + 4 * g) = f64x2{X0[0], X0[1]};
        *reinterpret_cast<f64x2 *>(w + 4 * g + 2) = f64x2{X0[2], X0[3]};
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++) w[g + 4 * r] = X0[r];
      }
      w[16 + g] = X1[0];
    }
    if (lane == 0) small_mask[wv] = mine;
    __syncthreads();  // X3 complete in C; every read of A and B done
    unsigned long long all = ~0ull;
#pragma unroll
    for (int cc = 0; cc < 4; cc++)
      all &= kWaves == 8 ? (small_mask[cc] | small_mask[cc + 4]) : small_mask[cc];
    if (threadIdx.x < kTS) {
      const int64_t site = base + threadIdx.x;
      const bool sc = (all >> threadIdx.x) & 1ull;
      if (site < n) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
    }
    {
      f64x2 *dst = reinterpret_cast<f64x2 *>(x3 + base * 80);
      f64x2 v[K];
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kThreads;
        const int sl = j / kCps, q = j - sl * kCps;
        v[i] = tC[sl * kStride + q];
        if ((all >> sl) & 1ull) v[i] = v[i] * Num<double>::two32();
      }
      if (base + kTS <= n) {
#pragma unroll
        for (int i = 0; i < K; i++) __builtin_nontemporal_store(v[i], dst + threadIdx.x + i * kThreads);
      } else {
        const int64_t lim = (n - base) * kCps;
#pragma unroll
        for (int i = 0; i < K; i++) {
          const int j = threadIdx.x + i * kThreads;
          if (j < lim) __builtin_nontemporal_store(v[i], dst + j);
        }
      }
    }
    if (nb < n) { put(tA, p1); put(tB, p2); }
    __syncthreads();  // next tiles visible; C and small_mask free again
  }
  if constexpr (kSum) {
    if (threadIdx.x < 64) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
      if (threadIdx.x == 0) ticket_publish(acc, ws, scaler_sum);
    }
  }
}

}  // namespace dev
}  // namespace plfx
