// prot_pair32.hpp -- tuning variant (not product code) of the f32 EXACT
// protein kernel: two sites per lane with packed f32 arithmetic.  Measured
// bit-identical and slower than plf_prot_lds_kernel<float> (78-82 vs 72.9 us at
// 2^18 sites, 309-311 vs 294-296 us at 2^20; profiles/r02_tune_protein_f32_pair.log):
// halving the VALU instructions and LDS broadcasts per site does not pay at two
// blocks per CU (its 234 VGPRs) against three.
#pragma once
#include "plf_prot_tune.hpp"

namespace plfx {
namespace dev {

// f32 EXACT mode, two sites per lane (dense children): lane l of wave c owns
// sites base + l and base + 64 + l of a 128-site tile, and every arithmetic
// operation is a packed f32 pair over the two sites (v_pk_mul_f32 /
// v_pk_add_f32: each half is one site's own IEEE f32 operation in plf()'s
// order), so the results are bit-identical to plf_prot_lds_kernel<float> while
// every matrix value read from LDS feeds both sites.  That kernel is bound by
// VALU issue (2420 f32 operations per site-category, one site per lane); here
// the instructions and the LDS broadcasts per site halve.  4-row groups in
// phases 1/2 (4 packed chains), 10-state halves in phase 3; the next child
// tile is prefetched in registers as in the one-site kernel.
template <bool kSum, int kMinWaves = 2>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_pair32_kernel(const float *__restrict__ x1, const float *__restrict__ x2,
                       float *__restrict__ x3, const float *__restrict__ EV,
                       const float *__restrict__ left, const float *__restrict__ right,
                       const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                       unsigned long long *ws, int64_t *scaler_sum,
                       const float *__restrict__ tipvec = nullptr) {
  constexpr int S = 20, kTS = 128;                  // sites per tile
  constexpr int kCps = 20, kStr = 21;               // 16-B chunks per site, padded row stride
  constexpr int K = kTS * kCps / kBlock;            // 10 chunks per thread per tile
  constexpr int kRows = 4;                          // phase 1/2 rows per group
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // P_L | P_R group-transposed ([c][k/4][l][k%4]: one f32x4 = rows 4g..4g+3 of
  // column l) and EV row-major: 3600 floats
  __shared__ f32x4 mats[900];
  __shared__ f32x4 tile[kTS * kStr];
  __shared__ unsigned long long small_mask[kWavesPerBlock][2];
  {
    float *md = reinterpret_cast<float *>(mats);
    for (int i = threadIdx.x; i < 4 * S * S; i += kBlock) {
      const int cc = i / (S * S), r = i - cc * S * S, k = r / S, l = r - k * S;
      const int d = cc * S * S + (k / kRows) * (S * kRows) + l * kRows + (k % kRows);
      md[d] = left[i];
      md[4 * S * S + d] = right[i];
    }
    for (int i = threadIdx.x; i < S * S; i += kBlock) md[8 * S * S + i] = EV[i];
  }
  const float m = Num<float>::minlik();
  auto fetch = [&](const float *g, int64_t b, f32x4 (&v)[K]) {
    const f32x4 *src = reinterpret_cast<const f32x4 *>(g + b * 80);
    if (b + kTS <= n) {
#pragma unroll
      for (int i = 0; i < K; i++) v[i] = __builtin_nontemporal_load(src + threadIdx.x + i * kBlock);
    } else {
      const int64_t lim = (n - b) * kCps;
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (j < lim) v[i] = __builtin_nontemporal_load(src + j);
      }
    }
  };
  auto put = [&](const f32x4 (&v)[K]) {
#pragma unroll
    for (int i = 0; i < K; i++) {
      const int j = threadIdx.x + i * kBlock;
      const int st = j / kCps, q = j - st * kCps;
      tile[st * kStr + q] = v[i];
    }
  };
  // this lane's two rows of category c as pairs {site A, site B}
  auto rows = [&](f32x2 (&xp)[S]) {
    const f32x4 *ra = tile + lane * kStr + c * 5, *rb = tile + (64 + lane) * kStr + c * 5;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const f32x4 a = ra[i], b = rb[i];
      xp[4 * i] = f32x2{a.x, b.x};
      xp[4 * i + 1] = f32x2{a.y, b.y};
      xp[4 * i + 2] = f32x2{a.z, b.z};
      xp[4 * i + 3] = f32x2{a.w, b.w};
    }
  };
  // phases 1/2: fn(k, {sum_l xA[l] M[k][l], sum_l xB[l] M[k][l]}) for every k,
  // each chain from its first product in ascending l (see site_cat)
  auto phase = [&](const f32x4 *M, const f32x2 (&xp)[S], auto &&fn) {
    int o = 0;
    float tok = 0.f;
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const f32x4 *G = M + gk * S;
      f32x4 ring[3];
      f32x2 u[kRows];
      asm volatile("" : "+v"(o) : "v"(tok));
      ring[0] = G[o];
      ring[1] = G[o + 1];
#pragma unroll
      for (int l = 0; l < S; l++) {
        asm volatile("" : "+v"(o) : "v"(tok));
        if (l + 2 < S) ring[(l + 2) % 3] = G[o + l + 2];
        const f32x4 col = ring[l % 3];
        f32x2 pr[kRows];
#pragma unroll
        for (int j = 0; j < kRows; j++) pr[j] = xp[l] * f32x2{col[j], col[j]};
        pin_chains(pr);
#pragma unroll
        for (int j = 0; j < kRows; j++) u[j] = l == 0 ? pr[j] : u[j] + pr[j];
        pin_chains(u);
        tok = u[kRows - 1].y;
      }
#pragma unroll
      for (int j = 0; j < kRows; j++) fn(gk * kRows + j, u[j]);
    }
  };
  const int64_t stride = (int64_t)gridDim.x * kTS;
  f32x4 pf[K];
  if ((int64_t)blockIdx.x * kTS < n) fetch(x1, (int64_t)blockIdx.x * kTS, pf);
  long long acc = 0;
  __syncthreads();  // matrices in LDS
  for (int64_t base = (int64_t)blockIdx.x * kTS; base < n; base += stride) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const f32x4 *mL = mats + off + c * 100, *mR = mats + off + 400 + c * 100, *mE = mats + off + 800;
    f32x2 U[S];
    {
      f32x2 xp[S];
      put(pf);
      __syncthreads();
      fetch(x2, base, pf);
      rows(xp);
      __syncthreads();  // the tile is free for the next put
      phase(mL, xp, [&](int k, f32x2 u) { U[k] = u; });
    }
    {
      f32x2 xp[S];
      put(pf);
      __syncthreads();
      if (base + stride < n) fetch(x1, base + stride, pf);
      rows(xp);
      __syncthreads();
      phase(mR, xp, [&](int k, f32x2 u) { U[k] = U[k] * u; });  // prod[k] = umpL[k] * umpR[k]
    }
    // phase 3: O[l] = sum_k U[k] EV[k][l] from +0.0 over ascending k, two halves
    // of 10 states (EV row k read as f32x4 chunks 3h .. 3h+2, h = 0 / chunks 2..4)
    f32x2 O[S];
    {
      int o = 0;
      float tok = 0.f;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int c0 = h == 0 ? 0 : 2, s0 = h == 0 ? 0 : 2;  // first chunk; state offset in it
        f32x2 v[10];
#pragma unroll
        for (int j = 0; j < 10; j++) v[j] = f32x2{0.f, 0.f};
#pragma unroll
        for (int k = 0; k < S; k++) {
          asm volatile("" : "+v"(o) : "v"(tok));
          const f32x4 *er = mE + o + k * 5 + c0;
          const f32x4 e0 = er[0], e1 = er[1], e2 = er[2];
          float e[12] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y, e2.z, e2.w};
          f32x2 pr[10];
#pragma unroll
          for (int j = 0; j < 10; j++) pr[j] = U[k] * f32x2{e[s0 + j], e[s0 + j]};
          pin_chains(pr);
#pragma unroll
          for (int j = 0; j < 10; j++) v[j] = v[j] + pr[j];
          pin_chains(v);
          tok = v[9].y;
        }
#pragma unroll
        for (int j = 0; j < 10; j++) O[10 * h + j] = v[j];
      }
    }
    // scale test per site (all 80 |values| < 2^-32, strict), across the 4 waves
    bool sa = base + lane < n, sb = base + 64 + lane < n;
#pragma unroll
    for (int l = 0; l < S; l++) {
      sa = sa && (Num<float>::abs(O[l].x) < m);
      sb = sb && (Num<float>::abs(O[l].y) < m);
    }
    const unsigned long long ma = __ballot(sa), mb = __ballot(sb);
    if (lane == 0) {
      small_mask[c][0] = ma;
      small_mask[c][1] = mb;
    }
    __syncthreads();
    const unsigned long long alla = small_mask[0][0] & small_mask[1][0] & small_mask[2][0] & small_mask[3][0];
    const unsigned long long allb = small_mask[0][1] & small_mask[1][1] & small_mask[2][1] & small_mask[3][1];
    const bool sca = (alla >> lane) & 1ull, scb = (allb >> lane) & 1ull;
#pragma unroll
    for (int l = 0; l < S; l++) {  // select, as every kernel: unscaled values pass through untouched
      const f32x2 sv = O[l] * f32x2{Num<float>::two32(), Num<float>::two32()};
      O[l] = f32x2{sca ? sv.x : O[l].x, scb ? sv.y : O[l].y};
    }
    f32x4 *wa = tile + lane * kStr + c * 5, *wb = tile + (64 + lane) * kStr + c * 5;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      wa[i] = f32x4{O[4 * i].x, O[4 * i + 1].x, O[4 * i + 2].x, O[4 * i + 3].x};
      wb[i] = f32x4{O[4 * i].y, O[4 * i + 1].y, O[4 * i + 2].y, O[4 * i + 3].y};
    }
    if (c == 0) {
      const int64_t sA = base + lane, sB = base + 64 + lane;
      if (sA < n) {
        if (scaler) scaler[sA] = (uint8_t)sca;
        if (kSum && sca) acc += wgt ? (long long)wgt[sA] : 1ll;
      }
      if (sB < n) {
        if (scaler) scaler[sB] = (uint8_t)scb;
        if (kSum && scb) acc += wgt ? (long long)wgt[sB] : 1ll;
      }
    }
    __syncthreads();
    {
      f32x4 *dst = reinterpret_cast<f32x4 *>(x3 + base * 80);
      f32x4 v[K];
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        const int st = j / kCps, q = j - st * kCps;
        v[i] = tile[st * kStr + q];
      }
      if (base + kTS <= n) {
#pragma unroll
        for (int i = 0; i < K; i++) __builtin_nontemporal_store(v[i], dst + threadIdx.x + i * kBlock);
      } else {
        const int64_t lim = (n - base) * kCps;
#pragma unroll
        for (int i = 0; i < K; i++) {
          const int j = threadIdx.x + i * kBlock;
          if (j < lim) __builtin_nontemporal_store(v[i], dst + j);
        }
      }
    }
    __syncthreads();  // tile and small_mask are reused by the next trip
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
