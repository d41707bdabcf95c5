// prot_wave32.hpp -- tuning copy (not product code): the f32 FMA protein node
// on the matrix cores with WAVE-PRIVATE 16-site tiles instead of the product's
// block-wide 64-site tile (plf_prot_mfma32_kernel, csrc/plf_prot.hpp).
//
// Mapping: wave = 16 consecutive sites (all 4 categories), lane group g =
// category g in the 4x4x1 parts.  The product kernel has wave = category, so
// all four waves need every site of the block's tile: 5 block barriers per
// trip and an LDS exchange of the four scale masks.  Here a wave holds the
// A fragments of all four categories (45 VGPRs), stages its own 16 sites
// (5 KiB per child) through its own LDS region, tests all 80 values of its
// sites itself (ballots, no exchange), and writes X3 back through the same
// region -- no block barrier inside the site loop.  The arithmetic is the
// product's, instruction for instruction per (site, category): the same
// k-ordered chains, so the output is bit-identical.
//   * 16x16x4 products: A = P_c with rows permuted (k = 4(i&3) + (i>>2)),
//     B = the tile's (site lo16, category c, state 4st + g), one accumulator
//     f32x4 per category;
//   * rows 16..19 (4x4x1_16b): block b = lane/4 = 4 sites of category g, A
//     lane l = P_g[16 + l%4][col] from the block's LDS copy, B = the lane's
//     own (site lo16, category g) row;
//   * back-transform per category: B fragments = the accumulators (k-step st
//     = reg st, k-step 4 = the transposed Q), rows 16..19 by 20 K = 1 steps on
//     p[k] brought to lane (g, lo16) by four 4x4 transposes.
#pragma once
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

constexpr int kWTileStride = 21;  // f32x4 chunks per site in LDS (20 + 1 pad)

__device__ __forceinline__ void wtile_fetch(const float *__restrict__ g, int64_t base, int64_t n, int lane,
                                            f32x4 (&v)[5]) {
  const f32x4 *src = reinterpret_cast<const f32x4 *>(g + base * 80);
  if (base + 16 <= n) {
#pragma unroll
    for (int i = 0; i < 5; i++) v[i] = __builtin_nontemporal_load(src + lane + 64 * i);
  } else {
    const int64_t lim = (n - base) * 20;
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int j = lane + 64 * i;
      v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (j < lim) v[i] = __builtin_nontemporal_load(src + j);
    }
  }
}

__device__ __forceinline__ void wtile_put(f32x4 *lds, int lane, const f32x4 (&v)[5]) {
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int j = lane + 64 * i;
    const int s = j / 20, q = j - 20 * s;
    lds[s * kWTileStride + q] = v[i];
  }
}

// kA: where the 16x16x4 A fragments of P_L / P_R come from -- 0: registers
// loaded from global memory per lane (40 scattered loads of a 12.8-KB matrix
// per wave), 1: registers loaded from a per-block LDS image of the fragments
// (built by coalesced loads), 2: read from that image inside every product
// (40 fewer VGPRs, 40 more ds_read_b32 per wave and trip).
template <bool kSum, int kMinBlocks, int kTips, int kA = 0>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
plf_prot_mfma32w_kernel(const float *__restrict__ x1, const float *__restrict__ x2,
                        float *__restrict__ x3, const float *__restrict__ EV,
                        const float *__restrict__ left, const float *__restrict__ right,
                        const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                        unsigned long long *ws, int64_t *scaler_sum,
                        const float *__restrict__ tipvec = nullptr) {
  constexpr int S = 20;
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  constexpr int kRow = 4 * kWTileStride;  // floats per site in the LDS tile (84)
  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int lo16 = lane & 15, g = lane >> 4;
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 16;
  const int64_t base0 = ((int64_t)blockIdx.x * kWavesPerBlock + wv) * 16;
  f32x4 pf[5];
  if constexpr (!(T1 && T2))
    if (base0 < n) wtile_fetch(T1 ? x2 : x1, base0, n, lane, pf);
  float AL[4][5], AR[4][5], AE[5];
  // afr[m][c][st][lane]: A fragment of lane for P_L (m = 0) / P_R (m = 1)
  __shared__ float afr[kA ? 2 : 1][4][5][64];
  if constexpr (kA) {
    for (int e = threadIdx.x; e < 2 * 4 * 5 * 64; e += kBlock) {
      const int mm = e / 1280, cc = (e / 320) & 3, st = (e / 64) % 5, l = e & 63;
      const int lo = l & 15, gg = l >> 4;
      const int k = 4 * (lo & 3) + (lo >> 2), col = 4 * st + gg;
      const float *Pm = mm ? right : left;
      afr[mm][cc][st][l] = ((mm == 0 && T1) || (mm == 1 && T2)) ? 0.f : Pm[cc * S * S + k * S + col];
    }
  }
  if constexpr (kA == 0) {
    const int k = 4 * (lo16 & 3) + (lo16 >> 2);  // pi: accumulators = back-transform B fragments
#pragma unroll
    for (int cc = 0; cc < 4; cc++)
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const int col = 4 * st + g;
        AL[cc][st] = T1 ? 0.f : left[cc * S * S + k * S + col];
        AR[cc][st] = T2 ? 0.f : right[cc * S * S + k * S + col];
      }
  }
#pragma unroll
  for (int st = 0; st < 5; st++) AE[st] = EV[(4 * st + g) * S + lo16];  // EV^T[l][k], natural rows
  __shared__ __attribute__((aligned(16))) float qm[3][4][4][S];
  for (int e = threadIdx.x; e < 4 * 4 * S; e += kBlock) {
    const int cc = e / (4 * S), i = (e / S) & 3, j = e % S;
    qm[0][cc][i][j] = T1 ? 0.f : left[cc * S * S + (16 + i) * S + j];
    qm[1][cc][i][j] = T2 ? 0.f : right[cc * S * S + (16 + i) * S + j];
    if (cc == 0) qm[2][0][i][j] = EV[j * S + 16 + i];
  }
  __shared__ float tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<float, true>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<float, true>(right, tipvec, tabs[1]);
  __syncthreads();
  if constexpr (kA == 1) {
#pragma unroll
    for (int cc = 0; cc < 4; cc++)
#pragma unroll
      for (int st = 0; st < 5; st++) {
        AL[cc][st] = afr[0][cc][st][lane];
        AR[cc][st] = afr[kA ? 1 : 0][cc][st][lane];
      }
  }
  // block b = lane/4 holds 4 sites of category g: A rows 16 + lane%4 of P_g
  const float *QL = &qm[0][g][lane & 3][0], *QR = &qm[1][g][lane & 3][0];
  const float *QE = &qm[2][0][lane & 3][0];
  const float m = Num<float>::minlik();
  __shared__ f32x4 tiles[kWavesPerBlock][16 * kWTileStride];
  f32x4 *tile = tiles[wv];
  const float *td = reinterpret_cast<const float *>(tile);
  float *tw = reinterpret_cast<float *>(tile);
  // U^T of a tip child, category c, in the accumulator layout (reg r of lane
  // group g = k 4r + g), and its rows 16..19 for the lane's (site, category g)
  auto tip_u = [&](const float *tab, int code, int cc) -> f32x4 {
    const float *r = tab + cc * kProtCodes * 20 + code * 20;
    return f32x4{r[g], r[g + 4], r[g + 8], r[g + 12]};
  };
  auto tip_q = [&](const float *tab, int code) -> f32x4 {
    const float *r = tab + g * kProtCodes * 20 + code * 20 + 16;
    return f32x4{r[0], r[1], r[2], r[3]};
  };
  long long acc = 0;
  auto product = [&](const float (&A)[4][5], int mA, const float *QA, f32x4 (&P)[4], f32x4 &Q, bool mul) {
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
    const float *xs = td + lo16 * kRow + g * S;  // the lane's own (site, category g) row
    const float *xr = td + lo16 * kRow + g;      // B: (site lo16, category c, state 4st + g)
#pragma unroll
    for (int cc = 0; cc < 4; cc++) {
      float bv[5];
#pragma unroll
      for (int st = 0; st < 5; st++) bv[st] = xr[cc * S + 4 * st];
      f32x4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const float a = kA == 2 ? afr[kA ? mA : 0][cc][st][lane] : A[cc][st];
        u = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[st], u, 0, 0, 0);
      }
      P[cc] = mul ? P[cc] * u : u;  // prod[k] = umpL[k] * umpR[k]
      const f32x4 xv = *reinterpret_cast<const f32x4 *>(xs + 4 * cc);
      const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 4 * cc);
#pragma unroll
      for (int j = 0; j < 4; j++) q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
    }
    const f32x4 xv = *reinterpret_cast<const f32x4 *>(xs + 16);
    const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 16);
#pragma unroll
    for (int j = 0; j < 4; j++) q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
    Q = mul ? Q * q : q;
  };
  for (int64_t base = base0; base < n; base += stride) {
    f32x4 P[4];
    f32x4 Q = {0.f, 0.f, 0.f, 0.f};  // p[16..19] of (site lo16, category g)
    const int64_t sq = base + lo16 < n ? base + lo16 : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (T1) {
#pragma unroll
      for (int cc = 0; cc < 4; cc++) P[cc] = tip_u(tabs[0], code1, cc);
      Q = tip_q(tabs[0], code1);
    } else {
      wtile_put(tile, lane, pf);
      __builtin_amdgcn_wave_barrier();
      if constexpr (T2) {
        if (base + stride < n) wtile_fetch(x1, base + stride, n, lane, pf);
      } else {
        wtile_fetch(x2, base, n, lane, pf);
      }
      product(AL, 0, QL, P, Q, false);
      __builtin_amdgcn_wave_barrier();
    }
    if constexpr (T2) {
#pragma unroll
      for (int cc = 0; cc < 4; cc++) P[cc] = P[cc] * tip_u(tabs[1], code2, cc);
      Q = Q * tip_q(tabs[1], code2);
    } else {
      wtile_put(tile, lane, pf);
      __builtin_amdgcn_wave_barrier();
      if (base + stride < n) wtile_fetch(T1 ? x2 : x1, base + stride, n, lane, pf);
      product(AR, 1, QR, P, Q, true);
      __builtin_amdgcn_wave_barrier();  // the tile takes X3 now
    }
    // lane (g, lo16): Qt[c] = p[16 + g] of (site lo16, category c)
    unsigned Qt[4] = {__float_as_uint(Q[0]), __float_as_uint(Q[1]), __float_as_uint(Q[2]),
                      __float_as_uint(Q[3])};
    transpose_groups44(Qt);
    // pk[k] = p[k] of (site lo16, category g), k = 0..15
    unsigned pk[16];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      unsigned v[4];
#pragma unroll
      for (int cc = 0; cc < 4; cc++) v[cc] = __float_as_uint(P[cc][r]);
      transpose_groups44(v);
#pragma unroll
      for (int gg = 0; gg < 4; gg++) pk[4 * r + gg] = v[gg];
    }
    unsigned long long mask = 0xFFFFull;  // bit s: site base + s scales
#pragma unroll
    for (int cc = 0; cc < 4; cc++) {
      f32x4 X0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const float b = st == 4 ? __uint_as_float(Qt[cc]) : P[cc][st];
        X0 = __builtin_amdgcn_mfma_f32_16x16x4f32(AE[st], b, X0, 0, 0, 0);
      }
      // lane group g holds states 4g..4g+3 of (site lo16, category cc)
      const bool small = (__builtin_fabsf(X0[0]) < m) && (__builtin_fabsf(X0[1]) < m) &&
                         (__builtin_fabsf(X0[2]) < m) && (__builtin_fabsf(X0[3]) < m);
      const unsigned long long b = __ballot(small);
      mask &= b & (b >> 16) & (b >> 32) & (b >> 48);
      *reinterpret_cast<f32x4 *>(tw + lo16 * kRow + cc * S + 4 * g) = X0;
    }
    {  // states 16..19 of (site lo16, category g): 20 K = 1 steps, k ascending
      f32x4 X1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 20; k++) {
        const float a = reinterpret_cast<const f32x4 *>(QE)[k >> 2][k & 3];
        const float b = k < 16 ? __uint_as_float(pk[k]) : Q[k & 3];
        X1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, X1, 0, 0, 0);
      }
      const bool small = (__builtin_fabsf(X1[0]) < m) && (__builtin_fabsf(X1[1]) < m) &&
                         (__builtin_fabsf(X1[2]) < m) && (__builtin_fabsf(X1[3]) < m);
      const unsigned long long b = __ballot(small);
      mask &= b & (b >> 16) & (b >> 32) & (b >> 48);
      *reinterpret_cast<f32x4 *>(tw + lo16 * kRow + g * S + 16) = X1;
    }
    __builtin_amdgcn_wave_barrier();
    if (g == 0) {
      const int64_t site = base + lo16;
      const bool sc = (mask >> lo16) & 1ull;
      if (site < n) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
    }
    {  // coalesced store with the rescale of the scaled sites (exact: x 2^32)
      f32x4 *dst = reinterpret_cast<f32x4 *>(x3 + base * 80);
      f32x4 v[5];
#pragma unroll
      for (int i = 0; i < 5; i++) {
        const int j = lane + 64 * i;
        const int s = j / 20, q = j - 20 * s;
        v[i] = tile[s * kWTileStride + q];
        if ((mask >> s) & 1ull) v[i] = v[i] * Num<float>::two32();
      }
      if (base + 16 <= n) {
#pragma unroll
        for (int i = 0; i < 5; i++) __builtin_nontemporal_store(v[i], dst + lane + 64 * i);
      } else {
        const int64_t lim = (n - base) * 20;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          const int j = lane + 64 * i;
          if (j < lim) __builtin_nontemporal_store(v[i], dst + j);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
