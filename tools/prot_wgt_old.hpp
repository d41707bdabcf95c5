// prot_wgt_old.hpp -- tuning copy (not product code): the protein exact and
// f32 FMA kernels as they were before the site weight moved to an
// unconditional load at the start of each trip (the old form loads wgt[site]
// inside the scaled-site branch, and its s_waitcnt vmcnt(0) there also waits
// for the next child tile already in flight).  For same-process A/B runs only.
#pragma once
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

template <typename T, bool kSum, int kTips, int kRows, bool kE3S>
__device__ __forceinline__ void prot_lds_body_old(const T *__restrict__ x1, const T *__restrict__ x2,
                                              T *__restrict__ x3, const T *__restrict__ EV,
                                              const T *__restrict__ left, const T *__restrict__ right,
                                              const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                              int64_t n, unsigned long long *ws, int64_t *scaler_sum,
                                              const T *__restrict__ tipvec) {
  constexpr int S = 20;
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  using PT = ProtTile<T>;
  using V = typename PT::V;
  constexpr int E = 16 / (int)sizeof(T);          // elements per 16-B LDS read
  constexpr int kPh3 = sizeof(T) == 8 ? 10 : 20;  // phase-3 chains per pass
  static_assert(kRows % E == 0 && S % kRows == 0, "kRows: a divisor of 20, whole 16-B reads");
  constexpr int RV = kRows / E, PV = kPh3 / E, kDist = 2;
  __shared__ T tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<T, false>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<T, false>(right, tipvec, tabs[1]);
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // P_L[4][400] (unless x1 is a tip) | P_R[4][400] (unless x2 is a tip) | EV[400]
  // in T elements; a tip child's matrix lives in its table instead
  constexpr int oR = T1 ? 0 : 4 * S * S, oE = oR + (T2 ? 0 : 4 * S * S);
  __shared__ V mats[(oE + S * S) / E];
  {
    T *md = reinterpret_cast<T *>(mats);
    for (int i = threadIdx.x; i < 4 * S * S; i += kBlock) {  // P[c][k][l] -> [c][k/kRows][l][k%kRows]
      const int cc = i / (S * S), r = i - cc * S * S, k = r / S, l = r - k * S;
      const int d = cc * S * S + (k / kRows) * (S * kRows) + l * kRows + (k % kRows);
      if constexpr (!T1) md[d] = left[i];
      if constexpr (!T2) md[oR + d] = right[i];
    }
    for (int i = threadIdx.x; i < S * S; i += kBlock) md[oE + i] = EV[i];
  }
  const T m = Num<T>::minlik();
  __shared__ V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  __syncthreads();
  // phases 1/2: M = the category's group-transposed matrix, x = the child's 20
  // values; fn(k, sum_l x[l] * M[k][l]) for every k
  auto gphase = [&](const V *M, const T (&x)[S], auto &&fn) {
    int o = 0;
    T tok = T(0);
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const V *G = M + gk * S * RV;
      V ring[kDist + 1][RV];
      T u[kRows];
      asm volatile("" : "+v"(o) : "v"(tok));  // the group's first columns after the last group's end
#pragma unroll
      for (int l = 0; l < kDist; l++)
#pragma unroll
        for (int j = 0; j < RV; j++) ring[l][j] = G[o + l * RV + j];
#pragma unroll
      for (int l = 0; l < S; l++) {
        asm volatile("" : "+v"(o) : "v"(tok));  // column l+kDist is read after column l-1 is used
        if (l + kDist < S) {
#pragma unroll
          for (int j = 0; j < RV; j++) ring[(l + kDist) % (kDist + 1)][j] = G[o + (l + kDist) * RV + j];
        }
        const V *col = ring[l % (kDist + 1)];
        // all kRows products, then all kRows adds: no add waits on the
        // multiply just before it (chains start at q0: site_cat, plf_dna.hpp)
        T pr[kRows];
#pragma unroll
        for (int j = 0; j < kRows; j++) pr[j] = x[l] * col[j / E][j % E];
        pin_chains(pr);
#pragma unroll
        for (int j = 0; j < kRows; j++) u[j] = l == 0 ? pr[j] : u[j] + pr[j];
        pin_chains(u);
        tok = u[kRows - 1];
      }
#pragma unroll
      for (int j = 0; j < kRows; j++) fn(gk * kRows + j, u[j]);
    }
  };
  constexpr bool kAnyDense = !(T1 && T2);
  const T *FD = T1 ? x2 : x1;  // the trip's first dense child
  const int64_t stride = (int64_t)gridDim.x * 64;
  constexpr int K = PT::kChunks / kBlock;
  V pf[K];  // unused (and eliminated) when both children are tips
  if constexpr (kAnyDense)
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<T>(FD, (int64_t)blockIdx.x * 64, n, pf);
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const V *mL = mats + off + c * (S * S / E), *mR = mats + off + (oR + c * S * S) / E,
            *mE = mats + off + oE / E;
    T U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    // stage a dense child's tile from the prefetch registers, then fetch the
    // next tile in the sequence
    auto stage = [&](const T *next, int64_t nbase) {
      tile_put<T>(tile, pf);
      __syncthreads();
      if (nbase < n) tile_fetch<T>(next, nbase, n, pf);
    };
    if constexpr (T1) {  // tip: U from the table row of the site's code
      const T *r = tabs[0] + c * kProtCodes * 20 + prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) * 20;
#pragma unroll
      for (int k = 0; k < S; k++) U[k] = r[k];
    } else {
      T a[S];
      // next in the sequence: this trip's x2, or the next trip's x1 when x2 is a tip
      stage(T2 ? x1 : x2, T2 ? base + stride : base);
      row_read<T>(tile, lane, c, a);
      __syncthreads();
      gphase(mL, a, [&](int k, T u) { U[k] = u; });
    }
    if constexpr (T2) {
      const T *r = tabs[1] + c * kProtCodes * 20 + prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) * 20;
#pragma unroll
      for (int k = 0; k < S; k++) U[k] = U[k] * r[k];
    } else {
      T b[S];
      stage(FD, base + stride);  // next: the next trip's first dense child
      row_read<T>(tile, lane, c, b);
      __syncthreads();
      gphase(mR, b, [&](int k, T u) { U[k] = U[k] * u; });
    }
    // phase 3: O[l] = sum_k U[k] * EV[k][l] from +0.0, kPh3 chains per pass
    T O[S];
    {
      int o = 0;
      T tok = T(0);
#pragma unroll
      for (int h = 0; h < S / kPh3; h++) {
        const V *G = mE + h * PV;  // EV row k, states h*kPh3..: G[o + k*(S/E) + j]
        V ring[3][PV];
        T v[kPh3];
#pragma unroll
        for (int j = 0; j < kPh3; j++) v[j] = T(0);
        asm volatile("" : "+v"(o) : "v"(tok));
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
          for (int j = 0; j < PV; j++) ring[k][j] = G[o + (S / E) * k + j];
#pragma unroll
        for (int k = 0; k < S; k++) {
          asm volatile("" : "+v"(o) : "v"(tok));
          if (k + 2 < S) {
#pragma unroll
            for (int j = 0; j < PV; j++) ring[(k + 2) % 3][j] = G[o + (S / E) * (k + 2) + j];
          }
          const V *e = ring[k % 3];
          T pr[kPh3];
          if constexpr (kE3S) {
            // EV row k straight from global memory at a wave-uniform address:
            // scalar loads, SGPR operands, one row ahead (the opaque offset);
            // the ring's LDS reads are dead and dropped
            int so = 0;
            asm volatile("" : "+s"(so) : "v"(tok));
            const T *er = EV + so + k * S + h * kPh3;
#pragma unroll
            for (int j = 0; j < kPh3; j++) pr[j] = U[k] * er[j];
          } else {
#pragma unroll
            for (int j = 0; j < kPh3; j++) pr[j] = U[k] * e[j / E][j % E];
          }
          pin_chains(pr);
#pragma unroll
          for (int j = 0; j < kPh3; j++) v[j] += pr[j];
          pin_chains(v);
          tok = v[kPh3 - 1];
        }
#pragma unroll
        for (int j = 0; j < kPh3; j++) O[h * kPh3 + j] = v[j];
      }
    }
    bool small = base + lane < n;
#pragma unroll
    for (int l = 0; l < S; l++) small = small && (Num<T>::abs(O[l]) < m);
    const unsigned long long mk = __ballot(small);
    if (lane == 0) small_mask[c] = mk;
    __syncthreads();  // also: every wave is done reading x2 from the tile
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    const bool sc = (all >> lane) & 1ull;
#pragma unroll
    for (int l = 0; l < S; l++) {
      const T sv = O[l] * Num<T>::two32();
      O[l] = sc ? sv : O[l];
    }
    row_write<T>(tile, lane, c, O);
    const int64_t site = base + lane;
    if (site < n && c == 0) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
    }
    __syncthreads();
    tile_store<T>(x3, base, n, tile);
    __syncthreads();  // tile and small_mask are reused by the next trip
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

template <typename T, bool kSum, int kMinWaves, int kTips, int kRows, bool kE3S>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_lds_old_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
                    const T *__restrict__ EV, const T *__restrict__ left, const T *__restrict__ right,
                    const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                    unsigned long long *ws, int64_t *scaler_sum, const T *__restrict__ tipvec = nullptr) {
  prot_lds_body_old<T, kSum, kTips, kRows, kE3S>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws,
                                              scaler_sum, tipvec);
}

template <bool kSum, int kMinWaves, int kTips, int kWaitAll = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma32_old_kernel(const float *__restrict__ x1, const float *__restrict__ x2,
                       float *__restrict__ x3, const float *__restrict__ EV,
                       const float *__restrict__ left, const float *__restrict__ right,
                       const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                       unsigned long long *ws, int64_t *scaler_sum,
                       const float *__restrict__ tipvec = nullptr) {
  constexpr int S = 20;
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  using PT = ProtTile<float>;
  constexpr int kRow = 4 * PT::kStride;  // floats per site in the LDS tile (84)
  constexpr int K = PT::kChunks / kBlock;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lo16 = lane & 15, g = lane >> 4;
  const int64_t stride = (int64_t)gridDim.x * 64;
  f32x4 pf[K];
  // the first dense child's first tile, before the matrix fragments
  if constexpr (!(T1 && T2))
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<float>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  float AL[2][5], AR[2][5], AE[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; mt++)
#pragma unroll
    for (int st = 0; st < 5; st++) {
      const int i = lo16, col = 4 * st + g;
      const int k = 16 * mt + 4 * (i & 3) + (i >> 2);  // pi: accumulators = back-transform B fragments
      AL[mt][st] = (k < S && !mt) ? left[c * S * S + k * S + col] : 0.f;   // P_L[k][l]
      AR[mt][st] = (k < S && !mt) ? right[c * S * S + k * S + col] : 0.f;
      const int lrow = 16 * mt + i;  // EV^T[l][k]: natural rows
      AE[mt][st] = (lrow < S && !mt) ? EV[col * S + lrow] : 0.f;
    }
  // A operands of the 4x4x1 chains in LDS (registers would cost 40-60 VGPRs
  // and the third block per CU): qm[0|1][cat][i][col] = P_L|P_R[16+i][col],
  // qm[2][0][i][k] = EV[k][16+i]; lane l reads row i = l%4 as 16-B pieces (4
  // distinct addresses per 16 lanes, 20 banks apart: no conflicts)
  __shared__ __attribute__((aligned(16))) float qm[3][4][4][S];
  for (int e = threadIdx.x; e < 4 * 4 * S; e += kBlock) {
    const int cc = e / (4 * S), i = (e / S) & 3, j = e % S;
    qm[0][cc][i][j] = T1 ? 0.f : left[cc * S * S + (16 + i) * S + j];
    qm[1][cc][i][j] = T2 ? 0.f : right[cc * S * S + (16 + i) * S + j];
    if (cc == 0) qm[2][0][i][j] = EV[j * S + 16 + i];
  }
  __syncthreads();
  const float *QL = &qm[0][c][lane & 3][0], *QR = &qm[1][c][lane & 3][0];
  const float *QE = &qm[2][0][lane & 3][0];
  const float m = Num<float>::minlik();
  __shared__ float tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<float, true>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<float, true>(right, tipvec, tabs[1]);
  if constexpr (T1) __syncthreads();
  // U^T of a tip child for sub-tile t in the accumulator layout (reg r of
  // lane group g = k 4r + g; tile 1 reg 0 = k 16 + g)
  auto tip_u = [&](const float *tab, int code_lane, int t, f32x4 &u0, f32x4 &u1) {
    const float *r = tab + c * kProtCodes * 20 + __shfl(code_lane, 16 * t + lo16) * 20;
    u0 = f32x4{r[g], r[g + 4], r[g + 8], r[g + 12]};
    u1 = f32x4{r[16 + g], 0.f, 0.f, 0.f};
  };
  __shared__ f32x4 tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const float *td = reinterpret_cast<const float *>(tile);
  float *tw = reinterpret_cast<float *>(tile);
  long long acc = 0;
  // one child's product U^T for the 4 sub-tiles from the LDS tile (mul: into P)
  // and rows 16..19 of the lane's own site into Q (4x4x1 chain, k ascending)
  auto product = [&](const float (&A)[2][5], const float *QA, f32x4 (&P)[4][2], f32x4 &Q, bool mul,
                     const float *tb) {
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
    const float *xs = tb + lane * kRow + c * S;  // the lane's own site row
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const float *xr = tb + (16 * t + lo16) * kRow + c * S + g;
      float bv[5];
#pragma unroll
      for (int st = 0; st < 5; st++) bv[st] = xr[4 * st];
      {
        f32x4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 5; st++) u = __builtin_amdgcn_mfma_f32_16x16x4f32(A[0][st], bv[st], u, 0, 0, 0);
        P[t][0] = mul ? P[t][0] * u : u;  // prod[k] = umpL[k] * umpR[k]
      }
      {  // four of the 20 K = 1 steps per sub-tile, interleaved
        const f32x4 xv = *reinterpret_cast<const f32x4 *>(xs + 4 * t);
        const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 4 * t);
#pragma unroll
        for (int j = 0; j < 4; j++) q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
      }
    }
    {
      const f32x4 xv = *reinterpret_cast<const f32x4 *>(xs + 16);
      const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 16);
#pragma unroll
      for (int j = 0; j < 4; j++) q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
      Q = mul ? Q * q : q;
    }
  };
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    f32x4 P[4][2];
    f32x4 Q = {0.f, 0.f, 0.f, 0.f};  // U[16..19] (then p[16..19]) of site `lane`
#pragma unroll
    for (int t = 0; t < 4; t++) P[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};  // rows 16..19 live in Q
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    // a tip child's U[16..19] of the lane's own site from its table row
    auto tip_q = [&](const float *tab, int code_lane) -> f32x4 {
      const float *r = tab + c * kProtCodes * 20 + code_lane * 20 + 16;
      return f32x4{r[0], r[1], r[2], r[3]};
    };
    if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
      Q = tip_q(tabs[0], code1);
    } else {
      tile_put<float>(tile, pf);
      __syncthreads();
      // next: this trip's x2, or the next trip's x1 when x2 is a tip
      if constexpr (T2) {
        if (base + stride < n) tile_fetch<float>(x1, base + stride, n, pf);
      } else {
        tile_fetch<float>(x2, base, n, pf);
      }
      product(AL, QL, P, Q, false, td);
      __syncthreads();
    }
    if constexpr (T2) {
#pragma unroll
      for (int t = 0; t < 4; t++) {
        f32x4 u0, u1;
        tip_u(tabs[1], code2, t, u0, u1);
        P[t][0] = P[t][0] * u0;
        P[t][1] = P[t][1] * u1;
      }
      Q = Q * tip_q(tabs[1], code2);
    } else {
      tile_put<float>(tile, pf);
      __syncthreads();
      if (base + stride < n) tile_fetch<float>(T1 ? x2 : x1, base + stride, n, pf);
      product(AR, QR, P, Q, true, td);
      __syncthreads();  // every wave is done reading x2: the tile takes X3 now
    }
    // lane group g gets p[16 + g] of sub-tile t's site lo16 as Qt[t]
    // (__float_as_uint: __builtin_bit_cast of a vector element reads element 0
    // with this compiler)
    unsigned Qt[4] = {__float_as_uint(Q[0]), __float_as_uint(Q[1]), __float_as_uint(Q[2]),
                      __float_as_uint(Q[3])};
    transpose_groups44(Qt);
    // p[k][site lane] for k = 0..15 (four transposes of the P rows)
    unsigned pk[16];
    {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        unsigned v[4];
#pragma unroll
        for (int t = 0; t < 4; t++) v[t] = __float_as_uint(P[t][0][r]);
        transpose_groups44(v);  // lane (t, lo16) reg g' = p[4r + g'][site 16t + lo16]
#pragma unroll
        for (int gg = 0; gg < 4; gg++) pk[4 * r + gg] = v[gg];
      }
    }
    // back-transform: B fragment of k-step s = P[t][0][s] (s < 4), Qt[t] (s = 4)
    unsigned long long mine = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      f32x4 X0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const float b = st == 4 ? __uint_as_float(Qt[t]) : P[t][st >> 2][st & 3];
        X0 = __builtin_amdgcn_mfma_f32_16x16x4f32(AE[0][st], b, X0, 0, 0, 0);
      }
      // lane group g holds states 4g..4g+3
      bool small = (__builtin_fabsf(X0[0]) < m) && (__builtin_fabsf(X0[1]) < m) &&
                   (__builtin_fabsf(X0[2]) < m) && (__builtin_fabsf(X0[3]) < m);
      const unsigned long long b = __ballot(small);
      mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
      float *w = tw + (16 * t + lo16) * kRow + c * S;
      *reinterpret_cast<f32x4 *>(w + 4 * g) = X0;
    }
    {  // states 16..19 of site `lane`: 20 K = 1 steps, k ascending
      f32x4 X1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 20; k++) {
        const float a = reinterpret_cast<const f32x4 *>(QE)[k >> 2][k & 3];
        const float b = k < 16 ? __uint_as_float(pk[k & 15]) : Q[k & 3];
        X1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, X1, 0, 0, 0);
      }
      const bool small = (__builtin_fabsf(X1[0]) < m) && (__builtin_fabsf(X1[1]) < m) &&
                         (__builtin_fabsf(X1[2]) < m) && (__builtin_fabsf(X1[3]) < m);
      mine &= __ballot(small);
      *reinterpret_cast<f32x4 *>(tw + lane * kRow + c * S + 16) = X1;
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
    // kWaitAll: every wave waits for its loads in flight before its share of
    // the store pass (the product: wave 0 only, through its weight load)
    if constexpr (kWaitAll == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // coalesced store with the rescale of the scaled sites (exact: x 2^32)
    {
      f32x4 *dst = reinterpret_cast<f32x4 *>(x3 + base * 80);
      f32x4 v[K];
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        const int sl = j / PT::kChunksPerSite, q = j - sl * PT::kChunksPerSite;
        v[i] = tile[sl * PT::kStride + q];
        if ((all >> sl) & 1ull) v[i] = v[i] * Num<float>::two32();
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
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
