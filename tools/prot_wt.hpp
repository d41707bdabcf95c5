// prot_wt.hpp -- (measured, not adopted: HISTORY.md section 3.3, round 4) exact-mode protein (S = 20, C = 4) node update with
// wave-private site tiles: plf()'s loop (app/src/plf.cpp:19-65, 4 -> 20
// states) with separate multiplies and adds in its order, bit-identical to
// plf_prot_lds_kernel and to the double / float instantiation of the loop.
//
// Why a second form (HISTORY.md section 3.3, round 4): plf_prot_lds_kernel
// runs one category per wave over a 64-site block tile, so every child tile and
// the 80-value scale test cross the block's four waves through LDS barriers,
// and its 42-KB tile plus a 28.8-KB matrix copy per block hold the CU to two
// blocks -- two waves per SIMD, whose VALU, LDS and HBM phases serialise
// (VALU busy ~60 % at its 2 700 f64 instructions per wave and tile).  Here:
//   * a wave owns 16 sites x 4 categories per trip: lane l = (category c, site
//     s) with c = (l >> 2) & 3, s = (l & 3) | ((l >> 4) << 2), so the four
//     categories of a site are lanes b, b+4, b+8, b+12 and the 80-value scale
//     test is ONE ballot: no LDS mask exchange, no block barrier in the loop;
//   * the child tile (16 x 640 B f64, coalesced 16-B loads) passes through the
//     wave's own LDS region only -- waves run independently;
//   * one block of kWtWaves = 12 waves per CU shares a single copy of P_L and
//     P_R (25.6 KB f64; EV rows are scalar loads, SGPR operands), so the 12
//     wave tiles fit beside it: THREE waves per SIMD (168 VGPRs each);
//   * matrix reads: lane c reads its category's group-transposed P, the four
//     category copies 816 dwords apart (= 48 mod 64: four disjoint bank sets
//     in a ds_read_b128 lane group); tile rows 44 chunks of 16 B per site,
//     categories 11 chunks apart: every row read, row write and staging access
//     of the lane map is conflict-free (bank model: HISTORY.md section 3.3).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "plf_dna.hpp"
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

constexpr int kWtWaves = 12;            // waves per block, one block per CU
constexpr int kWtThreads = 64 * kWtWaves;

template <typename T>
struct WtLayout {
  static constexpr int E = 16 / (int)sizeof(T);      // values per 16-B chunk
  static constexpr int kCatChunks = 20 / E;          // a (site, category) row: 10 f64 / 5 f32
  static constexpr int kCatStride = sizeof(T) == 8 ? 11 : 6;   // chunks between categories
  static constexpr int kSiteStride = sizeof(T) == 8 ? 44 : 24; // chunks per site
  static constexpr int kSiteChunks = 4 * kCatChunks;           // 40 / 20 in HBM
  static constexpr int kTileChunks = 16 * kSiteChunks;         // 640 / 320 per child tile
  static constexpr int kLoads = kTileChunks / 64;              // 10 / 5 per lane
  static constexpr int kMatStride = sizeof(T) == 8 ? 408 : 400 + 12;  // values per category (padded)
  typedef typename ProtTile<T>::V V;
};

// LDS chunk of tile chunk j (j = site * kSiteChunks + category * kCatChunks + i)
template <typename T>
__device__ __forceinline__ int wt_slot(int j) {
  using L = WtLayout<T>;
  const int sl = j / L::kSiteChunks, q = j - sl * L::kSiteChunks;
  const int c = q / L::kCatChunks, i = q - c * L::kCatChunks;
  return sl * L::kSiteStride + c * L::kCatStride + i;
}

// the wave's 16-site tile of child x (sites base..base+15, zero past n) into
// its LDS region: every load in flight before the first LDS write
template <typename T>
__device__ __forceinline__ void wt_stage(const T *__restrict__ x, int64_t base, int64_t n, int lane,
                                         typename WtLayout<T>::V *tile) {
  using L = WtLayout<T>;
  using V = typename L::V;
  V v[L::kLoads];
  const V *src = reinterpret_cast<const V *>(x + base * 80);
  if (base + 16 <= n) {
#pragma unroll
    for (int r = 0; r < L::kLoads; r++) v[r] = __builtin_nontemporal_load(src + lane + 64 * r);
  } else {
    const int lim = (int)(n - base) * L::kSiteChunks;
#pragma unroll
    for (int r = 0; r < L::kLoads; r++) {
      v[r] = V{};
      if (lane + 64 * r < lim) v[r] = __builtin_nontemporal_load(src + lane + 64 * r);
    }
  }
#pragma unroll
  for (int r = 0; r < L::kLoads; r++) tile[wt_slot<T>(lane + 64 * r)] = v[r];
}

// LDS accesses of one wave to its own tile are executed in issue order; this
// keeps the compiler from moving them across each other between phases
__device__ __forceinline__ void wt_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// kXL: the child row is read from the wave's LDS tile one 16-B chunk at a
// time as the phase streams its columns (2 steps ahead) instead of being held
// in 20 registers -- the registers pay for kRows = 10 chains.
// kAb (timing ablations of the tuning harness only; 0 in the product):
// bit 0 no HBM traffic (tiles staged from registers, no x3 stores), bit 1 no
// LDS matrix reads (a register constant instead), bit 2 no phase 3
template <typename T, bool kSum, int kRows, int kAb = 0, bool kXL = false>
__device__ __forceinline__ void prot_wt_body(const T *__restrict__ x1, const T *__restrict__ x2,
                                             T *__restrict__ x3, const T *__restrict__ EV,
                                             const T *__restrict__ left, const T *__restrict__ right,
                                             const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                             int64_t n, unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using L = WtLayout<T>;
  using V = typename L::V;
  constexpr int E = L::E;
  constexpr int kPh3 = sizeof(T) == 8 ? 10 : 20;  // phase-3 chains per pass
  static_assert(kRows % E == 0 && S % kRows == 0, "kRows: a divisor of 20, whole 16-B reads");
  constexpr int RV = kRows / E, kDist = 2, CS = L::kMatStride;
  __shared__ V mats[2 * 4 * CS / E];                   // P_L | P_R, [c][k/kRows][l][k%kRows]
  __shared__ V tiles[kWtWaves][16 * L::kSiteStride];
  __shared__ long long part[kWtWaves];
  {
    T *md = reinterpret_cast<T *>(mats);
    for (int i = threadIdx.x; i < 4 * S * S; i += kWtThreads) {
      const int cc = i / (S * S), r = i - cc * S * S, k = r / S, l = r - k * S;
      const int d = cc * CS + (k / kRows) * (S * kRows) + l * kRows + (k % kRows);
      md[d] = left[i];
      md[4 * CS + d] = right[i];
    }
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = (lane >> 2) & 3, s = (lane & 3) | ((lane >> 4) << 2);
  V *tile = tiles[w];
  V *row = tile + s * L::kSiteStride + c * L::kCatStride;
  const T m = Num<T>::minlik();
  long long acc = 0;
  // phases 1/2: M = this lane's category matrix (group-transposed), x = the
  // child row; fn(k, sum_l x[l] * M[k][l]) for every k, kRows chains at a time,
  // each chain in plf()'s order (first product, then ascending l)
  auto gphase = [&](const V *M, const T (&x)[S], auto &&fn) {
    int o = 0;
    T tok = T(0);
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const V *G = M + gk * S * RV;
      V ring[kDist + 1][RV];
      T u[kRows];
      asm volatile("" : "+v"(o) : "v"(tok));
#pragma unroll
      for (int l = 0; l < kDist; l++)
#pragma unroll
        for (int j = 0; j < RV; j++) ring[l][j] = G[o + l * RV + j];
#pragma unroll
      for (int l = 0; l < S; l++) {
        asm volatile("" : "+v"(o) : "v"(tok));
        if (l + kDist < S) {
#pragma unroll
          for (int j = 0; j < RV; j++) {
            if constexpr (kAb & 2) ring[(l + kDist) % (kDist + 1)][j] = V{} + (T)(o + l + j);
            else ring[(l + kDist) % (kDist + 1)][j] = G[o + (l + kDist) * RV + j];
          }
        }
        const V *col = ring[l % (kDist + 1)];
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
  // gphase with the child row streamed from the tile (kXL)
  auto gphase_xl = [&](const V *M, auto &&fn) {
    int o = 0;
    T tok = T(0);
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const V *G = M + gk * S * RV;
      V ring[kDist + 1][RV];
      V xc[2];
      T u[kRows];
      asm volatile("" : "+v"(o) : "v"(tok));
#pragma unroll
      for (int l = 0; l < kDist; l++)
#pragma unroll
        for (int j = 0; j < RV; j++) ring[l][j] = G[o + l * RV + j];
      xc[0] = row[o];
#pragma unroll
      for (int l = 0; l < S; l++) {
        asm volatile("" : "+v"(o) : "v"(tok));
        if (l + kDist < S) {
#pragma unroll
          for (int j = 0; j < RV; j++) {
            if constexpr (kAb & 2) ring[(l + kDist) % (kDist + 1)][j] = V{} + (T)(o + l + j);
            else ring[(l + kDist) % (kDist + 1)][j] = G[o + (l + kDist) * RV + j];
          }
        }
        if (l % E == 0 && l / E + 1 < L::kCatChunks) xc[(l / E + 1) % 2] = row[o + l / E + 1];
        const T xl = xc[(l / E) % 2][l % E];
        const V *col = ring[l % (kDist + 1)];
        T pr[kRows];
#pragma unroll
        for (int j = 0; j < kRows; j++) pr[j] = xl * col[j / E][j % E];
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
  auto read_row = [&](T (&v)[S]) {
#pragma unroll
    for (int i = 0; i < L::kCatChunks; i++) {
      const V t = row[i];
#pragma unroll
      for (int e = 0; e < E; e++) v[E * i + e] = t[e];
    }
  };
  const int64_t ntiles = (n + 15) / 16;
  const int64_t G = (int64_t)gridDim.x * kWtWaves;
  for (int64_t t = (int64_t)blockIdx.x * kWtWaves + w; t < ntiles; t += G) {
    const int64_t base = t * 16, site = base + s;
    const int64_t sq = site < n ? site : n - 1;
    const int wsite = kSum ? wgt_at(wgt, sq, ws) : 0;
    int off = 0;
    asm volatile("" : "+v"(off));  // keeps the matrix reads inside the trip
    const V *mL = mats + off + c * (CS / E), *mR = mats + off + (4 * CS + c * CS) / E;
    T U[S];
    if constexpr (kXL) {
      if constexpr (kAb & 1) tile[lane] = V{} + (T)t;
      else wt_stage<T>(x1, base, n, lane, tile);
      wt_wave_sync();
      gphase_xl(mL, [&](int k, T u) { U[k] = u; });
      wt_wave_sync();
      if constexpr (kAb & 1) tile[lane + 64] = V{} + (T)t;
      else wt_stage<T>(x2, base, n, lane, tile);
      wt_wave_sync();
      gphase_xl(mR, [&](int k, T u) { U[k] = U[k] * u; });
      wt_wave_sync();
    } else {
      {
        T a[S];
        if constexpr (kAb & 1) tile[lane] = V{} + (T)t;
        else wt_stage<T>(x1, base, n, lane, tile);
        wt_wave_sync();
        read_row(a);
        wt_wave_sync();
        gphase(mL, a, [&](int k, T u) { U[k] = u; });
      }
      {
        T b[S];
        if constexpr (kAb & 1) tile[lane + 64] = V{} + (T)t;
        else wt_stage<T>(x2, base, n, lane, tile);
        wt_wave_sync();
        read_row(b);
        wt_wave_sync();
        gphase(mR, b, [&](int k, T u) { U[k] = U[k] * u; });
      }
    }
    // phase 3: O[l] = sum_k U[k] * EV[k][l] from +0.0; EV rows by scalar
    // loads (SGPR operands, one row ahead through the opaque offset)
    T O[S];
    if constexpr (kAb & 4) {
#pragma unroll
      for (int l = 0; l < S; l++) O[l] = U[l];
    } else {
      T tok = T(0);
#pragma unroll
      for (int h = 0; h < S / kPh3; h++) {
        T v[kPh3];
#pragma unroll
        for (int j = 0; j < kPh3; j++) v[j] = T(0);
#pragma unroll
        for (int k = 0; k < S; k++) {
          int so = 0;
          asm volatile("" : "+s"(so) : "v"(tok));
          const T *er = EV + so + k * S + h * kPh3;
          T pr[kPh3];
#pragma unroll
          for (int j = 0; j < kPh3; j++) pr[j] = U[k] * er[j];
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
    // the site's 80-value test: this lane's 20, then the 4 category lanes of
    // the site (bits b, b+4, b+8, b+12 of the ballot, b = its category-0 lane)
    bool small = site < n;
#pragma unroll
    for (int l = 0; l < S; l++) small = small && (Num<T>::abs(O[l]) < m);
    const unsigned long long mk = __ballot(small);
    const unsigned long long all = mk & (mk >> 4) & (mk >> 8) & (mk >> 12);
    const bool sc = (all >> (lane & 0x33)) & 1ull;  // bit of lane (c = 0, s)
#pragma unroll
    for (int l = 0; l < S; l++) {
      const T sv = O[l] * Num<T>::two32();
      O[l] = sc ? sv : O[l];
    }
#pragma unroll
    for (int i = 0; i < L::kCatChunks; i++) {
      V t;
#pragma unroll
      for (int e = 0; e < E; e++) t[e] = O[E * i + e];
      row[i] = t;
    }
    if (c == 0 && site < n) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wsite;
    }
    wt_wave_sync();
    {
      V v[L::kLoads];
#pragma unroll
      for (int r = 0; r < L::kLoads; r++) v[r] = tile[wt_slot<T>(lane + 64 * r)];
      V *dst = reinterpret_cast<V *>(x3 + base * 80);
      if constexpr (kAb & 1) {
        if (v[0][0] == T(-1.2345)) __builtin_nontemporal_store(v[0], dst + lane);  // keep the reads
      } else if (base + 16 <= n) {
#pragma unroll
        for (int r = 0; r < L::kLoads; r++) __builtin_nontemporal_store(v[r], dst + lane + 64 * r);
      } else {
        const int lim = (int)(n - base) * L::kSiteChunks;
#pragma unroll
        for (int r = 0; r < L::kLoads; r++)
          if (lane + 64 * r < lim) __builtin_nontemporal_store(v[r], dst + lane + 64 * r);
      }
    }
    wt_wave_sync();  // the tile is restaged by the next trip
  }
  if constexpr (kSum) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) part[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      long long tot = 0;
#pragma unroll
      for (int i = 0; i < kWtWaves; i++) tot += part[i];
      ticket_publish(tot, ws, scaler_sum);
    }
  }
}

template <typename T, bool kSum, int kRows, int kAb = 0, bool kXL = false>
__global__ void __launch_bounds__(kWtThreads, 1)
plf_prot_wt_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
                   const T *__restrict__ EV, const T *__restrict__ left, const T *__restrict__ right,
                   const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                   unsigned long long *ws, int64_t *scaler_sum) {
  prot_wt_body<T, kSum, kRows, kAb, kXL>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
