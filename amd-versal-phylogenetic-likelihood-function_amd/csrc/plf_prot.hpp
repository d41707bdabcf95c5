// plf_prot.hpp -- fused PLF inner-node update for S=20 states (protein) x C=4
// Gamma categories (extension: the reference hard-wires DNA, SURVEY F9 /
// BASELINE configs[4]).  Same loop as plf() (app/src/plf.cpp:19-65) with 4
// replaced by 20: ump[k] = sum_l x[c][l]*P_c[k][l] (ascending l from +0.0),
// prod[k] = umpL*umpR, x3[c][l] = sum_k prod[k]*EV[k][l] (ascending k from
// +0.0), site scaled iff all 80 |x3| < 2^-32.
//
// Common mapping: a 256-thread block owns 64 consecutive sites per trip of a
// grid-stride loop; wave w = category c.  Child tiles pass through LDS
// (coalesced 16-B non-temporal loads into padded, conflict-free rows; lane =
// site straight on HBM re-read every line once per category-wave and thrashed
// L2).  The 80-value scale test of a site spans the 4 waves: each wave ballots
// its 20-value test, the 4 masks meet in LDS and are ANDed.  X3 leaves through
// the same tile with coalesced non-temporal stores.
//
// Only what csrc/plf_kernels.hip launches lives here:
//   plf_prot_lds_kernel     exact mode (plf()'s separate multiply and add), f64
//                           and f32: matrices as LDS broadcasts, row groups
//   plf_prot_mfma_kernel    FMA mode, f64, on the matrix cores
//   plf_prot_mfma32_kernel  FMA mode, f32, on the matrix cores
// each as a device body with a one-node kernel and a batched-nodes kernel
// (*_batch_kernel: node = blockIdx.y, plf_dna.hpp NodeBatch).
// The measured-and-not-adopted forms and knobs (the round-1 readlane kernel,
// ablations, swizzles, rings, SGPR operands, ...) live in the tuning copy
// tools/plf_prot_tune.hpp@f9b3af3; HISTORY.md section 3.3 has the measurements.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

#include "plf_dna.hpp"

namespace plfx {
namespace dev {

template <typename T, bool kFma>
__device__ __forceinline__ T madd(T a, T b, T c) {
  if constexpr (kFma) return __builtin_fma(a, b, c);
  else return c + a * b;
}
template <>
__device__ __forceinline__ float madd<float, true>(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}

// One 64-site tile of one child through LDS: the block's 256 threads load the
// tile's 64 x 80 values with coalesced 16-B (non-temporal) loads and store them
// at chunk (site*41 + chunk) -- one pad chunk per site makes every lane's
// ds_read_b128 of its own (site, category) row bank-conflict-free.
template <typename T>
struct ProtTile {
  static constexpr int kChunksPerSite = 80 * (int)sizeof(T) / 16;  // 40 (f64) / 20 (f32)
  static constexpr int kStride = kChunksPerSite + 1;
  static constexpr int kChunks = 64 * kChunksPerSite;
  typedef typename std::conditional<sizeof(T) == 8, f64x2, f32x4>::type V;
};

// fetch: all K 16-B loads of a thread in flight at once (a load->wait->write
// chain per chunk would serialise K HBM round trips per tile); put: into the
// padded LDS layout.  Split so a kernel can keep a fetch in flight across work.
template <typename T>
__device__ __forceinline__ void tile_fetch(const T *__restrict__ g, int64_t base, int64_t n,
                                           typename ProtTile<T>::V (&v)[ProtTile<T>::kChunks / kBlock]) {
  using PT = ProtTile<T>;
  constexpr int K = PT::kChunks / kBlock;
  const typename PT::V *src = reinterpret_cast<const typename PT::V *>(g + base * 80);
  if (base + 64 <= n) {
#pragma unroll
    for (int i = 0; i < K; i++) v[i] = __builtin_nontemporal_load(src + threadIdx.x + i * kBlock);
  } else {
    const int64_t lim = (n - base) * PT::kChunksPerSite;  // chunks of valid sites
#pragma unroll
    for (int i = 0; i < K; i++) {
      const int j = threadIdx.x + i * kBlock;
      v[i] = typename PT::V{};
      if (j < lim) v[i] = __builtin_nontemporal_load(src + j);
    }
  }
}

template <typename T>
__device__ __forceinline__ void tile_put(typename ProtTile<T>::V *lds,
                                         const typename ProtTile<T>::V (&v)[ProtTile<T>::kChunks / kBlock]) {
  using PT = ProtTile<T>;
#pragma unroll
  for (int i = 0; i < PT::kChunks / kBlock; i++) {
    const int j = threadIdx.x + i * kBlock;
    const int s = j / PT::kChunksPerSite, q = j - s * PT::kChunksPerSite;
    lds[s * PT::kStride + q] = v[i];
  }
}

template <typename T>
__device__ __forceinline__ void tile_load(const T *__restrict__ g, int64_t base, int64_t n,
                                          typename ProtTile<T>::V *lds) {
  typename ProtTile<T>::V v[ProtTile<T>::kChunks / kBlock];
  tile_fetch<T>(g, base, n, v);
  tile_put<T>(lds, v);
}

template <typename T>
__device__ __forceinline__ void tile_store(T *__restrict__ g, int64_t base, int64_t n,
                                           const typename ProtTile<T>::V *lds) {
  using PT = ProtTile<T>;
  constexpr int K = PT::kChunks / kBlock;
  typename PT::V *dst = reinterpret_cast<typename PT::V *>(g + base * 80);
  typename PT::V v[K];
#pragma unroll
  for (int i = 0; i < K; i++) {
    const int j = threadIdx.x + i * kBlock;
    const int s = j / PT::kChunksPerSite, q = j - s * PT::kChunksPerSite;
    v[i] = lds[s * PT::kStride + q];
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

// this lane's (site, category) row of 20 values <-> the LDS tile
template <typename T>
__device__ __forceinline__ void row_read(const typename ProtTile<T>::V *lds, int site, int c,
                                         T (&v)[20]) {
  using PT = ProtTile<T>;
  const typename PT::V *r = lds + site * PT::kStride + c * (PT::kChunksPerSite / 4);
  if constexpr (sizeof(T) == 8) {
#pragma unroll
    for (int i = 0; i < 10; i++) { const f64x2 t = r[i]; v[2 * i] = t.x; v[2 * i + 1] = t.y; }
  } else {
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const f32x4 t = r[i];
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  }
}

template <typename T>
__device__ __forceinline__ void row_write(typename ProtTile<T>::V *lds, int site, int c,
                                          const T (&v)[20]) {
  using PT = ProtTile<T>;
  typename PT::V *r = lds + site * PT::kStride + c * (PT::kChunksPerSite / 4);
  if constexpr (sizeof(T) == 8) {
#pragma unroll
    for (int i = 0; i < 10; i++) r[i] = f64x2{v[2 * i], v[2 * i + 1]};
  } else {
#pragma unroll
    for (int i = 0; i < 5; i++) r[i] = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
  }
}

// ---------------------------------------------------------------------------
// Protein tips (extension of SURVEY section 8f row 4 to S = 20): a leaf is one
// uint8 code per site, index into a table of kProtCodes dense rows of 20 values
// (tipvec, codes x 20, device, dtype of the CLVs), codes >= kProtCodes read row
// kProtCodes-1.  Default table (tipvec == NULL), states in ARNDCQEGHILKMFPSTWYV
// order: codes 0..19 one state, 20 = B (N|D), 21 = Z (Q|E), 22 = X / unknown,
// 23 = gap (all states).  A tip child's ump[c][k] = sum_l tv[code][l] * P_c[k][l]
// (ascending l from +0.0, the kernel's multiply-add) comes from a per-block LDS
// table built with exactly plf()'s operations on the expanded row, so results
// are bit-identical to plf() on the dense CLV x[i][c][s] = tv[code_i][s].
constexpr int kProtCodes = 24;

template <typename T>
__device__ __forceinline__ T prot_tip_value(const T *tipvec, int code, int l) {
  if (tipvec) return tipvec[code * 20 + l];
  if (code < 20) return l == code ? T(1) : T(0);
  if (code == 20) return (l == 2 || l == 3) ? T(1) : T(0);  // B = N | D
  if (code == 21) return (l == 5 || l == 6) ? T(1) : T(0);  // Z = Q | E
  return T(1);                                               // X, gap
}

__device__ __forceinline__ int prot_code(uint8_t v) { return v < kProtCodes ? v : kProtCodes - 1; }

// tab[c * kProtCodes * 20 + code * 20 + k] for the 4 categories of P (C x 400)
template <typename T, bool kFma>
__device__ void build_prot_tip_table(const T *__restrict__ P, const T *__restrict__ tipvec,
                                     T *tab) {
  for (int e = threadIdx.x; e < 4 * kProtCodes * 20; e += kBlock) {
    const int c = e / (kProtCodes * 20), r = e % (kProtCodes * 20), code = r / 20, k = r % 20;
    T u = T(0);
#pragma unroll 4
    for (int l = 0; l < 20; l++) u = madd<T, kFma>(prot_tip_value<T>(tipvec, code, l), P[c * 400 + k * 20 + l], u);
    tab[e] = u;
  }
}


// An empty asm that takes and returns every chain value: the compiler can no
// longer finish one independent chain before starting the next (it did, and
// held all the chains' operands in registers -- 256 VGPRs and spills).
template <typename T, int R>
__device__ __forceinline__ void pin_chains(T (&u)[R]) {
  if constexpr (R == 2) {
    asm volatile("" : "+v"(u[0]), "+v"(u[1]));
  } else if constexpr (R == 4) {
    asm volatile("" : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]));
  } else if constexpr (R == 10) {
    asm volatile("" : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]),
                 "+v"(u[6]), "+v"(u[7]), "+v"(u[8]), "+v"(u[9]));
  } else {
#pragma unroll
    for (int j = 0; j < R; j++) asm volatile("" : "+v"(u[j]));
  }
}

// A child tile gathered from its combination table by code pair (kTab in the bodies below):
// chunk j of the tile is site j / 40's row chunk j % 40, as tile_fetch.
template <typename T>
__device__ __forceinline__ void tab_fetch(const T *__restrict__ x, const uint8_t *__restrict__ ca,
                                          const uint8_t *__restrict__ cb, int64_t b, int64_t n,
                                          typename ProtTile<T>::V (&pf)[ProtTile<T>::kChunks / kBlock]) {
  using PT = ProtTile<T>;
  using V = typename PT::V;
  const V *tab = reinterpret_cast<const V *>(x);
  // lane l reads site l's two codes (one byte load per array for the whole
  // tile), each chunk takes its site's code pair from that lane (the kernel
  // runs at its 256-VGPR bound: per-chunk code loads spilled)
  const int lane = threadIdx.x & 63;
  const int lim = (int)(n - b < 64 ? n - b : 64);
  const int ls = lane < lim ? lane : lim - 1;
  const int mine = prot_code(ca[b + ls]) * kProtCodes + prot_code(cb[b + ls]);
#pragma unroll
  for (int i = 0; i < PT::kChunks / kBlock; i++) {
    const int j = threadIdx.x + i * kBlock;
    const int sl = j / PT::kChunksPerSite, q = j - sl * PT::kChunksPerSite;
    const int combo = __shfl(mine, sl < lim ? sl : lim - 1);
    pf[i] = sl < lim ? tab[(unsigned)(combo * PT::kChunksPerSite + q)] : V{};
  }
}

// The LDS-matrix protein kernel (exact mode, f64 and f32): the matrices live
// in LDS (P_L and P_R of the 4 categories and EV; 28.8 KB f64) and every value
// is a wave-uniform ds_read_b128 broadcast, where a register-distributed form
// pays v_readlane per value on the VALU, the binding unit.  Lane = site, wave
// = category; per 64-site tile, each with plf()'s order:
//   1: U[k]  = sum_l x1[l] * P_L[k][l]        2: U[k] *= sum_l x2[l] * P_R[k][l]
//   3: O[l]  = sum_k U[k] * EV[k][l]
// Phases 1 and 2 run kRows rows k at a time, streaming the group's columns l
// (P_L / P_R sit in LDS group-transposed: [category][group][l][kRows]), so a
// wave carries kRows independent chains; phase 3 streams EV rows in pieces of
// kPh3 states (kPh3 chains).  A single chain waits the f64 add's ~22-cycle
// dependent latency after every add (tools/probes/valu_f64.hip), which at two
// waves per SIMD held the round-1 row form (one chain per row k) to ~40 % of
// the VALU issue rate.  Each chain keeps plf()'s order (ascending l from the
// first product; x3 from +0.0), so the results are bit-identical to it.  The
// column reads run kDist steps ahead of their use (a register ring; an empty
// asm on a token from the previous step pins the distance, and an opaque
// per-trip offset keeps the reads inside the site loop).  Each dense child
// tile is fetched into registers while the previous phase computes: x2 during
// phase 1, the next trip's first dense child during phases 2 and 3.
// kE3S: phase 3's EV rows by scalar loads (SGPR operands) instead of LDS
// broadcasts: 145.8 vs 148.8 us at 2^18 f64 (profiles/r02_tune_protein_exact_rows.log).
// kTab: as prot_mfma_body's (children staged from their combination tables).
template <typename T, bool kSum, int kTips, int kRows, bool kE3S, bool kTab = false>
__device__ __forceinline__ void prot_lds_body(const T *__restrict__ x1, const T *__restrict__ x2,
                                              T *__restrict__ x3, const T *__restrict__ EV,
                                              const T *__restrict__ left, const T *__restrict__ right,
                                              const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                              int64_t n, unsigned long long *ws, int64_t *scaler_sum,
                                              const T *__restrict__ tipvec,
                                              const uint8_t *__restrict__ t1a = nullptr,
                                              const uint8_t *__restrict__ t1b = nullptr,
                                              const uint8_t *__restrict__ t2a = nullptr,
                                              const uint8_t *__restrict__ t2b = nullptr) {
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
        __builtin_amdgcn_sched_barrier(0);  // column l+kDist is read after column l-1 is used
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
  if constexpr (kTab) {
    if ((int64_t)blockIdx.x * 64 < n) tab_fetch<T>(x1, t1a, t1b, (int64_t)blockIdx.x * 64, n, pf);
  } else if constexpr (kAnyDense) {
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<T>(FD, (int64_t)blockIdx.x * 64, n, pf);
  }
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const V *mL = mats + off + c * (S * S / E), *mR = mats + off + (oR + c * S * S) / E,
            *mE = mats + off + oE / E;
    T U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    // the site weight up front, unconditionally (wgt_at, plf_dna.hpp): loaded
    // inside the scaled-site branch, its wait also drained the next child tile
    // in flight (2^18: f64 142.2 -> 138.9 us, f32 76.5 -> 74.6 us; the FMA
    // kernels ran 1-2 % slower this way and keep the branch load,
    // tools/tune_prot_wgt.hip@f9b3af3, profiles/r03_tune_protein_wgt.log)
    const int wsite = kSum ? wgt_at(wgt, sq, ws) : 0;
    // stage a dense child's tile from the prefetch registers, then fetch the
    // next tile in the sequence
    auto stage = [&](const T *next, int64_t nbase) {
      tile_put<T>(tile, pf);
      __syncthreads();
      if constexpr (kTab) {
        const bool one = next == x1;
        if (nbase < n) tab_fetch<T>(next, one ? t1a : t2a, one ? t1b : t2b, nbase, n, pf);
      } else {
        if (nbase < n) tile_fetch<T>(next, nbase, n, pf);
      }
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
    // x 2^32 on a scaled site as one v_ldexp by 32 or 0 per value (exact
    // either way: the same bits as the multiply-and-select, one VALU
    // instruction per value instead of three)
    int e = sc ? 32 : 0;
    asm volatile("" : "+v"(e));  // else LLVM turns it back into ldexp(O, 32) + select
#pragma unroll
    for (int l = 0; l < S; l++) {
      if constexpr (sizeof(T) == 8) O[l] = ldexp(O[l], e);
      else O[l] = ldexpf(O[l], e);
    }
    row_write<T>(tile, lane, c, O);
    const int64_t site = base + lane;
    if (site < n && c == 0) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wsite;
    }
    __syncthreads();
    tile_store<T>(x3, base, n, tile);
    __syncthreads();  // tile and small_mask are reused by the next trip
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

template <typename T, bool kSum, int kMinWaves, int kTips, int kRows, bool kE3S>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_lds_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
                    const T *__restrict__ EV, const T *__restrict__ left, const T *__restrict__ right,
                    const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                    unsigned long long *ws, int64_t *scaler_sum, const T *__restrict__ tipvec = nullptr) {
  prot_lds_body<T, kSum, kTips, kRows, kE3S>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws,
                                              scaler_sum, tipvec);
}

template <typename T, bool kSum, int kMinWaves, int kTips, int kRows, bool kE3S>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_lds_batch_kernel(const NodeBatch nodes, const T *__restrict__ EV, const int32_t *__restrict__ wgt,
                          int64_t n, unsigned long long *ws, const T *__restrict__ tipvec) {
  const NodeDesc &d = nodes.d[blockIdx.y];
  prot_lds_body<T, kSum, kTips, kRows, kE3S>((const T *)d.x1, (const T *)d.x2, (T *)d.x3, EV,
                                             (const T *)d.left, (const T *)d.right, wgt, d.scaler, n,
                                             ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, tipvec);
}

// ---------------------------------------------------------------------------
// FMA mode on the matrix cores (f64).  v_mfma_f64_16x16x4_f64 is bit-for-bit a
// k-ordered fma chain (probed on MI355X: tools/probes/mfma_f64_numerics.hip),
// so this kernel reproduces plf()'s loop with every multiply-add fused, in the
// same order -- identical to the oracle's fma() restatement.  Per category
// (wave) and 16-site sub-tile:
//   U^T[k][site]   = P[k][l]  . X^T[l][site]   (M = k: 2 tiles, N = 16 sites,
//                                               K = l: 5 steps of 4)
//   p              = U_L^T * U_R^T             (accumulator registers, VALU)
//   X3^T[l][site]  = EV^T[l][k] . p[k][site]   (the accumulators of the first
//                                               product ARE the B fragments:
//                                               k-step s = tile s>>2, reg s&3)
// A fragments (P rows, EV columns) stay in VGPRs for the whole kernel; B
// fragments (X^T) come from the LDS tile, conflict-free.
// Rows 16..19 of each product (M = 20 = 16 + 4) run on v_mfma_f64_4x4x4_4b_f64
// -- four 4x4x4 blocks = the 16 sites, 20 cycles -- instead of a zero-padded
// second 16x16x4 tile (64 cycles): 420 instead of 640 matrix-core cycles per
// product and sub-tile.  Its operand maps make the two forms interchangeable
// (A lane 16k+4b+i, B lane 16k+4b+j, D lane 16i+4b+j: the B fragment is the
// same LDS value, and D lands as row 16 + lane/16 of site lane%16 -- exactly
// the k-step-4 B fragment of the back-transform), and it too is bit-for-bit a
// k-ordered fma chain (tools/probes/mfma_f64_4x4x4_numerics.hip).
// X3 reaches the LDS tile through permuted back-transform rows: A row i of the
// first tile computes state 4(i%4) + i/4, so a lane's four 16x16x4 results are
// four consecutive states of its site -- 2 conflict-free ds_write_b128 + 1
// ds_write_b64, no lane movement (a row permutation of the A operand permutes
// the outputs, nothing else; 90.2 vs 91.2 us at 2^18, profiles/r02_tune_protein_v3.log).
// The next child tile's loads are in flight while the current one is
// multiplied (x2 during phase 1, the next trip's first dense child during
// phase 2); the first tile's loads go out before the matrix fragments'.
typedef double f64x4 __attribute__((ext_vector_type(4)));

// Device-wide tile queue for the protein kernels (kDyn).  Why: with two or
// three co-resident blocks per CU the oldest block's waves win the SIMD's issue
// arbitration -- at 2^18 sites the first block on each CU finished its 8 fixed
// trips at ~75 us, the second at ~83 us (tools/probes/prot_timeline.hip@f9b3af3) -- so
// a fixed grid stride leaves CUs half idle at the end, more so the more trips a
// block makes.  Tiles: trip 0 takes blockIdx.x, trip 1 G + blockIdx.x, trip
// i >= 2 2G + d, d from a returning atomic add on a head word that thread 0
// issues in the middle of trip i - 2 (right after the wave's next-tile loads,
// so no wait lands on it before the next trip's start) and publishes in LDS at
// the start of trip i - 1 (its only use: any use makes the wave wait for the
// atomic there).  The head address carries an offset laundered through an
// empty asm (a VGPR 0), so the compiler's atomic optimizer (a uniform address
// makes it aggregate lanes and read the result at once) leaves the single-lane
// add alone, and the address stays global (a laundered pointer turns it into
// a flat atomic, which every LDS wait would then wait for).  Words: the stream
// workspace's second region (ws + kWsWords; the protein launches use only the
// first): [0] head, [16] exit count.  The last block out zeroes both for the
// next launch; a block's last dequeue has returned before its exit add (the
// add depends on the returned value).  Every dequeued tile index is consumed
// in order, and one past the end ends the block, so no tile is lost.
struct ProtQueue {
  unsigned long long *head, *done;
  int64_t G, ntiles;
  long long pend = 0;  // thread 0: the dequeued value for the tile of trip i + 2
  bool dyn;
  __device__ ProtQueue(unsigned long long *ws, int64_t n, bool on) {
    int zero = 0;  // a divergent-looking 0: the address stays global, not uniform
    if (on) asm volatile("" : "+v"(zero));
    head = ws + kWsWords + zero;
    done = ws + kWsWords + 16;
    G = gridDim.x;
    ntiles = (n + 63) / 64;
    dyn = ntiles > 2 * G;
  }
  __device__ __forceinline__ void dequeue() {
    if (dyn && threadIdx.x == 0)
      pend = (long long)__hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // thread 0: the base of trip i + 1 (n * 64 sentinel clipped by the caller's loop)
  __device__ __forceinline__ int64_t next_base(int i) const {
    int64_t t = ntiles;
    if (i == 0) t = G + blockIdx.x;
    else if (dyn) t = 2 * G + pend;
    return (t < ntiles ? t : ntiles) * 64;
  }
  __device__ __forceinline__ void finish() const {
    if (threadIdx.x != 0) return;
    const unsigned long long after = (unsigned long long)(pend >> 62);  // 0, once it returned
    const unsigned long long d = __hip_atomic_fetch_add(done, 1ull + after, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned long long)G - 1) {
      __hip_atomic_store(head, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
};

// kTab: both children are tip/tip nodes of the same traversal whose values
// sit in their combination tables (prot_tiptip_gather_kernel below): x1 / x2
// point at the two tables (576 code pairs x 80), t1a/t1b and t2a/t2b at each
// child's two tip-code arrays, and a child tile is gathered from its table by
// code pair (L2-resident, 368 KB) instead of read back from HBM.  The values
// are the ones the gather wrote to the children's CLVs, so results are
// bit-identical.
template <bool kSum, int kTips, bool kDyn, bool kTab = false>
__device__ __forceinline__ void prot_mfma_body(const double *__restrict__ x1, const double *__restrict__ x2,
                                               double *__restrict__ x3, const double *__restrict__ EV,
                                               const double *__restrict__ left, const double *__restrict__ right,
                                               const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                               int64_t n, unsigned long long *ws, int64_t *scaler_sum,
                                               const double *__restrict__ tipvec,
                                               const uint8_t *__restrict__ t1a = nullptr,
                                               const uint8_t *__restrict__ t1b = nullptr,
                                               const uint8_t *__restrict__ t2a = nullptr,
                                               const uint8_t *__restrict__ t2b = nullptr) {
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
  if constexpr (!T2) {  // the first dense child's first tile, before the matrix fragments
    if constexpr (kTab) {
      if ((int64_t)blockIdx.x * 64 < n) tab_fetch<double>(x1, t1a, t1b, (int64_t)blockIdx.x * 64, n, pf);
    } else {
      if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
    }
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
  ProtQueue pq(ws, n, kDyn);
  __shared__ long long qslot;
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
  auto trip = [&](const int64_t base) -> int64_t {
    int64_t next = base + stride;  // kDyn: read from qslot after the trip's first barrier
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
      if constexpr (kDyn) next = qslot;
      if constexpr (kTab) tab_fetch<double>(x2, t2a, t2b, base, n, pf);
      else tile_fetch<double>(x2, base, n, pf);
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
      if constexpr (kDyn) {
        next = qslot;  // published before the trip's extra barrier
        pq.dequeue();
      }
    } else {
      tile_put<double>(tile, pf);
      __syncthreads();
      if constexpr (kDyn && T1) next = qslot;
      // next trip's first dense child: x1, or x2 when x1 is a tip
      if constexpr (kTab) {
        if (next < n) tab_fetch<double>(x1, t1a, t1b, next, n, pf);
      } else {
        if (next < n) tile_fetch<double>(T1 ? x2 : x1, next, n, pf);
      }
      if constexpr (kDyn) pq.dequeue();
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
  if constexpr (kDyn) {
    int64_t base = (int64_t)blockIdx.x * 64;
    for (int i = 0; base < n; i++) {
      if (threadIdx.x == 0) qslot = pq.next_base(i);
      if constexpr (T1 && T2) __syncthreads();
      base = trip(base);
    }
    pq.finish();
  } else {
    int64_t base = (int64_t)blockIdx.x * 64;
    for (; base < n; base += stride) trip(base);
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

// One node per launch (the grid strides over its sites)
template <bool kSum, int kMinWaves, int kTips, bool kDyn = false>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum,
                     const double *__restrict__ tipvec = nullptr) {
  prot_mfma_body<kSum, kTips, kDyn>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum, tipvec);
}

// Batched protein nodes (a tree level, a shard of independent nodes): node =
// blockIdx.y, descriptors by value as the DNA batches (plf_dna.hpp NodeBatch),
// each node with its own kWsWords of scaler-sum workspace; the fixed grid stride
// (no tile queue: its words would overlap the next node's sum region).
template <bool kSum, int kMinWaves, int kTips>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_batch_kernel(const NodeBatch nodes, const double *__restrict__ EV,
                           const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                           const double *__restrict__ tipvec) {
  const NodeDesc &d = nodes.d[blockIdx.y];
  prot_mfma_body<kSum, kTips, false>((const double *)d.x1, (const double *)d.x2, (double *)d.x3, EV,
                                     (const double *)d.left, (const double *)d.right, wgt, d.scaler, n,
                                     ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, tipvec);
}

// Batched protein nodes whose children are both tip/tip nodes held in
// combination tables (kTab above): the parents of a coded tree's first level.
// One kernel per mode and dtype: f64 FMA (matrix cores, below), exact f64 and
// f32 (the LDS-matrix body), f32 FMA (matrix cores) -- the traversal uses the
// tables in every mode (plfx_api.hip tab_mode).
struct ProtTabDesc {
  const void *tab1, *tab2;               // the children's tables (576 x 80 f64)
  const uint8_t *c1a, *c1b, *c2a, *c2b;  // each child's two tip-code arrays
  void *x3;
  const void *left, *right;
  uint8_t *scaler;
  int64_t *scaler_sum;
};
struct ProtTabBatch {
  ProtTabDesc d[kMaxBatch];
};

template <bool kSum>
__global__ void __launch_bounds__(kBlock, 2)
plf_prot_mfma_tab_batch_kernel(const ProtTabBatch b, const double *__restrict__ EV,
                               const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws) {
  const ProtTabDesc &d = b.d[blockIdx.y];
  prot_mfma_body<kSum, 0, false, true>((const double *)d.tab1, (const double *)d.tab2, (double *)d.x3, EV,
                                       (const double *)d.left, (const double *)d.right, wgt, d.scaler, n,
                                       ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, nullptr, d.c1a,
                                       d.c1b, d.c2a, d.c2b);
}

// exact mode (the LDS-matrix body), f64 and f32
template <typename T, bool kSum, int kRows, bool kE3S>
__global__ void __launch_bounds__(kBlock, 2)
plf_prot_lds_tab_batch_kernel(const ProtTabBatch b, const T *__restrict__ EV, const int32_t *__restrict__ wgt,
                              int64_t n, unsigned long long *ws) {
  const ProtTabDesc &d = b.d[blockIdx.y];
  prot_lds_body<T, kSum, 0, kRows, kE3S, true>((const T *)d.tab1, (const T *)d.tab2, (T *)d.x3, EV,
                                               (const T *)d.left, (const T *)d.right, wgt, d.scaler, n,
                                               ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, nullptr,
                                               d.c1a, d.c1b, d.c2a, d.c2b);
}

template <bool kSum>
__global__ void __launch_bounds__(kBlock, 3)
plf_prot_mfma32_tab_batch_kernel(const ProtTabBatch b, const float *__restrict__ EV,
                                 const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws);


// ---------------------------------------------------------------------------
// FMA mode on the matrix cores, f32: v_mfma_f32_16x16x4_f32 is exact f32, a
// k-ordered fmaf chain bit for bit (MI355X_MICROARCH.md, FP32-input MFMA), so
// this kernel is bit-identical to the oracle's fused restatement.  The f64
// kernel's scheme with the f32 operand maps (A: lane l = A[row l&15][k l>>4],
// B: lane l = B[k l>>4][col l&15], C/D: lane l reg r = D[row 4(l>>4) + r][col
// l&15] -- rows by 4 per lane group, where f64 interleaves them):
//   U^T[k][site] = P[k][l] . X^T[l][site]: A row i computes
//     k = pi(i) = 4 (i&3) + (i>>2), so lane group g, reg r holds k = 4 r + g --
//     exactly the B fragment of k-step r of the back-transform (lane group g =
//     k 4s + g);
//   X3^T[l][site] = EV^T[l][k] . p[k][site]: natural rows, so lane group g
//     holds states 4g..4g+3 of its site: one 16-B LDS write, no lane movement.
// Rows 16..19 of both child products and of the back-transform run on
// v_mfma_f32_4x4x1_16b_f32 (f32 has no 4x4x4 form).  Its maps (probed on the
// MI355X, tools/probes/mfma_f32_4x4x1.hip: block b = lane/4, A lane l =
// A_b[l%4][0], B lane l = B_b[0][l%4], D lane l reg r = D_b[r][l%4]; 20
// chained K = 1 steps are bit for bit a k-ordered fmaf chain) give, with A =
// P[16 + l%4][col] and B = x[site l][col], lane l = the trip's site l holding
// U[16..19] of its own site after 20 steps (14 cycles each) for all 64 sites
// at once -- 280 cycles per product and trip instead of 640 for padded 16x16x4
// tiles.  One 4x4 transpose of (lane group x register) by v_permlane32_swap +
// v_permlane16_swap then hands lane group g the k = 16 + g row of every
// sub-tile, the back-transform's B fragment of k-step 4; the back-transform's
// states 16..19 run the same way (B = p[k][site l] for all 20 k: rows 0..15
// brought to lane l by four more transposes), so a lane writes states 16..19
// of its site as one 16-B row (52.4 -> 46.5 us at 2^18,
// profiles/r02_tune_protein_f32_q.log).
// 4x4 transpose of (lane group g = lane >> 4) x (register r) on 32-bit values:
// afterwards v[r] of group g holds what v[g] of group r held.  (Unsigned
// values; convert with __float_as_uint / __uint_as_float: __builtin_bit_cast of
// a vector element, e.g. a builtin's pair result p[1], reads element 0 with
// this compiler.)
__device__ __forceinline__ void transpose_groups44(unsigned (&v)[4]) {
#pragma unroll
  for (int r = 0; r < 2; r++) {  // off-diagonal 2x2 blocks: groups 2,3 of v[r] <-> groups 0,1 of v[r+2]
    const auto p = __builtin_amdgcn_permlane32_swap(v[r], v[r + 2], false, false);
    v[r] = p[0];
    v[r + 2] = p[1];
  }
#pragma unroll
  for (int r = 0; r < 4; r += 2) {  // inside each block: odd groups of v[r] <-> even groups of v[r+1]
    const auto p = __builtin_amdgcn_permlane16_swap(v[r], v[r + 1], false, false);
    v[r] = p[0];
    v[r + 1] = p[1];
  }
}

// kTab: as prot_mfma_body's (children staged from their combination tables).
template <bool kSum, int kTips, bool kTab = false>
__device__ __forceinline__ void prot_mfma32_body(const float *__restrict__ x1, const float *__restrict__ x2,
                                                 float *__restrict__ x3, const float *__restrict__ EV,
                                                 const float *__restrict__ left, const float *__restrict__ right,
                                                 const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                                 int64_t n, unsigned long long *ws, int64_t *scaler_sum,
                                                 const float *__restrict__ tipvec,
                                                 const uint8_t *__restrict__ t1a = nullptr,
                                                 const uint8_t *__restrict__ t1b = nullptr,
                                                 const uint8_t *__restrict__ t2a = nullptr,
                                                 const uint8_t *__restrict__ t2b = nullptr) {
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
  if constexpr (!(T1 && T2)) {
    if constexpr (kTab) {
      if ((int64_t)blockIdx.x * 64 < n) tab_fetch<float>(x1, t1a, t1b, (int64_t)blockIdx.x * 64, n, pf);
    } else {
      if ((int64_t)blockIdx.x * 64 < n) tile_fetch<float>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
    }
  }
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
        if constexpr (kTab) tab_fetch<float>(x2, t2a, t2b, base, n, pf);
        else tile_fetch<float>(x2, base, n, pf);
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
      if constexpr (kTab) {
        if (base + stride < n) tab_fetch<float>(x1, t1a, t1b, base + stride, n, pf);
      } else {
        if (base + stride < n) tile_fetch<float>(T1 ? x2 : x1, base + stride, n, pf);
      }
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

template <bool kSum, int kMinWaves, int kTips>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma32_kernel(const float *__restrict__ x1, const float *__restrict__ x2,
                       float *__restrict__ x3, const float *__restrict__ EV,
                       const float *__restrict__ left, const float *__restrict__ right,
                       const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                       unsigned long long *ws, int64_t *scaler_sum,
                       const float *__restrict__ tipvec = nullptr) {
  prot_mfma32_body<kSum, kTips>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum, tipvec);
}

template <bool kSum, int kMinWaves, int kTips>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma32_batch_kernel(const NodeBatch nodes, const float *__restrict__ EV,
                             const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                             const float *__restrict__ tipvec) {
  const NodeDesc &d = nodes.d[blockIdx.y];
  prot_mfma32_body<kSum, kTips>((const float *)d.x1, (const float *)d.x2, (float *)d.x3, EV,
                                (const float *)d.left, (const float *)d.right, wgt, d.scaler, n,
                                ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, tipvec);
}

template <bool kSum>
__global__ void __launch_bounds__(kBlock, 3)
plf_prot_mfma32_tab_batch_kernel(const ProtTabBatch b, const float *__restrict__ EV,
                                 const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws) {
  const ProtTabDesc &d = b.d[blockIdx.y];
  prot_mfma32_body<kSum, 0, true>((const float *)d.tab1, (const float *)d.tab2, (float *)d.x3, EV,
                                  (const float *)d.left, (const float *)d.right, wgt, d.scaler, n,
                                  ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, nullptr, d.c1a, d.c1b,
                                  d.c2a, d.c2b);
}

// ---------------------------------------------------------------------------
// Tip/tip protein nodes by combination tables.  A node whose children are both
// coded tips has at most kProtCodes^2 = 576 distinct sites: its x3 row and
// scaler byte depend only on (code1, code2) and the node's matrices.  The
// library evaluates the 576 combinations with the node's own kernel (a batched
// launch over a constant 576-"site" alignment: combo k = code1 * 24 + code2,
// so every table row is bit for bit what that kernel computes for such a
// site), then this kernel writes the node: x3[i] = T[combo(i)], scaler[i] =
// S[combo(i)], scaler_sum = sum_i wgt_i * S[combo(i)] -- a write stream with
// the tables read from L2, where the direct tip/tip kernel is bound by its
// compute path (77 us f64 / 95 us f32 per 2^18 sites, no HBM reads at all).
// node = blockIdx.y; each block copies 64-site tiles with coalesced 16-B
// non-temporal stores (the protein kernels' tile order).
struct ProtGatherDesc {
  const uint8_t *c1, *c2;  // the children's codes
  void *x3;
  uint8_t *scaler;         // may be null
  int64_t *scaler_sum;     // may be null
  const void *tab;         // 576 x 80 values of the node's dtype
  const uint8_t *tsc;      // 576 scaler bytes
};
struct ProtGatherBatch {
  ProtGatherDesc d[kMaxBatch];
};
constexpr int kProtCombos = kProtCodes * kProtCodes;

template <typename T, bool kSum>
__global__ void __launch_bounds__(kBlock)
prot_tiptip_gather_kernel(const ProtGatherBatch b, const int32_t *__restrict__ wgt, int64_t n,
                          unsigned long long *ws) {
  using PT = ProtTile<T>;
  using V = typename PT::V;
  constexpr int K = PT::kChunks / kBlock;
  const ProtGatherDesc &d = b.d[blockIdx.y];
  const V *tab = static_cast<const V *>(d.tab);
  V *x3 = static_cast<V *>(d.x3);
  long long acc = 0;
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
    V v[K];
#pragma unroll
    for (int i = 0; i < K; i++) {  // all table loads first
      const int j = threadIdx.x + i * kBlock;
      const int sl = j / PT::kChunksPerSite, q = j - sl * PT::kChunksPerSite;
      const int64_t site = base + sl < n ? base + sl : n - 1;
      const int combo = prot_code(d.c1[site]) * kProtCodes + prot_code(d.c2[site]);
      v[i] = tab[(int64_t)combo * PT::kChunksPerSite + q];
    }
    if (base + 64 <= n) {
#pragma unroll
      for (int i = 0; i < K; i++) __builtin_nontemporal_store(v[i], x3 + base * PT::kChunksPerSite + threadIdx.x + i * kBlock);
    } else {
      const int64_t lim = (n - base) * PT::kChunksPerSite;
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        if (j < lim) __builtin_nontemporal_store(v[i], x3 + base * PT::kChunksPerSite + j);
      }
    }
    if (threadIdx.x < 64) {
      const int64_t site = base + threadIdx.x;
      if (site < n) {
        const uint8_t sc = d.tsc[prot_code(d.c1[site]) * kProtCodes + prot_code(d.c2[site])];
        if (d.scaler) d.scaler[site] = sc;
        if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
    }
  }
  if constexpr (kSum) block_ticket_sum(acc, ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum);
}

}  // namespace dev
}  // namespace plfx
