// plf_prot_tune.hpp -- TUNING COPY (not product code): csrc/plf_prot.hpp as it
// stood at the end of round 2, with every measured-and-not-adopted kernel and
// knob (plf_prot_kernel, plf_prot_exact_f64_kernel, plf_prot_exact64_kernel,
// prot_group_transpose, kAblate, kSwz, kSpread, kRing, kSplitB, kPS, kPack,
// kX3 = 0/1/3, kFirstX2, kQ = 0/1) for the same-process A/B harnesses in
// tools/.  A harness includes this INSTEAD of csrc/plf_prot.hpp (same names,
// same namespace); its product-knob instantiations are the product kernels'
// code as of that commit.  The product header keeps only what
// csrc/plf_kernels.hip instantiates.
//
// plf_prot.hpp -- fused PLF inner-node update for S=20 states (protein) x C=4
// Gamma categories (extension: the reference hard-wires DNA, SURVEY F9 /
// BASELINE configs[4]).  Same loop as plf() (app/src/plf.cpp:19-65) with 4
// replaced by 20: ump[k] = sum_l x[c][l]*P_c[k][l] (ascending l from +0.0),
// prod[k] = umpL*umpR, x3[c][l] = sum_k prod[k]*EV[k][l] (ascending k from
// +0.0), site scaled iff all 80 |x3| < 2^-32.
//
// Mapping: a 256-thread block owns 64 consecutive sites; wave w = category c,
// lane = site.  Child tiles pass through LDS (coalesced global access, padded
// conflict-free rows; lane = site directly on HBM re-read every line 4x and
// thrashed L2).  The wave's category matrices P_L, P_R and EV (3 x 400 values)
// stay resident in VGPRs for the whole kernel, spread over the 64 lanes (value
// e lives in lane e%64 of register e/64: 7 registers per matrix), and every
// use broadcasts one value with v_readlane at a compile-time lane -- no memory
// latency in the inner loop.  (Measured alternatives, both at 14 % of the HBM
// roofline: s_load from the scalar cache, which cannot hold 4 x 9.6 KB, and
// LDS broadcasts, which move a full 1 KiB per ds_read_b128 and were each
// waited on immediately.)  Each
// lane keeps its 20 x1, 20 x2 and 20 running x3 values in VGPRs and streams
// over k, accumulating x3 in plf()'s k order.  The 80-value scale test of a
// site spans the 4 waves: each wave ballots its 20-value test, the 4 masks meet
// in LDS and are ANDed.  The four waves of a block read the same contiguous
// 64 x 640 B of each child, so HBM/L2 see whole lines.
//
// kFma=false: separate multiply and add in plf()'s order (bit-identical to the
// oracle's generic restatement); kFma=true: fused multiply-add (one rounding
// per term), half the VALU issue, within 1e-12 relative of it.
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

// Value e of a lane-distributed matrix (lane e%64 of register e/64), broadcast
// to the wave; e is a compile-time constant after unrolling.
template <typename T, int R>
__device__ __forceinline__ T bcast(const T (&M)[R], int e) {
  if constexpr (sizeof(T) == 8) {
    const long long v = __builtin_bit_cast(long long, M[e >> 6]);
    const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), e & 63);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), e & 63);
    return __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned int)lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, M[e >> 6]), e & 63));
  }
}

template <typename T>
__device__ __forceinline__ void load20(const T *__restrict__ p, T (&v)[20]) {
  if constexpr (sizeof(T) == 8) {
    const f64x2 *q = reinterpret_cast<const f64x2 *>(p);
#pragma unroll
    for (int i = 0; i < 10; i++) {
      const f64x2 t = __builtin_nontemporal_load(q + i);
      v[2 * i] = t.x;
      v[2 * i + 1] = t.y;
    }
  } else {
    const f32x4 *q = reinterpret_cast<const f32x4 *>(p);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const f32x4 t = __builtin_nontemporal_load(q + i);
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  }
}

template <typename T>
__device__ __forceinline__ void store20(T *__restrict__ p, const T (&v)[20]) {
  if constexpr (sizeof(T) == 8) {
    f64x2 *q = reinterpret_cast<f64x2 *>(p);
#pragma unroll
    for (int i = 0; i < 10; i++) {
      f64x2 t = {v[2 * i], v[2 * i + 1]};
      __builtin_nontemporal_store(t, q + i);
    }
  } else {
    f32x4 *q = reinterpret_cast<f32x4 *>(p);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      f32x4 t = {v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
      __builtin_nontemporal_store(t, q + i);
    }
  }
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

// kAblate (tuning only, tools/tune_plf.hip): 0 = the kernel; 1 = skip the
// arithmetic (o = a + b); 2 = skip the child-tile traffic (a, b synthesised).
// kTips: 1 = x1 is a tip (uint8 codes), 2 = both children are tips.
template <typename T, bool kFma, bool kSum, int kAblate = 0, int kMinWaves = 2, int kTips = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
                const T *__restrict__ EV, const T *__restrict__ left, const T *__restrict__ right,
                const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                unsigned long long *ws, int64_t *scaler_sum, const T *__restrict__ tipvec = nullptr) {
  constexpr int S = 20;
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  using PT = ProtTile<T>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform category
  const int lane = threadIdx.x & 63;
  __shared__ T tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<T, kFma>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<T, kFma>(right, tipvec, tabs[1]);
  if constexpr (T1) __syncthreads();
  const T *tabL = tabs[0] + c * kProtCodes * 20, *tabR = tabs[T2 ? 1 : 0] + c * kProtCodes * 20;
  constexpr int R = (S * S + 63) / 64;  // registers per lane-distributed matrix
  T ML[R], MR[R], ME[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int e = r * 64 + lane;
    ML[r] = e < S * S ? left[c * S * S + e] : T(0);
    MR[r] = e < S * S ? right[c * S * S + e] : T(0);
    ME[r] = e < S * S ? EV[e] : T(0);
  }
  const T m = Num<T>::minlik();
  __shared__ typename PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
    const int64_t site = base + lane;
    const bool valid = site < n;
    T a[S], b[S], o[S];
    const int64_t sq = valid ? site : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (kAblate == 2) {
#pragma unroll
      for (int l = 0; l < S; l++) { a[l] = T(site + l) * T(1e-3); b[l] = T(lane + l) * T(1e-3); }
    } else {
      if constexpr (!T1) {
        tile_load<T>(x1, base, n, tile);
        __syncthreads();
        row_read<T>(tile, lane, c, a);
        __syncthreads();
      }
      if constexpr (!T2) {
        tile_load<T>(x2, base, n, tile);
        __syncthreads();
        row_read<T>(tile, lane, c, b);
      }
    }
#pragma unroll
    for (int l = 0; l < S; l++) o[l] = kAblate == 1 ? a[l] + b[l] : T(0);
#pragma unroll
    for (int k = 0; k < (kAblate == 1 ? 0 : S); k++) {
      // ump chains start at q0 (fma(a, b, +0) and a*b differ only in the sign
      // of a zero, which the x3 chain from +0 absorbs: site_cat, plf_dna.hpp)
      T u1, u2;
      if constexpr (T1) u1 = tabL[code1 * 20 + k];
      else u1 = a[0] * bcast<T>(ML, k * S);
      if constexpr (T2) u2 = tabR[code2 * 20 + k];
      else u2 = b[0] * bcast<T>(MR, k * S);
#pragma unroll
      for (int l = 1; l < S; l++) {
        if constexpr (!T1) u1 = madd<T, kFma>(a[l], bcast<T>(ML, k * S + l), u1);
        if constexpr (!T2) u2 = madd<T, kFma>(b[l], bcast<T>(MR, k * S + l), u2);
      }
      const T p = u1 * u2;
#pragma unroll
      for (int l = 0; l < S; l++) o[l] = madd<T, kFma>(p, bcast<T>(ME, k * S + l), o[l]);
    }
    bool small = valid;
#pragma unroll
    for (int l = 0; l < S; l++) small = small && (Num<T>::abs(o[l]) < m);
    const unsigned long long mk = __ballot(small);
    if (lane == 0) small_mask[c] = mk;
    __syncthreads();  // also: every wave is done reading x2 from the tile
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    const bool sc = (all >> lane) & 1ull;
#pragma unroll
    for (int l = 0; l < S; l++) {
      const T sv = o[l] * Num<T>::two32();
      o[l] = sc ? sv : o[l];
    }
    row_write<T>(tile, lane, c, o);
    if (valid && c == 0) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
    }
    __syncthreads();
    if constexpr (kAblate != 2) tile_store<T>(x3, base, n, tile);
    __syncthreads();  // tile and small_mask are reused by the next trip
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

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

// The LDS-matrix protein kernel (f64 exact, f32 exact and f32 FMA): the
// matrices live in LDS (P_L and P_R of the 4 categories and EV; 28.8 KB f64)
// and every value is a wave-uniform ds_read_b128 broadcast, where the
// register-distributed form (plf_prot_kernel) pays v_readlane per value on
// the VALU, the binding unit.  Lane = site, wave = category; per 64-site tile,
// each with plf()'s order:
//   1: U[k]  = sum_l x1[l] * P_L[k][l]        2: U[k] *= sum_l x2[l] * P_R[k][l]
//   3: O[l]  = sum_k U[k] * EV[k][l]
// Phases 1 and 2 run kRows rows k at a time, streaming the group's columns l
// (P_L / P_R sit in LDS group-transposed: [category][group][l][kRows]), so a
// wave carries kRows independent chains; phase 3 streams EV rows in pieces of
// kPh3 states (kPh3 chains).  A single chain waits the f64 add's ~22-cycle
// dependent latency after every add (tools/probes/valu_f64.hip), which at two
// waves per SIMD held the round-1 row form (one chain per row k) to ~40 % of
// the VALU issue rate.  Each chain keeps plf()'s order (ascending l from the
// first product; x3 from +0.0), so the results are bit-identical to it (exact)
// or to its fused restatement (kFma: every multiply-add one fma).  The column
// reads run kDist steps ahead of their use (a register ring; an empty asm on a
// token from the previous step pins the distance, and an opaque per-trip
// offset keeps the reads inside the site loop).  kPf: each dense child tile is
// fetched into registers while the previous phase computes (the FMA kernel's
// schedule): x2 during phase 1, the next trip's first dense child during
// phases 2 and 3.
// kPS (tuning, exact mode, dense children): phase 1 (bit 0) / phase 2 (bit 1)
// reads its matrix as SGPR operands by scalar loads from a group-transposed
// global copy (pl_t / pr_t: [c][k / kRows][l][k % kRows], prot_group_transpose)
// instead of LDS broadcasts, one column ahead; a null copy keeps the LDS path.
// Bit-identical; within the run-to-run spread of the LDS form on two boxes
// (profiles/r02_tune_protein_exact_sgpr.log), so the product keeps the LDS form.
template <typename T, bool kFma, bool kSum, int kTips, int kRows, bool kPf, bool kPack,
          bool kE3S = false, int kPS = 0, bool kNoMats = false>
__device__ __forceinline__ void prot_lds_body(const T *__restrict__ x1, const T *__restrict__ x2,
                                              T *__restrict__ x3, const T *__restrict__ EV,
                                              const T *__restrict__ left, const T *__restrict__ right,
                                              const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                                              int64_t n, unsigned long long *ws, int64_t *scaler_sum,
                                              const T *__restrict__ tipvec,
                                              const T *__restrict__ pl_t = nullptr,
                                              const T *__restrict__ pr_t = nullptr) {
  constexpr int S = 20;
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  using PT = ProtTile<T>;
  using V = typename PT::V;
  constexpr int E = 16 / (int)sizeof(T);          // elements per 16-B LDS read
  constexpr int kPh3 = sizeof(T) == 8 ? 10 : 20;  // phase-3 chains per pass
  static_assert(kRows % E == 0 && S % kRows == 0, "kRows: a divisor of 20, whole 16-B reads");
  constexpr int RV = kRows / E, PV = kPh3 / E, kDist = 2;
  constexpr bool kPacked = kPack && sizeof(T) == 4;  // f32: packed VALU on chain pairs
  // elements 2q, 2q+1 of a run of 16-B reads, as a pair
  auto pair2 = [](const V *r, int q) -> f32x2 {
    if constexpr (sizeof(T) == 4) {
      const f32x4 w = r[(2 * q) / 4];
      return (q & 1) ? f32x2{w.z, w.w} : f32x2{w.x, w.y};
    } else {
      return f32x2{};
    }
  };
  __shared__ T tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<T, kFma>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<T, kFma>(right, tipvec, tabs[1]);
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // P_L[4][400] (unless x1 is a tip) | P_R[4][400] (unless x2 is a tip) | EV[400]
  // in T elements; a tip child's matrix lives in its table instead
  constexpr int oR = T1 ? 0 : 4 * S * S, oE = oR + (T2 ? 0 : 4 * S * S);
  // kNoMats (with kPS = 3 and kE3S: every matrix as SGPR operands): no LDS copy,
  // so the block's LDS is the tile alone and three blocks fit a CU
  __shared__ V mats[kNoMats ? 1 : (oE + S * S) / E];
  if constexpr (!kNoMats) {
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
  // values; fn(k, sum_l x[l] * M[k][l]) for every k.  gsrc (kPS): the same
  // layout in global memory, read by scalar loads (SGPR operands)
  auto gphase = [&](const V *M, const T (&x)[S], auto &&fn, const T *gsrc = nullptr) {
    int o = 0;
    T tok = T(0);
    if constexpr (kPS != 0 && !kFma && !kPacked) {
      if (kNoMats || gsrc) {
#pragma unroll
        for (int gk = 0; gk < S / kRows; gk++) {
          const T *gp = gsrc + gk * S * kRows;
          int so = 0;
          asm volatile("" : "+s"(so) : "v"(tok));
          T cur[kRows], nxt[kRows], u[kRows];
#pragma unroll
          for (int j = 0; j < kRows; j++) cur[j] = gp[so + j];
#pragma unroll
          for (int l = 0; l < S; l++) {
            asm volatile("" : "+s"(so) : "v"(tok));  // column l+1's loads after column l-1's chains
            if (l + 1 < S) {
#pragma unroll
              for (int j = 0; j < kRows; j++) nxt[j] = gp[so + (l + 1) * kRows + j];
            }
            T pr[kRows];
#pragma unroll
            for (int j = 0; j < kRows; j++) pr[j] = x[l] * cur[j];
            pin_chains(pr);
#pragma unroll
            for (int j = 0; j < kRows; j++) u[j] = l == 0 ? pr[j] : u[j] + pr[j];
            pin_chains(u);
            tok = u[kRows - 1];
#pragma unroll
            for (int j = 0; j < kRows; j++) cur[j] = nxt[j];
          }
#pragma unroll
          for (int j = 0; j < kRows; j++) fn(gk * kRows + j, u[j]);
        }
        return;
      }
    }
    if constexpr (kNoMats) return;
#pragma unroll
    for (int gk = 0; gk < S / kRows; gk++) {
      const V *G = M + gk * S * RV;
      V ring[kDist + 1][RV];
      T u[kPacked ? 1 : kRows];
      f32x2 u2[kPacked ? kRows / 2 : 1];
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
        if constexpr (kPacked) {
          // f32: chain pairs on the packed VALU (v_pk_mul/add/fma_f32, two
          // IEEE f32 operations per lane and instruction)
          const f32x2 xv = {x[l], x[l]};
          if (l == 0 || !kFma) {
            f32x2 pr[kRows / 2];
#pragma unroll
            for (int q = 0; q < kRows / 2; q++) pr[q] = xv * pair2(col, q);
            pin_chains(pr);
#pragma unroll
            for (int q = 0; q < kRows / 2; q++) u2[q] = l == 0 ? pr[q] : u2[q] + pr[q];
          } else {
#pragma unroll
            for (int q = 0; q < kRows / 2; q++) u2[q] = __builtin_elementwise_fma(xv, pair2(col, q), u2[q]);
          }
          pin_chains(u2);
          tok = u2[kRows / 2 - 1].y;
        } else {
        if (l == 0 || !kFma) {
          // all kRows products, then all kRows adds: no add waits on the
          // multiply just before it (chains start at q0: site_cat, plf_dna.hpp)
          T pr[kRows];
#pragma unroll
          for (int j = 0; j < kRows; j++) pr[j] = x[l] * col[j / E][j % E];
          pin_chains(pr);
#pragma unroll
          for (int j = 0; j < kRows; j++) u[j] = l == 0 ? pr[j] : u[j] + pr[j];
        } else {
#pragma unroll
          for (int j = 0; j < kRows; j++) u[j] = madd<T, true>(x[l], col[j / E][j % E], u[j]);
        }
        pin_chains(u);
        tok = u[kRows - 1];
        }
      }
      if constexpr (kPacked) {
#pragma unroll
        for (int q = 0; q < kRows / 2; q++) {
          fn(gk * kRows + 2 * q, (T)u2[q].x);
          fn(gk * kRows + 2 * q + 1, (T)u2[q].y);
        }
      } else {
#pragma unroll
        for (int j = 0; j < kRows; j++) fn(gk * kRows + j, u[j]);
      }
    }
  };
  constexpr bool kAnyDense = !(T1 && T2);
  const T *FD = T1 ? x2 : x1;  // the trip's first dense child
  const int64_t stride = (int64_t)gridDim.x * 64;
  constexpr int K = PT::kChunks / kBlock;
  V pf[kPf ? K : 1];  // unused (and eliminated) when both children are tips
  if constexpr (kPf && kAnyDense)
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<T>(FD, (int64_t)blockIdx.x * 64, n, pf);
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const V *mL = mats + off + c * (S * S / E), *mR = mats + off + (oR + c * S * S) / E,
            *mE = mats + off + oE / E;
    T U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    // stage a dense child's tile: from the prefetch registers (then fetch the
    // next tile in the sequence) or straight from HBM
    auto stage = [&](const T *g, const T *next, int64_t nbase) {
      if constexpr (kPf) {
        tile_put<T>(tile, pf);
        __syncthreads();
        if (nbase < n) tile_fetch<T>(next, nbase, n, pf);
      } else {
        tile_load<T>(g, base, n, tile);
        __syncthreads();
      }
    };
    if constexpr (T1) {  // tip: U from the table row of the site's code
      const T *r = tabs[0] + c * kProtCodes * 20 + prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) * 20;
#pragma unroll
      for (int k = 0; k < S; k++) U[k] = r[k];
    } else {
      T a[S];
      // next in the sequence: this trip's x2, or the next trip's x1 when x2 is a tip
      stage(x1, T2 ? x1 : x2, T2 ? base + stride : base);
      row_read<T>(tile, lane, c, a);
      __syncthreads();
      gphase(mL, a, [&](int k, T u) { U[k] = u; }, ((kPS & 1) && pl_t) ? pl_t + c * S * S : nullptr);
    }
    if constexpr (T2) {
      const T *r = tabs[1] + c * kProtCodes * 20 + prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) * 20;
#pragma unroll
      for (int k = 0; k < S; k++) U[k] = U[k] * r[k];
    } else {
      T b[S];
      stage(x2, FD, base + stride);  // next: the next trip's first dense child
      row_read<T>(tile, lane, c, b);
      __syncthreads();
      gphase(mR, b, [&](int k, T u) { U[k] = U[k] * u; }, ((kPS & 2) && pr_t) ? pr_t + c * S * S : nullptr);
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
        T v[kPacked ? 1 : kPh3];
        f32x2 v2[kPacked ? kPh3 / 2 : 1];
#pragma unroll
        for (int j = 0; j < (kPacked ? 1 : kPh3); j++) v[j] = T(0);
#pragma unroll
        for (int q = 0; q < (kPacked ? kPh3 / 2 : 1); q++) v2[q] = f32x2{0.f, 0.f};
        asm volatile("" : "+v"(o) : "v"(tok));
        if constexpr (!kNoMats)
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
          for (int j = 0; j < PV; j++) ring[k][j] = G[o + (S / E) * k + j];
#pragma unroll
        for (int k = 0; k < S; k++) {
          asm volatile("" : "+v"(o) : "v"(tok));
          if (!kNoMats && k + 2 < S) {
#pragma unroll
            for (int j = 0; j < PV; j++) ring[(k + 2) % 3][j] = G[o + (S / E) * (k + 2) + j];
          }
          const V *e = ring[k % 3];
          if constexpr (kE3S && !kPacked && !kFma) {
            // tuning (kE3S): EV row k straight from global memory at a
            // wave-uniform address -- scalar loads, SGPR operands -- instead
            // of LDS broadcasts (one row ahead: the opaque offset)
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
            continue;
          }
          if constexpr (kPacked) {
            const f32x2 uv = {(float)U[k], (float)U[k]};
            if constexpr (kFma) {
#pragma unroll
              for (int q = 0; q < kPh3 / 2; q++) v2[q] = __builtin_elementwise_fma(uv, pair2(e, q), v2[q]);
            } else {
              f32x2 pr[kPh3 / 2];
#pragma unroll
              for (int q = 0; q < kPh3 / 2; q++) pr[q] = uv * pair2(e, q);
              pin_chains(pr);
#pragma unroll
              for (int q = 0; q < kPh3 / 2; q++) v2[q] += pr[q];
            }
            pin_chains(v2);
            tok = v2[kPh3 / 2 - 1].y;
            continue;
          }
          if constexpr (kFma) {
#pragma unroll
            for (int j = 0; j < kPh3; j++) v[j] = madd<T, true>(U[k], e[j / E][j % E], v[j]);
          } else {
            T pr[kPh3];
#pragma unroll
            for (int j = 0; j < kPh3; j++) pr[j] = U[k] * e[j / E][j % E];
            pin_chains(pr);
#pragma unroll
            for (int j = 0; j < kPh3; j++) v[j] += pr[j];
          }
          pin_chains(v);
          tok = v[kPh3 - 1];
        }
        if constexpr (kPacked) {
#pragma unroll
          for (int q = 0; q < kPh3 / 2; q++) {
            O[h * kPh3 + 2 * q] = (T)v2[q].x;
            O[h * kPh3 + 2 * q + 1] = (T)v2[q].y;
          }
        } else {
#pragma unroll
          for (int j = 0; j < kPh3; j++) O[h * kPh3 + j] = v[j];
        }
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

// kPack (f32): chain pairs on v_pk_* -- faster in FMA mode (one v_pk_fma_f32
// per two multiply-adds), slower in exact mode at 4-row groups
// (tools/tune_prot32.hip, profiles/r02_tune_protein_f32.log).
// kE3S (exact mode): phase 3's EV rows by scalar loads (SGPR operands) instead of
// LDS broadcasts: 145.8 vs 148.8 us at 2^18 f64 (profiles/r02_tune_protein_exact_rows.log).
template <typename T, bool kFma, bool kSum, int kMinWaves, int kTips, int kRows, bool kPf = true,
          bool kPack = kFma, bool kE3S = false>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_lds_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
                    const T *__restrict__ EV, const T *__restrict__ left, const T *__restrict__ right,
                    const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                    unsigned long long *ws, int64_t *scaler_sum, const T *__restrict__ tipvec = nullptr) {
  prot_lds_body<T, kFma, kSum, kTips, kRows, kPf, kPack, kE3S>(x1, x2, x3, EV, left, right, wgt,
                                                                scaler, n, ws, scaler_sum, tipvec);
}

// Tuning form of the exact f64 kernel with phase 2's matrix as SGPR operands
// (kPS = 2; not launched by the product): plf_prot_lds_kernel plus pr_t, the
// group-transposed P_R made by prot_group_transpose on the same stream.
template <bool kSum, int kMinWaves, int kTips>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_exact64_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                        double *__restrict__ x3, const double *__restrict__ EV,
                        const double *__restrict__ left, const double *__restrict__ right,
                        const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                        unsigned long long *ws, int64_t *scaler_sum, const double *__restrict__ tipvec,
                        const double *__restrict__ pr_t) {
  prot_lds_body<double, false, kSum, kTips, 10, true, false, true, 2>(
      x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum, tipvec, nullptr, pr_t);
}

// Tuning form of the exact f64 kernel with EVERY matrix as SGPR operands (kPS =
// 3 from the group-transposed copies pl_t / pr_t, kE3S for EV) and no LDS copy
// of the matrices (kNoMats), so up to three blocks fit a CU (LDS = the tile).
template <bool kSum, int kMinWaves, bool kPf>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_exact_sgpr_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                           double *__restrict__ x3, const double *__restrict__ EV,
                           const double *__restrict__ left, const double *__restrict__ right,
                           const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                           unsigned long long *ws, int64_t *scaler_sum, const double *__restrict__ pl_t,
                           const double *__restrict__ pr_t) {
  prot_lds_body<double, false, kSum, 0, 10, kPf, false, true, 3, true>(
      x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum, nullptr, pl_t, pr_t);
}

// The group-transposed copy of a 4-category S = 20 matrix for kPS:
// Pt[c][k / kRows][l][k % kRows] = P[c][k][l] (one block; stream-ordered before
// the kernel that reads it).
template <typename T, int kRows>
__global__ void __launch_bounds__(kBlock) prot_group_transpose(const T *__restrict__ P, T *__restrict__ Pt) {
  constexpr int S = 20;
  for (int i = threadIdx.x; i < 4 * S * S; i += kBlock) {
    const int cc = i / (S * S), r = i - cc * S * S, k = r / S, l = r - k * S;
    Pt[cc * S * S + (k / kRows) * (S * kRows) + l * kRows + (k % kRows)] = P[i];
  }
}

// The round-1 EXACT f64 form, kept for same-process comparisons
// (tools/tune_prot.hip): one chain per row k, the row streamed one ahead.
// kRows > 0 runs the product body (plf_prot_lds_kernel) instead.
template <bool kSum, int kMinWaves = 2, int kTips = 0, int kRows = 0, bool kPf = false,
          bool kE3S = false, int kPS = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_exact_f64_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                          double *__restrict__ x3, const double *__restrict__ EV,
                          const double *__restrict__ left, const double *__restrict__ right,
                          const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                          unsigned long long *ws, int64_t *scaler_sum,
                          const double *__restrict__ tipvec = nullptr,
                          const double *__restrict__ pl_t = nullptr,
                          const double *__restrict__ pr_t = nullptr) {
  if constexpr (kRows > 0) {
    prot_lds_body<double, false, kSum, kTips, kRows, kPf, false, kE3S, kPS>(
        x1, x2, x3, EV, left, right, wgt, scaler, n, ws, scaler_sum, tipvec, pl_t, pr_t);
    return;
  } else {
  constexpr int S = 20;
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  __shared__ double tabs[(T1 ? 1 : 0) + (T2 ? 1 : 0) + (T1 ? 0 : 1)][T1 ? 4 * kProtCodes * 20 : 1];
  if constexpr (T1) build_prot_tip_table<double, false>(left, tipvec, tabs[0]);
  if constexpr (T2) build_prot_tip_table<double, false>(right, tipvec, tabs[1]);
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  constexpr int oR = T1 ? 0 : 800, oE = oR + (T2 ? 0 : 800);
  __shared__ f64x2 mats[oE + 200];
  {
    const f64x2 *gl = reinterpret_cast<const f64x2 *>(left);
    const f64x2 *gr = reinterpret_cast<const f64x2 *>(right);
    const f64x2 *ge = reinterpret_cast<const f64x2 *>(EV);
    for (int i = threadIdx.x; i < 800; i += kBlock) {
      if constexpr (!T1) mats[i] = gl[i];
      if constexpr (!T2) mats[oR + i] = gr[i];
    }
    for (int i = threadIdx.x; i < 200; i += kBlock) mats[oE + i] = ge[i];
  }
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  __syncthreads();
  // rows M[k] (10 x f64x2) feed fn(k, row), which returns a value of its result
  auto phase = [&](const f64x2 *M, auto &&fn) {
    f64x2 cur[10], nxt[10];
    int o = 0;
    double tok = 0.0;
#pragma unroll
    for (int i = 0; i < 10; i++) cur[i] = M[i];
#pragma unroll
    for (int k = 0; k < S; k++) {
      asm volatile("" : "+v"(o) : "v"(tok));  // row k+1 is read after row k-1 is used
      if (k + 1 < S) {
#pragma unroll
        for (int i = 0; i < 10; i++) nxt[i] = M[o + (k + 1) * 10 + i];
      }
      tok = fn(k, cur);
#pragma unroll
      for (int i = 0; i < 10; i++) cur[i] = nxt[i];
    }
  };
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const f64x2 *mL = mats + off + c * 200, *mR = mats + off + oR + c * 200, *mE = mats + off + oE;
    double U[S];
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    if constexpr (T1) {  // tip: U from the table row of the site's code
      const double *r = tabs[0] + c * kProtCodes * 20 + prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) * 20;
#pragma unroll
      for (int k = 0; k < S; k++) U[k] = r[k];
    } else {
      double a[S];
      tile_load<double>(x1, base, n, tile);
      __syncthreads();
      row_read<double>(tile, lane, c, a);
      __syncthreads();
      phase(mL, [&](int k, const f64x2 (&p)[10]) {
        double u = a[0] * p[0].x;  // chain starts at q0: same x3 bits (site_cat, plf_dna.hpp)
        u += a[1] * p[0].y;
#pragma unroll
        for (int i = 1; i < 10; i++) {
          u += a[2 * i] * p[i].x;
          u += a[2 * i + 1] * p[i].y;
        }
        U[k] = u;
        return u;
      });
    }
    if constexpr (T2) {
      const double *r = tabs[1] + c * kProtCodes * 20 + prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) * 20;
#pragma unroll
      for (int k = 0; k < S; k++) U[k] = U[k] * r[k];
    } else {
      double b[S];
      tile_load<double>(x2, base, n, tile);
      __syncthreads();
      row_read<double>(tile, lane, c, b);
      __syncthreads();
      phase(mR, [&](int k, const f64x2 (&p)[10]) {
        double u = b[0] * p[0].x;  // chain starts at q0: same x3 bits (site_cat, plf_dna.hpp)
        u += b[1] * p[0].y;
#pragma unroll
        for (int i = 1; i < 10; i++) {
          u += b[2 * i] * p[i].x;
          u += b[2 * i + 1] * p[i].y;
        }
        U[k] = U[k] * u;
        return U[k];
      });
    }
    double O[S];
#pragma unroll
    for (int l = 0; l < S; l++) O[l] = 0.0;
    phase(mE, [&](int k, const f64x2 (&e)[10]) {
#pragma unroll
      for (int i = 0; i < 10; i++) {
        O[2 * i] += U[k] * e[i].x;
        O[2 * i + 1] += U[k] * e[i].y;
      }
      return O[S - 1];
    });
    bool small = base + lane < n;
#pragma unroll
    for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[l]) < m);
    const unsigned long long mk = __ballot(small);
    if (lane == 0) small_mask[c] = mk;
    __syncthreads();  // also: every wave is done reading x2 from the tile
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    const bool sc = (all >> lane) & 1ull;
#pragma unroll
    for (int l = 0; l < S; l++) {
      const double sv = O[l] * Num<double>::two32();
      O[l] = sc ? sv : O[l];
    }
    row_write<double>(tile, lane, c, O);
    const int64_t site = base + lane;
    if (site < n && c == 0) {
      if (scaler) scaler[site] = (uint8_t)sc;
      if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
    }
    __syncthreads();
    tile_store<double>(x3, base, n, tile);
    __syncthreads();  // tile and small_mask are reused by the next trip
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
  }
}

// ---------------------------------------------------------------------------
// FMA mode on the matrix cores (f64).  v_mfma_f64_16x16x4_f64 is bit-for-bit a
// k-ordered fma chain (probed on MI355X: tools/probes/mfma_f64_numerics.hip),
// so this kernel reproduces plf()'s loop with every multiply-add fused, in the
// same order -- identical to the VALU FMA kernel above and to the oracle's
// fma() restatement.  Per category (wave) and 16-site sub-tile:
//   U^T[k][site]   = P[k][l]  . X^T[l][site]   (M = k: 2 tiles, N = 16 sites,
//                                               K = l: 5 steps of 4)
//   p              = U_L^T * U_R^T             (accumulator registers, VALU)
//   X3^T[l][site]  = EV^T[l][k] . p[k][site]   (the accumulators of the first
//                                               product ARE the B fragments:
//                                               k-step s = tile s>>2, reg s&3)
// A fragments (P rows, EV columns) stay in VGPRs for the whole kernel; B
// fragments (X^T) come from the LDS tile, conflict-free.
// kMix4: rows 16..19 of each product (M = 20 = 16 + 4) on v_mfma_f64_4x4x4_4b_f64
// -- four 4x4x4 blocks = the 16 sites, 20 cycles -- instead of a zero-padded
// second 16x16x4 tile (64 cycles): 420 instead of 640 matrix-core cycles per
// product and sub-tile.  Its operand maps make the two forms interchangeable
// (A lane 16k+4b+i, B lane 16k+4b+j, D lane 16i+4b+j: the B fragment is the
// same LDS value, and D lands as row 16 + lane/16 of site lane%16 -- exactly
// the k-step-4 B fragment of the back-transform), and it too is bit-for-bit a
// k-ordered fma chain (tools/probes/mfma_f64_4x4x4_numerics.hip).
typedef double f64x4 __attribute__((ext_vector_type(4)));

// Exchange the upper 16-lane row of each 32-lane half of v (lanes 16-31,
// 48-63) with the lower row of w (lanes 0-15, 32-47), per 64-bit value
// (v_permlane16_swap, gfx950).
__device__ __forceinline__ void swap_rows16(double &v, double &w) {
  const long long a = __builtin_bit_cast(long long, v), b = __builtin_bit_cast(long long, w);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(a >> 32), (unsigned)(b >> 32), false,
                                                   false);
  v = __builtin_bit_cast(double, ((long long)hi[0] << 32) | (unsigned)lo[0]);
  w = __builtin_bit_cast(double, ((long long)hi[1] << 32) | (unsigned)lo[1]);
}

// kAblate (tuning only, tools/tune_prot.hip): 0 = the kernel; 1 = no matrix-core
// work (VALU stand-ins keep the LDS reads); 2 = no HBM loads or stores.
// kX3 = how the back-transform's results reach the LDS tile: 0 = five
// ds_write_b64 per lane and sub-tile (2-way bank conflicts: sites lo16 and
// lo16+8 share banks at the 82-double row stride); 1 = 16-B pairs (l, l+1)
// after row swaps (swap_rows16), 3 ds_write_b128, conflict-free; 2 = the
// back-transform's A rows permuted (row g + 4r computes state 4g + r) so a
// lane's four 16x16x4 results are four consecutive states: 2 conflict-free
// ds_write_b128 + 1 ds_write_b64, no lane movement (bit-identical: a row
// permutation of the A operand permutes the outputs, nothing else).
// kEarly: the first child tile's loads go out before the matrix fragments'.
// kFirstX2 (dense children): the first trip's x2 tile is fetched at kernel
// start too, instead of after the first x1 tile has landed (one HBM latency
// less in the start-up; the first trip is peeled so the extra registers are
// not live in the loop).
// kSplitB: the B-fragment reads stay separate ds_read_b64 (banks (a/4) mod 64,
// 2 x 32 lanes: conflict-free at the 164-dword row stride); left alone the
// compiler pairs the k-steps 32 B apart into ds_read2_b64, which banks mod 32
// in 16-lane groups (sites lo16 and lo16+8 collide: 2-way) and takes 8 LDS
// cycles instead of 2 x 2.
// kSwz (with kPrefetch, kX3 = 2): the two doubles of every 16-B chunk of the
// tile rows of sites 8..15 of each 16-site group are stored swapped (double
// index d -> d ^ 1 in those rows).  The paired B reads keep their ds_read2_b64
// (the pair's 32-B offset is unchanged by the swap) but sites lo16 and lo16+8
// now start 8 B apart, so the 16 lanes of a read2 group cover all 32 banks
// once; the rows-16..19 ds_write_b64 of X3 becomes conflict-free the same way.
// The b128 tile writes and the store pass move whole chunks and swap the two
// halves back with a select (tools/lds_banks.py, swizzle rows).
// kSpread (tuning, with kPrefetch): the next child tile's ten 16-B loads per
// thread go out in four parts, part t right after sub-tile t's B-fragment
// reads, instead of all at the start of the phase (fewer requests in flight
// at once: the stream probes' V = 1..2 regime).
template <bool kSum, int kMinWaves = 2, bool kPrefetch = true, int kAblate = 0, bool kMix4 = true,
          int kTips = 0, int kX3 = 0, bool kEarly = false, bool kFirstX2 = false,
          bool kSplitB = false, bool kSwz = false, bool kSpread = false>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
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
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lo16 = lane & 15, g = lane >> 4;
  // kPrefetch: the next child tile's loads are in flight while the current
  // one is multiplied (x2 during phase 1, the next trip's x1 during phase 2)
  f64x2 pf[PT::kChunks / kBlock];
  const int64_t stride = (int64_t)gridDim.x * 64;
  if constexpr (kAblate == 2)
    for (auto &q : pf) q = f64x2{1.0, 1.0};
  constexpr bool kX2Early = kFirstX2 && kEarly && kPrefetch && kAblate != 2 && kTips == 0;
  f64x2 pf2[kX2Early ? PT::kChunks / kBlock : 1];
  if constexpr (kEarly && kPrefetch && kAblate != 2 && !T2)  // the first dense child's first tile
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  if constexpr (kX2Early)
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(x2, (int64_t)blockIdx.x * 64, n, pf2);
  // A fragments: [mt][s] -> lane holds M[row = 16mt + lo16][col = 4s + g]
  // (kMix4: [1][s] -> M[row = 16 + lane%4][col = 4s + g], the 4x4x4_4b form)
  double AL[2][5], AR[2][5], AE[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; mt++)
#pragma unroll
    for (int st = 0; st < 5; st++) {
      const int row = (kMix4 && mt == 1) ? 16 + (lane & 3) : 16 * mt + lo16, col = 4 * st + g;
      AL[mt][st] = row < S ? left[c * S * S + row * S + col] : 0.0;   // P_L[k=row][l=col]
      AR[mt][st] = row < S ? right[c * S * S + row * S + col] : 0.0;
      // EV^T[l=row][k=col]; kX3 == 2: A row i of the first tile computes state 4*(i%4) + i/4
      const int erow = (kX3 >= 2 && mt == 0) ? 4 * (lo16 & 3) + (lo16 >> 2) : row;
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
  static_assert(!kSwz || (kPrefetch && kX3 == 2), "kSwz: the prefetch path with kX3 = 2");
  const int sw = kSwz ? (lo16 >> 3) & 1 : 0;  // this lane's rows are swizzled
  auto swap2 = [](f64x2 v, bool on) { return on ? f64x2{v.y, v.x} : v; };
  // a prefetched child tile into LDS (kSwz: halves of the swizzled rows swapped)
  auto put = [&](const f64x2 (&v)[PT::kChunks / kBlock]) {
    if constexpr (kSwz) {
#pragma unroll
      for (int i = 0; i < PT::kChunks / kBlock; i++) {
        const int j = threadIdx.x + i * kBlock;
        const int s_ = j / PT::kChunksPerSite, q = j - s_ * PT::kChunksPerSite;
        tile[s_ * PT::kStride + q] = swap2(v[i], (s_ >> 3) & 1);
      }
    } else {
      tile_put<double>(tile, v);
    }
  };
  // the five B-fragment values of sub-tile row xr (kSplitB: each read from its
  // own laundered LDS address, so no two are paired into a ds_read2_b64)
  auto bfrag = [&](const double *xr, double (&bv)[5]) {
#pragma unroll
    for (int st = 0; st < 5; st++) {
      if constexpr (kSplitB) {
        using L = const __attribute__((address_space(3))) double;
        L *q = (L *)(xr + 4 * st);
        asm volatile("" : "+v"(q));
        bv[st] = *q;
      } else {
        bv[st] = xr[4 * st];
      }
    }
  };
  // kSpread: part `part` (of 4) of a tile fetch into pf; z is an opaque zero
  // tied to the sub-tile's B reads, so the part cannot be hoisted above them
  auto fetch_part = [&](const double *src, int64_t b, int part, int z) {
    constexpr int K = PT::kChunks / kBlock;
    const f64x2 *sp = reinterpret_cast<const f64x2 *>(src + b * 80) + z;
    const int i0 = part * K / 4, i1 = (part + 1) * K / 4;
    if (b + 64 <= n) {
#pragma unroll
      for (int i = 0; i < K; i++)
        if (i >= i0 && i < i1) pf[i] = __builtin_nontemporal_load(sp + threadIdx.x + i * kBlock);
    } else {
      const int64_t lim = (n - b) * PT::kChunksPerSite;
#pragma unroll
      for (int i = 0; i < K; i++) {
        if (i < i0 || i >= i1) continue;
        const int j = threadIdx.x + i * kBlock;
        pf[i] = f64x2{0.0, 0.0};
        if (j < lim) pf[i] = __builtin_nontemporal_load(sp + j);
      }
    }
  };
  if constexpr (!kEarly && kPrefetch && kAblate != 2 && !T2)  // the first dense child's first tile
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<double>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  auto trip = [&](const int64_t base, auto first_tag) {
    constexpr bool kFirst = decltype(first_tag)::value;
    f64x4 P[4][2];  // per sub-tile: U_L^T, then p = U_L^T * U_R^T
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
    } else if constexpr (kPrefetch) {
      put(pf);
      __syncthreads();
      if constexpr (kFirst && kX2Early) {
#pragma unroll
        for (int i = 0; i < PT::kChunks / kBlock; i++) pf[i] = pf2[i];
      } else if constexpr (kAblate != 2 && !kSpread) {
        tile_fetch<double>(x2, base, n, pf);
      }
    } else {
      tile_load<double>(x1, base, n, tile);
      __syncthreads();
    }
    constexpr bool kSp1 = kSpread && kPrefetch && kAblate != 2 && !(kFirst && kX2Early);
    if constexpr (!T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) {
        double bv[5];
        bfrag(td + (16 * t + lo16) * kRow + c * S + (g ^ sw), bv);
        if constexpr (kSp1) {
          int z = 0;
          asm volatile("" : "+v"(z) : "v"(bv[0]));
          fetch_part(x2, base, t, z);
        }
#pragma unroll
        for (int mt = 0; mt < 2; mt++) {
          f64x4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int st = 0; st < 5; st++) {
            if constexpr (kAblate == 1) u[st & 3] += bv[st] * AL[mt][st];
            else if (kMix4 && mt == 1) u[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AL[1][st], bv[st], u[0], 0, 0, 0);
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
    if constexpr (kPrefetch) {
      put(pf);
      __syncthreads();
      // next trip's first dense child: x1, or x2 when x1 is a tip
      if (!kSpread && kAblate != 2 && base + stride < n) tile_fetch<double>(T1 ? x2 : x1, base + stride, n, pf);
    } else {
      tile_load<double>(x2, base, n, tile);
      __syncthreads();
    }
    const bool sp2 = kSpread && kPrefetch && kAblate != 2 && base + stride < n;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      double bv[5];
      bfrag(td + (16 * t + lo16) * kRow + c * S + (g ^ sw), bv);
      if constexpr (kSpread) {
        if (sp2) {
          int z = 0;
          asm volatile("" : "+v"(z) : "v"(bv[0]));
          fetch_part(T1 ? x2 : x1, base + stride, t, z);
        }
      }
#pragma unroll
      for (int mt = 0; mt < 2; mt++) {
        f64x4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 5; st++) {
          if constexpr (kAblate == 1) u[st & 3] += bv[st] * AR[mt][st];
          else if (kMix4 && mt == 1) u[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AR[1][st], bv[st], u[0], 0, 0, 0);
          else u = __builtin_amdgcn_mfma_f64_16x16x4f64(AR[mt][st], bv[st], u, 0, 0, 0);
        }
        P[t][mt] = P[t][mt] * u;  // prod[k] = umpL[k] * umpR[k]
      }
    }
    __syncthreads();  // every wave is done reading x2: the tile takes X3 now
    }
    // back-transform: lane holds X3[site 16t+lo16][l = 16mt + g + 4r]; written
    // unscaled into the tile, the x2^32 rescale happens in the store pass
    unsigned long long mine = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      f64x4 X0 = {0.0, 0.0, 0.0, 0.0}, X1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        if constexpr (kAblate == 1) {
          X0[st & 3] += AE[0][st] * P[t][st >> 2][st & 3];
          X1[st & 3] += AE[1][st] * P[t][st >> 2][st & 3];
        } else {
          X0 = __builtin_amdgcn_mfma_f64_16x16x4f64(AE[0][st], P[t][st >> 2][st & 3], X0, 0, 0, 0);
          if constexpr (kMix4) X1[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(AE[1][st], P[t][st >> 2][st & 3], X1[0], 0, 0, 0);
          else X1 = __builtin_amdgcn_mfma_f64_16x16x4f64(AE[1][st], P[t][st >> 2][st & 3], X1, 0, 0, 0);
        }
      }
      const bool small = (__builtin_fabs(X0[0]) < m) && (__builtin_fabs(X0[1]) < m) &&
                         (__builtin_fabs(X0[2]) < m) && (__builtin_fabs(X0[3]) < m) &&
                         (__builtin_fabs(X1[0]) < m);
      const unsigned long long b = __ballot(small);
      // site lo16 of sub-tile t is small in category c iff its 4 lanes agree
      mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
      double *w = tw + (16 * t + lo16) * kRow + c * S;
      if constexpr (kX3 == 2) {
        *reinterpret_cast<f64x2 *>(w + 4 * g) = swap2(f64x2{X0[0], X0[1]}, sw);
        *reinterpret_cast<f64x2 *>(w + 4 * g + 2) = swap2(f64x2{X0[2], X0[3]}, sw);
        w[16 + (g ^ sw)] = X1[0];
      } else if constexpr (kX3 == 3) {
        // kX3 == 2, and states 16..19 as 16-B pairs: after swap_rows16(X1,
        // copy) the lanes of even rows hold (16 + g, 17 + g)
        *reinterpret_cast<f64x2 *>(w + 4 * g) = f64x2{X0[0], X0[1]};
        *reinterpret_cast<f64x2 *>(w + 4 * g + 2) = f64x2{X0[2], X0[3]};
        double b0 = X1[0], b1 = X1[0];
        swap_rows16(b0, b1);
        if (!(g & 1)) *reinterpret_cast<f64x2 *>(w + 16 + g) = f64x2{b0, b1};
      } else if constexpr (kX3 == 1) {
        // lane of row g holds l = g + 4r (X0[r]) and 16 + g (X1).  After
        // swap_rows16(X0[1], X0[0]) a lane of an even row holds (g+4, g+5),
        // of an odd row (g-1, g); after swap_rows16(X0[3], X0[2]) (g+12, g+13)
        // resp. (g+7, g+8); after swap_rows16(X1, copy) even rows hold
        // (16+g, 17+g).  b128 groups of 8 lanes: row stride 164 dwords = 4
        // banks, so 8 sites x 4 dwords cover the 32 banks once.
        double a0 = X0[0], a1 = X0[1], a2 = X0[2], a3 = X0[3], b0 = X1[0], b1 = X1[0];
        swap_rows16(a1, a0);
        swap_rows16(a3, a2);
        swap_rows16(b0, b1);
        const bool odd = g & 1;
        *reinterpret_cast<f64x2 *>(w + (odd ? g - 1 : g + 4)) = f64x2{a1, a0};
        *reinterpret_cast<f64x2 *>(w + (odd ? g + 7 : g + 12)) = f64x2{a3, a2};
        if (!odd) *reinterpret_cast<f64x2 *>(w + 16 + g) = f64x2{b0, b1};
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++) w[g + 4 * r] = X0[r];
        w[16 + g] = X1[0];
      }
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
      constexpr int K = PT::kChunks / kBlock;
      f64x2 *dst = reinterpret_cast<f64x2 *>(x3 + base * 80);
      f64x2 v[K];
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        const int sl = j / PT::kChunksPerSite, q = j - sl * PT::kChunksPerSite;
        v[i] = tile[sl * PT::kStride + q];
        if constexpr (kSwz) v[i] = swap2(v[i], (sl >> 3) & 1);
        if ((all >> sl) & 1ull) v[i] = v[i] * Num<double>::two32();
      }
      if (kAblate == 2) {
        f64x2 t = v[0];
#pragma unroll
        for (int i = 1; i < K; i++) t += v[i];
        if (t.x == -1.25) dst[threadIdx.x] = t;  // keeps the LDS reads alive
      } else if (base + 64 <= n) {
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
  };
  int64_t base = (int64_t)blockIdx.x * 64;
  if constexpr (kX2Early) {
    if (base < n) trip(base, std::true_type{});
    base += stride;
  }
  for (; base < n; base += stride) trip(base, std::false_type{});
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}


// ---------------------------------------------------------------------------
// FMA mode on the matrix cores, f32: v_mfma_f32_16x16x4_f32 is exact f32, a
// k-ordered fmaf chain bit for bit (MI355X_MICROARCH.md, FP32-input MFMA), so
// this kernel is bit-identical to the f32 VALU FMA kernels and the oracle's
// fused restatement.  The f64 kernel's scheme with the f32 operand maps
// (A: lane l = A[row l&15][k l>>4], B: lane l = B[k l>>4][col l&15],
// C/D: lane l reg r = D[row 4(l>>4) + r][col l&15] -- rows by 4 per lane group,
// where f64 interleaves them):
//   U^T[k][site] = P[k][l] . X^T[l][site]: A row i of tile mt computes
//     k = pi(16 mt + i) = 16 mt + 4 (i&3) + (i>>2), so lane group g, reg r holds
//     k = 16 mt + 4 r + g -- exactly the B fragment of k-step s = 4 mt + r of
//     the back-transform (lane group g = k 4s + g); tile 1 keeps only reg 0
//     (k = 16 + g), its other rows are zero;
//   X3^T[l][site] = EV^T[l][k] . p[k][site]: natural rows, so lane group g
//     holds states 4g..4g+3 of its site (tile 0) and lane group 0 states 16..19
//     (tile 1): one 16-B LDS write each, no lane movement.
// Per 16-site sub-tile and category: 20 + 10 MFMAs of 32 cycles (960 cycles;
// f32 has no 4x4x4 form for rows 16..19).  Tiles as the f64 kernel (prefetch:
// x2 during phase 1, the next trip's first dense child during phase 2).
//
// kQ >= 1: rows 16..19 of both child products on v_mfma_f32_4x4x1_16b_f32
// instead of a zero-padded 16x16x4 tile.  Its maps (probed on the MI355X,
// tools/probes/mfma_f32_4x4x1.hip: block b = lane/4, A lane l = A_b[l%4][0],
// B lane l = B_b[0][l%4], D lane l reg r = D_b[r][l%4]; 20 chained K = 1 steps
// are bit for bit a k-ordered fmaf chain) give, with A = P[16 + l%4][col] and
// B = x[site l][col], lane l = the trip's site l holding U[16..19] of its own
// site after 20 steps (14 cycles each) for all 64 sites at once -- 280 cycles
// per product and trip instead of 640.  One 4x4 transpose of (lane group x
// register) by v_permlane32_swap + v_permlane16_swap then hands lane group g
// the k = 16 + g row of every sub-tile, the back-transform's B fragment of
// k-step 4.  kQ = 2: the back-transform's states 16..19 the same way (B =
// p[k][site l] for all 20 k: the rows 0..15 brought to lane l by four more
// transposes), so a lane writes states 16..19 of its site as one 16-B row.
typedef float f32x4m __attribute__((ext_vector_type(4)));

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

// kAblate (tuning only, tools/tune_prot32.hip): 1 = every MFMA replaced by one
// VALU multiply-add (no matrix cores), 2 = no HBM loads or stores, 3 = the
// tile data movement alone (x2's tile goes back out as x3: no products, no
// back-transform).
// kRing (tuning only): 1 = two child tiles in flight (x2 of this trip and x1 of
// the next during phase 1, x1 and x2 of the next trip during phase 2); 2 = both
// children staged together in two LDS tiles, the next trip's two in flight
// through both products.
template <bool kSum, int kMinWaves = 2, int kTips = 0, int kQ = 0, int kAblate = 0, int kRing = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma32_kernel(const float *__restrict__ x1, const float *__restrict__ x2,
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
  static_assert(!kRing || (kTips == 0 && kAblate != 2), "kRing: dense children");
  f32x4 pf[K];
  f32x4 pf2[kRing ? K : 1];
  // the first dense child's first tile, before the matrix fragments
  if constexpr (kAblate == 2)
    for (auto &q : pf) q = f32x4{1.f, 1.f, 1.f, 1.f};
  if constexpr (!(T1 && T2) && kAblate != 2)
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<float>(T1 ? x2 : x1, (int64_t)blockIdx.x * 64, n, pf);
  if constexpr (kRing)
    if ((int64_t)blockIdx.x * 64 < n) tile_fetch<float>(x2, (int64_t)blockIdx.x * 64, n, pf2);
  float AL[2][5], AR[2][5], AE[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; mt++)
#pragma unroll
    for (int st = 0; st < 5; st++) {
      const int i = lo16, col = 4 * st + g;
      const int k = 16 * mt + 4 * (i & 3) + (i >> 2);  // pi: accumulators = back-transform B fragments
      AL[mt][st] = (k < S && !(kQ && mt)) ? left[c * S * S + k * S + col] : 0.f;   // P_L[k][l]
      AR[mt][st] = (k < S && !(kQ && mt)) ? right[c * S * S + k * S + col] : 0.f;
      const int lrow = 16 * mt + i;  // EV^T[l][k]: natural rows
      AE[mt][st] = (lrow < S && !(kQ == 2 && mt)) ? EV[col * S + lrow] : 0.f;
    }
  // kQ: A operands of the 4x4x1 chains in LDS (registers would cost 40-60
  // VGPRs and the third block per CU): qm[0|1][cat][i][col] = P_L|P_R[16+i][col],
  // qm[2][0][i][k] = EV[k][16+i]; lane l reads row i = l%4 (4 distinct 16-B
  // addresses per 16 lanes, 20 banks apart: no conflicts)
  __shared__ float qm[kQ ? 3 : 1][kQ ? 4 : 1][4][kQ ? S : 1];
  if constexpr (kQ) {
    for (int e = threadIdx.x; e < 4 * 4 * S; e += kBlock) {
      const int cc = e / (4 * S), i = (e / S) & 3, j = e % S;
      qm[0][cc][i][j] = T1 ? 0.f : left[cc * S * S + (16 + i) * S + j];
      qm[1][cc][i][j] = T2 ? 0.f : right[cc * S * S + (16 + i) * S + j];
      if (cc == 0) qm[2][0][i][j] = EV[j * S + 16 + i];
    }
    __syncthreads();
  }
  const float *QL = &qm[0][kQ ? c : 0][lane & 3][0], *QR = &qm[kQ ? 1 : 0][kQ ? c : 0][lane & 3][0];
  const float *QE = &qm[kQ ? 2 : 0][0][lane & 3][0];
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
  __shared__ f32x4 tile2[kRing == 2 ? 64 * PT::kStride : 1];
  const float *td2 = reinterpret_cast<const float *>(tile2);
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const float *td = reinterpret_cast<const float *>(tile);
  float *tw = reinterpret_cast<float *>(tile);
  long long acc = 0;
  // one child's product U^T for the 4 sub-tiles from the LDS tile (mul: into P);
  // kQ: rows 16..19 of the lane's own site into Q (4x4x1 chain, k ascending)
  auto product = [&](const float (&A)[2][5], const float *QA, f32x4 (&P)[4][2], f32x4 &Q, bool mul,
                     const float *tb) {
    if constexpr (kAblate == 3) return;
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
    const float *xs = tb + lane * kRow + c * S;  // the lane's own site row
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const float *xr = tb + (16 * t + lo16) * kRow + c * S + g;
      float bv[5];
#pragma unroll
      for (int st = 0; st < 5; st++) bv[st] = xr[4 * st];
#pragma unroll
      for (int mt = 0; mt < (kQ ? 1 : 2); mt++) {
        f32x4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 5; st++) {
          if constexpr (kAblate == 1) u[st & 3] += bv[st] * A[mt][st];
          else u = __builtin_amdgcn_mfma_f32_16x16x4f32(A[mt][st], bv[st], u, 0, 0, 0);
        }
        P[t][mt] = mul ? P[t][mt] * u : u;  // prod[k] = umpL[k] * umpR[k]
      }
      if constexpr (kQ) {  // four of the 20 K = 1 steps per sub-tile, interleaved
        const f32x4 xv = *reinterpret_cast<const f32x4 *>(xs + 4 * t);
        const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 4 * t);
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if constexpr (kAblate == 1) q[j] += av[j] * xv[j];
          else q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
        }
      }
    }
    if constexpr (kQ) {
      const f32x4 xv = *reinterpret_cast<const f32x4 *>(xs + 16);
      const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 16);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if constexpr (kAblate == 1) q[j] += av[j] * xv[j];
        else q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
      }
      Q = mul ? Q * q : q;
    }
  };
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    f32x4 P[4][2];
    f32x4 Q = {0.f, 0.f, 0.f, 0.f};  // kQ: U[16..19] (then p[16..19]) of site `lane`
    if constexpr (kQ)  // rows 16..19 live in Q: the padded tiles stay zero (and unused)
#pragma unroll
      for (int t = 0; t < 4; t++) P[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t sq = base + lane < n ? base + lane : n - 1;
    const int code1 = T1 ? prot_code(reinterpret_cast<const uint8_t *>(x1)[sq]) : 0;
    const int code2 = T2 ? prot_code(reinterpret_cast<const uint8_t *>(x2)[sq]) : 0;
    // kQ: a tip child's U[16..19] of the lane's own site from its table row
    auto tip_q = [&](const float *tab, int code_lane) -> f32x4 {
      const float *r = tab + c * kProtCodes * 20 + code_lane * 20 + 16;
      return f32x4{r[0], r[1], r[2], r[3]};
    };
    if constexpr (kRing == 2) {  // both children staged together
      tile_put<float>(tile, pf);
      tile_put<float>(tile2, pf2);
      __syncthreads();
      if (base + stride < n) {
        tile_fetch<float>(x1, base + stride, n, pf);
        tile_fetch<float>(x2, base + stride, n, pf2);
      }
      product(AL, QL, P, Q, false, td);
      product(AR, QR, P, Q, true, td2);
      __syncthreads();
    } else if constexpr (T1) {
#pragma unroll
      for (int t = 0; t < 4; t++) tip_u(tabs[0], code1, t, P[t][0], P[t][1]);
      if constexpr (kQ) Q = tip_q(tabs[0], code1);
    } else {
      tile_put<float>(tile, pf);
      __syncthreads();
      // next: this trip's x2, or the next trip's x1 when x2 is a tip
      if constexpr (T2) {
        if (kAblate != 2 && base + stride < n) tile_fetch<float>(x1, base + stride, n, pf);
      } else if constexpr (kRing) {
        if (base + stride < n) tile_fetch<float>(x1, base + stride, n, pf);
      } else if constexpr (kAblate != 2) {
        tile_fetch<float>(x2, base, n, pf);
      }
      product(AL, QL, P, Q, false, td);
      __syncthreads();
    }
    if constexpr (kRing == 2) {
    } else if constexpr (T2) {
#pragma unroll
      for (int t = 0; t < 4; t++) {
        f32x4 u0, u1;
        tip_u(tabs[1], code2, t, u0, u1);
        P[t][0] = P[t][0] * u0;
        P[t][1] = P[t][1] * u1;
      }
      if constexpr (kQ) Q = Q * tip_q(tabs[1], code2);
    } else {
      if constexpr (kRing) {
        tile_put<float>(tile, pf2);
        __syncthreads();
        if (base + stride < n) tile_fetch<float>(x2, base + stride, n, pf2);
      } else {
        tile_put<float>(tile, pf);
        __syncthreads();
        if (kAblate != 2 && base + stride < n) tile_fetch<float>(T1 ? x2 : x1, base + stride, n, pf);
      }
      product(AR, QR, P, Q, true, td);
      __syncthreads();  // every wave is done reading x2: the tile takes X3 now
    }
    // kQ: lane group g gets p[16 + g] of sub-tile t's site lo16 as Qt[t]
    // (__float_as_uint: __builtin_bit_cast of a vector element reads element 0
    // with this compiler)
    unsigned Qt[4] = {__float_as_uint(Q[0]), __float_as_uint(Q[1]), __float_as_uint(Q[2]),
                      __float_as_uint(Q[3])};
    if constexpr (kQ) transpose_groups44(Qt);
    // kQ == 2: p[k][site lane] for k = 0..15 (four transposes of the P rows)
    unsigned pk[kQ == 2 ? 16 : 1];
    if constexpr (kQ == 2) {
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
    // back-transform: B fragment of k-step s = P[t][s >> 2][s & 3] (kQ: k-step 4 = Qt[t])
    unsigned long long mine = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      if constexpr (kAblate == 3) break;
      f32x4 X0 = {0.f, 0.f, 0.f, 0.f}, X1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const float b = (kQ && st == 4) ? __uint_as_float(Qt[t]) : P[t][st >> 2][st & 3];
        if constexpr (kAblate == 1) {
          X0[st & 3] += AE[0][st] * b;
          if constexpr (kQ != 2) X1[st & 3] += AE[1][st] * b;
          continue;
        }
        X0 = __builtin_amdgcn_mfma_f32_16x16x4f32(AE[0][st], b, X0, 0, 0, 0);
        if constexpr (kQ != 2) X1 = __builtin_amdgcn_mfma_f32_16x16x4f32(AE[1][st], b, X1, 0, 0, 0);
      }
      // lane group g holds states 4g..4g+3 (X0) and, for g = 0, 16..19 (X1)
      bool small = (__builtin_fabsf(X0[0]) < m) && (__builtin_fabsf(X0[1]) < m) &&
                   (__builtin_fabsf(X0[2]) < m) && (__builtin_fabsf(X0[3]) < m);
      if (kQ != 2 && g == 0)
        small = small && (__builtin_fabsf(X1[0]) < m) && (__builtin_fabsf(X1[1]) < m) &&
                (__builtin_fabsf(X1[2]) < m) && (__builtin_fabsf(X1[3]) < m);
      const unsigned long long b = __ballot(small);
      mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
      float *w = tw + (16 * t + lo16) * kRow + c * S;
      *reinterpret_cast<f32x4 *>(w + 4 * g) = X0;
      if (kQ != 2 && g == 0) *reinterpret_cast<f32x4 *>(w + 16) = X1;
    }
    if constexpr (kQ == 2 && kAblate != 3) {  // states 16..19 of site `lane`: 20 K = 1 steps, k ascending
      f32x4 X1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 20; k++) {
        const float a = reinterpret_cast<const f32x4 *>(QE)[k >> 2][k & 3];
        const float b = k < 16 ? __uint_as_float(pk[k & 15]) : Q[k & 3];
        if constexpr (kAblate == 1) X1[k & 3] += a * b;
        else X1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, X1, 0, 0, 0);
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
      if (kAblate == 2) {
        f32x4 t = v[0];
#pragma unroll
        for (int i = 1; i < K; i++) t += v[i];
        if (t.x == -1.25f) dst[threadIdx.x] = t;  // keeps the LDS reads alive
      } else if (base + 64 <= n) {
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
