// plf_dna.hpp -- device code of the fused DNA PLF kernels (instantiated by
// plf_kernels.hip; the tuning harnesses in tools/ include it too).
//
// Semantics: app/src/plf.cpp:19-65 (+ s2mm scaler byte,
// hls/src/s2mm_memDNAwindowComb.cpp:70-97, and the weighted scaler sum,
// app/src/host_mem.cpp:384-388).  See plf_kernels.hip for the mapping.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace plfx {
namespace dev {

constexpr int kBlock = 256;  // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename T>
struct Num;
template <>
struct Num<float> {
  __device__ static constexpr float two32() { return 4294967296.0f; }
  __device__ static constexpr float minlik() { return 2.3283064365386963e-10f; }  // 2^-32
  __device__ static inline float abs(float x) { return __builtin_fabsf(x); }
  template <bool NT>
  __device__ static inline void load4(const float *p, float (&v)[4]) {
    f32x4 a;
    if constexpr (NT) a = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    else a = *reinterpret_cast<const f32x4 *>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  __device__ static inline void store4_nt(float *p, const float (&v)[4]) {
    f32x4 a = {v[0], v[1], v[2], v[3]};
    __builtin_nontemporal_store(a, reinterpret_cast<f32x4 *>(p));
  }
};
template <>
struct Num<double> {
  __device__ static constexpr double two32() { return 4294967296.0; }
  __device__ static constexpr double minlik() { return 1.0 / 4294967296.0; }
  __device__ static inline double abs(double x) { return __builtin_fabs(x); }
  template <bool NT>
  __device__ static inline void load4(const double *p, double (&v)[4]) {
    f64x2 a, b;
    if constexpr (NT) {
      a = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(p));
      b = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(p) + 1);
    } else {
      a = reinterpret_cast<const f64x2 *>(p)[0];
      b = reinterpret_cast<const f64x2 *>(p)[1];
    }
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
  __device__ static inline void store4_nt(double *p, const double (&v)[4]) {
    f64x2 a = {v[0], v[1]};
    f64x2 b = {v[2], v[3]};
    __builtin_nontemporal_store(a, reinterpret_cast<f64x2 *>(p));
    __builtin_nontemporal_store(b, reinterpret_cast<f64x2 *>(p) + 1);
  }
};

// Cross-block sum without a memset launch and without a serialised fan-in.
// Workspace (kWsWords int64, zero at rest, restored to zero by the last
// arrivals): slot[s] at ws[s*16] (one 128-B line each, s = blockIdx % kSlots)
// and top at ws[kSlots*16].  Every add carries its own arrival count:
// word += kTick + partial, so after A arrivals word = A*kTick + sum and the
// count decodes as round(word / kTick) whenever |any partial sum| < kTick/2.
// Each block makes ONE returned atomic on its slot; the last arrival of a slot
// makes ONE returned atomic on top; the last arrival there knows the total.
// Two dependent round trips instead of a count+sum+acquire chain, and at most
// ceil(G/kSlots) arrivals serialise on a word (~12 ns each, MI355X_MICROARCH.md
// row fanin).  Precondition: sum |wgt| < 2^40 (the reference's own
// scalerIncrement is an int).
constexpr int kSlots = 32;
constexpr int kWsWords = (kSlots + 1) * 16;
constexpr long long kTick = 1ll << 41;

__device__ __forceinline__ long long decode_count(long long word) {
  return (word + (kTick >> 1)) >> 41;  // floor((word + kTick/2) / kTick)
}

// The two round trips for one block total `tot` (one thread).
// Site weight, loaded unconditionally: wgt == nullptr (all weights 1) reads a
// dummy word instead of branching round the load.  A load inside a branch got
// its value sign-extended inside the branch, i.e. an s_waitcnt vmcnt(0) right
// after it -- every CLV load of the trip issued so far had to land first.
__device__ __forceinline__ int wgt_at(const int32_t *wgt, int64_t site, const void *dummy) {
  const int32_t *p = wgt ? wgt + site : static_cast<const int32_t *>(dummy);
  const int v = __builtin_nontemporal_load(p);
  return wgt ? v : 1;
}

__device__ inline void ticket_publish(long long tot, unsigned long long *wsu, int64_t *out) {
  long long *ws = reinterpret_cast<long long *>(wsu);
  const long long G = gridDim.x;
  const long long slot = blockIdx.x % kSlots;
  const long long nslots = G < kSlots ? G : kSlots;
  const long long arrivals = (G - slot + kSlots - 1) / kSlots;
  const long long old = __hip_atomic_fetch_add(ws + slot * 16, kTick + tot, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
  if (decode_count(old) != arrivals - 1) return;
  const long long slot_sum = old + kTick + tot - arrivals * kTick;
  __hip_atomic_store(ws + slot * 16, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long told = __hip_atomic_fetch_add(ws + kSlots * 16, kTick + slot_sum, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
  if (decode_count(told) != nslots - 1) return;
  if (out) *out = (int64_t)(told + kTick + slot_sum - nslots * kTick);
  __hip_atomic_store(ws + kSlots * 16, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline void block_ticket_sum(long long v, unsigned long long *wsu, int64_t *out) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __shared__ long long part[kWavesPerBlock];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x != 0) return;
  long long tot = 0;
#pragma unroll
  for (int i = 0; i < kWavesPerBlock; i++) tot += part[i];
  ticket_publish(tot, wsu, out);
}

// Three independent sums (consecutive kWsWords regions of ws), published by
// threads 0..2 in parallel.
__device__ inline void block_ticket_sum3(long long v0, long long v1, long long v2,
                                         unsigned long long *wsu, int64_t *o0, int64_t *o1,
                                         int64_t *o2) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    v0 += __shfl_xor(v0, off);
    v1 += __shfl_xor(v1, off);
    v2 += __shfl_xor(v2, off);
  }
  __shared__ long long part3[3][kWavesPerBlock];
  if ((threadIdx.x & 63) == 0) {
    part3[0][threadIdx.x >> 6] = v0;
    part3[1][threadIdx.x >> 6] = v1;
    part3[2][threadIdx.x >> 6] = v2;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= 3) return;
  long long tot = 0;
#pragma unroll
  for (int i = 0; i < kWavesPerBlock; i++) tot += part3[t][i];
  ticket_publish(tot, wsu + (size_t)t * kWsWords, t == 0 ? o0 : (t == 1 ? o1 : o2));
}

// Swap 64-bit values between adjacent lanes with DPP quad_perm patterns:
// dpp_even(x) = x of lane (l & ~1), dpp_odd(x) = x of lane (l | 1).
// mov_dpp with bound_ctrl: every lane has a valid quad_perm source, so no
// "old" value is needed (update_dpp(0, ...) made the compiler zero the
// destination first: one extra v_mov_b32 per DPP move, ~15 % of the VALU
// issue of the headline kernel's loop).
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), kCtrl, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), kCtrl, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kQuadEven = 0 | (0 << 2) | (2 << 4) | (2 << 6);  // quad_perm [0,0,2,2]
constexpr int kQuadOdd = 1 | (1 << 2) | (3 << 4) | (3 << 6);   // quad_perm [1,1,3,3]

// Tip children: a tip is one DNA state code per site (bit s
// set = state s allowed, the RAxML/PLL convention); its dense CLV would be
// x[c][l] = tv[code][l] for every category c, with tv the tip-vector table
// (NULL: the 0/1 state indicator, bit l of the code; the eigen convention of
// plfx.h section 9 passes V^-1 applied to the indicator).  A block
// precomputes tab[c*64 + code*4 + k] = sum_l tv[code][l] * P_c[k][l] in plf()'s
// order from +0.0, so a tip's ump values are one LDS read and every result is
// bit-identical to running plf() on the expanded dense CLV.
template <typename T>
__device__ __forceinline__ void build_tip_table(const T *__restrict__ P, const T *__restrict__ tv,
                                                T *tab) {
  const int t = threadIdx.x;  // kBlock == 256 == 4 cats x 16 codes x 4 k
  const int cc = t >> 6, code = (t >> 2) & 15, k = t & 3;
  T v = T(0);
#pragma unroll
  for (int l = 0; l < 4; l++)
    v += (tv ? tv[code * 4 + l] : T((code >> l) & 1)) * P[cc * 16 + k * 4 + l];
  tab[t] = v;
}

// One site-category (4 values of x1, 4 of x2) -> 4 values of x3, before the
// scale test.  plf.cpp:31-50: ump from +0.0 ascending l, product per k, x3 from
// +0.0 ascending k.
//
// Leading +0.0 of the ump chains.  plf() sums ump = ((0 + q0) + q1) + ... ; here
// the chains start at q0.  The two differ only in the sign of a zero (0 + q0
// turns -0 into +0 and is the identity otherwise, NaN payloads included), and
// an ump value reaches x3 only through p = ump1*ump2 and the x3 chain, which
// DOES start at +0.0: (+0 + r) maps +0 and -0 to +0 and every later term of a
// chain that has reached +0 or a nonzero value ignores the sign of a zero
// term.  So x3, the scale test and the scaler bytes are bit-identical to
// plf()'s; the x3 chain keeps its +0.0.  (Saves 2 of the 14 f64 ops per
// site-category-k in the headline kernel; the GPU tests compare bit-for-bit.)
template <typename T>
__device__ __forceinline__ void site_cat(const T (&a)[4], const T (&b)[4], const T (&PL)[16],
                                         const T (&PR)[16], const T (&E)[16], T (&o)[4]) {
  T p[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    T u1 = a[0] * PL[k * 4], u2 = b[0] * PR[k * 4];  // chains start at q0 (see above)
#pragma unroll
    for (int l = 1; l < 4; l++) {
      u1 += a[l] * PL[k * 4 + l];
      u2 += b[l] * PR[k * 4 + l];
    }
    p[k] = u1 * u2;
  }
#pragma unroll
  for (int l = 0; l < 4; l++) o[l] = T(0);
#pragma unroll
  for (int k = 0; k < 4; k++) {
#pragma unroll
    for (int l = 0; l < 4; l++) o[l] += p[k] * E[4 * k + l];
  }
}

// site_cat with tip children: a tip's ump[k] comes from its table row.
template <typename T, bool T1, bool T2>
__device__ __forceinline__ void site_cat_tips(const T (&a)[4], const T (&b)[4], const T (&PL)[16],
                                              const T (&PR)[16], const T (&E)[16],
                                              const T *row1, const T *row2, T (&o)[4]) {
  T p[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    T u1, u2;
    if constexpr (T1) {
      u1 = row1[k];
    } else {
      u1 = a[0] * PL[k * 4];  // chains start at q0 (site_cat)
#pragma unroll
      for (int l = 1; l < 4; l++) u1 += a[l] * PL[k * 4 + l];
    }
    if constexpr (T2) {
      u2 = row2[k];
    } else {
      u2 = b[0] * PR[k * 4];
#pragma unroll
      for (int l = 1; l < 4; l++) u2 += b[l] * PR[k * 4 + l];
    }
    p[k] = u1 * u2;
  }
#pragma unroll
  for (int l = 0; l < 4; l++) o[l] = T(0);
#pragma unroll
  for (int k = 0; k < 4; k++) {
#pragma unroll
    for (int l = 0; l < 4; l++) o[l] += p[k] * E[4 * k + l];
  }
}

// Site -> wave mapping of the node kernels.  kSegL2 = 0: every wave strides
// over all n sites, so the whole chip works inside one window of each CLV.
// kSegL2 = 3: blocks b, b + 8, ... -- one XCD's blocks (blocks are dealt
// round-robin over the 8 XCDs, MI355X_MICROARCH.md) -- stride over the
// (b % 8)-th eighth of the sites only, eight windows far apart.  On very
// long CLVs the one-window pattern loses HBM rate (f32 0.59-0.62 of 8 TB/s at
// 1e8-5e8 sites against 0.70-0.75 at 2^20-2^22); eight windows recover it,
// but cost 6-8 % at 2^24 sites -- so the launchers pick the mapping by size
// (plf_kernels.hip segment_grid; tools/probes/size_scaling.hip,
// tools/max_sites.py --ab).  The grid must be a multiple of 2^kSegL2.
// Out: this wave's index within its segment, the stride, and its segment's
// first site and end (lo = 0, hi = n without segments).
template <int kSegL2, int kSitesPerStep>
__device__ __forceinline__ void wave_sites(int64_t n, int64_t &wave, int64_t &stride, int64_t &lo,
                                           int64_t &hi) {
  if constexpr (kSegL2 == 0) {
    wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    stride = (int64_t)gridDim.x * kWavesPerBlock * kSitesPerStep;
    lo = 0;
    hi = n;
  } else {
    constexpr int64_t S = 1 << kSegL2;
    wave = (int64_t)(blockIdx.x >> kSegL2) * kWavesPerBlock + (threadIdx.x >> 6);
    stride = (int64_t)(gridDim.x >> kSegL2) * kWavesPerBlock * kSitesPerStep;
    const int64_t steps = (n + kSitesPerStep - 1) / kSitesPerStep;
    const int64_t per = (steps + S - 1) / S * kSitesPerStep;  // sites per segment, whole steps
    lo = (int64_t)(blockIdx.x & (S - 1)) * per;
    hi = lo + per < n ? lo + per : n;
  }
}

// Knobs: U = 16-site wave steps per loop trip (bytes in flight per lane =
// 2*U*4*sizeof(T)); NT = non-temporal CLV loads; kSum = produce the weighted
// scaler sum; kMinWaves = __launch_bounds__ occupancy hint (waves per SIMD).
template <typename T, int U, bool kSum, bool NT, bool T1 = false, bool T2 = false, int kSegL2 = 0>
__device__ __forceinline__ void dna_cat_body(const T *__restrict__ x1, const T *__restrict__ x2,
                                             T *__restrict__ x3, const T *__restrict__ EV,
                                             const T *__restrict__ left, const T *__restrict__ right,
                                             const int32_t *__restrict__ wgt,
                                             uint8_t *__restrict__ scaler, int64_t n,
                                             unsigned long long *ws, int64_t *scaler_sum,
                                             const uint8_t *__restrict__ tip1 = nullptr,
                                             const uint8_t *__restrict__ tip2 = nullptr,
                                             const T *__restrict__ tipvec = nullptr) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 3;     // Gamma category owned by this lane
  const int q = lane >> 2;    // site slot within a 16-site wave step
  const int nib = lane & 60;  // bit offset of this site's nibble in the ballot
  __shared__ T tab1[T1 ? 256 : 1], tab2[T2 ? 256 : 1];
  if constexpr (T1) build_tip_table<T>(left, tipvec, tab1);
  if constexpr (T2) build_tip_table<T>(right, tipvec, tab2);
  if constexpr (T1 || T2) __syncthreads();

  T PL[16], PR[16], E[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    PL[i] = left[c * 16 + i];  // left[c*16 + k*4 + l]
    PR[i] = right[c * 16 + i];
    E[i] = EV[i];  // uniform: scalar loads
  }
  const T m = Num<T>::minlik();

  long long acc = 0;
  int64_t wave, stride, lo, hi;
  wave_sites<kSegL2, 16 * U>(n, wave, stride, lo, hi);
  const int64_t nfull = hi - (16 * U - 1);  // base < nfull  <=>  whole step in range

  int64_t base = lo + wave * 16 * U;
  // full steps: no bounds checks, every load of the step issued up front
  for (; base < nfull; base += stride) {
    T a[U][4], b[U][4];
    int w[U], k1[U], k2[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t site = base + u * 16 + q;
      if constexpr (T1) k1[u] = tip1[site] & 15;
      else Num<T>::template load4<NT>(x1 + site * 16 + c * 4, a[u]);
      if constexpr (T2) k2[u] = tip2[site] & 15;
      else Num<T>::template load4<NT>(x2 + site * 16 + c * 4, b[u]);
      if (kSum) w[u] = wgt_at(wgt, site, ws);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t site = base + u * 16 + q;
      T o[4];
      if constexpr (T1 || T2)
        site_cat_tips<T, T1, T2>(a[u], b[u], PL, PR, E, tab1 + c * 64 + 4 * (T1 ? k1[u] : 0),
                                 tab2 + c * 64 + 4 * (T2 ? k2[u] : 0), o);
      else
        site_cat<T>(a[u], b[u], PL, PR, E, o);
      const bool small = (Num<T>::abs(o[0]) < m) && (Num<T>::abs(o[1]) < m) &&
                         (Num<T>::abs(o[2]) < m) && (Num<T>::abs(o[3]) < m);
      const unsigned long long mask = __ballot(small);
      const bool sc = ((mask >> nib) & 0xFull) == 0xFull;
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const T s = o[l] * Num<T>::two32();  // exact: power-of-two scaling
        o[l] = sc ? s : o[l];
      }
      Num<T>::store4_nt(x3 + site * 16 + c * 4, o);
      if (c == 0) {
        if (scaler) scaler[site] = (uint8_t)sc;
      }
      if (kSum) acc += (c == 0 && sc) ? (long long)w[u] : 0ll;
    }
  }
  // tail (at most one partial step per wave)
  if (base < hi) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t site = base + u * 16 + q;
      const bool valid = site < hi;
      T a[4] = {T(0), T(0), T(0), T(0)}, b[4] = {T(0), T(0), T(0), T(0)};
      int k1 = 0, k2 = 0;
      if (valid) {
        if constexpr (T1) k1 = tip1[site] & 15;
        else Num<T>::template load4<false>(x1 + site * 16 + c * 4, a);
        if constexpr (T2) k2 = tip2[site] & 15;
        else Num<T>::template load4<false>(x2 + site * 16 + c * 4, b);
      }
      T o[4];
      if constexpr (T1 || T2)
        site_cat_tips<T, T1, T2>(a, b, PL, PR, E, tab1 + c * 64 + 4 * k1, tab2 + c * 64 + 4 * k2, o);
      else
        site_cat<T>(a, b, PL, PR, E, o);
      const bool small = valid && (Num<T>::abs(o[0]) < m) && (Num<T>::abs(o[1]) < m) &&
                         (Num<T>::abs(o[2]) < m) && (Num<T>::abs(o[3]) < m);
      const unsigned long long mask = __ballot(small);
      const bool sc = ((mask >> nib) & 0xFull) == 0xFull;
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const T s = o[l] * Num<T>::two32();
        o[l] = sc ? s : o[l];
      }
      if (valid) {
        Num<T>::store4_nt(x3 + site * 16 + c * 4, o);
        if (c == 0) {
          if (scaler) scaler[site] = (uint8_t)sc;
          if (kSum && sc) acc += wgt ? (long long)wgt[site] : 1ll;
        }
      }
    }
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

template <typename T, int U, bool kSum, bool NT, int kMinWaves, int kSegL2 = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
               const T *__restrict__ EV, const T *__restrict__ left,
               const T *__restrict__ right, const int32_t *__restrict__ wgt,
               uint8_t *__restrict__ scaler, int64_t n, unsigned long long *ws,
               int64_t *scaler_sum) {
  dna_cat_body<T, U, kSum, NT, false, false, kSegL2>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws,
                                                     scaler_sum);
}

// f64 DNA kernel, lane-pair mapping: every wave memory instruction touches one
// contiguous 1 KiB (lane l <-> bytes 16l..16l+15 of an 8-site block), i.e. lane
// l holds states {2h, 2h+1} (h = l&1) of category c = (l>>1)&3 of site l>>3.
// The two lanes of a pair rebuild the category's 4 states with DPP, each
// computes ump/prod for two of the four k (k = 2h, 2h+1), the pair swaps the
// products with DPP, and each lane produces its two output states -- every
// value with exactly plf()'s operation order (ascending l, then ascending k,
// from +0.0).  Per site: 16 lanes x 16 B per child, 8 lanes per site, the
// site's 16-value scale test is one byte of the wave ballot.
template <bool NT>
__device__ __forceinline__ f64x2 ld16(const f64x2 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// T1/T2: child 1/2 is a tip (one state code per site, see build_tip_table);
// its lane pair reads ump[2h], ump[2h+1] as one 16-B LDS row slice.
template <int U, bool kSum, bool NTL, bool T1 = false, bool T2 = false, int kSegL2 = 0>
__device__ __forceinline__ void dna_pair_body(const double *__restrict__ x1,
                                              const double *__restrict__ x2,
                                              double *__restrict__ x3,
                                              const double *__restrict__ EV,
                                              const double *__restrict__ left,
                                              const double *__restrict__ right,
                                              const int32_t *__restrict__ wgt,
                                              uint8_t *__restrict__ scaler, int64_t n,
                                              unsigned long long *ws, int64_t *scaler_sum,
                                              const uint8_t *__restrict__ tip1 = nullptr,
                                              const uint8_t *__restrict__ tip2 = nullptr,
                                              const double *__restrict__ tipvec = nullptr) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 1;          // which half of the category's states / k range
  const int c = (lane >> 1) & 3;   // Gamma category
  const int g = lane >> 3;         // site within the 8-site block of one instruction
  const int sh = lane & 56;        // bit offset of this site's byte in the ballot
  __shared__ double tab1[T1 ? 256 : 1], tab2[T2 ? 256 : 1];
  if constexpr (T1) build_tip_table<double>(left, tipvec, tab1);
  if constexpr (T2) build_tip_table<double>(right, tipvec, tab2);
  if constexpr (T1 || T2) __syncthreads();
  const int trow = c * 64 + 2 * h;  // + 4*code: this lane's slice of a table row

  double PL[2][4], PR[2][4], E[4][2];
#pragma unroll
  for (int kk = 0; kk < 2; kk++)
#pragma unroll
    for (int l = 0; l < 4; l++) {
      PL[kk][l] = left[c * 16 + (2 * h + kk) * 4 + l];
      PR[kk][l] = right[c * 16 + (2 * h + kk) * 4 + l];
    }
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int t = 0; t < 2; t++) E[k][t] = EV[4 * k + 2 * h + t];
  const double m = Num<double>::minlik();

  long long acc = 0;
  int64_t wave, stride, lo, hi;
  wave_sites<kSegL2, 16 * U>(n, wave, stride, lo, hi);
  const int64_t nfull = hi - (16 * U - 1);

  // one 8-site block: loads are done by the caller
  auto body = [&](const f64x2 a, const f64x2 b, int k1, int k2, int64_t site0, bool valid,
                  int w) {
    double u1[2], u2[2];
    if constexpr (T1) {
      const f64x2 r = *reinterpret_cast<const f64x2 *>(tab1 + trow + 4 * k1);
      u1[0] = r.x; u1[1] = r.y;
    } else {
      // rebuild the 4 states of x1_c in every lane of the pair
      const double a0 = dpp_f64<kQuadEven>(a.x), a1 = dpp_f64<kQuadEven>(a.y);
      const double a2 = dpp_f64<kQuadOdd>(a.x), a3 = dpp_f64<kQuadOdd>(a.y);
#pragma unroll
      for (int kk = 0; kk < 2; kk++) {
        double v = a0 * PL[kk][0];  // chain starts at q0 (site_cat)
        v += a1 * PL[kk][1]; v += a2 * PL[kk][2]; v += a3 * PL[kk][3];
        u1[kk] = v;
      }
    }
    if constexpr (T2) {
      const f64x2 r = *reinterpret_cast<const f64x2 *>(tab2 + trow + 4 * k2);
      u2[0] = r.x; u2[1] = r.y;
    } else {
      const double b0 = dpp_f64<kQuadEven>(b.x), b1 = dpp_f64<kQuadEven>(b.y);
      const double b2 = dpp_f64<kQuadOdd>(b.x), b3 = dpp_f64<kQuadOdd>(b.y);
#pragma unroll
      for (int kk = 0; kk < 2; kk++) {
        double v = b0 * PR[kk][0];  // chain starts at q0 (site_cat)
        v += b1 * PR[kk][1]; v += b2 * PR[kk][2]; v += b3 * PR[kk][3];
        u2[kk] = v;
      }
    }
    double pm[2];
#pragma unroll
    for (int kk = 0; kk < 2; kk++) pm[kk] = u1[kk] * u2[kk];
    const double p0 = dpp_f64<kQuadEven>(pm[0]), p1 = dpp_f64<kQuadEven>(pm[1]);
    const double p2 = dpp_f64<kQuadOdd>(pm[0]), p3 = dpp_f64<kQuadOdd>(pm[1]);
    double o[2];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      double x = 0.0;
      x += p0 * E[0][t]; x += p1 * E[1][t]; x += p2 * E[2][t]; x += p3 * E[3][t];
      o[t] = x;
    }
    const bool small = valid && (__builtin_fabs(o[0]) < m) && (__builtin_fabs(o[1]) < m);
    const unsigned long long mask = __ballot(small);
    const bool sc = ((mask >> sh) & 0xFFull) == 0xFFull;
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const double s = o[t] * Num<double>::two32();
      o[t] = sc ? s : o[t];
    }
    if (valid) {
      f64x2 ov = {o[0], o[1]};
      __builtin_nontemporal_store(ov, reinterpret_cast<f64x2 *>(x3 + site0 * 16) + lane);
      if ((lane & 7) == 0 && scaler) scaler[site0 + g] = (uint8_t)sc;
      if ((lane & 7) == 0) {
        if (kSum && sc) acc += w;
      }
    }
  };

  int64_t base = lo + wave * 16 * U;
  for (; base < nfull; base += stride) {
    f64x2 a[U][2], b[U][2];
    int w[U][2], k1[U][2], k2[U][2];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int64_t site0 = base + u * 16 + j * 8;
        if constexpr (T1) k1[u][j] = tip1[site0 + g] & 15;
        else a[u][j] = ld16<NTL>(reinterpret_cast<const f64x2 *>(x1 + site0 * 16) + lane);
        if constexpr (T2) k2[u][j] = tip2[site0 + g] & 15;
        else b[u][j] = ld16<NTL>(reinterpret_cast<const f64x2 *>(x2 + site0 * 16) + lane);
        if (kSum) w[u][j] = wgt ? wgt[site0 + g] : 1;  // (wgt_at measured 1.6 % slower here)
      }
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < 2; j++)
        body(T1 ? f64x2{} : a[u][j], T2 ? f64x2{} : b[u][j], T1 ? k1[u][j] : 0,
             T2 ? k2[u][j] : 0, base + u * 16 + j * 8, true, kSum ? w[u][j] : 0);
  }
  if (base < hi) {  // tail: at most one partial step per wave
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int64_t site0 = base + u * 16 + j * 8;
        const bool valid = site0 + g < hi;
        f64x2 a = {0.0, 0.0}, b = {0.0, 0.0};
        int w = 0, k1 = 0, k2 = 0;
        if (valid) {
          if constexpr (T1) k1 = tip1[site0 + g] & 15;
          else a = reinterpret_cast<const f64x2 *>(x1 + site0 * 16)[lane];
          if constexpr (T2) k2 = tip2[site0 + g] & 15;
          else b = reinterpret_cast<const f64x2 *>(x2 + site0 * 16)[lane];
          if (kSum) w = wgt ? wgt[site0 + g] : 1;
        }
        body(a, b, k1, k2, site0, valid, w);
      }
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

template <int U, bool kSum, int kMinWaves, bool NTL = false, int kSegL2 = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_f64_pair_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                        double *__restrict__ x3, const double *__restrict__ EV,
                        const double *__restrict__ left, const double *__restrict__ right,
                        const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                        unsigned long long *ws, int64_t *scaler_sum) {
  dna_pair_body<U, kSum, NTL, false, false, kSegL2>(x1, x2, x3, EV, left, right, wgt, scaler, n, ws,
                                                   scaler_sum);
}

// Batched inner-node updates: one launch evaluates gridDim.y <= kMaxBatch
// independent nodes (a tree level, or a shard of independent nodes) that share
// EV, n and wgt; node = blockIdx.y.  The descriptors travel by value in the
// kernel arguments (no staging copy, graph-capture safe) and are read through
// the scalar cache.  Each node has its own kWsWords of scaler-sum workspace.
struct NodeDesc {
  const void *x1, *x2;
  void *x3;
  const void *left, *right;
  uint8_t *scaler;      // may be null
  int64_t *scaler_sum;  // may be null
};
constexpr int kMaxBatch = 32;
struct NodeBatch {
  NodeDesc d[kMaxBatch];
};

// kTips: 0 = both children dense CLVs, 1 = child 1 is a tip (x1 points at its
// state codes), 2 = both children are tips.  (A dense/tip node is run as
// tip/dense with the children swapped: u1*u2 == u2*u1 exactly.)
template <int U, bool kSum, int kMinWaves, bool NTL = false, int kTips = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_f64_pair_batch_kernel(const NodeBatch nodes, const double *__restrict__ EV,
                              const int32_t *__restrict__ wgt, int64_t n,
                              unsigned long long *ws, const double *__restrict__ tipvec) {
  const NodeDesc &d = nodes.d[blockIdx.y];
  dna_pair_body<U, kSum, NTL, (kTips >= 1), (kTips == 2)>(
      (const double *)d.x1, (const double *)d.x2, (double *)d.x3, EV, (const double *)d.left,
      (const double *)d.right, wgt, d.scaler, n, ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum,
      (const uint8_t *)d.x1, (const uint8_t *)d.x2, tipvec);
}

template <typename T, int U, bool kSum, bool NT, int kMinWaves, int kTips = 0>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_batch_kernel(const NodeBatch nodes, const T *__restrict__ EV,
                     const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                     const T *__restrict__ tipvec) {
  const NodeDesc &d = nodes.d[blockIdx.y];
  dna_cat_body<T, U, kSum, NT, (kTips >= 1), (kTips == 2)>(
      (const T *)d.x1, (const T *)d.x2, (T *)d.x3, EV, (const T *)d.left, (const T *)d.right, wgt,
      d.scaler, n, ws + (size_t)blockIdx.y * kWsWords, d.scaler_sum, (const uint8_t *)d.x1,
      (const uint8_t *)d.x2, tipvec);
}

#ifndef PLFX_SECONDARY_TU  // the one non-template kernel: defined in plf_kernels.hip only
__global__ void __launch_bounds__(kBlock)
scaler_sum_kernel(const uint8_t *__restrict__ scaler, const int32_t *__restrict__ wgt, int64_t n,
                  unsigned long long *ws, int64_t *out) {
  long long acc = 0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride)
    acc += (long long)scaler[j] * (wgt ? (long long)wgt[j] : 1ll);
  block_ticket_sum(acc, ws, out);
}
#endif

// ---------------------------------------------------------------------------
// Fused level pair ("triple"): parent P of two inner nodes A, B that are
// computed in the same pass -- A from (a1, a2), B from (b1, b2), then P from
// (A, B) -- so the two intermediate CLVs are written once and never read back
// (per site and f64: 4 child reads + 3 writes = 896 B instead of 3 x 384).
// The lane-pair layout of a node's output (states 2h, 2h+1 of category c of
// site g) is exactly the layout the next node's body reads, so A and B feed P
// from registers.  Every node keeps plf()'s arithmetic, scale test, scaler
// byte and weighted scaler sum: results are bit-identical to three separate
// updates.  kTips: 0 = a1, a2, b1, b2 dense; 1 = a1 and b1 are tips (a2, b2
// dense); 2 = all four are tips.
struct TripleDesc {
  const void *a1, *a2, *b1, *b2;
  void *xa, *xb, *xp;
  const double *la, *ra, *lb, *rb, *lp, *rp;
  uint8_t *sa, *sb, *sp;
  int64_t *ssa, *ssb, *ssp;
};
constexpr int kMaxTriples = 10;
struct TripleBatch {
  TripleDesc d[kMaxTriples];
};

struct PairMats {
  double PL[2][4], PR[2][4];
};

__device__ __forceinline__ void pair_mats(const double *__restrict__ left,
                                          const double *__restrict__ right, int c, int h,
                                          PairMats &M) {
#pragma unroll
  for (int kk = 0; kk < 2; kk++)
#pragma unroll
    for (int l = 0; l < 4; l++) {
      M.PL[kk][l] = left[c * 16 + (2 * h + kk) * 4 + l];
      M.PR[kk][l] = right[c * 16 + (2 * h + kk) * 4 + l];
    }
}

// One node on one 8-site block in the lane-pair layout (dna_pair_body's body):
// returns the (possibly rescaled) output pair and the site's scale flag.
template <bool TL, bool TR>
__device__ __forceinline__ f64x2 pair_node(const f64x2 a, const f64x2 b, const double *rowL,
                                           const double *rowR, const PairMats &M,
                                           const double (&E)[4][2], bool valid, int sh,
                                           double m, bool &sc) {
  double u1[2], u2[2];
  if constexpr (TL) {
    const f64x2 r = *reinterpret_cast<const f64x2 *>(rowL);
    u1[0] = r.x; u1[1] = r.y;
  } else {
    const double a0 = dpp_f64<kQuadEven>(a.x), a1 = dpp_f64<kQuadEven>(a.y);
    const double a2 = dpp_f64<kQuadOdd>(a.x), a3 = dpp_f64<kQuadOdd>(a.y);
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      double v = a0 * M.PL[kk][0];  // chain starts at q0 (site_cat)
      v += a1 * M.PL[kk][1]; v += a2 * M.PL[kk][2]; v += a3 * M.PL[kk][3];
      u1[kk] = v;
    }
  }
  if constexpr (TR) {
    const f64x2 r = *reinterpret_cast<const f64x2 *>(rowR);
    u2[0] = r.x; u2[1] = r.y;
  } else {
    const double b0 = dpp_f64<kQuadEven>(b.x), b1 = dpp_f64<kQuadEven>(b.y);
    const double b2 = dpp_f64<kQuadOdd>(b.x), b3 = dpp_f64<kQuadOdd>(b.y);
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      double v = b0 * M.PR[kk][0];  // chain starts at q0 (site_cat)
      v += b1 * M.PR[kk][1]; v += b2 * M.PR[kk][2]; v += b3 * M.PR[kk][3];
      u2[kk] = v;
    }
  }
  double pm[2];
#pragma unroll
  for (int kk = 0; kk < 2; kk++) pm[kk] = u1[kk] * u2[kk];
  const double p0 = dpp_f64<kQuadEven>(pm[0]), p1 = dpp_f64<kQuadEven>(pm[1]);
  const double p2 = dpp_f64<kQuadOdd>(pm[0]), p3 = dpp_f64<kQuadOdd>(pm[1]);
  double o[2];
#pragma unroll
  for (int t = 0; t < 2; t++) {
    double x = 0.0;
    x += p0 * E[0][t]; x += p1 * E[1][t]; x += p2 * E[2][t]; x += p3 * E[3][t];
    o[t] = x;
  }
  const bool small = valid && (__builtin_fabs(o[0]) < m) && (__builtin_fabs(o[1]) < m);
  const unsigned long long mask = __ballot(small);
  sc = ((mask >> sh) & 0xFFull) == 0xFFull;
#pragma unroll
  for (int t = 0; t < 2; t++) {
    const double s = o[t] * Num<double>::two32();
    o[t] = sc ? s : o[t];
  }
  return f64x2{o[0], o[1]};
}

template <bool kSum, int kMinWaves, bool NTL, int kTips, int U = 1>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_f64_triple_kernel(const TripleBatch tb, const double *__restrict__ EV,
                          const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                          const double *__restrict__ tipvec) {
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  const TripleDesc &d = tb.d[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int h = lane & 1, c = (lane >> 1) & 3, g = lane >> 3, sh = lane & 56;
  // tip tables: [0] A's left, [1] B's left, [2] A's right, [3] B's right
  __shared__ double tab[T2 ? 4 : (T1 ? 2 : 1)][T1 ? 256 : 1];
  if constexpr (T1) {
    build_tip_table<double>(d.la, tipvec, tab[0]);
    build_tip_table<double>(d.lb, tipvec, tab[1]);
  }
  if constexpr (T2) {
    build_tip_table<double>(d.ra, tipvec, tab[2]);
    build_tip_table<double>(d.rb, tipvec, tab[3]);
  }
  if constexpr (T1) __syncthreads();
  const int trow = c * 64 + 2 * h;
  PairMats MA, MB, MP;
  pair_mats(d.la, d.ra, c, h, MA);
  pair_mats(d.lb, d.rb, c, h, MB);
  pair_mats(d.lp, d.rp, c, h, MP);
  double E[4][2];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int t = 0; t < 2; t++) E[k][t] = EV[4 * k + 2 * h + t];
  const double m = Num<double>::minlik();
  const uint8_t *ta1 = (const uint8_t *)d.a1, *ta2 = (const uint8_t *)d.a2;
  const uint8_t *tb1 = (const uint8_t *)d.b1, *tb2 = (const uint8_t *)d.b2;
  const double *xa1 = (const double *)d.a1, *xa2 = (const double *)d.a2;
  const double *xb1 = (const double *)d.b1, *xb2 = (const double *)d.b2;
  double *xa = (double *)d.xa, *xb = (double *)d.xb, *xp = (double *)d.xp;

  long long accA = 0, accB = 0, accP = 0;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 16 * U;
  for (int64_t base = wave * 16 * U; base < n; base += stride) {
    f64x2 va1[2 * U], va2[2 * U], vb1[2 * U], vb2[2 * U];
    int ka1[2 * U], ka2[2 * U], kb1[2 * U], kb2[2 * U], w[2 * U];
    bool valid[2 * U];
#pragma unroll
    for (int j = 0; j < 2 * U; j++) {  // all loads of the 16*U sites first
      const int64_t site0 = base + j * 8;
      valid[j] = site0 + g < n;
      // past n: reload the last site (unconditional loads, no wait-all; results unused)
      const int64_t sq = valid[j] ? site0 + g : n - 1;
      const int64_t rec = sq * 8 + (lane & 7);  // f64x2 index of this lane's pair (8 per site)
      va1[j] = va2[j] = vb1[j] = vb2[j] = f64x2{0.0, 0.0};
      ka1[j] = ka2[j] = kb1[j] = kb2[j] = 0;
      w[j] = 0;
      if constexpr (T1) {
        ka1[j] = ta1[sq] & 15;
        kb1[j] = tb1[sq] & 15;
      } else {
        va1[j] = ld16<NTL>(reinterpret_cast<const f64x2 *>(xa1) + rec);
        vb1[j] = ld16<NTL>(reinterpret_cast<const f64x2 *>(xb1) + rec);
      }
      if constexpr (T2) {
        ka2[j] = ta2[sq] & 15;
        kb2[j] = tb2[sq] & 15;
      } else {
        va2[j] = ld16<NTL>(reinterpret_cast<const f64x2 *>(xa2) + rec);
        vb2[j] = ld16<NTL>(reinterpret_cast<const f64x2 *>(xb2) + rec);
      }
      if (kSum) w[j] = wgt_at(wgt, sq, ws);
    }
#pragma unroll
    for (int j = 0; j < 2 * U; j++) {
      const int64_t site0 = base + j * 8;
      const int64_t rec = site0 * 8 + lane;
      bool sA, sB, sP;
      const f64x2 oA = pair_node<T1, T2>(va1[j], va2[j], tab[0] + trow + 4 * ka1[j],
                                         tab[T2 ? 2 : 0] + trow + 4 * ka2[j], MA, E, valid[j], sh,
                                         m, sA);
      const f64x2 oB = pair_node<T1, T2>(vb1[j], vb2[j], tab[T1 ? 1 : 0] + trow + 4 * kb1[j],
                                         tab[T2 ? 3 : 0] + trow + 4 * kb2[j], MB, E, valid[j], sh,
                                         m, sB);
      const f64x2 oP = pair_node<false, false>(oA, oB, nullptr, nullptr, MP, E, valid[j], sh, m, sP);
      if (valid[j]) {
        __builtin_nontemporal_store(oA, reinterpret_cast<f64x2 *>(xa) + rec);
        __builtin_nontemporal_store(oB, reinterpret_cast<f64x2 *>(xb) + rec);
        __builtin_nontemporal_store(oP, reinterpret_cast<f64x2 *>(xp) + rec);
        if ((lane & 7) == 0) {
          if (d.sa) d.sa[site0 + g] = (uint8_t)sA;
          if (d.sb) d.sb[site0 + g] = (uint8_t)sB;
          if (d.sp) d.sp[site0 + g] = (uint8_t)sP;
          if (kSum) {
            if (sA) accA += w[j];
            if (sB) accB += w[j];
            if (sP) accP += w[j];
          }
        }
      }
    }
  }
  if constexpr (kSum)
    block_ticket_sum3(accA, accB, accP, ws + (size_t)blockIdx.y * 3 * kWsWords, d.ssa, d.ssb,
                      d.ssp);
}

// Fused level pair in the lane = category mapping (f32): a node's output
// (category c of site q, 4 states) is again exactly the next node's input.
template <typename T, bool TL, bool TR>
__device__ __forceinline__ void cat_node(const T (&a)[4], const T (&b)[4], const T *rowL,
                                         const T *rowR, const T (&PL)[16], const T (&PR)[16],
                                         const T (&E)[16], bool valid, int nib, T m, T (&o)[4],
                                         bool &sc) {
  if constexpr (TL || TR) site_cat_tips<T, TL, TR>(a, b, PL, PR, E, rowL, rowR, o);
  else site_cat<T>(a, b, PL, PR, E, o);
  const bool small = valid && (Num<T>::abs(o[0]) < m) && (Num<T>::abs(o[1]) < m) &&
                     (Num<T>::abs(o[2]) < m) && (Num<T>::abs(o[3]) < m);
  const unsigned long long mask = __ballot(small);
  sc = ((mask >> nib) & 0xFull) == 0xFull;
#pragma unroll
  for (int l = 0; l < 4; l++) {
    const T s = o[l] * Num<T>::two32();
    o[l] = sc ? s : o[l];
  }
}

template <typename T, bool kSum, int kMinWaves, bool NT, int kTips, int U = 1>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_cat_triple_kernel(const TripleBatch tb, const T *__restrict__ EV,
                          const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                          const T *__restrict__ tipvec) {
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  const TripleDesc &d = tb.d[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int c = lane & 3, q = lane >> 2, nib = lane & 60;
  __shared__ T tab[T2 ? 4 : (T1 ? 2 : 1)][T1 ? 256 : 1];
  const T *la = (const T *)d.la, *ra = (const T *)d.ra, *lb = (const T *)d.lb;
  const T *rb = (const T *)d.rb, *lp = (const T *)d.lp, *rp = (const T *)d.rp;
  if constexpr (T1) {
    build_tip_table<T>(la, tipvec, tab[0]);
    build_tip_table<T>(lb, tipvec, tab[1]);
  }
  if constexpr (T2) {
    build_tip_table<T>(ra, tipvec, tab[2]);
    build_tip_table<T>(rb, tipvec, tab[3]);
  }
  if constexpr (T1) __syncthreads();
  T LA[16], RA[16], LB[16], RB[16], LP[16], RP[16], E[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    LA[i] = la[c * 16 + i]; RA[i] = ra[c * 16 + i];
    LB[i] = lb[c * 16 + i]; RB[i] = rb[c * 16 + i];
    LP[i] = lp[c * 16 + i]; RP[i] = rp[c * 16 + i];
    E[i] = EV[i];
  }
  const T m = Num<T>::minlik();
  const uint8_t *ta1 = (const uint8_t *)d.a1, *ta2 = (const uint8_t *)d.a2;
  const uint8_t *tb1 = (const uint8_t *)d.b1, *tb2 = (const uint8_t *)d.b2;
  const T *xa1 = (const T *)d.a1, *xa2 = (const T *)d.a2;
  const T *xb1 = (const T *)d.b1, *xb2 = (const T *)d.b2;
  T *xa = (T *)d.xa, *xb = (T *)d.xb, *xp = (T *)d.xp;
  const int trow = c * 64;

  long long accA = 0, accB = 0, accP = 0;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 16 * U;
  for (int64_t base = wave * 16 * U; base < n; base += stride) {
    T va1[U][4], va2[U][4], vb1[U][4], vb2[U][4];
    int ka1[U], ka2[U], kb1[U], kb2[U], w[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t site = base + u * 16 + q;
      valid[u] = site < n;
      const int64_t sq = valid[u] ? site : n - 1;  // past n: reload the last site (unused)
      ka1[u] = ka2[u] = kb1[u] = kb2[u] = w[u] = 0;
#pragma unroll
      for (int l = 0; l < 4; l++) va1[u][l] = va2[u][l] = vb1[u][l] = vb2[u][l] = T(0);
      const int64_t off = sq * 16 + c * 4;
      if constexpr (T1) {
        ka1[u] = ta1[sq] & 15;
        kb1[u] = tb1[sq] & 15;
      } else {
        Num<T>::template load4<NT>(xa1 + off, va1[u]);
        Num<T>::template load4<NT>(xb1 + off, vb1[u]);
      }
      if constexpr (T2) {
        ka2[u] = ta2[sq] & 15;
        kb2[u] = tb2[sq] & 15;
      } else {
        Num<T>::template load4<NT>(xa2 + off, va2[u]);
        Num<T>::template load4<NT>(xb2 + off, vb2[u]);
      }
      if (kSum) w[u] = wgt_at(wgt, sq, ws);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t site = base + u * 16 + q;
      const int64_t off = site * 16 + c * 4;
      T oA[4], oB[4], oP[4];
      bool sA, sB, sP;
      cat_node<T, T1, T2>(va1[u], va2[u], tab[0] + trow + 4 * ka1[u],
                          tab[T2 ? 2 : 0] + trow + 4 * ka2[u], LA, RA, E, valid[u], nib, m, oA, sA);
      cat_node<T, T1, T2>(vb1[u], vb2[u], tab[T1 ? 1 : 0] + trow + 4 * kb1[u],
                          tab[T2 ? 3 : 0] + trow + 4 * kb2[u], LB, RB, E, valid[u], nib, m, oB, sB);
      cat_node<T, false, false>(oA, oB, nullptr, nullptr, LP, RP, E, valid[u], nib, m, oP, sP);
      if (valid[u]) {
        Num<T>::store4_nt(xa + off, oA);
        Num<T>::store4_nt(xb + off, oB);
        Num<T>::store4_nt(xp + off, oP);
        if (c == 0) {
          if (d.sa) d.sa[site] = (uint8_t)sA;
          if (d.sb) d.sb[site] = (uint8_t)sB;
          if (d.sp) d.sp[site] = (uint8_t)sP;
          if (kSum) {
            if (sA) accA += w[u];
            if (sB) accB += w[u];
            if (sP) accP += w[u];
          }
        }
      }
    }
  }
  if constexpr (kSum)
    block_ticket_sum3(accA, accB, accP, ws + (size_t)blockIdx.y * 3 * kWsWords, d.ssa, d.ssb,
                      d.ssp);
}

// ---------------------------------------------------------------------------
// Fused three-level subtree ("septet", f64 lane-pair mapping): four nodes A_i
// over eight children g, their two parents B_1 = (A_1, A_2), B_2 = (A_3, A_4)
// and the root R = (B_1, B_2) in one pass: 8 child reads + 7 writes per site
// (15 CLV transfers for 7 nodes, 2.14 per node; a triple moves 7 for 3).  The
// 7 nodes' matrices (128 values each) sit in LDS and every lane reads its 16
// per node just in time (registers could not hold 7 x 16 doubles).  Results
// are bit-identical to seven separate updates.  kTips as the triple kernel,
// for the A level: 1 = g_1, g_3, g_5, g_7 tips; 2 = all eight.
struct SeptetDesc {
  const void *g[8];
  void *x[7];               // A1..A4, B1, B2, R
  const void *mat[14];      // left, right of A1..A4, B1, B2, R (element type T)
  uint8_t *sc[7];
  int64_t *ss[7];
};
constexpr int kMaxSeptets = 8;
struct SeptetBatch {
  SeptetDesc d[kMaxSeptets];
};

// the lane's P rows of one node from its LDS image (left 64 | right 64)
__device__ __forceinline__ void pair_mats_lds(const double *m, int c, int h, PairMats &M) {
  const f64x2 *L = reinterpret_cast<const f64x2 *>(m + c * 16 + 8 * h);
  const f64x2 *R = reinterpret_cast<const f64x2 *>(m + 64 + c * 16 + 8 * h);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const f64x2 a = L[i], b = R[i];
    M.PL[i >> 1][2 * (i & 1)] = a.x;
    M.PL[i >> 1][2 * (i & 1) + 1] = a.y;
    M.PR[i >> 1][2 * (i & 1)] = b.x;
    M.PR[i >> 1][2 * (i & 1) + 1] = b.y;
  }
}

__device__ inline void block_ticket_sum7(const long long (&v)[7], unsigned long long *wsu,
                                         int64_t *const (&out)[7]) {
  __shared__ long long part7[7][kWavesPerBlock];
#pragma unroll
  for (int q = 0; q < 7; q++) {
    long long x = v[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if ((threadIdx.x & 63) == 0) part7[q][threadIdx.x >> 6] = x;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= 7) return;
  long long tot = 0;
#pragma unroll
  for (int i = 0; i < kWavesPerBlock; i++) tot += part7[t][i];
  ticket_publish(tot, wsu + (size_t)t * kWsWords, out[t]);
}

// The matrices are re-read from LDS on every trip (an opaque zero offset
// stops the compiler hoisting the 224 loop-invariant values into registers),
// trading LDS traffic for occupancy.  U: 8-site blocks per trip (one matrix
// read serves all U).  kPf: issue the next trip's loads before this trip's
// arithmetic (software pipelining; twice the input registers).
template <bool kSum, int kMinWaves, bool NTL, int kTips, int U = 1, bool kPf = false>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_f64_septet_kernel(const SeptetBatch sb, const double *__restrict__ EV,
                          const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                          const double *__restrict__ tipvec) {
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  const SeptetDesc &d = sb.d[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int h = lane & 1, c = (lane >> 1) & 3, g = lane >> 3, sh = lane & 56;
  __shared__ double mats[7][128];
  // tip tables: [i] = A_i's left (g_{2i-1}), [4 + i] = A_i's right (g_{2i})
  __shared__ double tab[T2 ? 8 : (T1 ? 4 : 1)][T1 ? 256 : 1];
  for (int e = threadIdx.x; e < 7 * 128; e += kBlock) {
    const int node = e >> 7, k = e & 127;
    mats[node][k] = static_cast<const double *>(d.mat[2 * node + (k >> 6)])[k & 63];
  }
  if constexpr (T1) {
#pragma unroll
    for (int i = 0; i < 4; i++) build_tip_table<double>((const double *)d.mat[2 * i], tipvec, tab[i]);
  }
  if constexpr (T2) {
#pragma unroll
    for (int i = 0; i < 4; i++) build_tip_table<double>((const double *)d.mat[2 * i + 1], tipvec, tab[4 + i]);
  }
  __syncthreads();
  const int trow = c * 64 + 2 * h;
  double E[4][2];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int t = 0; t < 2; t++) E[k][t] = EV[4 * k + 2 * h + t];
  const double m = Num<double>::minlik();

  long long acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 8 * U;
  struct Trip {
    f64x2 v[U][8];
    int k8[U][8], w[U];
  };
  auto fetch = [&](int64_t base, Trip &t) {  // all loads of one trip
#pragma unroll
    for (int j = 0; j < U; j++) {
      const int64_t site0 = base + 8 * j;
      // past n (or a trip past the end, when prefetching): reload the last site;
      // unconditional loads keep the compiler's wait counts exact (results unused)
      const int64_t sq = site0 + g < n ? site0 + g : n - 1;
      const int64_t rec = sq * 8 + (lane & 7);  // f64x2 index of this lane's pair (8 per site)
      t.w[j] = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        t.v[j][q] = f64x2{0.0, 0.0};
        t.k8[j][q] = 0;
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const bool tip = (q & 1) ? T2 : T1;
        if (tip) t.k8[j][q] = ((const uint8_t *)d.g[q])[sq] & 15;
        else t.v[j][q] = ld16<NTL>(reinterpret_cast<const f64x2 *>(d.g[q]) + rec);
      }
      if (kSum) t.w[j] = wgt_at(wgt, sq, ws);
    }
  };
  Trip nxt;
  if constexpr (kPf) fetch(wave * 8 * U, nxt);
  for (int64_t base = wave * 8 * U; base < n; base += stride) {
    int z = 0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    const double *mz = &mats[0][0] + z;
    Trip cur;
    if constexpr (kPf) {  // the next trip's loads stay in flight while this one computes
      cur = nxt;
      fetch(base + stride, nxt);  // unconditional (see fetch)
    } else {
      fetch(base, cur);
    }
    auto &v = cur.v;
    auto &k8 = cur.k8;
    auto &w = cur.w;
    bool valid[U];
#pragma unroll
    for (int j = 0; j < U; j++) valid[j] = base + 8 * j + g < n;
    f64x2 o[U][7];
    bool sc[U][7];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      PairMats M;
      pair_mats_lds(mz + 128 * i, c, h, M);
#pragma unroll
      for (int j = 0; j < U; j++)
        o[j][i] = pair_node<T1, T2>(v[j][2 * i], v[j][2 * i + 1],
                                    tab[T1 ? i : 0] + trow + 4 * k8[j][2 * i],
                                    tab[T2 ? 4 + i : 0] + trow + 4 * k8[j][2 * i + 1], M, E,
                                    valid[j], sh, m, sc[j][i]);
    }
#pragma unroll
    for (int i = 4; i < 7; i++) {  // B1 = (A1, A2), B2 = (A3, A4), R = (B1, B2)
      PairMats M;
      pair_mats_lds(mz + 128 * i, c, h, M);
      const int l = 2 * (i - 4);
#pragma unroll
      for (int j = 0; j < U; j++)
        o[j][i] = pair_node<false, false>(o[j][l], o[j][l + 1], nullptr, nullptr, M, E, valid[j],
                                          sh, m, sc[j][i]);
    }
#pragma unroll
    for (int j = 0; j < U; j++) {
      if (!valid[j]) continue;
      const int64_t site0 = base + 8 * j;
      const int64_t rec = site0 * 8 + lane;
#pragma unroll
      for (int q = 0; q < 7; q++)
        __builtin_nontemporal_store(o[j][q], reinterpret_cast<f64x2 *>(d.x[q]) + rec);
      if ((lane & 7) == 0) {
#pragma unroll
        for (int q = 0; q < 7; q++) {
          if (d.sc[q]) d.sc[q][site0 + g] = (uint8_t)sc[j][q];
          if (kSum && sc[j][q]) acc[q] += w[j];
        }
      }
    }
  }
  if constexpr (kSum) block_ticket_sum7(acc, ws + (size_t)blockIdx.y * 7 * kWsWords, d.ss);
}

// Fused six-level subtree ("deep", f64 lane-pair mapping; built for depth D =
// 4, 5, 6 -- the numbers below are D = 6): the 63 ops of a complete binary
// subtree over 64 dense leaves in one pass -- 64 leaf reads + 63 writes per site (2.02 CLV transfers per node; three-level passes move
// 2.14, and a 64-taxon tree as nine of them reads the eight level-3 CLVs
// back).  Node numbering is heap order by level: level 1 = 0..31 (node i over
// leaves 2i, 2i+1), level 2 = 32..47, level 3 = 48..55, level 4 = 56..59,
// level 5 = 60, 61, root 62; node 32+i's children are nodes 2i, 2i+1 and so
// on up.  A trip evaluates eight three-level groups (group q: leaves
// 8q..8q+7, nodes 4q..4q+3, 32+2q, 33+2q, 48+q) and folds the upper three
// levels in as a binary carry (at most one pending value per level), so the
// code is one group body plus three node bodies.  The 63 nodes' matrices sit
// in LDS (63 KB, one copy per 512-thread block) and every lane reads its 16 per
// node just in time; each node's weighted scaler sum collects in an LDS
// counter (a wave reduction + atomic per node and 8-site block, only where a
// site scaled) and is published by the per-region ticket at the end.  Results
// are bit-identical to 63 separate updates.  (Measured, tools/gpu_deep.sh@f9b3af3,
// profiles/r01_deep.log: 256/512/768-thread blocks, U = 1/2, next-group
// prefetch.)
// kTips = 2: every leaf is a tip (one uint8 state code per site, see
// build_tip_table).  The level-1 nodes then read their ump values from
// per-child LDS tables instead of multiplying: 2 x 2^(D-1) tables of 256
// doubles (128 KiB at D = 6) built once per block, and only the upper levels'
// matrices sit in LDS (31 KiB) -- 159.5 KiB of the 160.  (Round 1 expanded the
// codes in registers instead and ran 20-40 % slower than the three-level
// passes' tables; with the tables a coded 64-taxon tree reads 64 code bytes
// and writes 63 CLVs per site in one pass.)
// Heap-order level offsets of a complete subtree of depth D (level 1 first):
// node numbers off(l) .. off(l) + 2^(D-1-l) - 1 hold level l+1.
template <int D>
__device__ constexpr int deep_off(int l) {
  int o = 0;
  for (int i = 0; i < l; i++) o += 1 << (D - 1 - i);
  return o;
}

// Wave-level chunk queue of the deep passes (kDyn).  Their waves run the
// grid stride independently (no block barriers), and with a fixed stride the
// launch ends when the slowest wave ends: a per-wave timeline of the 2^20-site
// six-level pass (tools/tune_deep_dyn.hip@f9b3af3) shows wave exits from 2.61 to
// 3.36 ms.  Chunk = one wave trip (8U f64 / 16U f32 sites); trip 0 takes
// chunk `wave`, trip 1 W + wave (W = waves in the grid), trip i >= 2 2W + d,
// d from a returning atomic add on the head word that lane 0 issues in trip
// i - 2 (after that trip's first leaf loads) and the wave reads at the end of
// that trip.  The head address carries an offset laundered through an empty
// asm (a VGPR 0): the compiler's atomic optimizer then leaves the single-lane
// add alone (with a uniform address it aggregates lanes and waits for the
// result at once) and the address stays global.  Words: region
// kDeepQueueRegion of the stream workspace ([0] head, [16] exit count); the
// last wave out zeroes both for the next launch, after every wave's last
// dequeue has returned (its exit add depends on the value).
constexpr int kDeepQueueRegion = 63;
struct WaveQueue {
  unsigned long long *head, *done;
  int64_t W, nch, chunk;
  long long pend = 0;  // lane 0: the dequeued chunk offset for trip i + 2
  bool dyn;
  __device__ WaveQueue(unsigned long long *ws, int64_t n, int64_t chunk_sites, int waves_per_block, bool on) {
    int zero = 0;
    if (on) asm volatile("" : "+v"(zero));
    head = ws + (size_t)kDeepQueueRegion * kWsWords + zero;
    done = ws + (size_t)kDeepQueueRegion * kWsWords + 16;
    chunk = chunk_sites;
    W = (int64_t)gridDim.x * waves_per_block;
    nch = (n + chunk_sites - 1) / chunk_sites;
    dyn = on && nch > 2 * W;
  }
  __device__ __forceinline__ void dequeue() {
    if (dyn && (threadIdx.x & 63) == 0)
      pend = (long long)__hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // base of trip i + 2, at the end of trip i (n: none)
  __device__ __forceinline__ int64_t after(int64_t n) const {
    if (!dyn) return n;
    const long long d = (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)pend) |
                        ((long long)__builtin_amdgcn_readfirstlane((int)(pend >> 32)) << 32);
    const int64_t b = (2 * W + d) * chunk;
    return b < n ? b : n;
  }
  __device__ __forceinline__ void finish() const {
    if ((threadIdx.x & 63) != 0) return;
    const unsigned long long later = (unsigned long long)(pend >> 62);  // 0, once it returned
    const unsigned long long d = __hip_atomic_fetch_add(done, 1ull + later, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned long long)W - 1) {
      __hip_atomic_store(head, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
};

struct DeepDesc {
  const void *g[64];
  void *x[63];
  const void *mat[126];  // left, right of node i at 2i, 2i+1
  uint8_t *sc[63];
  int64_t *ss[63];
};

template <int D, bool kSum, bool NTL, int U, int kThreads, int kTips = 0, bool kDyn = false>
__global__ void __launch_bounds__(kThreads, 1)
plf_dna_f64_deep_kernel(const DeepDesc d, const double *__restrict__ EV,
                        const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                        const double *__restrict__ tipvec = nullptr) {
  static_assert(D >= 4 && D <= 6, "depth 4..6");
  static_assert(kTips == 0 || kTips == 2, "dense leaves or every leaf a tip");
  constexpr int kWaves = kThreads / 64, kNodes = (1 << D) - 1, kGroups = 1 << (D - 3);
  constexpr bool kT = kTips == 2;
  constexpr int kLeafOps = 1 << (D - 1);        // level-1 nodes
  constexpr int kM0 = kT ? kLeafOps : 0;        // first node whose matrices sit in LDS
  const int lane = threadIdx.x & 63;
  const int h = lane & 1, c = (lane >> 1) & 3, g = lane >> 3, sh = lane & 56;
  __shared__ double mats[kNodes - kM0][128];
  __shared__ double tabs[kT ? 2 * kLeafOps : 1][kT ? 256 : 1];  // [2i | 2i+1]: node i's left | right
  __shared__ unsigned long long nacc[kNodes];
  for (int e = threadIdx.x; e < (kNodes - kM0) * 128; e += kThreads) {
    const int node = kM0 + (e >> 7), k = e & 127;
    mats[node - kM0][k] = static_cast<const double *>(d.mat[2 * node + (k >> 6)])[k & 63];
  }
  if constexpr (kT) {  // build_tip_table's entries and order, 2^D tables at once
    for (int e = threadIdx.x; e < 2 * kLeafOps * 256; e += kThreads) {
      const int t = e >> 8, cc = (e >> 6) & 3, code = (e >> 2) & 15, k = e & 3;
      const double *P = static_cast<const double *>(d.mat[t]);
      double v = 0.0;
#pragma unroll
      for (int l = 0; l < 4; l++)
        v += (tipvec ? tipvec[code * 4 + l] : double((code >> l) & 1)) * P[cc * 16 + k * 4 + l];
      tabs[t][e & 255] = v;
    }
  }
  if (threadIdx.x < kNodes) nacc[threadIdx.x] = 0;
  __syncthreads();
  const int trow = c * 64 + 2 * h;  // + 4*code: this lane's slice of a table row
  double E[4][2];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int t = 0; t < 2; t++) E[k][t] = EV[4 * k + 2 * h + t];
  const double m = Num<double>::minlik();
  const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWaves * 8 * U;
  WaveQueue wq(ws, n, 8 * U, kWaves, kDyn);
  int64_t nbase = wave * 8 * U + stride;  // kDyn: the base of the next trip
  for (int64_t base = wave * 8 * U; base < n;) {
    int z = 0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));  // keep the matrix reads inside the loop
    const double *mz = &mats[0][0] + z;
    bool valid[U];
    int64_t sq[U];
    int w[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
      valid[j] = base + 8 * j + g < n;
      sq[j] = valid[j] ? base + 8 * j + g : n - 1;  // past n: any valid record (unused)
      w[j] = kSum ? wgt_at(wgt, sq[j], ws) : 0;
    }
    // node `node` of this trip on inputs a, b (kT level 1: codes ka, kb):
    // output stored, scaler byte and sum
    auto node_eval = [&](int node, const f64x2 (&a)[U], const f64x2 (&b)[U], f64x2 (&o)[U],
                         const int *ka = nullptr, const int *kb = nullptr) {
      PairMats M;
      const bool tipn = kT && node < kLeafOps;  // compile-time after unrolling
      if (!tipn) pair_mats_lds(mz + 128 * (node - kM0), c, h, M);
      f64x2 *dst = static_cast<f64x2 *>(d.x[node]);
      uint8_t *scp = d.sc[node];
#pragma unroll
      for (int j = 0; j < U; j++) {
        bool sc;
        if (tipn)
          o[j] = pair_node<true, true>(a[j], b[j], &tabs[kT ? 2 * node : 0][trow + 4 * ka[j]],
                                       &tabs[kT ? 2 * node + 1 : 0][trow + 4 * kb[j]], M, E, valid[j],
                                       sh, m, sc);
        else
          o[j] = pair_node<false, false>(a[j], b[j], nullptr, nullptr, M, E, valid[j], sh, m, sc);
        if (valid[j]) {
          __builtin_nontemporal_store(o[j], dst + (base + 8 * j) * 8 + lane);
          if ((lane & 7) == 0 && scp) scp[base + 8 * j + g] = (uint8_t)sc;
        }
        if (kSum) {
          const bool mine = (lane & 7) == 0 && valid[j] && sc;
          if (__ballot(mine)) {  // rare: some site of the block scaled
            long long v = mine ? (long long)w[j] : 0ll;
            v += __shfl_xor(v, 8);
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane == 0) atomicAdd(&nacc[node], (unsigned long long)v);
          }
        }
      }
    };
    f64x2 s3[U], s4[U], s5[U];  // pending level-3/4/5 values of the carry
#pragma unroll 1
    for (int q = 0; q < kGroups; q++) {
      f64x2 v[8][U];
      int k8[8][U];
#pragma unroll
      for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int j = 0; j < U; j++) {
          if constexpr (kT) {
            k8[i][j] = static_cast<const uint8_t *>(d.g[8 * q + i])[sq[j]] & 15;
            v[i][j] = f64x2{0.0, 0.0};
          } else {
            v[i][j] = ld16<NTL>(static_cast<const f64x2 *>(d.g[8 * q + i]) + sq[j] * 8 + (lane & 7));
          }
        }
      }
      if (kDyn && q == 0) wq.dequeue();
      f64x2 a1[4][U], a2[2][U], r[U];
#pragma unroll
      for (int i = 0; i < 4; i++) node_eval(4 * q + i, v[2 * i], v[2 * i + 1], a1[i], k8[2 * i], k8[2 * i + 1]);
#pragma unroll
      for (int i = 0; i < 2; i++) node_eval(deep_off<D>(1) + 2 * q + i, a1[2 * i], a1[2 * i + 1], a2[i]);
      node_eval(deep_off<D>(2) + q, a2[0], a2[1], r);
      // levels 4..D: a binary carry over the groups, one pending value per level
#pragma unroll
      for (int l = 3; l < D; l++) {
        f64x2 (&pend)[U] = l == 3 ? s3 : (l == 4 ? s4 : s5);
        if (!((q >> (l - 3)) & 1)) {
#pragma unroll
          for (int j = 0; j < U; j++) pend[j] = r[j];
          break;
        }
        f64x2 up[U];
        node_eval(deep_off<D>(l) + (q >> (l - 2)), pend, r, up);
#pragma unroll
        for (int j = 0; j < U; j++) r[j] = up[j];
      }
    }
    if constexpr (kDyn) {
      base = nbase;
      nbase = wq.after(n);
    } else {
      base += stride;
    }
  }
  if constexpr (kDyn) wq.finish();
  if constexpr (kSum) {
    __syncthreads();
    if (threadIdx.x < kNodes)
      ticket_publish((long long)nacc[threadIdx.x], ws + (size_t)threadIdx.x * kWsWords, d.ss[threadIdx.x]);
  }
}

// The same six-level pass in the lane = category mapping (f32; any T): lane =
// (site q, category c), 16 sites per wave and block of U; a lane reads its
// category's 32 matrix values per node from the LDS copy (31.5 KB f32).
// kTips = 2: every leaf a tip, as the f64 pass (2^D per-child tables of 256
// values, 64 KiB f32 at D = 6, beside the upper levels' 15.5 KiB of matrices).
template <int D, typename T, bool kSum, bool NT, int U, int kThreads, int kTips = 0, bool kDyn = false>
__global__ void __launch_bounds__(kThreads, 1)
plf_dna_cat_deep_kernel(const DeepDesc d, const T *__restrict__ EV,
                        const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                        const T *__restrict__ tipvec = nullptr) {
  static_assert(D >= 4 && D <= 6, "depth 4..6");
  static_assert(kTips == 0 || kTips == 2, "dense leaves or every leaf a tip");
  constexpr int kWaves = kThreads / 64, kNodes = (1 << D) - 1, kGroups = 1 << (D - 3);
  constexpr bool kT = kTips == 2;
  constexpr int kLeafOps = 1 << (D - 1);  // level-1 nodes
  constexpr int kM0 = kT ? kLeafOps : 0;  // first node whose matrices sit in LDS
  const int lane = threadIdx.x & 63;
  const int c = lane & 3, qs = lane >> 2, nib = lane & 60;
  __shared__ T mats[(kNodes - kM0) * 128];  // node i: left [c][16] | right [c][16]
  __shared__ T tabs[kT ? 2 * kLeafOps : 1][kT ? 256 : 1];  // [2i | 2i+1]: node i's left | right
  __shared__ unsigned long long nacc[kNodes];
  for (int e = threadIdx.x; e < (kNodes - kM0) * 128; e += kThreads) {
    const int node = kM0 + (e >> 7), k = e & 127;
    mats[e] = static_cast<const T *>(d.mat[2 * node + (k >> 6)])[k & 63];
  }
  if constexpr (kT) {  // build_tip_table's entries and order, 2^D tables at once
    for (int e = threadIdx.x; e < 2 * kLeafOps * 256; e += kThreads) {
      const int t = e >> 8, cc = (e >> 6) & 3, code = (e >> 2) & 15, k = e & 3;
      const T *P = static_cast<const T *>(d.mat[t]);
      T v = T(0);
#pragma unroll
      for (int l = 0; l < 4; l++)
        v += (tipvec ? tipvec[code * 4 + l] : T((code >> l) & 1)) * P[cc * 16 + k * 4 + l];
      tabs[t][e & 255] = v;
    }
  }
  if (threadIdx.x < kNodes) nacc[threadIdx.x] = 0;
  __syncthreads();
  const int trow = c * 64;  // + 4*code: this lane's table row
  T E[16];
#pragma unroll
  for (int i = 0; i < 16; i++) E[i] = EV[i];
  const T m = Num<T>::minlik();
  const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWaves * 16 * U;
  WaveQueue wq(ws, n, 16 * U, kWaves, kDyn);
  int64_t nbase = wave * 16 * U + stride;  // kDyn: the base of the next trip
  for (int64_t base = wave * 16 * U; base < n;) {
    int z = 0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));  // keep the matrix reads inside the loop
    const T *mz = mats + z;
    bool valid[U];
    int64_t sq[U];
    int w[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      valid[u] = base + u * 16 + qs < n;
      sq[u] = valid[u] ? base + u * 16 + qs : n - 1;  // past n: any valid record (unused)
      w[u] = kSum ? wgt_at(wgt, sq[u], ws) : 0;
    }
    // kT level-1 nodes: codes ka, kb instead of matrices
    auto node_eval = [&](int node, const T (&a)[U][4], const T (&b)[U][4], T (&o)[U][4],
                         const int *ka = nullptr, const int *kb = nullptr) {
      const bool tipn = kT && node < kLeafOps;  // compile-time after unrolling
      T PL[16], PR[16];
      if (!tipn) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
          PL[j] = mz[128 * (node - kM0) + c * 16 + j];
          PR[j] = mz[128 * (node - kM0) + 64 + c * 16 + j];
        }
      }
      T *dst = static_cast<T *>(d.x[node]);
      uint8_t *scp = d.sc[node];
#pragma unroll
      for (int u = 0; u < U; u++) {
        bool sc;
        if (tipn)
          cat_node<T, true, true>(a[u], b[u], &tabs[kT ? 2 * node : 0][trow + 4 * ka[u]],
                                  &tabs[kT ? 2 * node + 1 : 0][trow + 4 * kb[u]], PL, PR, E, valid[u],
                                  nib, m, o[u], sc);
        else
          cat_node<T, false, false>(a[u], b[u], nullptr, nullptr, PL, PR, E, valid[u], nib, m, o[u], sc);
        if (valid[u]) {
          Num<T>::store4_nt(dst + sq[u] * 16 + c * 4, o[u]);
          if (c == 0 && scp) scp[sq[u]] = (uint8_t)sc;
        }
        if (kSum) {
          const bool mine = c == 0 && valid[u] && sc;
          if (__ballot(mine)) {  // rare: some site of the block scaled
            long long v = mine ? (long long)w[u] : 0ll;
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane == 0) atomicAdd(&nacc[node], (unsigned long long)v);
          }
        }
      }
    };
    T s3[U][4], s4[U][4], s5[U][4];  // pending level-3/4/5 values of the carry
#pragma unroll 1
    for (int q = 0; q < kGroups; q++) {
      T v[8][U][4];
      int k8[8][U];
#pragma unroll
      for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          if constexpr (kT) {
            k8[i][u] = static_cast<const uint8_t *>(d.g[8 * q + i])[sq[u]] & 15;
#pragma unroll
            for (int l = 0; l < 4; l++) v[i][u][l] = T(0);
          } else {
            Num<T>::template load4<NT>(static_cast<const T *>(d.g[8 * q + i]) + sq[u] * 16 + c * 4, v[i][u]);
          }
        }
      }
      if (kDyn && q == 0) wq.dequeue();
      T a1[4][U][4], a2[2][U][4], r[U][4];
#pragma unroll
      for (int i = 0; i < 4; i++) node_eval(4 * q + i, v[2 * i], v[2 * i + 1], a1[i], k8[2 * i], k8[2 * i + 1]);
#pragma unroll
      for (int i = 0; i < 2; i++) node_eval(deep_off<D>(1) + 2 * q + i, a1[2 * i], a1[2 * i + 1], a2[i]);
      node_eval(deep_off<D>(2) + q, a2[0], a2[1], r);
      auto keep = [&](T (&dst)[U][4], const T (&src)[U][4]) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int l = 0; l < 4; l++) dst[u][l] = src[u][l];
      };
      // levels 4..D: a binary carry over the groups, one pending value per level
#pragma unroll
      for (int l = 3; l < D; l++) {
        T (&pend)[U][4] = l == 3 ? s3 : (l == 4 ? s4 : s5);
        if (!((q >> (l - 3)) & 1)) {
          keep(pend, r);
          break;
        }
        T up[U][4];
        node_eval(deep_off<D>(l) + (q >> (l - 2)), pend, r, up);
        keep(r, up);
      }
    }
    if constexpr (kDyn) {
      base = nbase;
      nbase = wq.after(n);
    } else {
      base += stride;
    }
  }
  if constexpr (kDyn) wq.finish();
  if constexpr (kSum) {
    __syncthreads();
    if (threadIdx.x < kNodes)
      ticket_publish((long long)nacc[threadIdx.x], ws + (size_t)threadIdx.x * kWsWords, d.ss[threadIdx.x]);
  }
}

// Fused three-level subtree in the lane = category mapping (f32; any T): the
// same seven-node pass as plf_dna_f64_septet_kernel, lane = (site q, category
// c), 16 sites per wave and block of U.  A lane needs 32 matrix values per
// node (its category's P_L and P_R rows): the 7 nodes' matrices sit in LDS
// (3.5 KB f32) and are read per node and trip (4 distinct 16-B addresses per
// read, one per category, on disjoint banks); an opaque zero offset keeps the
// reads inside the loop (hoisted they need 224 VGPRs).
template <typename T, bool kSum, int kMinWaves, bool NT, int kTips, int U = 2>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_dna_cat_septet_kernel(const SeptetBatch sb, const T *__restrict__ EV,
                          const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                          const T *__restrict__ tipvec) {
  constexpr bool T1 = kTips >= 1, T2 = kTips == 2;
  const SeptetDesc &d = sb.d[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int c = lane & 3, q = lane >> 2, nib = lane & 60;
  __shared__ T mats[7 * 128];  // node i: left [c][16] | right [c][16]
  __shared__ T tab[T2 ? 8 : (T1 ? 4 : 1)][T1 ? 256 : 1];
  for (int e = threadIdx.x; e < 7 * 128; e += kBlock) {
    const int node = e >> 7, k = e & 127;
    mats[e] = static_cast<const T *>(d.mat[2 * node + (k >> 6)])[k & 63];
  }
  if constexpr (T1) {
#pragma unroll
    for (int i = 0; i < 4; i++) build_tip_table<T>((const T *)d.mat[2 * i], tipvec, tab[i]);
  }
  if constexpr (T2) {
#pragma unroll
    for (int i = 0; i < 4; i++) build_tip_table<T>((const T *)d.mat[2 * i + 1], tipvec, tab[4 + i]);
  }
  __syncthreads();
  T E[16];
#pragma unroll
  for (int i = 0; i < 16; i++) E[i] = EV[i];
  const T m = Num<T>::minlik();
  const int trow = c * 64;

  long long acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 16 * U;
  for (int64_t base = wave * 16 * U; base < n; base += stride) {
    int z = 0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    const T *mz = mats + z;
    T v[U][8][4];
    int k8[U][8], w[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; u++) {  // all loads of the trip first, unconditional (clamped)
      const int64_t site = base + u * 16 + q;
      valid[u] = site < n;
      const int64_t sq = valid[u] ? site : n - 1;
#pragma unroll
      for (int g = 0; g < 8; g++) {
        const bool tip = (g & 1) ? T2 : T1;
        k8[u][g] = 0;
#pragma unroll
        for (int l = 0; l < 4; l++) v[u][g][l] = T(0);
        if (tip) k8[u][g] = ((const uint8_t *)d.g[g])[sq] & 15;
        else Num<T>::template load4<NT>((const T *)d.g[g] + sq * 16 + c * 4, v[u][g]);
      }
      w[u] = kSum ? wgt_at(wgt, sq, ws) : 0;
    }
    T o[U][7][4];
    bool sc[U][7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
      T PL[16], PR[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        PL[j] = mz[128 * i + c * 16 + j];
        PR[j] = mz[128 * i + 64 + c * 16 + j];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (i < 4)
          cat_node<T, T1, T2>(v[u][2 * i], v[u][2 * i + 1], tab[T1 ? (i & 3) : 0] + trow + 4 * k8[u][2 * i],
                              tab[T2 ? 4 + (i & 3) : 0] + trow + 4 * k8[u][2 * i + 1], PL, PR, E,
                              valid[u], nib, m, o[u][i], sc[u][i]);
        else  // B1 = (A1, A2), B2 = (A3, A4), R = (B1, B2)
          cat_node<T, false, false>(o[u][2 * (i - 4)], o[u][2 * (i - 4) + 1], nullptr, nullptr, PL,
                                    PR, E, valid[u], nib, m, o[u][i], sc[u][i]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!valid[u]) continue;
      const int64_t site = base + u * 16 + q;
#pragma unroll
      for (int i = 0; i < 7; i++) Num<T>::store4_nt((T *)d.x[i] + site * 16 + c * 4, o[u][i]);
      if (c == 0) {
#pragma unroll
        for (int i = 0; i < 7; i++) {
          if (d.sc[i]) d.sc[i][site] = (uint8_t)sc[u][i];
          if (kSum && sc[u][i]) acc[i] += w[u];
        }
      }
    }
  }
  if constexpr (kSum) block_ticket_sum7(acc, ws + (size_t)blockIdx.y * 7 * kWsWords, d.ss);
}

}  // namespace dev
}  // namespace plfx
