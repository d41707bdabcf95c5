// plf_kernels.hip -- fused PLF inner-node update for CDNA4 (gfx950).
//
// One kernel replaces the reference's whole accelerator pipeline for one PLF
// call: the PL input movers (hls/src/mm2sleft_memDNAwindowComb.cpp:16-100,
// mm2sright_*, transpose.cpp:6-24), the AIE lane chain mmul_branch x2 ->
// combine -> ev (aie/src/128x9DNAwindow8192Comb/kernels/*.cpp) and the PL
// output mover with the underflow test/rescale and the char scaler
// (hls/src/s2mm_memDNAwindowComb.cpp:45-99), plus the host's weighted scaler
// reduction (app/src/host_mem.cpp:384-388).  Arithmetic follows the CPU
// definition plf() (app/src/plf.cpp:19-65) operation for operation.
//
// Mapping (DNA, S=4 states, C=4 Gamma categories, V=16 values per site):
//   * 4 consecutive lanes own one site, lane c = category c (the reference's
//     4 AIE lanes, app graph.h:6,34-46); a wave covers 16 sites per step and
//     unrolls U steps so 2*U*32 bytes (f64) per child are in flight per lane.
//   * lane c streams its 4 states of x1 and x2 with 16-byte loads (the 4 lanes
//     of a site read one contiguous 64/128-byte site record, the wave one
//     contiguous 1/2 KiB block) and writes its 4 results with non-temporal
//     16-byte stores.
//   * P_L[c], P_R[c] (16 values each) live in VGPRs for the whole grid-stride
//     loop; EV is wave-uniform and is loaded through the scalar cache.
//   * per-site scale test: each lane tests its 4 values, a wave ballot gives a
//     64-bit mask, and the site's nibble == 0xF decides; the rescale is a
//     select (no divergent branch).  Lane c==0 writes the site's scaler byte
//     and accumulates wgt into a register; one 64-bit atomic per block feeds a
//     self-resetting ticket reduction, so no memset launch is needed per call.
//   * no FMA contraction (-ffp-contract=off) and the reference's ascending
//     accumulation order from +0.0: bit-exact against plf() in f32 and against
//     its double instantiation in f64.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "plf_kernels.hpp"

namespace plfx {
namespace {

constexpr int kBlock = 256;       // 4 waves
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
  __device__ static inline void load4(const float *p, float (&v)[4]) {
    f32x4 a = *reinterpret_cast<const f32x4 *>(p);
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
  __device__ static inline void load4(const double *p, double (&v)[4]) {
    f64x2 a = reinterpret_cast<const f64x2 *>(p)[0];
    f64x2 b = reinterpret_cast<const f64x2 *>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
  __device__ static inline void store4_nt(double *p, const double (&v)[4]) {
    f64x2 a = {v[0], v[1]};
    f64x2 b = {v[2], v[3]};
    __builtin_nontemporal_store(a, reinterpret_cast<f64x2 *>(p));
    __builtin_nontemporal_store(b, reinterpret_cast<f64x2 *>(p) + 1);
  }
};

// Block-wide sum of one int64 per thread, then one returned 64-bit atomic per
// block into ws[0] and a ticket in ws[1]; the last block publishes the total
// and resets both words for the next launch on the stream.
__device__ inline void block_ticket_sum(long long v, unsigned long long *ws, int64_t *out) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __shared__ long long part[kWavesPerBlock];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long tot = 0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; i++) tot += part[i];
    long long *sum = reinterpret_cast<long long *>(ws);
    // returned atomic: performed at the device coherence point before the
    // ticket below is taken
    long long prev = __hip_atomic_fetch_add(sum, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)prev;
    unsigned long long t =
        __hip_atomic_fetch_add(ws + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned long long)gridDim.x - 1) {
      long long total = __hip_atomic_exchange(sum, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *out = (int64_t)total;
      __hip_atomic_store(ws + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <typename T, int U, bool kSum>
__global__ void __launch_bounds__(kBlock)
plf_dna_kernel(const T *__restrict__ x1, const T *__restrict__ x2, T *__restrict__ x3,
               const T *__restrict__ EV, const T *__restrict__ left,
               const T *__restrict__ right, const int32_t *__restrict__ wgt,
               uint8_t *__restrict__ scaler, int64_t n, unsigned long long *ws,
               int64_t *scaler_sum) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 3;         // Gamma category owned by this lane
  const int q = lane >> 2;        // site slot within a 16-site wave step
  const int nib = lane & 60;      // bit offset of this site's nibble in the ballot

  T PL[16], PR[16], E[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    PL[i] = left[c * 16 + i];     // left[c*16 + k*4 + l]
    PR[i] = right[c * 16 + i];
    E[i] = EV[i];                 // uniform: scalar loads
  }

  long long acc = 0;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * 16 * U;
  for (int64_t base = wave * 16 * U; base < n; base += stride) {
    T a[U][4], b[U][4];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t site = base + u * 16 + q;
      valid[u] = site < n;
      if (valid[u]) {
        Num<T>::load4(x1 + site * 16 + c * 4, a[u]);
        Num<T>::load4(x2 + site * 16 + c * 4, b[u]);
      } else {
#pragma unroll
        for (int l = 0; l < 4; l++) { a[u][l] = T(0); b[u][l] = T(0); }
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      // plf.cpp:31-43: ump_x1/ump_x2 from +0.0, ascending l; product per k
      T p[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        T u1 = T(0), u2 = T(0);
#pragma unroll
        for (int l = 0; l < 4; l++) {
          u1 += a[u][l] * PL[k * 4 + l];
          u2 += b[u][l] * PR[k * 4 + l];
        }
        p[k] = u1 * u2;
      }
      // plf.cpp:25-27,45-50: x3 from +0.0, ascending k
      T o[4];
#pragma unroll
      for (int l = 0; l < 4; l++) o[l] = T(0);
#pragma unroll
      for (int k = 0; k < 4; k++) {
#pragma unroll
        for (int l = 0; l < 4; l++) o[l] += p[k] * E[4 * k + l];
      }
      // plf.cpp:53-64 / s2mm:70-85: scale iff all 16 |x3| < 2^-32
      const T m = Num<T>::minlik();
      const bool small = valid[u] && (Num<T>::abs(o[0]) < m) && (Num<T>::abs(o[1]) < m) &&
                         (Num<T>::abs(o[2]) < m) && (Num<T>::abs(o[3]) < m);
      const unsigned long long mask = __ballot(small);
      const bool sc = ((mask >> nib) & 0xFull) == 0xFull;
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const T s = o[l] * Num<T>::two32();  // exact: power-of-two scaling
        o[l] = sc ? s : o[l];
      }
      if (valid[u]) {
        const int64_t site = base + u * 16 + q;
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

__global__ void __launch_bounds__(kBlock)
scaler_sum_kernel(const uint8_t *__restrict__ scaler, const int32_t *__restrict__ wgt, int64_t n,
                  unsigned long long *ws, int64_t *out) {
  long long acc = 0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride)
    acc += (long long)scaler[j] * (wgt ? (long long)wgt[j] : 1ll);
  block_ticket_sum(acc, ws, out);
}

template <typename T, int U>
hipError_t launch_dna(const DnaArgs &a, int max_blocks, hipStream_t s) {
  const int64_t sites_per_block = (int64_t)kWavesPerBlock * 16 * U;
  int64_t blocks = (a.n + sites_per_block - 1) / sites_per_block;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  if (a.scaler_sum) {
    hipLaunchKernelGGL((plf_dna_kernel<T, U, true>), dim3((unsigned)blocks), dim3(kBlock), 0, s,
                       (const T *)a.x1, (const T *)a.x2, (T *)a.x3, (const T *)a.EV,
                       (const T *)a.left, (const T *)a.right, a.wgt, a.scaler, a.n, a.ws,
                       a.scaler_sum);
  } else {
    hipLaunchKernelGGL((plf_dna_kernel<T, U, false>), dim3((unsigned)blocks), dim3(kBlock), 0, s,
                       (const T *)a.x1, (const T *)a.x2, (T *)a.x3, (const T *)a.EV,
                       (const T *)a.left, (const T *)a.right, a.wgt, a.scaler, a.n, a.ws,
                       a.scaler_sum);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_plf_dna_f32(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return launch_dna<float, 4>(a, max_blocks, s);
}
hipError_t launch_plf_dna_f64(const DnaArgs &a, int max_blocks, hipStream_t s) {
  return launch_dna<double, 2>(a, max_blocks, s);
}

hipError_t launch_scaler_sum(const uint8_t *scaler, const int32_t *wgt, int64_t n, int64_t *out,
                             unsigned long long *ws, int max_blocks, hipStream_t s) {
  int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(scaler_sum_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, scaler, wgt, n,
                     ws, out);
  return hipGetLastError();
}

}  // namespace plfx
