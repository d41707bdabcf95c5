// prot_dma32.hpp -- tuning copy (not product code): the f32 FMA protein kernel
// (plf_prot_mfma32_kernel, dense children) with its child tiles moved by
// LDS-DMA (global_load_lds_dwordx4: HBM -> LDS with no VGPR destination)
// into two LDS tiles per block, the VERDICT r02 item-5 candidate:
//   A <- x1 of the trip, B <- x2 of the trip (then X3 of the trip);
//   wait A, barrier, phase 1 on A; wait B, barrier, DMA x1(next) -> A;
//   phase 2 on B; barrier, back-transform into B, barrier; scaler bytes and
//   the store pass from B; barrier, DMA x2(next) -> B.
// Five barriers per trip instead of six, no tile_put pass (5 ds_write_b128 per
// thread and child) and no 20-VGPR register prefetch.  One DMA instruction
// fills 64 consecutive 16-B LDS slots (lane order), so the padded conflict-free
// row layout of the product cannot be written; instead the four-float chunks
// of site s are rotated by r(s) = (s >> 2) & 3 inside the site's 20 slots (slot
// (s, (q + r(s)) % 20) holds chunk q), which puts the B-fragment reads of 16
// sites x 4 lane groups on 64 distinct banks (except where the rotation wraps).
// The lane that fills slot j loads global chunk (s, (j % 20 - r(s)) mod 20), so
// every DMA instruction still reads one contiguous 1-KiB window of the child.
// Sites past n load the last valid site's record (never stored).
#pragma once
#include "plf_prot.hpp"

namespace plfx {
namespace dev {

// one 16-B LDS-DMA per lane: LDS bytes [m0 + 16 * lane, +16) <- *src (per lane)
__device__ __forceinline__ void glds16_nt(const void *src, unsigned lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_byte)
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ int rot_of(int s) { return (s >> 2) & 3; }
// float offset of (site s, chunk q) in a rotated tile
__device__ __forceinline__ int rslot(int s, int q) {
  int p = q + rot_of(s);
  p = p >= 20 ? p - 20 : p;
  return s * 80 + 4 * p;
}

// the block's 1280 chunk slots of one child tile, 5 DMA instructions per thread
__device__ __forceinline__ void tile_dma32(const float *__restrict__ g, int64_t base, int64_t n,
                                           unsigned tile_byte) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const int j = threadIdx.x + i * kBlock;
    const int s = j / 20, ql = j - s * 20;
    int q = ql - rot_of(s);
    q = q < 0 ? q + 20 : q;
    const int64_t site = base + s < n ? base + s : n - 1;
    glds16_nt(g + site * 80 + q * 4, tile_byte + (unsigned)(i * kBlock + wv * 64) * 16u);
  }
}

template <bool kSum, int kMinWaves>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma32d_kernel(const float *__restrict__ x1, const float *__restrict__ x2,
                        float *__restrict__ x3, const float *__restrict__ EV,
                        const float *__restrict__ left, const float *__restrict__ right,
                        const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                        unsigned long long *ws, int64_t *scaler_sum,
                        const float *__restrict__ tipvec = nullptr) {
  constexpr int S = 20;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lo16 = lane & 15, g = lane >> 4;
  const int64_t stride = (int64_t)gridDim.x * 64;
  __shared__ __attribute__((aligned(16))) float tA[64 * 80];
  __shared__ __attribute__((aligned(16))) float tB[64 * 80];
  const unsigned bA = (unsigned)(uintptr_t)tA, bB = (unsigned)(uintptr_t)tB;
  if ((int64_t)blockIdx.x * 64 < n) {
    tile_dma32(x1, (int64_t)blockIdx.x * 64, n, bA);
    tile_dma32(x2, (int64_t)blockIdx.x * 64, n, bB);
  }
  float AL[2][5], AR[2][5], AE[2][5];
#pragma unroll
  for (int mt = 0; mt < 2; mt++)
#pragma unroll
    for (int st = 0; st < 5; st++) {
      const int i = lo16, col = 4 * st + g;
      const int k = 16 * mt + 4 * (i & 3) + (i >> 2);
      AL[mt][st] = (k < S && !mt) ? left[c * S * S + k * S + col] : 0.f;
      AR[mt][st] = (k < S && !mt) ? right[c * S * S + k * S + col] : 0.f;
      const int lrow = 16 * mt + i;
      AE[mt][st] = (lrow < S && !mt) ? EV[col * S + lrow] : 0.f;
    }
  __shared__ __attribute__((aligned(16))) float qm[3][4][4][S];
  for (int e = threadIdx.x; e < 4 * 4 * S; e += kBlock) {
    const int cc = e / (4 * S), i = (e / S) & 3, j = e % S;
    qm[0][cc][i][j] = left[cc * S * S + (16 + i) * S + j];
    qm[1][cc][i][j] = right[cc * S * S + (16 + i) * S + j];
    if (cc == 0) qm[2][0][i][j] = EV[j * S + 16 + i];
  }
  const float *QL = &qm[0][c][lane & 3][0], *QR = &qm[1][c][lane & 3][0];
  const float *QE = &qm[2][0][lane & 3][0];
  const float m = Num<float>::minlik();
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  auto product = [&](const float (&A)[2][5], const float *QA, f32x4 (&P)[4][2], f32x4 &Q, bool mul,
                     const float *tb) {
    f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int s = 16 * t + lo16;
      float bv[5];
#pragma unroll
      for (int st = 0; st < 5; st++) bv[st] = tb[rslot(s, 5 * c + st) + g];
      {
        f32x4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 5; st++) u = __builtin_amdgcn_mfma_f32_16x16x4f32(A[0][st], bv[st], u, 0, 0, 0);
        P[t][0] = mul ? P[t][0] * u : u;
      }
      {
        const f32x4 xv = *reinterpret_cast<const f32x4 *>(tb + rslot(lane, 5 * c + t));
        const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 4 * t);
#pragma unroll
        for (int j = 0; j < 4; j++) q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
      }
    }
    {
      const f32x4 xv = *reinterpret_cast<const f32x4 *>(tb + rslot(lane, 5 * c + 4));
      const f32x4 av = *reinterpret_cast<const f32x4 *>(QA + 16);
#pragma unroll
      for (int j = 0; j < 4; j++) q = __builtin_amdgcn_mfma_f32_4x4x1f32(av[j], xv[j], q, 0, 0, 0);
      Q = mul ? Q * q : q;
    }
  };
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += stride) {
    const int64_t next = base + stride;
    f32x4 P[4][2];
    f32x4 Q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; t++) P[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // x1 of this trip in A (B's five DMAs may still be in flight: loads retire
    // in order, so at most 5 outstanding means A's have landed)
    wait_vm<5>();
    __syncthreads();  // also: qm written (first trip)
    product(AL, QL, P, Q, false, tA);
    wait_vm<0>();     // x2 of this trip in B
    __syncthreads();  // every wave is done with A
    if (next < n) tile_dma32(x1, next, n, bA);
    product(AR, QR, P, Q, true, tB);
    __syncthreads();  // every wave is done reading x2: B takes X3 now
    unsigned Qt[4] = {__float_as_uint(Q[0]), __float_as_uint(Q[1]), __float_as_uint(Q[2]),
                      __float_as_uint(Q[3])};
    transpose_groups44(Qt);
    unsigned pk[16];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      unsigned v[4];
#pragma unroll
      for (int t = 0; t < 4; t++) v[t] = __float_as_uint(P[t][0][r]);
      transpose_groups44(v);
#pragma unroll
      for (int gg = 0; gg < 4; gg++) pk[4 * r + gg] = v[gg];
    }
    unsigned long long mine = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      f32x4 X0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 5; st++) {
        const float b = st == 4 ? __uint_as_float(Qt[t]) : P[t][st >> 2][st & 3];
        X0 = __builtin_amdgcn_mfma_f32_16x16x4f32(AE[0][st], b, X0, 0, 0, 0);
      }
      bool small = (__builtin_fabsf(X0[0]) < m) && (__builtin_fabsf(X0[1]) < m) &&
                   (__builtin_fabsf(X0[2]) < m) && (__builtin_fabsf(X0[3]) < m);
      const unsigned long long b = __ballot(small);
      mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
      *reinterpret_cast<f32x4 *>(tB + rslot(16 * t + lo16, 5 * c + g)) = X0;
    }
    {
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
      *reinterpret_cast<f32x4 *>(tB + rslot(lane, 5 * c + 4)) = X1;
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
    // store pass: slot j of B holds chunk (s, (j % 20 - r(s)) mod 20)
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int j = threadIdx.x + i * kBlock;
      const int s = j / 20, ql = j - s * 20;
      int q = ql - rot_of(s);
      q = q < 0 ? q + 20 : q;
      f32x4 v = reinterpret_cast<const f32x4 *>(tB)[j];
      if ((all >> s) & 1ull) v = v * Num<float>::two32();
      if (base + s < n) __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(x3 + (base + s) * 80 + q * 4));
    }
    __syncthreads();  // every wave is done reading B
    if (next < n) tile_dma32(x2, next, n, bB);
  }
  wait_vm<0>();
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
