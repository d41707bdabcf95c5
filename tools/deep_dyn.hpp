// deep_dyn.hpp -- tuning copy (not product code): the f64 six-level pass
// (plf_dna_f64_deep_kernel, csrc/plf_dna.hpp) with per-wave timestamps and an
// optional wave-level chunk queue (kDyn) in place of the fixed wave stride.
#pragma once
#include "plf_dna.hpp"

namespace plfx {
namespace dev {

template <int D, bool kSum, bool NTL, int U, int kThreads, int kTips = 0, bool kDyn = false>
__global__ void __launch_bounds__(kThreads, 1)
plf_dna_f64_deep_dyn_kernel(const DeepDesc d, const double *__restrict__ EV,
                        const int32_t *__restrict__ wgt, int64_t n, unsigned long long *ws,
                        const double *__restrict__ tipvec, unsigned long long *queue, uint64_t *stamps) {
  const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
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
  // kDyn: chunks of 8U sites; trip 0 = chunk `wave`, trip 1 = W + wave, trip
  // i >= 2 = 2W + d, d from lane 0's dequeue issued at the start of trip i - 1
  // (after the first leaf loads are issued, used at trip i's start)
  const int64_t W = (int64_t)gridDim.x * kWaves, nch = (n + 8 * U - 1) / (8 * U);
  const bool dyn = kDyn && nch > 2 * W;
  int zero = 0;
  if (kDyn) asm volatile("" : "+v"(zero));
  unsigned long long *head = queue + zero;
  long long dq_pend = 0;
  int trips = 0;
  int64_t nbase = (W + wave) * 8 * U;
  for (int64_t base = wave * 8 * U; base < n; trips++) {
    bool deq_issued = false;
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
      if (dyn && q == 0 && !deq_issued) {
        deq_issued = true;
        if (lane == 0)
          dq_pend = (long long)__hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
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
      if (dyn) {
        const long long dq = (long long)(unsigned)__builtin_amdgcn_readfirstlane((int)dq_pend) |
                             ((long long)__builtin_amdgcn_readfirstlane((int)(dq_pend >> 32)) << 32);
        nbase = (2 * W + dq) * 8 * U;
      } else {
        nbase = n;
      }
    } else {
      base += stride;
    }
    if (stamps && lane == 0 && trips < 37) stamps[(size_t)wave * 40 + 2 + trips] = __builtin_amdgcn_s_memrealtime();
  }
  if (kDyn && lane == 0) {
    const unsigned long long after = (unsigned long long)(dq_pend >> 62);
    const unsigned long long dn = __hip_atomic_fetch_add(queue + 16, 1ull + after, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dn == (unsigned long long)W - 1) {
      __hip_atomic_store(queue, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(queue + 16, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (stamps && lane == 0) {
    stamps[(size_t)wave * 40] = t_entry | ((uint64_t)(__builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15) << 56);
    stamps[(size_t)wave * 40 + 1] = (uint64_t)trips;
    stamps[(size_t)wave * 40 + 39] = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (kSum) {
    __syncthreads();
    if (threadIdx.x < kNodes)
      ticket_publish((long long)nacc[threadIdx.x], ws + (size_t)threadIdx.x * kWsWords, d.ss[threadIdx.x]);
  }
}

}  // namespace dev
}  // namespace plfx
