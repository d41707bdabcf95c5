// prot_variants.hpp -- experimental protein (S=20) exact-mode kernels for the
// tuning harness tools/tune_prot.hip (not product code).
//
// Phased variant of plf_prot_kernel (csrc/plf_prot.hpp): each lane owns NS
// sites (sites base + s*64 + lane) of one category (wave = category) and runs
//   phase 1: U[s][k]  = sum_l x1[s][l] * PL[k][l]        (ascending l)
//   phase 2: U[s][k] *= sum_l x2[s][l] * PR[k][l]        (prod = umpL * umpR)
//   phase 3: O[s][l]  = sum_k U[s][k] * EV[k][l]         (ascending k)
// -- every value with plf()'s operation order, so the results are bit-identical
// to the product kernel.  One broadcast matrix value serves NS sites.
// kScalar: matrix values come from scalar loads (s_load through the scalar
// cache) instead of v_readlane broadcasts of lane-distributed registers.
#pragma once
#include "plf_prot_tune.hpp"

namespace plfx {
namespace dev {

template <bool kScalar, int NS, int kMinBlocks = 2>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
prot_phased_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                   double *__restrict__ x3, const double *__restrict__ EV,
                   const double *__restrict__ left, const double *__restrict__ right,
                   const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                   unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  constexpr int R = (S * S + 63) / 64;
  double ML[R], MR[R], ME[R];
  const double *gL = left + c * S * S, *gR = right + c * S * S, *gE = EV;
  if constexpr (!kScalar) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int e = r * 64 + lane;
      ML[r] = e < S * S ? gL[e] : 0.0;
      MR[r] = e < S * S ? gR[e] : 0.0;
      ME[r] = e < S * S ? EV[e] : 0.0;
    }
  }
  auto mL = [&](int e) { if constexpr (kScalar) return gL[e]; else return bcast<double>(ML, e); };
  auto mR = [&](int e) { if constexpr (kScalar) return gR[e]; else return bcast<double>(MR, e); };
  auto mE = [&](int e) { if constexpr (kScalar) return gE[e]; else return bcast<double>(ME, e); };
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock][NS];
  long long acc = 0;
  for (int64_t base = (int64_t)blockIdx.x * 64 * NS; base < n; base += (int64_t)gridDim.x * 64 * NS) {
    // opaque per trip: keeps the 3 x 400 broadcasts / scalar loads inside the
    // loop instead of hoisted (and spilled) as loop invariants
    if constexpr (kScalar) {
      asm volatile("" : "+s"(gL), "+s"(gR), "+s"(gE));
    } else {
#pragma unroll
      for (int r = 0; r < R; r++) asm volatile("" : "+v"(ML[r]), "+v"(MR[r]), "+v"(ME[r]));
    }
    double U[NS][S];
    {
      double a[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x1, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, a[s]);
        __syncthreads();
      }
#pragma unroll
      for (int k = 0; k < S; k++) {
        double u[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) u[s] = 0.0;
#pragma unroll
        for (int l = 0; l < S; l++) {
          const double p = mL(k * S + l);
#pragma unroll
          for (int s = 0; s < NS; s++) u[s] += a[s][l] * p;
        }
#pragma unroll
        for (int s = 0; s < NS; s++) U[s][k] = u[s];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    {
      double b[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x2, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, b[s]);
        __syncthreads();
      }
#pragma unroll
      for (int k = 0; k < S; k++) {
        double u[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) u[s] = 0.0;
#pragma unroll
        for (int l = 0; l < S; l++) {
          const double p = mR(k * S + l);
#pragma unroll
          for (int s = 0; s < NS; s++) u[s] += b[s][l] * p;
        }
#pragma unroll
        for (int s = 0; s < NS; s++) U[s][k] = U[s][k] * u[s];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    double O[NS][S];
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int l = 0; l < S; l++) O[s][l] = 0.0;
#pragma unroll
    for (int k = 0; k < S; k++) {
#pragma unroll
      for (int l = 0; l < S; l++) {
        const double e = mE(k * S + l);
#pragma unroll
        for (int s = 0; s < NS; s++) O[s][l] += U[s][k] * e;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
      bool small = base + 64 * s + lane < n;
#pragma unroll
      for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[s][l]) < m);
      const unsigned long long mk = __ballot(small);
      if (lane == 0) small_mask[c][s] = mk;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const unsigned long long all =
          small_mask[0][s] & small_mask[1][s] & small_mask[2][s] & small_mask[3][s];
      const bool sc = (all >> lane) & 1ull;
#pragma unroll
      for (int l = 0; l < S; l++) {
        const double sv = O[s][l] * Num<double>::two32();
        O[s][l] = sc ? sv : O[s][l];
      }
      row_write<double>(tile, lane, c, O[s]);
      const int64_t site = base + 64 * s + lane;
      if (site < n && c == 0) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
      __syncthreads();
      tile_store<double>(x3, base + 64 * s, n, tile);
      __syncthreads();
    }
  }
  block_ticket_sum(acc, ws, scaler_sum);
}

// Matrices in LDS, read as wave-uniform ds_read_b128 broadcasts (2 values per
// 4 LDS cycles, no VALU cost) instead of v_readlane; NS sites per lane.  Rows
// are double-buffered in registers by hand: row k+1 is read, then an empty
// asm with a memory clobber pins the order, then row k is used -- otherwise
// the compiler hoists a whole phase's 200 reads and spills them.
template <int NS>
struct RowPipe {
  f64x2 cur[10], nxt[10];
  __device__ __forceinline__ void load(f64x2 (&d)[10], const f64x2 *row) {
#pragma unroll
    for (int i = 0; i < 10; i++) d[i] = row[i];
  }
};

template <int NS, int kMinBlocks = 2>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
prot_ldsmat_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                   double *__restrict__ x3, const double *__restrict__ EV,
                   const double *__restrict__ left, const double *__restrict__ right,
                   const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                   unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ f64x2 mats[(2 * 4 * S * S + S * S) / 2];  // PL[4][400] | PR[4][400] | EV[400]
  {
    const f64x2 *gl = reinterpret_cast<const f64x2 *>(left);
    const f64x2 *gr = reinterpret_cast<const f64x2 *>(right);
    const f64x2 *ge = reinterpret_cast<const f64x2 *>(EV);
    for (int i = threadIdx.x; i < 800; i += kBlock) { mats[i] = gl[i]; mats[800 + i] = gr[i]; }
    for (int i = threadIdx.x; i < 200; i += kBlock) mats[1600 + i] = ge[i];
  }
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock][NS];
  long long acc = 0;
  __syncthreads();
  // one phase: for k, rows M[k] (10 x f64x2) feed fn(k, row)
  auto phase = [&](const f64x2 *M, auto &&fn) {
    f64x2 cur[10], nxt[10];
    int o = 0;
    double tok = 0.0;
#pragma unroll
    for (int i = 0; i < 10; i++) cur[i] = M[i];
#pragma unroll
    for (int k = 0; k < S; k++) {
      // row k+1's reads wait for row k-1's arithmetic (tok): at most two rows
      // of the matrix are in registers, whatever the scheduler prefers
      asm volatile("" : "+v"(o) : "v"(tok));
      if (k + 1 < S) {
#pragma unroll
        for (int i = 0; i < 10; i++) nxt[i] = M[o + (k + 1) * 10 + i];
      }
      tok = fn(k, cur);
#pragma unroll
      for (int i = 0; i < 10; i++) cur[i] = nxt[i];
    }
  };
  for (int64_t base = (int64_t)blockIdx.x * 64 * NS; base < n; base += (int64_t)gridDim.x * 64 * NS) {
    int off = 0;  // opaque per trip: the matrix reads are not hoisted out of the loop
    asm volatile("" : "+v"(off));
    const f64x2 *mL = mats + off + c * 200, *mR = mats + off + 800 + c * 200, *mE = mats + off + 1600;
    double U[NS][S];
    {
      double a[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x1, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, a[s]);
        __syncthreads();
      }
      phase(mL, [&](int k, const f64x2 (&p)[10]) {
        double u[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) u[s] = 0.0;
#pragma unroll
        for (int l2 = 0; l2 < S / 2; l2++)
#pragma unroll
          for (int s = 0; s < NS; s++) { u[s] += a[s][2 * l2] * p[l2].x; u[s] += a[s][2 * l2 + 1] * p[l2].y; }
#pragma unroll
        for (int s = 0; s < NS; s++) U[s][k] = u[s];
        return u[0];
      });
    }
    {
      double b[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x2, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, b[s]);
        __syncthreads();
      }
      phase(mR, [&](int k, const f64x2 (&p)[10]) {
        double u[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) u[s] = 0.0;
#pragma unroll
        for (int l2 = 0; l2 < S / 2; l2++)
#pragma unroll
          for (int s = 0; s < NS; s++) { u[s] += b[s][2 * l2] * p[l2].x; u[s] += b[s][2 * l2 + 1] * p[l2].y; }
#pragma unroll
        for (int s = 0; s < NS; s++) U[s][k] = U[s][k] * u[s];
        return U[0][k];
      });
    }
    double O[NS][S];
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int l = 0; l < S; l++) O[s][l] = 0.0;
    phase(mE, [&](int k, const f64x2 (&e)[10]) {
#pragma unroll
      for (int l2 = 0; l2 < S / 2; l2++)
#pragma unroll
        for (int s = 0; s < NS; s++) {
          O[s][2 * l2] += U[s][k] * e[l2].x;
          O[s][2 * l2 + 1] += U[s][k] * e[l2].y;
        }
      return O[0][S - 1];
    });
#pragma unroll
    for (int s = 0; s < NS; s++) {
      bool small = base + 64 * s + lane < n;
#pragma unroll
      for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[s][l]) < m);
      const unsigned long long mk = __ballot(small);
      if (lane == 0) small_mask[c][s] = mk;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const unsigned long long all =
          small_mask[0][s] & small_mask[1][s] & small_mask[2][s] & small_mask[3][s];
      const bool sc = (all >> lane) & 1ull;
#pragma unroll
      for (int l = 0; l < S; l++) {
        const double sv = O[s][l] * Num<double>::two32();
        O[s][l] = sc ? sv : O[s][l];
      }
      row_write<double>(tile, lane, c, O[s]);
      const int64_t site = base + 64 * s + lane;
      if (site < n && c == 0) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
      __syncthreads();
      tile_store<double>(x3, base + 64 * s, n, tile);
      __syncthreads();
    }
  }
  block_ticket_sum(acc, ws, scaler_sum);
}

// As prot_ldsmat_kernel, pipelined by half rows (10 values): row k of a
// matrix is two halves q = 2k, 2k+1; at most two halves are in registers.
template <int NS, int kMinBlocks = 2>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
prot_ldsmat_h_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ f64x2 mats[(2 * 4 * S * S + S * S) / 2];  // PL[4][400] | PR[4][400] | EV[400]
  {
    const f64x2 *gl = reinterpret_cast<const f64x2 *>(left);
    const f64x2 *gr = reinterpret_cast<const f64x2 *>(right);
    const f64x2 *ge = reinterpret_cast<const f64x2 *>(EV);
    for (int i = threadIdx.x; i < 800; i += kBlock) { mats[i] = gl[i]; mats[800 + i] = gr[i]; }
    for (int i = threadIdx.x; i < 200; i += kBlock) mats[1600 + i] = ge[i];
  }
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock][NS];
  long long acc = 0;
  __syncthreads();
  // fn(q, half) for q = 0..39 (row q>>1, values 10*(q&1) .. +9); returns a token
  auto phase = [&](const f64x2 *M, auto &&fn) {
    f64x2 cur[5], nxt[5];
    int o = 0;
    double tok = 0.0;
#pragma unroll
    for (int i = 0; i < 5; i++) cur[i] = M[i];
#pragma unroll
    for (int q = 0; q < 2 * S; q++) {
      asm volatile("" : "+v"(o) : "v"(tok));
      if (q + 1 < 2 * S) {
#pragma unroll
        for (int i = 0; i < 5; i++) nxt[i] = M[o + (q + 1) * 5 + i];
      }
      tok = fn(q, cur);
#pragma unroll
      for (int i = 0; i < 5; i++) cur[i] = nxt[i];
    }
    return tok;
  };
  for (int64_t base = (int64_t)blockIdx.x * 64 * NS; base < n; base += (int64_t)gridDim.x * 64 * NS) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const f64x2 *mL = mats + off + c * 200, *mR = mats + off + 800 + c * 200, *mE = mats + off + 1600;
    double U[NS][S];
    double tok;
    {
      double a[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x1, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, a[s]);
        __syncthreads();
      }
      double u[NS];
      tok = phase(mL, [&](int q, const f64x2 (&p)[5]) {
        const int k = q >> 1, h = q & 1;
        if (h == 0) {
#pragma unroll
          for (int s = 0; s < NS; s++) u[s] = 0.0;
        }
#pragma unroll
        for (int i = 0; i < 5; i++)
#pragma unroll
          for (int s = 0; s < NS; s++) {
            u[s] += a[s][10 * h + 2 * i] * p[i].x;
            u[s] += a[s][10 * h + 2 * i + 1] * p[i].y;
          }
        if (h == 1) {
#pragma unroll
          for (int s = 0; s < NS; s++) U[s][k] = u[s];
        }
        return u[0];
      });
    }
    {
      // the x2 tile's loads may not start before phase 1 is done (registers)
      const double *x2t = x2;
      asm volatile("" : "+s"(x2t) : "v"(tok));
      double b[NS][S];
#pragma unroll
      for (int s = 0; s < NS; s++) {
        tile_load<double>(x2t, base + 64 * s, n, tile);
        __syncthreads();
        row_read<double>(tile, lane, c, b[s]);
        __syncthreads();
      }
      double u[NS];
      phase(mR, [&](int q, const f64x2 (&p)[5]) {
        const int k = q >> 1, h = q & 1;
        if (h == 0) {
#pragma unroll
          for (int s = 0; s < NS; s++) u[s] = 0.0;
        }
#pragma unroll
        for (int i = 0; i < 5; i++)
#pragma unroll
          for (int s = 0; s < NS; s++) {
            u[s] += b[s][10 * h + 2 * i] * p[i].x;
            u[s] += b[s][10 * h + 2 * i + 1] * p[i].y;
          }
        if (h == 1) {
#pragma unroll
          for (int s = 0; s < NS; s++) U[s][k] = U[s][k] * u[s];
        }
        return u[0];
      });
    }
    double O[NS][S];
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int l = 0; l < S; l++) O[s][l] = 0.0;
    phase(mE, [&](int q, const f64x2 (&e)[5]) {
      const int k = q >> 1, h = q & 1;
#pragma unroll
      for (int i = 0; i < 5; i++)
#pragma unroll
        for (int s = 0; s < NS; s++) {
          O[s][10 * h + 2 * i] += U[s][k] * e[i].x;
          O[s][10 * h + 2 * i + 1] += U[s][k] * e[i].y;
        }
      return O[0][10 * h + 9];
    });
#pragma unroll
    for (int s = 0; s < NS; s++) {
      bool small = base + 64 * s + lane < n;
#pragma unroll
      for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[s][l]) < m);
      const unsigned long long mk = __ballot(small);
      if (lane == 0) small_mask[c][s] = mk;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const unsigned long long all =
          small_mask[0][s] & small_mask[1][s] & small_mask[2][s] & small_mask[3][s];
      const bool sc = (all >> lane) & 1ull;
#pragma unroll
      for (int l = 0; l < S; l++) {
        const double sv = O[s][l] * Num<double>::two32();
        O[s][l] = sc ? sv : O[s][l];
      }
      row_write<double>(tile, lane, c, O[s]);
      const int64_t site = base + 64 * s + lane;
      if (site < n && c == 0) {
        if (scaler) scaler[site] = (uint8_t)sc;
        if (sc) acc += wgt ? (long long)wgt[site] : 1ll;
      }
      __syncthreads();
      tile_store<double>(x3, base + 64 * s, n, tile);
      __syncthreads();
    }
  }
  block_ticket_sum(acc, ws, scaler_sum);
}

// NS = 1, rows taken in pairs (k, k+1) by half rows so that phases 1 and 2
// carry two independent add chains (a single u += a*p chain per row leaves
// the f64 pipe waiting on its own latency).
template <int kMinBlocks = 2>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
prot_ldsmat_p_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ f64x2 mats[(2 * 4 * S * S + S * S) / 2];  // PL[4][400] | PR[4][400] | EV[400]
  {
    const f64x2 *gl = reinterpret_cast<const f64x2 *>(left);
    const f64x2 *gr = reinterpret_cast<const f64x2 *>(right);
    const f64x2 *ge = reinterpret_cast<const f64x2 *>(EV);
    for (int i = threadIdx.x; i < 800; i += kBlock) { mats[i] = gl[i]; mats[800 + i] = gr[i]; }
    for (int i = threadIdx.x; i < 200; i += kBlock) mats[1600 + i] = ge[i];
  }
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  __syncthreads();
  // steps q = 0..19: rows 2(q>>1), 2(q>>1)+1, values 10(q&1) .. +9 of each
  auto phase2 = [&](const f64x2 *M, auto &&fn) {
    f64x2 cur[10], nxt[10];
    int o = 0;
    double tok = 0.0;
#pragma unroll
    for (int i = 0; i < 5; i++) { cur[i] = M[i]; cur[5 + i] = M[10 + i]; }
#pragma unroll
    for (int q = 0; q < S; q++) {
      asm volatile("" : "+v"(o) : "v"(tok));
      if (q + 1 < S) {
        const int r = 2 * ((q + 1) >> 1), h = (q + 1) & 1;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          nxt[i] = M[o + r * 10 + 5 * h + i];
          nxt[5 + i] = M[o + (r + 1) * 10 + 5 * h + i];
        }
      }
      tok = fn(q, cur);
#pragma unroll
      for (int i = 0; i < 10; i++) cur[i] = nxt[i];
    }
    return tok;
  };
  auto phase1 = [&](const f64x2 *M, auto &&fn) {  // one row per step (EV)
    f64x2 cur[10], nxt[10];
    int o = 0;
    double tok = 0.0;
#pragma unroll
    for (int i = 0; i < 10; i++) cur[i] = M[i];
#pragma unroll
    for (int k = 0; k < S; k++) {
      asm volatile("" : "+v"(o) : "v"(tok));
      if (k + 1 < S) {
#pragma unroll
        for (int i = 0; i < 10; i++) nxt[i] = M[o + (k + 1) * 10 + i];
      }
      tok = fn(k, cur);
#pragma unroll
      for (int i = 0; i < 10; i++) cur[i] = nxt[i];
    }
    return tok;
  };
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const f64x2 *mL = mats + off + c * 200, *mR = mats + off + 800 + c * 200, *mE = mats + off + 1600;
    double U[S], tok;
    {
      double a[S];
      tile_load<double>(x1, base, n, tile);
      __syncthreads();
      row_read<double>(tile, lane, c, a);
      __syncthreads();
      double u0 = 0.0, u1 = 0.0;
      tok = phase2(mL, [&](int q, const f64x2 (&p)[10]) {
        const int k = 2 * (q >> 1), h = q & 1;
        if (h == 0) { u0 = 0.0; u1 = 0.0; }
#pragma unroll
        for (int i = 0; i < 5; i++) {
          u0 += a[10 * h + 2 * i] * p[i].x;
          u1 += a[10 * h + 2 * i] * p[5 + i].x;
          u0 += a[10 * h + 2 * i + 1] * p[i].y;
          u1 += a[10 * h + 2 * i + 1] * p[5 + i].y;
        }
        if (h == 1) { U[k] = u0; U[k + 1] = u1; }
        return u0;
      });
    }
    {
      const double *x2t = x2;
      asm volatile("" : "+s"(x2t) : "v"(tok));
      double b[S];
      tile_load<double>(x2t, base, n, tile);
      __syncthreads();
      row_read<double>(tile, lane, c, b);
      __syncthreads();
      double u0 = 0.0, u1 = 0.0;
      phase2(mR, [&](int q, const f64x2 (&p)[10]) {
        const int k = 2 * (q >> 1), h = q & 1;
        if (h == 0) { u0 = 0.0; u1 = 0.0; }
#pragma unroll
        for (int i = 0; i < 5; i++) {
          u0 += b[10 * h + 2 * i] * p[i].x;
          u1 += b[10 * h + 2 * i] * p[5 + i].x;
          u0 += b[10 * h + 2 * i + 1] * p[i].y;
          u1 += b[10 * h + 2 * i + 1] * p[5 + i].y;
        }
        if (h == 1) { U[k] = U[k] * u0; U[k + 1] = U[k + 1] * u1; }
        return u0;
      });
    }
    double O[S];
#pragma unroll
    for (int l = 0; l < S; l++) O[l] = 0.0;
    phase1(mE, [&](int k, const f64x2 (&e)[10]) {
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
    __syncthreads();
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
      if (sc) acc += wgt ? (long long)wgt[site] : 1ll;
    }
    __syncthreads();
    tile_store<double>(x3, base, n, tile);
    __syncthreads();
  }
  block_ticket_sum(acc, ws, scaler_sum);
}

// Phases 1 and 2 merged (two independent add chains per row: u1 over x1 and
// P_L, u2 over x2 and P_R), half rows streamed one ahead; phase 3 as before.
template <int kMinBlocks = 2>
__global__ void __launch_bounds__(kBlock, kMinBlocks)
prot_ldsmat_c_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                     double *__restrict__ x3, const double *__restrict__ EV,
                     const double *__restrict__ left, const double *__restrict__ right,
                     const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n,
                     unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  __shared__ f64x2 mats[(2 * 4 * S * S + S * S) / 2];
  {
    const f64x2 *gl = reinterpret_cast<const f64x2 *>(left);
    const f64x2 *gr = reinterpret_cast<const f64x2 *>(right);
    const f64x2 *ge = reinterpret_cast<const f64x2 *>(EV);
    for (int i = threadIdx.x; i < 800; i += kBlock) { mats[i] = gl[i]; mats[800 + i] = gr[i]; }
    for (int i = threadIdx.x; i < 200; i += kBlock) mats[1600 + i] = ge[i];
  }
  const double m = Num<double>::minlik();
  __shared__ PT::V tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  long long acc = 0;
  __syncthreads();
  for (int64_t base = (int64_t)blockIdx.x * 64; base < n; base += (int64_t)gridDim.x * 64) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const f64x2 *mL = mats + off + c * 200, *mR = mats + off + 800 + c * 200, *mE = mats + off + 1600;
    double a[S], b[S], U[S];
    tile_load<double>(x1, base, n, tile);
    __syncthreads();
    row_read<double>(tile, lane, c, a);
    __syncthreads();
    tile_load<double>(x2, base, n, tile);
    __syncthreads();
    row_read<double>(tile, lane, c, b);
    {
      // half row q of both matrices: row q>>1, values 10*(q&1) .. +9
      f64x2 cl[5], cr[5], nl[5], nr[5];
      int o = 0;
      double tok = 0.0, u1 = 0.0, u2 = 0.0;
#pragma unroll
      for (int i = 0; i < 5; i++) { cl[i] = mL[i]; cr[i] = mR[i]; }
#pragma unroll
      for (int q = 0; q < 2 * S; q++) {
        asm volatile("" : "+v"(o) : "v"(tok));
        if (q + 1 < 2 * S) {
#pragma unroll
          for (int i = 0; i < 5; i++) { nl[i] = mL[o + (q + 1) * 5 + i]; nr[i] = mR[o + (q + 1) * 5 + i]; }
        }
        const int k = q >> 1, h = q & 1;
        if (h == 0) { u1 = 0.0; u2 = 0.0; }
#pragma unroll
        for (int i = 0; i < 5; i++) {
          u1 += a[10 * h + 2 * i] * cl[i].x;
          u2 += b[10 * h + 2 * i] * cr[i].x;
          u1 += a[10 * h + 2 * i + 1] * cl[i].y;
          u2 += b[10 * h + 2 * i + 1] * cr[i].y;
        }
        if (h == 1) U[k] = u1 * u2;
        tok = u1;
#pragma unroll
        for (int i = 0; i < 5; i++) { cl[i] = nl[i]; cr[i] = nr[i]; }
      }
    }
    double O[S];
#pragma unroll
    for (int l = 0; l < S; l++) O[l] = 0.0;
    {
      f64x2 cur[10], nxt[10];
      int o = 0;
      double tok = 0.0;
#pragma unroll
      for (int i = 0; i < 10; i++) cur[i] = mE[i];
#pragma unroll
      for (int k = 0; k < S; k++) {
        asm volatile("" : "+v"(o) : "v"(tok));
        if (k + 1 < S) {
#pragma unroll
          for (int i = 0; i < 10; i++) nxt[i] = mE[o + (k + 1) * 10 + i];
        }
#pragma unroll
        for (int i = 0; i < 10; i++) {
          O[2 * i] += U[k] * cur[i].x;
          O[2 * i + 1] += U[k] * cur[i].y;
        }
        tok = O[S - 1];
#pragma unroll
        for (int i = 0; i < 10; i++) cur[i] = nxt[i];
      }
    }
    bool small = base + lane < n;
#pragma unroll
    for (int l = 0; l < S; l++) small = small && (__builtin_fabs(O[l]) < m);
    const unsigned long long mk = __ballot(small);
    if (lane == 0) small_mask[c] = mk;
    __syncthreads();
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
      if (sc) acc += wgt ? (long long)wgt[site] : 1ll;
    }
    __syncthreads();
    tile_store<double>(x3, base, n, tile);
    __syncthreads();
  }
  block_ticket_sum(acc, ws, scaler_sum);
}

// ---------------------------------------------------------------------------
// Measured and not adopted (profiles/r01_tune_protein_ring.log): with static
// wait counts it keeps two tiles in flight per block, but at 2 blocks/CU it
// ties the product kernel (91 us); the tile traffic structure alone runs at
// 83-85 us, so the rest is the MFMA phases' issue pattern, not bytes in flight.
// Branch-free tile traffic through buffer descriptors: one descriptor per tile
// whose range is the tile's valid sites, so the hardware range check returns 0
// for loads past n and drops stores past n.  Every thread then issues the same
// number of vector memory instructions on every trip, which lets the
// compiler's wait counting keep later loads in flight across a tile_put (the
// bounds-checked global form branches per chunk, and its unknown count makes
// the compiler wait for everything).  A tile past n gets an empty range: its
// loads are issued (keeping the count static) but move no data.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const double *g, int64_t base,
                                                             int64_t n) {
  const int64_t left = n - base, sites = left < 0 ? 0 : (left < 64 ? left : 64);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(g + base * 80), 0,
                                           (int)(sites * 640), 0x00020000);
}
template <int K>
__device__ __forceinline__ void tile_fetch_buf(__amdgpu_buffer_rsrc_t r, f64x2 (&v)[K]) {
#pragma unroll
  for (int i = 0; i < K; i++)  // aux 2 = nt
    v[i] = __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(
                                         r, (threadIdx.x + i * kBlock) * 16, 0, 2));
}

// Depth-2 ring form of plf_prot_mfma_kernel (same arithmetic, bit-identical): the
// A fragments are read from an LDS copy of the matrices at the start of each
// phase (20 VGPRs live instead of 60 for the whole kernel), which makes room
// for a second prefetch register set, so two child tiles are always in flight
// per block -- x2(i) and x1(i+1) during phase 1, x1(i+1) and x2(i+1) during
// phases 2 and 3 -- where the single set leaves gaps with none.
template <bool kSum, int kMinWaves = 2>
__global__ void __launch_bounds__(kBlock, kMinWaves)
plf_prot_mfma_ring_kernel(const double *__restrict__ x1, const double *__restrict__ x2,
                          double *__restrict__ x3, const double *__restrict__ EV,
                          const double *__restrict__ left, const double *__restrict__ right,
                          const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler,
                          int64_t n, unsigned long long *ws, int64_t *scaler_sum) {
  constexpr int S = 20;
  using PT = ProtTile<double>;
  constexpr int K = PT::kChunks / kBlock;
  constexpr int kRow = 2 * PT::kStride;  // doubles per site in the LDS tile (82)
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lo16 = lane & 15, g = lane >> 4;
  __shared__ double mats[2 * 4 * S * S + S * S];  // P_L[4][400] | P_R[4][400] | EV[400]
  for (int i = threadIdx.x; i < 4 * S * S; i += kBlock) {
    mats[i] = left[i];
    mats[4 * S * S + i] = right[i];
  }
  for (int i = threadIdx.x; i < S * S; i += kBlock) mats[8 * S * S + i] = EV[i];
  // A fragment rows/cols of this lane: [0][s] 16x16x4 (row lo16), [1][s] 4x4x4_4b (row 16 + lane%4)
  const int rA0 = lo16, rA1 = 16 + (lane & 3);
  const double m = Num<double>::minlik();
  __shared__ f64x2 tile[64 * PT::kStride];
  __shared__ unsigned long long small_mask[kWavesPerBlock];
  const double *td = reinterpret_cast<const double *>(tile);
  double *tw = reinterpret_cast<double *>(tile);
  long long acc = 0;
  f64x2 pfA[K], pfB[K];  // x1 / x2 tiles in flight
  const int64_t stride = (int64_t)gridDim.x * 64;
  const int64_t first = (int64_t)blockIdx.x * 64;
  tile_fetch_buf(tile_rsrc(x1, first, n), pfA);
  tile_fetch_buf(tile_rsrc(x2, first, n), pfB);
  {  // the trip's trailing stores, mimicked with an empty range (they move no data), so
     // the loop entry and the back edge see the same vector-memory counts: the compiler
     // merges the two and would otherwise wait for both prefetched tiles every trip
    const __amdgpu_buffer_rsrc_t er = __builtin_amdgcn_make_buffer_rsrc(x3, 0, 0, 0x00020000);
    if (c == 0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, er, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < K; i++) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0, 0, 0, 0}, er, 0, 0, 2);
  }
  __syncthreads();  // mats
  for (int64_t base = first; base < n; base += stride) {
    int z = 0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));  // keeps the fragment reads per phase
    const double *mL = mats + z + c * S * S, *mR = mats + z + 4 * S * S + c * S * S;
    const double *mE = mats + z + 8 * S * S;
    // this trip's site weights, issued before the prefetches so that waiting
    // for them does not wait for the tiles in flight (the counter is in order)
    int wv = 0;
    if constexpr (kSum) {
      const int64_t vs = n - base < 64 ? n - base : 64;
      const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t *>(wgt ? wgt + base : wgt), 0, wgt ? (int)(vs * 4) : 0, 0x00020000);
      wv = __builtin_amdgcn_raw_buffer_load_b32(wr, lane * 4, 0, 0);
    }
    f64x4 P[4][2];
    tile_put<double>(tile, pfA);
    __syncthreads();
    tile_fetch_buf(tile_rsrc(x1, base + stride, n), pfA);  // unconditional: see tile_rsrc
    {
      double A[2][5];
#pragma unroll
      for (int st = 0; st < 5; st++) {
        A[0][st] = mL[rA0 * S + 4 * st + g];
        A[1][st] = mL[rA1 * S + 4 * st + g];
      }
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const double *xr = td + (16 * t + lo16) * kRow + c * S + g;
        f64x4 u = {0.0, 0.0, 0.0, 0.0}, v = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 5; st++) {
          u = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0][st], xr[4 * st], u, 0, 0, 0);
          v[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[1][st], xr[4 * st], v[0], 0, 0, 0);
        }
        P[t][0] = u;
        P[t][1] = v;
      }
    }
    __syncthreads();
    tile_put<double>(tile, pfB);
    __syncthreads();
    tile_fetch_buf(tile_rsrc(x2, base + stride, n), pfB);
    {
      double A[2][5];
#pragma unroll
      for (int st = 0; st < 5; st++) {
        A[0][st] = mR[rA0 * S + 4 * st + g];
        A[1][st] = mR[rA1 * S + 4 * st + g];
      }
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const double *xr = td + (16 * t + lo16) * kRow + c * S + g;
        f64x4 u = {0.0, 0.0, 0.0, 0.0}, v = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 5; st++) {
          u = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0][st], xr[4 * st], u, 0, 0, 0);
          v[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[1][st], xr[4 * st], v[0], 0, 0, 0);
        }
        P[t][0] = P[t][0] * u;  // prod[k] = umpL[k] * umpR[k]
        P[t][1] = P[t][1] * v;
      }
    }
    __syncthreads();  // every wave is done reading x2: the tile takes X3 now
    unsigned long long mine = 0;
    {
      double A[2][5];  // EV^T[l = row][k = col]
#pragma unroll
      for (int st = 0; st < 5; st++) {
        A[0][st] = mE[(4 * st + g) * S + rA0];
        A[1][st] = mE[(4 * st + g) * S + rA1];
      }
#pragma unroll
      for (int t = 0; t < 4; t++) {
        f64x4 X0 = {0.0, 0.0, 0.0, 0.0};
        double X1 = 0.0;
#pragma unroll
        for (int st = 0; st < 5; st++) {
          X0 = __builtin_amdgcn_mfma_f64_16x16x4f64(A[0][st], P[t][st >> 2][st & 3], X0, 0, 0, 0);
          X1 = __builtin_amdgcn_mfma_f64_4x4x4f64(A[1][st], P[t][st >> 2][st & 3], X1, 0, 0, 0);
        }
        const bool small = (__builtin_fabs(X0[0]) < m) && (__builtin_fabs(X0[1]) < m) &&
                           (__builtin_fabs(X0[2]) < m) && (__builtin_fabs(X0[3]) < m) &&
                           (__builtin_fabs(X1) < m);
        const unsigned long long b = __ballot(small);
        mine |= (b & (b >> 16) & (b >> 32) & (b >> 48) & 0xFFFFull) << (16 * t);
        double *w = tw + (16 * t + lo16) * kRow + c * S;
#pragma unroll
        for (int r = 0; r < 4; r++) w[g + 4 * r] = X0[r];
        w[16 + g] = X1;
      }
    }
    if (lane == 0) small_mask[c] = mine;
    __syncthreads();
    const unsigned long long all = small_mask[0] & small_mask[1] & small_mask[2] & small_mask[3];
    if (c == 0) {  // scaler bytes through a range-checked descriptor (no divergent store)
      const bool sc = (all >> lane) & 1ull;
      const int64_t vs = n - base < 64 ? n - base : 64;
      const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
          scaler ? scaler + base : scaler, 0, scaler ? (int)vs : 0, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)sc, sr, lane, 0, 0);
      if (kSum && sc && base + lane < n) acc += wgt ? (long long)wv : 1ll;
    }
    {
      const __amdgpu_buffer_rsrc_t r = tile_rsrc(x3, base, n);
#pragma unroll
      for (int i = 0; i < K; i++) {
        const int j = threadIdx.x + i * kBlock;
        const int sl = j / PT::kChunksPerSite, q = j - sl * PT::kChunksPerSite;
        f64x2 v = tile[sl * PT::kStride + q];
        if ((all >> sl) & 1ull) v = v * Num<double>::two32();
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, j * 16, 0, 2);
      }
    }
    __syncthreads();
  }
  if constexpr (kSum) block_ticket_sum(acc, ws, scaler_sum);
}

}  // namespace dev
}  // namespace plfx
