// tune_pair2.hip -- tuning only: headline DNA f64 node kernel variants with
// the P/EV matrices in LDS instead of 48 VGPRs (read once per matrix per trip,
// shared by the trip's four 8-site blocks), with and without software
// pipelining (the next trip's CLV loads issued before this trip's math).
// Same lane map and per-value operation order as csrc dna_pair_body, checked
// bit-for-bit against it before timing.  Interleaved with the csrc kernel and
// a 2-read/1-write stream over 4 rotating buffer sets (> Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I amd-versal-phylogenetic-likelihood-function_amd/csrc tools/tune_pair2.hip -o build/tune_pair2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "plf_dna.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using namespace plfx::dev;

__device__ __forceinline__ int opaque0() {
  int z = 0;
  asm volatile("; opaque %0" : "+v"(z));
  return z;
}

// n must be a multiple of 16*U*4 (full trips only; tuning harness)
template <int U, bool PIPE, int MINW>
__global__ void __launch_bounds__(256, MINW)
pair_lds(const double *__restrict__ x1, const double *__restrict__ x2, double *__restrict__ x3,
         const double *__restrict__ EV, const double *__restrict__ left, const double *__restrict__ right,
         const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n, unsigned long long *ws,
         int64_t *scaler_sum) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 1, c = (lane >> 1) & 3, g = lane >> 3, sh = lane & 56;
  // sM[0..63] = left, [64..127] = right, [128 + h*16 + k*2 + t] = EV[4k + 2h + t]
  __shared__ __attribute__((aligned(16))) double sM[160];
  if (threadIdx.x < 64) sM[threadIdx.x] = left[threadIdx.x];
  else if (threadIdx.x < 128) sM[threadIdx.x] = right[threadIdx.x - 64];
  else if (threadIdx.x < 160) {
    const int i = threadIdx.x - 128, hh = i >> 4, k = (i >> 1) & 7, t = i & 1;
    sM[threadIdx.x] = EV[4 * (k & 3) + 2 * hh + t];
  }
  __syncthreads();
  const int pofs = c * 16 + 2 * h * 4;  // rows 2h, 2h+1 of P_c: 8 contiguous doubles
  const int eofs = 128 + h * 16;
  const double m = Num<double>::minlik();
  long long acc = 0;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 4 * 16 * U;
  constexpr int B = 2 * U;  // 8-site blocks per trip

  f64x2 a[B], b[B];
  int w[B];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int i = 0; i < B; i++) {
      const int64_t site0 = base + i * 8;
      a[i] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(x1 + site0 * 16) + lane);
      b[i] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(x2 + site0 * 16) + lane);
      w[i] = wgt ? wgt[site0 + g] : 1;
    }
  };
  auto compute = [&](int64_t base, const f64x2 (&A)[B], const f64x2 (&Bv)[B], const int (&W)[B]) {
    const int z = opaque0();
    const double *pm = sM + z;
    double u1[B][2], u2[B][2];
    {
      double P[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int l = 0; l < 4; l++) P[kk][l] = pm[pofs + kk * 4 + l];
#pragma unroll
      for (int i = 0; i < B; i++) {
        const double a0 = dpp_f64<kQuadEven>(A[i].x), a1 = dpp_f64<kQuadEven>(A[i].y);
        const double a2 = dpp_f64<kQuadOdd>(A[i].x), a3 = dpp_f64<kQuadOdd>(A[i].y);
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
          double v = 0.0;
          v += a0 * P[kk][0]; v += a1 * P[kk][1]; v += a2 * P[kk][2]; v += a3 * P[kk][3];
          u1[i][kk] = v;
        }
      }
    }
    {
      double P[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int l = 0; l < 4; l++) P[kk][l] = pm[64 + pofs + kk * 4 + l];
#pragma unroll
      for (int i = 0; i < B; i++) {
        const double b0 = dpp_f64<kQuadEven>(Bv[i].x), b1 = dpp_f64<kQuadEven>(Bv[i].y);
        const double b2 = dpp_f64<kQuadOdd>(Bv[i].x), b3 = dpp_f64<kQuadOdd>(Bv[i].y);
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
          double v = 0.0;
          v += b0 * P[kk][0]; v += b1 * P[kk][1]; v += b2 * P[kk][2]; v += b3 * P[kk][3];
          u2[i][kk] = v;
        }
      }
    }
    double E[4][2];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int t = 0; t < 2; t++) E[k][t] = pm[eofs + k * 2 + t];
#pragma unroll
    for (int i = 0; i < B; i++) {
      const int64_t site0 = base + i * 8;
      double p[2];
#pragma unroll
      for (int kk = 0; kk < 2; kk++) p[kk] = u1[i][kk] * u2[i][kk];
      const double p0 = dpp_f64<kQuadEven>(p[0]), p1 = dpp_f64<kQuadEven>(p[1]);
      const double p2 = dpp_f64<kQuadOdd>(p[0]), p3 = dpp_f64<kQuadOdd>(p[1]);
      double o[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        double x = 0.0;
        x += p0 * E[0][t]; x += p1 * E[1][t]; x += p2 * E[2][t]; x += p3 * E[3][t];
        o[t] = x;
      }
      const bool small = (__builtin_fabs(o[0]) < m) && (__builtin_fabs(o[1]) < m);
      const unsigned long long mask = __ballot(small);
      const bool sc = ((mask >> sh) & 0xFFull) == 0xFFull;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const double s = o[t] * Num<double>::two32();
        o[t] = sc ? s : o[t];
      }
      f64x2 ov = {o[0], o[1]};
      __builtin_nontemporal_store(ov, reinterpret_cast<f64x2 *>(x3 + site0 * 16) + lane);
      if ((lane & 7) == 0) {
        if (scaler) scaler[site0 + g] = (uint8_t)sc;
        if (sc) acc += W[i];
      }
    }
  };
  int64_t base = wave * 16 * U;
  if constexpr (PIPE) {
    if (base < n) load(base);
    for (; base < n; base += stride) {
      f64x2 ca[B], cb[B];
      int cw[B];
#pragma unroll
      for (int i = 0; i < B; i++) { ca[i] = a[i]; cb[i] = b[i]; cw[i] = w[i]; }
      if (base + stride < n) load(base + stride);
      compute(base, ca, cb, cw);
    }
  } else {
    for (; base < n; base += stride) {
      load(base);
      compute(base, a, b, w);
    }
  }
  block_ticket_sum(acc, ws, scaler_sum);
}


// Wave-level dynamic scheduling inside a block: the block owns the wave-trip
// chunks ((k * gridDim.x + blockIdx.x) * WPB + s) * 16U, k = 0, 1, ...,
// s < WPB (the same sweep order as the grid-stride kernels), and its waves
// claim them in order from an LDS counter, so a wave the memory system serves
// faster takes more of them.  n must be a multiple of 16U (tuning harness).
template <int BLK, int U>
__global__ void __launch_bounds__(BLK, 1)
pair_q(const double *__restrict__ x1, const double *__restrict__ x2, double *__restrict__ x3,
       const double *__restrict__ EV, const double *__restrict__ left, const double *__restrict__ right,
       const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n, unsigned long long *ws,
       int64_t *scaler_sum) {
  constexpr int WPB = BLK / 64;
  const int lane = threadIdx.x & 63;
  const int h = lane & 1, c = (lane >> 1) & 3, g = lane >> 3, sh = lane & 56;
  __shared__ int ctr;
  __shared__ long long part[WPB];
  if (threadIdx.x == 0) ctr = 0;
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
  __syncthreads();
  const double m = Num<double>::minlik();
  long long acc = 0;
  int idx = threadIdx.x >> 6;  // first chunk: static
  auto site_of = [&](int i) -> int64_t {
    return (((int64_t)(i / WPB) * gridDim.x + blockIdx.x) * WPB + (i % WPB)) * (16 * U);
  };
  for (int64_t base = site_of(idx); base < n; ) {
    int nx = 0;
    if (lane == 0) nx = atomicAdd(&ctr, 1);
    f64x2 a[U][2], b[U][2];
    int w[U][2];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int64_t site0 = base + u * 16 + j * 8;
        a[u][j] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(x1 + site0 * 16) + lane);
        b[u][j] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(x2 + site0 * 16) + lane);
        w[u][j] = wgt ? wgt[site0 + g] : 1;
      }
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int64_t site0 = base + u * 16 + j * 8;
        const double a0 = dpp_f64<kQuadEven>(a[u][j].x), a1 = dpp_f64<kQuadEven>(a[u][j].y);
        const double a2 = dpp_f64<kQuadOdd>(a[u][j].x), a3 = dpp_f64<kQuadOdd>(a[u][j].y);
        const double b0 = dpp_f64<kQuadEven>(b[u][j].x), b1 = dpp_f64<kQuadEven>(b[u][j].y);
        const double b2 = dpp_f64<kQuadOdd>(b[u][j].x), b3 = dpp_f64<kQuadOdd>(b[u][j].y);
        double pm[2];
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
          double v = a0 * PL[kk][0];
          v += a1 * PL[kk][1]; v += a2 * PL[kk][2]; v += a3 * PL[kk][3];
          double y = b0 * PR[kk][0];
          y += b1 * PR[kk][1]; y += b2 * PR[kk][2]; y += b3 * PR[kk][3];
          pm[kk] = v * y;
        }
        const double p0 = dpp_f64<kQuadEven>(pm[0]), p1 = dpp_f64<kQuadEven>(pm[1]);
        const double p2 = dpp_f64<kQuadOdd>(pm[0]), p3 = dpp_f64<kQuadOdd>(pm[1]);
        double o[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
          double x = 0.0;
          x += p0 * E[0][t]; x += p1 * E[1][t]; x += p2 * E[2][t]; x += p3 * E[3][t];
          o[t] = x;
        }
        const bool small = (__builtin_fabs(o[0]) < m) && (__builtin_fabs(o[1]) < m);
        const unsigned long long mask = __ballot(small);
        const bool sc = ((mask >> sh) & 0xFFull) == 0xFFull;
#pragma unroll
        for (int t = 0; t < 2; t++) {
          const double s2 = o[t] * Num<double>::two32();
          o[t] = sc ? s2 : o[t];
        }
        f64x2 ov = {o[0], o[1]};
        __builtin_nontemporal_store(ov, reinterpret_cast<f64x2 *>(x3 + site0 * 16) + lane);
        if ((lane & 7) == 0) {
          if (scaler) scaler[site0 + g] = (uint8_t)sc;
          if (sc) acc += w[u][j];
        }
      }
    idx = __builtin_amdgcn_readfirstlane(nx) + WPB;
    base = site_of(idx);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x != 0) return;
  long long tot = 0;
  for (int i = 0; i < WPB; i++) tot += part[i];
  ticket_publish(tot, ws, scaler_sum);
}


// Rolling prefetch ("ring"): the trip's 2U 8-site blocks are loaded one trip
// ahead, block by block -- block i of the next trip is issued right after
// block i of this trip is computed -- so every wave keeps ~2U blocks of loads
// in flight at all times without a second register set.  Loop trips issue
// their next loads unconditionally (exact vmcnt waits); the last trip of a
// wave runs as an epilogue without loads.  Full trips only (tuning harness).
template <int U, int MINW>
__global__ void __launch_bounds__(256, MINW)
pair_ring(const double *__restrict__ x1, const double *__restrict__ x2, double *__restrict__ x3,
          const double *__restrict__ EV, const double *__restrict__ left, const double *__restrict__ right,
          const int32_t *__restrict__ wgt, uint8_t *__restrict__ scaler, int64_t n, unsigned long long *ws,
          int64_t *scaler_sum) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 1, c = (lane >> 1) & 3, g = lane >> 3, sh = lane & 56;
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
  constexpr int B = 2 * U;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 4 * 16 * U;
  const int64_t first = wave * 16 * U;
  if (first >= n) { block_ticket_sum(0, ws, scaler_sum); return; }
  const int64_t trips = (n - first + stride - 1) / stride;  // >= 1
  f64x2 a[B], b[B];
  int w[B];
  auto load = [&](int i, int64_t base) {
    const int64_t site0 = base + i * 8;
    a[i] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(x1 + site0 * 16) + lane);
    b[i] = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(x2 + site0 * 16) + lane);
    w[i] = wgt_at(wgt, site0 + g, ws);
  };
  auto compute = [&](int i, int64_t base) {
    const int64_t site0 = base + i * 8;
    const double a0 = dpp_f64<kQuadEven>(a[i].x), a1 = dpp_f64<kQuadEven>(a[i].y);
    const double a2 = dpp_f64<kQuadOdd>(a[i].x), a3 = dpp_f64<kQuadOdd>(a[i].y);
    const double b0 = dpp_f64<kQuadEven>(b[i].x), b1 = dpp_f64<kQuadEven>(b[i].y);
    const double b2 = dpp_f64<kQuadOdd>(b[i].x), b3 = dpp_f64<kQuadOdd>(b[i].y);
    double pm[2];
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      double v = a0 * PL[kk][0];
      v += a1 * PL[kk][1]; v += a2 * PL[kk][2]; v += a3 * PL[kk][3];
      double y = b0 * PR[kk][0];
      y += b1 * PR[kk][1]; y += b2 * PR[kk][2]; y += b3 * PR[kk][3];
      pm[kk] = v * y;
    }
    const double p0 = dpp_f64<kQuadEven>(pm[0]), p1 = dpp_f64<kQuadEven>(pm[1]);
    const double p2 = dpp_f64<kQuadOdd>(pm[0]), p3 = dpp_f64<kQuadOdd>(pm[1]);
    double o[2];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      double x = 0.0;
      x += p0 * E[0][t]; x += p1 * E[1][t]; x += p2 * E[2][t]; x += p3 * E[3][t];
      o[t] = x;
    }
    const bool small = (__builtin_fabs(o[0]) < m) && (__builtin_fabs(o[1]) < m);
    const unsigned long long mask = __ballot(small);
    const bool sc = ((mask >> sh) & 0xFFull) == 0xFFull;
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const double s2 = o[t] * Num<double>::two32();
      o[t] = sc ? s2 : o[t];
    }
    f64x2 ov = {o[0], o[1]};
    __builtin_nontemporal_store(ov, reinterpret_cast<f64x2 *>(x3 + site0 * 16) + lane);
    if ((lane & 7) == 0) {
      if (scaler) scaler[site0 + g] = (uint8_t)sc;
      if (sc) acc += w[i];
    }
  };
  int64_t base = first;
#pragma unroll
  for (int i = 0; i < B; i++) load(i, base);
  for (int64_t t = 1; t < trips; t++, base += stride) {
#pragma unroll
    for (int i = 0; i < B; i++) {
      compute(i, base);
      load(i, base + stride);
    }
  }
#pragma unroll
  for (int i = 0; i < B; i++) compute(i, base);
  block_ticket_sum(acc, ws, scaler_sum);
}

__global__ void fill(double *p, int64_t n, uint64_t seed, double scale4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    double v = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    if (scale4 != 1.0 && ((i / 16) % 4) == 0) v *= scale4;
    p[i] = v;
  }
}

typedef double f64x2v __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) stream3(const f64x2v *__restrict__ a, const f64x2v *__restrict__ b,
                                               f64x2v *__restrict__ c, int64_t nrec) {
  constexpr int V = 4;
  const int64_t stride = (int64_t)gridDim.x * 256 * V;
  for (int64_t i = (int64_t)blockIdx.x * 256 * V + threadIdx.x; i < nrec; i += stride) {
    f64x2v x[V], y[V];
#pragma unroll
    for (int v = 0; v < V; v++) {
      x[v] = __builtin_nontemporal_load(a + i + 256 * v);
      y[v] = __builtin_nontemporal_load(b + i + 256 * v);
    }
#pragma unroll
    for (int v = 0; v < V; v++) __builtin_nontemporal_store(x[v] + y[v], c + i + 256 * v);
  }
}

__global__ void __launch_bounds__(256) stream1(const f64x2v *__restrict__ a, const f64x2v *__restrict__ b,
                                               f64x2v *__restrict__ c, int64_t nrec) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nrec; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i), c + i);
}

struct Set { double *x1, *x2, *x3; int *wgt; uint8_t *sc; int64_t *sum; };

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const int reps = argc > 2 ? atoi(argv[2]) : 40, rounds = 5, R = 4;
  if (n % 512) { printf("n must be a multiple of 512\n"); return 1; }
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  double *EV, *L, *Rm; unsigned long long *ws;
  CK(hipMalloc(&EV, 16 * 8)); CK(hipMalloc(&L, 64 * 8)); CK(hipMalloc(&Rm, 64 * 8));
  CK(hipMalloc(&ws, kWsWords * 8)); CK(hipMemset(ws, 0, kWsWords * 8));
  fill<<<1, 64>>>(EV, 16, 1, 1.0); fill<<<1, 64>>>(L, 64, 2, 1.0); fill<<<1, 64>>>(Rm, 64, 3, 1.0);
  std::vector<Set> sets(R);
  for (int r = 0; r < R; r++) {
    Set &s = sets[r];
    CK(hipMalloc(&s.x1, n * 128)); CK(hipMalloc(&s.x2, n * 128)); CK(hipMalloc(&s.x3, n * 128));
    CK(hipMalloc(&s.wgt, n * 4)); CK(hipMalloc(&s.sc, n)); CK(hipMalloc(&s.sum, 8));
    fill<<<2048, 256>>>(s.x1, n * 16, 10 + r, 1e-12);
    fill<<<2048, 256>>>(s.x2, n * 16, 20 + r, 1.0);
    std::vector<int> wv(n);
    for (int64_t i = 0; i < n; i++) wv[i] = 1 + (int)(i % 3);
    CK(hipMemcpy(s.wgt, wv.data(), n * 4, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  auto occ = [&](const void *k) { int b = 0; CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, 256, 0)); return b; };
  struct V { std::string name; double bytes; std::function<void(const Set &)> run; std::vector<float> us; };
  std::vector<V> vs;
  vs.push_back({"stream 2R+1W V=4 grid 4/CU", 384.0 * n, [&](const Set &s) {
    stream3<<<CUs * 4, 256>>>((const f64x2v *)s.x1, (const f64x2v *)s.x2, (f64x2v *)s.x3, n * 8); }, {}});
  vs.push_back({"stream 2R+1W V=1 grid 2/CU", 384.0 * n, [&](const Set &s) {
    stream1<<<CUs * 2, 256>>>((const f64x2v *)s.x1, (const f64x2v *)s.x2, (f64x2v *)s.x3, n * 8); }, {}});
  std::vector<std::string> checkme;
#define ADD(NAME, K, MUL)                                                                          \
  {                                                                                                \
    auto k = K;                                                                                    \
    const int o = occ((const void *)k);                                                            \
    const int64_t grid = std::min<int64_t>((n + 127) / 128, (int64_t)(o * CUs * MUL));               \
    vs.push_back({std::string(NAME) + " occ " + std::to_string(o) + " grid " + std::to_string(grid), 389.0 * n, \
                  [=](const Set &s) {                                                              \
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,    \
                         s.wgt, s.sc, n, ws, s.sum); }, {}});                                      \
  }
#define ADDB(NAME, K, BLK, PER)                                                                    \
  {                                                                                                \
    auto k = K;                                                                                    \
    const int64_t grid = (int64_t)PER * CUs;                                                       \
    vs.push_back({std::string(NAME) + " grid " + std::to_string(grid), 389.0 * n, [=](const Set &s) { \
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(BLK), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,    \
                         s.wgt, s.sc, n, ws, s.sum); }, {}});                                      \
  }
  ADD("csrc pair U=2", (&plf_dna_f64_pair_kernel<2, true, 1, true>), 1)
  ADD("csrc pair U=2 x0.5", (&plf_dna_f64_pair_kernel<2, true, 1, true>), 0.5)
  ADD("csrc pair U=2 x0.75", (&plf_dna_f64_pair_kernel<2, true, 1, true>), 0.75)
  ADD("csrc pair U=1 x1", (&plf_dna_f64_pair_kernel<1, true, 1, true>), 1)
  ADD("csrc pair U=1 x0.5", (&plf_dna_f64_pair_kernel<1, true, 1, true>), 0.5)
  ADD("csrc pair U=1 x0.25", (&plf_dna_f64_pair_kernel<1, true, 1, true>), 0.25)
  ADD("csrc pair U=1 x0.375", (&plf_dna_f64_pair_kernel<1, true, 1, true>), 0.375)
  ADD("csrc pair U=1 x0.75", (&plf_dna_f64_pair_kernel<1, true, 1, true>), 0.75)
  ADD("lds U=1 pipe x0.5", (&pair_lds<1, true, 1>), 0.5)
  ADD("lds U=1 pipe x0.375", (&pair_lds<1, true, 1>), 0.375)
  ADD("ring U=1 x0.5", (&pair_ring<1, 1>), 0.5)
  ADD("ring U=1 x0.25", (&pair_ring<1, 1>), 0.25)

  // bit-exact check of every variant against the csrc kernel on set 0
  {
    const size_t bytes = n * 128;
    std::vector<char> ref(bytes), got(bytes), rsc(n), gsc(n);
    int64_t rsum = 0, gsum = 0;
    vs[2].run(sets[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), sets[0].x3, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rsc.data(), sets[0].sc, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&rsum, sets[0].sum, 8, hipMemcpyDeviceToHost));
    for (size_t i = 3; i < vs.size(); i++) {
      CK(hipMemset(sets[0].x3, 0xFF, bytes)); CK(hipMemset(sets[0].sc, 7, n)); CK(hipMemset(sets[0].sum, 0, 8));
      vs[i].run(sets[0]);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), sets[0].x3, bytes, hipMemcpyDeviceToHost));
      CK(hipMemcpy(gsc.data(), sets[0].sc, n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&gsum, sets[0].sum, 8, hipMemcpyDeviceToHost));
      const bool ok = !memcmp(ref.data(), got.data(), bytes) && !memcmp(rsc.data(), gsc.data(), n) && rsum == gsum;
      printf("check %-40s %s (sum %lld vs %lld)\n", vs[i].name.c_str(), ok ? "bit-exact" : "MISMATCH",
             (long long)gsum, (long long)rsum);
    }
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs) {
      for (int i = 0; i < 3; i++) v.run(sets[i % R]);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; i++) v.run(sets[i % R]);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / reps);
    }
  CK(hipGetLastError());
  printf("n=%lld sites, %d reps x %d rounds interleaved, %d buffer sets\n", (long long)n, reps, rounds, R);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6;
    printf("%-44s median %8.2f us (min %8.2f)  %5.1f%% of 8 TB/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           v.us[0], 100.0 * v.bytes / t / 8e12);
  }
  return 0;
}
