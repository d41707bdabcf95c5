// Same-process A/B of the exact-mode protein node kernel (f64, S = 20, C = 4;
// plf()'s separate multiply and add) at more waves per SIMD (VERDICT r05,
// next-round item 4):
//   A   plf_prot_lds_kernel<double, kSum, 2, 0, 10, true>      product: 256-thread
//       blocks, one 64-site tile, 70.8 KB LDS -> 2 blocks = 2 waves per SIMD
//   B   <..., kMinWaves 3, kRows 10, kTiles 3>  768-thread blocks, three 64-site
//       tiles sharing one LDS copy of the matrices (155 KB) -> 3 waves per SIMD
//       (VGPRs capped at 168 by the launch bounds)
//   C   as B with 4-row chains (fewer live registers per chain group)
//   D   as B with 2-row chains
// The tile-group form (kTiles = 3) also reads each child row from the LDS
// tile per column pair instead of 20 registers, runs phase 3 as 4-state
// passes whose values go straight to the tile, and rescales on the way out
// (tile_store_scaled): the register cuts that fit 168 VGPRs (B/C/D spill
// 140/42/26 VGPRs to scratch at that cap, mostly outside the inner loops).
// Every variant is checked bit for bit against A (x3, scaler bytes, scaler
// sum) before it is timed.  Timing: hipEvents over `reps` launches rotating 4
// buffer sets (> the 256-MiB Infinity Cache), after a warm-up of the same
// length, variants alternating, 3 rounds.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I amd-versal-phylogenetic-likelihood-function_amd/csrc tools/ab_prot_tiles.hip -o build/ab_prot_tiles
//   build/ab_prot_tiles [sites ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "plf_prot.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

using namespace plfx::dev;

typedef void (*ProtK)(const double *, const double *, double *, const double *, const double *,
                      const double *, const int32_t *, uint8_t *, int64_t, unsigned long long *, int64_t *,
                      const double *);

struct Var {
  const char *name;
  ProtK k;
  int threads, tiles, per_cu;
};

struct Set {
  double *x1, *x2, *x3;
  uint8_t *sc;
  int64_t *sum;
};

int main(int argc, char **argv) {
  std::vector<long> sizes;
  for (int i = 1; i < argc; i++) sizes.push_back(std::atol(argv[i]));
  if (sizes.empty()) sizes = {1 << 18, 4099, 1 << 20};
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  Var vs[] = {
      {"A product", &plf_prot_lds_kernel<double, true, 2, 0, 10, true, 1>, 256, 1, 0},
      {"B 3 tiles r10", &plf_prot_lds_kernel<double, true, 3, 0, 10, true, 3>, 768, 3, 0},
      {"C 3 tiles r4", &plf_prot_lds_kernel<double, true, 3, 0, 4, true, 3>, 768, 3, 0},
      {"D 3 tiles r2", &plf_prot_lds_kernel<double, true, 3, 0, 2, true, 3>, 768, 3, 0},
  };
  const int nv = sizeof(vs) / sizeof(vs[0]);
  for (auto &v : vs) {
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void *)v.k));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&v.per_cu, (const void *)v.k, v.threads, 0));
    std::printf("# %-14s %d threads, %d VGPRs, %zu B scratch, %zu B LDS, %d block(s)/CU = %d waves/SIMD\n",
                v.name, v.threads, fa.numRegs, fa.localSizeBytes, fa.sharedSizeBytes, v.per_cu,
                v.per_cu * v.threads / 256);
  }
  std::mt19937_64 g(20250117);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<double> EV(400), L(1600), R(1600);
  for (auto &v : EV) v = U(g) - 0.25;
  for (auto &v : L) v = U(g);
  for (auto &v : R) v = U(g);
  double *dEV, *dL, *dR;
  CK(hipMalloc(&dEV, 400 * 8));
  CK(hipMalloc(&dL, 1600 * 8));
  CK(hipMalloc(&dR, 1600 * 8));
  CK(hipMemcpy(dEV, EV.data(), 400 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dL, L.data(), 1600 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dR, R.data(), 1600 * 8, hipMemcpyHostToDevice));
  unsigned long long *ws;
  CK(hipMalloc(&ws, 1 << 20));
  CK(hipMemset(ws, 0, 1 << 20));
  for (long n : sizes) {
    const size_t V = 80 * (size_t)n;
    std::vector<double> h1(V), h2(V);
    for (size_t i = 0; i < V; i++) {
      h1[i] = U(g) * ((i / 80) % 4 == 0 ? 1e-14 : 1.0);
      h2[i] = U(g);
    }
    std::vector<int> hw(n, 1);
    int *wgt;
    CK(hipMalloc(&wgt, n * 4));
    CK(hipMemcpy(wgt, hw.data(), n * 4, hipMemcpyHostToDevice));
    const int R4 = 4;
    Set set[R4];
    for (auto &s : set) {
      CK(hipMalloc(&s.x1, V * 8));
      CK(hipMalloc(&s.x2, V * 8));
      CK(hipMalloc(&s.x3, V * 8));
      CK(hipMalloc(&s.sc, n));
      CK(hipMalloc(&s.sum, 8));
      CK(hipMemcpy(s.x1, h1.data(), V * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(s.x2, h2.data(), V * 8, hipMemcpyHostToDevice));
    }
    auto run = [&](const Var &v, Set &s) {
      const long per_block = 64L * v.tiles;
      const long grid = std::max(1L, std::min<long>((n + per_block - 1) / per_block, (long)v.per_cu * cus));
      hipLaunchKernelGGL(v.k, dim3(grid), dim3(v.threads), 0, 0, s.x1, s.x2, s.x3, dEV, dL, dR, wgt, s.sc,
                         (int64_t)n, ws, s.sum, nullptr);
    };
    std::vector<double> a3(V), b3(V);
    std::vector<uint8_t> asc(n), bsc(n);
    int64_t asum = 0, bsum = 0;
    for (int k = 0; k < nv; k++) {
      CK(hipMemset(set[0].x3, 0, V * 8));
      CK(hipMemset(set[0].sc, 7, n));
      run(vs[k], set[0]);
      CK(hipDeviceSynchronize());
      std::vector<double> &o3 = k == 0 ? a3 : b3;
      std::vector<uint8_t> &osc = k == 0 ? asc : bsc;
      int64_t &os = k == 0 ? asum : bsum;
      CK(hipMemcpy(o3.data(), set[0].x3, V * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(osc.data(), set[0].sc, n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&os, set[0].sum, 8, hipMemcpyDeviceToHost));
      if (k == 0) continue;
      const bool same = std::memcmp(a3.data(), b3.data(), V * 8) == 0 &&
                        std::memcmp(asc.data(), bsc.data(), n) == 0 && asum == bsum;
      std::printf("n=%ld  %s vs A: %s (sums %lld / %lld)\n", n, vs[k].name, same ? "bit-identical" : "MISMATCH",
                  (long long)asum, (long long)bsum);
      if (!same) return 2;
    }
    const int reps = n >= (1 << 20) ? 200 : 800;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 3; round++) {
      for (int k = 0; k < nv; k++) {
        for (int i = 0; i < reps; i++) run(vs[k], set[i % R4]);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; i++) run(vs[k], set[i % R4]);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        std::printf("n=%ld round %d %-14s %8.2f us/launch  %.3f of 8 TB/s (1921 B/site)\n", n, round,
                    vs[k].name, us, 1921.0 * n / (us * 1e-6) / 8e12);
        std::fflush(stdout);
      }
    }
    for (auto &s : set) {
      CK(hipFree(s.x1));
      CK(hipFree(s.x2));
      CK(hipFree(s.x3));
      CK(hipFree(s.sc));
      CK(hipFree(s.sum));
    }
    CK(hipFree(wgt));
  }
  return 0;
}
