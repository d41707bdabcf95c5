// Same-process A/B of the exact-mode protein node kernels (f64, S = 20, C = 4):
//   A  plf_prot_lds_kernel<double, kSum, 2, 0, 10, true>  (the product form until round 4)
//   B  plf_prot_wt_kernel<double, kSum, kRows>            (wave-private tiles, tools/prot_wt.hpp)
// Both include the product headers; B is checked bit for bit against A (x3,
// scaler bytes, scaler sum) before anything is timed.  Timing: hipEvents over
// `reps` launches rotating 4 buffer sets (4 x 1.5 GB at 2^20 sites > the
// 256-MiB Infinity Cache), after a warm-up of the same length.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I amd-versal-phylogenetic-likelihood-function_amd/csrc -I tools tools/ab_prot_exact.hip -o build/ab_prot_exact
//     [-DB_ROWS=4|10 -DB_XL=false|true]
//   build/ab_prot_exact [sites ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "plf_prot.hpp"
#include "prot_wt.hpp"  // the variant under test (tools/)

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

using namespace plfx::dev;

struct Set {
  double *x1, *x2, *x3;
  uint8_t *sc;
  int64_t *sum;
};

int main(int argc, char **argv) {
  std::vector<long> sizes;
  for (int i = 1; i < argc; i++) sizes.push_back(std::atol(argv[i]));
  if (sizes.empty()) sizes = {1 << 18, 1 << 20, 4099};
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto kA = &plf_prot_lds_kernel<double, true, 2, 0, 10, true>;
#ifndef B_ROWS
#define B_ROWS 4
#endif
#ifndef B_XL
#define B_XL false
#endif
  auto kB = &plf_prot_wt_kernel<double, true, B_ROWS, 0, B_XL>;
  int occA = 0, occB = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occA, kA, kBlock, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occB, kB, kWtThreads, 0));
  hipFuncAttributes fa, fb;
  CK(hipFuncGetAttributes(&fa, (const void *)kA));
  CK(hipFuncGetAttributes(&fb, (const void *)kB));
  std::printf("A lds: %d blocks/CU, %d VGPR-regs?, lds %zu B | B wt: %d blocks/CU, lds %zu B\n", occA,
              fa.numRegs, fa.sharedSizeBytes, occB, fb.sharedSizeBytes);
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
  int *wgt;
  for (long n : sizes) {
    const size_t V = 80 * (size_t)n;
    std::vector<double> h1(V), h2(V);
    for (size_t i = 0; i < V; i++) {
      h1[i] = U(g) * ((i / 80) % 4 == 0 ? 1e-14 : 1.0);
      h2[i] = U(g);
    }
    std::vector<int> hw(n, 1);
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
    const long gA = std::min<long>((n + 63) / 64, (long)occA * cus);
    const long gB = std::min<long>((n + 16 * kWtWaves - 1) / (16 * kWtWaves), (long)occB * cus);
    auto runA = [&](Set &s) {
      hipLaunchKernelGGL(kA, dim3(gA), dim3(kBlock), 0, 0, s.x1, s.x2, s.x3, dEV, dL, dR, wgt, s.sc,
                         (int64_t)n, ws, s.sum, nullptr);
    };
    auto runB = [&](Set &s) {
      hipLaunchKernelGGL(kB, dim3(gB), dim3(kWtThreads), 0, 0, s.x1, s.x2, s.x3, dEV, dL, dR, wgt, s.sc,
                         (int64_t)n, ws + 4096, s.sum);
    };
    // correctness: B against A on set 0
    std::vector<double> a3(V), b3(V);
    std::vector<uint8_t> asc(n), bsc(n);
    int64_t asum = 0, bsum = 0;
    runA(set[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a3.data(), set[0].x3, V * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(asc.data(), set[0].sc, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&asum, set[0].sum, 8, hipMemcpyDeviceToHost));
    CK(hipMemset(set[0].x3, 0, V * 8));
    runB(set[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b3.data(), set[0].x3, V * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(bsc.data(), set[0].sc, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&bsum, set[0].sum, 8, hipMemcpyDeviceToHost));
    const bool same = std::memcmp(a3.data(), b3.data(), V * 8) == 0 &&
                      std::memcmp(asc.data(), bsc.data(), n) == 0 && asum == bsum;
    long nsc = 0;
    for (auto v : asc) nsc += v;
    std::printf("n=%ld  B vs A: %s (scaled sites %ld, sums %lld / %lld)\n", n, same ? "bit-identical" : "MISMATCH",
                nsc, (long long)asum, (long long)bsum);
    if (!same) {
      for (size_t i = 0; i < V; i++)
        if (std::memcmp(&a3[i], &b3[i], 8)) {
          std::printf("  first diff at site %zu value %zu: %.17g vs %.17g\n", i / 80, i % 80, a3[i], b3[i]);
          break;
        }
      return 2;
    }
    const int reps = n >= (1 << 20) ? 200 : 800;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 3; round++) {
      for (int which = 0; which < 2; which++) {
        auto run = [&](int i) { which ? runB(set[i % R4]) : runA(set[i % R4]); };
        for (int i = 0; i < reps; i++) run(i);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; i++) run(i);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        std::printf("  round %d %s: %8.2f us/launch  %.3f of 8 TB/s (1921 B/site)\n", round,
                    which ? "B wt " : "A lds", us, 1921.0 * n / (us * 1e-6) / 8e12);
      }
    }
    // timing ablations of B (not bit-checked): 1 no HBM traffic, 2 no LDS
    // matrix reads, 4 no phase 3, and their sums
    if (argc <= 1 || std::getenv("AB_ABLATE")) {
      auto ab = [&](auto kern, const char *name) {
        auto run = [&](int i) {
          Set &s = set[i % R4];
          hipLaunchKernelGGL(kern, dim3(gB), dim3(kWtThreads), 0, 0, s.x1, s.x2, s.x3, dEV, dL, dR, wgt, s.sc,
                             (int64_t)n, ws + 4096, s.sum);
        };
        for (int i = 0; i < reps; i++) run(i);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; i++) run(i);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("  ablation %-28s %8.2f us/launch\n", name, ms * 1e3 / reps);
      };
      ab(&plf_prot_wt_kernel<double, true, B_ROWS, 1, B_XL>, "no HBM");
      ab(&plf_prot_wt_kernel<double, true, B_ROWS, 2, B_XL>, "no LDS matrix reads");
      ab(&plf_prot_wt_kernel<double, true, B_ROWS, 4, B_XL>, "no phase 3");
      ab(&plf_prot_wt_kernel<double, true, B_ROWS, 3, B_XL>, "no HBM, no LDS matrix");
      ab(&plf_prot_wt_kernel<double, true, B_ROWS, 5, B_XL>, "no HBM, no phase 3");
      ab(&plf_prot_wt_kernel<double, true, B_ROWS, 7, B_XL>, "no HBM, no LDS mat, no ph3");
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
