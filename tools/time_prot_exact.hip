// Timing of the product's exact-mode protein node kernel (f64, S = 20, C = 4,
// plf_prot_lds_kernel<double, kSum, 2, 0, 10, true>) built against whichever
// plf_prot.hpp is on the include path -- so two builds (the previous header
// and the current one) can be run back to back on one box and compared: each
// run prints us per launch at 2^18 and 2^20 sites (hipEvents over `reps`
// launches rotating 4 buffer sets > the 256-MiB Infinity Cache, after a warm-up
// of the same length) and an FNV-1a hash of x3, the scaler bytes and the sum
// of buffer set 0, which must be equal across the builds (bit-identical).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I <dir of plf_prot.hpp> tools/time_prot_exact.hip -o build/time_prot_exact
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

static unsigned long long fnv(const void *p, size_t n, unsigned long long h = 1469598103934665603ull) {
  const unsigned char *b = static_cast<const unsigned char *>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

int main(int argc, char **argv) {
  const char *tag = argc > 1 ? argv[1] : "build";
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto k = &plf_prot_lds_kernel<double, true, 2, 0, 10, true>;
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kBlock, 0));
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
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (long n : {1L << 18, 1L << 20}) {
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
    struct Set {
      double *x1, *x2, *x3;
      uint8_t *sc;
      int64_t *sum;
    } set[4];
    for (auto &s : set) {
      CK(hipMalloc(&s.x1, V * 8));
      CK(hipMalloc(&s.x2, V * 8));
      CK(hipMalloc(&s.x3, V * 8));
      CK(hipMalloc(&s.sc, n));
      CK(hipMalloc(&s.sum, 8));
      CK(hipMemcpy(s.x1, h1.data(), V * 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(s.x2, h2.data(), V * 8, hipMemcpyHostToDevice));
    }
    const long grid = std::min<long>((n + 63) / 64, (long)occ * cus);
    auto run = [&](int i) {
      Set &s = set[i % 4];
      hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, 0, s.x1, s.x2, s.x3, dEV, dL, dR, wgt, s.sc,
                         (int64_t)n, ws, s.sum, nullptr);
    };
    run(0);
    CK(hipDeviceSynchronize());
    std::vector<double> x3(V);
    std::vector<uint8_t> sc(n);
    int64_t sum = 0;
    CK(hipMemcpy(x3.data(), set[0].x3, V * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sc.data(), set[0].sc, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&sum, set[0].sum, 8, hipMemcpyDeviceToHost));
    const unsigned long long h = fnv(&sum, 8, fnv(sc.data(), n, fnv(x3.data(), V * 8)));
    const int reps = n >= (1 << 20) ? 200 : 800;
    for (int i = 0; i < reps; i++) run(i);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; i++) run(i);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    std::printf("%-6s n=%8ld  %8.2f us/launch  %.3f of 8 TB/s (1921 B/site)  %d blocks/CU  hash %016llx  sum %lld\n",
                tag, n, us, 1921.0 * n / (us * 1e-6) / 8e12, occ, h, (long long)sum);
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
