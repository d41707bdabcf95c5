// Timing of the product's f32 protein FMA kernel (S = 20, C = 4,
// plf_prot_mfma32_kernel<kSum = true, 3, kTips = 0>) built against whichever
// plf_prot.hpp is on the include path, like time_prot_exact.hip: two builds
// (the previous header and the current one) run back to back on one box.
// With -DPROT_F32_DYN (a header whose kernel takes the kDyn queue parameter:
// round 5 tried one, ProtQueue wired into prot_mfma32_body as in
// prot_mfma_body -- bit-identical but 20-30 % slower, not kept,
// profiles/r05_prot_f32_queue_ab.log) the queued form is timed too.  Per size: us per launch (hipEvents over
// `reps` launches rotating up to 4 buffer sets, after a warm-up of the same
// length) and an FNV-1a hash of x3, the scaler bytes and the sum of buffer
// set 0, which must be equal for every form and build (bit-identical).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DPROT_F32_DYN] \
//     -I <dir of plf_prot.hpp> tools/time_prot_f32.hip -o build/time_prot_f32
#include <hip/hip_runtime.h>

#include <algorithm>
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

typedef void (*Kern)(const float *, const float *, float *, const float *, const float *, const float *,
                     const int32_t *, uint8_t *, int64_t, unsigned long long *, int64_t *, const float *);

int main(int argc, char **argv) {
  const char *tag = argc > 1 ? argv[1] : "build";
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<std::pair<const char *, Kern>> forms = {
      {"static", &plf_prot_mfma32_kernel<true, 3, 0>}};
#ifdef PROT_F32_DYN
  forms.push_back({"queue", &plf_prot_mfma32_kernel<true, 3, 0, true>});
#endif
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)forms[0].second, kBlock, 0));
  std::mt19937_64 g(20250117);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::vector<float> EV(400), L(1600), R(1600);
  for (auto &v : EV) v = U(g) - 0.25f;
  for (auto &v : L) v = U(g);
  for (auto &v : R) v = U(g);
  float *dEV, *dL, *dR;
  CK(hipMalloc(&dEV, 400 * 4));
  CK(hipMalloc(&dL, 1600 * 4));
  CK(hipMalloc(&dR, 1600 * 4));
  CK(hipMemcpy(dEV, EV.data(), 400 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dL, L.data(), 1600 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dR, R.data(), 1600 * 4, hipMemcpyHostToDevice));
  unsigned long long *ws;
  CK(hipMalloc(&ws, 1 << 20));
  CK(hipMemset(ws, 0, 1 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // one 2^20-site pattern on the host, tiled onto the device for larger n
  const long P = 1L << 20;
  std::vector<float> h1(80 * P), h2(80 * P);
  for (size_t i = 0; i < h1.size(); i++) {
    h1[i] = U(g) * ((i / 80) % 4 == 0 ? 1e-14f : 1.f);
    h2[i] = U(g);
  }
  for (long n : {1L << 18, 1L << 20, 1L << 22, 1L << 24}) {
    const size_t V = 80 * (size_t)n;
    const int nsets = n <= (1L << 22) ? 4 : 1;
    int *wgt;
    CK(hipMalloc(&wgt, n * 4));
    std::vector<int> hw(n, 1);
    CK(hipMemcpy(wgt, hw.data(), n * 4, hipMemcpyHostToDevice));
    struct Set {
      float *x1, *x2, *x3;
      uint8_t *sc;
      int64_t *sum;
    } set[4];
    for (int si = 0; si < nsets; si++) {
      Set &s = set[si];
      CK(hipMalloc(&s.x1, V * 4));
      CK(hipMalloc(&s.x2, V * 4));
      CK(hipMalloc(&s.x3, V * 4));
      CK(hipMalloc(&s.sc, n));
      CK(hipMalloc(&s.sum, 8));
      for (size_t o = 0; o < V; o += 80 * (size_t)P) {
        const size_t m = std::min(V - o, 80 * (size_t)P);
        CK(hipMemcpy(s.x1 + o, h1.data(), m * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(s.x2 + o, h2.data(), m * 4, hipMemcpyHostToDevice));
      }
    }
    const long grid = std::min<long>((n + 63) / 64, (long)occ * cus);
    for (auto &f : forms) {
      auto run = [&](int i) {
        Set &s = set[i % nsets];
        hipLaunchKernelGGL(f.second, dim3(grid), dim3(kBlock), 0, 0, s.x1, s.x2, s.x3, dEV, dL, dR, wgt,
                           s.sc, (int64_t)n, ws, s.sum, nullptr);
      };
      run(0);
      CK(hipDeviceSynchronize());
      std::vector<float> x3(V);
      std::vector<uint8_t> sc(n);
      int64_t sum = 0;
      CK(hipMemcpy(x3.data(), set[0].x3, V * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(sc.data(), set[0].sc, n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&sum, set[0].sum, 8, hipMemcpyDeviceToHost));
      const unsigned long long h = fnv(&sum, 8, fnv(sc.data(), n, fnv(x3.data(), V * 4)));
      const int reps = std::max(8L, 1100000000L / n);  // ~0.2 s of launches
      for (int i = 0; i < reps; i++) run(i);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; i++) run(i);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      std::printf("%-6s %-6s n=%9ld  %9.2f us/launch  %.3f of 8 TB/s (961 B/site)  grid %ld  hash %016llx  sum %lld\n",
                  tag, f.first, n, us, 961.0 * n / (us * 1e-6) / 8e12, grid, h, (long long)sum);
      std::fflush(stdout);
    }
    for (int si = 0; si < nsets; si++) {
      Set &s = set[si];
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
