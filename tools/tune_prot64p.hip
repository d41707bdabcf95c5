// tune_prot64p.hip -- A/B harness (not product code): the f64 FMA protein
// product kernel (plf_prot_mfma_kernel, fixed grid stride, and its tile-queue
// form) against the wave-priority copy (tools/prot_prio.hpp), dense, each
// checked bit for bit against the product on the first buffer set (and the
// queue words checked back at zero after every launch), then timed over
// rotating buffer sets in one process.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I amd-versal-phylogenetic-likelihood-function_amd/csrc -I tools tools/tune_prot64p.hip -o build/tune_prot64p
//   build/tune_prot64p [sites] [reps] [sel]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "prot_prio.hpp"

using namespace plfx::dev;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void fill(double *p, int64_t n, uint64_t seed, double scale_every4, int rec) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    double v = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    if (((i / rec) % 4) == 0) v *= scale_every4;
    p[i] = v;
  }
}

struct Set { double *x1, *x2, *x3; int *wgt; uint8_t *sc; int64_t *sum; };
typedef void (*Kern)(const double *, const double *, double *, const double *, const double *, const double *,
                     const int32_t *, uint8_t *, int64_t, unsigned long long *, int64_t *, const double *);
typedef void (*KernS)(const double *, const double *, double *, const double *, const double *, const double *,
                      const int32_t *, uint8_t *, int64_t, unsigned long long *, int64_t *, const double *, uint64_t *);

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 18);
  const int R = 4, reps = argc > 2 ? atoi(argv[2]) : 40, rounds = 5;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  std::vector<Set> sets(R);
  double *EV, *L, *Rm; unsigned long long *ws;
  CK(hipMalloc(&EV, 400 * 8)); CK(hipMalloc(&L, 1600 * 8)); CK(hipMalloc(&Rm, 1600 * 8));
  CK(hipMalloc(&ws, 2 * kWsWords * 8)); CK(hipMemset(ws, 0, 2 * kWsWords * 8));  // queue: region 1
  fill<<<8, 64>>>(EV, 400, 7, 1.0, 1); fill<<<32, 64>>>(L, 1600, 8, 1.0, 1); fill<<<32, 64>>>(Rm, 1600, 9, 1.0, 1);
  for (int r = 0; r < R; r++) {
    Set &s = sets[r];
    // + 64 sites of slack: tip kernels read x1/x2 as bytes; ragged sizes stay in bounds
    CK(hipMalloc(&s.x1, (n + 64) * 640)); CK(hipMalloc(&s.x2, (n + 64) * 640)); CK(hipMalloc(&s.x3, (n + 64) * 640));
    CK(hipMalloc(&s.wgt, n * 4)); CK(hipMalloc(&s.sc, n)); CK(hipMalloc(&s.sum, 8));
    fill<<<2048, 256>>>(s.x1, (n + 64) * 80, 10 + r, 1e-14, 80);
    fill<<<2048, 256>>>(s.x2, (n + 64) * 80, 20 + r, 1.0, 80);
    std::vector<int> ones(n, 1); CK(hipMemcpy(s.wgt, ones.data(), n * 4, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  auto occ = [&](const void *k) { int b = 0; CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, 256, 0)); return b; };
  struct V { std::string name; int mode; std::function<void(const Set &)> run; std::vector<float> us; };
  std::vector<V> vs;
  auto add = [&](const char *name, int mode, Kern k, int sites_per_block) {
    const int o = occ((const void *)k);
    const int64_t grid = std::min<int64_t>((n + sites_per_block - 1) / sites_per_block, (int64_t)o * CUs);
    char nm[200]; snprintf(nm, sizeof nm, "%s occ=%d/CU grid=%lld", name, o, (long long)grid);
    vs.push_back({nm, mode, [=](const Set &s) {
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,
                         s.wgt, s.sc, n, ws, s.sum, nullptr); }, {}});
  };
  auto adds = [&](const char *name, int mode, KernS k, int sites_per_block) {
    const int o = occ((const void *)k);
    const int64_t grid = std::min<int64_t>((n + sites_per_block - 1) / sites_per_block, (int64_t)o * CUs);
    char nm[200]; snprintf(nm, sizeof nm, "%s occ=%d/CU grid=%lld", name, o, (long long)grid);
    vs.push_back({nm, mode, [=](const Set &s) {
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,
                         s.wgt, s.sc, n, ws, s.sum, nullptr, nullptr); }, {}});
  };
  const int sel = argc > 3 ? atoi(argv[3]) : 0;
  if (sel == 0 || sel == 1) {
    add("product static", 0, &plf_prot_mfma_kernel<true, 2, 0, false>, 64);
    add("prio mode 0 (copy, no setprio)", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 0, 0>, 64);
    add("prio young hi first 4 trips", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 1, 4>, 64);
    add("prio young hi first 3 trips", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 1, 3>, 64);
    add("prio young hi first 5 trips", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 1, 5>, 64);
    add("prio young hi first 2 trips", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 1, 2>, 64);
    add("prio young hi always", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 2, 0>, 64);
    add("prio alternating", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 3, 0>, 64);
    add("product kDyn", 0, &plf_prot_mfma_kernel<true, 2, 0, true>, 64);
    add("product static again", 0, &plf_prot_mfma_kernel<true, 2, 0, false>, 64);
    add("prio young hi first 4 trips again", 0, &plf_prot_mfma_prio_kernel<true, 2, 0, 1, 4>, 64);
  }
  if (sel == 2) {
    add("product tip/inner", 1, &plf_prot_mfma_kernel<true, 2, 1, false>, 64);
    add("prio tip/inner young hi first 4", 1, &plf_prot_mfma_prio_kernel<true, 2, 1, 1, 4>, 64);
    add("prio tip/inner alternating", 1, &plf_prot_mfma_prio_kernel<true, 2, 1, 3, 0>, 64);
  }
  std::vector<uint64_t> ref[3], got(n * 80);
  std::vector<uint8_t> rsc[3], gsc(n);
  int64_t rsum[3] = {0, 0, 0}, gsum = 0;
  int failures = 0;
  for (auto &v : vs) {
    CK(hipMemset(sets[0].x3, 0xff, n * 640)); CK(hipMemset(sets[0].sc, 7, n));
    v.run(sets[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), sets[0].x3, n * 640, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gsc.data(), sets[0].sc, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&gsum, sets[0].sum, 8, hipMemcpyDeviceToHost));
    if (ref[v.mode].empty()) { ref[v.mode] = got; rsc[v.mode] = gsc; rsum[v.mode] = gsum; }
    int64_t bad = 0;
    for (int64_t i = 0; i < n * 80; i++) bad += got[i] != ref[v.mode][i];
    for (int64_t i = 0; i < n; i++) bad += gsc[i] != rsc[v.mode][i];
    std::vector<unsigned long long> qw(kWsWords);
    for (int rep = 0; rep < 3; rep++) v.run(sets[rep % R]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(qw.data(), ws + kWsWords, kWsWords * 8, hipMemcpyDeviceToHost));
    for (auto w : qw) bad += w != 0;
    const bool ok = bad == 0 && gsum == rsum[v.mode];
    failures += !ok;
    printf("%-50s check %s (%lld mismatches, sum %lld)\n", v.name.c_str(), ok ? "bit-exact" : "DIFFERS",
           (long long)bad, (long long)gsum);
  }
  if (reps == 0) return failures ? 1 : 0;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 300; i++) vs[0].run(sets[i % R]);  // past the post-idle clock dip
  for (int round = 0; round < rounds; round++)
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
  printf("n=%lld f64 protein sites, %d reps x %d rounds, %d buffer sets, %% at 1921 B/site (dense)\n",
         (long long)n, reps, rounds, R);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6, bytes = 1921.0 * n;
    printf("%-50s median %8.2f us  %5.1f%% of 8 TB/s  %6.3f Gsites/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           100.0 * bytes / t / 8e12, n / t / 1e9);
  }
  return failures ? 1 : 0;
}
