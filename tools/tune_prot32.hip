// tune_prot32.hip -- tuning harness for the f32 protein (S=20) kernels (not
// product code): the register-distributed readlane kernel (plf_prot_kernel,
// the round-1 f32 path) against the LDS-matrix grouped kernel
// (plf_prot_lds_kernel) in exact and FMA mode, each checked bit-for-bit
// against the readlane kernel of the same mode on the first buffer set, then
// timed over rotating buffer sets in one process.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I amd-versal-phylogenetic-likelihood-function_amd/csrc -I tools tools/tune_prot32.hip -o build/tune_prot32
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "plf_prot_tune.hpp"
#include "prot_pair32.hpp"

using namespace plfx::dev;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void fill(float *p, int64_t n, uint64_t seed, float scale_every4, int rec) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    float v = (float)((double)(z >> 11) * (1.0 / 9007199254740992.0));
    if (((i / rec) % 4) == 0) v *= scale_every4;
    p[i] = v;
  }
}

struct Set { float *x1, *x2, *x3; int *wgt; uint8_t *sc; int64_t *sum; };

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 18);
  const int R = 4, reps = argc > 2 ? atoi(argv[2]) : 40, rounds = 5;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  std::vector<Set> sets(R);
  float *EV, *L, *Rm; unsigned long long *ws;
  CK(hipMalloc(&EV, 400 * 4)); CK(hipMalloc(&L, 1600 * 4)); CK(hipMalloc(&Rm, 1600 * 4));
  CK(hipMalloc(&ws, kWsWords * 8)); CK(hipMemset(ws, 0, kWsWords * 8));
  fill<<<8, 64>>>(EV, 400, 7, 1.0f, 1); fill<<<32, 64>>>(L, 1600, 8, 1.0f, 1); fill<<<32, 64>>>(Rm, 1600, 9, 1.0f, 1);
  for (int r = 0; r < R; r++) {
    Set &s = sets[r];
    CK(hipMalloc(&s.x1, n * 320)); CK(hipMalloc(&s.x2, n * 320)); CK(hipMalloc(&s.x3, n * 320));
    CK(hipMalloc(&s.wgt, n * 4)); CK(hipMalloc(&s.sc, n)); CK(hipMalloc(&s.sum, 8));
    fill<<<2048, 256>>>(s.x1, n * 80, 10 + r, 1e-14f, 80);
    fill<<<2048, 256>>>(s.x2, n * 80, 20 + r, 1.0f, 80);
    std::vector<int> ones(n, 1); CK(hipMemcpy(s.wgt, ones.data(), n * 4, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  auto occ = [&](const void *k) { int b = 0; CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, 256, 0)); return b; };
  struct V { std::string name; int mode; std::function<void(const Set &)> run; std::vector<float> us; };
  std::vector<V> vs;
#define ADD(NAME, MODE, KERNEL)                                                                    \
  {                                                                                                \
    auto k = KERNEL;                                                                               \
    const int o = occ((const void *)k);                                                            \
    const int64_t grid = std::min<int64_t>((n + 63) / 64, (int64_t)o * CUs);                       \
    char nm[200]; snprintf(nm, sizeof nm, "%s occ=%d/CU grid=%lld", NAME, o, (long long)grid);      \
    vs.push_back({nm, MODE, [=](const Set &s) {                                                    \
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,    \
                         s.wgt, s.sc, n, ws, s.sum, nullptr); }, {}});                              \
  }
  const bool q = argc > 3 && atoi(argv[3]) == 1;  // round-2 kQ session: FMA kernels only
  if (!q) {
  ADD("readlane exact (r01 product)", 0, (&plf_prot_kernel<float, false, true>))
  ADD("readlane fma (r01 product)", 1, (&plf_prot_kernel<float, true, true>))
  ADD("lds exact rows=4", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 4, true, false>))
  ADD("lds exact rows=4 packed", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 4, true, true>))
  ADD("lds exact rows=20", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 20, true, false>))
  ADD("lds exact rows=20 packed", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 20, true, true>))
  ADD("lds exact rows=4 no prefetch", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 4, false, false>))
  ADD("lds fma rows=4", 1, (&plf_prot_lds_kernel<float, true, true, 2, 0, 4, true, false>))
  ADD("lds fma rows=4 packed", 1, (&plf_prot_lds_kernel<float, true, true, 2, 0, 4, true, true>))
  ADD("lds fma rows=20 packed", 1, (&plf_prot_lds_kernel<float, true, true, 2, 0, 20, true, true>))
  ADD("lds fma rows=4 packed no prefetch", 1, (&plf_prot_lds_kernel<float, true, true, 2, 0, 4, false, true>))
  ADD("mfma32 fma", 1, (&plf_prot_mfma32_kernel<true, 2>))
  ADD("mfma32 fma minw1", 1, (&plf_prot_mfma32_kernel<true, 1>))
  ADD("mfma32 fma minw3", 1, (&plf_prot_mfma32_kernel<true, 3>))
  ADD("mfma32 fma minw4", 1, (&plf_prot_mfma32_kernel<true, 4>))
  } else {
  // rows 16..19 on v_mfma_f32_4x4x1_16b (kQ = 1: the products; 2: also the
  // back-transform), against the readlane FMA kernel (the check) and the product
  ADD("readlane fma (r01, the check)", 1, (&plf_prot_kernel<float, true, true>))
  ADD("mfma32 fma minw3 (product)", 1, (&plf_prot_mfma32_kernel<true, 3>))
  ADD("mfma32 fma minw3 kQ=1", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 1>))
  ADD("mfma32 fma minw3 kQ=2", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
  ADD("mfma32 fma minw2 kQ=1", 1, (&plf_prot_mfma32_kernel<true, 2, 0, 1>))
  ADD("mfma32 fma minw2 kQ=2", 1, (&plf_prot_mfma32_kernel<true, 2, 0, 2>))
  ADD("mfma32 fma minw4 kQ=2", 1, (&plf_prot_mfma32_kernel<true, 4, 0, 2>))
  ADD("mfma32 fma minw3 (product, again)", 1, (&plf_prot_mfma32_kernel<true, 3>))
  }
  if (argc > 3 && atoi(argv[3]) == 2) {  // round-2 pair session: exact, two sites per lane
    vs.clear();
    ADD("readlane exact (r01, the check)", 0, (&plf_prot_kernel<float, false, true>))
    ADD("lds exact rows=4 (product)", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 4, true, false>))
    ADD("pair32 exact minw2", 0, (&plf_prot_pair32_kernel<true, 2>))
    ADD("pair32 exact minw1", 0, (&plf_prot_pair32_kernel<true, 1>))
    ADD("lds exact rows=4 (product, again)", 0, (&plf_prot_lds_kernel<float, false, true, 2, 0, 4, true, false>))
    ADD("pair32 exact minw2 again", 0, (&plf_prot_pair32_kernel<true, 2>))
  }
  if (argc > 3 && atoi(argv[3]) == 3) {  // round-2 grid session: the product kernel at fixed grids
    vs.clear();
#define ADDG(NAME, MODE, KERNEL, GRID)                                                             \
  {                                                                                                \
    auto k = KERNEL;                                                                               \
    const int64_t grid = std::min<int64_t>((n + 63) / 64, (int64_t)(GRID));                        \
    char nm[200]; snprintf(nm, sizeof nm, "%s grid=%lld trips<=%lld", NAME, (long long)grid,       \
                           (long long)(((n + 63) / 64 + grid - 1) / grid));                         \
    vs.push_back({nm, MODE, [=](const Set &s) {                                                    \
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,    \
                         s.wgt, s.sc, n, ws, s.sum, nullptr); }, {}});                              \
  }
    const int64_t tiles = (n + 63) / 64, res = 3LL * CUs;
    const int64_t trips = (tiles + res - 1) / res, bal = (tiles + trips - 1) / trips;
    auto kp = &plf_prot_mfma32_kernel<true, 3, 0, 2>;
    ADDG("readlane fma (r01, the check)", 1, (&plf_prot_kernel<float, true, true>), 2LL * CUs)
    ADDG("product, resident 3/CU", 1, kp, res)
    ADDG("product, balanced trips", 1, kp, bal)
    ADDG("product, 2/CU", 1, kp, 2LL * CUs)
    ADDG("product, balanced+1 trip", 1, kp, (tiles + trips) / (trips + 1))
    ADDG("product, resident 3/CU again", 1, kp, res)
    ADDG("product, balanced trips again", 1, kp, bal)
  }
  if (argc > 3 && atoi(argv[3]) == 4) {  // round-2 ablation session (the ablated forms DIFFER by design)
    vs.clear();
    ADD("readlane fma (r01, the check)", 1, (&plf_prot_kernel<float, true, true>))
    ADD("product", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
    ADD("product ablate: no matrix cores", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 1>))
    ADD("product ablate: no HBM", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 2>))
    ADD("product ablate: tile movement only", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 3>))
    ADD("product ablate: tile movement only, 4/CU", 1, (&plf_prot_mfma32_kernel<true, 4, 0, 2, 3>))
    ADD("product again", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
  }
  if (argc > 3 && atoi(argv[3]) == 5) {  // round-2 ring session: two tiles in flight per block
    vs.clear();
    ADD("readlane fma (r01, the check)", 1, (&plf_prot_kernel<float, true, true>))
    ADD("product", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
    ADD("ring minw3", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 0, true>))
    ADD("ring minw2", 1, (&plf_prot_mfma32_kernel<true, 2, 0, 2, 0, true>))
    ADD("product again", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
    ADD("ring minw3 again", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 0, true>))
    ADD("ring minw2 again", 1, (&plf_prot_mfma32_kernel<true, 2, 0, 2, 0, true>))
  }
  if (argc > 3 && atoi(argv[3]) == 6) {  // round-2 session: both children staged together
    vs.clear();
    ADD("readlane fma (r01, the check)", 1, (&plf_prot_kernel<float, true, true>))
    ADD("product", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
    ADD("both minw3", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 0, 2>))
    ADD("both minw2", 1, (&plf_prot_mfma32_kernel<true, 2, 0, 2, 0, 2>))
    ADD("product again", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2>))
    ADD("both minw3 again", 1, (&plf_prot_mfma32_kernel<true, 3, 0, 2, 0, 2>))
    ADD("both minw2 again", 1, (&plf_prot_mfma32_kernel<true, 2, 0, 2, 0, 2>))
  }
  std::vector<uint32_t> ref[2], got(n * 80);
  std::vector<uint8_t> rsc[2], gsc(n);
  int64_t rsum[2] = {0, 0}, gsum = 0;
  for (auto &v : vs) {
    CK(hipMemset(sets[0].x3, 0xff, n * 320)); CK(hipMemset(sets[0].sc, 7, n));
    v.run(sets[0]);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), sets[0].x3, n * 320, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gsc.data(), sets[0].sc, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&gsum, sets[0].sum, 8, hipMemcpyDeviceToHost));
    if (ref[v.mode].empty()) { ref[v.mode] = got; rsc[v.mode] = gsc; rsum[v.mode] = gsum; }
    int64_t bad = 0;
    for (int64_t i = 0; i < n * 80; i++) bad += got[i] != ref[v.mode][i];
    for (int64_t i = 0; i < n; i++) bad += gsc[i] != rsc[v.mode][i];
    printf("%-50s check %s (%lld mismatches, sum %lld)\n", v.name.c_str(),
           bad == 0 && gsum == rsum[v.mode] ? "bit-exact" : "DIFFERS", (long long)bad, (long long)gsum);
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 300; i++) vs[1].run(sets[i % R]);  // past the first launches' transient
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
  printf("n=%lld f32 protein sites, %d reps x %d rounds, %d buffer sets, %% at 961 B/site\n", (long long)n, reps,
         rounds, R);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6, bytes = 961.0 * n;
    printf("%-50s median %8.2f us  %5.1f%% of 8 TB/s  %6.3f Gsites/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           100.0 * bytes / t / 8e12, n / t / 1e9);
  }
  return 0;
}
