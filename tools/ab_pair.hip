// ab_pair.hip -- interleaved A/B/C of the headline DNA f64 node kernel
// (plf_dna_f64_pair_kernel, U=2, scaler sum, NT loads) from up to three copies
// of plf_dna.hpp (tuning only): A = csrc, B = B_HEADER (plfx::dev_b), C =
// C_HEADER (plfx::dev_c), with a 2-read/1-write stream of the same bytes,
// round-robin over rotating buffer sets larger than the Infinity Cache.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -I amd-versal-phylogenetic-likelihood-function_amd/csrc -DB_HEADER='"/tmp/b/plf_dna.hpp"' \
//     -DC_HEADER='"/tmp/c/plf_dna.hpp"' tools/ab_pair.hip -o build/ab_pair
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "plf_dna.hpp"
#define dev dev_b
#include B_HEADER
#undef dev
#define dev dev_c
#include C_HEADER
#undef dev

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

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

struct Set { double *x1, *x2, *x3; int *wgt; uint8_t *sc; int64_t *sum; };

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const int R = 4, reps = argc > 2 ? atoi(argv[2]) : 60, rounds = 5;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  std::vector<Set> sets(R);
  double *EV, *L, *Rm; unsigned long long *ws;
  CK(hipMalloc(&EV, 16 * 8)); CK(hipMalloc(&L, 64 * 8)); CK(hipMalloc(&Rm, 64 * 8));
  CK(hipMalloc(&ws, plfx::dev::kWsWords * 8)); CK(hipMemset(ws, 0, plfx::dev::kWsWords * 8));
  fill<<<1, 64>>>(EV, 16, 1, 1.0); fill<<<1, 64>>>(L, 64, 2, 1.0); fill<<<1, 64>>>(Rm, 64, 3, 1.0);
  for (int r = 0; r < R; r++) {
    Set &s = sets[r];
    CK(hipMalloc(&s.x1, n * 128)); CK(hipMalloc(&s.x2, n * 128)); CK(hipMalloc(&s.x3, n * 128));
    CK(hipMalloc(&s.wgt, n * 4)); CK(hipMalloc(&s.sc, n)); CK(hipMalloc(&s.sum, 8));
    fill<<<2048, 256>>>(s.x1, n * 16, 10 + r, 1e-12);
    fill<<<2048, 256>>>(s.x2, n * 16, 20 + r, 1.0);
    std::vector<int> ones(n, 1); CK(hipMemcpy(s.wgt, ones.data(), n * 4, hipMemcpyHostToDevice));
  }
  CK(hipDeviceSynchronize());
  struct V { std::string name; double bytes; std::function<void(const Set &)> run; std::vector<float> us; };
  std::vector<V> vs;
  auto occ = [&](const void *k) { int b = 0; CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, 256, 0)); return b; };
  vs.push_back({"stream 2R+1W V=4 grid 4/CU", 384.0 * n, [&](const Set &s) {
    stream3<<<CUs * 4, 256>>>((const f64x2v *)s.x1, (const f64x2v *)s.x2, (f64x2v *)s.x3, n * 8); }, {}});
#define ADD(NAME, K)                                                                               \
  {                                                                                                \
    auto k = K;                                                                                    \
    const int64_t grid = std::min<int64_t>((n + 127) / 128, (int64_t)occ((const void *)k) * CUs); \
    vs.push_back({NAME, 389.0 * n, [=](const Set &s) {                                             \
      hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), 0, 0, s.x1, s.x2, s.x3, EV, L, Rm,    \
                         s.wgt, s.sc, n, ws, s.sum); }, {}});                                      \
  }
  ADD("A pair (csrc)", (&plfx::dev::plf_dna_f64_pair_kernel<2, true, 1, true>))
  ADD("B pair (" B_HEADER ")", (&plfx::dev_b::plf_dna_f64_pair_kernel<2, true, 1, true>))
  ADD("C pair (" C_HEADER ")", (&plfx::dev_c::plf_dna_f64_pair_kernel<2, true, 1, true>))
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
    printf("%-40s median %8.2f us (min %8.2f)  %5.1f%% of 8 TB/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           v.us[0], 100.0 * v.bytes / t / 8e12);
  }
  return 0;
}
