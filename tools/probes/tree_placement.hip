// tree_placement.hip -- probe (not product code): does the placement of the
// 127 CLVs of a 64-taxon sweep set the HBM rate of the fused six-level pass?
// Round 5: tree64 f64 ran at 0.65 of 8 TB/s on some boxes and 0.77 on others
// with the same code (the round-4 tree included), and on one box 0.77 with
// one allocation per CLV but 0.65 with every CLV carved from one slab at any
// stagger (tools/gpu_r05_tree_stagger.sh).  This streams the pass's memory
// pattern with no arithmetic -- per wave and 8-site step, 64 leaf reads and 63
// CLV writes of 1 KiB each in the lane-pair layout (lane l: bytes 16l..16l+15
// of the step's 8 x 128-B records), non-temporal, 512-thread blocks, one per
// CU, wave-level grid stride -- over the same 127 x 128-MiB buffers placed in
// several ways, alternated in one process:
//   sep        127 hipMalloc calls (the bench's default: torch allocates so)
//   slab       one hipMalloc of 127 x 128 MiB, buffer j at j x 128 MiB
//   slab+G     one hipMalloc, buffer j at j x (128 MiB + G)
//   sep-rev    127 hipMalloc calls, used in reverse order
// Rates are GB/s of the 127 x 128 B per site it moves (the pass's bytes).
// Each placement runs with the grid stride of the product pass and blocked
// (every wave its own contiguous range of sites); with PLACEMENT_POLICIES set,
// the strided form with write-back loads and/or stores instead; with
// PLACEMENT_XCD set, one segment of the sites per XCD instead of blocked.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/tree_placement.hip -o build/tree_placement
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kIn = 64, kOut = 63;
struct Ptrs {
  const f64x2 *in[kIn];
  f64x2 *out[kOut];
};

// kBlocked: wave w streams its own contiguous 1/waves of the sites (so the
// addresses in flight at once sit all over every buffer) instead of the
// grid stride (all waves inside one 512-KiB window of every buffer at once).
// kLdNT / kStNT: non-temporal loads / stores (the product pass uses both).
template <int U, bool kBlocked, bool kLdNT = true, bool kStNT = true>
__global__ void __launch_bounds__(512, 1) pass(Ptrs p, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int64_t waves = (int64_t)gridDim.x * 8;
  const int64_t step = 8 * U;
  const int64_t per = (n / step + waves - 1) / waves * step;  // sites per wave (blocked)
  const int64_t first = kBlocked ? wave * per : wave * step;
  const int64_t last = kBlocked ? (first + per < n ? first + per : n) : n;
  const int64_t stride = kBlocked ? step : waves * step;
  for (int64_t base = first; base < last; base += stride) {
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = f64x2{0.0, 0.0};
#pragma unroll 8
    for (int s = 0; s < kIn; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t b = base + 8 * u < n ? base + 8 * u : n - 8;
        if constexpr (kLdNT) acc[u] += __builtin_nontemporal_load(p.in[s] + b * 8 + lane);
        else acc[u] += p.in[s][b * 8 + lane];
      }
#pragma unroll 8
    for (int o = 0; o < kOut; o++)
#pragma unroll
      for (int u = 0; u < U; u++)
        if (base + 8 * u < n) {
          if constexpr (kStNT) __builtin_nontemporal_store(acc[u], p.out[o] + (base + 8 * u) * 8 + lane);
          else p.out[o][(base + 8 * u) * 8 + lane] = acc[u];
        }
  }
}

// kXcd: blocks b, b + 8, ... (one XCD's) stride over the (b % 8)-th eighth of
// the sites only -- the node kernels' segmented mapping (plf_dna.hpp
// wave_sites) applied to the 127-stream pattern
template <int U>
__global__ void __launch_bounds__(512, 1) pass_xcd(Ptrs p, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t step = 8 * U;
  const int64_t wave = (int64_t)(blockIdx.x >> 3) * 8 + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)(gridDim.x >> 3) * 8 * step;
  const int64_t per = ((n + step - 1) / step + 7) / 8 * step;
  const int64_t lo = (int64_t)(blockIdx.x & 7) * per;
  const int64_t hi = lo + per < n ? lo + per : n;
  for (int64_t base = lo + wave * step; base < hi; base += stride) {
    f64x2 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = f64x2{0.0, 0.0};
#pragma unroll 8
    for (int s = 0; s < kIn; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t b = base + 8 * u < n ? base + 8 * u : n - 8;
        acc[u] += __builtin_nontemporal_load(p.in[s] + b * 8 + lane);
      }
#pragma unroll 8
    for (int o = 0; o < kOut; o++)
#pragma unroll
      for (int u = 0; u < U; u++)
        if (base + 8 * u < hi) __builtin_nontemporal_store(acc[u], p.out[o] + (base + 8 * u) * 8 + lane);
  }
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? std::atol(argv[1]) : (1 << 20);  // sites per CLV
  const size_t clv = (size_t)n * 128;                            // f64, 16 values per site
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<void *> sep(kIn + kOut);
  for (auto &q : sep) {
    CK(hipMalloc(&q, clv));
    CK(hipMemset(q, 0, clv));
  }
  const size_t gaps[] = {0, 2u << 20, 6u << 20, 68u << 20};
  std::vector<char *> slabs;
  // PLACEMENT_SEP_ONLY: the 127 separate allocations only (long CLVs: four
  // 127-CLV slabs would not fit beside them)
  const bool sep_only = std::getenv("PLACEMENT_SEP_ONLY") != nullptr;
  for (size_t g : gaps) {
    if (sep_only) break;
    char *s = nullptr;
    CK(hipMalloc((void **)&s, (kIn + kOut) * (clv + g)));
    CK(hipMemset(s, 0, (kIn + kOut) * (clv + g)));
    slabs.push_back(s);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // PLACEMENT_BPC: 512-thread blocks per CU (default 1 = 2 waves per SIMD, the
  // six-level pass's occupancy; 2 = 4 waves per SIMD)
  const int bpc = std::getenv("PLACEMENT_BPC") ? std::atoi(std::getenv("PLACEMENT_BPC")) : 1;
  {
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, pass<2, false>, 512, 0));
    std::printf("# %d block(s) of 512 per CU requested, %d co-resident\n", bpc, occ);
  }
  auto time1 = [&](const char *name, const std::vector<void *> &bufs, auto kern, const char *mode) {
    Ptrs p;
    for (int s = 0; s < kIn; s++) p.in[s] = static_cast<const f64x2 *>(bufs[s]);
    for (int o = 0; o < kOut; o++) p.out[o] = static_cast<f64x2 *>(bufs[kIn + o]);
    const int reps = 10;
    for (int i = 0; i < 2; i++) hipLaunchKernelGGL(kern, dim3(bpc * cus), dim3(512), 0, 0, p, n);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL(kern, dim3(bpc * cus), dim3(512), 0, 0, p, n);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps, gbs = 127.0 * 128 * n / (us * 1e-6) / 1e9;
    std::printf("%-12s %-8s %9.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", name, mode, us, gbs, gbs / 8000);
  };
  const bool policies = std::getenv("PLACEMENT_POLICIES") != nullptr;
  auto time = [&](const char *name, const std::vector<void *> &bufs) {
    time1(name, bufs, pass<2, false>, "stride");
    if (policies) {  // cache policies of the strided form
      time1(name, bufs, pass<2, false, false, true>, "ld-wb");
      time1(name, bufs, pass<2, false, true, false>, "st-wb");
      time1(name, bufs, pass<2, false, false, false>, "both-wb");
    } else if (std::getenv("PLACEMENT_XCD")) {
      time1(name, bufs, pass_xcd<2>, "xcd");
    } else {
      time1(name, bufs, pass<2, true>, "blocked");
    }
  };
  for (int round = 0; round < 3; round++) {
    time("sep", sep);
    std::vector<void *> rev(sep.rbegin(), sep.rend());
    time("sep-rev", rev);
    for (size_t k = 0; k < slabs.size(); k++) {
      std::vector<void *> b(kIn + kOut);
      for (int j = 0; j < kIn + kOut; j++) b[j] = slabs[k] + (size_t)j * (clv + gaps[k]);
      char name[32];
      std::snprintf(name, sizeof name, "slab+%zuM", gaps[k] >> 20);
      time(name, b);
    }
  }
  CK(hipGetLastError());
  return 0;
}
