// stream_writes.hip -- probe (not product code): the HBM rate of write-dominated
// streaming on gfx950, the ceiling of the coded-leaf six-level pass (64 code
// bytes read, 63 CLVs of 128 B written per site; plf_dna_f64_deep_kernel
// kTips = 2).  Each wave writes W output streams in the lane-pair layout the
// pass uses (lane l stores 16 B at site0 * 128 + 16 l: 1 KiB per wave
// instruction, non-temporal or write-back), U 8-site blocks per trip, and reads R one-byte
// code streams per site; 512-thread blocks, grid = blocks per CU x CUs,
// grid-stride loop.  Rates in GB/s of algorithmic bytes (W * 128 + R per site).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/stream_writes.hip -o build/stream_writes
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kMaxW = 64;
struct Ptrs {
  f64x2 *out[kMaxW];
  const unsigned char *codes[kMaxW];
};

template <int W, int R, int U, bool NT>
__global__ void __launch_bounds__(512, 1) writes(Ptrs p, int64_t n) {
  const int lane = threadIdx.x & 63, g = lane >> 3;
  const int64_t wave = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 8 * 8 * U;
  for (int64_t base = wave * 8 * U; base < n; base += stride) {
    int code[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t s = base + 8 * u + g < n ? base + 8 * u + g : n - 1;
      int c = 0;
#pragma unroll
      for (int r = 0; r < R; r++) c += p.codes[r][s];
      code[u] = c;
    }
#pragma unroll 1
    for (int w = 0; w < W; w++) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t site0 = base + 8 * u;
        if (site0 + g < n) {
          const f64x2 v = {(double)(code[u] + w), (double)lane};
          if (NT) __builtin_nontemporal_store(v, p.out[w] + site0 * 8 + lane);
          else p.out[w][site0 * 8 + lane] = v;
        }
      }
    }
  }
}

template <int W, int R, int U, bool NT = true>
void run(const Ptrs &p, int64_t n, int cus, int per_cu) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = cus * per_cu;
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL((writes<W, R, U, NT>), dim3(grid), dim3(512), 0, 0, p, n);
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int rep = 0; rep < 10; rep++) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((writes<W, R, U, NT>), dim3(grid), dim3(512), 0, 0, p, n);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double bytes = (double)n * (W * 128.0 + R);
  printf("W=%2d R=%2d U=%d %s blocks/CU=%d: %8.3f ms  %7.0f GB/s  %5.1f%% of 8 TB/s\n", W, R, U, NT ? "nt " : "wb ", per_cu,
         t[t.size() / 2], bytes / (t[t.size() / 2] * 1e-3) / 1e9, bytes / (t[t.size() / 2] * 1e-3) / 8e12 * 100);
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t n = 1 << 20;
  Ptrs p{};
  for (int w = 0; w < kMaxW; w++) {
    CK(hipMalloc(&p.out[w], n * 128));
    unsigned char *c;
    CK(hipMalloc(&c, n));
    CK(hipMemset(c, 1, n));
    p.codes[w] = c;
  }
  CK(hipDeviceSynchronize());
  for (int bpc : {1, 2}) {
    run<1, 0, 4>(p, n, cus, bpc);
    run<2, 0, 4>(p, n, cus, bpc);
    run<8, 0, 4>(p, n, cus, bpc);
    run<63, 64, 2>(p, n, cus, bpc);
    run<63, 64, 4>(p, n, cus, bpc);
    run<63, 0, 4>(p, n, cus, bpc);
    run<63, 64, 8>(p, n, cus, bpc);
    run<8, 0, 4, false>(p, n, cus, bpc);
    run<63, 64, 4, false>(p, n, cus, bpc);
  }
  return 0;
}
