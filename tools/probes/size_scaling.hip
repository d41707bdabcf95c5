// size_scaling.hip -- probe (not product code): why does one f64 node call
// run at 0.67 of 8 TB/s at 5e8 sites (192 GB of CLVs, tools/max_sites.py)
// but 0.74-0.77 at 2^20-2^22 sites?  Streams the node kernel's memory pattern
// (2 reads + 1 write of 128 B per site, lane-pair layout: lane l <-> bytes
// 16l..16l+15 of an 8-site block, non-temporal, 256-thread blocks, 2 x 8-site
// blocks per wave step) with no arithmetic, over prefixes of three 64-GB
// buffers, with three site->wave mappings:
//   stride  the product's: every wave strides over the whole array, so all
//           waves (on all 8 XCDs) work inside one ~12-MB window of each buffer
//   xcd     blocks of XCD x (= blockIdx % 8, the dispatcher's round robin)
//           stride over the x-th eighth of the sites only: each XCD's address
//           translations cover 1/8 of the pages
//   blocked every wave its own contiguous range
//   segS    (second run: not kept) S = 16, 32, 64 segments -- at best like xcd
//   tileT   block b takes tiles b, b + G, ... of T contiguous sites (the
//           protein kernels' shape), its 4 waves the tile's steps in turn
//   queueC  (QUEUE=1 with MODES) chunks of 2^C sites from a device-wide counter
//   chunkK  (first run: not kept) sites cut into chunks of 2^K, chunk j to XCD
//           j % 8, each XCD striding over its own chunks -- ran like stride
// GB/s are of the 385 B per site the node kernel moves (the 1-B scaler omitted
// here, counted in the rate as the product counts it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/size_scaling.hip -o build/size_scaling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kWaves = 4;  // 256-thread blocks
constexpr int U = 2;       // 8-site blocks per wave step (x2 = 16 sites)

template <int K>
__global__ void __launch_bounds__(256) pass_chunk(const f64x2 *__restrict__ x1,
                                                  const f64x2 *__restrict__ x2,
                                                  f64x2 *__restrict__ x3, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t step = 8 * U;
  const int64_t xcd = blockIdx.x & 7;
  const int64_t wave = (int64_t)(blockIdx.x >> 3) * kWaves + (threadIdx.x >> 6);
  const int64_t stride = (int64_t)(gridDim.x / 8) * kWaves * step;
  const int64_t mask = (1ll << K) - 1;
  for (int64_t v = wave * step;; v += stride) {
    const int64_t base = ((((v >> K) << 3) + xcd) << K) + (v & mask);  // monotonic in v
    if (base >= n) break;
    f64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t s = base + 8 * u < n ? base + 8 * u : n - 8;
      a[u] = __builtin_nontemporal_load(x1 + s * 8 + lane);
      b[u] = __builtin_nontemporal_load(x2 + s * 8 + lane);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + 8 * u < n) __builtin_nontemporal_store(a[u] * b[u], x3 + (base + 8 * u) * 8 + lane);
  }
}

// tileT: the protein kernels' shape -- block b takes tiles b, b + G, ... of T
// contiguous sites; the block's 4 waves take the tile's 16-site steps in turn
template <int T>
__global__ void __launch_bounds__(256) pass_tile(const f64x2 *__restrict__ x1,
                                                 const f64x2 *__restrict__ x2,
                                                 f64x2 *__restrict__ x3, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  constexpr int64_t step = 8 * U;
  for (int64_t tile = blockIdx.x; tile * T < n; tile += gridDim.x) {
    const int64_t t0 = tile * T, t1 = t0 + T < n ? t0 + T : n;
    for (int64_t base = t0 + w * step; base < t1; base += kWaves * step) {
      f64x2 a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t s = base + 8 * u < n ? base + 8 * u : n - 8;
        a[u] = __builtin_nontemporal_load(x1 + s * 8 + lane);
        b[u] = __builtin_nontemporal_load(x2 + s * 8 + lane);
      }
#pragma unroll
      for (int u = 0; u < U; u++)
        if (base + 8 * u < t1) __builtin_nontemporal_store(a[u] * b[u], x3 + (base + 8 * u) * 8 + lane);
    }
  }
}

// UU: 8-site blocks per wave trip (2 = 16 sites; the product's f64 kernel
// covers 32 sites per trip, UU = 4)
// queueC: blocks take chunks of 2^C contiguous sites from a device-wide
// counter (one returning atomic per chunk, thread 0, broadcast through LDS);
// the block's 4 waves take the chunk's 16-site steps in turn.  `ctr` is zero
// at launch and reset by the last block out (done counter).
template <int C>
__global__ void __launch_bounds__(256) pass_queue(const f64x2 *__restrict__ x1,
                                                  const f64x2 *__restrict__ x2,
                                                  f64x2 *__restrict__ x3, int64_t n,
                                                  unsigned long long *ctr) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  constexpr int64_t step = 8 * U;
  const int64_t nchunks = (n + (1ll << C) - 1) >> C;
  __shared__ long long chunk;
  for (;;) {
    if (threadIdx.x == 0)
      chunk = (long long)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const long long c = chunk;
    __syncthreads();
    if (c >= nchunks) break;
    const int64_t t0 = c << C, t1 = t0 + (1ll << C) < n ? t0 + (1ll << C) : n;
    for (int64_t base = t0 + w * step; base < t1; base += kWaves * step) {
      f64x2 a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t s = base + 8 * u < n ? base + 8 * u : n - 8;
        a[u] = __builtin_nontemporal_load(x1 + s * 8 + lane);
        b[u] = __builtin_nontemporal_load(x2 + s * 8 + lane);
      }
#pragma unroll
      for (int u = 0; u < U; u++)
        if (base + 8 * u < t1) __builtin_nontemporal_store(a[u] * b[u], x3 + (base + 8 * u) * 8 + lane);
    }
  }
  if (threadIdx.x == 0) {
    const unsigned long long d = __hip_atomic_fetch_add(ctr + 16, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1) {
      __hip_atomic_store(ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 16, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int kMode, int S = 8, int UU = U>  // 0 stride, 1 segments (S = 8: one per XCD), 2 blocked
__global__ void __launch_bounds__(256) pass(const f64x2 *__restrict__ x1, const f64x2 *__restrict__ x2,
                                            f64x2 *__restrict__ x3, int64_t n) {
  constexpr int U = UU;
  const int lane = threadIdx.x & 63;
  const int64_t step = 8 * U;
  int64_t first, last, stride;
  if constexpr (kMode == 0) {
    const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    first = wave * step;
    last = n;
    stride = (int64_t)gridDim.x * kWaves * step;
  } else if constexpr (kMode == 1) {
    const int xcd = blockIdx.x % S;
    const int64_t blocks_x = gridDim.x / S;  // grid is a multiple of S
    const int64_t wave = (int64_t)(blockIdx.x / S) * kWaves + (threadIdx.x >> 6);
    const int64_t per = (n / step + S - 1) / S * step;  // sites of this segment
    const int64_t lo = xcd * per;
    first = lo + wave * step;
    last = lo + per < n ? lo + per : n;
    stride = blocks_x * kWaves * step;
  } else {
    const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    const int64_t waves = (int64_t)gridDim.x * kWaves;
    const int64_t per = (n / step + waves - 1) / waves * step;
    first = wave * per;
    last = first + per < n ? first + per : n;
    stride = step;
  }
  for (int64_t base = first; base < last; base += stride) {
    f64x2 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t s = base + 8 * u < n ? base + 8 * u : n - 8;
      a[u] = __builtin_nontemporal_load(x1 + s * 8 + lane);
      b[u] = __builtin_nontemporal_load(x2 + s * 8 + lane);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (base + 8 * u < last) __builtin_nontemporal_store(a[u] * b[u], x3 + (base + 8 * u) * 8 + lane);
  }
}

int main(int argc, char **argv) {
  const int64_t nmax = argc > 1 ? std::atoll(argv[1]) : 500000000LL;  // sites
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t bytes = (size_t)nmax * 128;
  void *p1, *p2, *p3;
  CK(hipMalloc(&p1, bytes));
  CK(hipMalloc(&p2, bytes));
  CK(hipMalloc(&p3, bytes));
  CK(hipMemset(p1, 0, bytes));
  CK(hipMemset(p2, 0, bytes));
  CK(hipMemset(p3, 0, bytes));
  auto *x1 = static_cast<const f64x2 *>(p1), *x2 = static_cast<const f64x2 *>(p2);
  auto *x3 = static_cast<f64x2 *>(p3);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // blocks per CU (argv[2], default 3): 256-thread blocks, so 1..8 = 1..8 waves per SIMD.
  // The 3 per CU resident for the product's shape (a multiple of 64 blocks);
  // MODES=sx runs only the stride and xcd mappings.
  const int bpc = argc > 2 ? std::atoi(argv[2]) : 3;
  const int grid = bpc * cus;
  const bool only_sx = std::getenv("MODES") != nullptr;
  auto time1 = [&](auto kern, const char *mode, int64_t n, int64_t off) {
    // rotate over prefixes at `off` apart so small sizes do not sit in the MALL
    const int sets = off ? 4 : 1;
    const int reps = n >= (1 << 26) ? 3 : 20;
    for (int i = 0; i < 2; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, x1, x2, x3, n);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; i++) {
      const int64_t o = (i % sets) * off * 8;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, x1 + o, x2 + o, x3 + o, n);
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps, gbs = 385.0 * n / (us * 1e-6) / 1e9;
    std::printf("bpc=%d n=%-11lld %-8s %11.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", bpc, (long long)n, mode,
                us, gbs, gbs / 8000);
  };
  unsigned long long *ctr = nullptr;
  CK(hipMalloc(&ctr, 4096));
  CK(hipMemset(ctr, 0, 4096));
  auto timeq = [&](auto kern, const char *mode, int64_t n, int64_t off) {
    const int sets = off ? 4 : 1;
    const int reps = n >= (1 << 26) ? 3 : 20;
    for (int i = 0; i < 2; i++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, x1, x2, x3, n, ctr);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; i++) {
      const int64_t o = (i % sets) * off * 8;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, x1 + o, x2 + o, x3 + o, n, ctr);
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps, gbs = 385.0 * n / (us * 1e-6) / 1e9;
    std::printf("bpc=%d n=%-11lld %-8s %11.1f us  %7.1f GB/s  %.3f of 8 TB/s\n", bpc, (long long)n, mode,
                us, gbs, gbs / 8000);
  };
  std::vector<int64_t> sizes = {1 << 20, 1 << 22, 1 << 24, 1 << 25, 1 << 26, 1 << 27, 1 << 28, nmax};
  if (const char *s = std::getenv("SIZES")) {  // comma-separated site counts
    sizes.clear();
    for (const char *q = s; *q;) {
      sizes.push_back(std::atoll(q));
      while (*q && *q != ',') q++;
      if (*q == ',') q++;
    }
  }
  for (int round = 0; round < 2; round++)
    for (int64_t n : sizes) {
      if (n > nmax) continue;
      const int64_t off = 4 * n <= nmax ? n : 0;  // 4 rotating sets where they fit
      time1(pass<0>, "stride", n, off);
      time1(pass<1>, "xcd", n, off);
      if (only_sx) {
        if (std::getenv("QUEUE")) {
          timeq(pass_queue<14>, "queue14", n, off);
          timeq(pass_queue<16>, "queue16", n, off);
        } else {
          time1(pass<0, 8, 4>, "stride32", n, off);
          time1(pass<1, 8, 4>, "xcd32", n, off);
        }
        continue;
      }
      time1(pass<2>, "blocked", n, off);
      time1(pass_tile<256>, "tile256", n, off);
      time1(pass_tile<1024>, "tile1k", n, off);
      time1(pass_tile<4096>, "tile4k", n, off);
    }
  CK(hipGetLastError());
  return 0;
}
