// Probe (not product code): HBM streaming rate on gfx950 vs the number of
// concurrent read and write streams per work item -- the ceiling for kernels
// that read R CLVs and write W (node 2:1, fused level pair 4:3, fused
// three-level subtree 8:7).  Each lane moves f64x2 records with non-temporal
// loads/stores, grid = resident blocks, grid-stride loop, like the PLF kernels.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/stream_mix.hip -o build/stream_mix
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Ptrs {
  const f64x2 *in[8];
  f64x2 *out[8];
};

template <int R, int W, int U>
__global__ void __launch_bounds__(256) mix(Ptrs p, int64_t nrec) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < nrec; i += stride) {
    f64x2 v[U][R];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int r = 0; r < R; r++)
        v[u][r] = i + 256 * u < nrec ? __builtin_nontemporal_load(p.in[r] + i + 256 * u) : f64x2{0, 0};
#pragma unroll
    for (int u = 0; u < U; u++) {
      f64x2 s = v[u][0];
#pragma unroll
      for (int r = 1; r < R; r++) s += v[u][r];
      if (W == 0 && s.x == -1.25) p.out[0][i] = s;  // keeps reads-only variants' loads alive
      if (i + 256 * u < nrec)
#pragma unroll
        for (int w = 0; w < W; w++) __builtin_nontemporal_store(s + (double)w, p.out[w] + i + 256 * u);
    }
  }
}

template <int R, int W, int U>
void run(Ptrs p, int64_t nrec, int CUs, int per_cu = 0) {
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, mix<R, W, U>, 256, 0));
  if (per_cu > 0 && per_cu < occ) occ = per_cu;  // fewer blocks (bytes in flight) per CU
  const int grid = occ * CUs;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int rep = 0; rep < 7; rep++) {
    mix<R, W, U><<<grid, 256>>>(p, nrec);
    CK(hipEventRecord(e0));
    for (int k = 0; k < 10; k++) mix<R, W, U><<<grid, 256>>>(p, nrec);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t; CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t / 10);
  }
  std::sort(ms.begin(), ms.end());
  const double bytes = 16.0 * nrec * (R + W);
  printf("reads %d writes %d U=%d occ=%d: %7.3f ms  %6.0f GB/s  %5.1f%% of 8 TB/s\n", R, W, U, occ,
         ms[3], bytes / (ms[3] * 1e-3) / 1e9, 100.0 * bytes / (ms[3] * 1e-3) / 8e12);
}

int main() {
  const int64_t nrec = (int64_t)1 << 23;  // 128 MiB per stream (a 2^20-site f64 CLV)
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  Ptrs p;
  for (int i = 0; i < 8; i++) {
    f64x2 *a, *b;
    CK(hipMalloc(&a, nrec * 16)); CK(hipMalloc(&b, nrec * 16));
    CK(hipMemset(a, 0, nrec * 16)); CK(hipMemset(b, 0, nrec * 16));
    p.in[i] = a;
    p.out[i] = b;
  }
  const int C = prop.multiProcessorCount;
  run<1, 0, 4>(p, nrec, C); run<2, 0, 4>(p, nrec, C); run<8, 0, 2>(p, nrec, C);
  run<1, 1, 4>(p, nrec, C); run<2, 1, 2>(p, nrec, C); run<2, 1, 4>(p, nrec, C);
  run<4, 3, 1>(p, nrec, C); run<4, 3, 2>(p, nrec, C);
  run<8, 7, 1>(p, nrec, C); run<8, 7, 2>(p, nrec, C);
  run<8, 1, 1>(p, nrec, C); run<1, 8, 2>(p, nrec, C); run<0 + 1, 4, 2>(p, nrec, C);
  // bytes in flight: the same mixes at 1..4 blocks per CU
  for (int pc : {1, 2, 3, 4}) {
    run<2, 1, 1>(p, nrec, C, pc); run<2, 1, 4>(p, nrec, C, pc);
    run<4, 3, 1>(p, nrec, C, pc); run<4, 3, 2>(p, nrec, C, pc);
    run<8, 7, 1>(p, nrec, C, pc); run<8, 7, 2>(p, nrec, C, pc);
  }
  return 0;
}
