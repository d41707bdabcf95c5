// Probe (not product code): 2-read/1-write stream rate vs bytes in flight
// per wave (V = 16-B loads per input per lane per trip) and grid (blocks per
// CU), 2^20 f64 DNA sites' worth of bytes (3 x 128 MiB), 4 rotating buffer
// sets.  The headline kernel issues its trip's loads in 4 groups with a wait
// after each (few bytes in flight per wave) and beats the V=4 stream at 2^22
// sites: is the V=4 stream the ceiling?
//   hipcc --offload-arch=gfx950 -O3 tools/probes/stream_depth.hip -o build/stream_depth
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int V, bool SER>
__global__ void __launch_bounds__(256) stream3(const f64x2 *__restrict__ a, const f64x2 *__restrict__ b,
                                               f64x2 *__restrict__ c, int64_t nrec) {
  const int64_t stride = (int64_t)gridDim.x * 256 * V;
  for (int64_t i = (int64_t)blockIdx.x * 256 * V + threadIdx.x; i < nrec; i += stride) {
    f64x2 x[V], y[V];
#pragma unroll
    for (int v = 0; v < V; v++) {
      x[v] = __builtin_nontemporal_load(a + i + 256 * v);
      y[v] = __builtin_nontemporal_load(b + i + 256 * v);
      if (SER) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int v = 0; v < V; v++) __builtin_nontemporal_store(x[v] + y[v], c + i + 256 * v);
  }
}

int main(int argc, char **argv) {
  const int64_t nrec = (argc > 1 ? atoll(argv[1]) : (1 << 20)) * 8;  // f64x2 records per stream
  const int R = 4, reps = 40, rounds = 5;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  std::vector<f64x2 *> A(R), B(R), C(R);
  for (int r = 0; r < R; r++) {
    CK(hipMalloc(&A[r], nrec * 16)); CK(hipMalloc(&B[r], nrec * 16)); CK(hipMalloc(&C[r], nrec * 16));
    CK(hipMemset(A[r], 0, nrec * 16)); CK(hipMemset(B[r], 0, nrec * 16));
  }
  struct Var { std::string name; std::function<void(int)> run; std::vector<float> us; };
  std::vector<Var> vs;
#define ADD(V, SER, G)                                                                             \
  vs.push_back({"V=" #V " ser=" #SER " grid " #G "/CU", [&, g = G](int r) {                       \
    stream3<V, SER><<<CUs * g, 256>>>(A[r], B[r], C[r], nrec); }, {}});
  ADD(1, false, 2) ADD(1, false, 4) ADD(1, false, 8)
  ADD(2, false, 2) ADD(2, false, 4) ADD(2, false, 8)
  ADD(4, false, 2) ADD(4, false, 4) ADD(4, false, 8)
  ADD(4, true, 4) ADD(4, true, 8) ADD(8, false, 4) ADD(2, true, 8)
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; rd++)
    for (auto &v : vs) {
      for (int i = 0; i < 3; i++) v.run(i % R);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; i++) v.run(i % R);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / reps);
    }
  printf("2R+1W stream, %lld MiB per stream, %d rounds interleaved\n", (long long)(nrec * 16 >> 20), rounds);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6;
    printf("%-28s median %8.2f us  %5.1f%% of 8 TB/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           100.0 * 48.0 * nrec / t / 8e12);
  }
  return 0;
}
