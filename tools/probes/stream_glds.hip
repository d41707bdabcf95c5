// Probe (not product code): the 2-read/1-write stream with its reads moved by
// LDS-DMA (`global_load_lds_dwordx4`, no VGPR destination) into a wave-private
// LDS ring D trips deep, then ds_read -> add -> NT store, against the
// register-staged streams of tools/probes/stream_depth.hip in the same
// process.  Question: is the headline kernel's ceiling (the V = 1..4 register
// streams, 78-81 % at 2^20 f64 sites) a property of HBM or of how many bytes a
// wave can keep in flight in VGPRs?  The DMA ring keeps D x 2 KiB per wave in
// flight with no registers held.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/stream_glds.hip -o build/stream_glds
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef double f64x2 __attribute__((ext_vector_type(2)));

// one 16-B LDS-DMA per lane: LDS bytes [dst + 16*lane, +16) <- *src (per-lane)
__device__ __forceinline__ void glds16(const void *src, unsigned dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

// Wave w owns LDS [w * D * 2048, +D*2048): slot s = x chunk (1 KiB) + y chunk.
// Every wave runs exactly T trips of 64 records per input (host guarantees).
template <int D>
__global__ void __launch_bounds__(256) stream_glds(const f64x2 *__restrict__ a, const f64x2 *__restrict__ b,
                                                   f64x2 *__restrict__ c, int64_t T) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  const unsigned ring = (unsigned)(uintptr_t)lds + (unsigned)wv * D * 2048u;
  auto rec = [&](int64_t t) { return (t * nwaves + w) * 64 + lane; };  // grid-strided wave trips
#pragma unroll
  for (int d = 0; d < D; d++) {
    glds16(a + rec(d), ring + d * 2048);
    glds16(b + rec(d), ring + d * 2048 + 1024);
  }
  for (int64_t t = 0; t < T; t++) {
    const int s = (int)(t % D);
    // glds(t) landed: 2(D-1) later DMA loads may still be in flight.  Loads
    // retire in order, stores need not (a count that also credits the
    // interleaved stores, 3(D-1), let glds(t) be read early), so the wait
    // also drains the stores issued since
    if (t + D <= T) wait_vm<2 * (D - 1)>();
    else wait_vm<0>();
    const f64x2 x = *reinterpret_cast<const f64x2 *>(lds + (ring - (unsigned)(uintptr_t)lds) + s * 2048 + lane * 16);
    const f64x2 y = *reinterpret_cast<const f64x2 *>(lds + (ring - (unsigned)(uintptr_t)lds) + s * 2048 + 1024 + lane * 16);
    __builtin_nontemporal_store(x + y, c + rec(t));
    if (t + D < T) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot s read before it is refilled
      glds16(a + rec(t + D), ring + s * 2048);
      glds16(b + rec(t + D), ring + s * 2048 + 1024);
    }
  }
}

template <int V>
__global__ void __launch_bounds__(256) stream3(const f64x2 *__restrict__ a, const f64x2 *__restrict__ b,
                                               f64x2 *__restrict__ c, int64_t nrec) {
  const int64_t stride = (int64_t)gridDim.x * 256 * V;
  for (int64_t i = (int64_t)blockIdx.x * 256 * V + threadIdx.x; i < nrec; i += stride) {
    f64x2 x[V], y[V];
#pragma unroll
    for (int v = 0; v < V; v++) {
      x[v] = __builtin_nontemporal_load(a + i + 256 * v);
      y[v] = __builtin_nontemporal_load(b + i + 256 * v);
    }
#pragma unroll
    for (int v = 0; v < V; v++) __builtin_nontemporal_store(x[v] + y[v], c + i + 256 * v);
  }
}

__global__ void fill(f64x2 *p, int64_t n, double s) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = f64x2{s + (double)(i & 1023), s - (double)(i & 511)};
}

int main(int argc, char **argv) {
  const int64_t sites = argc > 1 ? atoll(argv[1]) : (1 << 20);
  const int64_t nrec = sites * 8;  // f64x2 records per stream (128 B per f64 DNA site)
  const int R = 4, reps = 40, rounds = 5;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  std::vector<f64x2 *> A(R), B(R), C(R);
  for (int r = 0; r < R; r++) {
    CK(hipMalloc(&A[r], nrec * 16)); CK(hipMalloc(&B[r], nrec * 16)); CK(hipMalloc(&C[r], nrec * 16));
    fill<<<1024, 256>>>(A[r], nrec, 1.0 + r); fill<<<1024, 256>>>(B[r], nrec, 2.0 + r);
  }
  CK(hipDeviceSynchronize());
  struct Var { std::string name; std::function<void(int)> run; std::vector<float> us; };
  std::vector<Var> vs;
#define ADDV(V, G) vs.push_back({"regs V=" #V " grid " #G "/CU", [&](int r) { \
    stream3<V><<<CUs * G, 256>>>(A[r], B[r], C[r], nrec); }, {}});
#define ADDG(D, G)                                                                                 \
  {                                                                                                \
    const int64_t waves = (int64_t)CUs * G * 4, T = nrec / 64 / waves;                           \
    if (T * 64 * waves == nrec && T >= D) {                                                        \
      CK(hipFuncSetAttribute((const void *)&stream_glds<D>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * D * 2048)); \
      vs.push_back({"glds D=" #D " grid " #G "/CU (" + std::to_string(T) + " trips)", [&, T](int r) { \
        stream_glds<D><<<CUs * G, 256, 4 * D * 2048>>>(A[r], B[r], C[r], T); }, {}});            \
    }                                                                                              \
  }
  ADDV(1, 2) ADDV(4, 2) ADDV(4, 4)
  ADDG(2, 1) ADDG(4, 1) ADDG(8, 1)
  ADDG(2, 2) ADDG(4, 2) ADDG(8, 2)
  ADDG(2, 4) ADDG(4, 4)
  // correctness of the DMA ring: c = a + b everywhere
  {
    std::vector<f64x2> ha(nrec), hb(nrec), hc(nrec);
    CK(hipMemcpy(ha.data(), A[0], nrec * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), B[0], nrec * 16, hipMemcpyDeviceToHost));
    for (size_t v = 3; v < vs.size(); v++) {
      CK(hipMemset(C[0], 0, nrec * 16));
      vs[v].run(0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(hc.data(), C[0], nrec * 16, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int64_t i = 0; i < nrec; i++) {
        const f64x2 e = ha[i] + hb[i];
        if (hc[i].x != e.x || hc[i].y != e.y) bad++;
      }
      printf("check %-36s %s (%lld bad)\n", vs[v].name.c_str(), bad ? "WRONG" : "ok", (long long)bad);
    }
  }
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
  CK(hipGetLastError());
  printf("2R+1W stream, %lld MiB per stream (%lld f64 DNA sites), %d rounds interleaved\n",
         (long long)(nrec * 16 >> 20), (long long)sites, rounds);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6;
    printf("%-40s median %8.2f us  %5.1f%% of 8 TB/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           100.0 * 3.0 * nrec * 16 / t / 8e12);
  }
  return 0;
}
