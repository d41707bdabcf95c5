// Probe (not product code): the 2-read/1-write stream of the headline node
// kernel's bytes (2^20 f64 DNA sites: 3 x 128 MiB, 6 rotating buffer sets)
// under each cache policy of the gfx950 vector memory instructions.  Loads and
// stores go through buffer instructions whose aux operand sets the policy bits
// (1 = sc0, 2 = nt, 16 = sc1; checked in the emitted .s), so a policy the
// product's __builtin_nontemporal_load / _store (global_* ... nt) cannot
// express is measured on the same access pattern: every wave memory
// instruction one contiguous 1 KiB, V 16-B loads per input per lane per trip.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/stream_policy.hip -o build/stream_policy
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// reference: the product's global loads / stores with the nt bit
template <int V>
__global__ void __launch_bounds__(256) stream_global(const f64x2 *__restrict__ a, const f64x2 *__restrict__ b,
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

// buffer form: LP / SP = aux policy of the loads / stores.  nrec * 16 < 2^31.
template <int V, int LP, int SP>
__global__ void __launch_bounds__(256) stream_buf(const f64x2 *__restrict__ a, const f64x2 *__restrict__ b,
                                                  f64x2 *__restrict__ c, int64_t nrec) {
  const int bytes = (int)(nrec * 16);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)a, 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)b, 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)c, 0, bytes, 0x00020000);
  const int stride = gridDim.x * 256 * V * 16;
  for (int o = (blockIdx.x * 256 * V + threadIdx.x) * 16; o < bytes; o += stride) {
    i32x4 x[V], y[V];
#pragma unroll
    for (int v = 0; v < V; v++) {
      x[v] = __builtin_amdgcn_raw_buffer_load_b128(ra, o + 4096 * v, 0, LP);
      y[v] = __builtin_amdgcn_raw_buffer_load_b128(rb, o + 4096 * v, 0, LP);
    }
#pragma unroll
    for (int v = 0; v < V; v++) {
      const f64x2 s = __builtin_bit_cast(f64x2, x[v]) + __builtin_bit_cast(f64x2, y[v]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, s), rc, o + 4096 * v, 0, SP);
    }
  }
}

int main(int argc, char **argv) {
  const int64_t nrec = (argc > 1 ? atoll(argv[1]) : (1 << 20)) * 8;  // f64x2 records per stream
  if (nrec * 16 >= (1ll << 31)) { printf("too large for 32-bit buffer offsets\n"); return 1; }
  const int R = 6, reps = 40, rounds = 5;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  std::vector<f64x2 *> A(R), B(R), C(R);
  for (int r = 0; r < R; r++) {
    CK(hipMalloc(&A[r], nrec * 16)); CK(hipMalloc(&B[r], nrec * 16)); CK(hipMalloc(&C[r], nrec * 16));
    CK(hipMemset(A[r], 0, nrec * 16)); CK(hipMemset(B[r], 0, nrec * 16));
  }
  struct Var { std::string name; std::function<void(int)> run; std::vector<float> us; };
  std::vector<Var> vs;
#define ADDG(V, G)                                                                                 \
  vs.push_back({"global nt/nt V=" #V " grid " #G "/CU", [&, g = G](int r) {                       \
    stream_global<V><<<CUs * g, 256>>>(A[r], B[r], C[r], nrec); }, {}});
#define ADDB(V, LP, SP, G, NAME)                                                                   \
  vs.push_back({"buffer " NAME " V=" #V " grid " #G "/CU", [&, g = G](int r) {                    \
    stream_buf<V, LP, SP><<<CUs * g, 256>>>(A[r], B[r], C[r], nrec); }, {}});
  ADDG(2, 4) ADDG(1, 2)
  ADDB(2, 2, 2, 4, "ld nt / st nt")
  ADDB(2, 0, 2, 4, "ld -- / st nt")
  ADDB(2, 3, 2, 4, "ld sc0 nt / st nt")
  ADDB(2, 18, 2, 4, "ld sc1 nt / st nt")
  ADDB(2, 19, 2, 4, "ld sc0 sc1 nt / st nt")
  ADDB(2, 17, 2, 4, "ld sc0 sc1 / st nt")
  ADDB(2, 2, 19, 4, "ld nt / st sc0 sc1 nt")
  ADDB(2, 2, 0, 4, "ld nt / st --")
  ADDB(2, 2, 17, 4, "ld nt / st sc0 sc1")
  ADDB(2, 19, 19, 4, "ld sc0 sc1 nt / st sc0 sc1 nt")
  ADDB(1, 2, 2, 2, "ld nt / st nt")
  ADDB(1, 19, 2, 2, "ld sc0 sc1 nt / st nt")
  ADDB(1, 18, 2, 2, "ld sc1 nt / st nt")
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
  printf("2R+1W stream, %lld x 16 B per stream, %d buffer sets, %d reps x %d rounds interleaved\n",
         (long long)nrec, R, reps, rounds);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6, bytes = 3.0 * nrec * 16;
    printf("%-48s median %8.2f us (min %8.2f)  %5.1f%% of 8 TB/s\n", v.name.c_str(), v.us[v.us.size() / 2],
           v.us[0], 100.0 * bytes / t / 8e12);
  }
  return 0;
}
