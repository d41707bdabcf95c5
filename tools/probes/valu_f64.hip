// Probe (not product code): f64 VALU issue rate and dependent latency on the
// MI355X, for the protein EXACT kernel (every multiply-add is a separate
// v_mul_f64 + v_add_f64, plf()'s rounding).  Each lane runs C independent
// chains x = x*a + b (mul, then a dependent add) for M steps; grid = W blocks
// of 256 threads per CU (W waves per SIMD).  Reports cycles per VALU
// instruction per SIMD (4 = full rate) from the kernel time at the measured
// shader clock (s_memrealtime vs s_memtime inside a spin kernel, and inside
// the measured kernel itself: block 0's first lane brackets its own run).
// Round 5: up to 8 waves per SIMD (the CDNA4 cap) x 16
// chains, and the exact kernel's row pattern (independent mul, dependent add)
// at the same occupancies, until the rate plateaus.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/probes/valu_f64.hip -o build/valu_f64
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int C, bool kChain>
__global__ void __launch_bounds__(256) chains(double *out, long long *clk_out, int M, double a, double b) {
  long long t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  double x[C];
#pragma unroll
  for (int i = 0; i < C; i++) x[i] = threadIdx.x * 1e-3 + i;
  for (int m = 0; m < M; m++) {
#pragma unroll
    for (int i = 0; i < C; i++) {
      if constexpr (kChain) {
        x[i] = x[i] * a;  // v_mul_f64
        x[i] = x[i] + b;  // v_add_f64, dependent
      } else {
        // the exact kernel's row: u = q0; u += a_l * p_l ... (mul independent
        // of the chain, add dependent on the previous add)
        const double p = (x[(i + 1) % C] * a);
        x[i] = x[i] + p;
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < C; i++) s += x[i];
  if (s == 1.2345) out[threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk_out[0] = __builtin_amdgcn_s_memtime() - t0;
    clk_out[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

__global__ void clk(long long *o, int spin) {
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  volatile int k = 0;
  for (int i = 0; i < spin; i++) k += i;
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; }
}

int main() {
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  double *out; CK(hipMalloc(&out, 4096));
  long long *o; CK(hipMalloc(&o, 16));
  long long *ko; CK(hipMalloc(&ko, 16));
  clk<<<1, 64>>>(o, 2000000);
  long long h[2]; CK(hipMemcpy(h, o, 16, hipMemcpyDeviceToHost));
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;  // memrealtime = 100 MHz
  printf("shader clock (s_memtime / s_memrealtime): %.3f GHz\n", ghz);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int M = 4096;
  auto run = [&](const char *name, auto kern, int C, int W, int instr_per_step) {
    std::vector<float> t;
    std::vector<double> kg;
    for (int r = 0; r < 7; r++) {
      CK(hipEventRecord(e0, 0));
      kern<<<CUs * W, 256>>>(out, ko, M, 0.999, 1e-3);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
      long long k[2]; CK(hipMemcpy(k, ko, 16, hipMemcpyDeviceToHost));
      kg.push_back((double)k[0] / ((double)k[1] / 100e6) / 1e9);
    }
    std::sort(t.begin(), t.end());
    std::sort(kg.begin(), kg.end());
    const double sec = t[3] * 1e-3, g = kg[3];
    const double instr_per_simd = (double)W * M * C * instr_per_step;  // W waves per SIMD
    printf("%-26s C=%2d W=%d  %8.1f us  %5.2f cycles/instr/SIMD at %.3f GHz (in-kernel clock; "
           "%5.2f at the spin clock)\n", name, C, W, sec * 1e6, sec * g * 1e9 / instr_per_simd, g,
           sec * ghz * 1e9 / instr_per_simd);
  };
#define RUN(C, W)                                                     \
  run("mul->add chains", chains<C, true>, C, W, 2);                   \
  run("exact row (mul, dep. add)", chains<C, false>, C, W, 2);

  RUN(1, 1) RUN(2, 1) RUN(4, 1) RUN(8, 1) RUN(16, 1)
  RUN(1, 2) RUN(2, 2) RUN(4, 2) RUN(8, 2) RUN(16, 2)
  RUN(1, 4) RUN(2, 4) RUN(4, 4) RUN(8, 4) RUN(16, 4)
  RUN(1, 8) RUN(2, 8) RUN(4, 8) RUN(8, 8) RUN(16, 8)
  CK(hipGetLastError());
  return 0;
}
