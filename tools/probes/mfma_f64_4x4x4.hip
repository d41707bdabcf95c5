// Probe of v_mfma_f64_4x4x4_4b_f64 on gfx950 (not product code): operand and
// result lane maps and issue cost against v_mfma_f64_16x16x4_f64 (numerics
// not probed here).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_4x4x4.hip -o build/probe_4x4
//
// Measured on MI355X (profiles/r01_probe_mfma_f64_4x4x4.log), block b = 0..3:
//   A: lane 16k + 4b + i holds A_b[i][k];  B: lane 16k + 4b + j holds B_b[k][j];
//   C/D: lane 16i + 4b + j holds D_b[i][j]  (so a result tile is the next
//   product's B operand with i -> k, as for the 16x16x4 form);
//   issue: 20.1 cycles (512 flop) vs 64.0 cycles (2048 flop) for 16x16x4 --
//   80 % of the 16x16x4 flop rate, but no 20 -> 32 row padding for S = 20.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

// raw: lane l supplies a = A_in[l], b = B_in[l], c = C_in[l]; D_out[l]
__global__ void raw(const double *A, const double *B, const double *C, double *D) {
  const int l = threadIdx.x;
  D[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[l], B[l], C[l], 0, 0, 0);
}

template <int kind>
__global__ void timing(double *out, long long *cycles, int iters) {
  const int l = threadIdx.x;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  d4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if constexpr (kind == 0) {
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    } else {
      e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e1, 0, 0, 0);
      e2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e2, 0, 0, 0);
      e3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, e3, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  out[l] = c0 + c1 + c2 + c3 + e0[0] + e1[1] + e2[2] + e3[3];
  if (l == 0) *cycles = t1 - t0;
}

int main() {
  double hA[64], hB[64], hC[64], hD[64];
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 512); hipMalloc(&dD, 512);
  // 1. maps: A one-hot at lane L, B = distinct integers, C = 0
  printf("A one-hot lane -> nonzero D lanes (value = B lane + 1)\n");
  for (int L = 0; L < 64; L++) {
    for (int l = 0; l < 64; l++) { hA[l] = l == L; hB[l] = l + 1; hC[l] = 0; }
    hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, 512, hipMemcpyHostToDevice);
    raw<<<1, 64>>>(dA, dB, dC, dD);
    hipMemcpy(hD, dD, 512, hipMemcpyDeviceToHost);
    printf("A%02d:", L);
    for (int l = 0; l < 64; l++) if (hD[l] != 0) printf(" D%02d=B%02d", l, (int)hD[l] - 1);
    printf("\n");
  }
  // C map: A = 0 -> D = C
  for (int l = 0; l < 64; l++) { hA[l] = 0; hB[l] = 0; hC[l] = l + 1; }
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC, 512, hipMemcpyHostToDevice);
  raw<<<1, 64>>>(dA, dB, dC, dD);
  hipMemcpy(hD, dD, 512, hipMemcpyDeviceToHost);
  int cid = 0;
  for (int l = 0; l < 64; l++) cid += hD[l] == l + 1;
  printf("C passes through lane-for-lane: %d/64\n", cid);
  // 2. timing
  double *out; long long *cyc, hc;
  hipMalloc(&out, 512); hipMalloc(&cyc, 8);
  const int iters = 4096;
  timing<0><<<1, 64>>>(out, cyc, iters);
  hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
  printf("4x4x4_4b: %.1f cycles per MFMA (4 independent accumulators)\n", (double)hc / (4.0 * iters));
  timing<1><<<1, 64>>>(out, cyc, iters);
  hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
  printf("16x16x4: %.1f cycles per MFMA (4 independent accumulators)\n", (double)hc / (4.0 * iters));
  return 0;
}
