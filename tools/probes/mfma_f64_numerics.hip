#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
// D = A(16x4) * B(4x16) + C ; check layout and numerics vs a k-ordered fma chain
__global__ void k(const double* A, const double* B, const double* C, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];      // A[i][k]
  double b = B[(l >> 4) * 16 + (l & 15)];     // B[k][j]
  d4 c;
  for (int r = 0; r < 4; r++) c[r] = C[((l >> 4) + 4 * r) * 16 + (l & 15)];
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; r++) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = d[r];
}
int main() {
  double hA[64], hB[64], hC[256], hD[256];
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) / 16777216.0) * 2.0 - 1.0 + 1e-3 * ((s >> 4) & 15); };
  for (auto &x : hA) x = rnd();
  for (auto &x : hB) x = rnd() * 1e3;
  for (auto &x : hC) x = rnd() * 1e-2;
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 2048); hipMalloc(&dD, 2048);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice); hipMemcpy(dC, hC, 2048, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dA, dB, dC, dD);
  hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
  int exact_chain = 0, exact_sum = 0, close = 0;
  for (int i = 0; i < 16; i++) for (int j = 0; j < 16; j++) {
    double acc = hC[i * 16 + j];
    for (int kk = 0; kk < 4; kk++) acc = fma(hA[i * 4 + kk], hB[kk * 16 + j], acc);
    double sum = hC[i * 16 + j] + (hA[i*4]*hB[j] + hA[i*4+1]*hB[16+j] + hA[i*4+2]*hB[32+j] + hA[i*4+3]*hB[48+j]);
    exact_chain += acc == hD[i * 16 + j];
    exact_sum += sum == hD[i * 16 + j];
    close += fabs(acc - hD[i * 16 + j]) <= 1e-12 * fabs(acc);
  }
  printf("k-ordered fma chain exact: %d/256, plain sum exact: %d/256, within 1e-12: %d/256\n", exact_chain, exact_sum, close);
  return 0;
}
