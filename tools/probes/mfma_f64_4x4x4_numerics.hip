// Probe (not product code): is v_mfma_f64_4x4x4_4b_f64 bit-for-bit a
// k-ordered fma chain, like v_mfma_f64_16x16x4_f64?  Lane maps from
// mfma_f64_4x4x4.hip: A lane 16k+4b+i = A_b[i][k], B lane 16k+4b+j = B_b[k][j],
// C/D lane 16i+4b+j = D_b[i][j].  Many trials with wide magnitudes and mixed
// signs (so reassociation or a single-rounding dot product would show).
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_f64_4x4x4_numerics.hip -o build/probe_4x4_num
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void k4(const double *A, const double *B, const double *C, double *D, int trials) {
  const int l = threadIdx.x;
  for (int t = blockIdx.x; t < trials; t += gridDim.x) {
    const double *a = A + 64 * t, *b = B + 64 * t, *c = C + 64 * t;
    D[64 * t + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 0);
  }
}

typedef double d4 __attribute__((ext_vector_type(4)));
// 16x16x4 on the same kind of data: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15],
// C/D register r of lane l = D[(l>>4) + 4r][l&15]
__global__ void k16(const double *A, const double *B, const double *C, double *D, int trials) {
  const int l = threadIdx.x;
  for (int t = blockIdx.x; t < trials; t += gridDim.x) {
    d4 c;
    for (int r = 0; r < 4; r++) c[r] = C[256 * t + 64 * r + l];
    const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[64 * t + l], B[64 * t + l], c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[256 * t + 64 * r + l] = d[r];
  }
}

int main() {
  const int trials = 20000;
  std::vector<double> hA(64 * trials), hB(64 * trials), hC(64 * trials), hD(64 * trials);
  uint64_t s = 0x123456789abcdefull;
  auto u01 = [&]() {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return (double)(s >> 11) * (1.0 / 9007199254740992.0);
  };
  auto val = [&]() {  // sign * 2^[-20, 20) * [1, 2)
    const double m = 1.0 + u01();
    const int e = (int)(u01() * 40) - 20;
    return (u01() < 0.5 ? -1.0 : 1.0) * std::ldexp(m, e);
  };
  for (int t = 0; t < trials; t++)
    for (int l = 0; l < 64; l++) {
      hA[64 * t + l] = val();
      hB[64 * t + l] = val();
      hC[64 * t + l] = (t % 3 == 0) ? 0.0 : val();
    }
  double *dA, *dB, *dC, *dD;
  const size_t bytes = 64 * trials * sizeof(double);
  hipMalloc(&dA, bytes); hipMalloc(&dB, bytes); hipMalloc(&dC, bytes); hipMalloc(&dD, bytes);
  hipMemcpy(dA, hA.data(), bytes, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB.data(), bytes, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC.data(), bytes, hipMemcpyHostToDevice);
  k4<<<256, 64>>>(dA, dB, dC, dD, trials);
  hipMemcpy(hD.data(), dD, bytes, hipMemcpyDeviceToHost);
  long chain = 0, rev = 0, plain = 0, total = 0;
  for (int t = 0; t < trials; t++)
    for (int b = 0; b < 4; b++)
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
          const double *A = &hA[64 * t], *B = &hB[64 * t];
          const double c = hC[64 * t + 16 * i + 4 * b + j];
          double acc = c, r = c, p = 0.0;
          for (int k = 0; k < 4; k++) acc = std::fma(A[16 * k + 4 * b + i], B[16 * k + 4 * b + j], acc);
          for (int k = 3; k >= 0; k--) r = std::fma(A[16 * k + 4 * b + i], B[16 * k + 4 * b + j], r);
          for (int k = 0; k < 4; k++) p += A[16 * k + 4 * b + i] * B[16 * k + 4 * b + j];
          p += c;
          const double d = hD[64 * t + 16 * i + 4 * b + j];
          chain += d == acc;
          rev += d == r;
          plain += d == p;
          total++;
        }
  printf("4x4x4_4b f64: k-ordered fma chain exact %ld/%ld, reversed chain %ld, separate mul/add %ld\n",
         chain, total, rev, plain);
  // 16x16x4 with the same generator (C of 256 values per trial)
  const int t16 = trials / 4;
  std::vector<double> C16(256 * t16), D16(256 * t16);
  for (auto &x : C16) x = u01() < 0.3 ? 0.0 : val();
  double *dC16, *dD16;
  hipMalloc(&dC16, 256 * t16 * sizeof(double)); hipMalloc(&dD16, 256 * t16 * sizeof(double));
  hipMemcpy(dC16, C16.data(), 256 * t16 * sizeof(double), hipMemcpyHostToDevice);
  k16<<<256, 64>>>(dA, dB, dC16, dD16, t16);
  hipMemcpy(D16.data(), dD16, 256 * t16 * sizeof(double), hipMemcpyDeviceToHost);
  long chain16 = 0, total16 = 0;
  for (int t = 0; t < t16; t++)
    for (int r = 0; r < 4; r++)
      for (int l = 0; l < 64; l++) {
        const int i = (l >> 4) + 4 * r, j = l & 15;
        double acc = C16[256 * t + 64 * r + l];
        for (int k = 0; k < 4; k++) acc = std::fma(hA[64 * t + 16 * k + i], hB[64 * t + 16 * k + j], acc);
        chain16 += D16[256 * t + 64 * r + l] == acc;
        total16++;
      }
  printf("16x16x4 f64: k-ordered fma chain exact %ld/%ld\n", chain16, total16);
  return chain == total && chain16 == total16 ? 0 : 1;
}
