// Probe of v_mfma_f32_4x4x1_16b_f32 on gfx950 (not product code): operand and
// result lane maps, issue cost against v_mfma_f32_16x16x4_f32, numerics of a
// K = 20 chain of K = 1 steps against a k-ordered fmaf chain, and the 4x4
// (lane group x register) transpose by v_permlane32_swap + v_permlane16_swap.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/mfma_f32_4x4x1.hip -o build/probe_f32_4x4x1
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

// raw: lane l supplies a = A_in[l], b = B_in[l], c = C_in[4l..4l+3]; D_out[4l..]
__global__ void raw(const float *A, const float *B, const float *C, float *D) {
  const int l = threadIdx.x;
  f4 c = {C[4 * l], C[4 * l + 1], C[4 * l + 2], C[4 * l + 3]};
  f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], c, 0, 0, 0);
  for (int r = 0; r < 4; r++) D[4 * l + r] = d[r];
}

// chain: per wave w, lane l: D = sum over k = 0..19 of a[w][k][l] * b[w][k][l]
// as 20 chained K = 1 MFMAs from C = 0
__global__ void chain(const float *A, const float *B, float *D) {
  const int w = blockIdx.x, l = threadIdx.x;
  f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 20; k++)
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(A[(w * 20 + k) * 64 + l], B[(w * 20 + k) * 64 + l], d, 0, 0, 0);
  for (int r = 0; r < 4; r++) D[(w * 64 + l) * 4 + r] = d[r];
}

template <int kind>
__global__ void timing(float *out, long long *cycles, int iters) {
  const int l = threadIdx.x;
  float a = 1.0f + l * 1e-3f, b = 1.0f - l * 1e-3f;
  f4 e0 = {0, 0, 0, 0}, e1 = e0, e2 = e0, e3 = e0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if constexpr (kind == 0) {
      e0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e1, 0, 0, 0);
      e2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e2, 0, 0, 0);
      e3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, e3, 0, 0, 0);
    } else {
      e0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, e1, 0, 0, 0);
      e2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, e2, 0, 0, 0);
      e3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, e3, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  out[l] = e0[0] + e1[1] + e2[2] + e3[3];
  if (l == 0) *cycles = t1 - t0;
}

// 4x4 transpose of (lane group g = l >> 4) x (register r): v[r] of group g
// becomes S[r][g] where S[g][r] was v[r] of group g on entry.  (The first run
// of this probe cast with __builtin_bit_cast, which on a vector element -- the
// builtin's pair result p[1] -- reads element 0 with this compiler: 64/256.)
__device__ __forceinline__ void transpose44(float (&v)[4]) {
  // stage 1: off-diagonal 2x2 blocks (groups 2,3 of v[r] <-> groups 0,1 of v[r+2])
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[r]), __float_as_uint(v[r + 2]), false, false);
    v[r] = __uint_as_float(p[0]);
    v[r + 2] = __uint_as_float(p[1]);
  }
  // stage 2: inside each 2x2 block (odd groups of v[r] <-> even groups of v[r+1])
#pragma unroll
  for (int r = 0; r < 4; r += 2) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[r]), __float_as_uint(v[r + 1]), false, false);
    v[r] = __uint_as_float(p[0]);
    v[r + 1] = __uint_as_float(p[1]);
  }
}

__global__ void tr(float *out) {
  const int l = threadIdx.x, g = l >> 4, lo = l & 15;
  float v[4];
  for (int r = 0; r < 4; r++) v[r] = 1000.f * lo + 10.f * g + r;  // S[g][r]
  transpose44(v);
  for (int r = 0; r < 4; r++) out[4 * l + r] = v[r];
}

static float fmaf_chain(const float *a, const float *b) {
  float s = 0.f;
  for (int k = 0; k < 20; k++) s = std::fmaf(a[k], b[k], s);
  return s;
}

static float draw(std::mt19937 &g, int mode) {
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::uniform_int_distribution<int> e(-30, 30), pick(0, 19);
  float v = u(g);
  switch (mode) {
    case 0: return v;
    case 1: return std::ldexp(v, e(g));           // wide exponents: cancellation, rounding ties
    case 2: return pick(g) == 0 ? 0.f * v : v;     // signed zeros
    case 3: return std::ldexp(v, -120 - (pick(g) % 10));  // denormal inputs / products
    default: return pick(g) < 2 ? -0.f : std::ldexp(v, e(g) - 60);
  }
}

int main() {
  float hA[64], hB[64], hC[256], hD[256];
  float *dA, *dB, *dC, *dD;
  hipMalloc(&dA, 256); hipMalloc(&dB, 256); hipMalloc(&dC, 1024); hipMalloc(&dD, 1024);
  // 1. maps: A one-hot at lane L, B = distinct integers, C = 0
  printf("A one-hot lane -> nonzero D (lane.reg = B lane)\n");
  for (int L = 0; L < 64; L += 5) {
    for (int l = 0; l < 64; l++) { hA[l] = l == L; hB[l] = l + 1; }
    for (int i = 0; i < 256; i++) hC[i] = 0;
    hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, 1024, hipMemcpyHostToDevice);
    raw<<<1, 64>>>(dA, dB, dC, dD);
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    printf("A%02d:", L);
    for (int i = 0; i < 256; i++) if (hD[i] != 0) printf(" D%02d.%d=B%02d", i / 4, i % 4, (int)hD[i] - 1);
    printf("\n");
  }
  // hypothesis: A lane l = A_b[l%4][0], B lane l = B_b[0][l%4], D lane l reg r = D_b[r][l%4], b = l/4
  int ok_map = 0;
  for (int L = 0; L < 64; L++) {
    for (int l = 0; l < 64; l++) { hA[l] = l == L; hB[l] = l + 1; }
    hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
    raw<<<1, 64>>>(dA, dB, dC, dD);
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    bool ok = true;
    for (int l = 0; l < 64; l++)
      for (int r = 0; r < 4; r++) {
        const float want = (l / 4 == L / 4 && r == L % 4) ? (float)(l + 1) : 0.f;
        ok = ok && hD[4 * l + r] == want;
      }
    ok_map += ok;
  }
  printf("map hypothesis (A lane l = A_b[l%%4], B lane l = B_b[l%%4], D lane l reg r = D_b[r][l%%4]): %d/64\n", ok_map);
  for (int l = 0; l < 64; l++) hA[l] = hB[l] = 0;
  for (int i = 0; i < 256; i++) hC[i] = i + 1;
  hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC, 1024, hipMemcpyHostToDevice);
  raw<<<1, 64>>>(dA, dB, dC, dD);
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  int cid = 0;
  for (int i = 0; i < 256; i++) cid += hD[i] == i + 1;
  printf("C passes through lane.reg for lane.reg: %d/256\n", cid);
  // 2. timing
  float *out; long long *cyc, hc;
  hipMalloc(&out, 256); hipMalloc(&cyc, 8);
  const int iters = 4096;
  timing<0><<<1, 64>>>(out, cyc, iters);
  hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b: %.1f cycles per MFMA (4 independent chains)\n", (double)hc / (4.0 * iters));
  timing<1><<<1, 64>>>(out, cyc, iters);
  hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
  printf("16x16x4:   %.1f cycles per MFMA (4 independent chains)\n", (double)hc / (4.0 * iters));
  // 3. numerics: K = 20 chains vs fmaf chains, per the map hypothesis
  const int W = 4096;
  std::vector<float> A((size_t)W * 20 * 64), B(A.size()), D((size_t)W * 64 * 4);
  float *gA, *gB, *gD;
  hipMalloc(&gA, A.size() * 4); hipMalloc(&gB, B.size() * 4); hipMalloc(&gD, D.size() * 4);
  std::mt19937 rng(7);
  long long bad[5] = {}, tot[5] = {};
  for (int mode = 0; mode < 5; mode++) {
    for (auto &x : A) x = draw(rng, mode);
    for (auto &x : B) x = draw(rng, mode == 3 ? 0 : mode);
    hipMemcpy(gA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(gB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    chain<<<W, 64>>>(gA, gB, gD);
    hipMemcpy(D.data(), gD, D.size() * 4, hipMemcpyDeviceToHost);
    for (int w = 0; w < W; w++)
      for (int l = 0; l < 64; l++)
        for (int r = 0; r < 4; r++) {
          // D_b[r][j] with b = l/4, j = l%4: A from lane 4b + r, B from lane l
          float a[20], b[20];
          for (int k = 0; k < 20; k++) {
            a[k] = A[((size_t)w * 20 + k) * 64 + 4 * (l / 4) + r];
            b[k] = B[((size_t)w * 20 + k) * 64 + l];
          }
          const float want = fmaf_chain(a, b), got = D[((size_t)w * 64 + l) * 4 + r];
          uint32_t x, y;
          memcpy(&x, &want, 4); memcpy(&y, &got, 4);
          bad[mode] += x != y;
          tot[mode]++;
        }
  }
  const char *names[5] = {"U(-1,1)", "wide exponents", "signed zeros", "denormal A", "mixed tiny/-0"};
  for (int mode = 0; mode < 5; mode++)
    printf("numerics %-16s: %lld / %lld outputs differ from the k-ordered fmaf chain (bitwise)\n", names[mode],
           bad[mode], tot[mode]);
  // 4. transpose
  tr<<<1, 64>>>(dD);
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  int tok = 0;
  for (int l = 0; l < 64; l++)
    for (int r = 0; r < 4; r++) tok += hD[4 * l + r] == 1000.f * (l & 15) + 10.f * r + (l >> 4);
  printf("permlane32/16 swap transpose (group x reg): %d/256 correct\n", tok);
  return 0;
}
