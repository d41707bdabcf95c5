// prot_movement.hip -- probe (not product code): the HBM rate of three data
// movement forms for the f32 protein node (320-B site records, x3 = f(x1, x2),
// 2 reads : 1 write), with no arithmetic beyond one add per value:
//   block : the product kernel's form -- a 64-site tile per 256-thread block,
//           staged through LDS with block barriers, one tile in flight
//           (plf_prot_mfma32_kernel's kAblate = 3 measures the same thing);
//   wave  : every wave owns 16-site sub-tiles (5 KB per child), staged
//           through a private LDS region with no block barrier; the next
//           sub-tile's loads are in flight while the current one is
//           written, read back and stored;
//   stream: 16 B per lane straight from registers (the 2R:1W ceiling).
// Each form is checked against x1 + x2 elementwise.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/prot_movement.hip -o build/prot_movement
//   (-DPROBE_CHUNKS=40: the f64 record, 640 B)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); }  \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
#ifndef PROBE_CHUNKS
#define PROBE_CHUNKS 20
#endif
constexpr int kChunks = PROBE_CHUNKS;  // 16-B chunks per site record: 20 (f32, 80 floats) or 40 (f64)

__global__ void fill(float *p, int64_t n, unsigned seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (float)((i * 2654435761u + seed) % 1000) * 0.001f;
}

// block form: 64 sites x 20 chunks = 1280 chunks per child, 5 per thread
__global__ void __launch_bounds__(256) mv_block(const f32x4 *__restrict__ x1, const f32x4 *__restrict__ x2,
                                                f32x4 *__restrict__ x3, int64_t tiles) {
  __shared__ f32x4 t1[64 * (kChunks + 1)], t2[64 * (kChunks + 1)];
  for (int64_t b = blockIdx.x; b < tiles; b += gridDim.x) {
    f32x4 a[kChunks / 4], c[kChunks / 4];
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) a[i] = __builtin_nontemporal_load(x1 + b * (64 * kChunks) + threadIdx.x + 256 * i);
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) c[i] = __builtin_nontemporal_load(x2 + b * (64 * kChunks) + threadIdx.x + 256 * i);
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) {
      const int j = threadIdx.x + 256 * i, s = j / kChunks, q = j % kChunks;
      t1[s * (kChunks + 1) + q] = a[i];
      t2[s * (kChunks + 1) + q] = c[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) {  // read back in another thread's order (site-major rows)
      const int j = threadIdx.x + 256 * i, s = j % 64, q = j / 64;
      t1[s * (kChunks + 1) + q] = t1[s * (kChunks + 1) + q] + t2[s * (kChunks + 1) + q];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) {
      const int j = threadIdx.x + 256 * i, s = j / kChunks, q = j % kChunks;
      __builtin_nontemporal_store(t1[s * (kChunks + 1) + q], x3 + b * (64 * kChunks) + j);
    }
    __syncthreads();
  }
}

// block form with x3 stored straight from registers in the f32 MFMA kernel's
// output layout (wave = category c; sub-tile t: lane (lo16, g) holds chunk
// 5c + g of site 16t + lo16; then lane l holds chunk 5c + 4 of site l): 64-B
// pieces at a 320-B stride instead of whole coalesced records (f32 only)
#if PROBE_CHUNKS == 20
__global__ void __launch_bounds__(256) mv_block_scatter(const f32x4 *__restrict__ x1, const f32x4 *__restrict__ x2,
                                                        f32x4 *__restrict__ x3, int64_t tiles) {
  __shared__ f32x4 t1[64 * (kChunks + 1)], t2[64 * (kChunks + 1)];
  const int c = threadIdx.x >> 6, lane = threadIdx.x & 63, lo16 = lane & 15, g = lane >> 4;
  for (int64_t b = blockIdx.x; b < tiles; b += gridDim.x) {
    f32x4 a[5], d[5];
#pragma unroll
    for (int i = 0; i < 5; i++) a[i] = __builtin_nontemporal_load(x1 + b * 1280 + threadIdx.x + 256 * i);
#pragma unroll
    for (int i = 0; i < 5; i++) d[i] = __builtin_nontemporal_load(x2 + b * 1280 + threadIdx.x + 256 * i);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int j = threadIdx.x + 256 * i, s = j / kChunks, q = j % kChunks;
      t1[s * (kChunks + 1) + q] = a[i];
      t2[s * (kChunks + 1) + q] = d[i];
    }
    __syncthreads();
    f32x4 o[5];
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int s = 16 * t + lo16, q = 5 * c + g;
      o[t] = t1[s * (kChunks + 1) + q] + t2[s * (kChunks + 1) + q];
    }
    o[4] = t1[lane * (kChunks + 1) + 5 * c + 4] + t2[lane * (kChunks + 1) + 5 * c + 4];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; t++)
      __builtin_nontemporal_store(o[t], x3 + b * 1280 + (16 * t + lo16) * kChunks + 5 * c + g);
    __builtin_nontemporal_store(o[4], x3 + b * 1280 + lane * kChunks + 5 * c + 4);
  }
}
#endif

// wave form: 16 sites x 20 chunks = 320 chunks per child, 5 per lane; a private
// LDS region per wave, the next sub-tile's loads issued before this one's LDS work
template <int kWaves>
__global__ void __launch_bounds__(64 * kWaves) mv_wave(const f32x4 *__restrict__ x1, const f32x4 *__restrict__ x2,
                                                       f32x4 *__restrict__ x3, int64_t subs) {
  __shared__ f32x4 reg[kWaves][2][16 * (kChunks + 1)];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  f32x4 *r1 = reg[w][0], *r2 = reg[w][1];
  const int64_t stride = (int64_t)gridDim.x * kWaves;
  int64_t s0 = (int64_t)blockIdx.x * kWaves + w;
  f32x4 a[kChunks / 4], c[kChunks / 4];
  if (s0 < subs) {
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) a[i] = __builtin_nontemporal_load(x1 + s0 * (16 * kChunks) + lane + 64 * i);
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) c[i] = __builtin_nontemporal_load(x2 + s0 * (16 * kChunks) + lane + 64 * i);
  }
  for (int64_t s = s0; s < subs; s += stride) {
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) {
      const int j = lane + 64 * i, st = j / kChunks, q = j % kChunks;
      r1[st * (kChunks + 1) + q] = a[i];
      r2[st * (kChunks + 1) + q] = c[i];
    }
    if (s + stride < subs) {
#pragma unroll
      for (int i = 0; i < kChunks / 4; i++) a[i] = __builtin_nontemporal_load(x1 + (s + stride) * (16 * kChunks) + lane + 64 * i);
#pragma unroll
      for (int i = 0; i < kChunks / 4; i++) c[i] = __builtin_nontemporal_load(x2 + (s + stride) * (16 * kChunks) + lane + 64 * i);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) {
      const int j = lane + 64 * i, st = j % 16, q = j / 16;
      r1[st * (kChunks + 1) + q] = r1[st * (kChunks + 1) + q] + r2[st * (kChunks + 1) + q];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    f32x4 o[kChunks / 4];
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) {
      const int j = lane + 64 * i, st = j / kChunks, q = j % kChunks;
      o[i] = r1[st * (kChunks + 1) + q];
    }
#pragma unroll
    for (int i = 0; i < kChunks / 4; i++) __builtin_nontemporal_store(o[i], x3 + s * (16 * kChunks) + lane + 64 * i);
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void __launch_bounds__(256) mv_stream(const f32x4 *__restrict__ x1, const f32x4 *__restrict__ x2,
                                                 f32x4 *__restrict__ x3, int64_t chunks) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < chunks; i += (int64_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(x1 + i) + __builtin_nontemporal_load(x2 + i), x3 + i);
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 18);  // sites (multiple of 64)
  const int reps = argc > 2 ? atoi(argv[2]) : 40, R = 4, rounds = 5;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int CUs = prop.multiProcessorCount;
  const int64_t chunks = n * kChunks;
  struct Set { f32x4 *x1, *x2, *x3; };
  std::vector<Set> sets(R);
  for (auto &s : sets) {
    CK(hipMalloc(&s.x1, chunks * 16)); CK(hipMalloc(&s.x2, chunks * 16)); CK(hipMalloc(&s.x3, chunks * 16));
    fill<<<2048, 256>>>((float *)s.x1, chunks * 4, 1); fill<<<2048, 256>>>((float *)s.x2, chunks * 4, 2);
  }
  CK(hipDeviceSynchronize());
  struct V { const char *name; int grid, block; void (*run)(const Set &, int); std::vector<float> us; };
  auto occ = [&](const void *k, int bs) { int b = 0; CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, bs, 0)); return b; };
  std::vector<V> vs;
  vs.push_back({"block (64-site tile, barriers)", occ((const void *)mv_block, 256) * CUs, 256,
                [](const Set &s, int g) { mv_block<<<g, 256>>>(s.x1, s.x2, s.x3, 0); }, {}});
  vs.push_back({"wave x4 (16-site sub-tiles, no barrier)", occ((const void *)mv_wave<4>, 256) * CUs, 256,
                [](const Set &s, int g) { mv_wave<4><<<g, 256>>>(s.x1, s.x2, s.x3, 0); }, {}});
  vs.push_back({"wave x4, 2 blocks/CU", 2 * CUs, 256,
                [](const Set &s, int g) { mv_wave<4><<<g, 256>>>(s.x1, s.x2, s.x3, 0); }, {}});
  vs.push_back({"wave x4, 3 blocks/CU", 3 * CUs, 256,
                [](const Set &s, int g) { mv_wave<4><<<g, 256>>>(s.x1, s.x2, s.x3, 0); }, {}});
#if PROBE_CHUNKS == 20
    vs.push_back({"block, x3 scattered from registers (MFMA layout)", occ((const void *)mv_block_scatter, 256) * CUs, 256,
                  [](const Set &s, int g) { mv_block_scatter<<<g, 256>>>(s.x1, s.x2, s.x3, 0); }, {}});
#endif
  vs.push_back({"stream (registers)", 2 * CUs, 256,
                [](const Set &s, int g) { mv_stream<<<g, 256>>>(s.x1, s.x2, s.x3, 0); }, {}});
  // the lambdas cannot capture n: pass it through a global
  static int64_t gN;
  gN = n;
  vs[0].run = [](const Set &s, int g) { mv_block<<<g, 256>>>(s.x1, s.x2, s.x3, gN / 64); };
  for (int i = 1; i <= 3; i++) vs[i].run = [](const Set &s, int g) { mv_wave<4><<<g, 256>>>(s.x1, s.x2, s.x3, gN / 16); };
#if PROBE_CHUNKS == 20
  vs[4].run = [](const Set &s, int g) { mv_block_scatter<<<g, 256>>>(s.x1, s.x2, s.x3, gN / 64); };
#endif
  vs.back().run = [](const Set &s, int g) { mv_stream<<<g, 256>>>(s.x1, s.x2, s.x3, gN * kChunks); };
  std::vector<float> h1(chunks * 4), h2(chunks * 4), h3(chunks * 4);
  CK(hipMemcpy(h1.data(), sets[0].x1, chunks * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), sets[0].x2, chunks * 16, hipMemcpyDeviceToHost));
  for (auto &v : vs) {
    CK(hipMemset(sets[0].x3, 0, chunks * 16));
    v.run(sets[0], v.grid);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h3.data(), sets[0].x3, chunks * 16, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < chunks * 4; i++) bad += h3[i] != h1[i] + h2[i];
    printf("%-45s grid=%d check %s (%lld mismatches)\n", v.name, v.grid, bad ? "DIFFERS" : "ok", (long long)bad);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 200; i++) vs[0].run(sets[i % R], vs[0].grid);
  for (int r = 0; r < rounds; r++)
    for (auto &v : vs) {
      for (int i = 0; i < 3; i++) v.run(sets[i % R], v.grid);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; i++) v.run(sets[i % R], v.grid);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / reps);
    }
  printf("n=%lld sites, %d B/site moved, %d reps x %d rounds, %d buffer sets\n", (long long)n, 48 * kChunks, reps, rounds, R);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const double t = v.us[v.us.size() / 2] * 1e-6;
    printf("%-45s median %8.2f us  %5.1f%% of 8 TB/s\n", v.name, v.us[v.us.size() / 2], 100.0 * 48.0 * kChunks * n / t / 8e12);
  }
  return 0;
}
