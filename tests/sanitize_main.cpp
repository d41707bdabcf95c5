// sanitize_main.cpp -- test infrastructure, not product code.  The host-side
// C++ of libplfx (instance sizing and packing, the partition, the host_mem
// input protocol, the sw_emu target, the model setup: csrc/testbench_api.cpp,
// csrc/swemu.cpp, csrc/model.cpp) built with AddressSanitizer and
// UndefinedBehaviorSanitizer ("build runs
// -fsanitize=address,undefined on the CPU ref/host lib"), driven over ragged
// and edge configurations, with the sw_emu results checked bit for bit against
// the oracle's plf() restatement (oracle/plf_oracle.c, linked in as the
// checker).  tests/test_sanitizers.py builds and runs it; it prints "OK <n>"
// and exits 0, or names the first failure and exits 1 (a sanitizer report
// aborts it: -fno-sanitize-recover).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../include/plfx.h"

extern "C" {
void plfo_plf_f32(const float *x1s, const float *x2s, float *x3s, const float *EV, long long n,
                  const float *left, const float *right, const int *wgt, int *scalerIncrement,
                  unsigned char *scaler);
void plfo_plf_f64(const double *x1s, const double *x2s, double *x3s, const double *EV, long long n,
                  const double *left, const double *right, const int *wgt, int *scalerIncrement,
                  unsigned char *scaler);
}

static int failures = 0, checks = 0;
#define EXPECT(cond, ...)                    \
  do {                                       \
    ++checks;                                \
    if (!(cond)) {                           \
      ++failures;                            \
      std::printf("FAIL: " __VA_ARGS__);     \
      std::printf("\n");                     \
    }                                        \
  } while (0)

template <typename T>
static void oracle_plf(const T *x1, const T *x2, T *x3, const T *EV, long long n, const T *l,
                       const T *r, const int *w, int *inc, unsigned char *sc) {
  if constexpr (sizeof(T) == 4) plfo_plf_f32(x1, x2, x3, EV, n, l, r, w, inc, sc);
  else plfo_plf_f64(x1, x2, x3, EV, n, l, r, w, inc, sc);
}

// One testbench configuration: pack every instance, run it on the sw_emu
// target into exactly-sized outputs plus a guard element, compare with plf().
template <typename T>
static void swemu_case(uint64_t sites, uint32_t inst, uint32_t window, int layout, int aie, uint32_t seed) {
  const int dtype = sizeof(T) == 4 ? PLFX_F32 : PLFX_F64;
  std::vector<T> EV(16), L(64), R(64), x1(16 * sites), x2(16 * sites), x3(16 * sites);
  std::vector<int32_t> w(sites);
  EXPECT(plfx_gen_hostmem(dtype, seed, sites, EV.data(), L.data(), R.data(), x1.data(), x2.data(), w.data()) == 0,
         "gen_hostmem sites=%llu", (unsigned long long)sites);
  for (uint64_t i = 0; i < sites; i++) w[i] = 1 + (int)(i % 5);
  std::vector<unsigned char> esc(sites);
  int inc = 0;
  oracle_plf<T>(x1.data(), x2.data(), x3.data(), EV.data(), (long long)sites, L.data(), R.data(), w.data(), &inc,
                esc.data());
  const plfx_testbench tb{sites, inst, window, layout, aie};
  uint64_t covered = 0;
  for (uint32_t k = 0; k < inst; k++) {
    const uint64_t off = plfx_tb_instance_site_offset(&tb, (int)k);
    const uint64_t nk = plfx_tb_alignments_per_instance(&tb, (int)k);
    uint64_t soff = 0, scnt = 0;
    EXPECT(plfx_shard(sites, inst, k, &soff, &scnt) == 0 && soff == off && scnt == nk,
           "shard vs testbench: sites=%llu inst=%u k=%u", (unsigned long long)sites, inst, k);
    std::vector<T> bl(plfx_tb_instance_elements_left(&tb)), br(plfx_tb_instance_elements_right(&tb));
    const int prc = plfx_pack_instance(&tb, (int)k, dtype, EV.data(), L.data(), R.data(), x1.data(), x2.data(),
                                       bl.data(), br.data());
    EXPECT(prc == 0, "pack rc=%d", prc);
    if (prc != 0) return;
    std::vector<T> out(16 * nk + 16, T(-7));  // one guard site
    std::vector<uint8_t> sc(nk + 1, 0xAB);
    const int rc = plfx_swemu_instance_run(bl.data(), br.data(), out.data(), sc.data(), (uint32_t)nk, window,
                                           layout, aie, dtype);
    EXPECT(rc == 0, "swemu rc=%d sites=%llu inst=%u window=%u layout=%d aie=%d", rc, (unsigned long long)sites,
           inst, window, layout, aie);
    if (rc != 0) return;
    EXPECT(std::memcmp(out.data(), x3.data() + 16 * off, 16 * nk * sizeof(T)) == 0,
           "sw_emu CLV != plf(): sites=%llu inst=%u k=%u window=%u layout=%d aie=%d", (unsigned long long)sites,
           inst, k, window, layout, aie);
    EXPECT(std::memcmp(sc.data(), esc.data() + off, nk) == 0, "sw_emu scaler != plf()");
    bool guard = true;
    for (int j = 0; j < 16; j++) guard = guard && out[16 * nk + j] == T(-7);
    EXPECT(guard && sc[nk] == 0xAB, "sw_emu wrote past alignment_sites (k=%u)", k);
    covered += nk;
  }
  EXPECT(covered == sites, "instances cover %llu of %llu sites", (unsigned long long)covered,
         (unsigned long long)sites);
}

static void model_case(int S, uint32_t seed) {
  std::vector<double> exch(S * (S - 1) / 2), freqs(S), eigen(S + 2 * S * S), EV(S * S), wts(S), tv(16 * S);
  uint32_t z = seed;
  auto u = [&]() { z = z * 1664525u + 1013904223u; return 0.05 + (z >> 8) / 16777216.0; };
  for (double &e : exch) e = u();
  for (double &f : freqs) f = u();
  EXPECT(plfx_model_eigen(S, exch.data(), freqs.data(), eigen.data()) == 0, "model_eigen S=%d", S);
  // Q = V diag(lambda) Vinv: rows sum to 0, lambda_0 = 0, V Vinv = I
  const double *lam = eigen.data(), *V = lam + S, *Vi = V + S * S;
  double worst_row = 0, worst_id = 0;
  for (int i = 0; i < S; i++) {
    double row = 0;
    for (int j = 0; j < S; j++) {
      double q = 0, id = 0;
      for (int k = 0; k < S; k++) {
        q += V[i * S + k] * lam[k] * Vi[k * S + j];
        id += V[i * S + k] * Vi[k * S + j];
      }
      row += q;
      worst_id = std::fmax(worst_id, std::fabs(id - (i == j ? 1.0 : 0.0)));
    }
    worst_row = std::fmax(worst_row, std::fabs(row));
  }
  EXPECT(std::fabs(lam[0]) < 1e-12 && worst_row < 1e-10 && worst_id < 1e-10,
         "eigensystem S=%d: lambda0 %g, row sums %g, V.Vinv-I %g", S, lam[0], worst_row, worst_id);
  std::vector<double> rates(4), rates_med(4);
  EXPECT(plfx_gamma_rates(0.5, 4, 0, rates.data()) == 0 && plfx_gamma_rates(0.5, 4, 1, rates_med.data()) == 0,
         "gamma_rates");
  double mean = 0;
  for (double r : rates) mean += r / 4;
  EXPECT(std::fabs(mean - 1.0) < 1e-12, "gamma rates mean %g", mean);
  for (int conv = PLFX_PMAT_STATE; conv <= PLFX_PMAT_EIGEN; conv++) {
    EXPECT(plfx_model_ev(S, conv, eigen.data(), EV.data()) == 0, "model_ev");
    EXPECT(plfx_model_root_weights(S, conv, eigen.data(), freqs.data(), wts.data()) == 0, "root_weights");
    if (S == 4) EXPECT(plfx_model_tip_vectors(S, conv, eigen.data(), tv.data()) == 0, "tip_vectors");
  }
}

int main() {
  // the partition: the reference's ceil split, and its underflow rejected
  uint64_t o = 0, c = 0;
  EXPECT(plfx_shard(10, 8, 0, &o, &c) != 0, "shard 10 over 8 must be rejected");
  EXPECT(plfx_shard(1000448, 9, 8, &o, &c) == 0 && o + c == 1000448, "shard last part");
  EXPECT(plfx_shard(512, 8, 7, &o, &c) == 0 && o == 448 && c == 64, "shard 512 nodes over 8");
  // sw_emu over windows, layouts, PLIO kinds, ragged instance splits, f32 and f64
  const uint64_t sites[] = {1, 7, 64, 1000, 1024, 4099};
  const uint32_t insts[] = {1, 3, 4, 9};
  const uint32_t windows[] = {32, 96, 1024, 8192, 16288};
  uint32_t seed = 20250117;
  for (uint64_t n : sites)
    for (uint32_t p : insts) {
      if (n < 2 * p) continue;  // the reference's split underflows; plfx_shard rejects it
      uint64_t o2 = 0, c2 = 0;
      bool ok = true;
      for (uint32_t k = 0; k < p; k++) ok = ok && plfx_shard(n, p, k, &o2, &c2) == 0;
      if (!ok) continue;
      for (uint32_t wnd : windows)
        for (int layout = PLFX_LAYOUT_COMBINED; layout <= PLFX_LAYOUT_SEPARATE; layout++) {
          swemu_case<float>(n, p, wnd, layout, PLFX_AIE_WINDOW, seed++);
          swemu_case<double>(n, p, wnd, layout, PLFX_AIE_WINDOW, seed++);
        }
      swemu_case<float>(n, p, 0, PLFX_LAYOUT_COMBINED, PLFX_AIE_STREAM, seed++);
      swemu_case<double>(n, p, 0, PLFX_LAYOUT_COMBINED, PLFX_AIE_STREAM, seed++);
    }
  model_case(4, 1);
  model_case(20, 2);
  if (failures) {
    std::printf("FAILED %d of %d checks\n", failures, checks);
    return 1;
  }
  std::printf("OK %d checks\n", checks);
  return 0;
}
