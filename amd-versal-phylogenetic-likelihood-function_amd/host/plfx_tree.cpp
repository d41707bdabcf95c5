// plfx_tree.cpp -- C++ tree-likelihood driver over the plfx C ABI (BASELINE
// configs[2]).  The reference evaluates one node
// per call (app/src/host_mem.cpp); this is the loop a likelihood program runs
// around it: a GTR+Gamma4 model (plfx_model_eigen, plfx_gamma_rates), a
// balanced tree of T taxa as a post-order descriptor, and per sweep the device
// P matrices from the branch lengths (plfx_pmatrix), the traversal
// (plfx_traverse_tips: tips dense or as state codes, subtrees fused) and the
// root log-likelihood (plfx_root_lnl), timed with HIP events.
//
//   usage: plfx_tree <taxa (power of 2)> <sites> <sweeps>
//                    [--dtype f32|f64] [--tips] [--alpha A] [--seed S] [--quiet]
//                    [--states 4|20] [--fma]
//
// --states 20: a 20-state reversible model (fixed exchangeabilities and
// frequencies), amino-acid tips (codes 0..19, 5 % X), the protein kernels
// (exact, or --fma on the matrix cores), tree levels as batched launches.
//
// Prints the per-sweep device time, the node-site rate and the lnL (%.17g);
// with the same seed, dense tips and coded tips give the identical lnL (the tip
// path is bit-exact), as do PLFX_FUSE=0 and the default fused schedule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../include/plfx.h"

namespace {

void die(const std::string &m) {
  std::fprintf(stderr, "plfx_tree: %s\n", m.c_str());
  std::exit(2);
}

#define HIPCHK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) die(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define PLFXCHK(ctx, x)                                                        \
  do {                                                                         \
    int rc_ = (x);                                                             \
    if (rc_ != PLFX_OK) die(std::string(#x) + ": " + plfx_last_error(ctx));    \
  } while (0)

template <typename T>
T *dalloc(size_t count) {
  T *p = nullptr;
  HIPCHK(hipMalloc(reinterpret_cast<void **>(&p), count * sizeof(T)));
  return p;
}

template <typename T>
T *upload(const std::vector<T> &v) {
  T *p = dalloc<T>(v.size());
  HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

struct Opts {
  int taxa = 0;
  int64_t sites = 0;
  int sweeps = 1;
  bool f64 = true, tips = false, quiet = false, fma = false;
  int states = 4;
  double alpha = 0.5;
  uint32_t seed = 20250117u;
};

template <typename T>
int run(const Opts &o) {
  plfx_ctx *ctx = nullptr;
  if (plfx_ctx_create(0, &ctx) != PLFX_OK) die("no gfx950 device");
  const int dt = o.f64 ? PLFX_F64 : PLFX_F32;
  const int T_ = o.taxa, nops = T_ - 1, nslots = 2 * T_ - 1;
  const int64_t n = o.sites;
  const int S = o.states, V = 4 * S, M = 4 * S * S;  // values per site, per P pair member

  // model: GTR exchangeabilities AC AG AT CG CT GT, frequencies, Gamma(alpha);
  // S = 20: a fixed pattern of the 190 exchangeabilities and 20 frequencies
  std::vector<double> exch = {1.2, 3.9, 0.8, 1.1, 4.6, 1.0};
  std::vector<double> freqs = {0.31, 0.19, 0.22, 0.28};
  if (S == 20) {
    exch.resize(190);
    for (int k = 0; k < 190; k++) exch[k] = 0.5 + (double)((k * 37) % 29) / 10.0;
    freqs.resize(20);
    double tot = 0.0;
    for (int s = 0; s < 20; s++) tot += (freqs[s] = 1.0 + (double)((s * 7) % 11));
    for (double &f : freqs) f /= tot;
  }
  std::vector<double> eig(S + 2 * S * S), rates(4), EVd(S * S), w(S);
  if (plfx_model_eigen(S, exch.data(), freqs.data(), eig.data()) != PLFX_OK) die("model_eigen");
  plfx_gamma_rates(o.alpha, 4, 0, rates.data());
  plfx_model_ev(S, PLFX_PMAT_STATE, eig.data(), EVd.data());
  plfx_model_root_weights(S, PLFX_PMAT_STATE, eig.data(), freqs.data(), w.data());

  // balanced tree: tips 0..T-1, inner slots T.. in post-order, op j = pmat j
  std::vector<plfx_trav_op> ops;
  std::vector<int> level(T_);
  for (int i = 0; i < T_; i++) level[i] = i;
  int next = T_;
  while (level.size() > 1) {
    std::vector<int> up;
    for (size_t i = 0; i < level.size(); i += 2) {
      ops.push_back({next, level[i], level[i + 1], (int32_t)ops.size()});
      up.push_back(next++);
    }
    level = up;
  }

  std::mt19937 gen(o.seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<double> blen(2 * nops);
  for (double &b : blen) b = 0.01 + 0.3 * U(gen);
  // alignment: A/C/G/T codes, 5 % ambiguous (random non-empty subsets);
  // S = 20: amino-acid codes 0..19, 5 % X (code 22: every state)
  std::vector<std::vector<uint8_t>> codes(T_, std::vector<uint8_t>(n));
  const uint8_t acgt[4] = {1, 2, 4, 8};
  for (auto &c : codes)
    for (auto &v : c) {
      if (S == 4) v = U(gen) < 0.05 ? (uint8_t)(1 + (int)(U(gen) * 15)) : acgt[(int)(U(gen) * 4) & 3];
      else {  // two draws per site, as the DNA form
        const double a = U(gen), b = U(gen);
        v = a < 0.05 ? (uint8_t)22 : (uint8_t)((int)(b * 20) % 20);
      }
    }

  // device state
  std::vector<void *> clv(nslots, nullptr);
  std::vector<const uint8_t *> tip(nslots, nullptr);
  for (int t = 0; t < T_; t++) {
    if (o.tips) {
      tip[t] = upload(codes[t]);
    } else {  // dense tip CLV: x[i][c][s] = bit s of the code (DNA) / state s of the code
      std::vector<T> x((size_t)V * n);
      for (int64_t i = 0; i < n; i++)
        for (int c = 0; c < 4; c++)
          for (int s = 0; s < S; s++) {
            const int code = codes[t][i];
            const bool on = S == 4 ? ((code >> s) & 1) : (code >= 20 || code == s);
            x[(size_t)V * i + S * c + s] = (T)(on ? 1 : 0);
          }
      clv[t] = upload(x);
    }
  }
  for (int s = T_; s < nslots; s++) clv[s] = dalloc<T>((size_t)V * n);
  double *d_eig = upload(eig), *d_rates = upload(rates), *d_blen = upload(blen);
  std::vector<T> EVt(EVd.begin(), EVd.end());
  T *d_EV = upload(EVt), *d_pm = dalloc<T>((size_t)2 * nops * M);
  double *d_w = upload(w), *d_lnl = dalloc<double>(1);
  int64_t *d_sums = dalloc<int64_t>(nops);
  hipStream_t st = reinterpret_cast<hipStream_t>(plfx_ctx_stream(ctx));
  std::vector<hipEvent_t> ev(o.sweeps + 1);
  for (auto &e : ev) HIPCHK(hipEventCreate(&e));

  auto sweep = [&]() {
    PLFXCHK(ctx, plfx_pmatrix(ctx, dt, S, PLFX_PMAT_STATE, d_eig, d_rates, 4, d_blen, 2 * nops, d_pm, st));
    PLFXCHK(ctx, plfx_traverse_tips(ctx, dt, S, o.fma ? PLFX_FMA : PLFX_EXACT, ops.data(), nops, clv.data(),
                                    o.tips ? tip.data() : nullptr, nslots, d_pm, nops, d_EV, n,
                                    nullptr, nullptr, d_sums, nullptr, st));
    PLFXCHK(ctx, plfx_root_lnl(ctx, dt, S, clv[nslots - 1], n, nullptr, d_w, nullptr, d_sums, nops,
                               d_lnl, nullptr, st));
  };
  sweep();  // warm-up
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(hipEventRecord(ev[0], st));
  for (int i = 0; i < o.sweeps; i++) {
    sweep();
    HIPCHK(hipEventRecord(ev[i + 1], st));
  }
  HIPCHK(hipStreamSynchronize(st));
  double lnl = 0.0;
  HIPCHK(hipMemcpy(&lnl, d_lnl, sizeof lnl, hipMemcpyDeviceToHost));
  std::vector<int64_t> sums(nops);
  HIPCHK(hipMemcpy(sums.data(), d_sums, nops * sizeof(int64_t), hipMemcpyDeviceToHost));
  long long scale_events = 0;
  for (int64_t v : sums) scale_events += v;
  float tot_ms = 0.f, mn = 1e30f, mx = 0.f;
  for (int i = 0; i < o.sweeps; i++) {
    float ms;
    HIPCHK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
    tot_ms += ms;
    mn = std::min(mn, ms);
    mx = std::max(mx, ms);
  }
  const double avg = tot_ms / o.sweeps;
  if (!o.quiet) {
    std::printf("==================================================================================\n");
    std::printf("| taxa / inner nodes:     | %24d / %26d |\n", T_, nops);
    std::printf("| alignment sites:        | %54lld |\n", (long long)n);
    std::printf("| element type / tips:    | %24s / %26s |\n", o.f64 ? "f64" : "f32",
                o.tips ? "state codes" : "dense CLVs");
    std::printf("| states / mode:          | %24d / %26s |\n", S, o.fma ? "FMA" : "exact");
    std::printf("| sweeps (P + traversal + lnL) | %49d |\n", o.sweeps);
    std::printf("==================================================================================\n");
    std::printf("| sweep time (ms) avg / min / max | %14.4f / %10.4f / %10.4f |\n", avg, mn, mx);
    std::printf("| inner-node sites per second     | %46.4e |\n", (double)nops * n / (avg * 1e-3));
    std::printf("| scaling events (last sweep)     | %46lld |\n", scale_events);
    std::printf("==================================================================================\n");
  }
  std::printf("lnL = %.17g\n", lnl);
  for (auto &e : ev) (void)hipEventDestroy(e);
  for (int s = 0; s < nslots; s++) (void)hipFree(s < T_ && o.tips ? (void *)tip[s] : clv[s]);
  (void)hipFree(d_eig); (void)hipFree(d_rates); (void)hipFree(d_blen); (void)hipFree(d_EV);
  (void)hipFree(d_pm); (void)hipFree(d_w); (void)hipFree(d_lnl); (void)hipFree(d_sums);
  plfx_ctx_destroy(ctx);
  return std::isfinite(lnl) ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 4)
    die("usage: plfx_tree <taxa (power of 2)> <sites> <sweeps> [--dtype f32|f64] [--tips] "
        "[--alpha A] [--seed S] [--quiet] [--states 4|20] [--fma]");
  Opts o;
  try {
    o.taxa = std::stoi(argv[1]);
    o.sites = std::stoll(argv[2]);
    o.sweeps = std::stoi(argv[3]);
  } catch (const std::exception &e) {
    die(std::string("bad numeric argument: ") + e.what());
  }
  for (int i = 4; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) die("missing value for " + a);
      return argv[++i];
    };
    if (a == "--dtype") {
      const std::string v = next();
      if (v == "f32") o.f64 = false;
      else if (v == "f64") o.f64 = true;
      else die("bad dtype " + v);
    } else if (a == "--tips") {
      o.tips = true;
    } else if (a == "--alpha") {
      o.alpha = std::stod(next());
    } else if (a == "--seed") {
      o.seed = (uint32_t)std::stoul(next());
    } else if (a == "--quiet") {
      o.quiet = true;
    } else if (a == "--states") {
      o.states = std::stoi(next());
      if (o.states != 4 && o.states != 20) die("states must be 4 or 20");
    } else if (a == "--fma") {
      o.fma = true;
    } else {
      die("unknown option " + a);
    }
  }
  if (o.taxa < 2 || (o.taxa & (o.taxa - 1))) die("taxa must be a power of 2 >= 2");
  if (o.sites < 1 || o.sweeps < 1) die("sites and sweeps must be >= 1");
  return o.f64 ? run<double>(o) : run<float>(o);
}
