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
//                    [--states 4|20] [--fma] [--devices D0,D1,...]
//                    [--reduce rccl|host]
//
// --states 20: a 20-state reversible model (fixed exchangeabilities and
// frequencies), amino-acid tips (codes 0..19, 5 % X), the protein kernels
// (exact, or --fma on the matrix cores), tree levels as batched launches.
//
// --devices D0,D1,...: the alignment's sites split over the listed GPUs by
// the reference's ceil rule (plfx_shard, include.h:181-189), one context per
// entry; every GPU sweeps the whole tree over its own site block (its P
// matrices, traversal and root lnL).  The per-GPU lnL and the per-node scaler
// totals are then summed by ONE RCCL all-reduce over the listed GPUs
// (--reduce rccl, the default when the list names at least two distinct GPUs:
// ncclCommInitAll over the list, a grouped
// ncclAllReduce of f64 lnL + int64[inner nodes] on the GPUs' streams,
// plfx_rccl.hpp) -- the north star's single all-reduce over xGMI -- or, with
// --reduce host -- the default for one GPU or a list that repeats a GPU --
// copied back and added on the host in list order (a device may then be
// listed twice: two contexts on one GPU; RCCL refuses that).  The
// reduction that ran is printed ("reduce = ...").  Same value as one GPU up
// to the summation order.
//
// Prints the per-sweep device time, the node-site rate and the lnL (%.17g);
// with the same seed, dense tips and coded tips give the identical lnL (the tip
// path is bit-exact), as do PLFX_FUSE=0 and the default fused schedule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../include/plfx.h"
#include "plfx_rccl.hpp"

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
  std::vector<int> devices{0};
  int reduce = -1;  // --reduce rccl (1) | host (0); default (-1): rccl over >= 2 distinct GPUs, else host
  bool rccl = false;  // resolved from `reduce` and the device list
};

// One GPU's share: its context, its site block [off, off + n) and the device
// state of the whole tree over that block.
template <typename T>
struct Part {
  int device = 0;
  plfx_ctx *ctx = nullptr;
  int64_t off = 0, n = 0;
  std::vector<void *> clv;
  std::vector<const uint8_t *> tip;
  double *d_eig = nullptr, *d_rates = nullptr, *d_blen = nullptr, *d_w = nullptr, *d_lnl = nullptr;
  T *d_EV = nullptr, *d_pm = nullptr;
  int64_t *d_sums = nullptr;
  hipStream_t st = nullptr;
  std::vector<hipEvent_t> ev;
};

template <typename T>
int run(const Opts &o) {
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

  // device state: one Part per listed GPU, its site block by the reference's
  // ceil rule
  const uint32_t nd = (uint32_t)o.devices.size();
  std::vector<Part<T>> parts(nd);
  for (uint32_t q = 0; q < nd; q++) {
    Part<T> &p = parts[q];
    p.device = o.devices[q];
    uint64_t off = 0, cnt = 0;
    if (plfx_shard((uint64_t)n, nd, q, &off, &cnt) != PLFX_OK) die("too many devices for this many sites");
    p.off = (int64_t)off;
    p.n = (int64_t)cnt;
    // DNA sweeps never use the protein tip/tip tables: no ~95 MB table pool
    if (plfx_ctx_create_ex(p.device, S == 4 ? PLFX_CTX_LAZY_TABLES : 0u, &p.ctx) != PLFX_OK)
      die("no gfx950 device " + std::to_string(p.device));
    HIPCHK(hipSetDevice(p.device));
    p.clv.assign(nslots, nullptr);
    p.tip.assign(nslots, nullptr);
    for (int t = 0; t < T_; t++) {
      if (o.tips) {
        p.tip[t] = upload(std::vector<uint8_t>(codes[t].begin() + p.off, codes[t].begin() + p.off + p.n));
      } else {  // dense tip CLV: x[i][c][s] = bit s of the code (DNA) / state s of the code
        std::vector<T> x((size_t)V * p.n);
        for (int64_t i = 0; i < p.n; i++)
          for (int c = 0; c < 4; c++)
            for (int s = 0; s < S; s++) {
              const int code = codes[t][p.off + i];
              const bool on = S == 4 ? ((code >> s) & 1) : (code >= 20 || code == s);
              x[(size_t)V * i + S * c + s] = (T)(on ? 1 : 0);
            }
        p.clv[t] = upload(x);
      }
    }
    for (int s = T_; s < nslots; s++) p.clv[s] = dalloc<T>((size_t)V * p.n);
    p.d_eig = upload(eig);
    p.d_rates = upload(rates);
    p.d_blen = upload(blen);
    std::vector<T> EVt(EVd.begin(), EVd.end());
    p.d_EV = upload(EVt);
    p.d_pm = dalloc<T>((size_t)2 * nops * M);
    p.d_w = upload(w);
    p.d_lnl = dalloc<double>(1);
    p.d_sums = dalloc<int64_t>(nops);
    p.st = reinterpret_cast<hipStream_t>(plfx_ctx_stream(p.ctx));
    p.ev.resize(o.sweeps + 1);
    for (auto &e : p.ev) HIPCHK(hipEventCreate(&e));
  }

  // the communicator of the one all-reduce (made before the sweeps: RCCL's
  // setup is not part of the timed work)
  std::unique_ptr<plfx_host::NodeComm> comm;
  if (o.rccl) {
    std::string err;
    comm.reset(new plfx_host::NodeComm(o.devices, err));
    if (!err.empty()) die(err);
  }
  const std::string reduce_desc =
      o.rccl ? "rccl (" + std::to_string(nd) + " rank" + (nd > 1 ? "s" : "") + ", RCCL " +
                   plfx_host::NodeComm::version() + ")"
             : "host (" + std::to_string(nd) + " part" + (nd > 1 ? "s" : "") + ", list order)";
  auto sweep = [&](Part<T> &p) {  // enqueued on the part's stream, returns at once
    plfx_ctx *ctx = p.ctx;
    PLFXCHK(ctx, plfx_pmatrix(ctx, dt, S, PLFX_PMAT_STATE, p.d_eig, p.d_rates, 4, p.d_blen, 2 * nops, p.d_pm,
                              p.st));
    PLFXCHK(ctx, plfx_traverse_tips(ctx, dt, S, o.fma ? PLFX_FMA : PLFX_EXACT, ops.data(), nops, p.clv.data(),
                                    o.tips ? p.tip.data() : nullptr, nslots, p.d_pm, nops, p.d_EV, p.n,
                                    nullptr, nullptr, p.d_sums, nullptr, p.st));
    PLFXCHK(ctx, plfx_root_lnl(ctx, dt, S, p.clv[nslots - 1], p.n, nullptr, p.d_w, nullptr, p.d_sums, nops,
                               p.d_lnl, nullptr, p.st));
  };
  for (auto &p : parts) sweep(p);  // warm-up
  for (auto &p : parts) HIPCHK(hipStreamSynchronize(p.st));
  for (auto &p : parts) HIPCHK(hipEventRecord(p.ev[0], p.st));
  for (int i = 0; i < o.sweeps; i++)
    for (auto &p : parts) {  // every GPU's sweep i before any GPU's sweep i + 1
      sweep(p);
      HIPCHK(hipEventRecord(p.ev[i + 1], p.st));
    }
  for (auto &p : parts) HIPCHK(hipStreamSynchronize(p.st));
  // the one reduction of the per-GPU partials: lnL (f64) and the scaler totals
  // of every inner node (int64)
  double lnl = 0.0, reduce_us = 0.0;
  long long scale_events = 0;
  std::vector<int64_t> sums(nops);
  if (o.rccl) {
    std::vector<double *> f;
    std::vector<int64_t *> iv;
    std::vector<hipStream_t> st;
    for (auto &p : parts) {
      f.push_back(p.d_lnl);
      iv.push_back(p.d_sums);
      st.push_back(p.st);
    }
    const auto t0 = std::chrono::steady_clock::now();
    const std::string err = comm->allreduce_sum(f, 1, iv, (size_t)nops, st);
    if (!err.empty()) die(err);
    for (auto &p : parts) HIPCHK(hipStreamSynchronize(p.st));
    reduce_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    // every rank holds the job's totals now: rank 0's
    HIPCHK(hipSetDevice(parts[0].device));
    HIPCHK(hipMemcpy(&lnl, parts[0].d_lnl, sizeof lnl, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(sums.data(), parts[0].d_sums, nops * sizeof(int64_t), hipMemcpyDeviceToHost));
    for (int64_t s : sums) scale_events += s;
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (auto &p : parts) {  // list order: a fixed summation order
      double v = 0.0;
      HIPCHK(hipSetDevice(p.device));
      HIPCHK(hipMemcpy(&v, p.d_lnl, sizeof v, hipMemcpyDeviceToHost));
      lnl += v;
      HIPCHK(hipMemcpy(sums.data(), p.d_sums, nops * sizeof(int64_t), hipMemcpyDeviceToHost));
      for (int64_t s : sums) scale_events += s;
    }
    reduce_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  // a sweep's time: the slowest GPU's
  float tot_ms = 0.f, mn = 1e30f, mx = 0.f;
  for (int i = 0; i < o.sweeps; i++) {
    float ms = 0.f;
    for (auto &p : parts) {
      float m;
      HIPCHK(hipEventElapsedTime(&m, p.ev[i], p.ev[i + 1]));
      ms = std::max(ms, m);
    }
    tot_ms += ms;
    mn = std::min(mn, ms);
    mx = std::max(mx, ms);
  }
  const double avg = tot_ms / o.sweeps;
  if (!o.quiet) {
    std::string dl;
    for (uint32_t q = 0; q < nd; q++) dl += (q ? "," : "") + std::to_string(o.devices[q]);
    std::printf("==================================================================================\n");
    std::printf("| taxa / inner nodes:     | %24d / %26d |\n", T_, nops);
    std::printf("| alignment sites:        | %54lld |\n", (long long)n);
    std::printf("| GPUs (site blocks):     | %54s |\n", dl.c_str());
    std::printf("| element type / tips:    | %24s / %26s |\n", o.f64 ? "f64" : "f32",
                o.tips ? "state codes" : "dense CLVs");
    std::printf("| states / mode:          | %24d / %26s |\n", S, o.fma ? "FMA" : "exact");
    std::printf("| sweeps (P + traversal + lnL) | %49d |\n", o.sweeps);
    std::printf("==================================================================================\n");
    std::printf("| sweep time (ms) avg / min / max | %14.4f / %10.4f / %10.4f |\n", avg, mn, mx);
    std::printf("| inner-node sites per second     | %46.4e |\n", (double)nops * n / (avg * 1e-3));
    std::printf("| scaling events (last sweep)     | %46lld |\n", scale_events);
    std::printf("| lnL reduction / time (us)       | %32s / %11.1f |\n", reduce_desc.c_str(), reduce_us);
    std::printf("==================================================================================\n");
  }
  std::printf("reduce = %s\n", reduce_desc.c_str());
  std::printf("lnL = %.17g\n", lnl);
  comm.reset();  // before the streams it reduced on go away
  for (auto &p : parts) {
    HIPCHK(hipSetDevice(p.device));
    for (auto &e : p.ev) (void)hipEventDestroy(e);
    for (int s = 0; s < nslots; s++) (void)hipFree(s < T_ && o.tips ? (void *)p.tip[s] : p.clv[s]);
    (void)hipFree(p.d_eig); (void)hipFree(p.d_rates); (void)hipFree(p.d_blen); (void)hipFree(p.d_EV);
    (void)hipFree(p.d_pm); (void)hipFree(p.d_w); (void)hipFree(p.d_lnl); (void)hipFree(p.d_sums);
    plfx_ctx_destroy(p.ctx);
  }
  return std::isfinite(lnl) ? 0 : 3;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 4)
    die("usage: plfx_tree <taxa (power of 2)> <sites> <sweeps> [--dtype f32|f64] [--tips] "
        "[--alpha A] [--seed S] [--quiet] [--states 4|20] [--fma] [--devices D0,D1,...] "
        "[--reduce rccl|host]");
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
    } else if (a == "--reduce") {
      const std::string v = next();
      if (v == "rccl") o.reduce = 1;
      else if (v == "host") o.reduce = 0;
      else die("bad reduction " + v + " (rccl|host)");
    } else if (a == "--devices") {
      o.devices.clear();
      const std::string v = next();
      size_t p = 0;
      while (p <= v.size()) {
        const size_t q = std::min(v.find(',', p), v.size());
        try {
          o.devices.push_back(std::stoi(v.substr(p, q - p)));
        } catch (const std::exception &) {
          die("bad device list " + v);
        }
        if (o.devices.back() < 0) die("bad device list " + v);
        p = q + 1;
      }
    } else {
      die("unknown option " + a);
    }
  }
  if (o.taxa < 2 || (o.taxa & (o.taxa - 1))) die("taxa must be a power of 2 >= 2");
  if (o.sites < 1 || o.sweeps < 1) die("sites and sweeps must be >= 1");
  {
    std::vector<int> d = o.devices;
    std::sort(d.begin(), d.end());
    const bool distinct = std::adjacent_find(d.begin(), d.end()) == d.end();
    o.rccl = o.reduce == 1 || (o.reduce < 0 && distinct && d.size() >= 2);
  }
  return o.f64 ? run<double>(o) : run<float>(o);
}
