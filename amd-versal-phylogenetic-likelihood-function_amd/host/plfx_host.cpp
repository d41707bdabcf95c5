// plfx_host.cpp -- C++ host program over the plfx C ABI; the counterpart of the
// reference's app/src/host_mem.cpp (XRT) with the accelerator replaced by HIP.
//
//   usage: plfx_host <alignment sites> <plf calls> <parallel instances>
//                    [--dtype f32|f64] [--layout comb|sep] [--aie window|stream]
//                    [--window BYTES] [--seed S] [--dump PREFIX] [--quiet]
//
// Mirrors host_mem.cpp:
//   * argv shape <sites> <calls> <instances> (host_mem.cpp:13-38); the xclbin
//     and BDF arguments are gone, layout/AIE type/window are explicit flags
//     instead of being parsed out of the xclbin file name;
//   * size table (host_mem.cpp:45-101) from testbench sizing (include.h:150-266);
//   * host_mem input protocol (host_mem.cpp:179-209) with a fixed seed (Q8);
//   * per-instance packing [EV|P_L|CLV_L], [EV|P_R|CLV_R] / [P_R|CLV_R]
//     (host_mem.cpp:221-243);
//   * per call, per instance on its own HIP stream: H2D left || H2D right ->
//     fused kernel -> D2H CLV || D2H scaler, with the begin/t1/t2/end regions
//     of timing.h:25-52 taken by HIP events (host_mem.cpp:283-325);
//   * host scaler reduction sum scaler[j]*wgt[j] (host_mem.cpp:384-388);
//   * timing table in the layout of timing.h:107-151 (no CPU "Reference" row:
//     the CPU check lives in the tests, which read --dump output).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/plfx.h"
#include "../csrc/testbench.hpp"

namespace {

void die(const std::string &m) {
  std::fprintf(stderr, "plfx_host: %s\n", m.c_str());
  std::exit(2);
}

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) die(std::string(#x) + ": " + hipGetErrorString(e_));      \
  } while (0)

struct Opts {
  uint64_t sites = 0;
  uint32_t calls = 1, instances = 1;
  bool f64 = true;
  int layout = plfx::SEPARATE;
  int aie = plfx::WINDOW;
  uint32_t window = 8192;
  uint32_t seed = 20250117u;
  std::string dump;
  bool quiet = false;
};

Opts parse(int argc, char **argv) {
  if (argc < 4)
    die("usage: plfx_host <alignment sites> <plf calls> <parallel instances> [--dtype f32|f64] "
        "[--layout comb|sep] [--aie window|stream] [--window BYTES] [--seed S] [--dump PREFIX]");
  Opts o;
  try {
    o.sites = std::stoull(argv[1]);
    o.calls = (uint32_t)std::stoul(argv[2]);
    o.instances = (uint32_t)std::stoul(argv[3]);
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
      std::string v = next();
      if (v == "f32") o.f64 = false;
      else if (v == "f64") o.f64 = true;
      else die("bad dtype " + v);
    } else if (a == "--layout") {
      std::string v = next();
      if (v == "comb") o.layout = plfx::COMBINED;
      else if (v == "sep") o.layout = plfx::SEPARATE;
      else die("bad layout " + v);
    } else if (a == "--aie") {
      std::string v = next();
      if (v == "window") o.aie = plfx::WINDOW;
      else if (v == "stream") o.aie = plfx::STREAM;
      else die("bad aie type " + v);
    } else if (a == "--window") {
      o.window = (uint32_t)std::stoul(next());
    } else if (a == "--seed") {
      o.seed = (uint32_t)std::stoul(next());
    } else if (a == "--dump") {
      o.dump = next();
    } else if (a == "--quiet") {
      o.quiet = true;
    } else {
      die("unknown option " + a);
    }
  }
  if (o.instances == 0 || o.calls == 0) die("calls and instances must be > 0");
  if (o.aie == plfx::WINDOW && (o.window < 16 || o.window % 16)) die("window must be a multiple of 16 bytes");
  return o;
}

struct Region {  // timing.h:25-52, device-event based
  std::vector<double> hm, msm, mh, total;
};

template <typename T>
int run(const Opts &o) {
  plfx::Testbench tb;
  tb.alignment_sites = o.sites;
  tb.parallel_instances = o.instances;
  tb.window_size = o.window;
  tb.layout = o.layout;
  tb.aie_type = o.aie;
  const uint64_t n0 = tb.alignments_per_instance();
  // The reference's partition silently underflows when the padding exceeds one
  // instance's share (e.g. 10 sites over 8 instances); reject it instead.
  if (tb.alignments_padding() >= n0 && o.instances > 1) die("too many instances for this many sites");
  const size_t es = sizeof(T);

  if (!o.quiet) {
    std::printf("==================================================================================\n");
    std::printf("| alignment sites:        | %54llu |\n", (unsigned long long)o.sites);
    std::printf("| plf calls:              | %54u |\n", o.calls);
    std::printf("| parallel plfs:          | %54u |\n", o.instances);
    std::printf("| element type:           | %54s |\n", o.f64 ? "f64" : "f32");
    std::printf("| layout / aie / window:  | %34s %8s %10u |\n", o.layout == plfx::COMBINED ? "COMBINED" : "SEPARATE",
                o.aie == plfx::WINDOW ? "window" : "stream", o.window);
    std::printf("==================================================================================\n");
    std::printf("|                         |       alignments |         elements |     size (bytes) |\n");
    std::printf("| instance left:          | %16llu | %16llu | %16llu |\n", (unsigned long long)n0,
                (unsigned long long)tb.instance_elements_left(), (unsigned long long)(tb.instance_elements_left() * es));
    std::printf("| instance right:         | %16llu | %16llu | %16llu |\n", (unsigned long long)n0,
                (unsigned long long)tb.instance_elements_right(), (unsigned long long)(tb.instance_elements_right() * es));
    std::printf("| instance out:           | %16llu | %16llu | %16llu |\n", (unsigned long long)n0,
                (unsigned long long)tb.instance_elements_out(), (unsigned long long)(tb.instance_elements_out() * es));
    std::printf("==================================================================================\n");
  }

  plfx_ctx *ctx = nullptr;
  int rc = plfx_ctx_create(0, &ctx);
  if (rc != PLFX_OK) die("plfx_ctx_create failed: " + std::to_string(rc));

  // host_mem.cpp:179-209 input protocol, fixed seed
  std::mt19937 gen(o.seed);
  std::uniform_real_distribution<> dis(0.0f, 1.0f);
  T ev[16], bl[64], br[64];
  const uint64_t elems = o.sites * 16;
  std::vector<T> xl(elems), xr(elems);
  for (int j = 0; j < 16; j++) ev[j] = (T)dis(gen);
  for (int j = 0; j < 64; j++) {
    bl[j] = (T)dis(gen);
    br[j] = (T)dis(gen);
  }
  for (uint64_t j = 0; j < elems; j++) {
    const double scale = (j % 64 < 16) ? 1.0e-12 : 1.0;
    xl[j] = (T)(dis(gen) * scale);
    xr[j] = (T)dis(gen);
  }
  std::vector<int> wgt(o.sites, 1);

  // per-instance pinned host buffers, device buffers, streams and events
  const uint32_t P = o.instances;
  std::vector<T *> hL(P), hR(P), dL(P), dR(P), dO(P);
  std::vector<uint8_t *> dS(P);
  std::vector<hipStream_t> st(P);
  std::vector<hipEvent_t> eb(P * o.calls), e1(P * o.calls), e2(P * o.calls), ee(P * o.calls);
  for (uint32_t k = 0; k < P; k++) {
    HIPCHK(hipHostMalloc((void **)&hL[k], tb.instance_elements_left() * es));
    HIPCHK(hipHostMalloc((void **)&hR[k], tb.instance_elements_right() * es));
    HIPCHK(hipMalloc((void **)&dL[k], tb.instance_elements_left() * es));
    HIPCHK(hipMalloc((void **)&dR[k], tb.instance_elements_right() * es));
    HIPCHK(hipMalloc((void **)&dO[k], std::max<uint64_t>(tb.instance_elements_out(), 16) * es));
    HIPCHK(hipMalloc((void **)&dS[k], std::max<uint64_t>(n0, 1)));
    HIPCHK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
    tb.pack<T>(k, ev, bl, br, xl.data(), xr.data(), hL[k], hR[k]);
  }
  for (auto *v : {&eb, &e1, &e2, &ee})
    for (auto &e : *v) HIPCHK(hipEventCreate(&e));

  std::vector<std::vector<T>> result(o.calls, std::vector<T>(elems));
  std::vector<std::vector<uint8_t>> scaler(o.calls, std::vector<uint8_t>(o.sites));
  std::vector<long long> inc(o.calls, 0);
  const int dt = o.f64 ? PLFX_F64 : PLFX_F32;

  auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0; i < o.calls; i++) {
    for (uint32_t k = 0; k < P; k++) {
      const uint64_t nk = tb.alignments_per_instance(k);
      const uint64_t off = tb.instance_site_offset(k);
      const size_t ev_i = (size_t)i * P + k;
      HIPCHK(hipEventRecord(eb[ev_i], st[k]));
      HIPCHK(hipMemcpyAsync(dL[k], hL[k], tb.instance_active_elements_left(k) * es, hipMemcpyHostToDevice, st[k]));
      HIPCHK(hipMemcpyAsync(dR[k], hR[k], tb.instance_active_elements_right(k) * es, hipMemcpyHostToDevice, st[k]));
      HIPCHK(hipEventRecord(e1[ev_i], st[k]));
      rc = plfx_instance_run(ctx, dL[k], dR[k], dO[k], dS[k], (uint32_t)nk,
                             o.aie == plfx::WINDOW ? o.window : 0, o.layout, dt, st[k]);
      if (rc != PLFX_OK) die(std::string("plfx_instance_run: ") + plfx_last_error(ctx));
      HIPCHK(hipEventRecord(e2[ev_i], st[k]));
      HIPCHK(hipMemcpyAsync(result[i].data() + off * 16, dO[k], nk * 16 * es, hipMemcpyDeviceToHost, st[k]));
      HIPCHK(hipMemcpyAsync(scaler[i].data() + off, dS[k], nk, hipMemcpyDeviceToHost, st[k]));
      HIPCHK(hipEventRecord(ee[ev_i], st[k]));
    }
    for (uint32_t k = 0; k < P; k++) HIPCHK(hipStreamSynchronize(st[k]));
    long long s = 0;  // host_mem.cpp:385-388
    for (uint64_t j = 0; j < o.sites; j++) s += (long long)scaler[i][j] * wgt[j];
    inc[i] = s;
  }
  const double wall_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

  // timing regions of instance 0 (as the reference prints, host_mem.cpp:449),
  // plus the slowest/fastest kernel over all instances and calls
  double hm = 0, msm = 0, mh = 0, mx = 0, mn = 1e300;
  for (uint32_t i = 0; i < o.calls; i++) {
    for (uint32_t k = 0; k < P; k++) {
      const size_t ev_i = (size_t)i * P + k;
      float a, b, c;
      HIPCHK(hipEventElapsedTime(&a, eb[ev_i], e1[ev_i]));
      HIPCHK(hipEventElapsedTime(&b, e1[ev_i], e2[ev_i]));
      HIPCHK(hipEventElapsedTime(&c, e2[ev_i], ee[ev_i]));
      if (k == 0) { hm += a; msm += b; mh += c; }
      mx = std::max(mx, (double)b);
      mn = std::min(mn, (double)b);
    }
  }
  const double total_sites = (double)o.sites * o.calls;
  const double bytes = (double)(tb.instance_elements_left() + tb.instance_elements_right() +
                                tb.instance_elements_out()) * es * P * o.calls;
  auto row = [&](const char *name, double ms, double nbytes, double nsites) {
    std::printf("| %-38s | %10.4f | %16.1f | %24.3f |\n", name, ms, nbytes / 1e6 / (ms / 1e3),
                nsites / (ms / 1e3) * 1e-6);
  };
  if (!o.quiet) {
    std::printf("=====================================================================================================\n");
    std::printf("| Timing region                          | time (ms)  | bandwidth (MB/s) |         bandwidth (MA/s) |\n");
    std::printf("=====================================================================================================\n");
    row("Host to GPU memory (instance 0):", hm, bytes / P, total_sites / P);
    row("GPU PLF kernel (instance 0):", msm, bytes / P, total_sites / P);
    row("  - slowest call/instance:", mx, bytes / P / o.calls, total_sites / P / o.calls);
    row("  - fastest call/instance:", mn, bytes / P / o.calls, total_sites / P / o.calls);
    row("GPU memory to host (instance 0):", mh, bytes / P, total_sites / P);
    row("Total wall time (all instances):", wall_ms, bytes, total_sites);
    std::printf("=====================================================================================================\n");
    for (uint32_t i = 0; i < o.calls; i++) std::printf("scalerIncrement[call %u] = %lld\n", i, inc[i]);
  }
  if (!o.dump.empty()) {
    for (uint32_t i = 0; i < o.calls; i++) {
      std::string base = o.dump + "_call" + std::to_string(i);
      FILE *f = std::fopen((base + "_x3.bin").c_str(), "wb");
      if (!f) die("cannot write " + base);
      std::fwrite(result[i].data(), es, elems, f);
      std::fclose(f);
      f = std::fopen((base + "_scaler.bin").c_str(), "wb");
      std::fwrite(scaler[i].data(), 1, o.sites, f);
      std::fclose(f);
      f = std::fopen((base + "_inc.txt").c_str(), "w");
      std::fprintf(f, "%lld\n", inc[i]);
      std::fclose(f);
    }
  }
  for (uint32_t k = 0; k < P; k++) {
    (void)hipHostFree(hL[k]); (void)hipHostFree(hR[k]);
    (void)hipFree(dL[k]); (void)hipFree(dR[k]); (void)hipFree(dO[k]); (void)hipFree(dS[k]);
    (void)hipStreamDestroy(st[k]);
  }
  for (auto *v : {&eb, &e1, &e2, &ee})
    for (auto &e : *v) (void)hipEventDestroy(e);
  plfx_ctx_destroy(ctx);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  Opts o = parse(argc, argv);
  return o.f64 ? run<double>(o) : run<float>(o);
}
