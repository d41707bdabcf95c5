// plfx_host.cpp -- C++ host program over the plfx C ABI; the counterpart of the
// reference's app/src/host_mem.cpp (XRT) with the accelerator replaced by HIP.
//
//   usage: plfx_host <alignment sites> <plf calls> <parallel instances>
//                    [--target hw|sw_emu] [--dtype f32|f64] [--layout comb|sep]
//                    [--aie window|stream] [--window BYTES] [--seed S]
//                    [--dump PREFIX] [--no-check] [--quiet]
//                    [--no-intermediate] [--csv FILE] [--devices D0,D1,...]
//                    [--reduce host|rccl]
//
// Mirrors host_mem.cpp:
//   * argv shape <sites> <calls> <instances> (host_mem.cpp:13-38); the xclbin
//     and BDF arguments are gone, layout/AIE type/window are explicit flags
//     instead of being parsed out of the xclbin file name;
//     --target picks the run mode as the Makefile's TARGET does
//     (Makefile:199-220): hw = the GPU, sw_emu = the accelerator instance
//     emulated on the CPU (plfx_swemu_instance_run, no GPU touched);
//   * size table (host_mem.cpp:45-101) from testbench sizing (include.h:150-266);
//   * host_mem input protocol (host_mem.cpp:179-209) with a fixed seed (Q8);
//   * per-instance packing [EV|P_L|CLV_L], [EV|P_R|CLV_R] / [P_R|CLV_R]
//     (host_mem.cpp:221-243);
//   * per call, per instance on two HIP streams joined by events, as the
//     reference's main/right queues (host_mem.cpp:283-325): H2D left (main)
//     || H2D right (right) -> fused kernel (main) -> D2H CLV (main) || D2H
//     scaler (right), with the begin/t1/t2/end regions of timing.h:25-52
//     taken by HIP events on the main stream;
//   * --no-intermediate: the reference's NO_INTERMEDIATE_RESULTS build
//     (host_mem.cpp:327-382,390-392,454-468): per call the instance buffers
//     are packed inside the timed region ("Prepare input"), all instances run
//     on main/right/output streams (H2D left || H2D right -> kernel -> D2H
//     scaler || D2H CLV), and the host scaler reduction is its own region
//     ("scaling wgt mult"), all on the host clock as the reference's t.elapsed();
//   * --csv FILE: the per-call timing CSV of write_to_csv (timing.h:153-194):
//     hm<k>,msasm<k>,mh<k> columns per instance, or preparation,plf,scaling
//     with --no-intermediate;
//   * --devices D0,D1,...: instance k runs on GPU D[k % count] (one plfx
//     context per GPU, the instance's buffers, streams and events on it):
//     the reference's instance partition (include.h:181-195) spread over the
//     GPUs of a node the way its instances share one card; a device may be
//     listed twice (two contexts on one GPU).  Default: GPU 0;
//   * host scaler reduction sum scaler[j]*wgt[j] (host_mem.cpp:384-388);
//     --reduce rccl instead: every instance's weighted sum on its GPU
//     (plfx_scaler_sum, in the kernel region) into its slot of a per-GPU
//     int64[instances] vector, then ONE RCCL all-reduce over the --devices
//     list (ncclCommInitAll, plfx_rccl.hpp; distinct GPUs only) and the
//     instance totals added on the host -- the north star's all-reduce over
//     xGMI in place of the host loop.  The reduction that ran is printed
//     ("reduce = ..."); the default stays the reference's host loop;
//   * the correctness check of host_mem.cpp:403-442: this program's own CPU
//     plf() (below, plf.cpp:19-65 restated) run plf_calls times and timed,
//     every CLV value and every scalerIncrement compared exactly, "Test result:
//     Passed" / "Failed with N errors" (a scalerIncrement mismatch counts as
//     an error here; the reference only prints it);
//   * the timing table of timing.h:107-151 per instance and for all instances
//     together (the reference prints instance 0 only), with the
//     Reference row and the speed-ups excluding / including the transfers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>
#include <unistd.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../../include/plfx.h"
#include "../csrc/testbench.hpp"
#include "plfx_rccl.hpp"

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
  bool sw_emu = false;
  bool check = true;
  int layout = plfx::SEPARATE;
  int aie = plfx::WINDOW;
  uint32_t window = 8192;
  uint32_t seed = 20250117u;
  std::string dump;
  std::string csv;
  bool quiet = false;
  bool no_intermediate = false;
  std::vector<int> devices{0};
  bool rccl = false;  // --reduce host (default, host_mem.cpp:384-388) | rccl
};

Opts parse(int argc, char **argv) {
  if (argc < 4)
    die("usage: plfx_host <alignment sites> <plf calls> <parallel instances> [--target hw|sw_emu] "
        "[--dtype f32|f64] [--layout comb|sep] [--aie window|stream] [--window BYTES] [--seed S] "
        "[--dump PREFIX] [--no-check] [--quiet] [--no-intermediate] [--csv FILE] [--devices D0,D1,...] "
        "[--reduce host|rccl]");
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
    } else if (a == "--target") {
      std::string v = next();
      if (v == "hw") o.sw_emu = false;
      else if (v == "sw_emu") o.sw_emu = true;
      else die("bad target " + v);
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
    } else if (a == "--no-check") {
      o.check = false;
    } else if (a == "--quiet") {
      o.quiet = true;
    } else if (a == "--no-intermediate") {
      o.no_intermediate = true;
    } else if (a == "--csv") {
      o.csv = next();
    } else if (a == "--reduce") {
      std::string v = next();
      if (v == "rccl") o.rccl = true;
      else if (v == "host") o.rccl = false;
      else die("bad reduction " + v + " (host|rccl)");
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
  if (o.instances == 0 || o.calls == 0) die("calls and instances must be > 0");
  if (o.aie == plfx::WINDOW && (o.window < 32 || o.window % 32)) die("window must be a multiple of 32 bytes");
  if (o.sw_emu && o.aie == plfx::STREAM && o.layout != plfx::COMBINED)
    die("stream movers exist in the COMBINED layout only");
  if (o.sw_emu && o.no_intermediate) die("--no-intermediate is a GPU (hw) run mode");
  if (o.sw_emu && (o.devices.size() != 1 || o.devices[0] != 0)) die("--devices is a GPU (hw) option");
  if (o.sw_emu && o.rccl) die("--reduce rccl is a GPU (hw) option");
  return o;
}

// The host program's own CPU plf() -- the reference host links plf.cpp for
// its "Reference" row and correctness check (host_mem.cpp:416-420); this is
// that loop (plf.cpp:19-65) restated, in T.  Built with -ffp-contract=off.
template <typename T>
void cpu_plf(const T *x1, const T *x2, T *x3, const T *EV, uint64_t n, const T *left, const T *right,
             const int *wgt, long long &scalerIncrement) {
  long long add = 0;
  for (uint64_t i = 0; i < n; i++) {
    const T *a = x1 + 16 * i, *b = x2 + 16 * i;
    T *o = x3 + 16 * i;
    for (int j = 0; j < 16; j++) o[j] = T(0);
    for (int c = 0; c < 4; c++) {
      for (int k = 0; k < 4; k++) {
        T ul = T(0), ur = T(0);
        for (int l = 0; l < 4; l++) {
          ul += a[c * 4 + l] * left[c * 16 + k * 4 + l];
          ur += b[c * 4 + l] * right[c * 16 + k * 4 + l];
        }
        const T p = ul * ur;
        for (int l = 0; l < 4; l++) o[c * 4 + l] += p * EV[k * 4 + l];
      }
    }
    bool scale = true;
    for (int j = 0; j < 16 && scale; j++) scale = std::fabs((double)o[j]) < 1.0 / 4294967296.0;
    if (scale) {
      for (int j = 0; j < 16; j++) o[j] = (T)(o[j] * 4294967296.0);
      add += wgt[i];
    }
  }
  scalerIncrement = add;
}

struct Regions {  // timing.h:25-52: begin/t1/t2/end of one call of one instance, ms
  double begin, t1, t2, end;
  double hm() const { return t1 - begin; }
  double msm() const { return t2 - t1; }
  double mh() const { return end - t2; }
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
  const char *target = o.sw_emu ? "sw_emu" : "hw";

  if (!o.quiet) {
    std::printf("==================================================================================\n");
    std::printf("| target:                  | %53s |\n", target);
    std::printf("| alignment sites:        | %54llu |\n", (unsigned long long)o.sites);
    std::printf("| plf calls:              | %54u |\n", o.calls);
    std::printf("| parallel plfs:          | %54u |\n", o.instances);
    std::printf("| element type:           | %54s |\n", o.f64 ? "f64" : "f32");
    std::printf("| layout / aie / window:  | %34s %8s %10u |\n", o.layout == plfx::COMBINED ? "COMBINED" : "SEPARATE",
                o.aie == plfx::WINDOW ? "window" : "stream", o.window);
    if (!o.sw_emu) {
      std::string dl;
      for (size_t q = 0; q < o.devices.size(); q++) dl += (q ? "," : "") + std::to_string(o.devices[q]);
      std::printf("| GPUs (instance k: #k%%n): | %54s |\n", dl.c_str());
    }
    std::printf("==================================================================================\n");
    std::printf("|                         |       alignments |         elements |     size (bytes) |\n");
    std::printf("| instance left:          | %16llu | %16llu | %16llu |\n", (unsigned long long)n0,
                (unsigned long long)tb.instance_elements_left(), (unsigned long long)(tb.instance_elements_left() * es));
    std::printf("| instance right:         | %16llu | %16llu | %16llu |\n", (unsigned long long)n0,
                (unsigned long long)tb.instance_elements_right(), (unsigned long long)(tb.instance_elements_right() * es));
    std::printf("| instance out:           | %16llu | %16llu | %16llu |\n", (unsigned long long)n0,
                (unsigned long long)tb.instance_elements_out(), (unsigned long long)(tb.instance_elements_out() * es));
    // host_mem.cpp:70-82: the instances' buffers together, and all plf calls
    const unsigned long long P_ = o.instances, S_ = o.sites;
    std::printf("----------------------------------------------------------------------------------\n");
    std::printf("| buffer left:            | %16llu | %16llu | %16llu |\n", S_,
                (unsigned long long)tb.instance_elements_left() * P_, (unsigned long long)(tb.instance_elements_left() * P_ * es));
    std::printf("| buffer right:           | %16llu | %16llu | %16llu |\n", S_,
                (unsigned long long)tb.instance_elements_right() * P_, (unsigned long long)(tb.instance_elements_right() * P_ * es));
    std::printf("| buffer out:             | %16llu | %16llu | %16llu |\n", S_,
                (unsigned long long)tb.instance_elements_out() * P_, (unsigned long long)(tb.instance_elements_out() * P_ * es));
    std::printf("----------------------------------------------------------------------------------\n");
    const unsigned long long data_el = (unsigned long long)tb.elements_per_instance() * P_ * o.calls;
    std::printf("| total (%3u plf calls):  | %16llu | %16llu | %16llu |\n", o.calls, S_ * o.calls, data_el,
                data_el * es);
    std::printf("==================================================================================\n");
    // host_mem.cpp:84-88: memory this run holds on the host and on the device
    // (capacities from the machine and the GPU instead of the VCK5000's 256 / 12 GB)
    const double host_b = (double)es * (2.0 * o.sites * 16 + (double)o.calls * o.sites * 16 +
                                        (o.check ? o.sites * 16.0 : 0.0)) +
                          (double)o.calls * o.sites + 4.0 * o.sites +
                          (o.sw_emu ? 0.0 : (double)P_ * (tb.instance_elements_left() + tb.instance_elements_right()) * es);
    const double host_cap = (double)sysconf(_SC_PHYS_PAGES) * (double)sysconf(_SC_PAGE_SIZE);
    std::printf("| RAM usage (host):       | %14.6f GB of %7.1f GB (%12.6f %%)      |\n", host_b / 1e9, host_cap / 1e9,
                host_cap > 0 ? 100.0 * host_b / host_cap : 0.0);
    const double dev_b = (double)P_ * ((tb.instance_elements_left() + tb.instance_elements_right() +
                                        tb.instance_elements_out()) * es + n0);
    if (o.sw_emu) {
      std::printf("| RAM usage (GPU):        | %54s |\n", "none (sw_emu: the instances run on the host)");
    } else {
      size_t free_b = 0, total_b = 0;
      HIPCHK(hipSetDevice(o.devices[0]));
      HIPCHK(hipMemGetInfo(&free_b, &total_b));
      const double per_gpu = dev_b / (double)std::min<size_t>(o.devices.size(), P_);
      std::printf("| RAM usage (GPU):        | %14.6f GB of %7.1f GB (%12.6f %%)      |\n", per_gpu / 1e9,
                  (double)total_b / 1e9, total_b ? 100.0 * per_gpu / (double)total_b : 0.0);
    }
    std::printf("==================================================================================\n");
  }

  // host_mem.cpp:179-209 input protocol, fixed seed
  T ev[16], bl[64], br[64];
  const uint64_t elems = o.sites * 16;
  std::vector<T> xl(elems), xr(elems);
  std::vector<int> wgt(o.sites, 1);
  plfx::gen_hostmem<T>(o.seed, o.sites, ev, bl, br, xl.data(), xr.data(), wgt.data());

  const uint32_t P = o.instances;
  std::vector<std::vector<T>> result(o.calls, std::vector<T>(elems));
  std::vector<std::vector<uint8_t>> scaler(o.calls, std::vector<uint8_t>(o.sites));
  std::vector<long long> inc(o.calls, 0);
  std::vector<Regions> reg((size_t)o.calls * P);  // [call][instance]
  std::vector<Regions> callreg(o.calls);           // --no-intermediate: [call], host clock
  const int dt = o.f64 ? PLFX_F64 : PLFX_F32;
  double wall_ms = 0;

  if (o.sw_emu) {
    // the instance dataflow on the CPU; no device memory, so no transfer regions
    std::vector<std::vector<T>> hL(P, std::vector<T>(tb.instance_elements_left())),
        hR(P, std::vector<T>(tb.instance_elements_right()));
    for (uint32_t k = 0; k < P; k++) tb.pack<T>(k, ev, bl, br, xl.data(), xr.data(), hL[k].data(), hR[k].data());
    auto t0 = std::chrono::steady_clock::now();
    auto ms_since = [&](std::chrono::steady_clock::time_point a) {
      return std::chrono::duration<double, std::milli>(a - t0).count();
    };
    roctxRangePush("plfx_host roundtrip (sw_emu)");  // the reference's XRT user range, host_mem.cpp:273,395
    for (uint32_t i = 0; i < o.calls; i++) {
      for (uint32_t k = 0; k < P; k++) {
        const uint64_t nk = tb.alignments_per_instance(k), off = tb.instance_site_offset(k);
        Regions &r = reg[(size_t)i * P + k];
        r.begin = r.t1 = ms_since(std::chrono::steady_clock::now());
        const int rc = plfx_swemu_instance_run(hL[k].data(), hR[k].data(), result[i].data() + off * 16,
                                               scaler[i].data() + off, (uint32_t)nk,
                                               o.aie == plfx::WINDOW ? o.window : 0, o.layout, o.aie, dt);
        if (rc != PLFX_OK) die("plfx_swemu_instance_run failed: " + std::to_string(rc));
        r.t2 = r.end = ms_since(std::chrono::steady_clock::now());
      }
      long long s = 0;  // host_mem.cpp:385-388
      for (uint64_t j = 0; j < o.sites; j++) s += (long long)scaler[i][j] * wgt[j];
      inc[i] = s;
    }
    roctxRangePop();
    wall_ms = ms_since(std::chrono::steady_clock::now());
  } else {
    // one context per listed GPU; instance k on list entry k % count
    const size_t nd = o.devices.size();
    std::vector<plfx_ctx *> ctxs(nd, nullptr);
    int rc = PLFX_OK;
    for (size_t q = 0; q < nd; q++) {
      rc = plfx_ctx_create_ex(o.devices[q], PLFX_CTX_LAZY_TABLES, &ctxs[q]);  // DNA only: no table pool
      if (rc != PLFX_OK) die("plfx_ctx_create(" + std::to_string(o.devices[q]) + ") failed: " + std::to_string(rc));
    }
    auto slot = [&](uint32_t k) { return (size_t)k % nd; };
    auto on = [&](uint32_t k) { HIPCHK(hipSetDevice(o.devices[slot(k)])); };
    // per-instance pinned host buffers, device buffers, the reference's three
    // queues (main / right / output, host_mem.cpp:123-127) as HIP streams, and
    // the events that join them
    std::vector<T *> hL(P), hR(P), dL(P), dR(P), dO(P);
    std::vector<uint8_t *> dS(P);
    std::vector<hipStream_t> st(P), sr(P), so(P);
    std::vector<hipEvent_t> eb(P * o.calls), e1(P * o.calls), e2(P * o.calls), ee(P * o.calls);
    std::vector<hipEvent_t> j_up(P), j_run(P), j_dn(P);  // joins: right upload, kernel, side download
    std::vector<hipEvent_t> e0(P);  // per instance: events time against one on their own GPU
    for (uint32_t k = 0; k < P; k++) {
      on(k);
      HIPCHK(hipHostMalloc((void **)&hL[k], tb.instance_elements_left() * es, hipHostMallocPortable));
      HIPCHK(hipHostMalloc((void **)&hR[k], tb.instance_elements_right() * es, hipHostMallocPortable));
      HIPCHK(hipMalloc((void **)&dL[k], tb.instance_elements_left() * es));
      HIPCHK(hipMalloc((void **)&dR[k], tb.instance_elements_right() * es));
      HIPCHK(hipMalloc((void **)&dO[k], std::max<uint64_t>(tb.instance_elements_out(), 16) * es));
      HIPCHK(hipMalloc((void **)&dS[k], std::max<uint64_t>(n0, 1)));
      for (auto *q : {&st, &sr, &so}) HIPCHK(hipStreamCreateWithFlags(&(*q)[k], hipStreamNonBlocking));
      for (auto *q : {&j_up, &j_run, &j_dn}) HIPCHK(hipEventCreateWithFlags(&(*q)[k], hipEventDisableTiming));
      HIPCHK(hipEventCreate(&e0[k]));
      for (uint32_t i = 0; i < o.calls; i++)
        for (auto *v : {&eb, &e1, &e2, &ee}) HIPCHK(hipEventCreate(&(*v)[(size_t)i * P + k]));
      if (!o.no_intermediate) tb.pack<T>(k, ev, bl, br, xl.data(), xr.data(), hL[k], hR[k]);
    }
    // --reduce rccl: the communicator over the list, per list entry a stream
    // and the int64[P] slot vector (dSlot: instance k's sum in slot k on its own
    // GPU, zeros elsewhere) with its reduced copy (dSum); per instance its
    // weights on the device
    std::unique_ptr<plfx_host::NodeComm> comm;
    std::vector<int64_t *> dSlot(nd, nullptr), dSum(nd, nullptr);
    std::vector<hipStream_t> sq(nd, nullptr);
    std::vector<int32_t *> dW(P, nullptr);
    if (o.rccl) {
      std::string err;
      comm.reset(new plfx_host::NodeComm(o.devices, err));
      if (!err.empty()) die(err);
      for (size_t q = 0; q < nd; q++) {
        HIPCHK(hipSetDevice(o.devices[q]));
        HIPCHK(hipMalloc((void **)&dSlot[q], P * sizeof(int64_t)));
        HIPCHK(hipMalloc((void **)&dSum[q], P * sizeof(int64_t)));
        HIPCHK(hipMemset(dSlot[q], 0, P * sizeof(int64_t)));
        HIPCHK(hipStreamCreateWithFlags(&sq[q], hipStreamNonBlocking));
      }
      for (uint32_t k = 0; k < P; k++) {
        on(k);
        const uint64_t nk = tb.alignments_per_instance(k);
        HIPCHK(hipMalloc((void **)&dW[k], std::max<uint64_t>(nk, 1) * sizeof(int32_t)));
        HIPCHK(hipMemcpy(dW[k], wgt.data() + tb.instance_site_offset(k), nk * sizeof(int32_t),
                         hipMemcpyHostToDevice));
      }
    }
    // instance k's weighted scaler sum on its GPU, into its slot (rccl only)
    auto device_sum = [&](uint32_t k) {
      if (!o.rccl) return;
      plfx_ctx *ctx = ctxs[slot(k)];
      rc = plfx_scaler_sum(ctx, dS[k], dW[k], (int64_t)tb.alignments_per_instance(k), dSlot[slot(k)] + k, st[k]);
      if (rc != PLFX_OK) die(std::string("plfx_scaler_sum: ") + plfx_last_error(ctx));
    };
    // the call's scalerIncrement: the reference's host loop (host_mem.cpp:
    // 385-388) over the downloaded bytes, or ONE RCCL all-reduce of the slot
    // vectors (after every instance of the call finished) and the P totals
    auto reduce_call = [&](uint32_t i) -> long long {
      long long s = 0;
      if (!o.rccl) {
        for (uint64_t j = 0; j < o.sites; j++) s += (long long)scaler[i][j] * wgt[j];
        return s;
      }
      const std::string err = comm->allreduce_sum(std::vector<double *>(nd, nullptr), 0, dSlot, P, sq, &dSum);
      if (!err.empty()) die(err);
      for (size_t q = 0; q < nd; q++) HIPCHK(hipStreamSynchronize(sq[q]));
      std::vector<int64_t> v(P);
      HIPCHK(hipSetDevice(o.devices[0]));
      HIPCHK(hipMemcpy(v.data(), dSum[0], P * sizeof(int64_t), hipMemcpyDeviceToHost));
      for (int64_t x : v) s += x;
      return s;
    };
    for (size_t q = 0; q < nd; q++) {
      HIPCHK(hipSetDevice(o.devices[q]));
      HIPCHK(hipDeviceSynchronize());
    }
    auto t0 = std::chrono::steady_clock::now();
    auto ms_since = [&](std::chrono::steady_clock::time_point a) {
      return std::chrono::duration<double, std::milli>(a - t0).count();
    };
    auto run_instance = [&](uint32_t k) {
      const uint64_t nk = tb.alignments_per_instance(k);
      plfx_ctx *ctx = ctxs[slot(k)];
      rc = plfx_instance_run(ctx, dL[k], dR[k], dO[k], dS[k], (uint32_t)nk,
                             o.aie == plfx::WINDOW ? o.window : 0, o.layout, dt, st[k]);
      if (rc != PLFX_OK) die(std::string("plfx_instance_run: ") + plfx_last_error(ctx));
    };
    // host-side ranges for rocprofv3 --marker-trace: the whole run (the
    // reference's XRT user range "roundtrip_exec_time", host_mem.cpp:273,395)
    // and each plf call's enqueue + wait; the H2D / kernel / D2H regions
    // themselves are the events below and the kernel trace
    roctxRangePush("plfx_host roundtrip");
    for (uint32_t k = 0; k < P; k++) HIPCHK(hipEventRecord(e0[k], st[k]));
    for (uint32_t i = 0; i < o.calls; i++) {
      roctxRangePush("plf call (all instances)");
      if (!o.no_intermediate) {
        for (uint32_t k = 0; k < P; k++) {
          const uint64_t nk = tb.alignments_per_instance(k);
          const uint64_t off = tb.instance_site_offset(k);
          const size_t ev_i = (size_t)i * P + k;
          // time: begin; the right stream starts after it (so after the
          // previous call's kernel and downloads of this instance)
          HIPCHK(hipEventRecord(eb[ev_i], st[k]));
          HIPCHK(hipStreamWaitEvent(sr[k], eb[ev_i], 0));
          HIPCHK(hipMemcpyAsync(dL[k], hL[k], tb.instance_active_elements_left(k) * es, hipMemcpyHostToDevice, st[k]));
          HIPCHK(hipMemcpyAsync(dR[k], hR[k], tb.instance_active_elements_right(k) * es, hipMemcpyHostToDevice, sr[k]));
          HIPCHK(hipEventRecord(j_up[k], sr[k]));
          HIPCHK(hipStreamWaitEvent(st[k], j_up[k], 0));
          HIPCHK(hipEventRecord(e1[ev_i], st[k]));  // time: t1
          run_instance(k);
          device_sum(k);
          HIPCHK(hipEventRecord(e2[ev_i], st[k]));  // time: t2
          HIPCHK(hipStreamWaitEvent(sr[k], e2[ev_i], 0));
          HIPCHK(hipMemcpyAsync(result[i].data() + off * 16, dO[k], nk * 16 * es, hipMemcpyDeviceToHost, st[k]));
          HIPCHK(hipMemcpyAsync(scaler[i].data() + off, dS[k], nk, hipMemcpyDeviceToHost, sr[k]));
          HIPCHK(hipEventRecord(j_dn[k], sr[k]));
          HIPCHK(hipStreamWaitEvent(st[k], j_dn[k], 0));
          HIPCHK(hipEventRecord(ee[ev_i], st[k]));  // time: end
        }
        for (uint32_t k = 0; k < P; k++) HIPCHK(hipStreamSynchronize(st[k]));
        inc[i] = reduce_call(i);
      } else {
        // NO_INTERMEDIATE_RESULTS (host_mem.cpp:327-392): prepare, run, reduce
        Regions &r = callreg[i];
        r.begin = ms_since(std::chrono::steady_clock::now());
        for (uint32_t k = 0; k < P; k++) tb.pack<T>(k, ev, bl, br, xl.data(), xr.data(), hL[k], hR[k]);
        r.t1 = ms_since(std::chrono::steady_clock::now());
        for (uint32_t k = 0; k < P; k++) {
          const uint64_t nk = tb.alignments_per_instance(k);
          const uint64_t off = tb.instance_site_offset(k);
          HIPCHK(hipMemcpyAsync(dL[k], hL[k], tb.instance_active_elements_left(k) * es, hipMemcpyHostToDevice, st[k]));
          HIPCHK(hipMemcpyAsync(dR[k], hR[k], tb.instance_active_elements_right(k) * es, hipMemcpyHostToDevice, sr[k]));
          HIPCHK(hipEventRecord(j_up[k], sr[k]));
          HIPCHK(hipStreamWaitEvent(st[k], j_up[k], 0));
          run_instance(k);
          device_sum(k);
          HIPCHK(hipEventRecord(j_run[k], st[k]));
          HIPCHK(hipStreamWaitEvent(so[k], j_run[k], 0));
          HIPCHK(hipMemcpyAsync(scaler[i].data() + off, dS[k], nk, hipMemcpyDeviceToHost, st[k]));
          HIPCHK(hipMemcpyAsync(result[i].data() + off * 16, dO[k], nk * 16 * es, hipMemcpyDeviceToHost, so[k]));
          HIPCHK(hipEventRecord(j_dn[k], so[k]));
          HIPCHK(hipStreamWaitEvent(st[k], j_dn[k], 0));
        }
        for (uint32_t k = 0; k < P; k++) HIPCHK(hipStreamSynchronize(st[k]));
        r.t2 = ms_since(std::chrono::steady_clock::now());
        inc[i] = reduce_call(i);  // the "scaling wgt mult" region
        r.end = ms_since(std::chrono::steady_clock::now());
      }
      roctxRangePop();
    }
    roctxRangePop();
    wall_ms = ms_since(std::chrono::steady_clock::now());
    if (!o.no_intermediate) {
      for (size_t q = 0; q < reg.size(); q++) {
        const hipEvent_t z = e0[q % P];
        float a, b, c, d;
        HIPCHK(hipEventElapsedTime(&a, z, eb[q]));
        HIPCHK(hipEventElapsedTime(&b, z, e1[q]));
        HIPCHK(hipEventElapsedTime(&c, z, e2[q]));
        HIPCHK(hipEventElapsedTime(&d, z, ee[q]));
        reg[q] = Regions{a, b, c, d};
      }
    }
    for (uint32_t k = 0; k < P; k++) {
      on(k);
      (void)plfx_ctx_release_stream(ctxs[slot(k)], st[k]);  // before the stream is destroyed (plfx.h)
      (void)hipHostFree(hL[k]); (void)hipHostFree(hR[k]);
      (void)hipFree(dL[k]); (void)hipFree(dR[k]); (void)hipFree(dO[k]); (void)hipFree(dS[k]);
      for (auto *q : {&st, &sr, &so}) (void)hipStreamDestroy((*q)[k]);
      for (auto *q : {&j_up, &j_run, &j_dn}) (void)hipEventDestroy((*q)[k]);
      (void)hipEventDestroy(e0[k]);
      for (uint32_t i = 0; i < o.calls; i++)
        for (auto *v : {&eb, &e1, &e2, &ee}) (void)hipEventDestroy((*v)[(size_t)i * P + k]);
    }
    comm.reset();  // before the streams it reduced on go away
    for (size_t q = 0; q < nd && o.rccl; q++) {
      HIPCHK(hipSetDevice(o.devices[q]));
      (void)hipStreamDestroy(sq[q]);
      (void)hipFree(dSlot[q]);
      (void)hipFree(dSum[q]);
    }
    for (uint32_t k = 0; k < P && o.rccl; k++) {
      on(k);
      (void)hipFree(dW[k]);
    }
    for (plfx_ctx *c : ctxs) plfx_ctx_destroy(c);
  }

  // ---- correctness check and the CPU "Reference" region (host_mem.cpp:403-442)
  double ref_ms = 0;
  std::string verdict = "skipped (--no-check)";
  unsigned errors = 0;
  if (o.check) {
    std::vector<T> cpu(elems);
    std::vector<long long> cinc(o.calls);
    for (uint32_t i = 0; i < o.calls; i++) {
      auto a = std::chrono::steady_clock::now();
      roctxRangePush("reference plf() (CPU)");
      cpu_plf<T>(xl.data(), xr.data(), cpu.data(), ev, o.sites, bl, br, wgt.data(), cinc[i]);
      roctxRangePop();
      ref_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
      for (uint64_t j = 0; j < elems && errors < 20; j++) {
        if (std::memcmp(&cpu[j], &result[i][j], sizeof(T)) != 0) {  // bit patterns, stricter than !=
          std::printf("ERROR: alignment data wrong for call %u at alignment %llu, probability %llu, "
                      "cpu!=%s: %.17g!=%.17g\n", i, (unsigned long long)(j >> 4),
                      (unsigned long long)(j % 16), target, (double)cpu[j], (double)result[i][j]);
          errors++;
        }
      }
      if (cinc[i] != inc[i]) {
        std::printf("ERROR: scalerIncrement wrong for call %u, cpu!=gpu: %lld!=%lld\n", i, cinc[i], inc[i]);
        errors++;
      }
    }
    verdict = errors == 0 ? "Passed"
                          : (errors >= 20 ? "Failed with more than 20 errors"
                                          : "Failed with " + std::to_string(errors) + " errors");
  }

  // ---- timing table (timing.h:107-151), per instance and for all instances
  const double bytes_inst = (double)(tb.instance_elements_left() + tb.instance_elements_right() +
                                     tb.instance_elements_out()) * es;
  const double total_sites = (double)o.sites * o.calls;
  auto row = [&](const std::string &name, double ms, double nbytes, double nsites) {
    std::printf("| %-38s | %10.4f | %16.1f | %24.3f |\n", name.c_str(), ms,
                ms > 0 ? nbytes / 1e6 / (ms / 1e3) : 0.0, ms > 0 ? nsites / (ms / 1e3) * 1e-6 : 0.0);
  };
  // all instances of a call together: first begin .. last end of each region
  // (--no-intermediate: the call's host-clock regions)
  double agg_hm = 0, agg_msm = 0, agg_mh = 0;
  for (uint32_t i = 0; i < o.calls && o.no_intermediate; i++) {
    agg_hm += callreg[i].hm();
    agg_msm += callreg[i].msm();
    agg_mh += callreg[i].mh();
  }
  for (uint32_t i = 0; i < o.calls && !o.no_intermediate; i++) {
    Regions a{1e300, -1e300, -1e300, -1e300};
    double b0 = 1e300;
    for (uint32_t k = 0; k < P; k++) {
      const Regions &r = reg[(size_t)i * P + k];
      b0 = std::min(b0, r.begin);
      a.t1 = std::max(a.t1, r.t1);
      a.t2 = std::max(a.t2, r.t2);
      a.end = std::max(a.end, r.end);
    }
    a.begin = b0;
    agg_hm += a.hm();
    agg_msm += a.msm();
    agg_mh += a.mh();
  }
  if (!o.quiet) {
    std::printf("=====================================================================================================\n");
    std::printf("| Timing region (%-6s)                 | time (ms)  | bandwidth (MB/s) |         bandwidth (MA/s) |\n", target);
    std::printf("=====================================================================================================\n");
  }
  if (!o.quiet && o.no_intermediate) {
    // the NO_INTERMEDIATE_RESULTS table (host_mem.cpp:454-468)
    row("Prepare input for GPU:", agg_hm, bytes_inst * P * o.calls, total_sites);
    row("PLF on GPU:", agg_msm, bytes_inst * P * o.calls, total_sites);
    row("scaling wgt mult:", agg_mh, bytes_inst * P * o.calls, total_sites);
  }
  if (!o.quiet && !o.no_intermediate) {
    for (uint32_t k = 0; k < P; k++) {
      const double nk_sites = (double)tb.alignments_per_instance(k) * o.calls;
      double hm = 0, msm = 0, mh = 0, mx = 0, mn = 1e300;
      for (uint32_t i = 0; i < o.calls; i++) {
        const Regions &r = reg[(size_t)i * P + k];
        hm += r.hm();
        msm += r.msm();
        mh += r.mh();
        mx = std::max(mx, r.msm());
        mn = std::min(mn, r.msm());
      }
      const std::string tag = "[instance " + std::to_string(k) + "] ";
      row(tag + "Host to GPU memory:", hm, bytes_inst * o.calls, nk_sites);
      row(tag + "GPU PLF kernel:", msm, bytes_inst * o.calls, nk_sites);
      row("  - slowest call:", mx, bytes_inst, nk_sites / o.calls);
      row("  - fastest call:", mn, bytes_inst, nk_sites / o.calls);
      row(tag + "GPU memory to host:", mh, bytes_inst * o.calls, nk_sites);
    }
    std::printf("|----------------------------------------+------------+------------------+--------------------------|\n");
    row("[all instances] Host to GPU memory:", agg_hm, bytes_inst * P * o.calls, total_sites);
    row("[all instances] GPU PLF kernel:", agg_msm, bytes_inst * P * o.calls, total_sites);
    row("[all instances] GPU memory to host:", agg_mh, bytes_inst * P * o.calls, total_sites);
  }
  if (!o.quiet) {
    row("Total execution time:", wall_ms, bytes_inst * P * o.calls, total_sites);
    std::printf("=====================================================================================================\n");
    if (o.check) {
      row("Reference (CPU plf, 1 thread):", ref_ms, bytes_inst * P * o.calls, total_sites);
      std::printf("|----------------------------------------+------------+------------------+--------------------------|\n");
      std::printf("| Speed up (excluding transfers):        | %56.3f |\n", agg_msm > 0 ? ref_ms / agg_msm : 0.0);
      std::printf("| Speed up (including transfers):        | %56.3f |\n", wall_ms > 0 ? ref_ms / wall_ms : 0.0);
      std::printf("=====================================================================================================\n");
    }
    for (uint32_t i = 0; i < o.calls; i++) std::printf("scalerIncrement[call %u] = %lld\n", i, inc[i]);
  }
  if (!o.sw_emu)
    std::printf("reduce = %s\n", o.rccl ? ("rccl (" + std::to_string(o.devices.size()) + " rank" +
                                           (o.devices.size() > 1 ? "s" : "") + ", RCCL " +
                                           plfx_host::NodeComm::version() + ")").c_str()
                                        : "host (host_mem.cpp:384-388 loop)");
  std::printf("Test result: %s\n", verdict.c_str());
  if (!o.csv.empty()) {  // write_to_csv (timing.h:153-194), ms per call
    FILE *f = std::fopen(o.csv.c_str(), "w");
    if (!f) die("cannot write " + o.csv);
    if (o.no_intermediate) {
      std::fprintf(f, "preparation,plf,scaling\n");
      for (uint32_t i = 0; i < o.calls; i++)
        std::fprintf(f, "%.6f,%.6f,%.6f\n", callreg[i].hm(), callreg[i].msm(), callreg[i].mh());
    } else {
      const char *col[3] = {"hm", "msasm", "mh"};
      for (int c = 0; c < 3; c++)
        for (uint32_t k = 0; k < P; k++) std::fprintf(f, "%s%s%u", c || k ? "," : "", col[c], k);
      std::fprintf(f, "\n");
      for (uint32_t i = 0; i < o.calls; i++) {
        for (int c = 0; c < 3; c++)
          for (uint32_t k = 0; k < P; k++) {
            const Regions &r = reg[(size_t)i * P + k];
            std::fprintf(f, "%s%.6f", c || k ? "," : "", c == 0 ? r.hm() : (c == 1 ? r.msm() : r.mh()));
          }
        std::fprintf(f, "\n");
      }
    }
    std::fclose(f);
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
  return errors == 0 ? 0 : 1;
}

}  // namespace

int main(int argc, char **argv) {
  Opts o = parse(argc, argv);
  return o.f64 ? run<double>(o) : run<float>(o);
}
