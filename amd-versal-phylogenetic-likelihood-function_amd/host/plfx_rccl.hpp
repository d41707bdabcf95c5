// plfx_rccl.hpp -- the north star's one RCCL all-reduce for the C++ host
// drivers (plfx_tree, plfx_host): a communicator over the GPUs of one node,
// one rank per listed device in this process (ncclCommInitAll), and a single
// grouped sum-all-reduce of per-GPU partials (lnL as f64, scaler totals as
// int64) on the ranks' own streams, over xGMI between MI355X GPUs.
//
// The reference has no collective at all -- its only multi-unit mechanism is
// the instance fan-out over xrt::queues on one card (app/src/host_mem.cpp:
// 249-325); this is the step BASELINE's north star adds for configs[3]
// ("a single RCCL all-reduce over xGMI for the final per-site log-likelihood
// sum").  RCCL refuses a device listed twice in one communicator, so
// --devices lists with repeats (two contexts on one GPU, the one-GPU test
// box's way to rehearse a split) reduce on the host (--reduce host) instead;
// that choice is explicit and printed, never a silent fallback.
#ifndef PLFX_RCCL_HPP
#define PLFX_RCCL_HPP

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

namespace plfx_host {

class NodeComm {
 public:
  // err: empty on success, else why the communicator could not be made
  NodeComm(const std::vector<int> &devices, std::string &err) {
    std::vector<int> d = devices;
    std::sort(d.begin(), d.end());
    if (std::adjacent_find(d.begin(), d.end()) != d.end()) {
      err = "RCCL needs distinct GPUs (ncclCommInitAll rejects a device listed twice); "
            "use --reduce host for a list with repeats";
      return;
    }
    comms_.assign(devices.size(), nullptr);
    const ncclResult_t r = ncclCommInitAll(comms_.data(), (int)devices.size(), devices.data());
    if (r != ncclSuccess) {
      comms_.clear();
      err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
    }
  }
  NodeComm(const NodeComm &) = delete;
  NodeComm &operator=(const NodeComm &) = delete;
  ~NodeComm() {
    for (ncclComm_t c : comms_)
      if (c) (void)ncclCommDestroy(c);
  }

  bool ok() const { return !comms_.empty(); }
  int ranks() const { return (int)comms_.size(); }
  static std::string version() {
    int v = 0;
    (void)ncclGetVersion(&v);
    return std::to_string(v / 10000) + "." + std::to_string(v / 100 % 100) + "." + std::to_string(v % 100);
  }

  // ONE grouped sum-all-reduce, in place: rank q's f64[nf] at f[q] and
  // int64[ni] at i[q] (device pointers on devices_[q], either count may be 0),
  // enqueued on st[q].  i_out (optional): the int64 sums go there instead
  // (out of place).  Returns an empty string or the RCCL error.
  std::string allreduce_sum(const std::vector<double *> &f, size_t nf, const std::vector<int64_t *> &i,
                            size_t ni, const std::vector<hipStream_t> &st,
                            const std::vector<int64_t *> *i_out = nullptr) {
    ncclResult_t r = ncclGroupStart();
    for (size_t q = 0; q < comms_.size() && r == ncclSuccess; q++) {
      if (nf) r = ncclAllReduce(f[q], f[q], nf, ncclFloat64, ncclSum, comms_[q], st[q]);
      if (ni && r == ncclSuccess)
        r = ncclAllReduce(i[q], i_out ? (*i_out)[q] : i[q], ni, ncclInt64, ncclSum, comms_[q], st[q]);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (r == ncclSuccess) r = e;
    return r == ncclSuccess ? std::string() : std::string("ncclAllReduce: ") + ncclGetErrorString(r);
  }

 private:
  std::vector<ncclComm_t> comms_;
};

}  // namespace plfx_host

#endif  // PLFX_RCCL_HPP
