// plfx_plf.hpp -- source-level drop-in for the reference's plf()
// (/root/reference/app/src/plf.h:1-5):
//
//   void plf(float* x1_start, float* x2_start, float* x3_start, float* EV,
//            const int n, float* left, float* right, int* wgt,
//            int& scalerIncrement);
//
// Include this header instead of "plf.h" and link -lplfx: the call runs on the
// MI355X through the C ABI (include/plfx.h) on a process-wide context bound to
// HIP device PLFX_DEVICE (default 0).  Same arguments, same results (bit-exact
// f32), same "no error return" contract as the reference -- a failure is
// reported on stderr and aborts, since the reference signature cannot carry a
// status.  A double overload is provided for the f64 path.
#pragma once
#include <cstdio>
#include <cstdlib>

#include "plfx.h"

namespace plfx_dropin {
inline plfx_ctx *context() {
  static plfx_ctx *ctx = [] {
    plfx_ctx *c = nullptr;
    const char *d = std::getenv("PLFX_DEVICE");
    const int rc = plfx_ctx_create(d ? std::atoi(d) : 0, &c);
    if (rc != PLFX_OK) {
      std::fprintf(stderr, "plfx: no usable gfx950 device (status %d)\n", rc);
      std::abort();
    }
    return c;
  }();
  return ctx;
}
inline void check(int rc) {
  if (rc != PLFX_OK) {
    std::fprintf(stderr, "plfx: plf() failed (%d): %s\n", rc, plfx_last_error(context()));
    std::abort();
  }
}
}  // namespace plfx_dropin

inline void plf(float *x1_start, float *x2_start, float *x3_start, float *EV, const int n,
                float *left, float *right, int *wgt, int &scalerIncrement) {
  plfx_dropin::check(plfx_plf_f32(plfx_dropin::context(), x1_start, x2_start, x3_start, EV, n,
                                  left, right, wgt, &scalerIncrement));
}

inline void plf(double *x1_start, double *x2_start, double *x3_start, double *EV, const int n,
                double *left, double *right, int *wgt, int &scalerIncrement) {
  plfx_dropin::check(plfx_plf_f64(plfx_dropin::context(), x1_start, x2_start, x3_start, EV, n,
                                  left, right, wgt, &scalerIncrement));
}
