// ref_shim_f64.cpp -- TEST INFRASTRUCTURE ONLY (see plf_oracle.c header).
//
// The reference's plf() (/root/reference/app/src/plf.cpp:8-68) is written for
// float.  Its double instantiation -- the same loop in f64, which libplfx's
// f64 entry points claim bit for bit -- is built here from the unmodified
// reference source, compiled where it lies: the standard header it uses is
// included first, then `float` is spelled `double` for the reference's own
// header and source.  Nothing of the reference is copied into this
// repository; the binary goes to oracle/_ref/ (git-ignored).
#include <iostream>

#define float double
#include "plf.cpp"
#undef float

extern "C" int plfref_plf_f64(double* x1, double* x2, double* x3, double* EV, int n,
                              double* left, double* right, int* wgt) {
  int scalerIncrement = 0;
  plf(x1, x2, x3, EV, n, left, right, wgt, scalerIncrement);
  return scalerIncrement;
}
