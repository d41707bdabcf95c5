// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY (see plf_oracle.c header).
//
// A C-linkage entry point over the reference's own plf() so that the tests
// can call the unmodified reference (/root/reference/app/src/plf.cpp:8-68,
// declared in app/src/plf.h:1-5) through ctypes.  The reference source is
// compiled where it lies; nothing of it is copied into this repository.
// The binary goes to oracle/_ref/ (git-ignored, shipped to the GPU box).
#include "plf.h"

extern "C" int plfref_plf(float* x1, float* x2, float* x3, float* EV, int n,
                          float* left, float* right, int* wgt) {
  int scalerIncrement = 0;
  plf(x1, x2, x3, EV, n, left, right, wgt, scalerIncrement);
  return scalerIncrement;
}
