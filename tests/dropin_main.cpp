// Compiles the reference-style call site against include/plfx_plf.hpp: the
// exact plf() signature of app/src/plf.h:1-5, backed by libplfx on the GPU.
// usage: dropin_main <in.bin> <out.bin>   (in = n, EV16, left64, right64,
// x1[16n], x2[16n], wgt[n] as float32/int32; out = x3[16n] then the int)
#include <cstdio>
#include <vector>

#include "plfx_plf.hpp"

int main(int argc, char **argv) {
  if (argc != 3) return 2;
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int n = 0;
  if (std::fread(&n, 4, 1, f) != 1) return 2;
  std::vector<float> ev(16), left(64), right(64), x1(16 * n), x2(16 * n), x3(16 * n);
  std::vector<int> wgt(n);
  size_t ok = std::fread(ev.data(), 4, 16, f) + std::fread(left.data(), 4, 64, f) +
              std::fread(right.data(), 4, 64, f) + std::fread(x1.data(), 4, 16 * n, f) +
              std::fread(x2.data(), 4, 16 * n, f) + std::fread(wgt.data(), 4, n, f);
  std::fclose(f);
  if (ok != (size_t)(144 + 33 * n)) return 2;
  int scalerIncrement = 0;
  plf(x1.data(), x2.data(), x3.data(), ev.data(), n, left.data(), right.data(), wgt.data(),
      scalerIncrement);  // the reference call, unchanged
  f = std::fopen(argv[2], "wb");
  std::fwrite(x3.data(), 4, 16 * n, f);
  std::fwrite(&scalerIncrement, 4, 1, f);
  std::fclose(f);
  return 0;
}
