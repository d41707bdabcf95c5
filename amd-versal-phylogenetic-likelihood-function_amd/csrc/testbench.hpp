// testbench.hpp -- instance sizing, partitioning and packing of the reference
// host program, restated with 64-bit sizes.
//
//   sizing/partition   app/src/include.h:150-266 (testbench_info)
//   instance offsets   app/src/host_mem.cpp:229,290-291 (k * n0 sites)
//   packing            app/src/host_mem.cpp:221-243
//
// Used by the C ABI (plfx_tb_*, plfx_pack_instance) and by the C++ host driver.
#pragma once
#include <cstdint>
#include <cstring>
#include <random>

namespace plfx {

// The reference's split of `total` items over `parts` instances
// (include.h:181-189, offsets host_mem.cpp:229,290-291): n0 = ceil(total /
// parts), part k starts at k*n0, the last part is short by n0*parts - total.
// Used for sites over accelerator instances and for independent nodes over
// ranks.  Returns false where the reference's arithmetic underflows (the
// padding reaches a whole share, e.g. 10 items over 8 parts).
inline bool shard(uint64_t total, uint32_t parts, uint32_t k, uint64_t *offset, uint64_t *count) {
  if (parts == 0 || k >= parts) return false;
  const uint64_t n0 = (total + parts - 1) / parts;
  const uint64_t pad = n0 * parts - total;
  if (parts > 1 && total > 0 && pad >= n0) return false;
  *offset = (uint64_t)k * n0;
  *count = total == 0 ? 0 : n0 - (k == parts - 1 ? pad : 0);
  return true;
}

// host_mem.cpp:179-209 input protocol with a fixed seed (the reference seeds
// from std::random_device): std::mt19937 +
// std::uniform_real_distribution<double>(0, 1); EV[16]; left/right P
// interleaved; then the CLVs interleaved element by element, the left CLV x1e-12
// on the first 16 of every 64 elements (every 4th site scales); wgt = 1.
template <typename T>
void gen_hostmem(uint32_t seed, uint64_t n, T *ev, T *left, T *right, T *x1, T *x2, int32_t *wgt) {
  std::mt19937 gen(seed);
  std::uniform_real_distribution<> dis(0.0, 1.0);
  for (int j = 0; j < 16; j++) ev[j] = (T)dis(gen);
  for (int j = 0; j < 64; j++) {
    left[j] = (T)dis(gen);
    right[j] = (T)dis(gen);
  }
  for (uint64_t j = 0; j < 16 * n; j++) {
    const double scale = (j % 64 < 16) ? 1.0e-12 : 1.0;
    x1[j] = (T)(dis(gen) * scale);
    x2[j] = (T)dis(gen);
  }
  if (wgt)
    for (uint64_t j = 0; j < n; j++) wgt[j] = 1;
}

enum Layout : int { COMBINED = 0, SEPARATE = 1 };  // include.h:20
enum Aie : int { STREAM = 0, WINDOW = 1 };         // include.h:21

struct Testbench {
  uint64_t alignment_sites = 0;
  uint32_t parallel_instances = 1;
  uint32_t window_size = 1024;  // include.h:155
  int layout = SEPARATE;
  int aie_type = WINDOW;
  static constexpr uint64_t elements_per_alignment = 16;  // include.h:153

  uint64_t alignments_per_window() const { return window_size >> 4; }
  // ceil(N / P) (include.h:184-186)
  uint64_t alignments_per_instance() const {
    return (alignment_sites + parallel_instances - 1) / parallel_instances;
  }
  // the last instance is short by the padding (include.h:181-183)
  uint64_t alignments_per_instance(uint32_t k) const {
    return alignments_per_instance() - (k == parallel_instances - 1 ? alignments_padding() : 0);
  }
  uint64_t alignments_padding() const {
    return alignments_per_instance() * parallel_instances - alignment_sites;
  }
  uint64_t alignmentelements_per_instance(uint32_t k) const {
    return alignments_per_instance(k) * elements_per_alignment;
  }
  // instance k starts at k * n0 sites (host_mem.cpp:229)
  uint64_t instance_site_offset(uint32_t k) const { return (uint64_t)k * alignments_per_instance(0); }
  uint64_t stream_padding() const { return alignment_sites & 1; }  // include.h:259-261
  uint64_t num_windows_per_instance() const {                      // include.h:262-266
    const uint64_t apw = alignments_per_window();
    if (apw == 0) return 0;
    const uint64_t full = alignments_per_instance() / apw;
    return full + ((alignments_per_instance() - full * apw) > 0);
  }
  uint64_t elements_per_instance() const {  // include.h:247-258
    const uint64_t r = aie_type == STREAM ? alignments_per_instance() + stream_padding()
                                          : num_windows_per_instance() * alignments_per_window();
    return r * elements_per_alignment;
  }
  uint64_t header_left() const { return 5 * 16; }                              // [EV|P_L]
  uint64_t header_right() const { return layout == SEPARATE ? 4 * 16 : 5 * 16; }  // [P_R] / [EV|P_R]
  uint64_t instance_elements_left() const { return elements_per_instance() + header_left(); }
  uint64_t instance_elements_right() const { return elements_per_instance() + header_right(); }
  uint64_t instance_elements_out() const { return elements_per_instance(); }
  uint64_t instance_active_elements_left(uint32_t k) const {
    return alignmentelements_per_instance(k) + header_left();
  }
  uint64_t instance_active_elements_right(uint32_t k) const {
    return alignmentelements_per_instance(k) + header_right();
  }

  // host_mem.cpp:221-243 for element type T; zero-fills the padded tail.
  template <typename T>
  void pack(uint32_t k, const T *EV, const T *left, const T *right, const T *x1, const T *x2,
            T *outL, T *outR) const {
    const uint64_t nl = instance_elements_left(), nr = instance_elements_right();
    std::memset(outL, 0, nl * sizeof(T));
    std::memset(outR, 0, nr * sizeof(T));
    const uint64_t off = instance_site_offset(k) * elements_per_alignment;
    const uint64_t cnt = alignmentelements_per_instance(k);
    std::memcpy(outL, EV, 16 * sizeof(T));
    std::memcpy(outL + 16, left, 64 * sizeof(T));
    std::memcpy(outL + 80, x1 + off, cnt * sizeof(T));
    if (layout == COMBINED) {
      std::memcpy(outR, EV, 16 * sizeof(T));
      std::memcpy(outR + 16, right, 64 * sizeof(T));
      std::memcpy(outR + 80, x2 + off, cnt * sizeof(T));
    } else {
      std::memcpy(outR, right, 64 * sizeof(T));
      std::memcpy(outR + 64, x2 + off, cnt * sizeof(T));
    }
  }
};

}  // namespace plfx
