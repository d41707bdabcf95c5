// testbench_api.cpp -- C ABI for the instance sizing / packing of the
// reference host (include/plfx.h section 5; app/src/include.h:150-266,
// app/src/host_mem.cpp:221-243).  Host-only code.
#include "../../include/plfx.h"
#include "testbench.hpp"

namespace {
plfx::Testbench to_tb(const plfx_testbench *t) {
  plfx::Testbench tb;
  tb.alignment_sites = t->alignment_sites;
  tb.parallel_instances = t->parallel_instances ? t->parallel_instances : 1;
  tb.window_size = t->window_size;
  tb.layout = t->layout;
  tb.aie_type = t->aie_type;
  return tb;
}
}  // namespace

extern "C" {

uint64_t plfx_tb_alignments_per_instance(const plfx_testbench *t, int k) {
  if (!t) return 0;
  plfx::Testbench tb = to_tb(t);
  return k < 0 ? tb.alignments_per_instance() : tb.alignments_per_instance((uint32_t)k);
}
uint64_t plfx_tb_alignments_padding(const plfx_testbench *t) {
  return t ? to_tb(t).alignments_padding() : 0;
}
uint64_t plfx_tb_instance_site_offset(const plfx_testbench *t, int k) {
  return (t && k >= 0) ? to_tb(t).instance_site_offset((uint32_t)k) : 0;
}
uint64_t plfx_tb_elements_per_instance(const plfx_testbench *t) {
  return t ? to_tb(t).elements_per_instance() : 0;
}
uint64_t plfx_tb_instance_elements_left(const plfx_testbench *t) {
  return t ? to_tb(t).instance_elements_left() : 0;
}
uint64_t plfx_tb_instance_elements_right(const plfx_testbench *t) {
  return t ? to_tb(t).instance_elements_right() : 0;
}
uint64_t plfx_tb_instance_elements_out(const plfx_testbench *t) {
  return t ? to_tb(t).instance_elements_out() : 0;
}
uint64_t plfx_tb_instance_active_elements_left(const plfx_testbench *t, int k) {
  return (t && k >= 0) ? to_tb(t).instance_active_elements_left((uint32_t)k) : 0;
}
uint64_t plfx_tb_instance_active_elements_right(const plfx_testbench *t, int k) {
  return (t && k >= 0) ? to_tb(t).instance_active_elements_right((uint32_t)k) : 0;
}
uint64_t plfx_tb_num_windows_per_instance(const plfx_testbench *t) {
  return t ? to_tb(t).num_windows_per_instance() : 0;
}

int plfx_pack_instance(const plfx_testbench *t, int k, int dtype, const void *EV, const void *left,
                       const void *right, const void *x1, const void *x2, void *outL, void *outR) {
  if (!t || k < 0 || (uint32_t)k >= (t->parallel_instances ? t->parallel_instances : 1) || !EV ||
      !left || !right || !x1 || !x2 || !outL || !outR)
    return PLFX_ERR_INVALID;
  if (t->layout != PLFX_LAYOUT_COMBINED && t->layout != PLFX_LAYOUT_SEPARATE) return PLFX_ERR_INVALID;
  plfx::Testbench tb = to_tb(t);
  if (tb.aie_type == plfx::WINDOW && tb.alignments_per_window() == 0) return PLFX_ERR_INVALID;
  if (dtype == PLFX_F32)
    tb.pack<float>((uint32_t)k, (const float *)EV, (const float *)left, (const float *)right,
                   (const float *)x1, (const float *)x2, (float *)outL, (float *)outR);
  else if (dtype == PLFX_F64)
    tb.pack<double>((uint32_t)k, (const double *)EV, (const double *)left, (const double *)right,
                    (const double *)x1, (const double *)x2, (double *)outL, (double *)outR);
  else
    return PLFX_ERR_INVALID;
  return PLFX_OK;
}

int plfx_shard(uint64_t total, uint32_t parts, uint32_t k, uint64_t *offset, uint64_t *count) {
  if (!offset || !count) return PLFX_ERR_INVALID;
  return plfx::shard(total, parts, k, offset, count) ? PLFX_OK : PLFX_ERR_INVALID;
}

int plfx_gen_hostmem(int dtype, uint32_t seed, uint64_t n, void *EV, void *left, void *right,
                     void *x1, void *x2, int32_t *wgt) {
  if (!EV || !left || !right || (n > 0 && (!x1 || !x2))) return PLFX_ERR_INVALID;
  if (dtype == PLFX_F32)
    plfx::gen_hostmem<float>(seed, n, (float *)EV, (float *)left, (float *)right, (float *)x1,
                             (float *)x2, wgt);
  else if (dtype == PLFX_F64)
    plfx::gen_hostmem<double>(seed, n, (double *)EV, (double *)left, (double *)right,
                              (double *)x1, (double *)x2, wgt);
  else
    return PLFX_ERR_INVALID;
  return PLFX_OK;
}

}  // extern "C"
