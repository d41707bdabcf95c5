// swemu.cpp -- the sw_emu target: one accelerator instance emulated on the
// host, as its dataflow (BASELINE configs[0]; the reference's TARGET=sw_emu,
// Makefile:199-220, host_mem.cpp:160-164).  Host-only code; include/plfx.h
// section (5b).
//
// Per window (window PLIO) or once (stream PLIO):
//   mm2sleft / mm2sright    hls/src/mm2s{left,right}_memDNAwindow{Comb,Sep}.cpp,
//                           mm2sleft_memDNAstreamComb.cpp: header words -> EV
//                           half + transposed P_c (transpose.cpp:6-24) per lane,
//                           then each 512-bit site word split into 4 lane beats
//                           (lane c = category c, bits 128c..128c+127)
//   AIE lane c              mmul_branch x2 (aie/.../kernels/mmul_branch.cpp:6-41:
//                           2 sites x 4 states times P^T per iteration, EV half
//                           passed through), combine (combine.cpp:4-39: EV
//                           reassembled from the halves, L (.) R), ev (ev.cpp:4-27)
//   s2mm                    hls/src/s2mm_memDNAwindowComb.cpp:45-99: lane beats
//                           -> 16 values, all |x| < 2^-32 and slot < n -> x 2^32,
//                           char scaler
// Lane traffic goes through FIFOs of 128-bit beats exactly as the PLIOs carry
// it, so the framing (header beats, window padding, the stream count beat
// and odd-count pad) is exercised, not assumed.  The arithmetic of each lane
// stage uses plf()'s operation order (app/src/plf.cpp:29-50: ump from +0.0
// over ascending l, x3 from +0.0 over ascending k; no FMA contraction, this
// file is built with -ffp-contract=off), so the results equal plf()'s and the
// GPU kernels' bit for bit.  Only alignment_sites CLVs / scaler bytes are
// stored, as plfx_instance_run does.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/plfx.h"

namespace {

template <typename T>
struct Beat {  // one 128-bit PLIO beat (4 values of the element type)
  T v[4];
};

template <typename T>
struct Fifo {  // an AXI stream / PLIO: written in order, read in order
  std::vector<Beat<T>> q;
  size_t rd = 0;
  void put(const T *p) {
    Beat<T> b;
    std::memcpy(b.v, p, sizeof b.v);
    q.push_back(b);
  }
  const Beat<T> &get() { return q[rd++]; }  // the caller reads what the producer wrote
  bool drained() const { return rd == q.size(); }
  void clear() {
    q.clear();
    rd = 0;
  }
};

// transpose.cpp:6-24: element i*4+j -> j*4+i of one 512-bit word
template <typename T>
void transpose16(const T *in, T *out) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) out[j * 4 + i] = in[i * 4 + j];
}

// One side's mover (mm2sleft or mm2sright) over its packed instance buffer.
template <typename T>
struct Mover {
  const T *mem;
  bool has_ev;      // COMBINED buffers and the SEPARATE left buffer start with EV
  bool left;        // left side sends EV rows 0-1, right side rows 2-3
  T branch[4][16];  // P_c^T per lane, transposed once at kernel start
  uint64_t data_word;

  Mover(const T *m, bool is_left, int layout) : mem(m), left(is_left) {
    has_ev = is_left || layout == PLFX_LAYOUT_COMBINED;
    const uint64_t pbase = has_ev ? 1 : 0;
    for (int c = 0; c < 4; c++) transpose16(mem + 16 * (pbase + c), branch[c]);
    data_word = pbase + 4;
  }
  const T *word(uint64_t i) const { return mem + 16 * i; }
  // the EV half this side sends in a lane header (2 beats)
  void ev_half(Fifo<T> &f) const {
    const T *ev = word(0);
    f.put(ev + (left ? 0 : 8));
    f.put(ev + (left ? 4 : 12));
  }
  void branch_beats(Fifo<T> &f, int c) const {
    for (int j = 0; j < 4; j++) f.put(branch[c] + 4 * j);
  }
  // sites [first, first + count) of the data region, one beat per lane each
  void sites(Fifo<T> (&lane)[4], uint64_t first, uint64_t count) const {
    for (uint64_t i = 0; i < count; i++) {
      const T *w = word(data_word + first + i);
      for (int c = 0; c < 4; c++) lane[c].put(w + 4 * c);
    }
  }
};

// AIE mmul_branch on one lane: [EV half passthrough] [P^T 4 beats, or from a
// side stream] then `slots` sites in 2-site blocks: out[s][k] = sum_l
// data[s][l] * Bt[l][k] (Bt = P^T as streamed, so Bt[l][k] = P_c[k][l]).
template <typename T>
void mmul_branch(Fifo<T> &in, Fifo<T> *side_branch, bool passthrough_ev, uint64_t slots,
                 Fifo<T> &out) {
  if (passthrough_ev) {
    out.put(in.get().v);
    out.put(in.get().v);
  }
  T Bt[16];
  Fifo<T> &bsrc = side_branch ? *side_branch : in;
  for (int j = 0; j < 4; j++) std::memcpy(Bt + 4 * j, bsrc.get().v, 4 * sizeof(T));
  for (uint64_t s = 0; s < slots; s++) {
    const T *x = in.get().v;
    T u[4];
    for (int k = 0; k < 4; k++) {
      T acc = T(0);  // plf.cpp:31-39 order: from +0.0, ascending l
      for (int l = 0; l < 4; l++) acc += x[l] * Bt[l * 4 + k];
      u[k] = acc;
    }
    out.put(u);
  }
}

// AIE combine + ev on one lane: EV = [left half | right half] (Comb, from the
// two mmul_branch passthroughs) or from the EV side stream (Sep); p = uL * uR;
// x3[s][l] = sum_k p[s][k] * EV[k][l] (row-major EV, ev.cpp:11-26).
template <typename T>
void combine_ev(Fifo<T> &L, Fifo<T> &R, const T *ev_side, uint64_t slots, Fifo<T> &out) {
  T EV[16];
  if (ev_side) {
    std::memcpy(EV, ev_side, sizeof EV);
  } else {
    std::memcpy(EV + 0, L.get().v, 4 * sizeof(T));
    std::memcpy(EV + 4, L.get().v, 4 * sizeof(T));
    std::memcpy(EV + 8, R.get().v, 4 * sizeof(T));
    std::memcpy(EV + 12, R.get().v, 4 * sizeof(T));
  }
  for (uint64_t s = 0; s < slots; s++) {
    const T *a = L.get().v, *b = R.get().v;
    T p[4], o[4];
    for (int k = 0; k < 4; k++) p[k] = a[k] * b[k];
    for (int l = 0; l < 4; l++) o[l] = T(0);
    for (int k = 0; k < 4; k++)  // plf.cpp:45-50 order: from +0.0, ascending k
      for (int l = 0; l < 4; l++) o[l] += p[k] * EV[4 * k + l];
    out.put(o);
  }
}

// s2mm: `slots` beats per lane from slot index `first` on; slots >= n are
// padding (never scaled, never stored).
template <typename T>
void s2mm(Fifo<T> (&lane)[4], uint64_t first, uint64_t slots, uint64_t n, T *out, uint8_t *sc) {
  const double minlik = 1.0 / 4294967296.0;
  for (uint64_t s = 0; s < slots; s++) {
    T x3[16];
    for (int c = 0; c < 4; c++) std::memcpy(x3 + 4 * c, lane[c].get().v, 4 * sizeof(T));
    const uint64_t slot = first + s;
    bool scale = slot < n;
    for (int l = 0; l < 16 && scale; l++) scale = std::fabs((double)x3[l]) < minlik;
    if (scale)
      for (int l = 0; l < 16; l++) x3[l] = (T)(x3[l] * 4294967296.0);
    if (slot < n) {
      std::memcpy(out + 16 * slot, x3, sizeof x3);
      if (sc) sc[slot] = scale ? 1 : 0;
    }
  }
}

template <typename T>
int run(const T *inL, const T *inR, T *out, uint8_t *sc, uint64_t n, uint32_t window_size,
        int layout, int aie) {
  const Mover<T> ml(inL, true, layout), mr(inR, false, layout);
  Fifo<T> lane_l[4], lane_r[4], side_bl[4], side_br[4], ul[4], ur[4], o[4];
  if (aie == PLFX_AIE_STREAM) {
    // mm2sleft_memDNAstreamComb.cpp:44-114: count beat, EV half, P^T, the n
    // sites, one zero site if n is odd (the AIE reads sites in pairs)
    const uint64_t pad = n & 1, slots = n + pad;
    const T zero[4] = {T(0), T(0), T(0), T(0)};
    for (const Mover<T> *m : {&ml, &mr}) {
      Fifo<T>(&lane)[4] = m == &ml ? lane_l : lane_r;
      T cnt[4] = {(T)(float)slots, T(0), T(0), T(0)};  // the count travels as a float (Q7)
      for (int c = 0; c < 4; c++) {
        lane[c].put(cnt);
        m->ev_half(lane[c]);
        m->branch_beats(lane[c], c);
      }
      m->sites(lane, 0, n);
      if (pad)
        for (int c = 0; c < 4; c++) lane[c].put(zero);
    }
    for (int c = 0; c < 4; c++) {
      // mmul_branch (stream): the count beat sets the iteration count
      const uint64_t it_l = (uint64_t)lane_l[c].get().v[0], it_r = (uint64_t)lane_r[c].get().v[0];
      if (it_l != slots || it_r != slots) return PLFX_ERR_INVALID;
      mmul_branch<T>(lane_l[c], nullptr, true, slots, ul[c]);
      mmul_branch<T>(lane_r[c], nullptr, true, slots, ur[c]);
      combine_ev<T>(ul[c], ur[c], nullptr, slots, o[c]);
    }
    s2mm(o, 0, slots, n, out, sc);
    return PLFX_OK;
  }
  const uint64_t apw = window_size >> 4;  // sites per window (mm2sleft:45)
  const uint64_t nwin = n / apw + (n % apw ? 1 : 0);
  const T *ev_full = inL;  // Sep: EV goes to the combine stage on its side stream
  for (uint64_t w = 0; w < nwin; w++) {
    for (Fifo<T> *f : {lane_l, lane_r, side_bl, side_br, ul, ur, o})
      for (int c = 0; c < 4; c++) f[c].clear();
    for (int c = 0; c < 4; c++) {
      if (layout == PLFX_LAYOUT_COMBINED) {  // header beats in front of every window
        ml.ev_half(lane_l[c]);
        ml.branch_beats(lane_l[c], c);
        mr.ev_half(lane_r[c]);
        mr.branch_beats(lane_r[c], c);
      } else {  // Sep: P^T on side streams, once per window
        ml.branch_beats(side_bl[c], c);
        mr.branch_beats(side_br[c], c);
      }
    }
    ml.sites(lane_l, w * apw, apw);  // whole windows: padded slots are read too
    mr.sites(lane_r, w * apw, apw);
    const bool comb = layout == PLFX_LAYOUT_COMBINED;
    for (int c = 0; c < 4; c++) {
      mmul_branch<T>(lane_l[c], comb ? nullptr : &side_bl[c], comb, apw, ul[c]);
      mmul_branch<T>(lane_r[c], comb ? nullptr : &side_br[c], comb, apw, ur[c]);
      combine_ev<T>(ul[c], ur[c], comb ? nullptr : ev_full, apw, o[c]);
      if (!lane_l[c].drained() || !lane_r[c].drained()) return PLFX_ERR_INVALID;
    }
    s2mm(o, w * apw, apw, n, out, sc);
  }
  return PLFX_OK;
}

}  // namespace

extern "C" int plfx_swemu_instance_run(const void *in_left, const void *in_right, void *out_clv,
                                       uint8_t *out_scaler, uint32_t alignment_sites,
                                       uint32_t window_size, int layout, int aie_type, int dtype) {
  if (!in_left || !in_right || (alignment_sites > 0 && !out_clv)) return PLFX_ERR_INVALID;
  if (layout != PLFX_LAYOUT_COMBINED && layout != PLFX_LAYOUT_SEPARATE) return PLFX_ERR_INVALID;
  if (aie_type == PLFX_AIE_WINDOW) {
    if (window_size < 32 || window_size % 32) return PLFX_ERR_INVALID;  // 2-site AIE blocks
  } else if (aie_type == PLFX_AIE_STREAM) {
    if (layout != PLFX_LAYOUT_COMBINED) return PLFX_ERR_INVALID;  // stream movers are Comb only
  } else {
    return PLFX_ERR_INVALID;
  }
  if (alignment_sites == 0) return PLFX_OK;
  if (dtype == PLFX_F32)
    return run<float>((const float *)in_left, (const float *)in_right, (float *)out_clv, out_scaler,
                      alignment_sites, window_size, layout, aie_type);
  if (dtype == PLFX_F64)
    return run<double>((const double *)in_left, (const double *)in_right, (double *)out_clv,
                       out_scaler, alignment_sites, window_size, layout, aie_type);
  return PLFX_ERR_INVALID;
}
