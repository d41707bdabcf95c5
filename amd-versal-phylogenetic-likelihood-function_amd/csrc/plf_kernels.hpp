// plf_kernels.hpp -- launchers of the fused PLF kernels (internal to libplfx).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace plfx {

// Self-resetting workspace of the in-kernel scaler-sum reduction
// (plf_dna.hpp block_ticket_sum): kWsWords 64-bit words, zero at rest.
constexpr int kWsWords = (32 + 1) * 16;

struct DnaArgs {
  const void *x1, *x2;
  void *x3;
  const void *EV, *left, *right;
  const int32_t *wgt;       // may be null (weights = 1)
  uint8_t *scaler;          // may be null
  int64_t *scaler_sum;      // may be null
  unsigned long long *ws;   // ticket words (needed iff scaler_sum); the f64 protein FMA
                            // launch also takes its tile queue from ws + kWsWords when
                            // non-null (2 x kWsWords words, zero at rest)
  int64_t n;
  int segments = -1;        // node kernels' XCD-segmented site mapping: -1 by size, 0 off,
                            // 1 on (plf_kernels.hip use_segments; PLFX_NODE_SEGMENTS)
  int streams = 1;          // one-node calls the caller keeps in flight (plfx_ctx_set_streams):
                            // the dense DNA node kernels and the protein FMA kernels
                            // take the co-resident blocks / streams
};

// Fused DNA (4 states x 4 Gamma categories) inner-node update.
// Returns the hipError_t of the launch.
hipError_t launch_plf_dna_f32(const DnaArgs &a, int max_blocks, hipStream_t s);
hipError_t launch_plf_dna_f64(const DnaArgs &a, int max_blocks, hipStream_t s);

// sum_j scaler[j]*wgt[j] (host_mem.cpp:384-388), self-resetting ws as above.
// Protein (S=20, C=4) kernel; fma selects fused multiply-add.
hipError_t launch_plf_prot(int dtype, bool fma, const DnaArgs &a, int max_blocks, hipStream_t s,
                           int tips = 0, const void *tipvec = nullptr);
// Protein f64 in FMA mode on the VALU with LDS-tiled matrices (plf_prot_valu.hip,
// PLFX_FMA | PLFX_VALU): bit-identical to the matrix-core FMA kernel, dense
// children, one node.
hipError_t launch_plf_prot_valu_f64(const DnaArgs &a, int max_blocks, hipStream_t s);
// Protein f64 in exact mode with the matrices as scalar operands
// (plf_prot_valu_exact.hip): bit-identical to the LDS-matrix exact kernel.
hipError_t launch_plf_prot_valu_exact_f64(const DnaArgs &a, int max_blocks, hipStream_t s);

// Batched nodes (<= kMaxBatch per launch) sharing EV, n, wgt.  dtype: 0 f32, 1 f64.
// tips: 0 dense children; 1 x1 of every node is a tip (uint8 state codes);
// 2 x1 and x2 are tips.  tipvec: 16 x 4 tip vectors of dtype (NULL = 0/1 bits).
struct NodeDescH {
  const void *x1, *x2;
  void *x3;
  const void *left, *right;
  uint8_t *scaler;
  int64_t *scaler_sum;
};
constexpr int kMaxBatch = 32;
hipError_t launch_plf_dna_batch(int dtype, const NodeDescH *nodes, int count, const void *EV,
                                const int32_t *wgt, int64_t n, unsigned long long *ws,
                                int max_blocks, hipStream_t s, int tips = 0,
                                const void *tipvec = nullptr, int share = 1);
// Tip/tip protein nodes from their 576-combination tables (plf_prot.hpp
// prot_tiptip_gather_kernel): x3 / scaler / sum of each node gathered by code pair.
struct ProtGatherDescH {
  const uint8_t *c1, *c2;
  void *x3;
  uint8_t *scaler;
  int64_t *scaler_sum;
  const void *tab;
  const uint8_t *tsc;
};
constexpr int kProtCombos = 24 * 24;
hipError_t launch_prot_tiptip_gather(int dtype, const ProtGatherDescH *d, int count, const int32_t *wgt,
                                     int64_t n, unsigned long long *ws, int max_blocks, hipStream_t s);

// Protein nodes (f64, f32; FMA or exact) whose two children are tip/tip nodes held in
// combination tables (plf_prot.hpp ProtTabDesc), batched as above.
struct ProtTabDescH {
  const void *tab1, *tab2;
  const uint8_t *c1a, *c1b, *c2a, *c2b;
  void *x3;
  const void *left, *right;
  uint8_t *scaler;
  int64_t *scaler_sum;
};
hipError_t launch_prot_tab_batch(int dtype, bool fma, const ProtTabDescH *d, int count, const void *EV,
                                 const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                                 hipStream_t s);

// Protein (S = 20) nodes batched the same way; fma as launch_plf_prot.
hipError_t launch_plf_prot_batch(int dtype, bool fma, const NodeDescH *nodes, int count, const void *EV,
                                 const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                                 hipStream_t s, int tips, const void *tipvec);

// Root log-likelihood; partials: >= kLnlMaxGrid doubles; ticket: kWsWords u64 (zero at rest).
constexpr int kLnlMaxGrid = 4096;
hipError_t launch_root_lnl(int dtype, int states, const void *x, int64_t n, const double *catw,
                           const double *freq, const int32_t *wgt, const int64_t *scaler_sums,
                           int nsums, double *partials, unsigned long long *ticket, double *out,
                           double *site_lnl, hipStream_t s);

hipError_t launch_scaler_sum(const uint8_t *scaler, const int32_t *wgt, int64_t n,
                             int64_t *out, unsigned long long *ws, int max_blocks,
                             hipStream_t s);

// P matrices from an eigensystem (plf_pmat.hpp).  dtype 0 f32 / 1 f64.
hipError_t launch_pmatrix(int dtype, bool eigen_conv, const double *eigen, int S,
                          const double *rates, int ncat, const double *blen, int64_t nbranch,
                          void *out, hipStream_t s);

// Fused level pairs (plf_dna.hpp TripleDesc), dtype 0 f32 / 1 f64; <= kMaxTriples per
// launch, ws >= 3 * count regions.  tips as plf_dna_f64_triple_kernel's kTips.
struct TripleDescH {
  const void *a1, *a2, *b1, *b2;
  void *xa, *xb, *xp;
  const double *la, *ra, *lb, *rb, *lp, *rp;
  uint8_t *sa, *sb, *sp;
  int64_t *ssa, *ssb, *ssp;
};
constexpr int kMaxTriples = 10;
hipError_t launch_plf_dna_triples(int dtype, const TripleDescH *t, int count, const void *EV,
                                  const int32_t *wgt, int64_t n, unsigned long long *ws,
                                  int max_blocks, hipStream_t s, int tips, const void *tipvec);

// Fused three-level subtrees (plf_dna.hpp SeptetDesc), dtype 0 f32 / 1 f64; <= kMaxSeptets
// per launch, ws >= 7 * count regions.  tips as plf_dna_f64_septet_kernel's kTips.
struct SeptetDescH {
  const void *g[8];
  void *x[7];
  const void *mat[14];
  uint8_t *sc[7];
  int64_t *ss[7];
};
constexpr int kMaxSeptets = 8;
hipError_t launch_plf_dna_septets(int dtype, const SeptetDescH *t, int count, const void *EV,
                                  const int32_t *wgt, int64_t n, unsigned long long *ws,
                                  int max_blocks, hipStream_t s, int tips, const void *tipvec);

// Fused complete subtree of depth 4..6 (plf_dna.hpp DeepDesc: 2^depth leaves,
// 2^depth - 1 nodes in heap order by level), dtype 0 f32 / 1 f64, one per
// launch, ws >= 2^depth - 1 regions.  tips: 0 dense leaves; 2 every leaf a tip
// (uint8 state codes), tipvec as launch_plf_dna_batch's.
struct DeepDescH {
  const void *g[64];
  void *x[63];
  const void *mat[126];
  uint8_t *sc[63];
  int64_t *ss[63];
};
constexpr int kDeepNodes = 63;
// the deep passes' chunk queue: this region of the stream workspace (plf_dna.hpp WaveQueue)
constexpr int kDeepQueueRegion = 63;
hipError_t launch_plf_dna_deep(int dtype, int depth, const DeepDescH *t, const void *EV,
                               const int32_t *wgt, int64_t n, unsigned long long *ws, int max_blocks,
                               hipStream_t s, int tips = 0, const void *tipvec = nullptr);

}  // namespace plfx
