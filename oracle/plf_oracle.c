/*
 * plf_oracle.c -- CPU restatement of the reference PLF hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libplfx, the HIP kernels,
 * the host driver) links, loads or calls this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
 * as the checker / the timed CPU baseline, never as the thing measured.
 *
 * Written from the semantics of the reference, not copied from it:
 *
 *   plf()            /root/reference/app/src/plf.cpp:8-68
 *                    - x[site*16 + cat*4 + state]                (plf.cpp:21-23)
 *                    - ump[k] = sum_l x[c*4+l]*P[c*16+k*4+l], accumulated
 *                      from 0.0 in ascending l                    (plf.cpp:31-39)
 *                    - prod[k] = umpL[k]*umpR[k]                  (plf.cpp:41)
 *                    - x3[c*4+l] = 0 + sum_k prod[k]*EV[4k+l],
 *                      ascending k                                (plf.cpp:25-27,45-50)
 *                    - scale iff every |x3| < 2^-32 (strict, NaN -> no scale),
 *                      then x3 *= 2^32 and addScale += wgt[i]      (plf.cpp:4-6,53-64)
 *   s2mm scaler byte /root/reference/hls/src/s2mm_memDNAwindowComb.cpp:70-97
 *                    (char 0/1 per site; the host sums char*wgt,
 *                     app/src/host_mem.cpp:384-388)
 *   input protocol   /root/reference/app/src/host_mem.cpp:179-209
 *                    (std::mt19937 + std::uniform_real_distribution<double>(0,1),
 *                     EV[16], then left/right P interleaved, then the CLVs
 *                     interleaved left/right with the left CLV x1e-12 on the first
 *                     16 of every 64 elements, i.e. every 4th site; wgt = 1)
 *
 * Parity pin: the float instantiation is checked bit-for-bit against the
 * reference plf() itself, compiled from /root/reference by oracle/Makefile into
 * oracle/_ref/ (tests/test_oracle.py), against the reference's AIE golden
 * vectors aie/data/golden{0..3}.txt, and against committed fixtures
 * (tests/golden/) that were produced by that reference build.
 * The double, the generic S-state (protein) and the tree/lnL routines are
 * extensions that the reference does not have: "parity unpinned" beyond being
 * the same loop as the pinned float instantiation.
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math (no FMA contraction, SSE
 * float arithmetic: the same rounding sequence as the reference's -O0 x86-64
 * build).
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PLFO_TWO_TO_32 4294967296.0
#define PLFO_MINLIK (1.0 / PLFO_TWO_TO_32)

/* ------------------------------------------------------------------------ */
/* DNA (4 states x 4 Gamma categories) inner-inner update, plf.cpp:19-65     */
/* ------------------------------------------------------------------------ */
#define PLFO_DNA_SITE(T, x1, x2, x3, EV, left, right, scale_out)                   \
  do {                                                                             \
    int j_, k_, l_;                                                                \
    T p_[4];                                                                       \
    for (j_ = 0; j_ < 16; j_++) x3[j_] = (T)0.0;                                   \
    for (j_ = 0; j_ < 4; j_++) {                                                   \
      for (k_ = 0; k_ < 4; k_++) {                                                 \
        T u1_ = (T)0.0, u2_ = (T)0.0;                                              \
        for (l_ = 0; l_ < 4; l_++) {                                               \
          u1_ += x1[j_ * 4 + l_] * left[j_ * 16 + k_ * 4 + l_];                    \
          u2_ += x2[j_ * 4 + l_] * right[j_ * 16 + k_ * 4 + l_];                   \
        }                                                                          \
        p_[k_] = u1_ * u2_;                                                        \
      }                                                                            \
      for (k_ = 0; k_ < 4; k_++)                                                   \
        for (l_ = 0; l_ < 4; l_++) x3[j_ * 4 + l_] += p_[k_] * EV[4 * k_ + l_];    \
    }                                                                              \
    scale_out = 1;                                                                 \
    for (l_ = 0; scale_out && l_ < 16; l_++)                                       \
      scale_out = (fabs((double)x3[l_]) < PLFO_MINLIK);                            \
    if (scale_out)                                                                 \
      for (l_ = 0; l_ < 16; l_++) x3[l_] = (T)((double)x3[l_] * PLFO_TWO_TO_32);   \
  } while (0)

#define PLFO_DEFINE_DNA(SUFFIX, T)                                                 \
  void plfo_plf_##SUFFIX(const T *x1s, const T *x2s, T *x3s, const T *EV,          \
                         long long n, const T *left, const T *right,               \
                         const int *wgt, int *scalerIncrement,                     \
                         unsigned char *scaler) {                                  \
    long long i;                                                                   \
    int addScale = 0;                                                              \
    for (i = 0; i < n; i++) {                                                      \
      const T *x1 = x1s + i * 16;                                                  \
      const T *x2 = x2s + i * 16;                                                  \
      T *x3 = x3s + i * 16;                                                        \
      int sc;                                                                      \
      PLFO_DNA_SITE(T, x1, x2, x3, EV, left, right, sc);                           \
      if (scaler) scaler[i] = (unsigned char)sc;                                   \
      if (sc) addScale += wgt ? wgt[i] : 1;                                        \
    }                                                                              \
    if (scalerIncrement) *scalerIncrement = addScale;                              \
  }                                                                                \
  /* OpenMP variant (static site split) used only as the multi-core CPU         \
   * baseline; per-site results are identical to the serial loop. */            \
  void plfo_plf_##SUFFIX##_omp(const T *x1s, const T *x2s, T *x3s, const T *EV,    \
                               long long n, const T *left, const T *right,         \
                               const int *wgt, int *scalerIncrement,               \
                               unsigned char *scaler, int threads) {               \
    long long i;                                                                   \
    long long addScale = 0;                                                        \
    (void)threads;                                                                 \
    _Pragma("omp parallel for schedule(static) reduction(+:addScale) num_threads(threads)") \
    for (i = 0; i < n; i++) {                                                      \
      const T *x1 = x1s + i * 16;                                                  \
      const T *x2 = x2s + i * 16;                                                  \
      T *x3 = x3s + i * 16;                                                        \
      int sc;                                                                      \
      PLFO_DNA_SITE(T, x1, x2, x3, EV, left, right, sc);                           \
      if (scaler) scaler[i] = (unsigned char)sc;                                   \
      if (sc) addScale += wgt ? wgt[i] : 1;                                        \
    }                                                                              \
    if (scalerIncrement) *scalerIncrement = (int)addScale;                         \
  }

PLFO_DEFINE_DNA(f32, float)
PLFO_DEFINE_DNA(f64, double)

/* ------------------------------------------------------------------------ */
/* Generic S states x C categories (protein S=20).  Extension: the reference */
/* hard-wires S=C=4.  Same loop nest and accumulation order as plf.cpp with  */
/* 4 replaced by S / C; for S=C=4 it reproduces plfo_plf_f64 bit-for-bit.   */
/* Layouts: x[site][c][s], P[c][k][l] (S*S per category), EV[k][l].         */
/* ------------------------------------------------------------------------ */
#define PLFO_DEFINE_GEN(SUFFIX, T)                                                 \
  void plfo_plf_gen_##SUFFIX(int S, int C, const T *x1s, const T *x2s, T *x3s,     \
                             const T *EV, long long n, const T *left,              \
                             const T *right, const int *wgt,                       \
                             long long *scalerIncrement, unsigned char *scaler) {  \
    long long i, addScale = 0;                                                     \
    T p[64];                                                                       \
    const int V = S * C;                                                           \
    for (i = 0; i < n; i++) {                                                      \
      const T *x1 = x1s + i * V;                                                   \
      const T *x2 = x2s + i * V;                                                   \
      T *x3 = x3s + i * V;                                                         \
      int j, k, l, sc;                                                             \
      for (j = 0; j < V; j++) x3[j] = (T)0.0;                                      \
      for (j = 0; j < C; j++) {                                                    \
        for (k = 0; k < S; k++) {                                                  \
          T u1 = (T)0.0, u2 = (T)0.0;                                              \
          for (l = 0; l < S; l++) {                                                \
            u1 += x1[j * S + l] * left[(j * S + k) * S + l];                       \
            u2 += x2[j * S + l] * right[(j * S + k) * S + l];                      \
          }                                                                        \
          p[k] = u1 * u2;                                                          \
        }                                                                          \
        for (k = 0; k < S; k++)                                                    \
          for (l = 0; l < S; l++) x3[j * S + l] += p[k] * EV[S * k + l];           \
      }                                                                            \
      sc = 1;                                                                      \
      for (l = 0; sc && l < V; l++) sc = (fabs((double)x3[l]) < PLFO_MINLIK);      \
      if (sc)                                                                      \
        for (l = 0; l < V; l++) x3[l] = (T)((double)x3[l] * PLFO_TWO_TO_32);       \
      if (scaler) scaler[i] = (unsigned char)sc;                                   \
      if (sc) addScale += wgt ? wgt[i] : 1;                                        \
    }                                                                              \
    if (scalerIncrement) *scalerIncrement = addScale;                              \
  }

PLFO_DEFINE_GEN(f32, float)
PLFO_DEFINE_GEN(f64, double)

/* The same loop with every multiply-add fused (fma(): one rounding per term),
 * in plf()'s order: the reference for the PLFX_FMA mode (extension). */
#define PLFO_DEFINE_GEN_FMA(SUFFIX, T, FMA)                                        \
  void plfo_plf_gen_fma_##SUFFIX(int S, int C, const T *x1s, const T *x2s, T *x3s, \
                                 const T *EV, long long n, const T *left,          \
                                 const T *right, const int *wgt,                   \
                                 long long *scalerIncrement, unsigned char *scaler) { \
    long long i, addScale = 0;                                                     \
    T p[64];                                                                       \
    const int V = S * C;                                                           \
    for (i = 0; i < n; i++) {                                                      \
      const T *x1 = x1s + i * V;                                                   \
      const T *x2 = x2s + i * V;                                                   \
      T *x3 = x3s + i * V;                                                         \
      int j, k, l, sc;                                                             \
      for (j = 0; j < V; j++) x3[j] = (T)0.0;                                      \
      for (j = 0; j < C; j++) {                                                    \
        for (k = 0; k < S; k++) {                                                  \
          T u1 = (T)0.0, u2 = (T)0.0;                                              \
          for (l = 0; l < S; l++) {                                                \
            u1 = FMA(x1[j * S + l], left[(j * S + k) * S + l], u1);                \
            u2 = FMA(x2[j * S + l], right[(j * S + k) * S + l], u2);               \
          }                                                                        \
          p[k] = u1 * u2;                                                          \
        }                                                                          \
        for (k = 0; k < S; k++)                                                    \
          for (l = 0; l < S; l++) x3[j * S + l] = FMA(p[k], EV[S * k + l], x3[j * S + l]); \
      }                                                                            \
      sc = 1;                                                                      \
      for (l = 0; sc && l < V; l++) sc = (fabs((double)x3[l]) < PLFO_MINLIK);      \
      if (sc)                                                                      \
        for (l = 0; l < V; l++) x3[l] = (T)((double)x3[l] * PLFO_TWO_TO_32);       \
      if (scaler) scaler[i] = (unsigned char)sc;                                   \
      if (sc) addScale += wgt ? wgt[i] : 1;                                        \
    }                                                                              \
    if (scalerIncrement) *scalerIncrement = addScale;                              \
  }

PLFO_DEFINE_GEN_FMA(f32, float, fmaf)
PLFO_DEFINE_GEN_FMA(f64, double, fma)

/* OpenMP variant of the generic loops (static site split, one contiguous
 * chunk per thread through the serial function) used only as the multi-core
 * CPU baseline; per-site results are identical to the serial loop. */
#define PLFO_DEFINE_GEN_OMP(SUFFIX, T)                                             \
  void plfo_plf_gen_omp_##SUFFIX(int fma, int S, int C, const T *x1s, const T *x2s, \
                                 T *x3s, const T *EV, long long n, const T *left,  \
                                 const T *right, const int *wgt,                   \
                                 long long *scalerIncrement, unsigned char *scaler, \
                                 int threads) {                                    \
    long long addScale = 0;                                                        \
    const long long V = (long long)S * C;                                          \
    _Pragma("omp parallel num_threads(threads) reduction(+:addScale)")            \
    {                                                                              \
      const long long t = omp_get_thread_num(), nt = omp_get_num_threads();        \
      const long long lo = n * t / nt, hi = n * (t + 1) / nt;                      \
      long long inc = 0;                                                           \
      if (hi > lo) {                                                               \
        if (fma)                                                                   \
          plfo_plf_gen_fma_##SUFFIX(S, C, x1s + lo * V, x2s + lo * V, x3s + lo * V, \
                                    EV, hi - lo, left, right, wgt ? wgt + lo : 0,  \
                                    &inc, scaler ? scaler + lo : 0);               \
        else                                                                       \
          plfo_plf_gen_##SUFFIX(S, C, x1s + lo * V, x2s + lo * V, x3s + lo * V, EV, \
                                hi - lo, left, right, wgt ? wgt + lo : 0, &inc,    \
                                scaler ? scaler + lo : 0);                         \
      }                                                                            \
      addScale += inc;                                                             \
    }                                                                              \
    if (scalerIncrement) *scalerIncrement = addScale;                              \
  }

PLFO_DEFINE_GEN_OMP(f32, float)
PLFO_DEFINE_GEN_OMP(f64, double)

/* Host-side scaler reduction, app/src/host_mem.cpp:384-388. */
long long plfo_scaler_sum(const unsigned char *scaler, const int *wgt, long long n) {
  long long s = 0, j;
  for (j = 0; j < n; j++) s += (long long)scaler[j] * (wgt ? wgt[j] : 1);
  return s;
}

/* ------------------------------------------------------------------------ */
/* std::mt19937 + std::uniform_real_distribution<double>(0,1), restated     */
/* (libstdc++ generate_canonical<double,53> over a 32-bit engine: two draws, */
/* (g0 + g1*2^32) / 2^64, clamped below 1).                                  */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint32_t mt[624];
  int idx;
} plfo_mt;

static void mt_seed(plfo_mt *g, uint32_t seed) {
  int i;
  g->mt[0] = seed;
  for (i = 1; i < 624; i++)
    g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
}

static uint32_t mt_next(plfo_mt *g) {
  uint32_t y;
  if (g->idx >= 624) {
    int k;
    for (k = 0; k < 624; k++) {
      y = (g->mt[k] & 0x80000000u) | (g->mt[(k + 1) % 624] & 0x7fffffffu);
      g->mt[k] = g->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->idx = 0;
  }
  y = g->mt[g->idx++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

static double mt_canonical(plfo_mt *g) {
  double sum = 0.0, tmp = 1.0, r;
  sum += (double)mt_next(g) * tmp;
  tmp *= 4294967296.0;
  sum += (double)mt_next(g) * tmp;
  tmp *= 4294967296.0;
  r = sum / tmp;
  if (r >= 1.0) r = nextafter(1.0, 0.0);
  return r;
}

/* Raw draws, used by the tests to pin this engine against std::mt19937. */
void plfo_mt_draws(uint32_t seed, long long count, uint32_t *out32, double *outd) {
  plfo_mt g;
  long long i;
  mt_seed(&g, seed);
  for (i = 0; i < count; i++) {
    if (out32) out32[i] = mt_next(&g);
  }
  if (outd) {
    mt_seed(&g, seed);
    for (i = 0; i < count; i++) outd[i] = mt_canonical(&g);
  }
}

/* host_mem.cpp:179-209 input protocol.  n sites, elements = 16*n.  The float
 * variant stores like the reference (double draw, optionally x1e-12 in double,
 * rounded to float); the double variant keeps the double. */
#define PLFO_DEFINE_GEN_INPUTS(SUFFIX, T)                                          \
  void plfo_gen_hostmem_##SUFFIX(uint32_t seed, long long n, T *ev, T *left,       \
                                 T *right, T *x1, T *x2, int *wgt) {               \
    plfo_mt g;                                                                     \
    long long j;                                                                   \
    mt_seed(&g, seed);                                                             \
    for (j = 0; j < 16; j++) ev[j] = (T)mt_canonical(&g);                          \
    for (j = 0; j < 64; j++) {                                                     \
      left[j] = (T)mt_canonical(&g);                                               \
      right[j] = (T)mt_canonical(&g);                                              \
    }                                                                              \
    for (j = 0; j < 16 * n; j++) {                                                 \
      double scale = (j % 64 < 16) ? 1.0e-12 : 1.0;                                \
      x1[j] = (T)(mt_canonical(&g) * scale);                                       \
      x2[j] = (T)mt_canonical(&g);                                                 \
    }                                                                              \
    if (wgt)                                                                       \
      for (j = 0; j < n; j++) wgt[j] = 1;                                          \
  }

PLFO_DEFINE_GEN_INPUTS(f32, float)
PLFO_DEFINE_GEN_INPUTS(f64, double)

/* ------------------------------------------------------------------------ */
/* Tree traversal and root log-likelihood (extensions: the reference has no  */
/* traversal or evaluate step, SURVEY F9 -- parity unpinned beyond reusing   */
/* the pinned plf() loop).  Ops run strictly in list order (the sequential   */
/* semantics the GPU's level-batched schedule must reproduce).               */
/* ------------------------------------------------------------------------ */
typedef struct {
  int parent, child1, child2, pmat;
} plfo_trav_op;

#define PLFO_DEFINE_TRAV(SUFFIX, T)                                                     \
  void plfo_traverse_##SUFFIX(int S, int C, const plfo_trav_op *ops, int nops, T **clv,  \
                              const T *pmats, const T *EV, long long n, const int *wgt,   \
                              unsigned char **scalers, long long *scaler_sums) {          \
    const long long mat = (long long)C * S * S;                                          \
    int j;                                                                               \
    for (j = 0; j < nops; j++) {                                                         \
      const plfo_trav_op *o = &ops[j];                                                   \
      long long inc = 0;                                                                 \
      plfo_plf_gen_##SUFFIX(S, C, clv[o->child1], clv[o->child2], clv[o->parent], EV, n,  \
                            pmats + (2LL * o->pmat) * mat, pmats + (2LL * o->pmat + 1) * mat, \
                            wgt, &inc, scalers ? scalers[j] : 0);                        \
      if (scaler_sums) scaler_sums[j] = inc;                                             \
    }                                                                                    \
  }

PLFO_DEFINE_TRAV(f32, float)
PLFO_DEFINE_TRAV(f64, double)

/* lnL = sum_i wgt_i log(sum_c catw[c] sum_s freq[s] x[i][c][s])
 *       + (sum of scaler_sums) * log(2^-32)           (sites in order) */
#define PLFO_DEFINE_LNL(SUFFIX, T)                                                      \
  double plfo_root_lnl_##SUFFIX(int S, int C, const T *x, long long n, const double *catw, \
                                const double *freq, const int *wgt,                      \
                                const long long *scaler_sums, int nsums,                 \
                                double *site_lnl) {                                      \
    double acc = 0.0;                                                                    \
    long long i, nsc = 0;                                                                \
    int c, s;                                                                            \
    for (i = 0; i < n; i++) {                                                            \
      double L = 0.0;                                                                    \
      for (c = 0; c < C; c++) {                                                          \
        double t = 0.0;                                                                  \
        for (s = 0; s < S; s++)                                                          \
          t += (freq ? freq[s] : 1.0 / S) * (double)x[i * S * C + c * S + s];            \
        L += (catw ? catw[c] : 1.0 / C) * t;                                             \
      }                                                                                  \
      {                                                                                  \
        double l = log(L);                                                               \
        if (site_lnl) site_lnl[i] = l;                                                   \
        acc += (wgt ? (double)wgt[i] : 1.0) * l;                                         \
      }                                                                                  \
    }                                                                                    \
    for (c = 0; c < nsums; c++) nsc += scaler_sums[c];                                   \
    return acc + (double)nsc * (-32.0 * 0.69314718055994530942);                         \
  }

PLFO_DEFINE_LNL(f32, float)
PLFO_DEFINE_LNL(f64, double)
