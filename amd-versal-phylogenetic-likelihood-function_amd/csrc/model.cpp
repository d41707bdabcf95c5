// model.cpp -- substitution-model setup for the PLF inputs (SURVEY section 8f
// row 3): the eigendecomposition of a time-reversible rate matrix and the
// discrete-Gamma category rates.  The reference has no model code -- its P
// matrices and EV are random (app/src/host_mem.cpp:189-197) or precomputed
// files (aie/data/inputbranch*, inputEV0.txt) -- so these follow the standard
// published definitions: GTR (Tavare 1986) normalised to one expected
// substitution per unit time, and Yang (1994) discrete Gamma (mean or median
// of each of K equal-probability categories).  Host-only code (no device
// work); the P matrices themselves are built on the device (plf_pmat.hpp).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/plfx.h"

namespace {

// Cyclic Jacobi on a symmetric S x S matrix A (row-major, destroyed):
// A = U diag(w) U^T, U's columns the eigenvectors.
void jacobi(int S, std::vector<double> &A, std::vector<double> &w, std::vector<double> &U) {
  U.assign((size_t)S * S, 0.0);
  for (int i = 0; i < S; i++) U[(size_t)i * S + i] = 1.0;
  auto a = [&](int i, int j) -> double & { return A[(size_t)i * S + j]; };
  for (int sweep = 0; sweep < 100; sweep++) {
    double off = 0.0, diag = 0.0;
    for (int i = 0; i < S; i++) {
      diag += a(i, i) * a(i, i);
      for (int j = i + 1; j < S; j++) off += a(i, j) * a(i, j);
    }
    if (off <= 1e-36 * diag || off == 0.0) break;
    for (int p = 0; p < S; p++)
      for (int q = p + 1; q < S; q++) {
        const double apq = a(p, q);
        if (apq == 0.0) continue;
        // rotation angle that zeroes a(p,q): t = tan(theta)
        const double theta = (a(q, q) - a(p, p)) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < S; k++) {  // A <- A J (columns p, q)
          const double akp = a(k, p), akq = a(k, q);
          a(k, p) = c * akp - s * akq;
          a(k, q) = s * akp + c * akq;
        }
        for (int k = 0; k < S; k++) {  // A <- J^T A (rows p, q)
          const double apk = a(p, k), aqk = a(q, k);
          a(p, k) = c * apk - s * aqk;
          a(q, k) = s * apk + c * aqk;
        }
        for (int k = 0; k < S; k++) {  // U <- U J
          double &ukp = U[(size_t)k * S + p], &ukq = U[(size_t)k * S + q];
          const double x = ukp, y = ukq;
          ukp = c * x - s * y;
          ukq = s * x + c * y;
        }
      }
  }
  w.resize(S);
  for (int i = 0; i < S; i++) w[i] = a(i, i);
}

// Regularised lower incomplete gamma P(a, x): series below a+1, Lentz's
// continued fraction for Q = 1 - P above.
double inc_gamma_p(double a, double x) {
  if (x <= 0.0) return 0.0;
  if (std::isinf(x)) return 1.0;
  const double lpre = -x + a * std::log(x) - std::lgamma(a);
  if (x < a + 1.0) {
    double term = 1.0 / a, sum = term;
    for (int n = 1; n < 100000; n++) {
      term *= x / (a + n);
      sum += term;
      if (std::fabs(term) < std::fabs(sum) * 1e-17) break;
    }
    return sum * std::exp(lpre);
  }
  const double tiny = 1e-300;
  double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
  for (int i = 1; i < 100000; i++) {
    const double an = -i * (i - a);
    b += 2.0;
    d = an * d + b;
    if (std::fabs(d) < tiny) d = tiny;
    c = b + an / c;
    if (std::fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    const double del = d * c;
    h *= del;
    if (std::fabs(del - 1.0) < 1e-17) break;
  }
  return 1.0 - std::exp(lpre) * h;
}

// y with P(a, y) = p (0 < p < 1), by bracketing and bisection to full precision.
double inc_gamma_p_inv(double a, double p) {
  double lo = 0.0, hi = a > 1.0 ? a : 1.0;
  while (inc_gamma_p(a, hi) < p) hi *= 2.0;
  for (int it = 0; it < 2000; it++) {
    const double mid = 0.5 * (lo + hi);
    if (mid <= lo || mid >= hi) break;
    if (inc_gamma_p(a, mid) < p) lo = mid;
    else hi = mid;
  }
  return 0.5 * (lo + hi);
}

}  // namespace

extern "C" {

int plfx_model_eigen(int states, const double *exch, const double *freqs, double *eigen) {
  const int S = states;
  if (S < 2 || S > 64 || !exch || !freqs || !eigen) return PLFX_ERR_INVALID;
  std::vector<double> pi(S);
  double fs = 0.0;
  for (int i = 0; i < S; i++) {
    if (!(freqs[i] > 0.0) || !std::isfinite(freqs[i])) return PLFX_ERR_INVALID;
    fs += freqs[i];
  }
  for (int i = 0; i < S; i++) pi[i] = freqs[i] / fs;
  // Q_ij = r_ij pi_j (i != j), rows sum to 0, scaled to sum_i pi_i (-Q_ii) = 1
  std::vector<double> R((size_t)S * S, 0.0);
  int e = 0;
  for (int i = 0; i < S; i++)
    for (int j = i + 1; j < S; j++, e++) {
      if (!(exch[e] >= 0.0) || !std::isfinite(exch[e])) return PLFX_ERR_INVALID;
      R[(size_t)i * S + j] = R[(size_t)j * S + i] = exch[e];
    }
  double mu = 0.0;
  for (int i = 0; i < S; i++)
    for (int j = 0; j < S; j++)
      if (j != i) mu += pi[i] * R[(size_t)i * S + j] * pi[j];
  if (!(mu > 0.0)) return PLFX_ERR_INVALID;
  // symmetric B = D^1/2 Q D^-1/2: B_ij = r_ij sqrt(pi_i pi_j) / mu, B_ii = Q_ii
  std::vector<double> B((size_t)S * S, 0.0);
  for (int i = 0; i < S; i++) {
    double qii = 0.0;
    for (int j = 0; j < S; j++)
      if (j != i) {
        B[(size_t)i * S + j] = R[(size_t)i * S + j] * std::sqrt(pi[i] * pi[j]) / mu;
        qii -= R[(size_t)i * S + j] * pi[j] / mu;
      }
    B[(size_t)i * S + i] = qii;
  }
  std::vector<double> w, U;
  jacobi(S, B, w, U);
  // order eigenvalues descending (lambda_0 = 0 first)
  std::vector<int> ord(S);
  for (int i = 0; i < S; i++) ord[i] = i;
  for (int i = 0; i < S; i++)
    for (int j = i + 1; j < S; j++)
      if (w[ord[j]] > w[ord[i]]) std::swap(ord[i], ord[j]);
  double *lam = eigen, *V = eigen + S, *Vi = eigen + S + (size_t)S * S;
  for (int m = 0; m < S; m++) {
    const int o = ord[m];
    lam[m] = w[o];
    for (int k = 0; k < S; k++) {
      V[(size_t)k * S + m] = U[(size_t)k * S + o] / std::sqrt(pi[k]);   // D^-1/2 U
      Vi[(size_t)m * S + k] = U[(size_t)k * S + o] * std::sqrt(pi[k]);  // U^T D^1/2
    }
  }
  return PLFX_OK;
}

int plfx_gamma_rates(double alpha, int ncat, int median, double *rates) {
  if (!(alpha > 0.0) || !std::isfinite(alpha) || ncat < 1 || !rates) return PLFX_ERR_INVALID;
  if (ncat == 1) {
    rates[0] = 1.0;
    return PLFX_OK;
  }
  // Gamma(shape alpha, rate alpha): mean 1; y = alpha * x is Gamma(alpha, 1)
  if (median) {
    double s = 0.0;
    for (int i = 0; i < ncat; i++) {
      rates[i] = inc_gamma_p_inv(alpha, (2.0 * i + 1.0) / (2.0 * ncat)) / alpha;
      s += rates[i];
    }
    for (int i = 0; i < ncat; i++) rates[i] *= ncat / s;
    return PLFX_OK;
  }
  // mean of category i = K * integral of x f(x) over [q_i, q_i+1)
  //                    = K * (P(alpha+1, y_i+1) - P(alpha+1, y_i))
  double prev = 0.0;
  for (int i = 0; i < ncat; i++) {
    const double cur =
        i + 1 == ncat ? 1.0 : inc_gamma_p(alpha + 1.0, inc_gamma_p_inv(alpha, (i + 1.0) / ncat));
    rates[i] = ncat * (cur - prev);
    prev = cur;
  }
  return PLFX_OK;
}

int plfx_model_ev(int states, int convention, const double *eigen, double *EV) {
  const int S = states;
  if (S < 2 || S > 64 || !EV || (convention != PLFX_PMAT_STATE && convention != PLFX_PMAT_EIGEN))
    return PLFX_ERR_INVALID;
  if (convention == PLFX_PMAT_STATE) {
    for (int k = 0; k < S; k++)
      for (int l = 0; l < S; l++) EV[k * S + l] = k == l ? 1.0 : 0.0;
    return PLFX_OK;
  }
  if (!eigen) return PLFX_ERR_INVALID;
  const double *Vi = eigen + S + (size_t)S * S;
  for (int k = 0; k < S; k++)
    for (int l = 0; l < S; l++) EV[k * S + l] = Vi[(size_t)l * S + k];
  return PLFX_OK;
}

int plfx_model_root_weights(int states, int convention, const double *eigen, const double *freqs,
                            double *w) {
  const int S = states;
  if (S < 2 || S > 64 || !freqs || !w || (convention != PLFX_PMAT_STATE && convention != PLFX_PMAT_EIGEN))
    return PLFX_ERR_INVALID;
  double fs = 0.0;
  for (int s = 0; s < S; s++) fs += freqs[s];
  if (!(fs > 0.0)) return PLFX_ERR_INVALID;
  if (convention == PLFX_PMAT_STATE) {
    for (int s = 0; s < S; s++) w[s] = freqs[s] / fs;
    return PLFX_OK;
  }
  if (!eigen) return PLFX_ERR_INVALID;
  const double *V = eigen + S;
  for (int k = 0; k < S; k++) {
    double a = 0.0;
    for (int s = 0; s < S; s++) a += freqs[s] / fs * V[(size_t)s * S + k];
    w[k] = a;
  }
  return PLFX_OK;
}

int plfx_model_tip_vectors(int states, int convention, const double *eigen, double *tv) {
  const int S = states;
  if (S != 4 || !tv || (convention != PLFX_PMAT_STATE && convention != PLFX_PMAT_EIGEN))
    return PLFX_ERR_INVALID;
  if (convention == PLFX_PMAT_EIGEN && !eigen) return PLFX_ERR_INVALID;
  const double *Vi = eigen ? eigen + S + (size_t)S * S : nullptr;
  for (int code = 0; code < 16; code++)
    for (int k = 0; k < S; k++) {
      if (convention == PLFX_PMAT_STATE) {
        tv[code * S + k] = (code >> k) & 1 ? 1.0 : 0.0;
      } else {
        double a = 0.0;
        for (int s = 0; s < S; s++)
          if ((code >> s) & 1) a += Vi[(size_t)k * S + s];
        tv[code * S + k] = a;
      }
    }
  return PLFX_OK;
}

}  // extern "C"
