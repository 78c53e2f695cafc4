// Elastic-net coordinate descent (reference
// ``linear_model/_cd_fast.pyx``: enet_coordinate_descent and
// enet_coordinate_descent_gram).  Minimises
//     1/2 ||y - X w||^2 + alpha ||w||_1 + beta/2 ||w||^2
// by cyclic (or xorshift-random) coordinate updates with soft-thresholding;
// after a sweep whose largest coordinate change is below tol * max|w| the
// duality gap is evaluated and the solve stops once it drops below
// tol * ||y||^2.  The random coordinate stream is the reference's 32-bit
// xorshift (shifts 13/17/5, modulo 2^31), seeded by the caller, so
// selection='random' reproduces the reference's visiting order.
//
// Host design: the dense variant walks a column-major X (one contiguous
// column per coordinate); the Gram variant works on Q = X^T X and q = X^T y,
// which the framework computes on the GPU (hipBLASLt) before handing the
// d x d problem to this loop.
#include <cmath>
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

inline uint32_t xorshift_next(uint32_t* s) {
  if (*s == 0) *s = 1;
  *s ^= (uint32_t)(*s << 13);
  *s ^= (uint32_t)(*s >> 17);
  *s ^= (uint32_t)(*s << 5);
  return *s % ((uint32_t)0x7FFFFFFF + 1u);
}

inline double fsign(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }

inline double dot(const double* a, const double* b, int64_t n) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

inline void axpy(int64_t n, double a, const double* x, double* y) {
  for (int64_t i = 0; i < n; ++i) y[i] += a * x[i];
}

}  // namespace

extern "C" {

// X column-major (n x d); w in/out; out: [gap, tol_scaled, n_iter, converged]
void sqh_enet_cd_dense(double* w, double alpha, double beta, const double* X, const double* y,
                       long long n, long long d, int max_iter, double tol, uint32_t seed,
                       int random, int positive, double* out) {
  std::vector<double> norm_cols(d), R(n), XtA(d);
  for (int64_t j = 0; j < d; ++j) norm_cols[j] = dot(X + j * n, X + j * n, n);
  for (int64_t i = 0; i < n; ++i) R[i] = y[i];
  for (int64_t j = 0; j < d; ++j)
    if (w[j] != 0.0) axpy(n, -w[j], X + j * n, R.data());
  const double d_w_tol = tol;
  tol *= dot(y, y, n);
  double gap = tol + 1.0;
  int it = 0;
  bool converged = false;
  uint32_t rs = seed;
  for (it = 0; it < max_iter; ++it) {
    double w_max = 0.0, d_w_max = 0.0;
    for (int64_t f = 0; f < d; ++f) {
      const int64_t ii = random ? (int64_t)(xorshift_next(&rs) % (uint32_t)d) : f;
      if (norm_cols[ii] == 0.0) continue;
      const double w_ii = w[ii];
      const double* xc = X + ii * n;
      if (w_ii != 0.0) axpy(n, w_ii, xc, R.data());
      const double tmp = dot(xc, R.data(), n);
      if (positive && tmp < 0)
        w[ii] = 0.0;
      else
        w[ii] = fsign(tmp) * std::fmax(std::fabs(tmp) - alpha, 0.0) / (norm_cols[ii] + beta);
      if (w[ii] != 0.0) axpy(n, -w[ii], xc, R.data());
      d_w_max = std::fmax(d_w_max, std::fabs(w[ii] - w_ii));
      w_max = std::fmax(w_max, std::fabs(w[ii]));
    }
    if (w_max == 0.0 || d_w_max / w_max < d_w_tol || it == max_iter - 1) {
      for (int64_t j = 0; j < d; ++j) XtA[j] = dot(X + j * n, R.data(), n) - beta * w[j];
      double dual = 0.0;
      for (int64_t j = 0; j < d; ++j) {
        const double v = positive ? XtA[j] : std::fabs(XtA[j]);
        if (j == 0 || v > dual) dual = v;
      }
      const double R2 = dot(R.data(), R.data(), n), w2 = dot(w, w, d);
      double cst;
      if (dual > alpha) {
        cst = alpha / dual;
        gap = 0.5 * (R2 + R2 * cst * cst);
      } else {
        cst = 1.0;
        gap = R2;
      }
      double l1 = 0.0;
      for (int64_t j = 0; j < d; ++j) l1 += std::fabs(w[j]);
      gap += alpha * l1 - cst * dot(R.data(), y, n) + 0.5 * beta * (1 + cst * cst) * w2;
      if (gap < tol) {
        converged = true;
        break;
      }
    }
  }
  out[0] = gap;
  out[1] = tol;
  out[2] = (double)(converged ? it + 1 : max_iter);
  out[3] = converged ? 1.0 : 0.0;
}

// Q row-major d x d (= X^T X), q = X^T y, y_norm2 = y.y
void sqh_enet_cd_gram(double* w, double alpha, double beta, const double* Q, const double* q,
                      double y_norm2, long long d, int max_iter, double tol, uint32_t seed,
                      int random, int positive, double* out) {
  std::vector<double> H(d, 0.0), XtA(d);
  for (int64_t i = 0; i < d; ++i) H[i] = dot(Q + i * d, w, d);
  const double d_w_tol = tol;
  tol *= y_norm2;
  double gap = tol + 1.0;
  int it = 0;
  bool converged = false;
  uint32_t rs = seed;
  for (it = 0; it < max_iter; ++it) {
    double w_max = 0.0, d_w_max = 0.0;
    for (int64_t f = 0; f < d; ++f) {
      const int64_t ii = random ? (int64_t)(xorshift_next(&rs) % (uint32_t)d) : f;
      if (Q[ii * d + ii] == 0.0) continue;
      const double w_ii = w[ii];
      if (w_ii != 0.0) axpy(d, -w_ii, Q + ii * d, H.data());
      const double tmp = q[ii] - H[ii];
      if (positive && tmp < 0)
        w[ii] = 0.0;
      else
        w[ii] = fsign(tmp) * std::fmax(std::fabs(tmp) - alpha, 0.0) / (Q[ii * d + ii] + beta);
      if (w[ii] != 0.0) axpy(d, w[ii], Q + ii * d, H.data());
      const double dw = std::fabs(w[ii] - w_ii);
      if (dw > d_w_max) d_w_max = dw;
      if (std::fabs(w[ii]) > w_max) w_max = std::fabs(w[ii]);
    }
    if (w_max == 0.0 || d_w_max / w_max < d_w_tol || it == max_iter - 1) {
      const double qw = dot(w, q, d);
      double dual = 0.0;
      for (int64_t j = 0; j < d; ++j) {
        XtA[j] = q[j] - H[j] - beta * w[j];
        const double v = positive ? XtA[j] : std::fabs(XtA[j]);
        if (j == 0 || v > dual) dual = v;
      }
      const double wH = dot(w, H.data(), d);
      const double R2 = y_norm2 + wH - 2.0 * qw, w2 = dot(w, w, d);
      double cst;
      if (dual > alpha) {
        cst = alpha / dual;
        gap = 0.5 * (R2 + R2 * cst * cst);
      } else {
        cst = 1.0;
        gap = R2;
      }
      double l1 = 0.0;
      for (int64_t j = 0; j < d; ++j) l1 += std::fabs(w[j]);
      gap += alpha * l1 - cst * y_norm2 + cst * qw + 0.5 * beta * (1 + cst * cst) * w2;
      if (gap < tol) {
        converged = true;
        break;
      }
    }
  }
  out[0] = gap;
  out[1] = tol;
  out[2] = (double)(converged ? it + 1 : max_iter);
  out[3] = converged ? 1.0 : 0.0;
}

}  // extern "C"
