// Trust-region Newton (TRON) for liblinear's L2-regularised primal problems
// (reference ``svm/src/liblinear/tron.cpp`` and the function objects of
// ``linear.cpp``: l2r_lr_fun, l2r_l2_svc_fun, l2r_l2_svr_fun; solver types
// 0, 2 and 11).
//
//   L2R_LR   f(w) = w.w / 2 + sum_i C_i log(1 + exp(-y_i w.x_i))
//   L2R_L2SVC       w.w / 2 + sum_i C_i max(0, 1 - y_i w.x_i)^2
//   L2R_L2SVR       w.w / 2 + sum_i C_i max(0, |w.x_i - y_i| - p)^2
//
// Each outer iteration solves the trust-region sub-problem with conjugate
// gradients on Hessian-vector products (stopping at |r| <= 0.1 |g| or at the
// region boundary), then accepts / rejects the step and resizes the region
// from the actual-vs-predicted reduction with liblinear's constants; the
// run stops when |g| <= eps |g(w0)|.  X v and X^T u (the only O(n d) work)
// run as OpenMP loops over rows / feature blocks with per-thread partials
// reduced in a fixed order (deterministic for a given thread count).
#include <cmath>
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

struct Data {
  const double* X;   // n x d, row major (bias column already appended)
  int64_t n, d;
  const double* y;
  const double* C;
};

// out = X v
void xv(const Data& D, const double* v, double* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < D.n; ++i) {
    const double* xi = D.X + i * D.d;
    double s = 0.0;
    for (int64_t f = 0; f < D.d; ++f) s += xi[f] * v[f];
    out[i] = s;
  }
}

// out = X^T u over the rows with mask[i] (mask null: all rows); feature
// blocks per thread, rows in order inside a block: deterministic
void xtu(const Data& D, const double* u, const char* mask, double* out) {
  const int64_t B = 64;
  const int64_t nb = (D.d + B - 1) / B;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t f0 = b * B, f1 = std::min(D.d, f0 + B);
    double acc[64];
    for (int64_t f = f0; f < f1; ++f) acc[f - f0] = 0.0;
    for (int64_t i = 0; i < D.n; ++i) {
      if (mask && !mask[i]) continue;
      const double ui = u[i];
      if (ui == 0.0) continue;
      const double* xi = D.X + i * D.d;
      for (int64_t f = f0; f < f1; ++f) acc[f - f0] += ui * xi[f];
    }
    for (int64_t f = f0; f < f1; ++f) out[f] = acc[f - f0];
  }
}

double dot(const std::vector<double>& a, const std::vector<double>& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
  return s;
}

double nrm(const std::vector<double>& a) { return std::sqrt(dot(a, a)); }

struct Objective {
  const Data& D;
  int kind;       // 0 LR, 1 L2-loss SVC, 2 L2-loss SVR
  double p;       // SVR insensitivity
  std::vector<double> z, dvec, u, tmp;
  std::vector<char> act;
  explicit Objective(const Data& d, int k, double pp)
      : D(d), kind(k), p(pp), z(d.n), dvec(d.n), u(d.n), tmp(d.n), act(d.n, 1) {}

  double fun(const std::vector<double>& w) {
    xv(D, w.data(), z.data());
    double f = 0.5 * dot(w, w);
    for (int64_t i = 0; i < D.n; ++i) {
      const double yz = D.y[i] * z[i];
      if (kind == 0) {
        f += D.C[i] * (yz >= 0 ? std::log1p(std::exp(-yz)) : -yz + std::log1p(std::exp(yz)));
      } else if (kind == 1) {
        const double m = 1.0 - yz;
        if (m > 0) f += D.C[i] * m * m;
      } else {
        const double r = z[i] - D.y[i];
        if (r < -p) f += D.C[i] * (r + p) * (r + p);
        else if (r > p) f += D.C[i] * (r - p) * (r - p);
      }
    }
    return f;
  }

  // gradient at the w of the last fun() call; also fixes the Hessian's
  // per-row weights dvec and active rows
  void grad(const std::vector<double>& w, std::vector<double>& g) {
    for (int64_t i = 0; i < D.n; ++i) {
      if (kind == 0) {
        const double s = 1.0 / (1.0 + std::exp(-D.y[i] * z[i]));
        dvec[i] = s * (1.0 - s);
        u[i] = D.C[i] * (s - 1.0) * D.y[i];
        act[i] = 1;
      } else if (kind == 1) {
        const double yz = D.y[i] * z[i];
        act[i] = yz < 1.0;
        u[i] = act[i] ? 2.0 * D.C[i] * D.y[i] * (yz - 1.0) : 0.0;
      } else {
        const double r = z[i] - D.y[i];
        act[i] = r < -p || r > p;
        u[i] = r < -p ? 2.0 * D.C[i] * (r + p) : (r > p ? 2.0 * D.C[i] * (r - p) : 0.0);
      }
    }
    xtu(D, u.data(), kind == 0 ? nullptr : act.data(), g.data());
    for (int64_t f = 0; f < D.d; ++f) g[f] += w[f];
  }

  void hv(const std::vector<double>& s, std::vector<double>& out) {
    xv(D, s.data(), tmp.data());
    for (int64_t i = 0; i < D.n; ++i) {
      if (kind == 0) tmp[i] *= D.C[i] * dvec[i];
      else tmp[i] = act[i] ? 2.0 * D.C[i] * tmp[i] : 0.0;
    }
    xtu(D, tmp.data(), kind == 0 ? nullptr : act.data(), out.data());
    for (int64_t f = 0; f < D.d; ++f) out[f] += s[f];
  }
};

// CG on the trust-region sub-problem min g.s + s.H s / 2, |s| <= delta
int trcg(Objective& obj, double delta, const std::vector<double>& g, std::vector<double>& s,
         std::vector<double>& r) {
  const size_t n = g.size();
  std::vector<double> dd(n), Hd(n);
  for (size_t i = 0; i < n; ++i) {
    s[i] = 0.0;
    r[i] = -g[i];
    dd[i] = r[i];
  }
  const double cgtol = 0.1 * nrm(g);
  int it = 0;
  double rTr = dot(r, r);
  while (std::sqrt(rTr) > cgtol) {
    ++it;
    obj.hv(dd, Hd);
    double alpha = rTr / dot(dd, Hd);
    for (size_t i = 0; i < n; ++i) s[i] += alpha * dd[i];
    if (nrm(s) > delta) {
      // back off and move to the boundary along dd
      for (size_t i = 0; i < n; ++i) s[i] -= alpha * dd[i];
      const double sd = dot(s, dd), ss = dot(s, s), d2 = dot(dd, dd);
      const double dsq = delta * delta;
      const double rad = std::sqrt(sd * sd + d2 * (dsq - ss));
      alpha = sd >= 0 ? (dsq - ss) / (sd + rad) : (rad - sd) / d2;
      for (size_t i = 0; i < n; ++i) {
        s[i] += alpha * dd[i];
        r[i] -= alpha * Hd[i];
      }
      break;
    }
    for (size_t i = 0; i < n; ++i) r[i] -= alpha * Hd[i];
    const double rn = dot(r, r);
    const double beta = rn / rTr;
    for (size_t i = 0; i < n; ++i) dd[i] = r[i] + beta * dd[i];
    rTr = rn;
  }
  return it;
}

}  // namespace

extern "C" {

// kind: 0 L2R_LR, 1 L2R_L2LOSS_SVC, 2 L2R_L2LOSS_SVR (p = epsilon).
// w: in = start, out = solution.  Returns the number of outer iterations.
int sqh_tron(const double* X, long long n, long long d, const double* y, const double* C,
             int kind, double p, double eps, int max_iter, double* w_io) {
  Data D{X, n, d, y, C};
  Objective obj(D, kind, p);
  const double eta0 = 1e-4, eta1 = 0.25, eta2 = 0.75;
  const double sigma1 = 0.25, sigma2 = 0.5, sigma3 = 4.0;
  std::vector<double> w(w_io, w_io + d), g(d), s(d), r(d), wn(d);
  double f = obj.fun(w);
  obj.grad(w, g);
  double delta = nrm(g);
  const double g0 = delta;
  double gnorm = g0;
  int iter = 1;
  bool search = gnorm > eps * g0;
  while (iter <= max_iter && search) {
    trcg(obj, delta, g, s, r);
    for (int64_t i = 0; i < d; ++i) wn[i] = w[i] + s[i];
    const double gs = dot(g, s);
    const double prered = -0.5 * (gs - dot(s, r));
    const double fnew = obj.fun(wn);
    const double actred = f - fnew;
    const double snorm = nrm(s);
    if (iter == 1) delta = std::min(delta, snorm);
    double alpha = fnew - f - gs <= 0 ? sigma3 : std::max(sigma1, -0.5 * (gs / (fnew - f - gs)));
    if (actred < eta0 * prered) delta = std::min(std::max(alpha, sigma1) * snorm, sigma2 * delta);
    else if (actred < eta1 * prered)
      delta = std::max(sigma1 * delta, std::min(alpha * snorm, sigma2 * delta));
    else if (actred < eta2 * prered)
      delta = std::max(sigma1 * delta, std::min(alpha * snorm, sigma3 * delta));
    else delta = std::max(delta, std::min(alpha * snorm, sigma3 * delta));
    if (actred > eta0 * prered) {
      ++iter;
      w = wn;
      f = fnew;
      obj.grad(w, g);
      gnorm = nrm(g);
      if (gnorm <= eps * g0) break;
    }
    if (f < -1.0e+32) break;
    if (std::fabs(actred) <= 0 && prered <= 0) break;
    if (std::fabs(actred) <= 1.0e-12 * std::fabs(f) && std::fabs(prered) <= 1.0e-12 * std::fabs(f))
      break;
  }
  for (int64_t i = 0; i < d; ++i) w_io[i] = w[i];
  return iter - 1;
}

}  // extern "C"
