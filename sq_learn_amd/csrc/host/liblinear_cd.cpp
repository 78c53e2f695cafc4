// Dual coordinate descent of liblinear (reference
// ``svm/src/liblinear/linear.cpp``: ``solve_l2r_l1l2_svc`` :820-1012 for
// L2-regularised L1-/L2-loss SVC, ``solve_l2r_l1l2_svr`` :1050-1240 for the
// SVR duals), with the reference's per-instance C (sample weights), its
// shrinking heuristics and its random visiting order: ``std::mt19937``
// seeded by the caller and the Lemire bounded integer of
// ``svm/src/newrand/newrand.h`` - so iterates, n_iter and the returned w are
// the reference's.  Rows are dense (row-major, bias column appended by the
// caller when fitting an intercept).  Also the Crammer-Singer multi-class
// dual (``Solver_MCSVM_CS``, linear.cpp:493-787): per-instance sub-problems
// over the class scores with per-class shrinking.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <random>
#include <utility>
#include <vector>

#include "host.h"

namespace {

constexpr double kInf = HUGE_VAL;

struct Rng {
  std::mt19937 mt;
  explicit Rng(uint32_t seed) : mt(seed) {}
  uint32_t bounded(uint32_t range) {
    uint32_t x = mt();
    uint64_t m = uint64_t(x) * uint64_t(range);
    uint32_t l = uint32_t(m);
    if (l < range) {
      uint32_t t = -range;
      if (t >= range) {
        t -= range;
        if (t >= range) t %= range;
      }
      while (l < t) {
        x = mt();
        m = uint64_t(x) * uint64_t(range);
        l = uint32_t(m);
      }
    }
    return (uint32_t)(m >> 32);
  }
};

inline double dot(const double* a, const double* b, int64_t d) {
  double s = 0;
  for (int64_t k = 0; k < d; ++k) s += a[k] * b[k];
  return s;
}

}  // namespace

extern "C" {

// The reference keeps ONE mt19937 across the one-vs-rest sub-problems of a
// fit (``newrand.h`` global): callers create a stream and pass it to every
// solve of that fit.
void* sqh_mt_new(uint32_t seed) { return new Rng(seed); }
void sqh_mt_free(void* h) { delete (Rng*)h; }

// L2-regularised L2-loss (l1loss=0) or L1-loss (l1loss=1) SVC dual.
// y in {+1,-1}; Cvec per instance (W_i * C_{class}).  Returns iterations.
int sqh_linear_svc_dual(const double* X, long long l, long long d, const double* y,
                        const double* Cvec, int l1loss, double eps, int max_iter, void* stream,
                        double* w, double* alpha_out) {
  Rng& rng = *(Rng*)stream;
  std::vector<double> diag(l), ub(l), QD(l), alpha(l, 0.0);
  std::vector<int> index(l);
  std::vector<int8_t> yy(l);
  for (int64_t i = 0; i < l; ++i) {
    diag[i] = l1loss ? 0.0 : 0.5 / Cvec[i];
    ub[i] = l1loss ? Cvec[i] : kInf;
    yy[i] = y[i] > 0 ? 1 : -1;
  }
  for (int64_t k = 0; k < d; ++k) w[k] = 0;
  for (int64_t i = 0; i < l; ++i) {
    QD[i] = diag[i] + dot(X + i * d, X + i * d, d);
    index[i] = (int)i;
  }
  int64_t active = l;
  double PGmax_old = kInf, PGmin_old = -kInf;
  int iter = 0;
  while (iter < max_iter) {
    double PGmax_new = -kInf, PGmin_new = kInf;
    for (int64_t i = 0; i < active; ++i) {
      int64_t j = i + rng.bounded((uint32_t)(active - i));
      std::swap(index[i], index[j]);
    }
    for (int64_t s = 0; s < active; ++s) {
      const int i = index[s];
      const double* xi = X + (int64_t)i * d;
      const int yi = yy[i];
      double G = dot(w, xi, d) * yi - 1;
      const double C = ub[i];
      G += alpha[i] * diag[i];
      double PG = 0;
      if (alpha[i] == 0) {
        if (G > PGmax_old) { --active; std::swap(index[s], index[active]); --s; continue; }
        else if (G < 0) PG = G;
      } else if (alpha[i] == C) {
        if (G < PGmin_old) { --active; std::swap(index[s], index[active]); --s; continue; }
        else if (G > 0) PG = G;
      } else {
        PG = G;
      }
      PGmax_new = std::max(PGmax_new, PG);
      PGmin_new = std::min(PGmin_new, PG);
      if (std::fabs(PG) > 1.0e-12) {
        double old = alpha[i];
        alpha[i] = std::min(std::max(alpha[i] - G / QD[i], 0.0), C);
        double dlt = (alpha[i] - old) * yi;
        for (int64_t k = 0; k < d; ++k) w[k] += dlt * xi[k];
      }
    }
    ++iter;
    if (PGmax_new - PGmin_new <= eps) {
      if (active == l) break;
      active = l;
      PGmax_old = kInf;
      PGmin_old = -kInf;
      continue;
    }
    PGmax_old = PGmax_new;
    PGmin_old = PGmin_new;
    if (PGmax_old <= 0) PGmax_old = kInf;
    if (PGmin_old >= 0) PGmin_old = -kInf;
  }
  if (alpha_out)
    for (int64_t i = 0; i < l; ++i) alpha_out[i] = alpha[i];
  return iter;
}

// L2-regularised L1-loss (l1loss=1, epsilon-insensitive) or L2-loss SVR dual.
int sqh_linear_svr_dual(const double* X, long long l, long long d, const double* y,
                        const double* Cvec, int l1loss, double p, double eps, int max_iter,
                        void* stream, double* w) {
  Rng& rng = *(Rng*)stream;
  std::vector<double> lambda(l), ub(l), beta(l, 0.0), QD(l);
  std::vector<int> index(l);
  for (int64_t i = 0; i < l; ++i) {
    lambda[i] = l1loss ? 0.0 : 0.5 / Cvec[i];
    ub[i] = l1loss ? Cvec[i] : kInf;
  }
  for (int64_t k = 0; k < d; ++k) w[k] = 0;
  for (int64_t i = 0; i < l; ++i) {
    QD[i] = dot(X + i * d, X + i * d, d);
    index[i] = (int)i;
  }
  int64_t active = l;
  double Gmax_old = kInf, Gnorm1_init = -1.0;
  int iter = 0;
  while (iter < max_iter) {
    double Gmax_new = 0, Gnorm1_new = 0;
    for (int64_t i = 0; i < active; ++i) {
      int64_t j = i + rng.bounded((uint32_t)(active - i));
      std::swap(index[i], index[j]);
    }
    for (int64_t s = 0; s < active; ++s) {
      const int i = index[s];
      const double* xi = X + (int64_t)i * d;
      double G = -y[i] + lambda[i] * beta[i] + dot(w, xi, d);
      const double H = QD[i] + lambda[i];
      const double Gp = G + p, Gn = G - p;
      double viol = 0;
      if (beta[i] == 0) {
        if (Gp < 0) viol = -Gp;
        else if (Gn > 0) viol = Gn;
        else if (Gp > Gmax_old && Gn < -Gmax_old) {
          --active; std::swap(index[s], index[active]); --s; continue;
        }
      } else if (beta[i] >= ub[i]) {
        if (Gp > 0) viol = Gp;
        else if (Gp < -Gmax_old) { --active; std::swap(index[s], index[active]); --s; continue; }
      } else if (beta[i] <= -ub[i]) {
        if (Gn < 0) viol = -Gn;
        else if (Gn > Gmax_old) { --active; std::swap(index[s], index[active]); --s; continue; }
      } else if (beta[i] > 0) {
        viol = std::fabs(Gp);
      } else {
        viol = std::fabs(Gn);
      }
      Gmax_new = std::max(Gmax_new, viol);
      Gnorm1_new += viol;
      double dd;
      if (Gp < H * beta[i]) dd = -Gp / H;
      else if (Gn > H * beta[i]) dd = -Gn / H;
      else dd = -beta[i];
      if (std::fabs(dd) < 1.0e-12) continue;
      double old = beta[i];
      beta[i] = std::min(std::max(beta[i] + dd, -ub[i]), ub[i]);
      dd = beta[i] - old;
      if (dd != 0)
        for (int64_t k = 0; k < d; ++k) w[k] += dd * xi[k];
    }
    if (iter == 0) Gnorm1_init = Gnorm1_new;
    ++iter;
    if (Gnorm1_new <= eps * Gnorm1_init) {
      if (active == l) break;
      active = l;
      Gmax_old = kInf;
      continue;
    }
    Gmax_old = Gmax_new;
  }
  return iter;
}

}  // extern "C"

// Crammer-Singer multi-class SVM dual (reference linear.cpp:493-787):
//   min_a 0.5 sum_m |w_m|^2 + sum_{i, m != y_i} a_i^m,  w_m = sum_i a_i^m x_i,
//   sum_m a_i^m = 0,  a_i^m <= C_i [m = y_i]  (C_i = W_i C_{y_i}),
// solved one instance at a time (all its class scores at once, the closed-
// form sub-problem below) in a random order, with the reference's per-class
// and per-instance shrinking and its stopping rule.  y: class ids 0..K-1
// (rows grouped by class).  w: [d][K] feature-major, like liblinear's model.
namespace {

struct McsCs {
  int K;
  std::vector<double> D;
  explicit McsCs(int k) : K(k), D(k) {}
  // new scores of one instance: the threshold beta of the sorted shifted
  // gradients, then a^m = min(bound_m, (beta - B_m) / A)
  void sub_problem(double A, int yi, double Cy, int na, const double* B, double* out) {
    for (int m = 0; m < na; ++m) D[m] = B[m];
    if (yi < na) D[yi] += A * Cy;
    std::sort(D.begin(), D.begin() + na, [](double a, double b) { return a > b; });
    double beta = D[0] - A * Cy;
    int r = 1;
    while (r < na && beta < r * D[r]) beta += D[r++];
    beta /= r;
    for (int m = 0; m < na; ++m) {
      const double v = (beta - B[m]) / A;
      out[m] = m == yi ? std::min(Cy, v) : std::min(0.0, v);
    }
  }
};

}  // namespace

extern "C" {

int sqh_linear_mcsvm_cs(const double* X, long long l, long long d, const int* y, int K,
                        const double* Cvec, double eps, int max_iter, void* stream, double* w) {
  Rng& rng = *(Rng*)stream;
  McsCs sp(K);
  std::vector<double> alpha((size_t)l * K, 0.0), QD(l), G(K), B(K), anew(K), dval(K);
  std::vector<int> aidx((size_t)l * K), index(l), yidx(l), na_i(l, K), dind(K);
  for (int64_t k = 0; k < d * K; ++k) w[k] = 0;
  for (int64_t i = 0; i < l; ++i) {
    for (int m = 0; m < K; ++m) aidx[(size_t)i * K + m] = m;
    QD[i] = dot(X + i * d, X + i * d, d);
    yidx[i] = y[i];
    index[i] = (int)i;
  }
  // a score sits at its bound with a gradient below every free one: shrink
  auto shrunk = [&](int64_t i, int m, double a, double minG) {
    const double bound = m == yidx[i] ? Cvec[i] : 0.0;
    return a == bound && G[m] < minG;
  };
  int64_t active = l;
  double eps_shrink = std::max(10.0 * eps, 1.0);
  bool from_all = true;
  int iter = 0;
  while (iter < max_iter) {
    double stopping = -kInf;
    for (int64_t i = 0; i < active; ++i) {
      int64_t j = i + rng.bounded((uint32_t)(active - i));
      std::swap(index[i], index[j]);
    }
    for (int64_t s = 0; s < active; ++s) {
      const int64_t i = index[s];
      const double A = QD[i];
      if (!(A > 0)) continue;
      double* ai = &alpha[(size_t)i * K];
      int* ix = &aidx[(size_t)i * K];
      const double* xi = X + i * d;
      int na = na_i[i];
      for (int m = 0; m < na; ++m) G[m] = 1.0;
      if (yidx[i] < na) G[yidx[i]] = 0.0;
      for (int64_t f = 0; f < d; ++f) {
        const double v = xi[f];
        const double* wf = w + f * K;
        for (int m = 0; m < na; ++m) G[m] += wf[ix[m]] * v;
      }
      double minG = kInf, maxG = -kInf;
      for (int m = 0; m < na; ++m) {
        if (ai[ix[m]] < 0 && G[m] < minG) minG = G[m];
        if (G[m] > maxG) maxG = G[m];
      }
      if (yidx[i] < na && ai[y[i]] < Cvec[i] && G[yidx[i]] < minG) minG = G[yidx[i]];
      for (int m = 0; m < na_i[i]; ++m) {
        if (!shrunk(i, m, ai[ix[m]], minG)) continue;
        --na_i[i];
        while (na_i[i] > m) {
          const int t = na_i[i];
          if (!shrunk(i, t, ai[ix[t]], minG)) {
            std::swap(ix[m], ix[t]);
            std::swap(G[m], G[t]);
            if (yidx[i] == t) yidx[i] = m;
            else if (yidx[i] == m) yidx[i] = t;
            break;
          }
          --na_i[i];
        }
      }
      na = na_i[i];
      if (na <= 1) {
        --active;
        std::swap(index[s], index[active]);
        --s;
        continue;
      }
      if (maxG - minG <= 1e-12) continue;
      stopping = std::max(stopping, maxG - minG);
      for (int m = 0; m < na; ++m) B[m] = G[m] - A * ai[ix[m]];
      sp.sub_problem(A, yidx[i], Cvec[i], na, B.data(), anew.data());
      int nz = 0;
      for (int m = 0; m < na; ++m) {
        const double dl = anew[m] - ai[ix[m]];
        ai[ix[m]] = anew[m];
        if (std::fabs(dl) >= 1e-12) {
          dind[nz] = ix[m];
          dval[nz++] = dl;
        }
      }
      for (int64_t f = 0; f < d; ++f) {
        const double v = xi[f];
        double* wf = w + f * K;
        for (int m = 0; m < nz; ++m) wf[dind[m]] += dval[m] * v;
      }
    }
    ++iter;
    if (stopping < eps_shrink) {
      if (stopping < eps && from_all) break;
      active = l;
      for (int64_t i = 0; i < l; ++i) na_i[i] = K;
      eps_shrink = std::max(eps_shrink / 2, eps);
      from_all = true;
    } else {
      from_all = false;
    }
  }
  return iter;
}

}  // extern "C"
