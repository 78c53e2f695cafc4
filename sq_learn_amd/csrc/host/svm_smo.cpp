// SMO solvers of libsvm (reference ``svm/src/libsvm/svm.cpp``:
// ``Solver::Solve`` :658, second-order working-set selection ``:935``,
// ``calculate_rho``, ``Solver_NU`` :1158, ``solve_c_svc`` / ``nu_svc`` /
// ``one_class`` / ``epsilon_svr`` / ``nu_svr`` :1589-1831).
//
// MI355X split of work: the kernel matrix is a GEMM (+ elementwise
// epilogue) and is formed on the GPU (or with BLAS on a CPU-only host) by the
// Python layer; this file runs the inherently sequential two-variable SMO
// iterations on the host over that dense matrix.  Variables map to kernel
// rows through ``idx`` (l for classification / one-class, 2l for the SVR
// doubled problem) with signs ``y`` (+1 / -1), so every libsvm formulation
// is one call: Q_ij = y_i y_j K[idx_i, idx_j].  Per-variable upper bounds C_i
// carry class weights and sample weights (the reference's per-instance C).
// No shrinking: the optimum and rho are the same; shrinking only saves time
// on problems far larger than a dense kernel allows.
#include <cmath>
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

constexpr double kTau = 1e-12;
constexpr double kInf = INFINITY;

struct Problem {
  int64_t l;             // number of variables
  const double* K;       // n x n kernel (row-major)
  int64_t n;
  const int32_t* idx;    // variable -> kernel row
  const int8_t* y;       // +1 / -1
  const double* p;       // linear term
  const double* C;       // per-variable upper bound
  double eps;
  int64_t max_iter;
  inline double Q(int64_t i, int64_t j) const {
    return (double)(y[i] * y[j]) * K[(int64_t)idx[i] * n + idx[j]];
  }
  inline double QD(int64_t i) const { return K[(int64_t)idx[i] * n + idx[i]]; }
};

struct Solver {
  const Problem& P;
  std::vector<double> alpha, G, QD;
  std::vector<int8_t> status;   // 0 lower, 1 upper, 2 free
  std::vector<double> Qi, Qj;
  explicit Solver(const Problem& p) : P(p) {}

  void update_status(int64_t i) {
    status[i] = alpha[i] >= P.C[i] ? 1 : (alpha[i] <= 0 ? 0 : 2);
  }
  bool upper(int64_t i) const { return status[i] == 1; }
  bool lower(int64_t i) const { return status[i] == 0; }

  void row(int64_t i, std::vector<double>& out) {
    const double* Kr = P.K + (int64_t)P.idx[i] * P.n;
    const double yi = P.y[i];
    for (int64_t j = 0; j < P.l; ++j) out[j] = yi * P.y[j] * Kr[P.idx[j]];
  }

  void init(const double* alpha0) {
    const int64_t l = P.l;
    alpha.assign(alpha0, alpha0 + l);
    status.resize(l);
    for (int64_t i = 0; i < l; ++i) update_status(i);
    QD.resize(l);
    for (int64_t i = 0; i < l; ++i) QD[i] = P.QD(i);
    G.assign(P.p, P.p + l);
    Qi.resize(l);
    Qj.resize(l);
    for (int64_t i = 0; i < l; ++i) {
      if (!lower(i)) {
        row(i, Qi);
        for (int64_t j = 0; j < l; ++j) G[j] += alpha[i] * Qi[j];
      }
    }
  }

  // two-variable update (reference Solver::Solve inner step)
  void update_pair(int64_t i, int64_t j) {
    row(i, Qi);
    row(j, Qj);
    const double Ci = P.C[i], Cj = P.C[j];
    const double ai = alpha[i], aj = alpha[j];
    if (P.y[i] != P.y[j]) {
      double qc = QD[i] + QD[j] + 2 * Qi[j];
      if (qc <= 0) qc = kTau;
      double delta = (-G[i] - G[j]) / qc;
      double diff = alpha[i] - alpha[j];
      alpha[i] += delta;
      alpha[j] += delta;
      if (diff > 0) { if (alpha[j] < 0) { alpha[j] = 0; alpha[i] = diff; } }
      else { if (alpha[i] < 0) { alpha[i] = 0; alpha[j] = -diff; } }
      if (diff > Ci - Cj) { if (alpha[i] > Ci) { alpha[i] = Ci; alpha[j] = Ci - diff; } }
      else { if (alpha[j] > Cj) { alpha[j] = Cj; alpha[i] = Cj + diff; } }
    } else {
      double qc = QD[i] + QD[j] - 2 * Qi[j];
      if (qc <= 0) qc = kTau;
      double delta = (G[i] - G[j]) / qc;
      double sum = alpha[i] + alpha[j];
      alpha[i] -= delta;
      alpha[j] += delta;
      if (sum > Ci) { if (alpha[i] > Ci) { alpha[i] = Ci; alpha[j] = sum - Ci; } }
      else { if (alpha[j] < 0) { alpha[j] = 0; alpha[i] = sum; } }
      if (sum > Cj) { if (alpha[j] > Cj) { alpha[j] = Cj; alpha[i] = sum - Cj; } }
      else { if (alpha[i] < 0) { alpha[i] = 0; alpha[j] = sum; } }
    }
    const double dai = alpha[i] - ai, daj = alpha[j] - aj;
    for (int64_t k = 0; k < P.l; ++k) G[k] += Qi[k] * dai + Qj[k] * daj;
    update_status(i);
    update_status(j);
  }

  // ------------------------------------------------------------ C-type
  bool select(int64_t* out_i, int64_t* out_j) {
    double Gmax = -kInf, Gmax2 = -kInf, obj_min = kInf;
    int64_t imax = -1, jmin = -1;
    for (int64_t t = 0; t < P.l; ++t) {
      if (P.y[t] == 1) { if (!upper(t) && -G[t] >= Gmax) { Gmax = -G[t]; imax = t; } }
      else { if (!lower(t) && G[t] >= Gmax) { Gmax = G[t]; imax = t; } }
    }
    const int64_t i = imax;
    if (i != -1) row(i, Qi);
    for (int64_t j = 0; j < P.l; ++j) {
      if (P.y[j] == 1) {
        if (!lower(j)) {
          double gd = Gmax + G[j];
          if (G[j] >= Gmax2) Gmax2 = G[j];
          if (gd > 0 && i != -1) {
            double qc = QD[i] + QD[j] - 2.0 * P.y[i] * Qi[j];
            double od = -(gd * gd) / (qc > 0 ? qc : kTau);
            if (od <= obj_min) { jmin = j; obj_min = od; }
          }
        }
      } else {
        if (!upper(j)) {
          double gd = Gmax - G[j];
          if (-G[j] >= Gmax2) Gmax2 = -G[j];
          if (gd > 0 && i != -1) {
            double qc = QD[i] + QD[j] + 2.0 * P.y[i] * Qi[j];
            double od = -(gd * gd) / (qc > 0 ? qc : kTau);
            if (od <= obj_min) { jmin = j; obj_min = od; }
          }
        }
      }
    }
    if (Gmax + Gmax2 < P.eps || jmin == -1) return true;
    *out_i = imax;
    *out_j = jmin;
    return false;
  }

  double rho() const {
    double ub = kInf, lb = -kInf, sum_free = 0;
    int64_t nr_free = 0;
    for (int64_t i = 0; i < P.l; ++i) {
      double yG = P.y[i] * G[i];
      if (upper(i)) { if (P.y[i] == -1) ub = std::min(ub, yG); else lb = std::max(lb, yG); }
      else if (lower(i)) { if (P.y[i] == 1) ub = std::min(ub, yG); else lb = std::max(lb, yG); }
      else { ++nr_free; sum_free += yG; }
    }
    return nr_free > 0 ? sum_free / nr_free : (ub + lb) / 2;
  }

  // ------------------------------------------------------------ nu-type
  bool select_nu(int64_t* out_i, int64_t* out_j) {
    double Gmaxp = -kInf, Gmaxp2 = -kInf, Gmaxn = -kInf, Gmaxn2 = -kInf, obj_min = kInf;
    int64_t ip = -1, in = -1, jmin = -1;
    for (int64_t t = 0; t < P.l; ++t) {
      if (P.y[t] == 1) { if (!upper(t) && -G[t] >= Gmaxp) { Gmaxp = -G[t]; ip = t; } }
      else { if (!lower(t) && G[t] >= Gmaxn) { Gmaxn = G[t]; in = t; } }
    }
    std::vector<double>& Qip = Qi;
    std::vector<double>& Qin = Qj;
    if (ip != -1) row(ip, Qip);
    if (in != -1) row(in, Qin);
    for (int64_t j = 0; j < P.l; ++j) {
      if (P.y[j] == 1) {
        if (!lower(j)) {
          double gd = Gmaxp + G[j];
          if (G[j] >= Gmaxp2) Gmaxp2 = G[j];
          if (gd > 0 && ip != -1) {
            double qc = QD[ip] + QD[j] - 2 * Qip[j];
            double od = -(gd * gd) / (qc > 0 ? qc : kTau);
            if (od <= obj_min) { jmin = j; obj_min = od; }
          }
        }
      } else {
        if (!upper(j)) {
          double gd = Gmaxn - G[j];
          if (-G[j] >= Gmaxn2) Gmaxn2 = -G[j];
          if (gd > 0 && in != -1) {
            double qc = QD[in] + QD[j] - 2 * Qin[j];
            double od = -(gd * gd) / (qc > 0 ? qc : kTau);
            if (od <= obj_min) { jmin = j; obj_min = od; }
          }
        }
      }
    }
    if (std::max(Gmaxp + Gmaxp2, Gmaxn + Gmaxn2) < P.eps || jmin == -1) return true;
    *out_i = P.y[jmin] == 1 ? ip : in;
    *out_j = jmin;
    return false;
  }

  void rho_nu(double* rho_out, double* r_out) const {
    int64_t nf1 = 0, nf2 = 0;
    double ub1 = kInf, ub2 = kInf, lb1 = -kInf, lb2 = -kInf, sf1 = 0, sf2 = 0;
    for (int64_t i = 0; i < P.l; ++i) {
      if (P.y[i] == 1) {
        if (upper(i)) lb1 = std::max(lb1, G[i]);
        else if (lower(i)) ub1 = std::min(ub1, G[i]);
        else { ++nf1; sf1 += G[i]; }
      } else {
        if (upper(i)) lb2 = std::max(lb2, G[i]);
        else if (lower(i)) ub2 = std::min(ub2, G[i]);
        else { ++nf2; sf2 += G[i]; }
      }
    }
    double r1 = nf1 > 0 ? sf1 / nf1 : (ub1 + lb1) / 2;
    double r2 = nf2 > 0 ? sf2 / nf2 : (ub2 + lb2) / 2;
    *r_out = (r1 + r2) / 2;
    *rho_out = (r1 - r2) / 2;
  }

  int run(bool nu) {
    int64_t it = 0;
    int status_code = 0;
    while (true) {
      if (P.max_iter > 0 && it >= P.max_iter) { status_code = 1; break; }
      int64_t i, j;
      bool done = nu ? select_nu(&i, &j) : select(&i, &j);
      if (done) break;
      ++it;
      update_pair(i, j);
    }
    return status_code;
  }

  double objective() const {
    double v = 0;
    for (int64_t i = 0; i < P.l; ++i) v += alpha[i] * (G[i] + P.p[i]);
    return v / 2;
  }
};

}  // namespace

extern "C" {

// Solve one libsvm sub-problem.  mode 0: C-type (C-SVC, eps-SVR, one-class);
// mode 1: nu-type (nu-SVC, nu-SVR).  alpha: in = initial point, out = solution.
// out: [rho, r (nu only), objective, n_iter_status]
void sqh_svm_solve(const double* K, long long n, const int32_t* idx, const int8_t* y,
                   const double* p, const double* C, long long l, double eps, long long max_iter,
                   int mode, double* alpha, double* out) {
  Problem P{l, K, n, idx, y, p, C, eps, max_iter};
  Solver S(P);
  S.init(alpha);
  int st = S.run(mode == 1);
  for (int64_t i = 0; i < l; ++i) alpha[i] = S.alpha[i];
  if (mode == 1) S.rho_nu(&out[0], &out[1]);
  else { out[0] = S.rho(); out[1] = 0; }
  out[2] = S.objective();
  out[3] = st;
}

}  // extern "C"
