// SMO solvers of libsvm (reference ``svm/src/libsvm/svm.cpp``:
// ``Solver::Solve`` :658, second-order working-set selection ``:935``,
// shrinking ``do_shrinking`` / ``be_shrunk`` / ``reconstruct_gradient``,
// ``calculate_rho``, ``Solver_NU`` :1158, ``solve_c_svc`` / ``nu_svc`` /
// ``one_class`` / ``epsilon_svr`` / ``nu_svr`` :1589-1831, ``Cache`` :70).
//
// Variables map to kernel rows through ``idx`` (l for classification /
// one-class, 2l for the SVR doubled problem) with signs ``y`` (+1 / -1), so
// every libsvm formulation is one call: Q_ij = y_i y_j K[idx_i, idx_j].
// Per-variable upper bounds C_i carry class weights and sample weights.
//
// Kernel rows come from a KernelSource:
//   * dense: the n x n kernel formed beforehand as one GEMM + epilogue on
//     the GPU (small / medium problems: every row is a pointer);
//   * computed: rows evaluated on demand from the training rows (dense fp64
//     or CSR, never densified) with OpenMP over the row's n entries, held in
//     an LRU cache of ``cache_bytes`` (the reference's ``cache_size``) - O(n)
//     memory beyond the cache, so the problem size is bounded by time, not
//     by an n x n matrix.
// Shrinking (libsvm's heuristic): every min(l, 1000) iterations the
// variables stuck at a bound whose gradient says they will stay there leave
// the active set; the selection and gradient updates then run over the
// active prefix of a variable permutation, and the full gradient is rebuilt
// from G_bar (sum of C_j Q_j over upper-bounded j) plus the free variables
// before the final optimality check and rho.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <unordered_map>
#include <vector>

#include "host.h"

namespace {

constexpr double kTau = 1e-12;
constexpr double kInf = INFINITY;

struct KernelSource {
  int64_t n = 0;
  // dense
  const double* K = nullptr;
  // computed
  int type = 0;   // 0 linear, 1 poly, 2 rbf, 3 sigmoid
  const double* X = nullptr;   // dense n x d
  int64_t d = 0;
  const int64_t* indptr = nullptr;   // CSR alternative
  const int32_t* indices = nullptr;
  const double* data = nullptr;
  double gamma = 0, coef0 = 0;
  int degree = 3;
  std::vector<double> sq;
  // LRU cache of computed rows (most recent at the front)
  size_t cap = 2;
  std::list<std::pair<int64_t, std::vector<double>>> lru;
  std::unordered_map<int64_t, std::list<std::pair<int64_t, std::vector<double>>>::iterator> where;
  std::vector<double> dense_row;   // scatter buffer of a CSR row
  int64_t hits = 0, misses = 0;

  double kfun(double dot, int64_t a, int64_t b) const {
    switch (type) {
      case 0: return dot;
      case 1: return std::pow(gamma * dot + coef0, degree);
      case 2: return a == b ? 1.0 : std::exp(-gamma * std::max(sq[a] + sq[b] - 2.0 * dot, 0.0));
      default: return std::tanh(gamma * dot + coef0);
    }
  }

  double dot_dense(int64_t a, int64_t b) const {
    const double* xa = X + a * d;
    const double* xb = X + b * d;
    double s = 0.0;
    for (int64_t f = 0; f < d; ++f) s += xa[f] * xb[f];
    return s;
  }

  double dot_csr(int64_t a, int64_t b) const {
    // sorted-index merge of two sparse rows
    int64_t p = indptr[a], pe = indptr[a + 1], q = indptr[b], qe = indptr[b + 1];
    double s = 0.0;
    while (p < pe && q < qe) {
      if (indices[p] == indices[q]) s += data[p++] * data[q++];
      else if (indices[p] < indices[q]) ++p;
      else ++q;
    }
    return s;
  }

  void prepare(size_t cache_bytes) {
    if (K) return;
    sq.assign(n, 0.0);
    for (int64_t i = 0; i < n; ++i) sq[i] = indptr ? dot_csr(i, i) : dot_dense(i, i);
    cap = std::max<size_t>(2, cache_bytes / (sizeof(double) * (size_t)std::max<int64_t>(n, 1)));
    if (indptr) dense_row.assign(d, 0.0);
  }

  double eval(int64_t a, int64_t b) const {
    if (K) return K[a * n + b];
    return kfun(indptr ? dot_csr(a, b) : dot_dense(a, b), a, b);
  }

  const double* row(int64_t r) {
    if (K) return K + r * n;
    auto it = where.find(r);
    if (it != where.end()) {
      ++hits;
      lru.splice(lru.begin(), lru, it->second);
      return lru.front().second.data();
    }
    ++misses;
    std::vector<double> v;
    if (lru.size() >= cap) {   // recycle the least recently used row's storage
      v.swap(lru.back().second);
      where.erase(lru.back().first);
      lru.pop_back();
    }
    v.resize(n);
    if (indptr) {
      for (int64_t p = indptr[r]; p < indptr[r + 1]; ++p) dense_row[indices[p]] = data[p];
      const double* xr = dense_row.data();
#pragma omp parallel for schedule(static) if (n > 4096)
      for (int64_t j = 0; j < n; ++j) {
        double s = 0.0;
        for (int64_t p = indptr[j]; p < indptr[j + 1]; ++p) s += data[p] * xr[indices[p]];
        v[j] = kfun(s, r, j);
      }
      for (int64_t p = indptr[r]; p < indptr[r + 1]; ++p) dense_row[indices[p]] = 0.0;
    } else {
#pragma omp parallel for schedule(static) if (n > 4096)
      for (int64_t j = 0; j < n; ++j) v[j] = kfun(dot_dense(r, j), r, j);
    }
    lru.emplace_front(r, std::move(v));
    where[r] = lru.begin();
    return lru.front().second.data();
  }
};

struct Problem {
  int64_t l;             // number of variables
  KernelSource* ks;
  const int32_t* idx;    // variable -> kernel row
  const int8_t* y;       // +1 / -1
  const double* p;       // linear term
  const double* C;       // per-variable upper bound
  double eps;
  int64_t max_iter;
  bool shrinking;
};

struct Solver {
  const Problem& P;
  int64_t l;
  std::vector<double> alpha, G, G_bar, QD;
  std::vector<int8_t> status;   // 0 lower, 1 upper, 2 free
  std::vector<int64_t> order;   // variables; the first `active` are active
  int64_t active;
  bool unshrink = false;
  std::vector<double> Qi, Qj;
  explicit Solver(const Problem& p) : P(p), l(p.l) {}

  void update_status(int64_t i) {
    status[i] = alpha[i] >= P.C[i] ? 1 : (alpha[i] <= 0 ? 0 : 2);
  }
  bool upper(int64_t i) const { return status[i] == 1; }
  bool lower(int64_t i) const { return status[i] == 0; }
  bool is_free(int64_t i) const { return status[i] == 2; }

  // Q row of variable i over the first `upto` variables of `order`
  void qrow(int64_t i, std::vector<double>& out, int64_t upto) {
    const double* Kr = P.ks->row(P.idx[i]);
    const double yi = P.y[i];
    for (int64_t k = 0; k < upto; ++k) {
      const int64_t j = order[k];
      out[j] = yi * P.y[j] * Kr[P.idx[j]];
    }
  }

  void init(const double* alpha0) {
    alpha.assign(alpha0, alpha0 + l);
    status.resize(l);
    for (int64_t i = 0; i < l; ++i) update_status(i);
    QD.resize(l);
    for (int64_t i = 0; i < l; ++i) QD[i] = P.ks->eval(P.idx[i], P.idx[i]);
    order.resize(l);
    for (int64_t i = 0; i < l; ++i) order[i] = i;
    active = l;
    G.assign(P.p, P.p + l);
    G_bar.assign(l, 0.0);
    Qi.resize(l);
    Qj.resize(l);
    for (int64_t i = 0; i < l; ++i) {
      if (!lower(i)) {
        qrow(i, Qi, l);
        for (int64_t j = 0; j < l; ++j) G[j] += alpha[i] * Qi[j];
        if (upper(i))
          for (int64_t j = 0; j < l; ++j) G_bar[j] += P.C[i] * Qi[j];
      }
    }
  }

  // two-variable update (reference Solver::Solve inner step)
  void update_pair(int64_t i, int64_t j) {
    qrow(i, Qi, l);
    qrow(j, Qj, l);
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
    for (int64_t k = 0; k < active; ++k) {
      const int64_t t = order[k];
      G[t] += Qi[t] * dai + Qj[t] * daj;
    }
    const bool ui = upper(i), uj = upper(j);
    update_status(i);
    update_status(j);
    // G_bar over every variable when an upper-bound status flips
    if (ui != upper(i)) {
      const double s = upper(i) ? Ci : -Ci;
      for (int64_t k = 0; k < l; ++k) G_bar[k] += s * Qi[k];
    }
    if (uj != upper(j)) {
      const double s = upper(j) ? Cj : -Cj;
      for (int64_t k = 0; k < l; ++k) G_bar[k] += s * Qj[k];
    }
  }

  // the gradient of the inactive (shrunk, at-bound) variables from G_bar
  // and the free active variables; then every variable is active again
  void reconstruct_gradient() {
    if (active == l) return;
    for (int64_t k = active; k < l; ++k) {
      const int64_t j = order[k];
      G[j] = G_bar[j] + P.p[j];
    }
    for (int64_t k = 0; k < active; ++k) {
      const int64_t i = order[k];
      if (!is_free(i)) continue;
      const double* Kr = P.ks->row(P.idx[i]);
      const double ai = alpha[i] * P.y[i];
      for (int64_t m = active; m < l; ++m) {
        const int64_t j = order[m];
        G[j] += ai * P.y[j] * Kr[P.idx[j]];
      }
    }
    active = l;
  }

  // ------------------------------------------------------------ C-type
  bool select(int64_t* out_i, int64_t* out_j) {
    double Gmax = -kInf, Gmax2 = -kInf, obj_min = kInf;
    int64_t imax = -1, jmin = -1;
    for (int64_t k = 0; k < active; ++k) {
      const int64_t t = order[k];
      if (P.y[t] == 1) { if (!upper(t) && -G[t] >= Gmax) { Gmax = -G[t]; imax = t; } }
      else { if (!lower(t) && G[t] >= Gmax) { Gmax = G[t]; imax = t; } }
    }
    const int64_t i = imax;
    if (i != -1) qrow(i, Qi, active);
    for (int64_t k = 0; k < active; ++k) {
      const int64_t j = order[k];
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

  bool be_shrunk(int64_t i, double Gmax1, double Gmax2) const {
    if (upper(i)) return P.y[i] == 1 ? -G[i] > Gmax1 : -G[i] > Gmax2;
    if (lower(i)) return P.y[i] == 1 ? G[i] > Gmax2 : G[i] > Gmax1;
    return false;
  }

  void do_shrinking() {
    double Gmax1 = -kInf, Gmax2 = -kInf;
    for (int64_t k = 0; k < active; ++k) {
      const int64_t i = order[k];
      if (P.y[i] == 1) {
        if (!upper(i)) Gmax1 = std::max(Gmax1, -G[i]);
        if (!lower(i)) Gmax2 = std::max(Gmax2, G[i]);
      } else {
        if (!upper(i)) Gmax2 = std::max(Gmax2, -G[i]);
        if (!lower(i)) Gmax1 = std::max(Gmax1, G[i]);
      }
    }
    if (!unshrink && Gmax1 + Gmax2 <= P.eps * 10) {
      unshrink = true;
      reconstruct_gradient();
    }
    for (int64_t k = 0; k < active;) {
      if (be_shrunk(order[k], Gmax1, Gmax2)) std::swap(order[k], order[--active]);
      else ++k;
    }
  }

  double rho() const {
    double ub = kInf, lb = -kInf, sum_free = 0;
    int64_t nr_free = 0;
    for (int64_t i = 0; i < l; ++i) {
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
    for (int64_t k = 0; k < active; ++k) {
      const int64_t t = order[k];
      if (P.y[t] == 1) { if (!upper(t) && -G[t] >= Gmaxp) { Gmaxp = -G[t]; ip = t; } }
      else { if (!lower(t) && G[t] >= Gmaxn) { Gmaxn = G[t]; in = t; } }
    }
    std::vector<double>& Qip = Qi;
    std::vector<double>& Qin = Qj;
    if (ip != -1) qrow(ip, Qip, active);
    if (in != -1) qrow(in, Qin, active);
    for (int64_t k = 0; k < active; ++k) {
      const int64_t j = order[k];
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

  bool be_shrunk_nu(int64_t i, double G1, double G2, double G3, double G4) const {
    if (upper(i)) return P.y[i] == 1 ? -G[i] > G1 : -G[i] > G4;
    if (lower(i)) return P.y[i] == 1 ? G[i] > G2 : G[i] > G3;
    return false;
  }

  void do_shrinking_nu() {
    double G1 = -kInf, G2 = -kInf, G3 = -kInf, G4 = -kInf;
    for (int64_t k = 0; k < active; ++k) {
      const int64_t i = order[k];
      if (!upper(i)) {
        if (P.y[i] == 1) G1 = std::max(G1, -G[i]);
        else G4 = std::max(G4, -G[i]);
      }
      if (!lower(i)) {
        if (P.y[i] == 1) G2 = std::max(G2, G[i]);
        else G3 = std::max(G3, G[i]);
      }
    }
    if (!unshrink && std::max(G1 + G2, G3 + G4) <= P.eps * 10) {
      unshrink = true;
      reconstruct_gradient();
    }
    for (int64_t k = 0; k < active;) {
      if (be_shrunk_nu(order[k], G1, G2, G3, G4)) std::swap(order[k], order[--active]);
      else ++k;
    }
  }

  void rho_nu(double* rho_out, double* r_out) const {
    int64_t nf1 = 0, nf2 = 0;
    double ub1 = kInf, ub2 = kInf, lb1 = -kInf, lb2 = -kInf, sf1 = 0, sf2 = 0;
    for (int64_t i = 0; i < l; ++i) {
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

  int run(bool nu, int64_t* iters) {
    int64_t it = 0;
    int status_code = 0;
    int64_t counter = std::min<int64_t>(l, 1000) + 1;
    while (true) {
      if (P.max_iter > 0 && it >= P.max_iter) { status_code = 1; break; }
      if (--counter == 0) {
        counter = std::min<int64_t>(l, 1000);
        if (P.shrinking) { if (nu) do_shrinking_nu(); else do_shrinking(); }
      }
      int64_t i, j;
      bool done = nu ? select_nu(&i, &j) : select(&i, &j);
      if (done) {
        if (active == l) break;
        // optimal on the active set: rebuild the whole gradient and check
        // every variable once more
        reconstruct_gradient();
        done = nu ? select_nu(&i, &j) : select(&i, &j);
        if (done) break;
        counter = 1;   // shrink again at the next iteration
      }
      ++it;
      update_pair(i, j);
    }
    reconstruct_gradient();   // (max_iter exit) rho needs every gradient
    *iters = it;
    return status_code;
  }

  double objective() const {
    double v = 0;
    for (int64_t i = 0; i < l; ++i) v += alpha[i] * (G[i] + P.p[i]);
    return v / 2;
  }
};

void solve(KernelSource& ks, const int32_t* idx, const int8_t* y, const double* p,
           const double* C, long long l, double eps, long long max_iter, int mode, int shrinking,
           double* alpha, double* out) {
  Problem P{l, &ks, idx, y, p, C, eps, max_iter, shrinking != 0};
  Solver S(P);
  S.init(alpha);
  int64_t iters = 0;
  int st = S.run(mode == 1, &iters);
  for (int64_t i = 0; i < l; ++i) alpha[i] = S.alpha[i];
  if (mode == 1) S.rho_nu(&out[0], &out[1]);
  else { out[0] = S.rho(); out[1] = 0; }
  out[2] = S.objective();
  out[3] = st;
  out[4] = (double)iters;
  out[5] = (double)ks.hits;
  out[6] = (double)ks.misses;
}

}  // namespace

extern "C" {

// Solve one libsvm sub-problem over a dense n x n kernel.  mode 0: C-type
// (C-SVC, eps-SVR, one-class); mode 1: nu-type (nu-SVC, nu-SVR).
// alpha: in = initial point, out = solution.
// out: [rho, r (nu only), objective, status, iterations, cache hits, misses]
void sqh_svm_solve(const double* K, long long n, const int32_t* idx, const int8_t* y,
                   const double* p, const double* C, long long l, double eps, long long max_iter,
                   int mode, int shrinking, double* alpha, double* out) {
  KernelSource ks;
  ks.n = n;
  ks.K = K;
  solve(ks, idx, y, p, C, l, eps, max_iter, mode, shrinking, alpha, out);
}

// Same, with kernel rows computed on demand from the n training rows (dense
// X n x d when indptr is null, else CSR indptr / indices / data with d
// columns) and kept in an LRU cache of cache_bytes.  ktype: 0 linear,
// 1 poly, 2 rbf, 3 sigmoid.
void sqh_svm_solve_rows(const double* X, const long long* indptr, const int32_t* indices,
                        const double* data, long long n, long long d, int ktype, double gamma,
                        double coef0, int degree, long long cache_bytes, const int32_t* idx,
                        const int8_t* y, const double* p, const double* C, long long l,
                        double eps, long long max_iter, int mode, int shrinking, double* alpha,
                        double* out) {
  KernelSource ks;
  ks.n = n;
  ks.d = d;
  ks.type = ktype;
  ks.X = X;
  ks.indptr = (const int64_t*)indptr;
  ks.indices = indices;
  ks.data = data;
  ks.gamma = gamma;
  ks.coef0 = coef0;
  ks.degree = degree;
  ks.prepare((size_t)std::max<long long>(cache_bytes, 0));
  solve(ks, idx, y, p, C, l, eps, max_iter, mode, shrinking, alpha, out);
}

// kernel rows [r0, r1) of the computed source against all n rows (for the
// decision values of held-out rows when no dense kernel exists)
void sqh_svm_kernel_rows(const double* X, const long long* indptr, const int32_t* indices,
                         const double* data, long long n, long long d, int ktype, double gamma,
                         double coef0, int degree, const int32_t* rows, long long m,
                         const int32_t* cols, long long nc, double* out) {
  KernelSource ks;
  ks.n = n;
  ks.d = d;
  ks.type = ktype;
  ks.X = X;
  ks.indptr = (const int64_t*)indptr;
  ks.indices = indices;
  ks.data = data;
  ks.gamma = gamma;
  ks.coef0 = coef0;
  ks.degree = degree;
  ks.prepare(0);
#pragma omp parallel for schedule(static)
  for (long long a = 0; a < m; ++a)
    for (long long b = 0; b < nc; ++b) out[a * nc + b] = ks.eval(rows[a], cols[b]);
}

}  // extern "C"
