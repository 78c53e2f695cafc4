// Host kernels for matrix-factorisation estimators (reference N28:
// decomposition/_cdnmf_fast.pyx and _online_lda_fast.pyx).
//
//  * sqh_cdnmf_update: one coordinate-descent sweep of NMF over the columns
//    of W in the given permutation order, using the precomputed Gram HH^T
//    and XH^T (the GEMMs happen on the device / BLAS before the call).
//    Returns the projected-gradient violation, as the reference.
//  * sqh_lda_estep: variational E-step of latent Dirichlet allocation over
//    CSR documents - per document fixed-point updates of the topic
//    distribution with the exp-digamma Dirichlet expectation, plus the
//    sufficient statistics.  Documents are independent: OpenMP over
//    documents with per-thread statistics buffers reduced at the end.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

double digamma(double x) {
  double r = 0.0;
  while (x < 6.0) {
    r -= 1.0 / x;
    x += 1.0;
  }
  double f = 1.0 / (x * x);
  double t = f * (-1.0 / 12 + f * (1.0 / 120 + f * (-1.0 / 252 + f * (1.0 / 240 +
             f * (-1.0 / 132 + f * (691.0 / 32760 + f * (-1.0 / 12)))))));
  return r + std::log(x) - 0.5 / x + t;
}

}  // namespace

extern "C" {

double sqh_cdnmf_update(double* W, const double* HHt, const double* XHt, const int64_t* perm,
                        int64_t n, int64_t k) {
  double violation = 0.0;
  for (int64_t s = 0; s < k; ++s) {
    const int64_t t = perm[s];
    const double hess = HHt[t * k + t];
    for (int64_t i = 0; i < n; ++i) {
      double* w = W + i * k;
      double grad = -XHt[i * k + t];
      for (int64_t r = 0; r < k; ++r) grad += HHt[t * k + r] * w[r];
      double pg = (w[t] == 0.0) ? std::min(0.0, grad) : grad;
      violation += std::fabs(pg);
      if (hess != 0.0) w[t] = std::max(w[t] - grad / hess, 0.0);
    }
  }
  return violation;
}

void sqh_dirichlet_expectation_2d(const double* a, int64_t rows, int64_t cols, double* out) {
  for (int64_t i = 0; i < rows; ++i) {
    double tot = 0.0;
    for (int64_t j = 0; j < cols; ++j) tot += a[i * cols + j];
    double pt = digamma(tot);
    for (int64_t j = 0; j < cols; ++j) out[i * cols + j] = digamma(a[i * cols + j]) - pt;
  }
}

// doc_topic (n x k) holds the initial distribution on entry and the result
// on exit; sstats (k x F) accumulates when non-null.
void sqh_lda_estep(const double* data, const int64_t* indices, const int64_t* indptr,
                   int64_t n_docs, int k, int64_t n_features, const double* exp_tw,
                   double prior, int max_iters, double tol, double* doc_topic, double* sstats,
                   int n_threads) {
  const double EPS = 2.220446049250313e-16;
  int nt = std::max(1, n_threads);
  std::vector<std::vector<double>> local(sstats ? nt : 0);
#pragma omp parallel num_threads(nt)
  {
    int tid = 0;
#ifdef _OPENMP
    tid = omp_get_thread_num();
#endif
    double* ss = nullptr;
    if (sstats) {
      local[tid].assign((size_t)k * n_features, 0.0);
      ss = local[tid].data();
    }
    std::vector<double> dt(k), last(k), edt(k), norm_phi, tw;
#pragma omp for schedule(dynamic, 8)
    for (int64_t d = 0; d < n_docs; ++d) {
      const int64_t s = indptr[d], e = indptr[d + 1], m = e - s;
      double* row = doc_topic + d * k;
      double tot = 0.0;
      for (int j = 0; j < k; ++j) tot += row[j];
      double pt = digamma(tot);
      for (int j = 0; j < k; ++j) { dt[j] = row[j]; edt[j] = std::exp(digamma(row[j]) - pt); }
      tw.resize((size_t)k * m);
      norm_phi.resize(m);
      for (int j = 0; j < k; ++j)
        for (int64_t t = 0; t < m; ++t) tw[j * m + t] = exp_tw[j * n_features + indices[s + t]];
      for (int it = 0; it < max_iters; ++it) {
        last = dt;
        for (int64_t t = 0; t < m; ++t) {
          double v = 0.0;
          for (int j = 0; j < k; ++j) v += edt[j] * tw[j * m + t];
          norm_phi[t] = v + EPS;
        }
        double total = 0.0;
        for (int j = 0; j < k; ++j) {
          double v = 0.0;
          for (int64_t t = 0; t < m; ++t) v += data[s + t] / norm_phi[t] * tw[j * m + t];
          dt[j] = edt[j] * v + prior;
          total += dt[j];
        }
        double ptot = digamma(total);
        for (int j = 0; j < k; ++j) edt[j] = std::exp(digamma(dt[j]) - ptot);
        double mc = 0.0;
        for (int j = 0; j < k; ++j) mc += std::fabs(last[j] - dt[j]);
        if (mc / k < tol) break;
      }
      for (int j = 0; j < k; ++j) row[j] = dt[j];
      if (ss) {
        for (int64_t t = 0; t < m; ++t) {
          double v = 0.0;
          for (int j = 0; j < k; ++j) v += edt[j] * tw[j * m + t];
          norm_phi[t] = v + EPS;
        }
        for (int j = 0; j < k; ++j)
          for (int64_t t = 0; t < m; ++t)
            ss[j * n_features + indices[s + t]] += edt[j] * data[s + t] / norm_phi[t];
      }
    }
  }
  if (sstats) {
    std::memset(sstats, 0, sizeof(double) * (size_t)k * n_features);
    for (auto& l : local)
      for (size_t i = 0; i < l.size(); ++i) sstats[i] += l[i];
  }
}

}  // extern "C"
