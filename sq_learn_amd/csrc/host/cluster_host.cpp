// Host kernels for clustering utilities:
//   * DBSCAN cluster expansion (reference ``cluster/_dbscan_inner.pyx:21``):
//     depth-first growth from each unlabelled core sample over the
//     precomputed radius-neighbourhood graph (CSR), non-core samples are
//     border points that join the first cluster reaching them;
//   * expected mutual information of a contingency table under the
//     hypergeometric model (reference
//     ``metrics/cluster/_expected_mutual_info_fast.pyx``), OpenMP over rows.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "host.h"

extern "C" {

void sqh_dbscan_inner(const uint8_t* is_core, const int64_t* indptr, const int64_t* indices,
                      long long n, int64_t* labels) {
  std::vector<int64_t> stack;
  int64_t label = 0;
  for (long long s = 0; s < n; ++s) {
    if (labels[s] != -1 || !is_core[s]) continue;
    int64_t i = s;
    while (true) {
      if (labels[i] == -1) {
        labels[i] = label;
        if (is_core[i]) {
          for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) {
            const int64_t v = indices[e];
            if (labels[v] == -1) stack.push_back(v);
          }
        }
      }
      if (stack.empty()) break;
      i = stack.back();
      stack.pop_back();
    }
    ++label;
  }
}

// a: row sums (R), b: column sums (C), N: total.  Returns E[MI] in nats.
double sqh_expected_mutual_info(const int64_t* a, long long R, const int64_t* b, long long C,
                                long long N) {
  if (N <= 1) return 0.0;
  long long maxab = 0;
  for (long long i = 0; i < R; ++i) maxab = std::max<long long>(maxab, a[i]);
  for (long long j = 0; j < C; ++j) maxab = std::max<long long>(maxab, b[j]);
  // log(nij / N) and lgamma(nij + 1) tables for nij = 0 .. maxab
  std::vector<double> log_nij(maxab + 1), gln_nij(maxab + 1);
  for (long long v = 0; v <= maxab; ++v) {
    log_nij[v] = v > 0 ? std::log((double)v) : 0.0;
    gln_nij[v] = std::lgamma((double)v + 1.0);
  }
  const double logN = std::log((double)N);
  const double gln_N = std::lgamma((double)N + 1.0);
  double emi = 0.0;
#pragma omp parallel for reduction(+ : emi) schedule(dynamic)
  for (long long i = 0; i < R; ++i) {
    const double ai = (double)a[i];
    const double gln_a = std::lgamma(ai + 1.0), gln_Na = std::lgamma((double)N - ai + 1.0);
    for (long long j = 0; j < C; ++j) {
      const double bj = (double)b[j];
      const double gln_b = std::lgamma(bj + 1.0), gln_Nb = std::lgamma((double)N - bj + 1.0);
      const long long lo = std::max<long long>(1, a[i] - N + b[j]);
      const long long hi = std::min<long long>(a[i], b[j]) + 1;
      const double log_ab = std::log(ai) + std::log(bj);
      for (long long nij = lo; nij < hi; ++nij) {
        const double term1 = (double)nij / (double)N;
        const double term2 = logN + log_nij[nij] - log_ab;
        const double gln = gln_a + gln_b + gln_Na + gln_Nb - gln_N - gln_nij[nij] -
                           std::lgamma(ai - (double)nij + 1.0) -
                           std::lgamma(bj - (double)nij + 1.0) -
                           std::lgamma((double)N - ai - bj + (double)nij + 1.0);
        emi += term1 * term2 * std::exp(gln);
      }
    }
  }
  return emi;
}

}  // extern "C"

// OPTICS ordering (reference cluster/_optics.py:compute_optics_graph and
// _set_reach_dist): repeatedly take the unprocessed point of smallest
// reachability (first index on ties) and relax the reachability of the
// unprocessed points within max_eps of it.  Distances are minkowski-p on
// the fly (p = inf for chebyshev); reachabilities are rounded to 15
// decimals exactly like np.around, so the ordering matches the reference.
extern "C" void sqh_optics_order(const double* X, int64_t n, int64_t d, const double* core,
                                 double max_eps, double p, double* reach, int64_t* pred,
                                 int64_t* ordering) {
  std::vector<uint8_t> done(n, 0);
  for (int64_t i = 0; i < n; ++i) { reach[i] = INFINITY; pred[i] = -1; }
  auto rnd = [](double v) {
    if (!std::isfinite(v)) return v;
    double y = v * 1e15;
    if (std::fabs(y) >= 4503599627370496.0) return v;
    return std::nearbyint(y) / 1e15;
  };
  for (int64_t step = 0; step < n; ++step) {
    int64_t pt = -1;
    double best = INFINITY;
    for (int64_t j = 0; j < n; ++j) {
      if (done[j]) continue;
      if (pt < 0 || reach[j] < best) { pt = j; best = reach[j]; }
    }
    done[pt] = 1;
    ordering[step] = pt;
    if (!std::isfinite(core[pt])) continue;
    const double* xp = X + pt * d;
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < n; ++j) {
      if (done[j]) continue;
      const double* xj = X + j * d;
      double s = 0.0;
      if (std::isinf(p)) {
        for (int64_t k = 0; k < d; ++k) s = std::max(s, std::fabs(xp[k] - xj[k]));
      } else if (p == 2.0) {
        // the reference's euclidean_distances expansion: -2 x.y + |x|^2 + |y|^2
        double dot = 0.0, xx = 0.0, yy = 0.0;
        for (int64_t k = 0; k < d; ++k) {
          dot += xp[k] * xj[k];
          xx += xp[k] * xp[k];
          yy += xj[k] * xj[k];
        }
        s = -2.0 * dot + xx + yy;
        s = std::sqrt(std::max(s, 0.0));
      } else if (p == 1.0) {
        for (int64_t k = 0; k < d; ++k) s += std::fabs(xp[k] - xj[k]);
      } else {
        for (int64_t k = 0; k < d; ++k) s += std::pow(std::fabs(xp[k] - xj[k]), p);
        s = std::pow(s, 1.0 / p);
      }
      if (s > max_eps) continue;
      double rd = rnd(std::max(s, core[pt]));
      if (rd < reach[j]) { reach[j] = rd; pred[j] = pt; }
    }
  }
}

// Norm groups of the ipe16 IPE screen (ops.kmeans.Ipe16.group_tiles): the
// first tile of each of G contiguous tile ranges of the |c|^2-sorted
// centroids minimising sum_g (centroids in g) x (|c|^2 range of g), by a DP
// over tile cuts - the same fp64 expressions and first-minimum ties as the
// numpy version, once per IPE step on the host (the numpy form cost ~0.1 ms
// of the step boundary, where the GPU waits for it).
extern "C" int sqh_group_tiles(const double* cs, int64_t k, int nt, int G, int* out) {
  if (nt < 1 || k < 1 || G < 1) return 1;
  if (G == 1) {
    out[0] = 0;
    return 0;
  }
  const double inf = INFINITY;
  std::vector<double> lo1(nt + 1, 0.0), hib(nt + 1, 0.0), cc(nt + 1, 0.0);
  for (int t = 0; t < nt; ++t) {
    const int64_t a = 64 * (int64_t)t < k - 1 ? 64 * (int64_t)t : k - 1;
    const int64_t b = 64 * (int64_t)t + 63 < k - 1 ? 64 * (int64_t)t + 63 : k - 1;
    lo1[t] = cs[a];
    hib[t + 1] = cs[b];
    const int64_t c = k - 64 * (int64_t)t;
    cc[t + 1] = cc[t] + (double)(c < 0 ? 0 : (c > 64 ? 64 : c));
  }
  std::vector<double> best((size_t)(G + 1) * (nt + 1), inf);
  std::vector<int> arg((size_t)(G + 1) * (nt + 1), 0);
  best[0] = 0.0;
  for (int g = 1; g <= G; ++g) {
    const double* bp = &best[(size_t)(g - 1) * (nt + 1)];
    for (int b = 0; b <= nt; ++b) {
      double m = inf;
      int am = 0;
      for (int a = 0; a <= nt; ++a) {
        double tv = inf;
        if (a >= g - 1 && a < b) tv = bp[a] + (cc[b] - cc[a]) * (hib[b] - lo1[a]);
        if (tv < m) {
          m = tv;
          am = a;
        }
      }
      arg[(size_t)g * (nt + 1) + b] = am;
      best[(size_t)g * (nt + 1) + b] = b < g ? inf : m;
    }
  }
  std::vector<int> cuts;
  int b = nt;
  for (int g = G; g >= 1; --g) {
    const int a = arg[(size_t)g * (nt + 1) + b];
    cuts.push_back(a);
    b = a;
  }
  std::sort(cuts.begin(), cuts.end());
  for (int g = 0; g < G; ++g) out[g] = cuts[g];
  return 0;
}
