// CSR polynomial expansion of one degree (reference
// ``preprocessing/_csr_polynomial_expansion.pyx``): for every row, all
// degree-D products of its non-zero features, written at the column index
// of the monomial in ``itertools.combinations[_with_replacement](range(F), D)``
// order (so rows come out column-sorted when the input rows are).  The rank
// of a monomial i_0 <= ... <= i_{D-1} is a sum of hockey-stick binomial
// differences, O(D) per product.
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

// C(n, k) for small k, exact in int64 for the sizes we handle (n < 2^21 at D <= 3)
inline int64_t binom(int64_t n, int k) {
  if (k < 0 || n < k) return 0;
  int64_t r = 1;
  for (int t = 1; t <= k; ++t) r = r * (n - k + t) / t;
  return r;
}

struct Ranker {
  int64_t F;
  int D;
  bool inter;
  // sum_{v=a}^{b-1} count(r, v): monomials of r more factors whose values
  // are >= v (with replacement) or > v (interaction only)
  int64_t block(int r, int64_t a, int64_t b) const {
    if (b <= a) return 0;
    if (!inter) return binom(F - a + r, r + 1) - binom(F - b + r, r + 1);
    return binom(F - a, r + 1) - binom(F - b, r + 1);
  }
  int64_t rank(const int64_t* idx) const {
    int64_t r = 0, lo = 0;
    for (int t = 0; t < D; ++t) {
      r += block(D - 1 - t, lo, idx[t]);
      lo = inter ? idx[t] + 1 : idx[t];
    }
    return r;
  }
};

template <typename Emit>
void for_each_monomial(const int32_t* ind, const double* val, int64_t nnz, int D, bool inter,
                       Emit emit) {
  int64_t pos[4];
  // iterative nested loops over positions into the row's non-zeros
  auto rec = [&](auto&& self, int t, int64_t start, double prod) -> void {
    if (t == D) {
      int64_t idx[4];
      for (int q = 0; q < D; ++q) idx[q] = ind[pos[q]];
      emit(idx, prod);
      return;
    }
    for (int64_t p = start; p < nnz; ++p) {
      pos[t] = p;
      self(self, t + 1, inter ? p + 1 : p, prod * val[p]);
    }
  };
  rec(rec, 0, 0, 1.0);
}

}  // namespace

extern "C" {

// pass 1 (out_data == nullptr): row counts into out_indptr[1..n]; pass 2 fills
long long sqh_csr_poly(const double* data, const int32_t* indices, const int64_t* indptr,
                       long long n, long long F, int D, int interaction_only, int64_t* out_indptr,
                       int64_t* out_indices, double* out_data) {
  if (D < 1 || D > 3) return -1;
  Ranker rk{F, D, interaction_only != 0};
  int64_t total = 0;
  if (!out_data) out_indptr[0] = 0;
  for (long long i = 0; i < n; ++i) {
    const int64_t b = indptr[i], e = indptr[i + 1];
    int64_t cnt = 0;
    int64_t w = out_data ? out_indptr[i] : 0;
    for_each_monomial(indices + b, data + b, e - b, D, rk.inter,
                      [&](const int64_t* idx, double prod) {
                        if (out_data) {
                          out_indices[w] = rk.rank(idx);
                          out_data[w] = prod;
                          ++w;
                        }
                        ++cnt;
                      });
    if (!out_data) out_indptr[i + 1] = out_indptr[i] + cnt;
    total += cnt;
  }
  return total;
}

}  // extern "C"
