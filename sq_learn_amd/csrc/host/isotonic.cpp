// Isotonic regression kernels (reference ``_isotonic.pyx``):
// in-place pool-adjacent-violators for a non-decreasing weighted fit, and the
// duplicate-x aggregation used before it.  Linear time: blocks are tracked
// by a pointer array holding, at each block's first and last index, the
// index of the other end, so merging and backtracking are O(1) per step.
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

template <typename T>
void pava(T* y, T* w, long long n) {
  if (n <= 1) return;
  std::vector<long long> other(n);
  for (long long i = 0; i < n; ++i) other[i] = i;
  long long i = 0;
  while (i < n) {
    long long k = other[i] + 1;          // first index after block i
    if (k == n) break;
    if (y[i] < y[k]) {                   // ordered: move to the next block
      i = k;
      continue;
    }
    // violation: absorb following blocks while the sequence does not increase
    T swy = w[i] * y[i], sw = w[i];
    while (true) {
      const T prev = y[k];
      swy += w[k] * y[k];
      sw += w[k];
      k = other[k] + 1;
      if (k == n || prev < y[k]) {
        y[i] = swy / sw;
        w[i] = sw;
        other[i] = k - 1;
        other[k - 1] = i;
        if (i > 0) i = other[i - 1];     // re-check against the previous block
        break;
      }
    }
  }
  for (long long b = 0; b < n;) {        // expand block values
    const long long e = other[b] + 1;
    for (long long t = b + 1; t < e; ++t) y[t] = y[b];
    b = e;
  }
}

// X sorted; merges runs with x - run_start < eps; returns the unique count
template <typename T>
long long make_unique(const T* x, const T* y, const T* w, long long n, T eps, T* xo, T* yo,
                      T* wo) {
  if (n == 0) return 0;
  long long u = 0;
  T cx = x[0], cy = 0, cw = 0;
  for (long long j = 0; j < n; ++j) {
    if (x[j] - cx >= eps) {
      xo[u] = cx;
      wo[u] = cw;
      yo[u] = cy / cw;
      ++u;
      cx = x[j];
      cw = w[j];
      cy = y[j] * w[j];
    } else {
      cw += w[j];
      cy += y[j] * w[j];
    }
  }
  xo[u] = cx;
  wo[u] = cw;
  yo[u] = cy / cw;
  return u + 1;
}

}  // namespace

extern "C" {

void sqh_pava_f64(double* y, double* w, long long n) { pava(y, w, n); }
void sqh_pava_f32(float* y, float* w, long long n) { pava(y, w, n); }

long long sqh_make_unique_f64(const double* x, const double* y, const double* w, long long n,
                              double eps, double* xo, double* yo, double* wo) {
  return make_unique(x, y, w, n, eps, xo, yo, wo);
}
long long sqh_make_unique_f32(const float* x, const float* y, const float* w, long long n,
                              float eps, float* xo, float* yo, float* wo) {
  return make_unique(x, y, w, n, eps, xo, yo, wo);
}

}  // extern "C"
