// Sparse-sparse L1 distances between CSR rows (reference
// ``metrics/_pairwise_fast.pyx: _sparse_manhattan``): sorted-index merge per
// (i, j) pair, OpenMP over the rows of X.  Also ``cholesky_delete``
// (reference ``utils/arrayfuncs.pyx``): remove column/row ``go_out`` from a
// lower-triangular Cholesky factor with Givens rotations (LARS downdate).
#include <cmath>
#include <cstdint>

#include "host.h"

extern "C" {

void sqh_sparse_manhattan(const double* xd, const int32_t* xi, const int64_t* xp,
                          const double* yd, const int32_t* yi, const int64_t* yp, long long n,
                          long long m, double* D) {
#pragma omp parallel for schedule(dynamic, 16)
  for (long long i = 0; i < n; ++i) {
    for (long long j = 0; j < m; ++j) {
      int64_t a = xp[i], ae = xp[i + 1], b = yp[j], be = yp[j + 1];
      double s = 0.0;
      while (a < ae && b < be) {
        if (xi[a] == yi[b]) {
          s += std::fabs(xd[a] - yd[b]);
          ++a;
          ++b;
        } else if (xi[a] < yi[b]) {
          s += std::fabs(xd[a++]);
        } else {
          s += std::fabs(yd[b++]);
        }
      }
      while (a < ae) s += std::fabs(xd[a++]);
      while (b < be) s += std::fabs(yd[b++]);
      D[i * m + j] = s;
    }
  }
}

// L: n x n row-major (lower triangular in the leading n rows/cols), in place
void sqh_cholesky_delete(double* L, long long n, long long ld, long long go_out) {
  // shift rows below go_out up by one, then restore lower-triangularity
  for (long long i = go_out; i < n - 1; ++i)
    for (long long k = 0; k < n; ++k) L[i * ld + k] = L[(i + 1) * ld + k];
  for (long long i = go_out; i < n - 1; ++i) {
    const double a = L[i * ld + i], b = L[i * ld + i + 1];
    const double r = std::hypot(a, b);
    if (r == 0.0) continue;
    const double c = a / r, s = b / r;
    for (long long k = i; k < n - 1; ++k) {
      const double u = L[k * ld + i], v = L[k * ld + i + 1];
      L[k * ld + i] = c * u + s * v;
      L[k * ld + i + 1] = -s * u + c * v;
    }
    L[i * ld + i + 1] = 0.0;
  }
}

}  // extern "C"
