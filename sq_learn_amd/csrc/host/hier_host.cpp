// Hierarchical clustering core (reference
// ``cluster/_hierarchical_fast.pyx`` + the scipy linkage the reference's
// unstructured trees delegate to).
//
//   * nearest-neighbour-chain agglomeration (Muellner 2011) on a condensed
//     distance matrix with Lance-Williams updates for ward / complete /
//     average / weighted linkage: O(n^2) time, no extra memory;
//   * single linkage as Prim's minimum spanning tree over the same matrix;
//   * merges stably sorted by height, then relabelled with a union-find
//     (new node n + i for the i-th merge, children ordered (min, max)),
//     giving a standard linkage matrix [child_a, child_b, height, size].
#include <cmath>
#include <cstdint>
#include <limits>
#include <numeric>
#include <vector>

#include "host.h"

namespace {

inline int64_t cidx(int64_t n, int64_t i, int64_t j) {   // condensed index, i != j
  if (i > j) std::swap(i, j);
  return n * i - (i * (i + 1)) / 2 + (j - i - 1);
}

enum Method { kSingle = 0, kComplete = 1, kAverage = 2, kWeighted = 3, kWard = 4 };

inline double lance_williams(int m, double dxi, double dyi, double dxy, double nx, double ny,
                             double ni) {
  switch (m) {
    case kComplete: return dxi > dyi ? dxi : dyi;
    case kAverage: return (nx * dxi + ny * dyi) / (nx + ny);
    case kWeighted: return 0.5 * (dxi + dyi);
    case kWard: {
      const double t = 1.0 / (nx + ny + ni);
      return std::sqrt((ni + nx) * t * dxi * dxi + (ni + ny) * t * dyi * dyi - ni * t * dxy * dxy);
    }
    default: return dxi < dyi ? dxi : dyi;
  }
}

// ordered: children as (min, max) root ids (scipy linkage convention);
// otherwise (root of child a, root of child b) as given (the reference's
// single-linkage labelling of an MST edge list)
void relabel(double* Z, int64_t n, bool ordered) {
  std::vector<int64_t> parent(2 * n - 1);
  std::vector<double> size(2 * n - 1, 1.0);
  std::iota(parent.begin(), parent.end(), 0);
  auto find = [&](int64_t x) {
    int64_t r = x;
    while (parent[r] != r) r = parent[r];
    while (parent[x] != r) {
      const int64_t nx = parent[x];
      parent[x] = r;
      x = nx;
    }
    return r;
  };
  int64_t next = n;
  for (int64_t i = 0; i < n - 1; ++i) {
    const int64_t a = find((int64_t)Z[4 * i]), b = find((int64_t)Z[4 * i + 1]);
    Z[4 * i] = (double)(ordered ? std::min(a, b) : a);
    Z[4 * i + 1] = (double)(ordered ? std::max(a, b) : b);
    parent[a] = parent[b] = next;
    size[next] = size[a] + size[b];
    Z[4 * i + 3] = size[next];
    ++next;
  }
}

void stable_sort_by_height(double* Z, int64_t n) {
  std::vector<int64_t> ord(n - 1);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(),
                   [&](int64_t a, int64_t b) { return Z[4 * a + 2] < Z[4 * b + 2]; });
  std::vector<double> tmp(Z, Z + 4 * (n - 1));
  for (int64_t i = 0; i < n - 1; ++i)
    for (int c = 0; c < 4; ++c) Z[4 * i + c] = tmp[4 * ord[i] + c];
}

}  // namespace

extern "C" {

// D: condensed distances (n(n-1)/2), overwritten for method != single.
// Z: (n-1) x 4 output.  Returns 0, or -1 for an unknown method.
int sqh_linkage(double* D, long long n, int method, int ordered_children, double* Z) {
  if (n < 2) return 0;
  const double inf = std::numeric_limits<double>::infinity();
  if (method == kSingle) {
    std::vector<char> merged(n, 0);
    std::vector<double> best(n, inf);
    int64_t x = 0;
    for (int64_t k = 0; k < n - 1; ++k) {
      double cur = inf;
      int64_t y = -1;
      merged[x] = 1;
      for (int64_t i = 0; i < n; ++i) {
        if (merged[i]) continue;
        const double d = D[cidx(n, x, i)];
        if (best[i] > d) best[i] = d;
        if (best[i] < cur || y < 0) {
          y = i;
          cur = best[i];
        }
      }
      Z[4 * k] = (double)x;
      Z[4 * k + 1] = (double)y;
      Z[4 * k + 2] = cur;
      Z[4 * k + 3] = 0.0;
      x = y;
    }
  } else if (method >= kComplete && method <= kWard) {
    std::vector<double> size(n, 1.0);
    std::vector<int64_t> chain;
    chain.reserve(n);
    for (int64_t k = 0; k < n - 1; ++k) {
      if (chain.empty()) {
        for (int64_t i = 0; i < n; ++i)
          if (size[i] > 0) {
            chain.push_back(i);
            break;
          }
      }
      int64_t x = 0, y = 0;
      double cur = inf;
      while (true) {
        x = chain.back();
        if (chain.size() > 1) {
          y = chain[chain.size() - 2];
          cur = D[cidx(n, x, y)];
        } else {
          cur = inf;
        }
        for (int64_t i = 0; i < n; ++i) {
          if (size[i] == 0 || i == x) continue;
          const double d = D[cidx(n, x, i)];
          if (d < cur) {
            cur = d;
            y = i;
          }
        }
        if (chain.size() > 1 && y == chain[chain.size() - 2]) break;
        chain.push_back(y);
      }
      chain.pop_back();
      chain.pop_back();
      if (x > y) std::swap(x, y);
      const double nx = size[x], ny = size[y];
      Z[4 * k] = (double)x;
      Z[4 * k + 1] = (double)y;
      Z[4 * k + 2] = cur;
      Z[4 * k + 3] = nx + ny;
      size[x] = 0;
      size[y] = nx + ny;
      for (int64_t i = 0; i < n; ++i) {
        const double ni = size[i];
        if (ni == 0 || i == y) continue;
        D[cidx(n, i, y)] = lance_williams(method, D[cidx(n, i, x)], D[cidx(n, i, y)], cur, nx,
                                          ny, ni);
      }
    }
  } else {
    return -1;
  }
  stable_sort_by_height(Z, n);
  relabel(Z, n, ordered_children != 0);
  return 0;
}

}  // extern "C"
