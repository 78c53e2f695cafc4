// Barnes-Hut t-SNE gradient (reference ``manifold/_barnes_hut_tsne.pyx:263``
// compute_gradient + ``neighbors/_quad_tree.pyx``), host-native.
//
//   grad_i = c (F_attr_i - F_rep_i / Z)
//   F_attr_i = sum_j p_ij q_ij (y_i - y_j)          over the sparse k-NN P
//   F_rep_i  = sum_j q_ij^2 Z^2... = sum_j w_ij^2 (y_i - y_j),  Z = sum_{i != j} w_ij
//   w_ij = (dof / (dof + |y_i - y_j|^2))^((dof + 1) / 2),   c = 2 (dof + 1) / dof
//
// The repulsion is approximated with a 2^dim-ary space-partitioning tree
// (quad-tree in 2-D, oct-tree in 3-D) over the embedding: a cell whose
// width w seen from y_i at distance r satisfies w / r < theta acts as one
// point of mass |cell| at its centre of mass (theta = 0: exact).  The tree
// is rebuilt every iteration in O(n log n) (flat node array, children
// contiguous); the per-point traversals and the sparse attraction run as
// OpenMP loops over points, each point's forces in a private accumulator,
// then Z and the optional KL error are reduced in a fixed order (per-point
// partials summed serially), so the result is deterministic for any thread
// count.  fp64 throughout (the reference computes in fp32).
#include <cmath>
#include <vector>

#include "host.h"

namespace {

constexpr int kMaxDim = 3;
constexpr int kMaxDepth = 64;   // below this cell size points count as duplicates

struct Cell {
  double center[kMaxDim];   // geometric centre
  double half;              // half width (cells are cubes)
  double com[kMaxDim];      // centre of mass of the points inside
  long long size;           // points inside (duplicates included)
  int child;                // first of 2^dim children, -1 for a leaf
  long long point;          // leaf: one representative point, -1 if empty
  int depth;
};

struct Tree {
  int dim;
  int nchild;
  std::vector<Cell> cells;

  int new_cell(const double* c, double half, int depth) {
    Cell cell;
    for (int a = 0; a < kMaxDim; ++a) {
      cell.center[a] = a < dim ? c[a] : 0.0;
      cell.com[a] = 0.0;
    }
    cell.half = half;
    cell.size = 0;
    cell.child = -1;
    cell.point = -1;
    cell.depth = depth;
    cells.push_back(cell);
    return (int)cells.size() - 1;
  }

  int child_index(const Cell& c, const double* y) const {
    int q = 0;
    for (int a = 0; a < dim; ++a)
      if (y[a] >= c.center[a]) q |= 1 << a;
    return q;
  }

  void split(int ci) {
    const double h = cells[ci].half * 0.5;
    const int depth = cells[ci].depth + 1;
    double c0[kMaxDim];
    int first = -1;
    for (int q = 0; q < nchild; ++q) {
      for (int a = 0; a < dim; ++a)
        c0[a] = cells[ci].center[a] + ((q >> a) & 1 ? h : -h);
      const int k = new_cell(c0, h, depth);   // may reallocate: index only
      if (q == 0) first = k;
    }
    cells[ci].child = first;
  }

  void insert(const double* Y, long long i) {
    const double* y = Y + i * dim;
    int ci = 0;
    while (true) {
      Cell& c = cells[ci];
      // running centre of mass of everything inserted below this cell
      const double s = (double)c.size;
      for (int a = 0; a < dim; ++a) c.com[a] = (c.com[a] * s + y[a]) / (s + 1.0);
      c.size += 1;
      if (c.child < 0) {
        if (c.point < 0) {   // empty leaf
          c.point = i;
          return;
        }
        const double* p = Y + c.point * dim;
        bool same = true;
        for (int a = 0; a < dim; ++a) same = same && p[a] == y[a];
        if (same || c.depth >= kMaxDepth) return;   // duplicate: mass only
        // subdivide: push the resident point one level down (its mass is
        // already counted here), then continue with the new point
        const long long old = c.point;
        const double* po = Y + old * dim;
        split(ci);
        Cell& c2 = cells[ci];
        c2.point = -1;
        Cell& oc = cells[c2.child + child_index(c2, po)];
        oc.point = old;
        oc.size = c2.size - 1;   // the resident point (+ its duplicates)
        for (int a = 0; a < dim; ++a) oc.com[a] = po[a];
        ci = c2.child + child_index(c2, y);
        continue;
      }
      ci = c.child + child_index(c, y);
    }
  }

  void build(const double* Y, long long n) {
    double lo[kMaxDim], hi[kMaxDim];
    for (int a = 0; a < dim; ++a) {
      lo[a] = INFINITY;
      hi[a] = -INFINITY;
    }
    for (long long i = 0; i < n; ++i)
      for (int a = 0; a < dim; ++a) {
        lo[a] = std::min(lo[a], Y[i * dim + a]);
        hi[a] = std::max(hi[a], Y[i * dim + a]);
      }
    double c[kMaxDim], w = 0.0;
    for (int a = 0; a < dim; ++a) {
      c[a] = 0.5 * (lo[a] + hi[a]);
      w = std::max(w, hi[a] - lo[a]);
    }
    // half width with a margin so the max corner lies strictly inside
    const double half = 0.5 * w * (1.0 + 1e-3) + 1e-12;
    cells.clear();
    cells.reserve((size_t)(4 * n + 16));
    new_cell(c, half, 0);
    for (long long i = 0; i < n; ++i) insert(Y, i);
  }
};

inline double kernel(double d2, double dof, double expo) {
  double w = dof / (dof + d2);
  return expo == 1.0 ? w : std::pow(w, expo);
}

}  // namespace

extern "C" {

// Y: n x dim (row major, fp64); P: CSR (indptr n+1, indices, values) of the
// symmetric joint probabilities.  grad: n x dim output.  Returns the KL
// divergence when compute_error != 0 (else 0).
double sqh_tsne_bh_grad(const double* Y, long long n, int dim, const long long* indptr,
                        const int* indices, const double* pval, double theta, double dof,
                        int compute_error, double* grad) {
  if (n <= 0 || dim < 1 || dim > kMaxDim) return 0.0;
  const double expo = (dof + 1.0) / 2.0;
  Tree t;
  t.dim = dim;
  t.nchild = 1 << dim;
  t.build(Y, n);
  const double theta2 = theta * theta;
  std::vector<double> zpart((size_t)n, 0.0), neg((size_t)n * dim, 0.0);
#pragma omp parallel
  {
    std::vector<int> stack;
    stack.reserve(256);
#pragma omp for schedule(dynamic, 256)
    for (long long i = 0; i < n; ++i) {
      const double* yi = Y + i * dim;
      double z = 0.0, f[kMaxDim] = {0.0, 0.0, 0.0};
      stack.clear();
      stack.push_back(0);
      while (!stack.empty()) {
        const Cell& c = t.cells[stack.back()];
        stack.pop_back();
        if (c.size == 0) continue;
        double delta[kMaxDim], d2 = 0.0;
        for (int a = 0; a < dim; ++a) {
          delta[a] = yi[a] - c.com[a];
          d2 += delta[a] * delta[a];
        }
        const bool leaf = c.child < 0;
        const double w = 2.0 * c.half;
        if (leaf || w * w < theta2 * d2) {
          long long m = c.size;
          if (leaf && d2 == 0.0) {
            // the cell holds y_i itself (and possibly duplicates of it):
            // the duplicates interact at distance 0, y_i does not
            m -= 1;
            if (m <= 0) continue;
          }
          const double q = kernel(d2, dof, expo);
          z += (double)m * q;
          const double mult = (double)m * q * q;
          for (int a = 0; a < dim; ++a) f[a] += mult * delta[a];
          continue;
        }
        for (int k = 0; k < t.nchild; ++k) stack.push_back(c.child + k);
      }
      zpart[i] = z;
      for (int a = 0; a < dim; ++a) neg[i * dim + a] = f[a];
    }
  }
  double Z = 0.0;
  for (long long i = 0; i < n; ++i) Z += zpart[i];
  if (!(Z > 0.0)) Z = 1e-300;
  const double cgrad = 2.0 * (dof + 1.0) / dof;
  std::vector<double> errpart(compute_error ? (size_t)n : 0, 0.0);
#pragma omp parallel for schedule(dynamic, 256)
  for (long long i = 0; i < n; ++i) {
    const double* yi = Y + i * dim;
    double pos[kMaxDim] = {0.0, 0.0, 0.0}, e = 0.0;
    for (long long p = indptr[i]; p < indptr[i + 1]; ++p) {
      const long long j = indices[p];
      const double* yj = Y + j * dim;
      double delta[kMaxDim], d2 = 0.0;
      for (int a = 0; a < dim; ++a) {
        delta[a] = yi[a] - yj[a];
        d2 += delta[a] * delta[a];
      }
      const double q = kernel(d2, dof, expo);
      const double pij = pval[p];
      for (int a = 0; a < dim; ++a) pos[a] += pij * q * delta[a];
      if (compute_error) {
        const double qn = std::max(q / Z, 2.220446049250313e-16);
        e += pij * std::log(std::max(pij, 2.220446049250313e-16) / qn);
      }
    }
    for (int a = 0; a < dim; ++a)
      grad[i * dim + a] = cgrad * (pos[a] - neg[i * dim + a] / Z);
    if (compute_error) errpart[i] = e;
  }
  double err = 0.0;
  if (compute_error)
    for (long long i = 0; i < n; ++i) err += errpart[i];
  return err;
}

}  // extern "C"
