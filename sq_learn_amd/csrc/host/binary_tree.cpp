// KD-tree / ball-tree for the host neighbour searches (reference
// sklearn/neighbors/_binary_tree.pxi, _kd_tree.pyx, _ball_tree.pyx; N12).
//
// Same layout as the reference: a complete binary tree with
// n_levels = 1 + floor(log2(max(1, (n-1)/leaf_size))) levels, node i has
// children 2i+1 / 2i+2, each split at the middle index along the dimension
// of largest spread (nth_element partition).  KD nodes keep per-dimension
// lower/upper bounds, ball nodes a centroid + radius.  Queries are
// depth-first, nearer child first, with pruning on the reduced distance
// ("rdist": |x|^p sums without the root, max for chebyshev); one query row
// per OpenMP iteration.  Metrics: minkowski p (p=2 euclidean, p=1
// manhattan, p=inf chebyshev).
//
// On the GPU the framework uses brute force (distance GEMM + top-k kernel);
// the trees serve non-euclidean metrics, small queries and radius searches
// on the host, where the reference uses them too.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <queue>
#include <utility>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct Tree {
  int64_t n;
  int d, leaf_size, kind;  // kind 0 = kd, 1 = ball
  double p;
  std::vector<double> X;
  std::vector<int64_t> idx;
  std::vector<int64_t> start, end;
  std::vector<uint8_t> leaf;
  std::vector<double> radius;  // ball radius (dist units)
  std::vector<double> bounds;  // kd: [node][2][d] lower, upper ; ball: [node][d] centroid
  int64_t n_nodes;

  bool cheb() const { return std::isinf(p); }
  double rdist(const double* a, const double* b) const {
    double s = 0.0;
    if (p == 2.0) {
      for (int j = 0; j < d; ++j) { double t = a[j] - b[j]; s += t * t; }
    } else if (p == 1.0) {
      for (int j = 0; j < d; ++j) s += std::fabs(a[j] - b[j]);
    } else if (cheb()) {
      for (int j = 0; j < d; ++j) s = std::max(s, std::fabs(a[j] - b[j]));
    } else {
      for (int j = 0; j < d; ++j) s += std::pow(std::fabs(a[j] - b[j]), p);
    }
    return s;
  }
  double r2d(double r) const {
    if (p == 2.0) return std::sqrt(r);
    if (p == 1.0 || cheb()) return r;
    return std::pow(r, 1.0 / p);
  }
  double d2r(double x) const {
    if (p == 2.0) return x * x;
    if (p == 1.0 || cheb()) return x;
    return std::pow(x, p);
  }
  const double* row(int64_t i) const { return X.data() + i * d; }

  void init_node(int64_t i, int64_t s, int64_t e) {
    start[i] = s;
    end[i] = e;
    if (kind == 0) {
      double* lo = bounds.data() + i * 2 * d;
      double* hi = lo + d;
      for (int j = 0; j < d; ++j) { lo[j] = INFINITY; hi[j] = -INFINITY; }
      for (int64_t t = s; t < e; ++t) {
        const double* x = row(idx[t]);
        for (int j = 0; j < d; ++j) { lo[j] = std::min(lo[j], x[j]); hi[j] = std::max(hi[j], x[j]); }
      }
      double r = 0.0;  // half-diagonal, as the reference stores for kd nodes
      if (cheb()) {
        for (int j = 0; j < d; ++j) r = std::max(r, 0.5 * std::fabs(hi[j] - lo[j]));
      } else {
        for (int j = 0; j < d; ++j) r += std::pow(0.5 * std::fabs(hi[j] - lo[j]), p);
        r = std::pow(r, 1.0 / p);
      }
      radius[i] = r;
    } else {
      double* c = bounds.data() + i * d;
      for (int j = 0; j < d; ++j) c[j] = 0.0;
      for (int64_t t = s; t < e; ++t) {
        const double* x = row(idx[t]);
        for (int j = 0; j < d; ++j) c[j] += x[j];
      }
      for (int j = 0; j < d; ++j) c[j] /= (double)(e - s);
      double r = 0.0;
      for (int64_t t = s; t < e; ++t) r = std::max(r, rdist(c, row(idx[t])));
      radius[i] = r2d(r);
    }
  }

  int spread_dim(int64_t s, int64_t e) const {
    int best = 0;
    double bs = -1.0;
    for (int j = 0; j < d; ++j) {
      double lo = INFINITY, hi = -INFINITY;
      for (int64_t t = s; t < e; ++t) {
        double v = X[idx[t] * d + j];
        lo = std::min(lo, v);
        hi = std::max(hi, v);
      }
      if (hi - lo > bs) { bs = hi - lo; best = j; }
    }
    return best;
  }

  void build(int64_t i, int64_t s, int64_t e) {
    init_node(i, s, e);
    if (2 * i + 1 >= n_nodes) {
      leaf[i] = 1;
      return;
    }
    leaf[i] = 0;
    int64_t mid = s + (e - s) / 2;
    int j = spread_dim(s, e);
    std::nth_element(idx.begin() + s, idx.begin() + mid, idx.begin() + e,
                     [&](int64_t a, int64_t b) { return X[a * d + j] < X[b * d + j]; });
    build(2 * i + 1, s, mid);
    build(2 * i + 2, mid, e);
  }

  double min_rdist(int64_t i, const double* x) const {
    if (kind == 0) {
      const double* lo = bounds.data() + i * 2 * d;
      const double* hi = lo + d;
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        double dl = lo[j] - x[j], dh = x[j] - hi[j];
        double g = 0.5 * ((dl + std::fabs(dl)) + (dh + std::fabs(dh)));
        if (cheb()) s = std::max(s, g);
        else if (p == 2.0) s += g * g;
        else if (p == 1.0) s += g;
        else s += std::pow(g, p);
      }
      return s;
    }
    double dc = r2d(rdist(x, bounds.data() + i * d));
    return d2r(std::max(0.0, dc - radius[i]));
  }
  double max_rdist(int64_t i, const double* x) const {
    if (kind == 0) {
      const double* lo = bounds.data() + i * 2 * d;
      const double* hi = lo + d;
      double s = 0.0;
      for (int j = 0; j < d; ++j) {
        double g = std::max(std::fabs(x[j] - lo[j]), std::fabs(x[j] - hi[j]));
        if (cheb()) s = std::max(s, g);
        else if (p == 2.0) s += g * g;
        else if (p == 1.0) s += g;
        else s += std::pow(g, p);
      }
      return s;
    }
    double dc = r2d(rdist(x, bounds.data() + i * d));
    return d2r(dc + radius[i]);
  }

  // k nearest: max-heap of (rdist, index)
  void knn(int64_t node, const double* x, int k,
           std::priority_queue<std::pair<double, int64_t>>& heap) const {
    double bound = (int)heap.size() < k ? INFINITY : heap.top().first;
    if (min_rdist(node, x) > bound) return;
    if (leaf[node]) {
      for (int64_t t = start[node]; t < end[node]; ++t) {
        double r = rdist(x, row(idx[t]));
        if ((int)heap.size() < k) {
          heap.emplace(r, idx[t]);
        } else if (r < heap.top().first) {
          heap.pop();
          heap.emplace(r, idx[t]);
        }
      }
      return;
    }
    int64_t a = 2 * node + 1, b = 2 * node + 2;
    double da = min_rdist(a, x), db = min_rdist(b, x);
    if (db < da) std::swap(a, b);
    knn(a, x, k, heap);
    knn(b, x, k, heap);
  }

  void radius_q(int64_t node, const double* x, double r_rd, bool want_dist,
                std::vector<int64_t>& out, std::vector<double>& dist) const {
    if (min_rdist(node, x) > r_rd) return;
    if (max_rdist(node, x) <= r_rd) {
      for (int64_t t = start[node]; t < end[node]; ++t) {
        out.push_back(idx[t]);
        if (want_dist) dist.push_back(rdist(x, row(idx[t])));
      }
      return;
    }
    if (leaf[node]) {
      for (int64_t t = start[node]; t < end[node]; ++t) {
        double r = rdist(x, row(idx[t]));
        if (r <= r_rd) {
          out.push_back(idx[t]);
          if (want_dist) dist.push_back(r);
        }
      }
      return;
    }
    radius_q(2 * node + 1, x, r_rd, want_dist, out, dist);
    radius_q(2 * node + 2, x, r_rd, want_dist, out, dist);
  }
};

struct RadiusResult {
  std::vector<std::vector<int64_t>> ind;
  std::vector<std::vector<double>> dist;
};

}  // namespace

extern "C" {

void* sqh_btree_build(const double* X, int64_t n, int d, int leaf_size, int kind, double p) {
  Tree* t = new Tree();
  t->n = n;
  t->d = d;
  t->leaf_size = leaf_size;
  t->kind = kind;
  t->p = p;
  t->X.assign(X, X + n * d);
  t->idx.resize(n);
  for (int64_t i = 0; i < n; ++i) t->idx[i] = i;
  int64_t q = std::max<int64_t>(1, (n - 1) / std::max(1, leaf_size));
  int n_levels = 1 + (int)std::floor(std::log2((double)q));
  t->n_nodes = ((int64_t)1 << n_levels) - 1;
  t->start.resize(t->n_nodes);
  t->end.resize(t->n_nodes);
  t->leaf.resize(t->n_nodes);
  t->radius.resize(t->n_nodes);
  t->bounds.resize(t->n_nodes * (kind == 0 ? 2 * d : d));
  if (n > 0) t->build(0, 0, n);
  return t;
}

void sqh_btree_free(void* h) { delete static_cast<Tree*>(h); }

void sqh_btree_info(void* h, int64_t* out) {
  Tree* t = static_cast<Tree*>(h);
  out[0] = t->n_nodes;
  out[1] = (int64_t)t->bounds.size();
}

void sqh_btree_copy(void* h, int64_t* idx, int64_t* start, int64_t* end, uint8_t* leaf,
                    double* radius, double* bounds) {
  Tree* t = static_cast<Tree*>(h);
  std::memcpy(idx, t->idx.data(), sizeof(int64_t) * t->n);
  std::memcpy(start, t->start.data(), sizeof(int64_t) * t->n_nodes);
  std::memcpy(end, t->end.data(), sizeof(int64_t) * t->n_nodes);
  std::memcpy(leaf, t->leaf.data(), t->n_nodes);
  std::memcpy(radius, t->radius.data(), sizeof(double) * t->n_nodes);
  std::memcpy(bounds, t->bounds.data(), sizeof(double) * t->bounds.size());
}

// k nearest neighbours of m query rows; outputs sorted ascending (dist units).
void sqh_btree_knn(void* h, const double* Q, int64_t m, int k, double* dist, int64_t* ind,
                   int n_threads) {
  Tree* t = static_cast<Tree*>(h);
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads)
  for (int64_t i = 0; i < m; ++i) {
    std::priority_queue<std::pair<double, int64_t>> heap;
    t->knn(0, Q + i * t->d, k, heap);
    int kk = (int)heap.size();
    for (int j = kk - 1; j >= 0; --j) {
      dist[i * k + j] = t->r2d(heap.top().first);
      ind[i * k + j] = heap.top().second;
      heap.pop();
    }
    for (int j = kk; j < k; ++j) { dist[i * k + j] = INFINITY; ind[i * k + j] = -1; }
  }
}

// Radius neighbours; r per query (dist units).  counts[i] filled always;
// returns a result handle unless count_only.
void* sqh_btree_radius(void* h, const double* Q, int64_t m, const double* r, int count_only,
                       int want_dist, int sort_results, int64_t* counts, int n_threads) {
  Tree* t = static_cast<Tree*>(h);
  RadiusResult* res = count_only ? nullptr : new RadiusResult();
  if (res) {
    res->ind.resize(m);
    res->dist.resize(m);
  }
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads)
  for (int64_t i = 0; i < m; ++i) {
    std::vector<int64_t> o;
    std::vector<double> dd;
    bool wd = want_dist || sort_results;
    t->radius_q(0, Q + i * t->d, t->d2r(r[i]), wd, o, dd);
    counts[i] = (int64_t)o.size();
    if (!res) continue;
    if (sort_results) {
      std::vector<size_t> ord(o.size());
      for (size_t j = 0; j < ord.size(); ++j) ord[j] = j;
      std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return dd[a] < dd[b]; });
      std::vector<int64_t> o2(o.size());
      std::vector<double> d2(o.size());
      for (size_t j = 0; j < ord.size(); ++j) { o2[j] = o[ord[j]]; d2[j] = dd[ord[j]]; }
      o.swap(o2);
      dd.swap(d2);
    }
    for (double& v : dd) v = t->r2d(v);
    res->ind[i].swap(o);
    if (want_dist) res->dist[i].swap(dd);
  }
  return res;
}

void sqh_radius_copy(void* r, int64_t* ind, double* dist) {
  RadiusResult* res = static_cast<RadiusResult*>(r);
  int64_t off = 0;
  for (size_t i = 0; i < res->ind.size(); ++i) {
    std::memcpy(ind + off, res->ind[i].data(), sizeof(int64_t) * res->ind[i].size());
    if (dist && !res->dist[i].empty())
      std::memcpy(dist + off, res->dist[i].data(), sizeof(double) * res->dist[i].size());
    off += (int64_t)res->ind[i].size();
  }
}

void sqh_radius_free(void* r) { delete static_cast<RadiusResult*>(r); }

}  // extern "C"
