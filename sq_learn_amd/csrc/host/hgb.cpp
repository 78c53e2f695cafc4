// Histogram gradient-boosting tree growth (reference
// ``ensemble/_hist_gradient_boosting``: ``_binning.pyx:_map_to_bins``,
// ``histogram.pyx`` brute / subtraction histograms, ``splitting.pyx``
// split finding (left-to-right and, with missing values, right-to-left
// scans, monotonic constraints, XGBoost gain / node value), ``grower.py``
// best-first growth with a gain max-heap and ``_predictor.pyx`` inference).
//
// One call grows one tree: binned features are column-major uint8, the
// gradients / hessians float32, sums float64.  Histograms of a node are
// built over its sample slice (OpenMP over features); the larger child gets
// parent - smaller (subtraction trick).  The heap is Python ``heapq``'s
// sift algorithm with "greater gain first" so equal-gain ties resolve in the
// reference's order; sample partitions are stable, so histogram sums see
// rows in the reference's order.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "host.h"

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct Bin { double g, h; uint32_t c; };

struct SplitInfo {
  double gain = -1.0;
  int feature = 0;
  int bin = 0;
  bool missing_left = false;
  double gl = 0, hl = 0, gr = 0, hr = 0;
  uint32_t nl = 0, nr = 0;
  double vl = 0, vr = 0;
  bool is_cat = false;
  uint32_t bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // categorical: bins that go left
};

struct CatInfo { unsigned bin; double value; };

// Merge sort with the reference's comparator (a < b ? -1 : 1) and glibc
// msort's merge rule (take left iff cmp <= 0), so ties order identically.
void cat_msort(CatInfo* a, CatInfo* tmp, size_t n) {
  if (n <= 1) return;
  size_t n1 = n / 2, n2 = n - n1;
  CatInfo *b1 = a, *b2 = a + n1;
  cat_msort(b1, tmp, n1);
  cat_msort(b2, tmp, n2);
  size_t k = 0;
  while (n1 > 0 && n2 > 0) {
    if (b1->value < b2->value) { tmp[k++] = *b1++; --n1; }
    else { tmp[k++] = *b2++; --n2; }
  }
  while (n1 > 0) { tmp[k++] = *b1++; --n1; }
  for (size_t i = 0; i < k; ++i) a[i] = tmp[i];
}

struct Node {
  int depth;
  int64_t start, stop;      // slice of the partition array
  double sum_g, sum_h;
  double value;
  double lower = -INFINITY, upper = INFINITY;
  bool is_leaf = false;
  SplitInfo split;
  int left = -1, right = -1;
  std::vector<Bin> hist;    // d * n_bins while needed
  uint32_t n() const { return (uint32_t)(stop - start); }
};

struct Params {
  int64_t n; int d; int n_bins;
  const uint8_t* Xb; const float* grad; const float* hess; bool hess_const;
  const uint32_t* nbnm; const uint8_t* has_missing; const int8_t* mono;
  const uint8_t* is_cat;
  int max_leaf_nodes, max_depth, min_samples_leaf;
  double min_gain, l2, min_hess, shrinkage;
};

inline double node_value(double g, double h, double lo, double hi, double l2) {
  double v = -g / (h + l2 + 1e-15);
  if (v < lo) v = lo;
  else if (v > hi) v = hi;
  return v;
}

inline double split_gain(double gl, double hl, double gr, double hr, double loss_cur, int8_t mono,
                         double lo, double hi, double l2) {
  double vl = node_value(gl, hl, lo, hi, l2), vr = node_value(gr, hr, lo, hi, l2);
  if ((mono == 1 && vl > vr) || (mono == -1 && vl < vr)) return -1.0;
  return loss_cur - gl * vl - gr * vr;
}

struct Grower {
  Params P;
  std::vector<uint32_t> part;   // sample indices, partitioned per node
  std::vector<uint32_t> tmp;
  std::vector<Node> nodes;
  std::vector<int> heap;        // indices into nodes (heapq order)
  std::vector<int> finalized;

  bool less(int a, int b) const { return nodes[a].split.gain > nodes[b].split.gain; }
  // Python heapq._siftdown / _siftup with the node '<' = greater gain
  void siftdown(int startpos, int pos) {
    int item = heap[pos];
    while (pos > startpos) {
      int parentpos = (pos - 1) >> 1;
      int parent = heap[parentpos];
      if (less(item, parent)) { heap[pos] = parent; pos = parentpos; continue; }
      break;
    }
    heap[pos] = item;
  }
  void siftup(int pos) {
    int endpos = (int)heap.size(), startpos = pos, item = heap[pos];
    int child = 2 * pos + 1;
    while (child < endpos) {
      int right = child + 1;
      if (right < endpos && !less(heap[child], heap[right])) child = right;
      heap[pos] = heap[child];
      pos = child;
      child = 2 * pos + 1;
    }
    heap[pos] = item;
    siftdown(startpos, pos);
  }
  void push(int i) { heap.push_back(i); siftdown(0, (int)heap.size() - 1); }
  int pop() {
    int last = heap.back();
    heap.pop_back();
    if (!heap.empty()) { int ret = heap[0]; heap[0] = last; siftup(0); return ret; }
    return last;
  }

  std::vector<float> og, oh;     // gradients / hessians gathered in node order

  void build_hist(Node& nd) {
    const int nb = P.n_bins;
    nd.hist.assign((size_t)P.d * nb, Bin{0, 0, 0});
    const uint32_t* idx = part.data() + nd.start;
    const int64_t m = nd.stop - nd.start;
    const bool root = m == P.n;     // identity partition: no indirection
    if (!root) {                    // one gather per node instead of one per feature
      og.resize(m);
      for (int64_t q = 0; q < m; ++q) og[q] = P.grad[idx[q]];
      if (!P.hess_const) {
        oh.resize(m);
        for (int64_t q = 0; q < m; ++q) oh[q] = P.hess[idx[q]];
      }
    }
    const float* g = root ? P.grad : og.data();
    const float* hh = root ? P.hess : oh.data();
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) if (m * P.d > 20000)
#endif
    for (int f = 0; f < P.d; ++f) {
      Bin* h = nd.hist.data() + (size_t)f * nb;
      const uint8_t* col = P.Xb + (size_t)f * P.n;
      if (root) {
        if (P.hess_const) {
          for (int64_t q = 0; q < m; ++q) { Bin& b = h[col[q]]; b.g += g[q]; b.c += 1; }
        } else {
          for (int64_t q = 0; q < m; ++q) { Bin& b = h[col[q]]; b.g += g[q]; b.h += hh[q]; b.c += 1; }
        }
      } else if (P.hess_const) {
        for (int64_t q = 0; q < m; ++q) { Bin& b = h[col[idx[q]]]; b.g += g[q]; b.c += 1; }
      } else {
        for (int64_t q = 0; q < m; ++q) {
          Bin& b = h[col[idx[q]]];
          b.g += g[q];
          b.h += hh[q];
          b.c += 1;
        }
      }
    }
  }

  void subtract_hist(const Node& parent, const Node& sib, Node& nd) {
    nd.hist.resize(parent.hist.size());
    for (size_t j = 0; j < parent.hist.size(); ++j) {
      nd.hist[j].g = parent.hist[j].g - sib.hist[j].g;
      nd.hist[j].h = parent.hist[j].h - sib.hist[j].h;
      nd.hist[j].c = parent.hist[j].c - sib.hist[j].c;
    }
  }

  void scan_feature(const Node& nd, int f, SplitInfo& si) const {
    const Bin* h = nd.hist.data() + (size_t)f * P.n_bins;
    const uint32_t ns = nd.n();
    const double sg = nd.sum_g, sh = nd.sum_h, lo = nd.lower, hi = nd.upper;
    const double loss_cur = sg * nd.value;
    const int8_t mono = P.mono[f];
    const bool miss = P.has_missing[f] != 0;
    si.feature = f;
    si.gain = -1.0;
    if (P.is_cat && P.is_cat[f]) { scan_categorical(nd, f, si); return; }
    // left to right: missing values (last bin) go right
    {
      const unsigned end = P.nbnm[f] - 1 + (miss ? 1 : 0);
      double gl = 0, hl = 0;
      uint32_t nl = 0;
      bool found = false;
      double best = -1.0, bgl = 0, bhl = 0;
      uint32_t bnl = 0;
      int bbin = 0;
      for (unsigned b = 0; b < end; ++b) {
        nl += h[b].c;
        uint32_t nr = ns - nl;
        hl += P.hess_const ? (double)h[b].c : h[b].h;
        double hr = sh - hl;
        gl += h[b].g;
        double gr = sg - gl;
        if (nl < (uint32_t)P.min_samples_leaf) continue;
        if (nr < (uint32_t)P.min_samples_leaf) break;
        if (hl < P.min_hess) continue;
        if (hr < P.min_hess) break;
        double gain = split_gain(gl, hl, gr, hr, loss_cur, mono, lo, hi, P.l2);
        if (gain > best && gain > P.min_gain) {
          found = true; best = gain; bbin = (int)b; bgl = gl; bhl = hl; bnl = nl;
        }
      }
      if (found) {
        si.gain = best; si.bin = bbin; si.missing_left = false;
        si.gl = bgl; si.hl = bhl; si.gr = sg - bgl; si.hr = sh - bhl;
        si.nl = bnl; si.nr = ns - bnl;
        si.vl = node_value(si.gl, si.hl, lo, hi, P.l2);
        si.vr = node_value(si.gr, si.hr, lo, hi, P.l2);
      }
    }
    // right to left: missing values go left
    if (miss) {
      double gr = 0, hr = 0;
      uint32_t nr = 0;
      bool found = false;
      double best = si.gain, bgl = 0, bhl = 0;
      uint32_t bnl = 0;
      int bbin = 0;
      for (int b = (int)P.nbnm[f] - 2; b >= 0; --b) {
        nr += h[b + 1].c;
        uint32_t nl = ns - nr;
        hr += P.hess_const ? (double)h[b + 1].c : h[b + 1].h;
        double hl = sh - hr;
        gr += h[b + 1].g;
        double gl = sg - gr;
        if (nr < (uint32_t)P.min_samples_leaf) continue;
        if (nl < (uint32_t)P.min_samples_leaf) break;
        if (hr < P.min_hess) continue;
        if (hl < P.min_hess) break;
        double gain = split_gain(gl, hl, gr, hr, loss_cur, mono, lo, hi, P.l2);
        if (gain > best && gain > P.min_gain) {
          found = true; best = gain; bbin = b; bgl = gl; bhl = hl; bnl = nl;
        }
      }
      if (found) {
        si.gain = best; si.bin = bbin; si.missing_left = true;
        si.gl = bgl; si.hl = bhl; si.gr = sg - bgl; si.hr = sh - bhl;
        si.nl = bnl; si.nr = ns - bnl;
        si.vl = node_value(si.gl, si.hl, lo, hi, P.l2);
        si.vr = node_value(si.gr, si.hr, lo, hi, P.l2);
      }
    }
  }

  // Fisher grouping: categories with enough support sorted by
  // g / (h + MIN_CAT_SUPPORT), scanned from both ends up to the middle
  // (reference splitting.pyx _find_best_bin_to_split_category).
  void scan_categorical(const Node& nd, int f, SplitInfo& si) const {
    const Bin* h = nd.hist.data() + (size_t)f * P.n_bins;
    const uint32_t ns = nd.n();
    const double sg = nd.sum_g, sh = nd.sum_h, lo = nd.lower, hi = nd.upper;
    const bool miss = P.has_missing[f] != 0;
    const unsigned nbm = P.nbnm[f], mbin = (unsigned)P.n_bins - 1;
    const double MIN_CAT_SUPPORT = 10.0, support = (double)ns / sh;
    std::vector<CatInfo> ci, tmp;
    ci.reserve(nbm + 1);
    auto consider = [&](unsigned b) {
      double hb = P.hess_const ? (double)h[b].c : h[b].h;
      if (hb * support >= MIN_CAT_SUPPORT) ci.push_back({b, h[b].g / (hb + MIN_CAT_SUPPORT)});
    };
    for (unsigned b = 0; b < nbm; ++b) consider(b);
    if (miss) consider(mbin);
    const size_t nu = ci.size();
    if (nu <= 1) return;
    tmp.resize(nu);
    cat_msort(ci.data(), tmp.data(), nu);
    const double loss_cur = sg * nd.value;
    bool found = false;
    double best = -1.0, bgl = 0, bhl = 0;
    uint32_t bnl = 0;
    size_t bthr = 0;
    int bdir = 0;
    for (int dir : {1, -1}) {
      const size_t middle = dir == 1 ? (nu + 1) / 2 : (nu + 1) / 2 - 1;
      double gl = 0, hl = 0;
      uint32_t nl = 0;
      for (size_t i = 0; i < middle; ++i) {
        const size_t sidx = dir == 1 ? i : nu - 1 - i;
        const unsigned b = ci[sidx].bin;
        nl += h[b].c;
        const uint32_t nr = ns - nl;
        hl += P.hess_const ? (double)h[b].c : h[b].h;
        const double hr = sh - hl;
        gl += h[b].g;
        const double gr = sg - gl;
        if (nl < (uint32_t)P.min_samples_leaf || hl < P.min_hess) continue;
        if (nr < (uint32_t)P.min_samples_leaf || hr < P.min_hess) break;
        double gain = split_gain(gl, hl, gr, hr, loss_cur, 0, lo, hi, P.l2);
        if (gain > best && gain > P.min_gain) {
          found = true; best = gain; bthr = sidx; bgl = gl; bhl = hl; bnl = nl; bdir = dir;
        }
      }
    }
    if (!found) return;
    si.gain = best; si.bin = 0; si.is_cat = true;
    si.gl = bgl; si.hl = bhl; si.gr = sg - bgl; si.hr = sh - bhl;
    si.nl = bnl; si.nr = ns - bnl;
    si.vl = node_value(si.gl, si.hl, lo, hi, P.l2);
    si.vr = node_value(si.gr, si.hr, lo, hi, P.l2);
    for (int w = 0; w < 8; ++w) si.bits[w] = 0;
    if (bdir == 1) {
      for (size_t k = 0; k <= bthr; ++k) si.bits[ci[k].bin >> 5] |= 1u << (ci[k].bin & 31);
    } else {
      for (size_t k = nu - 1; k + 1 > bthr; --k) {
        si.bits[ci[k].bin >> 5] |= 1u << (ci[k].bin & 31);
        if (k == 0) break;
      }
    }
    si.missing_left = miss ? ((si.bits[mbin >> 5] >> (mbin & 31)) & 1u) != 0 : false;
  }

  void find_split(Node& nd) {
    std::vector<SplitInfo> infos(P.d);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) if (P.d > 4)
#endif
    for (int f = 0; f < P.d; ++f) scan_feature(nd, f, infos[f]);
    int best = 0;
    double bg = -1.0;
    for (int f = 0; f < P.d; ++f)
      if (infos[f].gain > bg) { bg = infos[f].gain; best = f; }
    nd.split = infos[best];
  }

  void finalize(int i) { nodes[i].is_leaf = true; finalized.push_back(i); }

  void split_and_push(int i) {
    find_split(nodes[i]);
    if (nodes[i].split.gain <= 0) finalize(i);
    else push(i);
  }

  bool goes_left(const SplitInfo& s, uint8_t b) const {
    if (s.is_cat) return ((s.bits[b >> 5] >> (b & 31)) & 1u) != 0;
    if (b == (uint8_t)(P.n_bins - 1)) return s.missing_left;
    return b <= (uint8_t)s.bin;
  }

  void grow() {
    nodes.reserve(2 * (size_t)std::max(P.max_leaf_nodes, 64) + 2);
    part.resize(P.n);
    for (int64_t i = 0; i < P.n; ++i) part[i] = (uint32_t)i;
    tmp.resize(P.n);
    Node root;
    root.depth = 0; root.start = 0; root.stop = P.n;
    double sg = 0, sh = 0;
    for (int64_t i = 0; i < P.n; ++i) sg += P.grad[i];
    if (P.hess_const) sh = (double)P.hess[0] * (double)P.n;
    else for (int64_t i = 0; i < P.n; ++i) sh += P.hess[i];
    root.sum_g = sg; root.sum_h = sh; root.value = 0.0;
    nodes.push_back(root);
    if (nodes[0].n() < 2u * (uint32_t)P.min_samples_leaf || sh < P.min_hess) {
      finalize(0);
    } else {
      build_hist(nodes[0]);
      split_and_push(0);
    }
    while (!heap.empty()) split_next();
    for (int i : finalized) nodes[i].value *= P.shrinkage;
  }

  void split_next() {
    int pi = pop();
    SplitInfo s = nodes[pi].split;
    const int64_t st = nodes[pi].start, sp = nodes[pi].stop;
    // stable partition of the node's slice
    const uint8_t* col = P.Xb + (size_t)s.feature * P.n;
    int64_t nl = 0, nr = 0;
    for (int64_t q = st; q < sp; ++q) {
      uint32_t i = part[q];
      if (goes_left(s, col[i])) part[st + nl++] = i;
      else tmp[nr++] = i;
    }
    std::memcpy(part.data() + st + nl, tmp.data(), sizeof(uint32_t) * nr);
    const int depth = nodes[pi].depth + 1;
    const int n_leaf_nodes = (int)(finalized.size() + heap.size()) + 2;
    Node L, R;
    L.depth = R.depth = depth;
    L.start = st; L.stop = st + nl;
    R.start = st + nl; R.stop = sp;
    L.sum_g = s.gl; L.sum_h = s.hl; L.value = s.vl;
    R.sum_g = s.gr; R.sum_h = s.hr; R.value = s.vr;
    if (!P.has_missing[s.feature]) nodes[pi].split.missing_left = L.n() > R.n();
    int li = (int)nodes.size();
    nodes.push_back(std::move(L));
    int ri = (int)nodes.size();
    nodes.push_back(std::move(R));
    nodes[pi].left = li;
    nodes[pi].right = ri;
    if (P.max_leaf_nodes > 0 && n_leaf_nodes == P.max_leaf_nodes) {
      finalize(li); finalize(ri);
      while (!heap.empty()) { int j = heap.back(); heap.pop_back(); finalize(j); }
      nodes[pi].hist.clear(); nodes[pi].hist.shrink_to_fit();
      return;
    }
    if (P.max_depth > 0 && depth == P.max_depth) {
      finalize(li); finalize(ri);
      nodes[pi].hist.clear(); nodes[pi].hist.shrink_to_fit();
      return;
    }
    if (nodes[li].n() < 2u * (uint32_t)P.min_samples_leaf) finalize(li);
    if (nodes[ri].n() < 2u * (uint32_t)P.min_samples_leaf) finalize(ri);
    const int8_t mono = P.mono[s.feature];
    if (mono == 0) {
      nodes[li].lower = nodes[ri].lower = nodes[pi].lower;
      nodes[li].upper = nodes[ri].upper = nodes[pi].upper;
    } else {
      double mid = (nodes[li].value + nodes[ri].value) / 2;
      if (mono == 1) {
        nodes[li].lower = nodes[pi].lower; nodes[li].upper = mid;
        nodes[ri].lower = mid; nodes[ri].upper = nodes[pi].upper;
      } else {
        nodes[li].lower = mid; nodes[li].upper = nodes[pi].upper;
        nodes[ri].lower = nodes[pi].lower; nodes[ri].upper = mid;
      }
    }
    bool sl = !nodes[li].is_leaf, sr = !nodes[ri].is_leaf;
    if (sl || sr) {
      int small = nodes[li].n() < nodes[ri].n() ? li : ri;
      int large = small == li ? ri : li;
      build_hist(nodes[small]);
      subtract_hist(nodes[pi], nodes[small], nodes[large]);
      if (sl) split_and_push(li);
      if (sr) split_and_push(ri);
      for (int c : {li, ri})
        if (nodes[c].is_leaf) { nodes[c].hist.clear(); nodes[c].hist.shrink_to_fit(); }
    }
    nodes[pi].hist.clear();
    nodes[pi].hist.shrink_to_fit();
  }
};

struct Result {
  // predictor nodes in depth-first preorder (reference _fill_predictor_arrays)
  std::vector<double> value, gain;
  std::vector<int32_t> count, feature, bin, left, right, depth;
  std::vector<uint8_t> missing_left, is_leaf, is_cat;
  std::vector<uint32_t> bits;            // 8 words per node (binned left bitset)
  std::vector<int32_t> leaf_of_sample;   // predictor node id of every training row
};

}  // namespace

extern "C" {

// Map float64 X (row-major n x d) to bins: thresholds concatenated per
// feature (offsets[f]..offsets[f+1]), NaN -> missing_bin.  Output column-major.
void sqh_hgb_map_bins(const double* X, long long n, int d, const double* thr,
                      const long long* offsets, int missing_bin, uint8_t* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (int f = 0; f < d; ++f) {
    const double* t = thr + offsets[f];
    const long long nt = offsets[f + 1] - offsets[f];
    for (long long i = 0; i < n; ++i) {
      double v = X[i * d + f];
      uint8_t b;
      if (std::isnan(v)) {
        b = (uint8_t)missing_bin;
      } else {
        long long lo = 0, hi = nt;
        while (lo < hi) {
          long long mid = lo + (hi - lo - 1) / 2;
          if (v <= t[mid]) hi = mid;
          else lo = mid + 1;
        }
        b = (uint8_t)lo;
      }
      out[(size_t)f * n + i] = b;
    }
  }
}

// prm: [max_leaf_nodes (<=0 none), max_depth (<=0 none), min_samples_leaf,
//       min_gain_to_split, l2, min_hessian_to_split, shrinkage, n_bins]
void* sqh_hgb_grow(const uint8_t* Xb, long long n, int d, const float* grad, const float* hess,
                   int hess_const, const uint32_t* nbnm, const uint8_t* has_missing,
                   const int8_t* mono, const double* prm, const uint8_t* is_cat) {
  Grower G;
  G.P = Params{n, d, (int)prm[7], Xb, grad, hess, hess_const != 0, nbnm, has_missing, mono,
               is_cat, (int)prm[0], (int)prm[1], (int)prm[2], prm[3], prm[4], prm[5], prm[6]};
  G.grow();
  auto* R = new Result();
  R->leaf_of_sample.assign(n, -1);
  // preorder renumbering
  std::vector<int> stack{0};
  std::vector<int> newid(G.nodes.size(), -1);
  std::vector<int> order;
  while (!stack.empty()) {
    int i = stack.back();
    stack.pop_back();
    newid[i] = (int)order.size();
    order.push_back(i);
    const Node& nd = G.nodes[i];
    if (!nd.is_leaf) { stack.push_back(nd.right); stack.push_back(nd.left); }
  }
  const size_t m = order.size();
  R->value.resize(m); R->gain.resize(m); R->count.resize(m); R->feature.resize(m);
  R->bin.resize(m); R->left.resize(m); R->right.resize(m); R->depth.resize(m);
  R->missing_left.resize(m); R->is_leaf.resize(m);
  R->is_cat.assign(m, 0); R->bits.assign(8 * m, 0u);
  for (size_t k = 0; k < m; ++k) {
    const Node& nd = G.nodes[order[k]];
    R->value[k] = nd.value;
    R->count[k] = (int32_t)nd.n();
    R->depth[k] = nd.depth;
    R->is_leaf[k] = nd.is_leaf ? 1 : 0;
    if (nd.is_leaf) {
      R->gain[k] = -1; R->feature[k] = 0; R->bin[k] = 0; R->missing_left[k] = 0;
      R->left[k] = R->right[k] = 0;
      for (int64_t q = nd.start; q < nd.stop; ++q) R->leaf_of_sample[G.part[q]] = (int32_t)k;
    } else {
      R->gain[k] = nd.split.gain; R->feature[k] = nd.split.feature; R->bin[k] = nd.split.bin;
      R->missing_left[k] = nd.split.missing_left ? 1 : 0;
      R->left[k] = newid[nd.left]; R->right[k] = newid[nd.right];
      if (nd.split.is_cat) {
        R->is_cat[k] = 1;
        for (int w = 0; w < 8; ++w) R->bits[8 * k + w] = nd.split.bits[w];
      }
    }
  }
  return R;
}

long long sqh_hgb_size(void* h) { return (long long)((Result*)h)->value.size(); }

void sqh_hgb_copy(void* h, double* value, double* gain, int* count, int* feature, int* bin,
                  int* left, int* right, int* depth, uint8_t* missing_left, uint8_t* is_leaf,
                  int* leaf_of_sample, long long n) {
  auto* R = (Result*)h;
  size_t m = R->value.size();
  std::memcpy(value, R->value.data(), m * 8);
  std::memcpy(gain, R->gain.data(), m * 8);
  std::memcpy(count, R->count.data(), m * 4);
  std::memcpy(feature, R->feature.data(), m * 4);
  std::memcpy(bin, R->bin.data(), m * 4);
  std::memcpy(left, R->left.data(), m * 4);
  std::memcpy(right, R->right.data(), m * 4);
  std::memcpy(depth, R->depth.data(), m * 4);
  std::memcpy(missing_left, R->missing_left.data(), m);
  std::memcpy(is_leaf, R->is_leaf.data(), m);
  if (leaf_of_sample) std::memcpy(leaf_of_sample, R->leaf_of_sample.data(), (size_t)n * 4);
}

void sqh_hgb_copy_cat(void* h, uint8_t* is_cat, uint32_t* bits) {
  auto* R = (Result*)h;
  std::memcpy(is_cat, R->is_cat.data(), R->is_cat.size());
  std::memcpy(bits, R->bits.data(), R->bits.size() * 4);
}

void sqh_hgb_free(void* h) { delete (Result*)h; }

// As sqh_hgb_predict, with categorical nodes: raw category c goes left if
// it is in the node's raw bitset, right if it is a known category, and
// follows the missing direction otherwise (reference _predictor.pyx).
void sqh_hgb_predict_cat(const double* X, long long n, int d, const int* feature,
                         const double* thr, const uint8_t* missing_left, const int* left,
                         const int* right, const uint8_t* is_leaf, const double* value,
                         const uint8_t* is_cat, const uint32_t* raw_bits,
                         const uint32_t* known_bits, const long long* offs, int T, double* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (long long i = 0; i < n; ++i) {
    const double* xi = X + i * d;
    double acc = 0.0;
    for (int t = 0; t < T; ++t) {
      const long long b = offs[t];
      long long k = 0;
      while (!is_leaf[b + k]) {
        const long long q = b + k;
        const int f = feature[q];
        const double v = xi[f];
        bool gl;
        if (std::isnan(v)) {
          gl = missing_left[q] != 0;
        } else if (is_cat[q]) {
          if (v >= 0 && v < 256) {
            const unsigned c = (unsigned)v;
            if ((raw_bits[8 * q + (c >> 5)] >> (c & 31)) & 1u) gl = true;
            else if ((known_bits[8 * f + (c >> 5)] >> (c & 31)) & 1u) gl = false;
            else gl = missing_left[q] != 0;
          } else {
            gl = missing_left[q] != 0;
          }
        } else {
          gl = v <= thr[q];
        }
        k = gl ? left[q] : right[q];
      }
      acc += value[b + k];
    }
    out[i] = acc;
  }
}

// Raw predictions of T stacked predictors on float64 rows (NaN-aware):
// out[i] = sum_t value_t[leaf].  Node arrays concatenated, offsets per tree.
void sqh_hgb_predict(const double* X, long long n, int d, const int* feature,
                     const double* thr, const uint8_t* missing_left, const int* left,
                     const int* right, const uint8_t* is_leaf, const double* value,
                     const long long* offs, int T, double* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (long long i = 0; i < n; ++i) {
    const double* xi = X + i * d;
    double acc = 0.0;
    for (int t = 0; t < T; ++t) {
      const long long b = offs[t];
      long long k = 0;
      while (!is_leaf[b + k]) {
        double v = xi[feature[b + k]];
        bool gl = std::isnan(v) ? missing_left[b + k] != 0 : v <= thr[b + k];
        k = gl ? left[b + k] : right[b + k];
      }
      acc += value[b + k];
    }
    out[i] = acc;
  }
}

}  // extern "C"
