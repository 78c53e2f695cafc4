// CART decision-tree induction (reference
// ``tree/_tree.pyx`` builders, ``tree/_splitter.pyx`` Best/Random splitters,
// ``tree/_criterion.pyx`` criteria, ``tree/_utils.pyx`` heap / weighted
// median).  Host-native: node splitting is branchy, data dependent and
// sequential per tree, so it runs on the CPU; forests build their trees in
// parallel with OpenMP (one tree per thread), and inference of fitted trees
// also has a device kernel (``csrc/forest.hip``).
//
// Semantics kept from the reference so fitted trees are the same trees:
//  * samples with zero weight are dropped before growing;
//  * feature draws are a Fisher-Yates walk over the non-constant features
//    with the reference's 32-bit xorshift stream (seeded by the caller with
//    ``random_state.randint(0, 2**31 - 1)``), constant features found in an
//    ancestor are remembered (depth-first builder) and skipped;
//  * best splits scan sorted feature values, skip gaps <= 1e-7, keep the
//    first strictly better proxy improvement, threshold = midpoint (or the
//    lower value when the midpoint rounds to the upper one);
//  * extra-trees draw one uniform threshold in (min, max) per feature;
//  * depth-first node order (left subtree first) or best-first growth with
//    the reference's binary max-heap on impurity improvement;
//  * criteria: gini, entropy (log2), squared error, Friedman MSE, absolute
//    error (weighted median; here with Fenwick order statistics instead of
//    the reference's O(n) weighted-median queue), Poisson (half deviance,
//    weighted proxy - the reference's unweighted proxy at
//    ``_criterion.pyx:1398-1401`` is a defect fixed upstream later).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

#include "host.h"

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

constexpr double kInf = INFINITY;
constexpr double kEps = DBL_EPSILON;
constexpr float kFeatThr = 1e-7f;
constexpr uint32_t kRandMax = 0x7FFFFFFFu;

enum Crit { GINI = 0, ENTROPY = 1, MSE = 2, FRIEDMAN = 3, MAE = 4, POISSON = 5 };

inline uint32_t rand_r32(uint32_t* s) {
  if (*s == 0) *s = 1;
  *s ^= (uint32_t)(*s << 13);
  *s ^= (uint32_t)(*s >> 17);
  *s ^= (uint32_t)(*s << 5);
  return *s % (kRandMax + 1u);
}
inline int64_t rand_int(int64_t lo, int64_t hi, uint32_t* s) {
  return lo + (int64_t)(rand_r32(s) % (uint32_t)(hi - lo));
}
inline double rand_uniform(double lo, double hi, uint32_t* s) {
  return (hi - lo) * (double)rand_r32(s) / (double)kRandMax + lo;
}
inline double log2d(double x) { return std::log(x) / std::log(2.0); }
inline double xlogy(double x, double y) { return x == 0.0 ? 0.0 : x * std::log(y); }

struct Data {
  const float* X;     // column-major: X[f * n + i]
  const double* y;    // row-major n x n_outputs
  const double* sw;   // n or null
  int64_t n, d;
  int n_outputs;
  const int64_t* n_classes;  // classification: per output; null for regression
  int64_t max_n_classes;
  inline float x(int64_t i, int64_t f) const { return X[f * n + i]; }
  inline double w(int64_t i) const { return sw ? sw[i] : 1.0; }
};

// Fenwick tree over y-ranks holding (weight, weight * y): weighted median and
// absolute deviations of a dynamic sample set in O(log n).
struct Fenwick {
  std::vector<double> W, WY;
  int64_t n = 0, top = 1;
  void init(int64_t n_) {
    n = n_;
    W.assign(n + 1, 0.0);
    WY.assign(n + 1, 0.0);
    top = 1;
    while (top * 2 <= n) top *= 2;
  }
  void add(int64_t r, double w, double wy) {
    for (int64_t i = r + 1; i <= n; i += i & -i) { W[i] += w; WY[i] += wy; }
  }
  void prefix(int64_t r, double* w, double* wy) const {  // ranks [0, r]
    double a = 0, b = 0;
    for (int64_t i = r + 1; i > 0; i -= i & -i) { a += W[i]; b += WY[i]; }
    *w = a; *wy = b;
  }
  // smallest rank r with prefix weight(r) >= t (or > t when strict)
  int64_t search(double t, bool strict) const {
    int64_t pos = 0;
    double acc = 0;
    for (int64_t step = top; step > 0; step >>= 1) {
      int64_t nxt = pos + step;
      if (nxt <= n) {
        double v = acc + W[nxt];
        if (strict ? (v <= t) : (v < t)) { pos = nxt; acc = v; }
      }
    }
    return pos;  // 0-based rank
  }
};

struct Criterion {
  const Data* D;
  int crit;
  int K;          // n_outputs
  int64_t S;      // stride of per-output sums (max_n_classes or 1)
  const int64_t* samples = nullptr;
  int64_t start = 0, end = 0, pos = 0;
  double wn_total = 0, wn_node = 0, wn_left = 0, wn_right = 0;
  std::vector<double> sum_total, sum_left, sum_right;
  double sq_total = 0;
  // absolute error: per-output Fenwick sets of the left / right children
  std::vector<Fenwick> fl, fr;
  const std::vector<std::vector<int64_t>>* rank = nullptr;
  const std::vector<std::vector<double>>* ysorted = nullptr;
  bool mae_active = false;

  void setup(const Data* d, int c, const std::vector<std::vector<int64_t>>* rk,
             const std::vector<std::vector<double>>* ys) {
    D = d; crit = c; K = d->n_outputs;
    S = (c == GINI || c == ENTROPY) ? d->max_n_classes : 1;
    sum_total.assign(K * S, 0.0); sum_left.assign(K * S, 0.0); sum_right.assign(K * S, 0.0);
    if (crit == MAE) {
      rank = rk; ysorted = ys;
      fl.resize(K); fr.resize(K);
      for (int k = 0; k < K; ++k) { fl[k].init(d->n); fr[k].init(d->n); }
    }
  }
  bool classif() const { return crit == GINI || crit == ENTROPY; }

  void init(const int64_t* smp, int64_t s, int64_t e) {
    mae_release();
    samples = smp; start = s; end = e;
    std::fill(sum_total.begin(), sum_total.end(), 0.0);
    wn_node = 0; sq_total = 0;
    for (int64_t p = s; p < e; ++p) {
      int64_t i = smp[p];
      double w = D->w(i);
      const double* yi = D->y + i * K;
      if (classif()) {
        for (int k = 0; k < K; ++k) sum_total[k * S + (int64_t)yi[k]] += w;
      } else {
        for (int k = 0; k < K; ++k) { sum_total[k] += w * yi[k]; sq_total += w * yi[k] * yi[k]; }
      }
      wn_node += w;
    }
    pos = start;
    reset();
  }

  void mae_add(int64_t from, int64_t to, std::vector<Fenwick>& f, double sign) {
    for (int64_t p = from; p < to; ++p) {
      int64_t i = samples[p];
      double w = D->w(i) * sign;
      for (int k = 0; k < K; ++k) {
        double yv = D->y[i * K + k];
        f[k].add((*rank)[k][i], w, w * yv);
      }
    }
  }
  // Empty both Fenwick sets (they hold samples[start:pos] left, [pos:end] right).
  // Must run before samples[start:end] is permuted.
  void mae_release() {
    if (crit != MAE || !mae_active) return;
    mae_add(start, pos, fl, -1.0);
    mae_add(pos, end, fr, -1.0);
    mae_active = false;
  }

  void reset() {
    if (crit == MAE) {
      if (mae_active) { mae_add(start, pos, fl, -1.0); mae_add(start, pos, fr, +1.0); }
      else { mae_add(start, end, fr, +1.0); mae_active = true; }
    }
    pos = start;
    wn_left = 0; wn_right = wn_node;
    std::fill(sum_left.begin(), sum_left.end(), 0.0);
    sum_right = sum_total;
  }

  // Moves samples[pos:new_pos] to the left child.  Like the reference
  // (``_criterion.pyx:439-465``) the sums are accumulated from whichever end
  // is closer, so the rounding of sum_left / sum_right matches its trees.
  void update(int64_t new_pos) {
    if (crit == MAE) {
      for (int64_t p = pos; p < new_pos; ++p) {
        int64_t i = samples[p];
        double w = D->w(i);
        const double* yi = D->y + i * K;
        for (int k = 0; k < K; ++k) {
          int64_t r = (*rank)[k][i];
          fr[k].add(r, -w, -w * yi[k]);
          fl[k].add(r, w, w * yi[k]);
        }
      }
    }
    if (new_pos - pos <= end - new_pos) {
      for (int64_t p = pos; p < new_pos; ++p) {
        int64_t i = samples[p];
        double w = D->w(i);
        const double* yi = D->y + i * K;
        if (classif()) {
          for (int k = 0; k < K; ++k) sum_left[k * S + (int64_t)yi[k]] += w;
        } else {
          for (int k = 0; k < K; ++k) sum_left[k] += w * yi[k];
        }
        wn_left += w;
      }
    } else {
      sum_left = sum_total;
      wn_left = wn_node;
      for (int64_t p = end - 1; p >= new_pos; --p) {
        int64_t i = samples[p];
        double w = D->w(i);
        const double* yi = D->y + i * K;
        if (classif()) {
          for (int k = 0; k < K; ++k) sum_left[k * S + (int64_t)yi[k]] -= w;
        } else {
          for (int k = 0; k < K; ++k) sum_left[k] -= w * yi[k];
        }
        wn_left -= w;
      }
    }
    pos = new_pos;
    wn_right = wn_node - wn_left;
    for (size_t j = 0; j < sum_left.size(); ++j) sum_right[j] = sum_total[j] - sum_left[j];
  }

  double class_imp(const double* sums, double wn) const {
    double acc = 0;
    for (int k = 0; k < K; ++k) {
      const double* c = sums + k * S;
      int64_t nc = D->n_classes[k];
      if (crit == GINI) {
        double sq = 0;
        for (int64_t j = 0; j < nc; ++j) sq += c[j] * c[j];
        acc += 1.0 - sq / (wn * wn);
      } else {
        double ent = 0;
        for (int64_t j = 0; j < nc; ++j)
          if (c[j] > 0.0) { double q = c[j] / wn; ent -= q * log2d(q); }
        acc += ent;
      }
    }
    return acc / K;
  }

  // weighted median (reference WeightedMedianCalculator definition) and
  // sum_i w_i |y_i - median| of one Fenwick set
  void mae_stats(const Fenwick& f, int k, double wn, double* med, double* dev) const {
    double half = wn / 2.0;
    int64_t r = f.search(half, false);
    double cw, cwy;
    f.prefix(r, &cw, &cwy);
    const std::vector<double>& ys = (*ysorted)[k];
    double m = ys[r];
    if (cw == half) {
      int64_t r2 = f.search(half, true);
      if (r2 < f.n) m = (ys[r] + ys[r2]) / 2.0;
    }
    double tw, twy;
    f.prefix(f.n - 1, &tw, &twy);
    *med = m;
    *dev = (m * cw - cwy) + ((twy - cwy) - m * (tw - cw));
  }

  double poisson_loss(int64_t s, int64_t e, const double* ysum, double wsum) const {
    double loss = 0;
    for (int k = 0; k < K; ++k) {
      if (ysum[k] <= kEps) return kInf;
      double ym = ysum[k] / wsum;
      for (int64_t p = s; p < e; ++p) {
        int64_t i = samples[p];
        double yv = D->y[i * K + k];
        loss += D->w(i) * xlogy(yv, yv / ym);
      }
    }
    return loss / (wsum * K);
  }

  double node_impurity() {
    if (classif()) return class_imp(sum_total.data(), wn_node);
    if (crit == MAE) {
      reset();
      double acc = 0;
      for (int k = 0; k < K; ++k) {
        double med, dev;
        mae_stats(fr[k], k, wn_node, &med, &dev);
        acc += dev / wn_node;
      }
      return acc / K;
    }
    if (crit == POISSON) return poisson_loss(start, end, sum_total.data(), wn_node);
    double imp = sq_total / wn_node;
    for (int k = 0; k < K; ++k) { double m = sum_total[k] / wn_node; imp -= m * m; }
    return imp / K;
  }

  void children_impurity(double* il, double* ir) {
    if (classif()) {
      *il = class_imp(sum_left.data(), wn_left);
      *ir = class_imp(sum_right.data(), wn_right);
      return;
    }
    if (crit == MAE) {
      double a = 0, b = 0;
      for (int k = 0; k < K; ++k) {
        double med, dev;
        mae_stats(fl[k], k, wn_left, &med, &dev); a += dev / wn_left;
        mae_stats(fr[k], k, wn_right, &med, &dev); b += dev / wn_right;
      }
      *il = a / K; *ir = b / K;
      return;
    }
    if (crit == POISSON) {
      *il = poisson_loss(start, pos, sum_left.data(), wn_left);
      *ir = poisson_loss(pos, end, sum_right.data(), wn_right);
      return;
    }
    double sql = 0;
    for (int64_t p = start; p < pos; ++p) {
      int64_t i = samples[p];
      double w = D->w(i);
      for (int k = 0; k < K; ++k) { double yv = D->y[i * K + k]; sql += w * yv * yv; }
    }
    double sqr = sq_total - sql;
    double a = sql / wn_left, b = sqr / wn_right;
    for (int k = 0; k < K; ++k) {
      double ml = sum_left[k] / wn_left, mr = sum_right[k] / wn_right;
      a -= ml * ml; b -= mr * mr;
    }
    *il = a / K; *ir = b / K;
  }

  double proxy_improvement() {
    if (crit == MSE) {
      double pl = 0, pr = 0;
      for (int k = 0; k < K; ++k) { pl += sum_left[k] * sum_left[k]; pr += sum_right[k] * sum_right[k]; }
      return pl / wn_left + pr / wn_right;
    }
    if (crit == FRIEDMAN) {
      double tl = 0, tr = 0;
      for (int k = 0; k < K; ++k) { tl += sum_left[k]; tr += sum_right[k]; }
      double diff = wn_right * tl - wn_left * tr;
      return diff * diff / (wn_left * wn_right);
    }
    if (crit == POISSON) {
      double pl = 0, pr = 0;
      for (int k = 0; k < K; ++k) {
        if (sum_left[k] <= kEps || sum_right[k] <= kEps) return -kInf;
        pl -= sum_left[k] * log2d(sum_left[k] / wn_left);
        pr -= sum_right[k] * log2d(sum_right[k] / wn_right);
      }
      return -pl - pr;
    }
    double il, ir;
    children_impurity(&il, &ir);
    return -wn_right * ir - wn_left * il;
  }

  double impurity_improvement(double parent, double il, double ir) const {
    if (crit == FRIEDMAN) {
      double tl = 0, tr = 0;
      for (int k = 0; k < K; ++k) { tl += sum_left[k]; tr += sum_right[k]; }
      double diff = (wn_right * tl - wn_left * tr) / K;
      return diff * diff / (wn_left * wn_right * wn_node);
    }
    return (wn_node / wn_total) *
           (parent - wn_right / wn_node * ir - wn_left / wn_node * il);
  }

  void node_value(double* out) {
    if (classif()) {
      std::memcpy(out, sum_total.data(), sizeof(double) * K * S);
    } else if (crit == MAE) {
      reset();
      for (int k = 0; k < K; ++k) { double dev; mae_stats(fr[k], k, wn_node, &out[k], &dev); }
    } else {
      for (int k = 0; k < K; ++k) out[k] = sum_total[k] / wn_node;
    }
  }
};

struct Split {
  int64_t feature = 0, pos = 0;
  double threshold = 0, improvement = -kInf, imp_left = kInf, imp_right = kInf;
};

struct Params {
  int crit, splitter;          // splitter: 0 best, 1 random
  int64_t max_depth, min_samples_split, min_samples_leaf, max_features, max_leaf_nodes;
  double min_weight_leaf, min_impurity_decrease;
};

struct TreeOut {
  std::vector<int64_t> left, right, feature, n_node;
  std::vector<double> threshold, impurity, wn, value;
  int64_t stride = 0, max_depth = 0;
  int64_t add(int64_t parent, bool is_left, bool leaf, int64_t f, double t, double imp,
              int64_t nn, double w) {
    int64_t id = (int64_t)left.size();
    left.push_back(-1); right.push_back(-1);
    feature.push_back(leaf ? -2 : f);
    threshold.push_back(leaf ? -2.0 : t);
    impurity.push_back(imp); n_node.push_back(nn); wn.push_back(w);
    value.resize(value.size() + stride, 0.0);
    if (parent >= 0) (is_left ? left : right)[parent] = id;
    return id;
  }
};

struct Splitter {
  const Data* D;
  Params P;
  Criterion crit;
  uint32_t rs;
  std::vector<int64_t> samples, features, constant_features;
  std::vector<float> Xf;
  std::vector<std::pair<float, int64_t>> tmp;
  double wn_samples = 0;

  int64_t init(const Data* d, const Params& p, uint32_t seed,
               const std::vector<std::vector<int64_t>>* rk,
               const std::vector<std::vector<double>>* ys) {
    D = d; P = p; rs = seed;
    samples.clear();
    wn_samples = 0;
    for (int64_t i = 0; i < d->n; ++i) {
      if (!d->sw || d->sw[i] != 0.0) { samples.push_back(i); wn_samples += d->w(i); }
    }
    features.resize(d->d);
    for (int64_t f = 0; f < d->d; ++f) features[f] = f;
    constant_features.assign(d->d, 0);
    Xf.assign(samples.size(), 0.f);
    crit.setup(d, p.crit, rk, ys);
    crit.wn_total = wn_samples;
    return (int64_t)samples.size();
  }

  void sort_range(int64_t s, int64_t e) {
    int64_t m = e - s;
    tmp.resize(m);
    for (int64_t q = 0; q < m; ++q) tmp[q] = {Xf[s + q], samples[s + q]};
    std::sort(tmp.begin(), tmp.end(),
              [](const std::pair<float, int64_t>& a, const std::pair<float, int64_t>& b) {
                return a.first < b.first;
              });
    for (int64_t q = 0; q < m; ++q) { Xf[s + q] = tmp[q].first; samples[s + q] = tmp[q].second; }
  }

  void node_split(int64_t start, int64_t end, double impurity, Split* out, int64_t* n_const) {
    int64_t f_i = D->d, n_visited = 0, n_found = 0, n_drawn = 0;
    const int64_t n_known = *n_const;
    int64_t n_total = n_known;
    Split best;
    best.pos = end;
    double best_proxy = -kInf;
    const bool random = P.splitter == 1;

    while (f_i > n_total && (n_visited < P.max_features || n_visited <= n_found + n_drawn)) {
      ++n_visited;
      int64_t f_j = rand_int(n_drawn, f_i - n_found, &rs);
      if (f_j < n_known) {
        std::swap(features[n_drawn], features[f_j]);
        ++n_drawn;
        continue;
      }
      f_j += n_found;
      Split cur;
      cur.feature = features[f_j];
      if (!random) {
        for (int64_t p = start; p < end; ++p) Xf[p] = D->x(samples[p], cur.feature);
        crit.mae_release();
        sort_range(start, end);
        if (Xf[end - 1] <= Xf[start] + kFeatThr) {
          std::swap(features[f_j], features[n_total]);
          ++n_found; ++n_total;
          continue;
        }
        --f_i;
        std::swap(features[f_i], features[f_j]);
        crit.reset();
        int64_t p = start;
        while (p < end) {
          while (p + 1 < end && Xf[p + 1] <= Xf[p] + kFeatThr) ++p;
          ++p;
          if (p >= end) continue;
          cur.pos = p;
          if (cur.pos - start < P.min_samples_leaf || end - cur.pos < P.min_samples_leaf) continue;
          crit.update(cur.pos);
          if (crit.wn_left < P.min_weight_leaf || crit.wn_right < P.min_weight_leaf) continue;
          double pr = crit.proxy_improvement();
          if (pr > best_proxy) {
            best_proxy = pr;
            cur.threshold = (double)Xf[p - 1] / 2.0 + (double)Xf[p] / 2.0;
            if (cur.threshold == (double)Xf[p] || std::isinf(cur.threshold))
              cur.threshold = Xf[p - 1];
            best = cur;
          }
        }
      } else {
        float mn = D->x(samples[start], cur.feature), mx = mn;
        Xf[start] = mn;
        for (int64_t p = start + 1; p < end; ++p) {
          float v = D->x(samples[p], cur.feature);
          Xf[p] = v;
          if (v < mn) mn = v;
          else if (v > mx) mx = v;
        }
        if (mx <= mn + kFeatThr) {
          std::swap(features[f_j], features[n_total]);
          ++n_found; ++n_total;
          continue;
        }
        --f_i;
        std::swap(features[f_i], features[f_j]);
        cur.threshold = rand_uniform(mn, mx, &rs);
        if (cur.threshold == (double)mx) cur.threshold = mn;
        crit.mae_release();
        int64_t p = start, pe = end;
        while (p < pe) {
          if ((double)Xf[p] <= cur.threshold) ++p;
          else { --pe; std::swap(Xf[p], Xf[pe]); std::swap(samples[p], samples[pe]); }
        }
        cur.pos = pe;
        if (cur.pos - start < P.min_samples_leaf || end - cur.pos < P.min_samples_leaf) continue;
        crit.reset();
        crit.update(cur.pos);
        if (crit.wn_left < P.min_weight_leaf || crit.wn_right < P.min_weight_leaf) continue;
        double pr = crit.proxy_improvement();
        if (pr > best_proxy) { best_proxy = pr; best = cur; }
      }
    }

    if (best.pos < end) {
      crit.mae_release();
      int64_t p = start, pe = end;
      while (p < pe) {
        if ((double)D->x(samples[p], best.feature) <= best.threshold) ++p;
        else { --pe; std::swap(samples[p], samples[pe]); }
      }
      best.pos = pe;
      crit.reset();
      crit.update(best.pos);
      crit.children_impurity(&best.imp_left, &best.imp_right);
      best.improvement = crit.impurity_improvement(impurity, best.imp_left, best.imp_right);
    }
    std::memcpy(features.data(), constant_features.data(), sizeof(int64_t) * n_known);
    std::memcpy(constant_features.data() + n_known, features.data() + n_known,
                sizeof(int64_t) * n_found);
    *out = best;
    *n_const = n_total;
  }

  void node_reset(int64_t s, int64_t e) { crit.init(samples.data(), s, e); }
};

struct StackRec { int64_t start, end, depth, parent; bool is_left; double impurity; int64_t n_const; };
struct HeapRec {
  int64_t node_id, start, end, pos, depth; bool is_leaf;
  double improvement, impurity, imp_left, imp_right;
};

struct MaxHeap {  // reference PriorityHeap (tree/_utils.pyx)
  std::vector<HeapRec> h;
  void up(size_t pos) {
    while (pos > 0) {
      size_t par = (pos - 1) / 2;
      if (h[par].improvement < h[pos].improvement) { std::swap(h[par], h[pos]); pos = par; }
      else break;
    }
  }
  void down(size_t pos, size_t len) {
    for (;;) {
      size_t l = 2 * pos + 1, r = 2 * pos + 2, big = pos;
      if (l < len && h[l].improvement > h[big].improvement) big = l;
      if (r < len && h[r].improvement > h[big].improvement) big = r;
      if (big == pos) break;
      std::swap(h[pos], h[big]);
      pos = big;
    }
  }
  void push(const HeapRec& r) { h.push_back(r); up(h.size() - 1); }
  HeapRec pop() {
    HeapRec r = h[0];
    std::swap(h[0], h.back());
    h.pop_back();
    if (h.size() > 1) down(0, h.size());
    return r;
  }
};

// Node bookkeeping shared by both builders: leaf tests, split, value.
struct NodeResult { int64_t id; bool leaf; Split s; double impurity; int64_t n_const; };

NodeResult grow_node(Splitter& sp, TreeOut& T, int64_t start, int64_t end, int64_t depth,
                     int64_t parent, bool is_left, double impurity, bool first,
                     int64_t n_const) {
  const Params& P = sp.P;
  int64_t nn = end - start;
  sp.node_reset(start, end);
  double wn = sp.crit.wn_node;
  bool leaf = depth >= P.max_depth || nn < P.min_samples_split || nn < 2 * P.min_samples_leaf ||
              wn < 2 * P.min_weight_leaf;
  if (first) impurity = sp.crit.node_impurity();
  leaf = leaf || impurity <= kEps;
  Split s;
  s.pos = end;
  if (!leaf) {
    sp.node_split(start, end, impurity, &s, &n_const);
    leaf = s.pos >= end || s.improvement + kEps < P.min_impurity_decrease;
  }
  int64_t id = T.add(parent, is_left, leaf, s.feature, s.threshold, impurity, nn, wn);
  sp.node_reset(start, end);   // node value over the whole node
  sp.crit.node_value(T.value.data() + id * T.stride);
  return {id, leaf, s, impurity, n_const};
}

void build_depth_first(Splitter& sp, TreeOut& T) {
  std::vector<StackRec> stack;
  int64_t n = (int64_t)sp.samples.size();
  stack.push_back({0, n, 0, -1, false, kInf, 0});
  bool first = true;
  int64_t max_depth_seen = -1;
  while (!stack.empty()) {
    StackRec r = stack.back();
    stack.pop_back();
    NodeResult nr = grow_node(sp, T, r.start, r.end, r.depth, r.parent, r.is_left, r.impurity,
                              first, r.n_const);
    first = false;
    if (!nr.leaf) {
      stack.push_back({nr.s.pos, r.end, r.depth + 1, nr.id, false, nr.s.imp_right, nr.n_const});
      stack.push_back({r.start, nr.s.pos, r.depth + 1, nr.id, true, nr.s.imp_left, nr.n_const});
    }
    if (r.depth > max_depth_seen) max_depth_seen = r.depth;
  }
  sp.crit.mae_release();
  T.max_depth = max_depth_seen;
}

HeapRec frontier_node(Splitter& sp, TreeOut& T, int64_t start, int64_t end, double impurity,
                      bool first, bool is_left, int64_t parent, int64_t depth) {
  NodeResult nr = grow_node(sp, T, start, end, depth, parent, is_left, impurity, first, 0);
  if (nr.leaf)
    return {nr.id, start, end, end, depth, true, 0.0, nr.impurity, nr.impurity, nr.impurity};
  return {nr.id, start, end, nr.s.pos, depth, false, nr.s.improvement, nr.impurity,
          nr.s.imp_left, nr.s.imp_right};
}

void build_best_first(Splitter& sp, TreeOut& T) {
  int64_t max_split = sp.P.max_leaf_nodes - 1;
  int64_t n = (int64_t)sp.samples.size();
  MaxHeap frontier;
  frontier.push(frontier_node(sp, T, 0, n, kInf, true, false, -1, 0));
  int64_t max_depth_seen = -1;
  while (!frontier.h.empty()) {
    HeapRec r = frontier.pop();
    bool leaf = r.is_leaf || max_split <= 0;
    if (leaf) {
      T.left[r.node_id] = -1; T.right[r.node_id] = -1;
      T.feature[r.node_id] = -2; T.threshold[r.node_id] = -2.0;
    } else {
      --max_split;
      HeapRec L = frontier_node(sp, T, r.start, r.pos, r.imp_left, false, true, r.node_id,
                                r.depth + 1);
      HeapRec R = frontier_node(sp, T, r.pos, r.end, r.imp_right, false, false, r.node_id,
                                r.depth + 1);
      frontier.push(L);
      frontier.push(R);
    }
    if (r.depth > max_depth_seen) max_depth_seen = r.depth;
  }
  sp.crit.mae_release();
  T.max_depth = max_depth_seen;
}

void make_ranks(const Data& D, std::vector<std::vector<int64_t>>& rank,
                std::vector<std::vector<double>>& ys) {
  int K = D.n_outputs;
  rank.assign(K, std::vector<int64_t>(D.n));
  ys.assign(K, std::vector<double>(D.n));
  std::vector<int64_t> idx(D.n);
  for (int k = 0; k < K; ++k) {
    for (int64_t i = 0; i < D.n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
      return D.y[a * K + k] < D.y[b * K + k];
    });
    for (int64_t r = 0; r < D.n; ++r) { rank[k][idx[r]] = r; ys[k][r] = D.y[idx[r] * K + k]; }
  }
}

TreeOut* grow(const Data& D, const Params& P, uint32_t seed,
              const std::vector<std::vector<int64_t>>* rk,
              const std::vector<std::vector<double>>* ys) {
  auto* T = new TreeOut();
  T->stride = (int64_t)D.n_outputs * ((P.crit == GINI || P.crit == ENTROPY) ? D.max_n_classes : 1);
  Splitter sp;
  sp.init(&D, P, seed, rk, ys);
  if (sp.samples.empty()) {  // no sample with positive weight: single empty leaf
    T->add(-1, false, true, 0, 0, 0.0, 0, 0.0);
    return T;
  }
  if (P.max_leaf_nodes > 0) build_best_first(sp, *T);
  else build_depth_first(sp, *T);
  return T;
}

Params make_params(const double* prm) {
  Params P;
  P.crit = (int)prm[0]; P.splitter = (int)prm[1];
  P.max_depth = (int64_t)prm[2]; P.min_samples_split = (int64_t)prm[3];
  P.min_samples_leaf = (int64_t)prm[4]; P.max_features = (int64_t)prm[5];
  P.max_leaf_nodes = (int64_t)prm[6]; P.min_weight_leaf = prm[7];
  P.min_impurity_decrease = prm[8];
  return P;
}

}  // namespace

extern "C" {

// params: [criterion, splitter, max_depth, min_samples_split, min_samples_leaf,
//          max_features, max_leaf_nodes (<=0: depth-first), min_weight_leaf,
//          min_impurity_decrease]
// sw: n_trees x n weights (bootstrap counts folded in) or null; seeds: n_trees.
// handles: n_trees output pointers.
void sqh_forest_build(const float* Xc, const double* y, const double* sw, long long n,
                      long long d, int n_outputs, const long long* n_classes,
                      long long max_n_classes, const double* prm, const uint32_t* seeds,
                      int n_trees, int n_threads, void** handles) {
  Params P = make_params(prm);
  std::vector<std::vector<int64_t>> rank;
  std::vector<std::vector<double>> ys;
  Data base{Xc, y, nullptr, n, d, n_outputs, (const int64_t*)n_classes, max_n_classes};
  if (P.crit == MAE) make_ranks(base, rank, ys);
#ifdef _OPENMP
  if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads)
#endif
  for (int t = 0; t < n_trees; ++t) {
    Data D = base;
    D.sw = sw ? sw + (int64_t)t * n : nullptr;
    handles[t] = grow(D, P, seeds[t], &rank, &ys);
  }
}

// sizes: [node_count, max_depth, value_stride]
void sqh_tree_sizes(void* h, long long* out) {
  auto* T = (TreeOut*)h;
  out[0] = (long long)T->left.size();
  out[1] = T->max_depth;
  out[2] = T->stride;
}

void sqh_tree_copy(void* h, long long* left, long long* right, long long* feature,
                   double* threshold, double* impurity, long long* n_node, double* wn,
                   double* value) {
  auto* T = (TreeOut*)h;
  size_t m = T->left.size();
  std::memcpy(left, T->left.data(), m * 8);
  std::memcpy(right, T->right.data(), m * 8);
  std::memcpy(feature, T->feature.data(), m * 8);
  std::memcpy(threshold, T->threshold.data(), m * 8);
  std::memcpy(impurity, T->impurity.data(), m * 8);
  std::memcpy(n_node, T->n_node.data(), m * 8);
  std::memcpy(wn, T->wn.data(), m * 8);
  std::memcpy(value, T->value.data(), T->value.size() * 8);
}

void sqh_tree_free(void* h) { delete (TreeOut*)h; }

// Leaf index of every row (row-major float32 X) for n_trees stacked trees:
// node arrays concatenated, offsets[t] = first node of tree t.  out: n x n_trees.
void sqh_forest_apply(const long long* left, const long long* right, const long long* feature,
                      const double* threshold, const long long* offsets, int n_trees,
                      const float* X, long long n, long long d, long long* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (long long i = 0; i < n; ++i) {
    const float* xi = X + i * d;
    for (int t = 0; t < n_trees; ++t) {
      long long base = offsets[t], node = 0;
      while (left[base + node] != -1) {
        node = ((double)xi[feature[base + node]] <= threshold[base + node]) ? left[base + node]
                                                                            : right[base + node];
      }
      out[i * n_trees + t] = node;
    }
  }
}

}  // extern "C"
