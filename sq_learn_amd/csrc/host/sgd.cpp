// Plain stochastic gradient descent for linear models (SGDClassifier /
// SGDRegressor / SGDOneClassSVM / Perceptron / PassiveAggressive*).
//
// Behavioural parity with the reference's Cython loop
// (sklearn/linear_model/_sgd_fast.pyx:_plain_sgd, lines ~344-700):
//   * the weight vector is kept as (w, wscale, sq_norm) so the L2 shrink
//     is O(1) per sample (reference utils/_weight_vector.pyx); averaged SGD
//     keeps (aw, average_a, average_b) with the same lazy-update algebra,
//   * per-epoch Fisher-Yates shuffle of a persistent index array with the
//     tree xorshift generator, the seed passed BY VALUE each epoch
//     (reference utils/_seq_dataset.pyx.tp:151-159),
//   * learning-rate schedules constant/optimal/invscaling/adaptive/PA1/PA2,
//     MAX_DLOSS clipping, truncated-gradient L1 with the cumulative
//     penalty u and per-feature q (Tsuruoka et al. 2009),
//   * early stopping on the training loss or on a validation score that
//     is evaluated with the RAW (unscaled) weight buffer, as the
//     reference's callback does.
// Rows are dense (row-major, every feature visited) or CSR.

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr uint32_t kRandMax = 0x7FFFFFFFu;
inline uint32_t rand_r32(uint32_t* s) {
  if (*s == 0) *s = 1;
  *s ^= (uint32_t)(*s << 13);
  *s ^= (uint32_t)(*s >> 17);
  *s ^= (uint32_t)(*s << 5);
  return *s % (kRandMax + 1u);
}

enum Loss { HINGE = 0, SQ_HINGE = 1, LOG = 2, MOD_HUBER = 3, SQUARED = 4, HUBER = 5,
            EPS_INS = 6, SQ_EPS_INS = 7 };
enum Penalty { P_NONE = 0, P_L1 = 1, P_L2 = 2, P_EN = 3 };
enum LR { CONSTANT = 1, OPTIMAL = 2, INVSCALING = 3, ADAPTIVE = 4, PA1 = 5, PA2 = 6 };

struct LossFn {
  int kind;
  double c;  // threshold (hinge), delta (huber), epsilon (eps-insensitive)
  double loss(double p, double y) const {
    double z, r;
    switch (kind) {
      case HINGE: z = p * y; return z <= c ? c - z : 0.0;
      case SQ_HINGE: z = c - p * y; return z > 0 ? z * z : 0.0;
      case LOG:
        z = p * y;
        if (z > 18) return std::exp(-z);
        if (z < -18) return -z;
        return std::log(1.0 + std::exp(-z));
      case MOD_HUBER:
        z = p * y;
        if (z >= 1.0) return 0.0;
        if (z >= -1.0) return (1.0 - z) * (1.0 - z);
        return -4.0 * z;
      case SQUARED: return 0.5 * (p - y) * (p - y);
      case HUBER:
        r = p - y;
        return std::fabs(r) <= c ? 0.5 * r * r : c * std::fabs(r) - 0.5 * c * c;
      case EPS_INS: r = std::fabs(y - p) - c; return r > 0 ? r : 0.0;
      case SQ_EPS_INS: r = std::fabs(y - p) - c; return r > 0 ? r * r : 0.0;
    }
    return 0.0;
  }
  double dloss(double p, double y) const {
    double z, r;
    switch (kind) {
      case HINGE: z = p * y; return z <= c ? -y : 0.0;
      case SQ_HINGE: z = c - p * y; return z > 0 ? -2 * y * z : 0.0;
      case LOG:
        z = p * y;
        if (z > 18.0) return std::exp(-z) * -y;
        if (z < -18.0) return -y;
        return -y / (std::exp(z) + 1.0);
      case MOD_HUBER:
        z = p * y;
        if (z >= 1.0) return 0.0;
        if (z >= -1.0) return 2.0 * (1.0 - z) * -y;
        return -4.0 * y;
      case SQUARED: return p - y;
      case HUBER:
        r = p - y;
        if (std::fabs(r) <= c) return r;
        return r > 0.0 ? c : -c;
      case EPS_INS:
        if (y - p > c) return -1;
        if (p - y > c) return 1;
        return 0;
      case SQ_EPS_INS:
        z = y - p;
        if (z > c) return -2 * (z - c);
        if (z < -c) return 2 * (-z - c);
        return 0;
    }
    return 0.0;
  }
};

struct Rows {
  const double* X;
  const int* indptr;   // null => dense
  const int* indices;
  int d;
  std::vector<int> iota;
  void row(int i, const double** xd, const int** xi, int* nnz) const {
    if (!indptr) {
      *xd = X + (int64_t)i * d;
      *xi = iota.data();
      *nnz = d;
    } else {
      *xd = X + indptr[i];
      *xi = indices + indptr[i];
      *nnz = indptr[i + 1] - indptr[i];
    }
  }
};

struct WeightVec {
  double* w;
  double* aw;  // null unless averaging
  int d;
  double wscale = 1.0, average_a = 0.0, average_b = 1.0, sq_norm = 0.0;

  double dot(const double* x, const int* ind, int nnz) const {
    double s = 0.0;
    for (int j = 0; j < nnz; ++j) s += w[ind[j]] * x[j];
    return s * wscale;
  }
  void add(const double* x, const int* ind, int nnz, double c) {
    double ip = 0.0, xs = 0.0;
    for (int j = 0; j < nnz; ++j) {
      int k = ind[j];
      double v = x[j];
      ip += w[k] * v;
      xs += v * v;
      w[k] += v * (c / wscale);
    }
    sq_norm += xs * c * c + 2.0 * ip * wscale * c;
  }
  void add_average(const double* x, const int* ind, int nnz, double c, double num_iter) {
    double mu = 1.0 / num_iter;
    for (int j = 0; j < nnz; ++j) aw[ind[j]] += average_a * x[j] * (-c / wscale);
    if (num_iter > 1) average_b /= (1.0 - mu);
    average_a += mu * average_b * wscale;
  }
  void reset_wscale() {
    if (aw) {
      for (int k = 0; k < d; ++k) aw[k] += average_a * w[k];
      for (int k = 0; k < d; ++k) aw[k] *= 1.0 / average_b;
      average_a = 0.0;
      average_b = 1.0;
    }
    for (int k = 0; k < d; ++k) w[k] *= wscale;
    wscale = 1.0;
  }
  void scale(double c) {
    wscale *= c;
    sq_norm *= c * c;
    if (wscale < 1e-9) reset_wscale();
  }
};

// Validation score of the raw weight buffer (reference
// _stochastic_gradient.py:_ValidationScoreCallback): weighted accuracy on
// {-1,+1} labels (classifiers) or weighted R^2 (regressors).
double val_score(const Rows& R, const double* w, double b, const double* y, const double* sw,
                 const uint8_t* vmask, int n, int score_type) {
  const double* xd;
  const int* xi;
  int nnz;
  if (score_type == 0) {
    double num = 0.0, den = 0.0;
    for (int i = 0; i < n; ++i) {
      if (!vmask[i]) continue;
      R.row(i, &xd, &xi, &nnz);
      double p = b;
      for (int j = 0; j < nnz; ++j) p += xd[j] * w[xi[j]];
      double pred = p > 0 ? 1.0 : -1.0;
      num += sw[i] * (pred == y[i] ? 1.0 : 0.0);
      den += sw[i];
    }
    return num / den;
  }
  double swsum = 0.0, ybar = 0.0;
  for (int i = 0; i < n; ++i)
    if (vmask[i]) { swsum += sw[i]; ybar += sw[i] * y[i]; }
  ybar /= swsum;
  double ssr = 0.0, sst = 0.0;
  for (int i = 0; i < n; ++i) {
    if (!vmask[i]) continue;
    R.row(i, &xd, &xi, &nnz);
    double p = b;
    for (int j = 0; j < nnz; ++j) p += xd[j] * w[xi[j]];
    ssr += sw[i] * (y[i] - p) * (y[i] - p);
    sst += sw[i] * (y[i] - ybar) * (y[i] - ybar);
  }
  if (sst == 0.0) return ssr == 0.0 ? 1.0 : 0.0;
  return 1.0 - ssr / sst;
}

}  // namespace

// iprm: [loss, penalty, lr_type, n_iter_no_change, max_iter, fit_intercept,
//        shuffle, one_class, early_stopping, score_type]
// dprm: [loss_param, alpha, C, l1_ratio, tol, weight_pos, weight_neg, eta0,
//        power_t, t, intercept_decay, average]
// io:   [intercept, average_intercept] in/out; out2: [t_end]
// Returns epochs run (>0) or -(epochs) when a weight/intercept went non-finite.
extern "C" int sqh_sgd_plain(double* w, double* aw, double* io, const double* X,
                             const int* indptr, const int* indices, const double* y,
                             const double* sw, int n, int d, const uint8_t* vmask,
                             const int* iprm, const double* dprm, uint32_t seed, int* index) {
  LossFn loss{iprm[0], dprm[0]};
  const int penalty = iprm[1], lr = iprm[2], n_iter_no_change = iprm[3], max_iter = iprm[4];
  const int fit_intercept = iprm[5], shuffle = iprm[6], one_class = iprm[7];
  const int early_stopping = iprm[8], score_type = iprm[9];
  const double alpha = dprm[1], C = dprm[2], tol = dprm[4];
  double l1_ratio = dprm[3];
  const double weight_pos = dprm[5], weight_neg = dprm[6], eta0 = dprm[7], power_t = dprm[8];
  double t = dprm[9];
  const double intercept_decay = dprm[10], average = dprm[11];
  double intercept = io[0], average_intercept = io[1];

  Rows R{X, indptr, indices, d, {}};
  if (!indptr) {
    R.iota.resize(d);
    for (int k = 0; k < d; ++k) R.iota[k] = k;
  }
  WeightVec W{w, average > 0 ? aw : nullptr, d};
  for (int k = 0; k < d; ++k) W.sq_norm += w[k] * w[k];

  std::vector<double> q;
  if (penalty == P_L1 || penalty == P_EN) q.assign(d, 0.0);
  double u = 0.0;
  if (penalty == P_L2) l1_ratio = 0.0;
  else if (penalty == P_L1) l1_ratio = 1.0;

  double eta = eta0, optimal_init = 0.0;
  if (lr == OPTIMAL) {
    double typw = std::sqrt(1.0 / std::sqrt(alpha));
    double initial_eta0 = typw / std::max(1.0, loss.dloss(-typw, 1.0));
    optimal_init = 1.0 / (initial_eta0 * alpha);
  }
  const bool is_hinge = loss.kind == HINGE;
  const double MAX_DLOSS = 1e12;
  double best_loss = INFINITY, best_score = -INFINITY;
  int no_improvement = 0, epoch = 0;
  bool infinity = false;
  const double* xd;
  const int* xi;
  int nnz;

  for (epoch = 0; epoch < max_iter; ++epoch) {
    double sumloss = 0.0;
    if (shuffle) {
      uint32_t s = seed;
      for (unsigned i = 0; i + 1 < (unsigned)n; ++i) {
        unsigned j = i + rand_r32(&s) % ((unsigned)n - i);
        std::swap(index[i], index[j]);
      }
    }
    for (int ii = 0; ii < n; ++ii) {
      const int si = index[ii];
      if (vmask[si]) continue;
      R.row(si, &xd, &xi, &nnz);
      const double yi = y[si], swi = sw[si];
      double p = W.dot(xd, xi, nnz) + intercept;
      if (lr == OPTIMAL) eta = 1.0 / (alpha * (optimal_init + t - 1));
      else if (lr == INVSCALING) eta = eta0 / std::pow(t, power_t);
      if (!early_stopping) sumloss += loss.loss(p, yi);
      double class_weight = yi > 0.0 ? weight_pos : weight_neg;
      double update;
      if (lr == PA1) {
        double nx = 0.0;
        for (int j = 0; j < nnz; ++j) nx += xd[j] * xd[j];
        if (nx == 0) continue;
        update = std::min(C, loss.loss(p, yi) / nx);
      } else if (lr == PA2) {
        double nx = 0.0;
        for (int j = 0; j < nnz; ++j) nx += xd[j] * xd[j];
        update = loss.loss(p, yi) / (nx + 0.5 / C);
      } else {
        double dl = loss.dloss(p, yi);
        if (dl < -MAX_DLOSS) dl = -MAX_DLOSS;
        else if (dl > MAX_DLOSS) dl = MAX_DLOSS;
        update = -eta * dl;
      }
      if (lr >= PA1) {
        if (is_hinge) update *= yi;
        else if (yi - p < 0) update *= -1;
      }
      update *= class_weight * swi;
      if (penalty >= P_L2) W.scale(std::max(0.0, 1.0 - ((1.0 - l1_ratio) * eta * alpha)));
      if (update != 0.0) W.add(xd, xi, nnz, update);
      if (fit_intercept == 1) {
        double iu = update;
        if (one_class) iu -= 2. * eta * alpha;
        if (iu != 0) intercept += iu * intercept_decay;
      }
      if (0 < average && average <= t) {
        W.add_average(xd, xi, nnz, update, t - average + 1);
        average_intercept += (intercept - average_intercept) / (t - average + 1);
      }
      if (penalty == P_L1 || penalty == P_EN) {
        u += l1_ratio * eta * alpha;
        const double wscale = W.wscale;
        for (int j = 0; j < nnz; ++j) {
          int k = xi[j];
          double z = w[k];
          if (wscale * z > 0.0) w[k] = std::max(0.0, w[k] - ((u + q[k]) / wscale));
          else if (wscale * z < 0.0) w[k] = std::min(0.0, w[k] + ((u - q[k]) / wscale));
          q[k] += wscale * (w[k] - z);
        }
      }
      t += 1;
    }
    bool nonfinite = !std::isfinite(intercept);
    for (int k = 0; k < d && !nonfinite; ++k) nonfinite = !std::isfinite(w[k]);
    if (nonfinite) {
      infinity = true;
      break;
    }
    if (early_stopping) {
      double score = val_score(R, w, intercept, y, sw, vmask, n, score_type);
      if (tol > -INFINITY && score < best_score + tol) ++no_improvement;
      else no_improvement = 0;
      if (score > best_score) best_score = score;
    } else {
      if (tol > -INFINITY && sumloss > best_loss - tol * n) ++no_improvement;
      else no_improvement = 0;
      if (sumloss < best_loss) best_loss = sumloss;
    }
    if (no_improvement >= n_iter_no_change) {
      if (lr == ADAPTIVE && eta > 1e-6) {
        eta = eta / 5;
        no_improvement = 0;
      } else {
        break;
      }
    }
  }
  if (infinity) return -(epoch + 1);
  W.reset_wscale();
  io[0] = intercept;
  io[1] = average_intercept;
  io[2] = t;
  return (epoch < max_iter ? epoch : max_iter - 1) + 1;
}
