// Stochastic Average Gradient (SAG, Schmidt et al. 2013) and SAGA (Defazio
// et al. 2014) for the ridge / logistic / multinomial losses - SURVEY.md
// N20-N22, reference ``linear_model/_sag.py:89`` (``sag_solver``) and its
// Cython core ``_sag_fast.pyx.tp``.
//
// Rows are dense, so every step touches every weight: the weights are
// updated eagerly (scaled by 1 - step alpha, corrected by the SAGA term, then
// moved by the averaged gradient and, for SAGA with an L1 part, soft-
// thresholded) instead of through the reference's just-in-time cumulative
// sums - the same iterates in exact arithmetic.  Samples are drawn with
// replacement by the reference's generator (xorshift ``our_rand_r`` seeded
// like ``make_dataset``), the step size and the stopping rule (max weight
// change / max weight <= tol after each epoch) are the reference's.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "host.h"

namespace {

inline uint32_t xorshift_rand(uint32_t& s) {
  if (s == 0) s = 1;
  s ^= (uint32_t)(s << 13);
  s ^= (uint32_t)(s >> 17);
  s ^= (uint32_t)(s << 5);
  return s % 0x80000000u;
}

// d loss / d prediction of the binary log loss, labels in {-1, +1}
inline double dlog(double p, double y) {
  const double z = p * y;
  if (z > 18.0) return std::exp(-z) * -y;
  if (z < -18.0) return -y;
  return -y / (std::exp(z) + 1.0);
}

inline double soft(double w, double t) {
  return w > t ? w - t : (w < -t ? w + t : 0.0);
}

}  // namespace

extern "C" {

// loss: 0 = log (binary, y in {-1, 1}, K = 1), 1 = squared (K = 1),
// 2 = multinomial (y = class id, K classes).  W [d][K] and b [K] hold the
// initial weights on entry and the solution on exit.  Returns the number of
// epochs run, or -1 - epoch on a floating-point overflow.
int sqh_sag(const double* X, const double* y, const double* sw, long long n, long long d, int K,
            int loss, double alpha, double beta, double step, int max_iter, double tol,
            int fit_intercept, double intercept_decay, int saga, uint32_t seed, double* W,
            double* b) {
  const int64_t dK = d * (int64_t)K;
  std::vector<double> gmem((size_t)n * K, 0.0), sg(dK, 0.0), isg(K, 0.0), prev(W, W + dK);
  std::vector<double> pred(K), g(K);
  std::vector<uint8_t> seen(n, 0);
  const bool prox = saga && beta > 0;
  const double decay = 1.0 - step * alpha;
  int64_t num_seen = 0;
  uint32_t s = seed;
  int epoch = 0;
  for (; epoch < max_iter; ++epoch) {
    for (int64_t it = 0; it < n; ++it) {
      const int64_t i = xorshift_rand(s) % (uint32_t)n;
      const double* xi = X + i * d;
      if (!seen[i]) {
        seen[i] = 1;
        ++num_seen;
      }
      const double ns = (double)num_seen;
      for (int c = 0; c < K; ++c) pred[c] = 0.0;
      for (int64_t f = 0; f < d; ++f) {
        const double v = xi[f];
        const double* wf = W + f * K;
        for (int c = 0; c < K; ++c) pred[c] += v * wf[c];
      }
      for (int c = 0; c < K; ++c) pred[c] += b[c];
      if (loss == 0) {
        g[0] = dlog(pred[0], y[i]) * sw[i];
      } else if (loss == 1) {
        g[0] = (pred[0] - y[i]) * sw[i];
      } else {
        double mx = pred[0];
        for (int c = 1; c < K; ++c) mx = std::max(mx, pred[c]);
        double se = 0.0;
        for (int c = 0; c < K; ++c) se += std::exp(pred[c] - mx);
        const double lse = mx + std::log(se);
        const int yc = (int)y[i];
        for (int c = 0; c < K; ++c)
          g[c] = sw[i] * (std::exp(pred[c] - lse) - (c == yc ? 1.0 : 0.0));
      }
      // L2 shrink, SAGA correction, gradient-table update
      double* gm = &gmem[(size_t)i * K];
      const double corr_step = step * (1.0 - 1.0 / ns);
      for (int64_t f = 0; f < d; ++f) {
        const double v = xi[f];
        double* wf = W + f * K;
        double* sf = &sg[f * K];
        for (int c = 0; c < K; ++c) {
          const double corr = v * (g[c] - gm[c]);
          wf[c] *= decay;
          if (saga) wf[c] -= corr * corr_step;
          sf[c] += corr;
        }
      }
      if (fit_intercept) {
        for (int c = 0; c < K; ++c) {
          const double gc = g[c] - gm[c];
          isg[c] += gc;
          const double avg = step * isg[c] / ns * intercept_decay;
          b[c] -= saga ? avg + gc * corr_step : avg;
          if (!std::isfinite(b[c])) return -1 - epoch;
        }
      }
      for (int c = 0; c < K; ++c) gm[c] = g[c];
      // the averaged-gradient step (+ the L1 proximal step)
      const double gstep = step / ns;
      for (int64_t k = 0; k < dK; ++k) {
        double w = W[k] - gstep * sg[k];
        if (prox) w = soft(w, step * beta);
        W[k] = w;
      }
    }
    double max_w = 0.0, max_dw = 0.0;
    for (int64_t k = 0; k < dK; ++k) {
      if (!std::isfinite(W[k])) return -1 - epoch;
      max_w = std::max(max_w, std::fabs(W[k]));
      max_dw = std::max(max_dw, std::fabs(W[k] - prev[k]));
      prev[k] = W[k];
    }
    if ((max_w != 0 && max_dw / max_w <= tol) || (max_w == 0 && max_dw == 0)) {
      ++epoch;
      break;
    }
  }
  return epoch;
}

}  // extern "C"
