// All-pairs shortest paths on positive-weight graphs (SURVEY.md N25,
// reference ``utils/graph_shortest_path.pyx``: Floyd-Warshall and Dijkstra).
// Conventions follow the reference: a zero weight means "no edge", the
// undirected case uses min(w_ij, w_ji) (FW) / both edge directions
// (Dijkstra), and unreachable pairs come back as 0.
//
// Host design: Dijkstra runs one binary-heap search per source with OpenMP
// over sources (the reference is single-threaded with Fibonacci heaps);
// Floyd-Warshall parallelises the row loop of each pivot.  A GPU
// Floyd-Warshall for large dense graphs lives in ``utils/graph.py`` (torch
// min-plus sweeps on the device).
#include <cmath>
#include <cstdint>
#include <limits>
#include <queue>
#include <utility>
#include <vector>

#include "host.h"

extern "C" {

// graph: N x N row-major, zero = no edge; overwritten with path lengths
void sqh_floyd_warshall(double* g, long long N, int directed) {
  const double inf = std::numeric_limits<double>::infinity();
  for (long long t = 0; t < N * N; ++t)
    if (g[t] == 0.0) g[t] = inf;
  for (long long i = 0; i < N; ++i) g[i * N + i] = 0.0;
  if (!directed) {
    for (long long i = 0; i < N; ++i)
      for (long long j = i + 1; j < N; ++j) {
        const double m = g[j * N + i] <= g[i * N + j] ? g[j * N + i] : g[i * N + j];
        g[i * N + j] = m;
        g[j * N + i] = m;
      }
  }
  for (long long k = 0; k < N; ++k) {
    const double* gk = g + k * N;
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < N; ++i) {
      double* gi = g + i * N;
      const double dik = gi[k];
      if (dik == inf) continue;
      for (long long j = 0; j < N; ++j) {
        const double s = dik + gk[j];
        if (s < gi[j]) gi[j] = s;
      }
    }
  }
  for (long long t = 0; t < N * N; ++t)
    if (std::isinf(g[t])) g[t] = 0.0;
}

// CSR graph (explicit zeros are not edges); out: N x N distances
void sqh_dijkstra(const int32_t* indptr, const int32_t* indices, const double* data,
                  const int32_t* tindptr, const int32_t* tindices, const double* tdata,
                  long long N, int directed, double* out) {
  const double inf = std::numeric_limits<double>::infinity();
#pragma omp parallel
  {
    std::vector<double> dist(N);
    std::vector<char> done(N);
    using Item = std::pair<double, int32_t>;
#pragma omp for schedule(dynamic, 4)
    for (long long s = 0; s < N; ++s) {
      std::fill(dist.begin(), dist.end(), inf);
      std::fill(done.begin(), done.end(), 0);
      std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
      dist[s] = 0.0;
      pq.push({0.0, (int32_t)s});
      while (!pq.empty()) {
        const auto [du, u] = pq.top();
        pq.pop();
        if (done[u]) continue;
        done[u] = 1;
        auto relax = [&](const int32_t* ip, const int32_t* ix, const double* dv) {
          for (int32_t e = ip[u]; e < ip[u + 1]; ++e) {
            const double w = dv[e];
            if (w == 0.0) continue;
            const int32_t v = ix[e];
            const double nd = du + w;
            if (nd < dist[v]) {
              dist[v] = nd;
              pq.push({nd, v});
            }
          }
        };
        relax(indptr, indices, data);
        if (!directed) relax(tindptr, tindices, tdata);
      }
      double* row = out + s * N;
      for (long long v = 0; v < N; ++v) row[v] = std::isinf(dist[v]) ? 0.0 : dist[v];
    }
  }
}

}  // extern "C"
