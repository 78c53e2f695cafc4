"""Graph utilities (reference ``utils/graph_shortest_path.pyx``
and ``utils/graph.py``).

``graph_shortest_path`` keeps the reference contract: zero weight = no edge,
unreachable pairs -> 0, ``directed=False`` walks edges both ways, method
'auto' | 'FW' | 'D' ('auto': Dijkstra when nnz < N^2 / 4).  Host kernels:
``csrc/host/graph.cpp`` (OpenMP Dijkstra over sources, Floyd-Warshall).
A dense graph given as a GPU tensor runs Floyd-Warshall on the device
(``floyd_warshall_device``: one fused min-plus rank-1 sweep per pivot over
the whole N x N matrix in HBM)."""

import numpy as np
import scipy.sparse as sp
import torch

from ..ops import _host


def floyd_warshall_device(G, directed=True):
    """All-pairs shortest paths of a dense (N, N) tensor on its device;
    zero = no edge, unreachable -> 0 (reference conventions)."""
    G = G.to(torch.float64).clone()
    N = G.shape[0]
    inf = torch.tensor(float("inf"), dtype=G.dtype, device=G.device)
    G = torch.where(G == 0, inf, G)
    G.fill_diagonal_(0.0)
    if not directed:
        G = torch.minimum(G, G.T)
    for k in range(N):
        torch.minimum(G, G[:, k:k + 1] + G[k:k + 1, :], out=G)
    G[torch.isinf(G)] = 0.0
    return G


def graph_shortest_path(dist_matrix, directed=True, method="auto"):
    """Shortest-path lengths between all pairs of a positive-weight graph."""
    if isinstance(dist_matrix, torch.Tensor) and dist_matrix.is_cuda and method in ("auto", "FW"):
        return floyd_warshall_device(dist_matrix, directed)
    if isinstance(dist_matrix, torch.Tensor):
        dist_matrix = dist_matrix.cpu().numpy()
    if not sp.isspmatrix_csr(dist_matrix):
        dist_matrix = sp.csr_matrix(dist_matrix)
    N = dist_matrix.shape[0]
    Nk = len(dist_matrix.data)
    if method == "auto":
        method = "D" if Nk < N * N / 4 else "FW"
    L = _host.lib()
    if method == "FW":
        graph = np.ascontiguousarray(dist_matrix.toarray(), dtype=np.float64)
        L.sqh_floyd_warshall(_host.ptr(graph), N, int(bool(directed)))
        return graph
    if method == "D":
        A = dist_matrix.astype(np.float64)
        A.sort_indices()
        T = A.T.tocsr()
        ip, ix, dv = (np.ascontiguousarray(A.indptr, np.int32),
                      np.ascontiguousarray(A.indices, np.int32),
                      np.ascontiguousarray(A.data, np.float64))
        tip, tix, tdv = (np.ascontiguousarray(T.indptr, np.int32),
                         np.ascontiguousarray(T.indices, np.int32),
                         np.ascontiguousarray(T.data, np.float64))
        graph = np.zeros((N, N), dtype=np.float64)
        L.sqh_dijkstra(_host.ptr(ip), _host.ptr(ix), _host.ptr(dv), _host.ptr(tip),
                       _host.ptr(tix), _host.ptr(tdv), N, int(bool(directed)), _host.ptr(graph))
        return graph
    raise ValueError("unrecognized method '%s'" % method)


def single_source_shortest_path_length(graph, source, *, cutoff=None):
    """Unweighted BFS hop counts from ``source`` (reference ``utils/graph.py``):
    dict {node: level} for nodes within ``cutoff`` levels."""
    if sp.isspmatrix(graph):
        graph = graph.tolil()
    else:
        graph = sp.lil_matrix(graph)
    seen = {}
    level = 0
    next_level = [source]
    while next_level:
        this_level = next_level
        next_level = set()
        for v in this_level:
            if v not in seen:
                seen[v] = level
                next_level.update(graph.rows[v])
        if cutoff is not None and cutoff <= level:
            break
        level += 1
    return seen
