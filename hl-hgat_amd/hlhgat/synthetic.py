"""Synthetic simplex graphs of the BASELINE.json shapes (no datasets offline).

ZINC-like molecules: n ~ clip(round(N(23.2, 4.5)), 9, 38) atoms,
a random tree with max degree 4 plus ring closures (E ≈ n + 1.7 on average),
atom / bond one-hots (21 / 3 classes) concatenated with keig Laplacian
eigenvector PEs, Hodge Laplacians exactly as the reference ZINC process()
builds them (lib/Hodge_Dataset.py:447-477) and the get()-time PE padding /
sign flips (:425-440).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from .hodge_dataset import (PairData, collate, dense_to_sparse, halo_tiles, hodge_laplacians,
                            locality_order, mlgc)

__all__ = ["zinc_like_graph", "zinc_like_batch", "molecule_edges", "tsp_like_graph",
           "cifar_like_graphs", "peptides_like_graphs", "two_level_batch", "knn_edges"]


def molecule_edges(rng: np.random.Generator, n: int, extra_mean: float = 2.7) -> np.ndarray:
    """Undirected edge list (i<j, sorted) of a random tree with max degree 4
    plus ring closures between atoms 4-5 bonds apart."""
    deg = np.zeros(n, dtype=np.int64)
    edges = set()
    adj = [[] for _ in range(n)]
    for v in range(1, n):
        cand = [u for u in range(v) if deg[u] < 4]
        u = int(rng.choice(cand))
        edges.add((u, v))
        adj[u].append(v)
        adj[v].append(u)
        deg[u] += 1
        deg[v] += 1
    n_extra = int(rng.poisson(extra_mean))
    tries = 0
    while n_extra > 0 and tries < 50:
        tries += 1
        a = int(rng.integers(n))
        if deg[a] >= 4:
            continue
        # BFS distances from a
        dist = -np.ones(n, dtype=np.int64)
        dist[a] = 0
        frontier = [a]
        while frontier:
            nxt = []
            for x in frontier:
                for y in adj[x]:
                    if dist[y] < 0:
                        dist[y] = dist[x] + 1
                        nxt.append(y)
            frontier = nxt
        cand = [b for b in range(n) if dist[b] in (4, 5) and deg[b] < 4]
        if not cand:
            continue
        b = int(rng.choice(cand))
        e = (min(a, b), max(a, b))
        if e in edges:
            continue
        edges.add(e)
        adj[a].append(b)
        adj[b].append(a)
        deg[a] += 1
        deg[b] += 1
        n_extra -= 1
    return np.array(sorted(edges), dtype=np.int64).T.reshape(2, -1)


def _eig_pe(L: torch.Tensor, k: int) -> torch.Tensor:
    """eig_pe (lib/Hodge_Dataset.py:97-112): eigenvectors 1..k-1 by ascending
    eigenvalue."""
    vals, vecs = np.linalg.eigh(L.numpy().astype(np.float64))
    vecs = vecs[:, vals.argsort()]
    return torch.from_numpy(vecs[:, 1:k].astype(np.float32))


def _pad_sign(x: torch.Tensor, width: int, n_fixed: int, rng: np.random.Generator):
    if x.shape[1] < width:
        return torch.cat([x, torch.zeros(x.shape[0], width - x.shape[1])], dim=-1)
    sign = torch.cat([torch.ones(n_fixed),
                      torch.from_numpy(rng.integers(0, 2, width - n_fixed) * 2.0 - 1.0).float()])
    return x[:, :width] * sign


def zinc_like_graph(seed: int, keig: int = 15) -> PairData:
    rng = np.random.default_rng(seed)
    n = int(np.clip(round(rng.normal(23.2, 4.5)), 9, 38))
    ei = molecule_edges(rng, n)
    E = ei.shape[1]
    L0, L1, maxeig, _ = hodge_laplacians(ei, n)
    atom = torch.from_numpy(rng.integers(0, 21, n))
    bond = torch.from_numpy(rng.integers(0, 3, E))
    x_t = torch.cat([torch.nn.functional.one_hot(atom, 21).float(), _eig_pe(L0, keig + 1)], -1)
    x_s = torch.cat([torch.nn.functional.one_hot(bond, 3).float(), _eig_pe(L1, keig + 1)], -1)
    x_t = _pad_sign(x_t, 21 + keig, 21, rng)
    x_s = _pad_sign(x_s, 3 + keig, 3, rng)
    eit, ewt = dense_to_sparse(L0)
    eis, ews = dense_to_sparse(L1)
    g = PairData(x_s=x_s, edge_index_s=eis, edge_weight_s=ews, x_t=x_t, edge_index_t=eit,
                 edge_weight_t=ewt, y=torch.tensor([float(rng.normal())]))
    g.edge_index = torch.from_numpy(ei)
    g.num_node1 = n
    g.num_edge1 = E
    g.num_nodes = n
    g._hodge_sorted = True  # dense_to_sparse of symmetric L: row-major, symmetric
    return g


def tsp_like_graph(seed: int, n: int = 10000, k: int = 9, row_order: bool = True,
                   halo: bool = True) -> PairData:
    """TSP-like simplex graph (BASELINE config 5): n uniform points in [0,1]^2,
    symmetric k-NN edges (i<j), L0 = 2 B1 B1^T / lmax and L1 = 2 B1^T B1 / lmax
    built SPARSE (a dense E x E L1 would be ~10 GB at n = 10k), lmax of L0 by
    Lanczos; COO row-major sorted like dense_to_sparse.  Features: node
    coordinates (2), edge length + mask (2) as in main_TSP (:99-176)."""
    import scipy.sparse as sp
    from scipy.sparse.linalg import eigsh
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    pts = rng.random((n, 2))
    _, nbr = cKDTree(pts).query(pts, k=k + 1)
    a = np.repeat(np.arange(n), k)
    b = nbr[:, 1:].reshape(-1)
    i, j = np.minimum(a, b), np.maximum(a, b)
    key = np.unique(i.astype(np.int64) * n + j)
    ei = np.stack([key // n, key % n])
    E = ei.shape[1]
    B = sp.csr_matrix((np.concatenate([-np.ones(E), np.ones(E)]).astype(np.float32),
                       (np.concatenate([ei[0], ei[1]]), np.concatenate([np.arange(E)] * 2))),
                      shape=(n, E))
    L0 = (B @ B.T).tocsr()
    lmax = float(eigsh(L0.astype(np.float64), k=1, which="LA", return_eigenvectors=False)[0])
    L0 = (2.0 * L0 / lmax).astype(np.float32).tocoo()
    L1 = (2.0 * (B.T @ B) / lmax).astype(np.float32).tocoo()

    def coo(M):
        M.sum_duplicates()
        o = np.lexsort((M.col, M.row))
        keep = M.data[o] != 0
        r, c, v = M.row[o][keep], M.col[o][keep], M.data[o][keep]
        return torch.from_numpy(np.stack([r, c]).astype(np.int64)), torch.from_numpy(v)

    eit, ewt = coo(L0)
    eis, ews = coo(L1)
    length = np.linalg.norm(pts[ei[0]] - pts[ei[1]], axis=1).astype(np.float32)
    x_s = torch.from_numpy(np.stack([length, np.ones(E, np.float32)], 1))
    g = PairData(x_s=x_s, edge_index_s=eis, edge_weight_s=ews,
                 x_t=torch.from_numpy(pts.astype(np.float32)), edge_index_t=eit,
                 edge_weight_t=ewt, y=torch.zeros(E))
    if row_order:  # L2-locality schedules of the two Laplacians (SpMM row order)
        g.row_order_s = locality_order(eis.numpy(), E)
        g.row_order_t = locality_order(eit.numpy(), n)
        if halo:  # LDS halo tiles along those schedules (k_poly_halo)
            for side, eix, rows, o in (("s", eis, E, g.row_order_s), ("t", eit, n, g.row_order_t)):
                ht = halo_tiles(eix.numpy(), rows, o.numpy())
                for key, val in (ht or {}).items():
                    setattr(g, key + "_" + side, val)
    g.edge_index = torch.from_numpy(ei)
    g.num_node1 = n
    g.num_edge1 = E
    g.num_nodes = n
    g._hodge_sorted = True
    return g


def zinc_like_batch(n_graphs: int, seed: int = 0, keig: int = 15,
                    check_hodge: bool = False):
    graphs: List[PairData] = [zinc_like_graph(seed * 1_000_003 + i, keig) for i in range(n_graphs)]
    return collate(graphs, check_hodge=check_hodge)


# ----------------------------------------------------------------------------
# two-level (MLGC) batches for the attention-pooling heads (configs 3 and 4)
# ----------------------------------------------------------------------------
def _two_level(ei: np.ndarray, n: int, x_t: torch.Tensor, x_s: torch.Tensor, y, seed: int):
    """Level-0 PairData with the MLGC cluster of each node / edge in feature
    column 0 (as CIFAR10SP_EigPE_MLGC.get / the pepfunc dataset prepend it,
    main_cifar10SP...:101-105) and the coarse level-1 PairData."""
    L0, L1, _, _ = hodge_laplacians(ei, n)
    eit, ewt = dense_to_sparse(L0)
    eis, ews = dense_to_sparse(L1)
    g = PairData(x_s=x_s, edge_index_s=eis, edge_weight_s=ews, x_t=x_t, edge_index_t=eit,
                 edge_weight_t=ewt, y=y)
    g.edge_index = torch.from_numpy(ei)
    g.num_node1 = n
    g.num_edge1 = int(ei.shape[1])
    g.num_nodes = n
    g._hodge_sorted = True
    coarse, c_node, c_edge = mlgc(g, seed=seed)
    g.x_t = torch.cat([c_node, g.x_t], dim=-1)
    g.x_s = torch.cat([c_edge, g.x_s], dim=-1)
    return g, coarse


def knn_edges(pts: np.ndarray, k: int) -> np.ndarray:
    """Symmetric k-NN edge list (i<j, sorted, unique)."""
    from scipy.spatial import cKDTree
    n = pts.shape[0]
    _, nbr = cKDTree(pts).query(pts, k=min(k + 1, n))
    a = np.repeat(np.arange(n), nbr.shape[1] - 1)
    b = nbr[:, 1:].reshape(-1)
    i, j = np.minimum(a, b), np.maximum(a, b)
    key = np.unique(i.astype(np.int64) * n + j)
    return np.stack([key // n, key % n])


def cifar_like_graphs(seed: int, n: int = 118, k: int = 8, keig: int = 10):
    """CIFAR10 superpixel-like graph (BASELINE config 3): n
    superpixels at uniform positions, symmetric 8-NN edges (~565 at n=118),
    node features node_dim 5 + keig, edge features edge_dim 4 + keig
    (lib/Hodge_ST_Model.py:958-961), one MLGC level.  Returns (level0, level1)."""
    rng = np.random.default_rng(seed)
    ei = knn_edges(rng.random((n, 2)), k)
    x_t = torch.from_numpy(rng.standard_normal((n, 5 + keig)).astype(np.float32))
    x_s = torch.from_numpy(rng.standard_normal((ei.shape[1], 4 + keig)).astype(np.float32))
    return _two_level(ei, n, x_t, x_s, torch.tensor([int(rng.integers(10))]), seed)


def peptides_like_graphs(seed: int, keig: int = 20):
    """Peptides-func-like molecule (BASELINE config 4, SURVEY §8d: ~151 atoms,
    ~154 bonds): node features 9 + keig, edge features 3 + keig
    (main_pepfunc...:37-39), 10 binary labels, one MLGC level."""
    rng = np.random.default_rng(seed)
    n = int(np.clip(round(rng.normal(150.9, 20.0)), 40, 300))
    ei = molecule_edges(rng, n)
    x_t = torch.from_numpy(rng.standard_normal((n, 9 + keig)).astype(np.float32))
    x_s = torch.from_numpy(rng.standard_normal((ei.shape[1], 3 + keig)).astype(np.float32))
    y = torch.from_numpy(rng.integers(0, 2, (1, 10)).astype(np.float32))
    return _two_level(ei, n, x_t, x_s, y, seed)


def two_level_batch(kind: str, n_graphs: int, seed: int = 0, **kw):
    """datas = [level-0 batch, level-1 batch] as the attpool heads take them."""
    make = {"cifar": cifar_like_graphs, "peptides": peptides_like_graphs}[kind]
    pairs = [make(seed * 1_000_003 + i, **kw) for i in range(n_graphs)]
    return [collate([p[0] for p in pairs], check_hodge=False),
            collate([p[1] for p in pairs], check_hodge=False)]
