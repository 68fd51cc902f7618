"""hlhgat_eig_pe (ops.eig_pe): the eigenvector PE and lambda_max of every
graph of a batch in one launch -- the reference's per-sample eig_pe(L0)
(lib/Hodge_Dataset.py:97-112: eigenvectors 1 .. k-1 of a dense eigh) and
torch.linalg.eigh(L0).max() (lib/Hodge_Dataset.py:782) -- against numpy's
fp64 eigh of the same dense L0 = B1 B1^T:

* lambda_max within 1e-12 relative;
* every PE column whose eigenvalue is separated from its neighbours by more
  than 1e-3 equals the reference eigenvector up to sign within 2e-6 (the
  output is float32 of an fp64 computation);
* every column (clusters included: disconnected graphs, isolated nodes, equal
  eigenvalues) is an eigenvector of its eigenvalue (residual <= 1e-5) and the
  columns of a graph are orthonormal within 1e-5;
* a graph with fewer than k nodes has zero columns past its own size;
* graphs too large for the LDS (the workspace path) agree as well.
"""
import numpy as np
import pytest
import torch

K = 10


def _dense_l0(ei, n):
    L = np.zeros((n, n))
    np.add.at(L, (ei[0], ei[1]), -1.0)
    np.add.at(L, (ei[1], ei[0]), -1.0)
    L[np.diag_indices(n)] = -L.sum(1)
    return L


def _graphs(seed):
    """Superpixel kNN graphs with dropout (isolated nodes appear), sizes on
    both sides of the LDS limit, a disconnected graph, a path, a star, tiny
    graphs."""
    from hlhgat.pipeline import superpixel_raw, to_undirected_min
    rng = np.random.default_rng(seed)
    out = []
    for i, n in enumerate([118, 40, 150, 97, 200, 64, 123, 130]):
        r = superpixel_raw(300 + i + 17 * seed, n=n)
        ei, _ = to_undirected_min(r.edge_index, r.edge_attr, n)
        ei = ei[:, ei[0] < ei[1]]
        if i % 2 == 0:
            ei = ei[:, rng.random(ei.shape[1]) >= 0.5]
        out.append((ei, n))
    # two disjoint 5-cycles + 3 isolated nodes; a path; a star; n < k; one node
    cyc = [(j, (j + 1) % 5) for j in range(5)]
    e = [(min(a, b), max(a, b)) for a, b in cyc] + [(min(a, b) + 5, max(a, b) + 5) for a, b in cyc]
    out.append((np.array(e, np.int64).T, 13))
    out.append((np.array([[j, j + 1] for j in range(29)], np.int64).T, 30))
    out.append((np.array([[0, j] for j in range(1, 25)], np.int64).T, 25))
    out.append((np.array([[0, 1], [1, 2], [2, 3], [0, 3], [1, 4]], np.int64).T, 6))
    out.append((np.zeros((2, 0), np.int64), 1))
    return out


def _batch(graphs, dev):
    offs = np.concatenate([[0], np.cumsum([n for _, n in graphs])])
    ei = np.concatenate([e + o for (e, _), o in zip(graphs, offs[:-1])], axis=1)
    return torch.from_numpy(np.ascontiguousarray(ei)).to(dev), [n for _, n in graphs], offs


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_eig_pe_matches_fp64_eigh(cuda, seed):
    from hlhgat import ops
    graphs = _graphs(seed)
    ei, ns, offs = _batch(graphs, cuda)
    pe, lmax = ops.eig_pe(ei, ns, K)
    torch.cuda.synchronize()
    pe, lmax = pe.cpu().numpy().astype(np.float64), lmax.cpu().numpy()
    assert pe.shape == (offs[-1], K - 1)
    for g, (e, n) in enumerate(graphs):
        L = _dense_l0(e, n)
        w, V = np.linalg.eigh(L)
        assert abs(lmax[g] - w[-1]) <= 1e-12 * max(w[-1], 1.0), (g, lmax[g], w[-1])
        P = pe[offs[g]:offs[g + 1]]
        m = min(K, n)
        assert np.all(P[:, m - 1:] == 0.0), g  # columns past the graph's size
        if m <= 1:
            continue
        P = P[:, :m - 1]
        lam = w[1:m]
        # eigenvectors of their eigenvalues, orthonormal
        res = np.abs(L @ P - P * lam[None, :]).max()
        assert res <= 1e-5 * max(1.0, w[-1]), (g, res)
        orth = np.abs(P.T @ P - np.eye(m - 1)).max()
        assert orth <= 1e-5, (g, orth)
        # separated eigenvalues: the reference vector up to sign
        for c in range(m - 1):
            j = c + 1
            gap = min(w[j] - w[j - 1], (w[j + 1] - w[j]) if j + 1 < n else np.inf)
            if gap > 1e-3:
                s = np.sign(P[:, c] @ V[:, j]) or 1.0
                err = np.abs(P[:, c] * s - V[:, j]).max()
                assert err <= 2e-6, (g, c, gap, err)


@pytest.mark.gpu
def test_eig_pe_device_counts_and_repeatability(cuda):
    """Device node counts (max_nodes given) give the same bits as host
    counts, and a second launch the same bits as the first."""
    from hlhgat import ops
    graphs = _graphs(2)
    ei, ns, _ = _batch(graphs, cuda)
    a, la = ops.eig_pe(ei, ns, K)
    b, lb = ops.eig_pe(ei, torch.tensor(ns, device=cuda), K, max_nodes=max(ns))
    c, lc = ops.eig_pe(ei, ns, K)
    assert torch.equal(a, b) and torch.equal(la, lb)
    assert torch.equal(a, c) and torch.equal(la, lc)
