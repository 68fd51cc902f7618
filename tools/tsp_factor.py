"""Experiment: L1 X through the Hodge factorisation L1 = alpha * B1^T B1
(lib/Hodge_Dataset.py:451-456: every L1 entry is fl(2 v / lmax) with v the
integer entry of B1^T B1, so L1 = alpha_e * (B1^T B1) exactly, alpha_e =
L1[e,e] / 2) versus the plain CSR SpMM, at BASELINE config 5.

    Z = B1 X          (node rows: signed sum of the incident edges' rows)
    Y = alpha B1^T Z  (edge rows: alpha_e (Z[j] - Z[i]))

~2 gathered rows per edge and ~2 per node instead of ~20 per edge.
Algorithmic bytes are those of the SpMM problem (8 nnz + 4 (n+1) + 8 n d,
SURVEY §8d) so the columns compare directly with tools/tsp_spmm.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from tsp_spmm import PEAK_GBPS, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=4)
    ap.add_argument("--d", type=int, nargs="+", default=[64, 128])
    args = ap.parse_args()
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph
    dev = torch.device("cuda:0")
    b = collate([tsp_like_graph(s, halo=False) for s in range(args.graphs)], check_hodge=False)
    eis, ws = b.edge_index_s.numpy(), b.edge_weight_s.numpy()
    ei = b.edge_index.numpy()
    n, nnz, N = b.x_s.shape[0], eis.shape[1], b.x_t.shape[0]
    E = ei.shape[1]
    assert E == n
    diag = eis[0] == eis[1]
    alpha = np.zeros(n, np.float32)
    alpha[eis[0][diag]] = ws[diag] / 2
    # exactness of the factorisation: rebuild every entry
    rows = np.concatenate([ei[0], ei[1]])
    sgn = np.concatenate([-np.ones(E), np.ones(E)]).astype(np.float32)
    import scipy.sparse as sp
    B = sp.csr_matrix((sgn, (rows, np.concatenate([np.arange(E)] * 2))), shape=(N, E))
    BtB = (B.T @ B).tocoo()
    Lr = sp.csr_matrix((BtB.data.astype(np.float32) * alpha[BtB.row], (BtB.row, BtB.col)),
                       shape=(n, n)).tocoo()
    L = sp.csr_matrix((ws, (eis[0], eis[1])), shape=(n, n))
    exact = bool((abs(L - Lr.tocsr()) > 0).nnz == 0)
    print(json.dumps({"factorisation_exact": exact, "n_edges": E, "n_nodes": N, "nnz_L1": nnz}))

    e = ops.set_row_order(ops.mark_hodge(b.edge_index_s.to(dev)), b.row_order_s)
    ops.set_hodge_factor(e, b.edge_index.to(dev), N, b.row_order_t)
    op = ops.hodge_operator(e, b.edge_weight_s.to(dev), n)
    nr, ne, ns, no, _, _, _ = op.factor
    node = ops.SparseCSR(nr, ne, ns, N, E, 2 * E, order=no)
    for d in args.d:
        X = torch.randn(n, d, device=dev)
        Zn = torch.empty(N, d, device=dev)
        Yr = ops.spmm(op.fwd, X)
        err = float((ops.hodge_spmm(op, X) - Yr).abs().max() / Yr.abs().max())
        by = 8 * nnz + 4 * (n + 1) + 8 * n * d
        t_all = timeit(lambda: ops.hodge_spmm(op, X))
        t_node = timeit(lambda: ops._poly_step(node, X, Zn))
        r = {"op": "factored spmm", "d": d, "us": round(t_all, 1), "stage1_node_us": round(t_node, 1),
             "stage2_edge_us": round(t_all - t_node, 1), "rel_err_vs_csr": err,
             "GBps_equiv": round(by / t_all / 1e3, 1),
             "hbm_frac_equiv": round(by / t_all / 1e3 / PEAK_GBPS, 4),
             "stage1_GBps": round((4 * n * d + 4 * N * d + 8 * 2 * E) / t_node / 1e3, 1),
             "stage2_GBps": round((4 * N * d + 4 * n * d + 12 * n) / (t_all - t_node) / 1e3, 1)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
