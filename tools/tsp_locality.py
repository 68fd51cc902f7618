"""Does gather locality decide the TSP-scale (BASELINE config 5) SpMM rate?

    python tools/tsp_locality.py [--graphs 4] [--d 128 64]

Times Y = L1 X on the batched TSP-like L1 (n ~ 207k edges, nnz ~ 4.1M) as
generated (edges sorted by their first node) and after renumbering the edges
in reverse Cuthill-McKee order (the same operator, permuted), plus a
midpoint space-filling-curve order.  Same kernel, same bytes; only which rows
are gathered together changes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=4)
    ap.add_argument("--d", type=int, nargs="+", default=[128, 64])
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph
    dev = torch.device("cuda:0")
    b = collate([tsp_like_graph(s) for s in range(args.graphs)], check_hodge=False)
    ei, w = b.edge_index_s.numpy(), b.edge_weight_s.numpy()
    n = b.x_s.shape[0]
    A = sp.csr_matrix((w, (ei[1], ei[0])), shape=(n, n))
    A.sort_indices()
    orders = {"as generated": np.arange(n)}
    orders["rcm"] = reverse_cuthill_mckee(A, symmetric_mode=True)
    # edge midpoint order along the node numbering of the incidence (proxy
    # without coordinates): sort edges by (min node, max node) of B1 = same as
    # generated; by (max node) instead
    eb = b.edge_index.numpy()
    orders["by max node"] = np.lexsort((eb[0], eb[1]))
    res = []
    # schedule-only variant: original numbering (bit-identical results), rows
    # visited in RCM order
    csr0 = ops.SparseCSR(torch.from_numpy(A.indptr.astype(np.int32)).to(dev),
                         torch.from_numpy(A.indices.astype(np.int32)).to(dev),
                         torch.from_numpy(A.data.astype(np.float32)).to(dev), n, n, A.nnz,
                         torch.from_numpy(orders["rcm"].astype(np.int32)).to(dev))
    for d in args.d:
        X = torch.randn(n, d, device=dev)
        Y = torch.empty(n, d, device=dev)
        Yref = torch.empty(n, d, device=dev)
        csr_nat = ops.SparseCSR(csr0.rowptr, csr0.col, csr0.val, n, n, A.nnz)
        ops._poly_step(csr_nat, X, Yref)
        ops._poly_step(csr0, X, Y)
        assert torch.equal(Y, Yref), "schedule changed results"
        us = timeit(lambda: ops._poly_step(csr0, X, Y))
        by = 8 * A.nnz + 4 * (n + 1) + 8 * n * d
        r = {"order": "as generated, rcm schedule", "d": d, "us": round(us, 1),
             "GBps": round(by / us / 1e3, 1), "hbm_frac": round(by / us / 1e3 / 8000, 4)}
        res.append(r)
        print(json.dumps(r), flush=True)
    for name, perm in orders.items():
        inv = np.empty_like(perm)
        inv[perm] = np.arange(n)
        P = A[perm][:, perm].tocsr()
        P.sort_indices()
        csr = ops.SparseCSR(torch.from_numpy(P.indptr.astype(np.int32)).to(dev),
                            torch.from_numpy(P.indices.astype(np.int32)).to(dev),
                            torch.from_numpy(P.data.astype(np.float32)).to(dev), n, n, P.nnz)
        bw = int(np.abs(P.tocoo().row - P.tocoo().col).max())
        for d in args.d:
            X = torch.randn(n, d, device=dev)
            Y = torch.empty(n, d, device=dev)
            us = timeit(lambda: ops._poly_step(csr, X, Y))
            by = 8 * P.nnz + 4 * (n + 1) + 8 * n * d
            r = {"order": name, "d": d, "us": round(us, 1), "GBps": round(by / us / 1e3, 1),
                 "hbm_frac": round(by / us / 1e3 / 8000, 4), "bandwidth": bw, "n": n, "nnz": P.nnz}
            res.append(r)
            print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
