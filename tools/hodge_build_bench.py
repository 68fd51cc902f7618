"""On-device Hodge builder (hlhgat_hodge_lmax + hlhgat_hodge_build) vs the host
sparse construction, at BASELINE config 3 (256 CIFAR-like superpixel graphs)
and config 5 (4 TSP-like graphs of 10k nodes): lmax agreement (Lanczos vs the
host eigh / eigsh), COO equality given the same lmax, and wall time.

    python tools/hodge_build_bench.py
"""
from __future__ import annotations

import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate, hodge_coo_from_boundary
    from hlhgat.synthetic import knn_edges
    from scipy.sparse.linalg import eigsh
    import scipy.sparse as sp
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    for name, n, k, B in (("cfg3 CIFAR-like", 118, 8, 256), ("cfg5 TSP-like", 10000, 9, 4)):
        eis, counts, lams_host = [], [], []
        t0 = time.perf_counter()
        off = 0
        for g in range(B):
            ei = knn_edges(rng.random((n, 2)), k)
            E = ei.shape[1]
            Bm = sp.csr_matrix((np.concatenate([-np.ones(E), np.ones(E)]),
                                (np.concatenate([ei[0], ei[1]]), np.concatenate([np.arange(E)] * 2))),
                               shape=(n, E))
            L0 = (Bm @ Bm.T).astype(np.float64)
            if n <= 500:
                lam = float(np.linalg.eigvalsh(L0.toarray()).max())
            else:
                lam = float(eigsh(L0, k=1, which="LA", return_eigenvectors=False)[0])
            hodge_coo_from_boundary(ei, n, lam)  # the host sparse build, timed
            lams_host.append(lam)
            eis.append(ei + off)
            counts.append(n)
            off += n
        t_host = time.perf_counter() - t0
        ei_all = torch.from_numpy(np.concatenate(eis, 1)).to(dev)
        torch.cuda.synchronize()
        for _ in range(2):
            ops.clear_caches()
            ops.hodge_build(ei_all, counts)
        torch.cuda.synchronize()
        ops.clear_caches()
        t0 = time.perf_counter()
        ei_t, w_t, ei_s, w_s, lam_d = ops.hodge_build(ei_all, counts)
        torch.cuda.synchronize()
        t_dev = time.perf_counter() - t0
        rel = np.abs(lam_d.double().cpu().numpy() - np.array(lams_host)) / np.array(lams_host)
        # same lmax -> same COO as the host construction (graph 0)
        e0 = torch.from_numpy(eis[0])
        h = hodge_coo_from_boundary(eis[0], n, float(np.float32(lam_d[0].item())))
        d = ops.hodge_build(e0.to(dev), [n], lam_d[:1].cpu())
        same = all(torch.equal(a.cpu(), b) for a, b in zip(d[:4], h))
        print(json.dumps({"batch": name, "graphs": B, "nodes": off, "edges": int(ei_all.shape[1]),
                          "nnz_L1": int(ei_s.shape[1]), "device_build_ms": round(t_dev * 1e3, 2),
                          "host_build_ms": round(t_host * 1e3, 1),
                          "lmax_rel_diff_max": float(rel.max()), "coo_equal_given_lmax": same}),
              flush=True)


if __name__ == "__main__":
    main()
