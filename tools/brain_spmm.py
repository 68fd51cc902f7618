"""L1 SpMM / Laguerre basis on the reference's brain skeleton (HL-HGAT-DEMO
data, the skewed-degree stress case: 8997 edges, nnz(L1) 1.37 M = 152 entries
per row), CSR vs the Hodge-factored L1, kernel time from hipExtLaunchKernel
stamps.  Batches of B copies of the skeleton (block-diagonal, as a DataLoader
batch of subjects would be).

    python tools/brain_spmm.py [--batch 1 8 32] [--d 32 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 32])
    ap.add_argument("--d", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import hodge_coo_from_boundary
    g = np.load(os.path.join(REPO, "tests", "golden", "brain_skeleton.npz"))
    n = int(g["n_nodes"])
    ei_t, w_t, ei_s, w_s = hodge_coo_from_boundary(g["edge_index"], n, float(g["lmax"]))
    E = g["edge_index"].shape[1]
    dev = torch.device("cuda:0")
    for B in args.batch:
        eis = torch.cat([ei_s + b * E for b in range(B)], 1)
        ws = w_s.repeat(B)
        eib = torch.cat([torch.from_numpy(g["edge_index"]) + b * n for b in range(B)], 1)
        rows, nnz = B * E, eis.shape[1]
        ops_ = {}
        for fac in (False, True):
            e = ops.mark_hodge(eis.to(dev))
            if fac:
                ops.set_hodge_factor(e, eib.to(dev), B * n)
            ops_[fac] = ops.hodge_operator(e, ws.to(dev), rows)
        for d in args.d:
            X = torch.randn(rows, d, device=dev)
            ref = ops.spmm(ops_[False].fwd, X)
            err = float((ops.hodge_spmm(ops_[True], X) - ref).abs().max() / ref.abs().max())
            by = 8 * nnz + 4 * (rows + 1) + 8 * rows * d
            res = {"graphs": B, "rows": rows, "nnz": nnz, "d": d, "factored_rel_err": err}
            for fac, name in ((False, "csr"), (True, "factored")):
                classes = ((hlhgat._lib.PROF_HODGE_NODE, hlhgat._lib.PROF_HODGE_EDGE) if fac
                           else (hlhgat._lib.PROF_POLY,))
                fn = (lambda: ops.hodge_spmm(ops_[True], X)) if fac else \
                    (lambda: ops.spmm(ops_[False].fwd, X))
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                ops.prof_reset()
                for c in classes:
                    ops.prof_enable(c, True)
                for _ in range(args.reps):
                    fn()
                torch.cuda.synchronize()
                for c in classes:
                    ops.prof_enable(c, False)
                us = sum(ops.prof_read(c)["ms"] for c in classes) * 1e3 / args.reps
                res[f"{name}_us"] = round(us, 2)
                res[f"{name}_equiv_frac"] = round(by / us / 1e3 / PEAK, 4)
            res["speedup"] = round(res["csr_us"] / res["factored_us"], 2)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
