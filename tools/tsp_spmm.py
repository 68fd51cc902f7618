"""SpMM / Laguerre step at BASELINE config 5 (TSP-like, 4 graphs of 10k
nodes, L1 n ~ 207k rows, nnz ~ 4.1M) against the HBM roofline.

    python tools/tsp_spmm.py [--graphs 4] [--d 64 128] [--tiles 128:256 64:128]

Variants, all on the same operator and bitwise-equal outputs (checked):
  plain   k_poly_step, natural row order
  rcm     k_poly_step, RCM row schedule (hodge_dataset.locality_order)
  halo    k_poly_halo, LDS halo tiles along the RCM schedule (max_rows:max_halo)
  factored  L1 = alpha B1^T B1 (hlhgat_hodge_factor_t): B1 X over the node rows,
          then one fused edge step; NOT bitwise (checked to 1e-5 relative)
Ops: spmm, laguerre_step (one fused step) and basis_k3 (T_1, T_2 of a K = 3
Laguerre basis: 2 steps, 16 nnz + 8 (n+1) + 20 n d bytes; the only form the
factored variant has besides spmm).
Algorithmic bytes: SpMM 8 nnz + 4 (n+1) + 8 n d; Laguerre step
(reads T_k, T_{k-1}) 8 nnz + 4 (n+1) + 12 n d.  Peak 8 TB/s.
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

import torch  # noqa: E402

PEAK_GBPS = 8000.0


def timeit(fn, reps=30):
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
    ap.add_argument("--d", type=int, nargs="+", default=[64, 128])
    ap.add_argument("--tiles", nargs="+", default=["24:160:768", "32:192:1024"])
    ap.add_argument("--out", default="")
    ap.add_argument("--no-factored", action="store_true")
    args = ap.parse_args()
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate, halo_tiles
    from hlhgat.synthetic import tsp_like_graph
    dev = torch.device("cuda:0")
    gs = [tsp_like_graph(s, halo=False) for s in range(args.graphs)]
    b = collate(gs, check_hodge=False)
    ei, w = b.edge_index_s, b.edge_weight_s
    n, nnz = b.x_s.shape[0], ei.shape[1]
    order = b.row_order_s
    variants = {"plain": ops.hodge_operator(ops.mark_hodge(ei.to(dev)), w.to(dev), n),
                "rcm": ops.hodge_operator(ops.set_row_order(ops.mark_hodge(ei.to(dev)), order),
                                          w.to(dev), n)}
    for spec in args.tiles:
        mr, mh, mn = (int(v) for v in spec.split(":"))
        ht = halo_tiles(ei.numpy(), n, order.numpy(), max_rows=mr, max_halo=mh, max_nnz=mn)
        e = ops.set_row_order(ops.mark_hodge(ei.to(dev)), order)
        ops.set_halo(e, ht)
        op = ops.hodge_operator(e, w.to(dev), n)
        op.info = {"tiles": ht["halo_tile_ptr"].numel() - 1,
                   "reuse": round(nnz / int(ht["halo_ptr"][-1]), 2)}
        variants[f"halo {spec}"] = op
    if not args.no_factored:
        ef = ops.set_row_order(ops.mark_hodge(ei.to(dev)), order)
        ops.set_hodge_factor(ef, b.edge_index.to(dev), b.x_t.shape[0], b.row_order_t)
        opf = ops.hodge_operator(ef, w.to(dev), n)
        assert opf.factor is not None
        variants["factored"] = opf
    res = []
    for d in args.d:
        X = torch.randn(n, d, device=dev)
        Z = torch.randn(n, d, device=dev)
        Y = torch.empty(n, d, device=dev)
        ref = None
        for name, op in variants.items():
            A = op.fwd
            fac = op.factor is not None
            if fac:
                Yf = ops.hodge_spmm(op, X)
                err = float((Yf - ref).abs().max() / ref.abs().max())
                assert err < 1e-5, f"{name}: {err}"
                cases = [("spmm", lambda: ops.hodge_spmm(op, X),
                          8 * nnz + 4 * (n + 1) + 8 * n * d)]
            else:
                ops._poly_step(A, X, Y)
                if ref is None:
                    ref = Y.clone()
                assert torch.equal(Y, ref), f"{name}: results differ"
                cases = [("spmm", lambda: ops._poly_step(A, X, Y),
                          8 * nnz + 4 * (n + 1) + 8 * n * d),
                         ("laguerre_step", lambda: ops._poly_step(A, X, Y, Z=Z, alpha=-1.0,
                                                                  beta=5.0, gamma=-2.0, div=3.0),
                          8 * nnz + 4 * (n + 1) + 12 * n * d)]
            cases.append(("basis_k3", lambda: ops.poly_basis(op, X, 3, ops.POLY_LAGUERRE),
                          16 * nnz + 8 * (n + 1) + 20 * n * d))
            for what, fn, by in cases:
                us = timeit(fn)
                r = {"variant": name, "op": what, "d": d, "n": n, "nnz": nnz, "us": round(us, 1),
                     "GBps": round(by / us / 1e3, 1),
                     "hbm_frac": round(by / us / 1e3 / PEAK_GBPS, 4)}
                r.update(getattr(op, "info", {}))
                res.append(r)
                print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
