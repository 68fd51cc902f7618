"""Per-kernel timings of the hlhgat HIP ops at the BASELINE.json shapes.

    python tools/microbench.py [--quick] [--out gpurun_out/microbench.json]

Times each op with HIP events on the current stream (median of R reps after
warm-up) and reports algorithmic bytes / flops per launch (SURVEY.md §8d
formulas) against the MI355X peaks (HBM 8 TB/s, fp32 MFMA 157.3 TF/s).
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

HBM = 8000.0
MFMA = 157.3


def timeit(fn, reps=50, warm=5):
    for _ in range(warm):
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
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "microbench.json"))
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph, zinc_like_batch

    dev = torch.device("cuda:0")
    res = []

    def rec(name, us, us_min, bytes_=None, flops=None, **kw):
        r = {"op": name, "us": round(us, 2), "us_min": round(us_min, 2)}
        if bytes_:
            r["GBps"] = round(bytes_ / us / 1e3, 1)
            r["hbm_frac"] = round(bytes_ / us / 1e3 / HBM, 4)
        if flops:
            r["TFps"] = round(flops / us / 1e6, 2)
            r["mfma_frac"] = round(flops / us / 1e6 / MFMA, 4)
        r.update(kw)
        res.append(r)
        print(json.dumps(r), flush=True)

    # ---- operators ------------------------------------------------------
    zb = zinc_like_batch(1000, seed=1).to(dev)
    tsp = collate([tsp_like_graph(s) for s in range(4)], check_hodge=False)
    tsp.hodge_sorted = {"edge_index_s": True, "edge_index_t": True}
    tsp = tsp.to(dev)
    shapes = [("zinc_L0", zb.edge_index_t, zb.edge_weight_t, zb.x_t.shape[0], [64]),
              ("zinc_L1", zb.edge_index_s, zb.edge_weight_s, zb.x_s.shape[0], [64]),
              ("tsp4_L1", tsp.edge_index_s, tsp.edge_weight_s, tsp.x_s.shape[0], [32, 64, 128]),
              ("tsp4_L0", tsp.edge_index_t, tsp.edge_weight_t, tsp.x_t.shape[0], [128])]
    for name, ei, w, n, ds in shapes:
        op = ops.hodge_operator(ei, w, n)
        A = op.fwd
        for d in ds:
            X = torch.randn(n, d, device=dev)
            Z = torch.randn(n, d, device=dev)
            Y = torch.empty(n, d, device=dev)
            csr_b = 8 * A.nnz + 4 * (n + 1)
            us, mn = timeit(lambda: ops._poly_step(A, X, Y), args.reps)
            rec(f"spmm {name} d={d}", us, mn, csr_b + 8 * n * d, 2 * A.nnz * d, n=n, nnz=A.nnz)
            us, mn = timeit(lambda: ops._poly_step(A, X, Y, Z=Z, alpha=-1.0, beta=3.0, gamma=-1.0,
                                                   div=2.0), args.reps)
            rec(f"laguerre_step {name} d={d}", us, mn, csr_b + 12 * n * d, 2 * A.nnz * d,
                n=n, nnz=A.nnz)
    # CSR builds (per step work)
    ei, w, n = zb.edge_index_s, zb.edge_weight_s, zb.x_s.shape[0]
    us, mn = timeit(lambda: ops._csr_sorted(ei[0], ei[1], w, n, n), args.reps)
    rec("csr_from_sorted zinc_L1", us, mn)
    us, mn = timeit(lambda: ops._csr_general(ei[1], ei[0], w, n, n), args.reps)
    rec("csr_from_coo(sort) zinc_L1", us, mn)
    us, mn = timeit(lambda: ops.incidence(zb.edge_index.clone(), zb.x_t.shape[0]), args.reps)
    rec("incidence_csr zinc", us, mn)

    # ---- projections ----------------------------------------------------
    for M, N, kbs, tag in [(23259, 64, [64, 64, 64], "conv K=3 d=64"),
                           (23259, 64, [36, 36, 36], "init conv d=36"),
                           (24927, 64, [384, 384], "MSI Linear(768,64)"),
                           (24927, 64, [64], "MSI Linear(64,64)"),
                           (206936, 128, [128] * 4, "tsp conv K=4 d=128")]:
        As = [torch.randn(M, k, device=dev) for k in kbs]
        W = torch.randn(N, sum(kbs), device=dev)
        Ws, o = [], 0
        for k in kbs:
            Ws.append(W[:, o:o + k])
            o += k
        out = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * sum(kbs)
        by = 4.0 * M * (sum(kbs) + N)
        us, mn = timeit(lambda: ops._proj_fwd(As, Ws, M, N, None, out), args.reps)
        rec(f"proj_fwd {tag}", us, mn, by, fl)
        G = torch.randn(M, N, device=dev)
        dAs = [torch.empty(M, k, device=dev) for k in kbs]
        us, mn = timeit(lambda: ops._proj_bwd_data(G, Ws, kbs, dAs), args.reps)
        rec(f"proj_bwd_data {tag}", us, mn, by, fl)
        dW = torch.empty_like(W)
        dWs, o = [], 0
        for k in kbs:
            dWs.append(dW[:, o:o + k])
            o += k
        db = torch.empty(N, device=dev)
        us, mn = timeit(lambda: ops._proj_bwd_weight(G, As, dWs, db), args.reps)
        rec(f"proj_bwd_weight {tag}", us, mn, by, fl)
        if len(kbs) == 1:
            Wt = W.t().contiguous()
            us, mn = timeit(lambda: torch.mm(As[0], W.t()), args.reps)
            rec(f"torch.mm (hipBLASLt) {tag}", us, mn, by, fl)

    # ---- batch norm --------------------------------------------------------
    for n, C in [(23259, 64), (24927, 64), (1000, 256)]:
        x = torch.randn(n, C, device=dev, requires_grad=True)
        bn = torch.nn.BatchNorm1d(C).to(dev).train()
        us, mn = timeit(lambda: ops.batch_norm_act(x, bn, relu=True), args.reps)
        rec(f"bn_relu_fwd hip [{n},{C}]", us, mn, 8.0 * n * C)
        y = ops.batch_norm_act(x, bn, relu=True)
        g = torch.randn_like(y)
        us, mn = timeit(lambda: torch.autograd.grad(y, x, g, retain_graph=True), args.reps)
        rec(f"bn_relu_bwd hip [{n},{C}]", us, mn, 16.0 * n * C)
        us, mn = timeit(lambda: torch.relu(bn(x)), args.reps)
        rec(f"bn_relu_fwd torch [{n},{C}]", us, mn, 8.0 * n * C)

    # ---- boundary operator / attention ------------------------------------
    inc = ops.incidence(zb.edge_index, zb.x_t.shape[0])
    for d in (64, 384):
        xs = torch.randn(zb.x_s.shape[0], d, device=dev)
        xt = torch.randn(zb.x_t.shape[0], d, device=dev)
        rD = torch.rand(zb.x_t.shape[0], device=dev) + 0.5
        us, mn = timeit(lambda: ops.node_from_edges(xs, inc, rD), args.reps)
        rec(f"node_from_edges d={d}", us, mn, 4.0 * d * (xs.shape[0] + xt.shape[0]))
        us, mn = timeit(lambda: ops.edge_from_nodes(xt, inc), args.reps)
        rec(f"edge_from_nodes d={d}", us, mn, 4.0 * d * (xs.shape[0] + xt.shape[0]))
    q = torch.randn(24927, 96, device=dev)
    us, mn = timeit(lambda: ops.att_score(q[:, :32], q[:, 32:64], q[:, 64:], 0.1, 0.9,
                                          5.656854, ops.SIGMA_SIGMOID), args.reps)
    rec("att_score n=24927 dk=32", us, mn, 4.0 * 24927 * 97)

    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
