"""Per-launch kernel cost at the cfg2 (ZINC, 1000 graphs) shapes.

    python tools/kbench.py [--only REGEX] [--reps 30] [--chain 20]

For every op: `iso` = median of single launches bracketed by events (includes
the event/launch latency), `chain` = median over reps of (CHAIN back-to-back
launches between two events) / CHAIN: what one launch costs inside a step.
HLHGAT_* env knobs select kernel variants (A/B in one process, run twice).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def timed(fn, reps, chain):
    """iso: single eager launch between events; chain: CHAIN launches captured
    in one hipGraph and replayed (host launch cost removed)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    iso, ch = [], []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        iso.append(a.elapsed_time(b) * 1e3)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(chain):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        b.synchronize()
        ch.append(a.elapsed_time(b) * 1e3 / chain)
    iso.sort()
    ch.sort()
    return iso[len(iso) // 2], ch[len(ch) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=".")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--chain", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--big", action="store_true",
                    help="config 3 / 5 projection shapes only (CIFAR / TSP heads)")
    ap.add_argument("--modes", default="0,1",
                    help="--big: hlhgat_set_gemm_big modes to time (0 small tiles, 1 large)")
    args = ap.parse_args()
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    dev = torch.device("cuda:0")
    pat = re.compile(args.only)
    res = []

    def run(name, fn, bytes_=None, flops=None):
        if not pat.search(name):
            return
        iso, ch = timed(fn, args.reps, args.chain)
        r = {"op": name, "iso_us": round(iso, 2), "chain_us": round(ch, 2)}
        if bytes_:
            r["chain_GBps"] = round(bytes_ / ch / 1e3, 1)
        if flops:
            r["chain_TFps"] = round(flops / ch / 1e6, 2)
        res.append(r)
        print(json.dumps(r), flush=True)

    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*s):
        return torch.randn(*s, generator=g).to(dev)

    if args.big:  # projection shapes of the config-3 / config-5 heads (M rows, N, blocks)
        # per-GPU config-5 batch: 4 TSP graphs of 2500 nodes -> 10000 nodes,
        # 51698 edges; widths of the dense-concat NodeEdgeInt (2 d) and the
        # K=4 convs; config 3: 256 CIFAR superpixel graphs
        from hlhgat import _lib
        shapes = [(51698, 128, [800, 800], "TSP edge NEInt L2 Linear(1600,128)"),
                  (10000, 128, [800, 800], "TSP node NEInt L2 Linear(1600,128)"),
                  (51698, 128, [128] * 4, "TSP edge conv K=4 d=128"),
                  (51698, 64, [352, 352], "TSP edge NEInt L1 Linear(704,64)"),
                  (51698, 64, [64] * 4, "TSP edge conv K=4 d=64"),
                  (51698, 32, [128, 128], "TSP edge NEInt L0 Linear(256,32)"),
                  (143192, 256, [448, 448], "CIFAR NEInt L2 edge Linear(896,256)"),
                  (143192, 64, [64] * 4, "CIFAR conv K=4 d=64")]
        modes = [int(m) for m in args.modes.split(",")]
        for M, N, kbs, tag in shapes:
            As = [rnd(M, k) for k in kbs]
            W = rnd(N, sum(kbs))
            Ws, o = [], 0
            for k in kbs:
                Ws.append(W[:, o:o + k])
                o += k
            out = torch.empty(M, N, device=dev)
            fl = 2.0 * M * N * sum(kbs)
            by = 4.0 * M * (sum(kbs) + N)
            G = rnd(M, N)
            dAs = [torch.empty(M, k, device=dev) for k in kbs]
            dW = torch.empty_like(W)
            dWs, o = [], 0
            for k in kbs:
                dWs.append(dW[:, o:o + k])
                o += k
            db = torch.empty(N, device=dev)
            for mode in modes:
                _lib.check(_lib.LIB.hlhgat_set_gemm_big(mode, 0), "set_gemm_big")
                tg = f"{tag} big={mode}"
                run(f"proj_fwd {tg}", lambda: ops._proj_fwd(As, Ws, M, N, None, out), by, fl)
                run(f"proj_bwd_data {tg}", lambda: ops._proj_bwd_data(G, Ws, kbs, dAs), by, fl)
                run(f"proj_bwd_weight {tg}", lambda: ops._proj_bwd_weight(G, As, dWs, db), by, fl)
            _lib.check(_lib.LIB.hlhgat_set_gemm_big(-1, 0), "set_gemm_big")
            Acat = torch.cat(As, 1)
            run(f"ref torch.mm fwd {tag}", lambda: torch.mm(Acat, W.t(), out=out), by, fl)
            run(f"ref torch.mm wgrad {tag}", lambda: torch.mm(G.t(), Acat, out=dW), by, fl)
            del As, G, dAs, Acat
        return
    zb = zinc_like_batch(1000, seed=1).to(dev)
    nt, ns = zb.x_t.shape[0], zb.x_s.shape[0]
    # ---- reference points: streaming copies / library GEMM at the same bytes --
    Xr = rnd(nt, 192)
    Yr = torch.empty_like(Xr)
    Wr = rnd(192, 64)
    Or = torch.empty(nt, 64, device=dev)
    run("ref copy [23k,192]", lambda: Yr.copy_(Xr), 8.0 * Xr.numel())
    run("ref rowsum [23k,192]", lambda: torch.sum(Xr, 1, out=Or[:, 0]), 4.0 * Xr.numel())
    run("ref torch.mm [23k,192]x[192,64]", lambda: torch.mm(Xr, Wr, out=Or),
        4.0 * (Xr.numel() + Or.numel()), 2.0 * nt * 192 * 64)
    X6 = rnd(nt, 64)
    Y6 = torch.empty_like(X6)
    run("ref copy [23k,64]", lambda: Y6.copy_(X6), 8.0 * X6.numel())
    # ---- projections (cfg2 shapes) ------------------------------------------
    for M, N, kbs, tag in [(nt, 64, [64, 64, 64], "conv K=3 d=64"),
                           (nt, 64, [36, 36, 36], "init conv d=36"),
                           (ns, 64, [18, 18, 18], "init conv d=18"),
                           (ns, 64, [384, 384], "MSI Linear(768,64)"),
                           (nt, 128, [64], "NEI Wt pack Linear(64,128) nodes"),
                           (ns, 128, [64], "NEI Ws pack Linear(64,128) edges"),
                           (ns, 64, [128, 128], "MSI Linear(256,64)"),
                           (ns, 64, [64], "MSI Linear(64,64)"),
                           (1000, 256, [128, 128], "mlp Linear(256,256)"),
                           (1000, 1, [256], "out Linear(256,1)")]:
        As = [rnd(M, k) for k in kbs]
        W = rnd(N, sum(kbs))
        bias = rnd(N)
        Ws, o = [], 0
        for k in kbs:
            Ws.append(W[:, o:o + k])
            o += k
        out = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * sum(kbs)
        by = 4.0 * M * (sum(kbs) + N)
        run(f"proj_fwd {tag}", lambda: ops._proj_fwd(As, Ws, M, N, bias, out), by, fl)
        G = rnd(M, N)
        dAs = [torch.empty(M, k, device=dev) for k in kbs]
        run(f"proj_bwd_data {tag}", lambda: ops._proj_bwd_data(G, Ws, kbs, dAs), by, fl)
        dW = torch.empty_like(W)
        dWs, o = [], 0
        for k in kbs:
            dWs.append(dW[:, o:o + k])
            o += k
        db = torch.empty(N, device=dev)
        run(f"proj_bwd_weight {tag}", lambda: ops._proj_bwd_weight(G, As, dWs, db), by, fl)
        # the product's Linear backward: weight partials + data gradient in one
        # launch, then the split reduction (torch.ops.hlhgat.proj_backward)
        Acat = [a.contiguous() for a in As]
        run(f"proj_bwd_fused {tag}",
            lambda: torch.ops.hlhgat.proj_backward(G, Acat, W, True), 2 * by, 2 * fl)
    # ---- projection + BatchNorm forward (hlhgat_proj_bn_fwd) -----------------
    import ctypes
    from hlhgat import _lib
    L = _lib.LIB
    for M, kbs, tag in [(nt, [64, 64, 64], "conv K=3 d=64"), (ns, [384, 384], "Linear(768,64)")]:
        N = 64
        As = [rnd(M, k) for k in kbs]
        W = rnd(N, sum(kbs))
        bias = rnd(N)
        bn = torch.nn.BatchNorm1d(N).to(dev).train()
        nb = len(kbs)
        offs = [sum(kbs[:i]) for i in range(nb)]
        A_p = (ctypes.c_void_p * nb)(*[a.data_ptr() for a in As])
        lda = (ctypes.c_int64 * nb)(*[a.stride(0) for a in As])
        W_p = (ctypes.c_void_p * nb)(*[W.data_ptr() + 4 * o for o in offs])
        ldw = (ctypes.c_int64 * nb)(*([W.stride(0)] * nb))
        kb_ = (ctypes.c_int64 * nb)(*kbs)
        x = torch.empty(M, N, device=dev)
        y = torch.empty(M, N, device=dev)
        mean = torch.empty(N, device=dev)
        inv = torch.empty(N, device=dev)
        ws = torch.zeros(int(L.hlhgat_bn_workspace_bytes(M, N)), dtype=torch.uint8, device=dev)

        def pb():
            L.hlhgat_proj_bn_fwd(nb, A_p, lda, W_p, ldw, kb_, M, N, bias.data_ptr(),
                                 x.data_ptr(), N, None, bn.weight.data_ptr(),
                                 bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                                 bn.running_var.data_ptr(), bn.num_batches_tracked.data_ptr(),
                                 0.1, 1e-5, 1, y.data_ptr(), N, mean.data_ptr(),
                                 inv.data_ptr(), ws.data_ptr(), ws.numel(),
                                 torch.cuda.current_stream().cuda_stream)
        fl = 2.0 * M * N * sum(kbs)
        L.hlhgat_set_proj_bn_fused(1)
        run(f"proj_bn_fwd fused {tag}", pb, None, fl)
        L.hlhgat_set_bn_wait_us(0)
        run(f"proj_bn_fwd fused, every tile handed to the finaliser {tag}", pb, None, fl)
        L.hlhgat_set_bn_wait_us(1000)
        L.hlhgat_set_proj_bn_fused(0)
        run(f"proj_bn_fwd two-call {tag}", pb, None, fl)
        L.hlhgat_set_proj_bn_fused(1)
    # ---- batch norm ----------------------------------------------------------
    for n, C in [(nt, 64), (ns, 64), (1000, 256)]:
        x = rnd(n, C).requires_grad_(True)
        bn = torch.nn.BatchNorm1d(C).to(dev).train()
        run(f"bn_relu_fwd [{n},{C}]", lambda: ops.batch_norm_act(x, bn, relu=True), 8.0 * n * C)
        gy = torch.randn(n, C, device=dev)
        run(f"bn_relu_fwd+bwd [{n},{C}]",
            lambda: torch.autograd.grad(ops.batch_norm_act(x, bn, relu=True), x, gy),
            24.0 * n * C)
    # ---- SpMM / Laguerre step ----------------------------------------------
    for name, ei, w, n in [("L0", zb.edge_index_t, zb.edge_weight_t, nt),
                           ("L1", zb.edge_index_s, zb.edge_weight_s, ns)]:
        op = ops.hodge_operator(ei, w, n)
        A = op.fwd
        X, Z, Y = rnd(n, 64), rnd(n, 64), torch.empty(n, 64, device=dev)
        by = 8 * A.nnz + 4 * (n + 1) + 12 * n * 64
        run(f"laguerre_step {name} d=64",
            lambda: ops._poly_step(A, X, Y, Z=Z, alpha=-1.0, beta=3.0, gamma=-1.0, div=2.0), by)
    # ---- Laguerre basis K=3 (two step launches) ----------------------------------
    for side in ("t", "s"):
        ei = getattr(zb, "edge_index_" + side)
        w = getattr(zb, "edge_weight_" + side)
        n = getattr(zb, "x_" + side).shape[0]
        X = rnd(n, 64)
        op = ops.hodge_operator(ops.mark_hodge(ei.clone()), w, n)
        by = 8 * op.fwd.nnz + 4 * (n + 1) + 4 * n * 64 * 3
        run(f"basis K=3 L_{side} d=64", lambda: ops.poly_basis(op, X, 3, ops.POLY_LAGUERRE), by)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
