"""Probe: is a grouped node+edge launch cheaper than the two concurrent chains?

At the bench's ZINC shape (1000 graphs), one HL conv->BN->ReLU forward +
backward on L0 (nodes) and on L1 (edges):
  two   : the two sides on two streams (ops.fork), as the model runs them;
  union : ONE conv over the block-diagonal union blockdiag(L0, L1) with the
          two sides' rows stacked -- the launch count of a grouped design
          (same kernels, twice the rows per launch; the weights / BN are
          shared here, which only changes numbers, not the cost);
  node / edge : one side alone.
Each variant is captured into a hipGraph of `reps` iterations and replayed.

    python tools/group_probe.py [--reps 20] [--layers 1]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hl-hgat_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--graphs", type=int, default=1000)
    args = ap.parse_args()
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    dev = torch.device("cuda:0")
    b = zinc_like_batch(args.graphs, seed=1).to(dev)
    nt, ns = b.x_t.shape[0], b.x_s.shape[0]
    opT = ops.hodge_operator(b.edge_index_t, b.edge_weight_t, nt)
    opS = ops.hodge_operator(b.edge_index_s, b.edge_weight_s, ns)
    ei_u = torch.cat([b.edge_index_t, b.edge_index_s + nt], 1).contiguous()
    w_u = torch.cat([b.edge_weight_t, b.edge_weight_s]).contiguous()
    ops.mark_hodge(ei_u)
    opU = ops.hodge_operator(ei_u, w_u, nt + ns)
    g = torch.Generator().manual_seed(0)
    F, K = 64, 3
    ws = [[(torch.randn(F, F, generator=g) / 8).to(dev).requires_grad_(True) for _ in range(K)]
          for _ in range(args.layers)]
    bias = [torch.zeros(F, device=dev, requires_grad=True) for _ in range(args.layers)]
    bns = [torch.nn.BatchNorm1d(F).to(dev) for _ in range(args.layers)]
    xt = torch.randn(nt, F, generator=g).to(dev).requires_grad_(True)
    xs = torch.randn(ns, F, generator=g).to(dev).requires_grad_(True)
    xu = torch.cat([xt.detach(), xs.detach()]).requires_grad_(True)
    params = [p for l in ws for p in l] + bias

    def chain(x, op):
        for i in range(args.layers):
            x = ops.hodge_poly_conv(x, op, ws[i], bias[i], bn=bns[i], relu=True)
        return x

    def it_two():
        yt, ys = ops.fork(lambda: chain(xt, opT), lambda: chain(xs, opS), device=dev)
        loss = yt.sum() + ys.sum()
        return torch.autograd.grad(loss, [xt, xs] + params)

    def it_union():
        return torch.autograd.grad(chain(xu, opU).sum(), [xu] + params)

    def it_node():
        return torch.autograd.grad(chain(xt, opT).sum(), [xt] + params)

    def it_edge():
        return torch.autograd.grad(chain(xs, opS).sum(), [xs] + params)

    out = {"graphs": args.graphs, "n_nodes": nt, "n_edges": ns, "layers": args.layers}
    for name, fn in (("two", it_two), ("union", it_union), ("node", it_node), ("edge", it_edge)):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(args.reps):
                fn()
            ops.join_capture_streams(dev)
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for _ in range(5):
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / args.reps)
        times.sort()
        out[name + "_us"] = round(times[len(times) // 2], 1)
        del graph
    out["union_vs_two"] = round(out["union_us"] / out["two_us"], 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
