"""Linear backward at the configs' shapes, per weight-gradient staging mode
(hlhgat_set_wgrad_stages: 0 = two-deep register ring, 3..6 = LDS-DMA ring
of that depth): the fused launch (weight partials + data gradient + split
reduction, torch.ops.hlhgat.proj_backward) and its weight-only half
(hlhgat_proj_bwd_weight + reduce), each as a hipGraph chain of one shape
(tools/kbench.timed).  Also checks that every mode gives the mode-0 bits.

    python tools/wgrad_bench.py [--stages 0,3,4,6] [--only cfg2]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd"), os.path.join(REPO, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from kbench import timed  # noqa: E402

# (tag, M, N, input blocks): the config-2 step (ZINC, 1000 graphs: 23.5k node
# rows, 25k edge rows) and the config-5 step (4 TSP graphs: 40.4k / 207k rows)
SHAPES = [
    ("cfg2 conv K=3 d=64 (edges)", 25088, 64, [64, 64, 64]),
    ("cfg2 NEInt fused Linear(320->128) (edges)", 25088, 128, [320]),
    ("cfg2 NEInt Linear(64,64)", 25088, 64, [64]),
    ("cfg5 conv K=4 d=128 (edges)", 207360, 128, [128, 128, 128, 128]),
    ("cfg5 NEInt fused Linear(800->256) (edges)", 207360, 256, [800]),
    ("cfg5 conv K=4 d=64 (edges)", 207360, 64, [64, 64, 64, 64]),
    ("cfg5 NEInt fused Linear(800->256) (nodes)", 40448, 256, [800]),
    ("cfg5 conv K=4 d=32 (edges)", 207360, 32, [32, 32, 32, 32]),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="0,3,4,5,6")
    ap.add_argument("--only", default=".")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--chain", type=int, default=5)
    args = ap.parse_args()
    from hlhgat import _lib, ops
    L = _lib.LIB
    dev = torch.device("cuda:0")
    stages = [int(v) for v in args.stages.split(",")]
    pat = re.compile(args.only)
    g = torch.Generator(device="cpu").manual_seed(0)
    for tag, M, N, kbs in SHAPES:
        if not pat.search(tag):
            continue
        As = [torch.randn(M, k, generator=g).to(dev) for k in kbs]
        W = (torch.randn(N, sum(kbs), generator=g) * 0.05).to(dev)
        G = torch.randn(M, N, generator=g).to(dev)
        dW = torch.empty_like(W)
        dWs, o = [], 0
        for k in kbs:
            dWs.append(dW[:, o:o + k])
            o += k
        db = torch.empty(N, device=dev)
        fl = 2.0 * M * N * sum(kbs)
        ref = None
        for st in stages:
            _lib.check(L.hlhgat_set_wgrad_stages(st), "set_wgrad_stages")
            try:
                out = torch.ops.hlhgat.proj_backward(G, As, W, True)
                ops._proj_bwd_weight(G, As, dWs, db)
                torch.cuda.synchronize()
                got = [out[0].clone(), out[1].clone()] + [t.clone() for t in out[2]] + \
                    [dW.clone(), db.clone()]
                if ref is None:
                    ref = got
                same = all(torch.equal(a, b) for a, b in zip(ref, got))
                _, t_f = timed(lambda: torch.ops.hlhgat.proj_backward(G, As, W, True),
                               args.reps, args.chain)
                _, t_w = timed(lambda: ops._proj_bwd_weight(G, As, dWs, db), args.reps,
                               args.chain)
            finally:
                L.hlhgat_set_wgrad_stages(0)
            print(json.dumps({"shape": tag, "M": M, "N": N, "kb": kbs, "stages": st,
                              "fused_us": round(t_f, 1), "fused_TFps": round(2 * fl / t_f / 1e6, 1),
                              "weight_us": round(t_w, 1),
                              "weight_TFps": round(fl / t_w / 1e6, 1),
                              "bitwise_mode0": same}), flush=True)
        del As, W, G, dW
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
