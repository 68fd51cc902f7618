"""Projection kernels at the exact shapes of a step (a HLHGAT_LOG_PROJ census,
tools/gpu_steps.sh census5): each distinct (call, M, N, blocks, ld) timed in
isolation per hlhgat_set_gemm_big mode, and the census-weighted sum -- the
step's GEMM time if every launch ran as fast as alone.

    python tools/kbench_census.py gpurun_out/r05g_census5.txt [--modes 0,1] [--min-gflop 1]
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

LINE = re.compile(r"^\s*(\d+) \[hlhgat proj\] (\w+) M=(\d+) N=(\d+) kb=([\d,]+)(?: ld=([\d,]+))?")


def parse(path):
    shapes = {}
    for ln in open(path):
        m = LINE.match(ln)
        if not m:
            continue
        cnt, kind, M, N, kb = int(m[1]), m[2], int(m[3]), int(m[4]), [int(x) for x in m[5].split(",")]
        ld = [int(x) for x in m[6].split(",")] if m[6] else list(kb)
        key = (kind, M, N, tuple(kb), tuple(ld))
        shapes[key] = shapes.get(key, 0) + cnt
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("census")
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--min-gflop", type=float, default=0.5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chain", type=int, default=3)
    args = ap.parse_args()
    from hlhgat import _lib, ops
    dev = torch.device("cuda:0")
    modes = [int(m) for m in args.modes.split(",")]
    shapes = parse(args.census)
    g = torch.Generator(device="cpu").manual_seed(0)
    total = {m: 0.0 for m in modes}
    total_small = 0.0
    for (kind, M, N, kb, ld), cnt in sorted(shapes.items(), key=lambda kv: -kv[0][1] * kv[0][2]
                                            * sum(kv[0][3])):
        fl = 2.0 * M * N * sum(kb)
        if fl * cnt < args.min_gflop * 1e9:
            total_small += fl * cnt
            continue
        As = [torch.randn(M, l, generator=g).to(dev)[:, :k] for k, l in zip(kb, ld)]
        W = torch.randn(N, sum(kb), generator=g).to(dev)
        Ws, o = [], 0
        for k in kb:
            Ws.append(W[:, o:o + k])
            o += k
        G = torch.randn(M, N, generator=g).to(dev)
        out = torch.empty(M, N, device=dev)
        dAs = [torch.empty(M, k, device=dev) for k in kb]
        dW = torch.empty_like(W)
        dWs, o = [], 0
        for k in kb:
            dWs.append(dW[:, o:o + k])
            o += k
        db = torch.empty(N, device=dev)
        fn = {"fwd": lambda: ops._proj_fwd(As, Ws, M, N, None, out),
              "bwd_d": lambda: ops._proj_bwd_data(G, Ws, list(kb), dAs),
              "bwd_w": lambda: ops._proj_bwd_weight(G, As, dWs, db)}[kind]
        row = {"call": kind, "M": M, "N": N, "kb": list(kb), "ld": list(ld), "count": cnt,
               "gflop": round(fl / 1e9, 2)}
        for m in modes:
            _lib.check(_lib.LIB.hlhgat_set_gemm_big(m, 0), "set_gemm_big")
            _, ch = timed(fn, args.reps, args.chain)
            row[f"us_{m}"] = round(ch, 1)
            row[f"TF_{m}"] = round(fl / ch / 1e6, 1)
            total[m] += ch * cnt
        print(json.dumps(row), flush=True)
        del As, W, G, out, dAs, dW
    _lib.check(_lib.LIB.hlhgat_set_gemm_big(-1, 0), "set_gemm_big")
    print(json.dumps({"census_weighted_ms": {str(m): round(v / 1e3, 3) for m, v in total.items()},
                      "gflop_not_timed": round(total_small / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
