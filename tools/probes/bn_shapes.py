"""BatchNorm kernels alone at the config-2 / config-5 shapes: each C-ABI call
replayed 20x in a captured hipGraph (events around the replays), µs per call
and GB/s on the algorithmic bytes (stats 4nC, apply 8nC, backward reduction
12nC: x, dy, y; backward apply 16nC: x, dy, y read, dx written).

    python3 tools/probes/bn_shapes.py [--reps 10] [--chain 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def timed(fn, reps, chain):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(chain):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gr.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / chain)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--chain", type=int, default=20)
    args = ap.parse_args()
    from hlhgat import _lib
    L = _lib.LIB
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for n, C, tag in [(23157, 64, "cfg2 nodes"), (24868, 64, "cfg2 edges"),
                      (40448, 32, "cfg5 nodes"), (40448, 128, "cfg5 nodes"),
                      (207360, 32, "cfg5 edges"), (207360, 64, "cfg5 edges"),
                      (207360, 128, "cfg5 edges"), (143360, 64, "cfg3 edges"),
                      (143360, 256, "cfg3 edges")]:
        x = (torch.randn(n, C, generator=g) * 2 + 0.5).to(dev)
        dy = torch.randn(n, C, generator=g).to(dev)
        y = torch.empty(n, C, device=dev)
        dx = torch.empty(n, C, device=dev)
        w = torch.rand(C, generator=g).to(dev) + 0.5
        b = torch.randn(C, generator=g).to(dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros(1, dtype=torch.int64, device=dev)
        mean, inv = torch.empty(C, device=dev), torch.empty(C, device=dev)
        coef = torch.empty(3 * C, device=dev)
        dw, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        ws = torch.zeros(int(L.hlhgat_bn_workspace_bytes(n, C)), dtype=torch.uint8, device=dev)

        def st():
            return torch.cuda.current_stream().cuda_stream

        def stats():
            _lib.check(L.hlhgat_bn_stats_train(x.data_ptr(), C, n, None, C, rm.data_ptr(),
                                               rv.data_ptr(), nbt.data_ptr(), 0.1, 1e-5,
                                               mean.data_ptr(), inv.data_ptr(), ws.data_ptr(),
                                               ws.numel(), st()), "stats")

        def apply():
            _lib.check(L.hlhgat_bn_apply(x.data_ptr(), C, n, None, C, w.data_ptr(), b.data_ptr(),
                                         mean.data_ptr(), inv.data_ptr(), 1, y.data_ptr(), C,
                                         st()), "apply")

        def fwd():
            _lib.check(L.hlhgat_bn_fwd_train(x.data_ptr(), C, n, None, C, w.data_ptr(),
                                             b.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                                             nbt.data_ptr(), 0.1, 1e-5, 1, y.data_ptr(), C,
                                             mean.data_ptr(), inv.data_ptr(), ws.data_ptr(),
                                             ws.numel(), st()), "fwd")

        def bred():
            _lib.check(L.hlhgat_bn_bwd_reduce(x.data_ptr(), C, y.data_ptr(), C, dy.data_ptr(), C, n,
                                              None, C, w.data_ptr(), mean.data_ptr(),
                                              inv.data_ptr(), coef.data_ptr(), dw.data_ptr(),
                                              db.data_ptr(), ws.data_ptr(), ws.numel(), st()),
                       "bwd_reduce")

        def bwd():
            _lib.check(L.hlhgat_bn_bwd_train(x.data_ptr(), C, y.data_ptr(), C, dy.data_ptr(), C, n,
                                             None, C, w.data_ptr(), mean.data_ptr(),
                                             inv.data_ptr(), dx.data_ptr(), C, dw.data_ptr(),
                                             db.data_ptr(), ws.data_ptr(), ws.numel(), st()),
                       "bwd")

        fwd()
        torch.cuda.synchronize()
        nC = float(n) * C
        r = {"shape": tag, "n": n, "C": C}
        for name, fn, by in (("stats", stats, 4 * nC), ("apply", apply, 8 * nC),
                             ("fwd", fwd, None), ("bwd_reduce", bred, 12 * nC),
                             ("bwd", bwd, 28 * nC)):
            us = timed(fn, args.reps, args.chain)
            r[name + "_us"] = round(us, 2)
            if by:
                r[name + "_GBps"] = round(by / us / 1e3, 1)
        r["bwd_apply_us_by_diff"] = round(r["bwd_us"] - r["bwd_reduce_us"], 2)
        r["bwd_apply_GBps_by_diff"] = round(16 * nC / max(r["bwd_apply_us_by_diff"], 1e-3) / 1e3, 1)
        print(json.dumps(r), flush=True)
        del x, dy, y, dx, ws
    from hlhgat import ops
    ops.check_device_errors()


if __name__ == "__main__":
    main()
