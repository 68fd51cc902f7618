"""Where the time of one k_proj_bn_fwd launch goes (config-2 shapes).

hlhgat_set_proj_bn_stamps: thread 0 of every workgroup stamps s_memrealtime
(100 MHz, 10 ns) at its phase boundaries.  One stamped launch after warm-up
(and the same launch timed with events, unstamped); reports, in µs from the
first workgroup's start: workgroup start skew, main-loop (GEMM) time, when
the last workgroup's partials were written, the finaliser's bump, the
pollers' detection lag, the y store, and the launch's event time.

    python3 tools/probes/proj_bn_phases.py [--reps 20]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def q(v):
    v = np.asarray(v, dtype=np.float64)
    return {"min": round(float(v.min()), 2), "med": round(float(np.median(v)), 2),
            "p90": round(float(np.percentile(v, 90)), 2), "max": round(float(v.max()), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from hlhgat import _lib
    from hlhgat.synthetic import zinc_like_batch
    L = _lib.LIB
    dev = torch.device("cuda:0")
    zb = zinc_like_batch(1000, seed=1)
    nt, ns = zb.x_t.shape[0], zb.x_s.shape[0]
    g = torch.Generator(device="cpu").manual_seed(0)
    out = []
    for M, kbs, tag in [(nt, [64, 64, 64], "conv K=3 d=64 (nodes)"),
                        (ns, [64, 64, 64], "conv K=3 d=64 (edges)"),
                        (ns, [384, 384], "Linear(768,64) (edges)")]:
        N = 64
        As = [torch.randn(M, k, generator=g).to(dev) for k in kbs]
        W = torch.randn(N, sum(kbs), generator=g).to(dev)
        bias = torch.randn(N, generator=g).to(dev)
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
        gx = (M + 63) // 64
        st = torch.zeros(gx * 8, dtype=torch.int64, device=dev)

        def pb():
            _lib.check(L.hlhgat_proj_bn_fwd(
                nb, A_p, lda, W_p, ldw, kb_, M, N, bias.data_ptr(), x.data_ptr(), N, None,
                bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                bn.running_var.data_ptr(), bn.num_batches_tracked.data_ptr(), 0.1, 1e-5, 1,
                y.data_ptr(), N, mean.data_ptr(), inv.data_ptr(), ws.data_ptr(), ws.numel(),
                torch.cuda.current_stream().cuda_stream), "proj_bn_fwd")

        res = measure(pb, st, gx, args.reps)
        res.update({"shape": tag, "M": M, "K": sum(kbs), "workgroups": gx})
        out.append(res)
        print(json.dumps(res), flush=True)


def measure(pb, st, gx, reps):
    from hlhgat import _lib
    L = _lib.LIB
    for _ in range(5):
        pb()
    torch.cuda.synchronize()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        pb()
        b.record()
        b.synchronize()
        ev.append(a.elapsed_time(b) * 1e3)
    runs = []
    for _ in range(reps):
        st.zero_()
        _lib.check(L.hlhgat_set_proj_bn_stamps(st.data_ptr(), st.numel()), "stamps")
        pb()
        torch.cuda.synchronize()
        _lib.check(L.hlhgat_set_proj_bn_stamps(None, 0), "stamps off")
        runs.append(st.view(gx, 8).cpu().numpy().astype(np.float64))
    from hlhgat import ops
    ops.check_device_errors()
    res = {"event_us": q(ev)}
    keys = ["start_skew", "gemm", "partials", "last_partials", "group_level",
            "finaliser_bump", "poll_lag", "y_store", "last_y_store"]
    agg = {k: [] for k in keys}
    for s in runs:
        t = (s[:, :6] - s[:, 0].min()) / 100.0  # µs
        flags = s[:, 6].astype(np.int64)
        top = np.nonzero(flags & 2)[0]
        if len(top) != 1:
            continue
        tp = top[0]
        others = np.nonzero((flags & 2) == 0)[0]
        agg["start_skew"].append(t[:, 0].max())
        agg["gemm"].append(np.median(t[:, 1] - t[:, 0]))
        agg["partials"].append(np.median(t[:, 2] - t[:, 1]))
        agg["last_partials"].append(t[:, 2].max())
        agg["group_level"].append(t[tp, 3] - t[:, 2].max())
        agg["finaliser_bump"].append(t[tp, 4])
        agg["poll_lag"].append(np.median(t[others, 4]) - t[tp, 4])
        agg["y_store"].append(np.median(t[:, 5] - t[:, 4]))
        agg["last_y_store"].append(t[:, 5].max())
    res["phases_us"] = {k: q(v) for k, v in agg.items() if v}
    res["stamped_runs"] = len(agg["gemm"])
    return res


if __name__ == "__main__":
    main()
