"""Probe: eager vs whole-step hipGraph replay (fwd + L1 + bwd + fused Adam) of
the cfg2 model, with and without the node/edge two-stream fork."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
import torch  # noqa: E402

import hlhgat  # noqa: E402
from hlhgat import ops  # noqa: E402
from hlhgat.synthetic import zinc_like_batch  # noqa: E402

KW = dict(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256], K=3, keig=15)
dev = torch.device("cuda:0")
b = zinc_like_batch(1000, seed=1).to(dev)


def run(fork: bool):
    ops.set_stream_fork(fork)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(dev).train()
    if os.environ.get("PROBE_NO_SPLIT"):
        from hlhgat.nn import Sequential
        for mod in m.modules():
            if isinstance(mod, Sequential):
                mod._split = None
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-3, fused=True,
                           capturable=True)
    crit = torch.nn.L1Loss()

    def step():
        ops.clear_caches()
        out = m(b)
        loss = crit(out.view(-1, 1), b.y.view(-1, 1))
        loss.backward()
        opt.step()
        return loss

    for _ in range(3):
        opt.zero_grad(set_to_none=False)
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        opt.zero_grad(set_to_none=False)
        loss = step()
    torch.cuda.synchronize()
    print(f"fork={fork} eager: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step "
          f"loss {loss.item():.5f}", flush=True)
    del loss  # drop the autograd graph: its AccumulateGrad nodes pin the default stream

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            opt.zero_grad(set_to_none=False)
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=False)
    with torch.cuda.graph(g, stream=s):
        for p in m.parameters():
            p.grad.zero_()
        static_loss = step()
    ops.clear_caches()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 50
    print(f"fork={fork} graph replay: {dt * 1e3:.3f} ms/step = {1000 / dt:.0f} graphs/s, "
          f"loss {static_loss.item():.5f}", flush=True)


run(False)
if not os.environ.get("PROBE_ONLY_NOFORK"):
    run(True)
