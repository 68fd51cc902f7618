"""Is the replayed step's launch lag per graph node?  The bench's config-2
step with N extra no-op kernels (torch.cuda._sleep(1), ~2 us of GPU time
each) captured at the start of the step's forward, same-process interleaved
timing.  If the GPU waits for the host's per-node packet writing (~7 us per
node), each no-op costs ~7 us of step time; if not, ~2 us.

    python tools/probes/packet_cost.py [--rounds 4] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import bench
    import hlhgat
    from hlhgat.train import TrainStep
    dev = torch.device("cuda:0")
    batches, _, _, _, _ = bench.make_batches(2, 0, dev)
    crit = hlhgat.nn.L1Loss()
    steps = {}
    for n in (0, 50, 100, 200):
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
        st = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                       weight_decay=1e-3, graphs=True)
        orig = st._fwd_bwd

        def fb(batch, orig=orig, n=n):
            for _ in range(n):
                torch.cuda._sleep(1)
            return orig(batch)
        st._fwd_bwd = fb
        for i in range(4):
            st(batches[i % 2])
        torch.cuda.synchronize()
        steps[n] = st
    res = {n: [] for n in steps}
    for r in range(args.rounds):
        for n, st in steps.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                st(batches[i % 2])
            torch.cuda.synchronize()
            res[n].append(round((time.perf_counter() - t0) / args.steps * 1e3, 4))
    # the no-op's own GPU time in a chain (no host involvement)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(200):
            torch.cuda._sleep(1)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    b.synchronize()
    print(json.dumps({"ms_per_step": {str(n): v for n, v in res.items()},
                      "noop_us_in_a_graph_chain": round(a.elapsed_time(b) * 1e3 / 200, 2)}))


if __name__ == "__main__":
    main()
