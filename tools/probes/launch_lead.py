"""Does the replayed step wait for the host's graph launch?  Times the bench
workload's replayed step with a GPU-side sleep of S us enqueued right before
every replay (after the batch copy-in).  If the first blocks stall because the
GPU catches up with the host writing the replay's packets, the step minus S
gets SHORTER as S grows (the host is ahead by then); if not, it stays flat.

    python tools/probes/launch_lead.py [--steps 20] [--rounds 3]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import bench
    import hlhgat
    from hlhgat import train
    from hlhgat.train import TrainStep
    dev = torch.device("cuda:0")
    batches, _, _, _, _ = bench.make_batches(4, 0, dev)
    crit = hlhgat.nn.L1Loss()
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
    st = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                   weight_decay=1e-3, graphs=True)
    for i in range(6):
        st(batches[i % len(batches)])
    torch.cuda.synchronize()
    # calibrate torch.cuda._sleep: cycles per us
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    torch.cuda._sleep(1_000_000)
    b.record()
    b.synchronize()
    cyc_per_us = 1_000_000 / (a.elapsed_time(b) * 1e3)
    lead = {"sleep_us": 0}
    orig_load = train._Captured.load

    def load(self, batch):
        orig_load(self, batch)
        if lead["sleep_us"]:
            torch.cuda._sleep(int(lead["sleep_us"] * cyc_per_us))

    train._Captured.load = load
    res = {}
    for r in range(args.rounds):
        for s_us in (0, 200, 400, 800):
            lead["sleep_us"] = s_us
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for i in range(args.steps):
                st(batches[i % len(batches)])
            b.record()
            b.synchronize()
            ms = a.elapsed_time(b) / args.steps
            res.setdefault(s_us, []).append(round(ms - s_us / 1e3, 4))
    # host time per step call (no synchronisation inside the loop)
    lead["sleep_us"] = 0
    torch.cuda.synchronize()
    hs = []
    for i in range(args.steps * 2):
        t0 = time.perf_counter()
        st(batches[i % len(batches)])
        hs.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    hs.sort()
    print(json.dumps({"cycles_per_us": round(cyc_per_us, 1),
                      "step_minus_sleep_ms": {str(k): v for k, v in res.items()},
                      "host_ms_per_call_median": round(hs[len(hs) // 2], 4),
                      "host_ms_per_call_min": round(hs[0], 4)}))


if __name__ == "__main__":
    main()
