"""Where the config-3 per-sample pipeline spends its time: SuperpixelPipeline
stage timings (device synchronised at every stage boundary) over a few
256-graph batches, plus pad_levels.

    python tools/probes/pipeline_stages.py [--batches 4]
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

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--graphs", type=int, default=256)
    args = ap.parse_args()
    from hlhgat.hodge_dataset import level_caps, pad_levels
    from hlhgat.pipeline import SuperpixelPipeline, superpixel_raw
    G, B = args.graphs, args.batches
    raw = [superpixel_raw(5000 + i) for i in range(B * G)]
    pipe = SuperpixelPipeline(raw, keig=11, aug=True)
    dev = torch.device("cuda:0")
    bs = [pipe.batch(range(b * G, (b + 1) * G), seed=b, device=dev) for b in range(B)]  # warm
    caps = level_caps(bs, 512)
    pipe.PROFILE = True
    pipe.stage_ms = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tp = 0.0
    pads = []
    for b in range(B):
        d = pipe.batch(range(b * G, (b + 1) * G), seed=b, device=dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        pad_levels(d, caps)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        pad_levels(d, caps)
        torch.cuda.synchronize()
        pads.append((round((t2 - t1) * 1e3, 2), round((time.perf_counter() - t2) * 1e3, 2)))
        tp += t2 - t1
    print("pad_levels ms (first, again) per batch:", pads, flush=True)
    tot = (time.perf_counter() - t0) / B * 1e3
    # where pad_levels spends its host time (torch.profiler, CPU ops)
    from torch.profiler import ProfilerActivity, profile
    d = pipe.batch(range(0, G), seed=0, device=dev)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        pad_levels(d, caps)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=12), flush=True)
    st = {k: round(v / B, 2) for k, v in pipe.stage_ms.items()}
    st["pad_levels"] = round(tp / B * 1e3, 2)
    print(json.dumps({"ms_per_batch": round(tot, 2), "graphs": G, "stages_ms": st}))


if __name__ == "__main__":
    main()
