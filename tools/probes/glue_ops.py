"""Which torch ops launch the non-hlhgat ("glue") kernels of a head's step.

One eager training step (fwd + loss + bwd + Adam) of a bench head under
torch.profiler recording input shapes; prints the ATen ops that ran
device kernels, grouped by input shape, sorted by device time.

    python3 tools/probes/glue_ops.py [--head cfg4_pepfunc_attpool]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--head", default="cfg4_pepfunc_attpool")
    ap.add_argument("--rows", type=int, default=70)
    args = ap.parse_args()
    import bench
    import hlhgat
    from hlhgat.hodge_dataset import level_caps, pad_batch, pad_levels, static_caps
    from hlhgat.train import TrainStep
    dev = torch.device("cuda:0")
    c = bench.HEADS[args.head]
    kind, G = c["kind"], c["graphs"]
    pool = bench._head_pool(kind, 2 * G)
    rng = np.random.RandomState(7)
    raw = bench._head_collate(kind, [pool[i] for i in rng.choice(len(pool), G, replace=False)])
    if kind == "tsp":
        b = pad_batch(raw, static_caps(raw, 512)).to(dev)
    else:
        b = [x.to(dev) for x in pad_levels(raw, level_caps([raw], 512))]
    torch.manual_seed(0)
    m = getattr(hlhgat, c["cls"])(**c["kw"]).to(dev).train()
    st = TrainStep(m, lambda o, d: bench._head_loss(kind, o, d), lr=1e-3, graphs=False)
    for _ in range(3):
        st(b)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        st(b)
        torch.cuda.synchronize()
    key = "self_device_time_total"
    rows = [e for e in prof.key_averages(group_by_input_shape=True)
            if e.key.startswith("aten::") and e.self_device_time_total > 0]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:args.rows]:
        print(f"{e.key:24s} calls {e.count:3d}  dev_us {e.self_device_time_total:9.1f}  "
              f"shapes {e.input_shapes}", flush=True)
    print(prof.key_averages().table(sort_by=key, row_limit=40, max_name_column_width=60),
          flush=True)


if __name__ == "__main__":
    main()
