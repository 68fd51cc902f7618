"""Host enqueue time per replayed step vs GPU time per step (bench workload)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
import hlhgat  # noqa: E402
from hlhgat.train import TrainStep  # noqa: E402

dev = torch.device("cuda:0")
batches, caps, _, _, ds = bench.make_batches(8, 0, dev)
torch.manual_seed(0)
model = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
crit = hlhgat.nn.L1Loss()
step = TrainStep(model, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                 weight_decay=1e-3, graphs=True)
for i in range(6):
    step(batches[i % 8])
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    parts = {"key": 0.0, "load": 0.0, "replay": 0.0}
    for i in range(40):
        b = batches[i % 8]
        a = time.perf_counter()
        key = hlhgat.train.batch_key(b)
        ent = step._graphs[key]
        c = time.perf_counter()
        ent.load(b)
        d = time.perf_counter()
        ent.graph.replay()
        e = time.perf_counter()
        parts["key"] += c - a
        parts["load"] += d - c
        parts["replay"] += e - d
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e3 * (t1 - t0) / 40:.3f} ms/step, total {1e3 * (t2 - t0) / 40:.3f} ms/step, "
          + ", ".join(f"{k} {1e3 * v / 40:.3f}" for k, v in parts.items()), flush=True)

# the loader-fed loop's host side: one pinned batch's H2D (all its tensors)
import numpy as np  # noqa: E402
idx = np.arange(1000)
pb = ds.collate(idx, caps, pin=True)
n_t = sum(1 for v in vars(pb).values() if torch.is_tensor(v))
for rep in range(3):
    t0 = time.perf_counter()
    for i in range(20):
        bd = pb.to(dev, non_blocking=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"upload: {n_t} tensors, host {1e3 * (t1 - t0) / 20:.3f} ms/batch", flush=True)
