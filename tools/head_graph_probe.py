"""Probe: can the config-5 TSP head (and the attpool heads) run as a
replayed hipGraph through TrainStep(graphs=True)?  For each head: 3 eager
steps vs 3 graph steps from the same initial weights and batches (losses and
final weights compared), then steps/s of both.  Prints one JSON line per
head."""
import json
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hl-hgat_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import hlhgat  # noqa: E402
from hlhgat.train import TrainStep  # noqa: E402


def run(name, graphs, steps=8):
    c = bench.HEADS[name]
    raw = [bench._head_batch(c["kind"], c["graphs"], s) for s in range(2)]
    dev = torch.device("cuda:0")
    batches = [b.to(dev) if c["kind"] == "tsp" else [x.to(dev) for x in b] for b in raw]
    torch.manual_seed(0)
    m = getattr(hlhgat, c["cls"])(**c["kw"]).to(dev).train()
    st = TrainStep(m, lambda o, d, k=c["kind"]: bench._head_loss(k, o, d), lr=1e-3,
                   graphs=graphs)
    losses = []
    for i in range(4):
        losses.append(float(st(batches[i % 2]).detach()))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        st(batches[i % 2])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    w = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()
    return losses, w, dt, dict(st.stats)


out = {}
for name in sys.argv[1:] or ["cfg5_tsp_pyr"]:
    le, we, de, se = run(name, False)
    try:
        lg, wg, dg, sg = run(name, True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"head": name, "graphs": "failed", "error": repr(e)[:300],
                          "where": traceback.format_exc()[-2500:]}), flush=True)
        break
    print(json.dumps({"head": name, "eager_ms": round(de * 1e3, 2), "graph_ms": round(dg * 1e3, 2),
                      "losses_eager": le, "losses_graph": lg,
                      "weights_max_abs_diff": float((we - wg).abs().max()),
                      "stats": sg}), flush=True)
