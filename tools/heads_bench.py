"""graphs/s (fwd + loss + bwd) of the attention-pooling heads at BASELINE
configs 3 and 4 on one GPU, eager (no hipGraph: the two MLGC levels change
shape every batch).

    python tools/heads_bench.py [--configs cifar peptides] [--steps 10]

cifar    (config 3): HL_HGCNN_CIFAR10SP_dense_int3_attpool(channels=[2,2,2],
         filters=[64,128,256], mlp=[256], K=4, keig=10, pool_loc=1, l=0.5),
         256 CIFAR-like superpixel graphs (118 nodes, 8-NN) per batch
         (main_cifar10SP...:35-36,186-187), cross-entropy loss.
peptides (config 4): HL_HGCNN_pepfunc_dense_int3_attpool(channels=[2,2,2],
         filters=[64,128,256], mlp=[256], K=6, pool_loc=1), 64 peptide-like
         molecules (~151 atoms) per batch (main_pepfunc...:27-28), BCE loss.
Synthetic data, random-init weights.  One JSON line per config.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

CONFIGS = {
    "cifar": dict(kind="cifar", graphs=256, cls="HL_HGCNN_CIFAR10SP_dense_int3_attpool",
                  kw=dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256], K=4,
                          keig=10, pool_loc=1, l=0.5), loss="ce"),
    "peptides": dict(kind="peptides", graphs=64, cls="HL_HGCNN_pepfunc_dense_int3_attpool",
                     kw=dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256],
                             K=6, pool_loc=1), loss="bce"),
}


def to_dev(b, dev):
    for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
              "edge_index", "num_node1", "num_edge1", "y"):
        v = getattr(b, k, None)
        if torch.is_tensor(v):
            setattr(b, k, v.to(dev))
    return b


def run(name, steps, warmup, n_batches, dev):
    import hlhgat
    from hlhgat.synthetic import two_level_batch
    c = CONFIGS[name]
    t0 = time.time()
    batches = [[to_dev(b, dev) for b in two_level_batch(c["kind"], c["graphs"], seed=s)]
               for s in range(n_batches)]
    t_data = time.time() - t0
    torch.manual_seed(0)
    m = getattr(hlhgat, c["cls"])(**c["kw"]).to(dev).train()
    n_params = sum(p.numel() for p in m.parameters())

    def step(i):
        datas = batches[i % n_batches]
        out = m(datas)
        y = datas[0].y
        if c["loss"] == "ce":
            loss = torch.nn.functional.cross_entropy(out, y.view(-1).long())
        else:
            loss = torch.nn.functional.binary_cross_entropy_with_logits(out, y.view(out.shape))
        m.zero_grad(set_to_none=True)
        loss.backward()

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    b0 = batches[0][0]
    return {"config": name, "head": c["cls"], "graphs_per_step": c["graphs"],
            "value": round(c["graphs"] / dt, 1), "unit": "graphs/s", "ms_per_step": round(dt * 1e3, 3),
            "mode": "eager fwd+loss+bwd", "params": n_params, "rows_t": int(b0.x_t.shape[0]),
            "rows_s": int(b0.x_s.shape[0]), "nnz_s": int(b0.edge_index_s.shape[1]),
            "data_gen_s": round(t_data, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["cifar", "peptides"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batches", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.configs:
        print(json.dumps(run(name, args.steps, args.warmup, args.batches, dev)), flush=True)


if __name__ == "__main__":
    main()
