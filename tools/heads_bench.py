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
tsp      (config 5): HL_HGCNN_TSP_dense_int3_pyr(channels=[4,4,4],
         filters=[32,64,128], mlp=[256], K=4), 4 TSP-like graphs (10k nodes,
         9-NN) per GPU, BCE on the masked edge logits
         (main_TSP...:316-321 trains a focal-BCE).
Synthetic data, random-init weights.  One JSON line per config.  The L1
operators of cifar / tsp batches run factored (hlhgat_hodge_factor_t) unless
HLHGAT_FACTOR=0.
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
    "tsp": dict(kind="tsp", graphs=4, cls="HL_HGCNN_TSP_dense_int3_pyr",
                kw=dict(channels=[4, 4, 4], filters=[32, 64, 128], mlp_channels=[256], K=4),
                loss="edge_bce"),
}


def make_batch(kind, graphs, seed):
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph, two_level_batch
    if kind == "tsp":
        return collate([tsp_like_graph(seed * graphs + i) for i in range(graphs)],
                       check_hodge=False)
    return two_level_batch(kind, graphs, seed=seed)


def run(name, steps, warmup, n_batches, dev):
    import hlhgat
    from hlhgat import ops
    c = CONFIGS[name]
    t0 = time.time()
    batches = []
    for s in range(n_batches):
        bb = make_batch(c["kind"], c["graphs"], s)
        # Batch.to also attaches the operator hints (row schedules, halo tiles,
        # hodge factor) that collate recorded
        batches.append(bb.to(dev) if c["kind"] == "tsp" else [b.to(dev) for b in bb])
    t_data = time.time() - t0
    torch.manual_seed(0)
    m = getattr(hlhgat, c["cls"])(**c["kw"]).to(dev).train()
    n_params = sum(p.numel() for p in m.parameters())

    def step(i):
        datas = batches[i % n_batches]
        out = m(datas)
        if c["loss"] == "edge_bce":
            logits, _ = out
            loss = torch.nn.functional.binary_cross_entropy_with_logits(
                logits.view(-1), datas.y.view(-1).float())
            m.zero_grad(set_to_none=True)
            loss.backward()
            return
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
    b0 = batches[0] if c["kind"] == "tsp" else batches[0][0]
    op = ops.hodge_operator(b0.edge_index_s, b0.edge_weight_s, b0.x_s.shape[0])
    return {"config": name, "head": c["cls"], "graphs_per_step": c["graphs"],
            "value": round(c["graphs"] / dt, 1), "unit": "graphs/s", "ms_per_step": round(dt * 1e3, 3),
            "mode": "eager fwd+loss+bwd", "params": n_params, "rows_t": int(b0.x_t.shape[0]),
            "rows_s": int(b0.x_s.shape[0]), "nnz_s": int(b0.edge_index_s.shape[1]),
            "data_gen_s": round(t_data, 1), "l1_factored": op.factor is not None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["cifar", "peptides", "tsp"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batches", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.configs:
        print(json.dumps(run(name, args.steps, args.warmup, args.batches, dev)), flush=True)


if __name__ == "__main__":
    main()
