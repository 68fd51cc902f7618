"""Data-parallel gradient check on the HIP path, 2 ranks.

    HLHGAT_DIST_BACKEND=gloo HLHGAT_SHARE_GPU=1 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/ddp_check.py [--out gpurun_out/ddp_check.json]

(on an 8-GPU node: the same without the two env variables, RCCL.)

- ZINC head (config 2), a different 64-graph shard per rank: the DDP gradient
  equals the mean of the two per-shard gradients, each computed in one process
  before the process group exists.
- TSP head (config 5), 2 x 1500-node graphs per rank: as ZINC.
- pepfunc attpool head (config 4), the SAME shard on both ranks: the attention
  is divided by the batch max over all ranks (hlhgat.distributed.global_max),
  which with identical shards equals the local max, so the DDP gradient equals
  the one-process gradient on that shard; this exercises the cross-rank max and
  its backward exchange.
Every rank checks; rank 0 writes the JSON summary.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

TOL = 1e-5  # relative to max(1, |g|_max) per parameter


def zinc_setup(dev):
    import hlhgat
    from hlhgat.synthetic import zinc_like_batch
    kw = dict(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256], K=3, keig=15)
    shards = [zinc_like_batch(64, seed=7 + r).to(dev) for r in range(2)]

    def model():
        torch.manual_seed(0)
        return hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**kw).to(dev).train()

    def loss(m, b):
        return torch.nn.functional.l1_loss(m(b).view(-1), b.y.view(-1))
    return model, loss, shards


def pep_setup(dev):
    import hlhgat
    from hlhgat.synthetic import two_level_batch
    kw = dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256], K=6, pool_loc=1)
    shard = [b.to(dev) for b in two_level_batch("peptides", 8, seed=3)]
    shards = [shard, shard]

    def model():
        torch.manual_seed(0)
        return hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(**kw).to(dev).train()

    def loss(m, datas):
        out = m(datas)
        return torch.nn.functional.binary_cross_entropy_with_logits(
            out, datas[0].y.view(out.shape))
    return model, loss, shards


def tsp_setup(dev):
    import hlhgat
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph
    kw = dict(channels=[4, 4, 4], filters=[32, 64, 128], mlp_channels=[256], K=4)
    shards = [collate([tsp_like_graph(11 + 2 * r + i, n=1500) for i in range(2)],
                      check_hodge=False).to(dev) for r in range(2)]

    def model():
        torch.manual_seed(0)
        return hlhgat.HL_HGCNN_TSP_dense_int3_pyr(**kw).to(dev).train()

    def loss(m, b):
        logits, _ = m(b)
        return torch.nn.functional.binary_cross_entropy_with_logits(
            logits.view(-1), b.y.view(-1).float())
    return model, loss, shards


def grads_of(m):
    return {k: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
            for k, p in m.named_parameters()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/ddp_check.json")
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    assert world == 2, "run with --nproc-per-node 2"
    dev0 = torch.device("cuda", 0 if os.environ.get("HLHGAT_SHARE_GPU") == "1"
                        else int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev0)
    cases = {"zinc": zinc_setup(dev0), "pepfunc": pep_setup(dev0), "tsp": tsp_setup(dev0)}
    # one-process references, before the process group exists
    refs, per_shard = {}, {}
    for name, (model, loss, shards) in cases.items():
        gs = []
        for r in range(world):
            m = model()
            torch.manual_seed(100)
            loss(m, shards[r]).backward()
            gs.append(grads_of(m))
        per_shard[name] = gs
        refs[name] = {k: sum(g[k] for g in gs) / world for k in gs[0]}
    from hlhgat.distributed import init_distributed, wrap_ddp
    r, w, dev = init_distributed()
    assert dev == dev0 and r == rank
    report = {}
    ok = True
    for name, (model, loss, shards) in cases.items():
        m = model()
        ddp = wrap_ddp(m, dev)
        torch.manual_seed(100)
        loss(ddp, shards[r]).backward()
        g = grads_of(m)
        errs = {}
        for k, ref in refs[name].items():
            scale = max(1.0, float(ref.abs().max()))
            errs[k] = float((g[k] - ref).abs().max()) / scale
        worst = max(errs.values())
        report[name] = {"params": len(g), "max_rel_err": worst, "tol": TOL,
                        "ok": worst <= TOL,
                        "worst_params": sorted(errs, key=errs.get)[-3:]}
        if name == "pepfunc":  # same shard twice: a one-process repeatability figure
            a, b = per_shard[name]
            report[name]["repeat_rel_err"] = max(
                float((a[k] - b[k]).abs().max()) / max(1.0, float(a[k].abs().max())) for k in a)
        ok &= worst <= TOL
    torch.cuda.synchronize()
    flags = torch.tensor([int(ok)], device="cpu" if dist.get_backend() == "gloo" else dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank == 0:
        report["backend"] = dist.get_backend()
        report["all_ranks_ok"] = bool(flags.item())
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(report, f, indent=1)
        print(json.dumps(report))
    print(f"[rank {rank}] {report}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
