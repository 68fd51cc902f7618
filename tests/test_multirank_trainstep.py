"""The data-parallel training step the multi-GPU bench runs (bench.py --gpus N:
hlhgat.train.TrainStep with world > 1), on the product models (-m gpu).

Two ranks share the one GPU of the test box (HLHGAT_SHARE_GPU=1, gloo: the
rehearsal mode of hlhgat.distributed.init_distributed; RCCL refuses two
ranks on one device).  Each rank trains its own shard of every step's graphs
(sharding by graph) through TrainStep -- captured hipGraph +
flat one-bucket all-reduce (mean over ranks, as DDP) + the HIP Adam -- for 4
steps.  The check: after every rank's 4 steps the parameters are BITWISE
those of a one-process emulation (per step: the two shards' gradients at the
same parameters, summed and halved as the all-reduce + div does, then the
same Adam step).

* ZINC (configs 1-2 head), every shard padded to one capacity bucket: one
  capture per rank, then replays;
* peptides attpool head (BASELINE configs[3] runs it under 8-GPU DDP): two
  level-batch shapes per rank, captured and replayed;
* CIFAR attpool head: its forward divides by the batch-global max
  (distributed.global_max, an all-reduce MAX inside the forward,
  lib/Hodge_ST_Model.py:1061-1062), which gloo cannot capture, so TrainStep
  runs it eagerly (graphs_off); the emulation takes the max over both shards.

The CPU test checks that TrainStep refuses a DDP-wrapped module (two
gradient reductions per step otherwise).
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import REPO
from test_sync_bn import _env, _run_ranks

STEPS = 4
ZKW = dict(channels=[1, 1], filters=[32, 32], mlp_channels=[32], K=3, keig=15)
HEADKW = {"peptides": dict(channels=[1, 1], filters=[32, 64], mlp_channels=[64], K=3,
                           pool_loc=0),
          "cifar": dict(channels=[1, 1], filters=[32, 64], mlp_channels=[64], K=3, keig=10,
                        pool_loc=0, l=0.5),
          # BASELINE configs[3] itself (peptides under 8-GPU DDP): K=6, pool_loc=1
          "peptides_cfg4": dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256],
                                K=6, pool_loc=1)}
HEADCLS = {"peptides": "HL_HGCNN_pepfunc_dense_int3_attpool",
           "peptides_cfg4": "HL_HGCNN_pepfunc_dense_int3_attpool",
           "cifar": "HL_HGCNN_CIFAR10SP_dense_int3_attpool"}


def _zinc_shards(world=2):
    """[step][rank] padded ZINC shards of one capacity bucket."""
    from hlhgat.hodge_dataset import PackedGraphs
    from hlhgat.synthetic import zinc_like_graph
    per = 12
    ds = PackedGraphs([zinc_like_graph(900 + i) for i in range(STEPS * world * per)],
                      check_hodge=False)
    idx = [[np.arange((s * world + r) * per, (s * world + r + 1) * per) for r in range(world)]
           for s in range(STEPS)]
    cs = [ds.caps_for(i, 128) for row in idx for i in row]
    caps = {k: max(c[k] for c in cs) for k in cs[0]}
    return [[ds.collate(i, caps) for i in row] for row in idx]


def _head_shards(kind, world=2):
    """[step][rank] level-batch lists; two shapes per rank, alternating."""
    from hlhgat.synthetic import two_level_batch
    gen = "peptides" if kind.startswith("peptides") else kind
    base = [[two_level_batch(gen, 6, seed=40 + 2 * r + a) for r in range(world)]
            for a in range(2)]
    return [base[s % 2] for s in range(STEPS)]


def _loss(kind):
    F = torch.nn.functional
    if kind.startswith("zinc"):
        import hlhgat
        crit = hlhgat.nn.L1Loss()
        return lambda out, b: crit(out.view(-1, 1), b.y.view(-1, 1))
    if kind == "cifar":
        return lambda out, d: F.cross_entropy(out, d[0].y.view(-1).long())
    return lambda out, d: F.binary_cross_entropy_with_logits(out, d[0].y.view(out.shape).float())


def _model(kind, dev):
    import hlhgat
    torch.manual_seed(0)
    if kind.startswith("zinc"):
        return hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**ZKW).to(dev).train()
    return getattr(hlhgat, HEADCLS[kind])(**HEADKW[kind]).to(dev).train()


def _to(b, dev):
    return [x.to(dev) for x in b] if isinstance(b, list) else b.to(dev)


def _save_shards(shards, path):
    """[step][rank] batches (a Batch or a level list) as plain tensor dicts."""
    def one(b):
        # (clones: PackedGraphs.collate carves every tensor from one arena,
        # which torch.save refuses to store as differently typed views)
        d = {k: v.clone() for k, v in vars(b).items()
             if torch.is_tensor(v) and not k.startswith("_")}
        d["__meta"] = {"num_graphs": int(b.num_graphs), "hodge_sorted": dict(b.hodge_sorted),
                       "l1_factor": bool(getattr(b, "l1_factor", False)),
                       "num_nodes": int(getattr(b, "num_nodes", 0))}
        return d
    torch.save([[[one(x) for x in b] if isinstance(b, list) else one(b) for b in row]
                for row in shards], path)


def _load_shards(path):
    from hlhgat.hodge_dataset import Batch

    def one(d):
        b = Batch()
        meta = d.pop("__meta")
        for k, v in d.items():
            setattr(b, k, v)
        for k, v in meta.items():
            setattr(b, k, v)
        return b
    raw = torch.load(path, weights_only=True)
    return [[[one(x) for x in b] if isinstance(b, list) else one(b) for b in row] for row in raw]


def _rank_worker(rank, world, port, q, kind, path):
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=True)  # a stuck rank shows where
    _env(rank, world, port, share_gpu=True)
    from hlhgat.distributed import init_distributed
    from hlhgat.train import TrainStep
    r, w, dev = init_distributed()
    shards = _load_shards(path)  # the parent's exact inputs
    model = _model(kind, dev)
    # zinc_overlap: eager steps (gloo's exchange cannot be captured) with the
    # gradient all-reduce in small buckets issued from the backward's hooks
    kw = dict(graphs=False, overlap=True, bucket_mb=0.02) if kind.endswith("_overlap") else \
        dict(graphs=True)
    st = TrainStep(model, _loss(kind), lr=1e-3, weight_decay=1e-3, **kw)
    losses = []
    for s in range(STEPS):
        losses.append(float(st(_to(shards[s][r], dev))))
    torch.cuda.synchronize()
    q.put((r, dict(flat=st.flat.cpu().numpy(), stats=dict(st.stats), graphs=st.graphs,
                   graphs_off=st.graphs_off, losses=losses, overlap=st.overlap,
                   overlap_stats=dict(st.overlap_stats))))
    dist.destroy_process_group()


def _emulate(kind, cuda, shards, world=2):
    """One process: per step, each shard's gradient at the same parameters,
    (g_0 + g_1) / 2 as all_reduce(SUM) + div_(world) computes it, one Adam.
    CIFAR: hodge_st_model.global_max replaced by an emulation that takes the
    max over both shards and, in the backward, the upstream gradients of both
    shards and their tie counts summed -- what _GlobalMax's two all-reduces
    give every rank (a first pass records the maxima, a second the upstream
    gradients)."""
    from hlhgat import hodge_st_model as HM
    from hlhgat.train import TrainStep
    model = _model(kind, cuda)
    st = TrainStep(model, _loss(kind), lr=1e-3, weight_decay=1e-3, graphs=False)
    real_gm = HM.global_max
    try:
        for s in range(STEPS):
            data = [_to(shards[s][r], cuda) for r in range(world)]
            emu = None
            if kind == "cifar":
                emu = _EmuMaxState(world)
                HM.global_max = emu
                for phase in ("max", "upstream"):
                    for r in range(world):
                        emu.begin(phase, r)
                        if phase == "max":
                            with torch.no_grad():
                                model(data[r])
                        else:
                            st._fwd_bwd(data[r])
            grads = []
            for r in range(world):
                if emu is not None:
                    emu.begin("final", r)
                st._fwd_bwd(data[r])
                grads.append(st.flat_grad.clone())
            HM.global_max = real_gm
            st.flat_grad.copy_(grads[0] + grads[1]).div_(world)
            st._opt_step()
    finally:
        HM.global_max = real_gm
    torch.cuda.synchronize()
    return st.flat.cpu().numpy()


class _EmuMaxState:
    """Stand-in for distributed.global_max over `world` emulated ranks,
    called once per max site in forward order."""

    def __init__(self, world):
        self.world = world
        self.maxima = [[] for _ in range(world)]   # per rank, per site (forward order)
        self.ups = [{} for _ in range(world)]      # per rank: site -> upstream gradient
        self.hits = [{} for _ in range(world)]     # per rank: site -> tie count

    def begin(self, phase, rank):
        self.phase, self.rank, self.site = phase, rank, 0

    def __call__(self, x):
        i = self.site
        self.site += 1
        if self.phase == "max":
            self.maxima[self.rank].append(x.detach().max().reshape(1).clone())
            return x.max()
        m = self.maxima[0][i]
        for r in range(1, self.world):
            m = torch.maximum(m, self.maxima[r][i])
        return _EmuMax.apply(x, m, self, i)


class _EmuMax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, m, state, i):
        ctx.save_for_backward(x, m)
        ctx.state, ctx.i, ctx.rank, ctx.phase = state, i, state.rank, state.phase
        return m.reshape(())

    @staticmethod
    def backward(ctx, g):
        x, m = ctx.saved_tensors
        hit = (x == m).to(x.dtype)
        S = ctx.state
        if ctx.phase == "upstream":  # this rank's contribution only
            S.ups[ctx.rank][ctx.i] = g.reshape(()).to(x.dtype)
            S.hits[ctx.rank][ctx.i] = hit.sum()
            return torch.zeros_like(x), None, None, None
        # all_reduce(SUM) of [g_r, hits_r] over the ranks
        gs, hs = S.ups[0][ctx.i], S.hits[0][ctx.i]
        for r in range(1, S.world):
            gs = gs + S.ups[r][ctx.i]
            hs = hs + S.hits[r][ctx.i]
        return hit * (gs / hs), None, None, None


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["zinc", "peptides", "peptides_cfg4", "cifar", "zinc_overlap"])
def test_trainstep_two_ranks_bitwise_one_process(cuda, kind, tmp_path):
    shards = _zinc_shards(2) if kind.startswith("zinc") else _head_shards(kind, 2)
    path = str(tmp_path / "shards.pt")
    _save_shards(shards, path)
    res = _run_ranks(_rank_worker, 2, kind, path, timeout=200)
    for r in range(2):
        st = res[r]["stats"]
        if kind == "cifar":
            assert res[r]["graphs_off"] and st["eager"] == STEPS, st
        elif kind.endswith("_overlap"):
            assert res[r]["overlap"] and st["eager"] == STEPS, st
            assert res[r]["overlap_stats"]["in_backward"] >= 3 * STEPS, res[r]["overlap_stats"]
        else:
            assert res[r]["graphs"] and st["replay"] >= 2, st
    assert np.array_equal(res[0]["flat"], res[1]["flat"]), "ranks hold different parameters"
    want = _emulate(kind, cuda, _load_shards(path))
    diff = np.abs(res[0]["flat"] - want).max()
    assert np.array_equal(res[0]["flat"], want), f"{kind}: max |diff| {diff:.3e}"


def test_trainstep_refuses_ddp_wrapper():
    import socket
    from hlhgat.train import TrainStep
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        m = torch.nn.Linear(3, 2)
        ddp = torch.nn.parallel.DistributedDataParallel(m)
        with pytest.raises(ValueError, match="DistributedDataParallel"):
            TrainStep(ddp, lambda o, b: o.sum(), graphs=False)
    finally:
        dist.destroy_process_group()
