"""SyncBatchNorm mode (hlhgat.distributed.convert_sync_batchnorm): batch
statistics over every rank's rows, so a batch sharded by graph normalises as
one process over the whole batch does (parity caveat 1).

CPU: the module conversion and the all-reduce (SUM) of the fp64 sums
(2 gloo ranks).  GPU: one rank is bitwise the plain HIP BatchNorm; two gloo
ranks sharing the card (HLHGAT_SHARE_GPU=1, the rehearsal mode of
hlhgat.distributed.init_distributed) equal one process over the concatenated
rows; the product ZINC model under DDP with SyncBatchNorm equals the
one-process model on the whole batch, and without it does not.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, close


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(target, world, *args, timeout=300):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, payload = q.get(timeout=timeout)
            res[r] = payload
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return res


def _env(rank, world, port, share_gpu=False):
    sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    if share_gpu:
        os.environ.update(HLHGAT_DIST_BACKEND="gloo", HLHGAT_SHARE_GPU="1")
    torch.set_num_threads(1)


# ---------------------------------------------------------------------------
# CPU
# ---------------------------------------------------------------------------
def test_convert_and_revert_mark_every_batchnorm():
    from hlhgat import ops
    from hlhgat.distributed import convert_sync_batchnorm, revert_sync_batchnorm
    from hlhgat.hodge_st_model import HL_HGCNN_zinc_dense_int3_pyr
    m = HL_HGCNN_zinc_dense_int3_pyr(channels=[1], filters=[16], mlp_channels=[8], K=2, keig=3)
    keys = set(m.state_dict())
    bns = [b for b in m.modules() if isinstance(b, torch.nn.BatchNorm1d)]
    assert len(bns) > 4
    convert_sync_batchnorm(m)
    assert all(ops.sync_bn_group(b) is not None for b in bns)
    assert set(m.state_dict()) == keys  # same modules, same checkpoint keys
    m.eval()  # running statistics: nothing to synchronise
    assert all(ops.sync_bn_group(b) is None for b in bns)
    m.train()
    revert_sync_batchnorm(m)
    assert all(ops.sync_bn_group(b) is None for b in bns)


def _sum_worker(rank, world, port, q):
    _env(rank, world, port)
    from hlhgat.ops import _sum_over_ranks
    dist.init_process_group("gloo")
    t = torch.arange(5, dtype=torch.float64) * (1.0 + rank) + 0.1 * rank
    g = _sum_over_ranks(t, None)
    q.put((rank, g.numpy()))
    dist.destroy_process_group()


def test_sum_over_ranks_gloo():
    """SyncBatchNorm's exchange: the fp64 sums of both ranks added, the same
    bits on every rank, one row (the apply kernels' gathered[1][2C+1])."""
    res = _run_ranks(_sum_worker, 2)
    want = (np.arange(5) * 1.0 + (np.arange(5) * 2.0 + 0.1)).reshape(1, -1)
    assert np.array_equal(res[0], res[1])
    assert res[0].shape == (1, 5) and np.allclose(res[0], want, rtol=0, atol=1e-12)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
def _bn_pair(C, seed=0):
    torch.manual_seed(seed)
    a = torch.nn.BatchNorm1d(C)
    with torch.no_grad():
        a.weight.uniform_(0.5, 1.5)
        a.bias.uniform_(-0.5, 0.5)
    b = torch.nn.BatchNorm1d(C)
    b.load_state_dict(a.state_dict())
    return a, b


@pytest.mark.gpu
@pytest.mark.parametrize("C,relu,pad", [(64, True, 0), (24, False, 0), (64, True, 37), (6, True, 0)])
def test_sync_bn_one_rank_bitwise(cuda, C, relu, pad):
    """One rank: the sync kernels give the plain HIP BatchNorm's bits (output,
    saved and running statistics, dx, dweight, dbias), padding rows too."""
    from hlhgat import ops
    from hlhgat.distributed import convert_sync_batchnorm
    n = 3001 + pad
    g = torch.Generator().manual_seed(C + pad)
    x = (torch.randn(n, C, generator=g) * 3 + 1).to(cuda)
    dy = torch.randn(n, C, generator=g).to(cuda)
    valid = torch.tensor([n - pad], dtype=torch.int32, device=cuda) if pad else None
    plain, sync = _bn_pair(C)
    plain, sync = plain.to(cuda), sync.to(cuda)
    convert_sync_batchnorm(sync)
    outs = []
    for bn in (plain, sync):
        xi = x.clone().requires_grad_(True)
        y = ops.batch_norm_act(xi, bn, relu=relu, valid=valid)
        y.backward(dy)
        outs.append((y.detach(), xi.grad, bn.weight.grad, bn.bias.grad, bn.running_mean.clone(),
                     bn.running_var.clone(), bn.num_batches_tracked.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _bn_rank_worker(rank, world, port, q, n, C, relu):
    _env(rank, world, port, share_gpu=True)
    from hlhgat import ops
    from hlhgat.distributed import convert_sync_batchnorm, init_distributed, shard_range
    r, w, dev = init_distributed()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, C, generator=g) * 2 + 0.5
    dy = torch.randn(n, C, generator=g)
    lo, hi = shard_range(n, r, w)
    bn, _ = _bn_pair(C)
    bn = convert_sync_batchnorm(bn.to(dev))
    xi = x[lo:hi].to(dev).requires_grad_(True)
    y = ops.batch_norm_act(xi, bn, relu=relu)
    y.backward(dy[lo:hi].to(dev))
    q.put((r, dict(y=y.detach().cpu().numpy(), dx=xi.grad.cpu().numpy(),
                   dw=bn.weight.grad.cpu().numpy(), db=bn.bias.grad.cpu().numpy(),
                   rm=bn.running_mean.cpu().numpy(), rv=bn.running_var.cpu().numpy())))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sync_bn_two_ranks_equal_one_process(cuda):
    """2 ranks x half the rows == one process over all rows (fp64 sums in a
    different order: 1e-6 / 1e-5 relative); each rank holds the same running
    statistics; local dweight / dbias sum to the full-batch ones."""
    from hlhgat import ops
    n, C, relu = 4099, 64, True
    res = _run_ranks(_bn_rank_worker, 2, n, C, relu)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, C, generator=g) * 2 + 0.5
    dy = torch.randn(n, C, generator=g)
    bn, _ = _bn_pair(C)
    bn = bn.to(cuda)
    xi = x.to(cuda).requires_grad_(True)
    y = ops.batch_norm_act(xi, bn, relu=relu)
    y.backward(dy.to(cuda))
    close(torch.from_numpy(np.concatenate([res[0]["y"], res[1]["y"]])), y.detach().cpu(), 1e-6,
          "sync bn y")
    close(torch.from_numpy(np.concatenate([res[0]["dx"], res[1]["dx"]])), xi.grad.cpu(), 1e-5,
          "sync bn dx")
    close(torch.from_numpy(res[0]["dw"] + res[1]["dw"]), bn.weight.grad.cpu(), 1e-5, "dweight")
    close(torch.from_numpy(res[0]["db"] + res[1]["db"]), bn.bias.grad.cpu(), 1e-5, "dbias")
    for k in ("rm", "rv"):
        assert np.array_equal(res[0][k], res[1][k])
    close(torch.from_numpy(res[0]["rm"]), bn.running_mean.cpu(), 1e-6, "running_mean")
    close(torch.from_numpy(res[0]["rv"]), bn.running_var.cpu(), 1e-6, "running_var")


ZKW = dict(channels=[1, 1], filters=[32, 32], mlp_channels=[32], K=3, keig=15)
N_GRAPHS = 24


def _zinc_graphs():
    from hlhgat.synthetic import zinc_like_graph
    return [zinc_like_graph(500 + i) for i in range(N_GRAPHS)]


def _zinc_step(model, batch):
    out = model(batch)
    loss = torch.nn.functional.l1_loss(out.view(-1), batch.y.view(-1))
    loss.backward()
    return out.detach()


def _zinc_rank_worker(rank, world, port, q, sync):
    import faulthandler
    faulthandler.dump_traceback_later(120, exit=True)  # a stuck rank shows where
    _env(rank, world, port, share_gpu=True)
    from hlhgat.distributed import (convert_sync_batchnorm, init_distributed, shard_graphs,
                                    wrap_ddp)
    from hlhgat.hodge_dataset import collate
    from hlhgat.hodge_st_model import HL_HGCNN_zinc_dense_int3_pyr
    r, w, dev = init_distributed()
    torch.manual_seed(0)
    model = HL_HGCNN_zinc_dense_int3_pyr(**ZKW).to(dev).train()
    if sync:
        convert_sync_batchnorm(model)
    ddp = wrap_ddp(model, dev)
    b = collate(shard_graphs(_zinc_graphs(), r, w)).to(dev)
    print(f"[rank {r}] sync={sync} forward+backward", file=sys.stderr, flush=True)
    out = _zinc_step(ddp, b)
    print(f"[rank {r}] done", file=sys.stderr, flush=True)
    grads = {k: p.grad.cpu().numpy() for k, p in model.named_parameters()}
    q.put((r, dict(out=out.cpu().numpy(), grads=grads)))
    dist.destroy_process_group()


def _bn_fed_bias(k):
    """biases whose output feeds a BatchNorm (conv / Linear before BN)"""
    import re
    return bool((re.search(r"module_[04]\.bias$", k) and not k.startswith("out."))
                or re.search(r"mlp\d+\.0\.bias$", k) or re.search(r"WV_(Node|Edge)\.[03]\.bias$", k))


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-12))


@pytest.mark.gpu
def test_zinc_ddp_sync_bn_equals_one_process(cuda):
    """The product ZINC model, 2 ranks x 12 graphs under DDP with
    SyncBatchNorm == one process on all 24 graphs: predictions to 1e-5 and
    every parameter gradient to 1e-4 (norm-wise; 1.5e-6 measured; the
    BN-fed biases, analytically zero, only bounded as noise);
    with per-rank statistics the predictions differ by far more."""
    from hlhgat.hodge_dataset import collate
    from hlhgat.hodge_st_model import HL_HGCNN_zinc_dense_int3_pyr
    torch.manual_seed(0)
    model = HL_HGCNN_zinc_dense_int3_pyr(**ZKW).to(cuda).train()
    b = collate(_zinc_graphs()).to(cuda)
    out = _zinc_step(model, b).cpu().numpy()
    ref = {k: p.grad.cpu().numpy() for k, p in model.named_parameters()}
    res = _run_ranks(_zinc_rank_worker, 2, True, timeout=150)
    got = np.concatenate([res[0]["out"], res[1]["out"]])
    assert _rel(got, out) < 1e-5, _rel(got, out)
    scale = max(float(np.abs(g).max()) for g in ref.values())
    for k in ref:
        if _bn_fed_bias(k):  # analytically zero (BN removes the shift): fp32 noise only
            assert float(np.abs(res[0]["grads"][k]).max()) < 1e-3 * scale, k
    worst = max((_rel(res[0]["grads"][k], ref[k]), k) for k in ref if not _bn_fed_bias(k))
    print("worst gradient rel err", worst)
    assert worst[0] < 1e-4, worst
    for k in ref:  # DDP: both ranks hold the same averaged gradient
        assert np.array_equal(res[0]["grads"][k], res[1]["grads"][k])
    res = _run_ranks(_zinc_rank_worker, 2, False, timeout=150)
    local = np.concatenate([res[0]["out"], res[1]["out"]])
    assert _rel(local, out) > 1e-3  # per-rank statistics: a different model output
