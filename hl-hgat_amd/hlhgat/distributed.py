"""Data parallelism for HL-HGAT: shard batches BY GRAPH, all-reduce gradients.

The reference is single-device ('cuda:0' hard-coded).
Simplex graphs are independent units (block-diagonal L0 / L1 / B1,
lib/Hodge_Dataset.py:40-48), so each rank owns whole graphs and the only
exchange step is the per-step gradient all-reduce (torch DDP over RCCL /
xGMI; backend "nccl" is RCCL on ROCm).  One graph never spans GPUs.

BatchNorm statistics stay per rank by default (like the reference's per-batch
statistics, computed on each rank's shard); convert_sync_batchnorm turns on
SyncBatchNorm mode, whose statistics span every rank (parity
caveat 1).
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

__all__ = ["world_info", "shard_range", "shard_graphs", "shard_by_weight", "init_distributed",
           "wrap_ddp", "max_over_ranks", "convert_sync_batchnorm", "revert_sync_batchnorm"]


def world_info() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) share of n items (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_graphs(graphs: Sequence, rank: int, world: int) -> List:
    lo, hi = shard_range(len(graphs), rank, world)
    return list(graphs[lo:hi])


def shard_by_weight(weights: Sequence[float], world: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment of items (e.g. graphs by
    nnz(L1), for the TSP config where graph sizes differ) to ranks."""
    order = sorted(range(len(weights)), key=lambda i: -weights[i])
    loads = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda j: (loads[j], j))
        out[r].append(i)
        loads[r] += weights[i]
    return [sorted(o) for o in out]


def init_distributed(backend: str = None) -> Tuple[int, int, torch.device]:
    """Initialise the process group (RCCL on GPU, gloo on CPU); one process
    per GPU.  Returns (rank, world, device)."""
    rank, world, local = world_info()
    # Rehearsal of the multi-rank path on a one-GPU box: HLHGAT_DIST_BACKEND=gloo
    # with HLHGAT_SHARE_GPU=1 puts every rank on cuda:0 and exchanges through
    # gloo (RCCL refuses two ranks on one device).  Production: nccl = RCCL.
    backend = os.environ.get("HLHGAT_DIST_BACKEND", backend)
    share = os.environ.get("HLHGAT_SHARE_GPU", "0") == "1"
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    elif share:
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, device


def wrap_ddp(model: torch.nn.Module, device: torch.device, bucket_cap_mb: int = 32,
             find_unused_parameters: bool = None):
    """DistributedDataParallel with one gradient bucket per ~32 MB: the whole
    0.6-16 MB gradient of the SURVEY configs fits in one or two ring
    all-reduces over the 7 xGMI links.  find_unused_parameters defaults to the
    model's ``ddp_find_unused_parameters`` flag (the attpool heads, whose
    unused NEAtt parameters would otherwise keep the bucket from ever being
    reduced, leaving every gradient pre-scaled by 1/W and un-summed)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return model
    if find_unused_parameters is None:
        find_unused_parameters = bool(getattr(model, "ddp_find_unused_parameters", False))
    ids = [device.index] if device.type == "cuda" else None
    return torch.nn.parallel.DistributedDataParallel(
        model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
        find_unused_parameters=find_unused_parameters)


def convert_sync_batchnorm(module: torch.nn.Module, process_group=None) -> torch.nn.Module:
    """SyncBatchNorm mode for every BatchNorm1d of ``module`` (the role of
    torch.nn.SyncBatchNorm.convert_sync_batchnorm): in training their batch
    statistics (and the input gradient's sums) span all ranks of
    ``process_group`` (None = the default group), so a model sharded by graph
    normalises exactly as one process over the whole batch does.  The
    modules stay BatchNorm1d (state_dict keys unchanged); the HIP kernels
    exchange one fp64 [2C+1] vector per layer and direction
    (include/hlhgat.h, hlhgat_bn_sums_*).  Returns ``module``."""
    from .ops import _SyncGroup
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm1d):
            m._hlhgat_sync = _SyncGroup(process_group)
    return module


def revert_sync_batchnorm(module: torch.nn.Module) -> torch.nn.Module:
    """Back to per-rank statistics (the default)."""
    for m in module.modules():
        if isinstance(m, torch.nn.BatchNorm1d) and hasattr(m, "_hlhgat_sync"):
            del m._hlhgat_sync
    return module


# Tests: run the collectives of a one-rank group too (RCCL on a world-size-1
# nccl group on a one-GPU box), so the captured-collective paths execute
COLLECTIVES_AT_WORLD_1 = False


def collectives_on(group=None) -> bool:
    """True when the data-parallel collectives run: an initialised process
    group of more than one rank (or of one, with COLLECTIVES_AT_WORLD_1)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or COLLECTIVES_AT_WORLD_1


def max_over_ranks(value: float, device: torch.device = torch.device("cpu")) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class _GlobalMax(torch.autograd.Function):
    """max over all elements on all ranks (all_reduce MAX; no host sync).
    Backward is the adjoint of that exchange: the data-parallel objective is
    (1/W)·Σ_r L_r and every L_r depends on the one global max, so dΣL/dM =
    Σ_r g_r is summed over ranks (one all_reduce with the tie count) and lands
    on the positions holding the max (torch.max's subgradient, ties split
    evenly); DDP's 1/W average then gives d/dθ of the global-batch loss."""

    @staticmethod
    def forward(ctx, x):
        m = x.max().reshape(1).clone()
        if collectives_on():
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
        ctx.save_for_backward(x, m)
        return m.reshape(())

    @staticmethod
    def backward(ctx, g):
        x, m = ctx.saved_tensors
        hit = (x == m).to(x.dtype)
        gc = torch.stack([g.reshape(()).to(x.dtype), hit.sum()])
        if collectives_on():
            dist.all_reduce(gc)
        return hit * (gc[0] / gc[1])


def global_max(x: torch.Tensor) -> torch.Tensor:
    """x.max() over the whole data-parallel batch: the attpool heads divide
    the attention by its batch max (lib/Hodge_ST_Model.py:1061-1062), which
    under graph sharding must span every rank's graphs to equal the
    single-process result (parity caveat 2).  One process: x.max()."""
    if not collectives_on():
        return x.max()
    return _GlobalMax.apply(x)

