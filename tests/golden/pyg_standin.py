"""Minimal stand-in for the third-party packages the reference imports
(torch_geometric, torch_scatter, torch_cluster, torchmetrics), none of which is
installed here.  Used ONLY by make_golden.py, in this container, to import the
reference's own lib/*.py class bodies and run them on CPU.

It restates the documented semantics of the few symbols the hot path touches:
  * MessagePassing.propagate (flow source_to_target, aggr='add'):
      x_j = x.index_select(0, edge_index[0]); msg = self.message(x_j, norm);
      out = zeros(x.size(0), ...).scatter_add_(0, edge_index[1], msg)
  * torch_geometric.nn.dense.linear.Linear (weight [out, in], glorot init)
  * torch_geometric.nn.BatchNorm (BatchNorm1d held as .module)
  * torch_geometric.nn.Sequential (entries registered as module_{i})
  * torch_geometric.utils.degree / dense_to_sparse, global_mean_pool,
    torch_scatter.scatter_mean
  * torch_sparse.SparseTensor(row, col, value) with .t() / .coo(), and
    torch_sparse.matmul(A, x, reduce='add'): out[r] = sum over A's row-r
    entries in column order of value * x[col] (the DEMO fork only)
Everything else is an inert placeholder.  It is not PyG.
"""
from __future__ import annotations

import math
import re
import sys
import types

import torch
import torch.nn as nn
import torch.nn.functional as F


def _mod(name):
    m = types.ModuleType(name)
    sys.modules[name] = m
    return m


class _Placeholder:
    def __init__(self, *a, **k):
        raise RuntimeError("placeholder from the golden stand-in (not available)")


class MessagePassing(nn.Module):
    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2, **kwargs):
        super().__init__()
        assert aggr == "add" and flow == "source_to_target"
        self.aggr = aggr

    def propagate(self, edge_index, size=None, **kwargs):
        x = kwargs["x"]
        x_j = x.index_select(0, edge_index[0])
        msg = self.message(x_j, kwargs["norm"])
        out = torch.zeros((x.size(0),) + tuple(msg.shape[1:]), dtype=msg.dtype)
        idx = edge_index[1].view(-1, *([1] * (msg.dim() - 1))).expand_as(msg)
        return out.scatter_add_(0, idx, msg)


class PygLinear(nn.Module):
    def __init__(self, in_channels, out_channels, bias=True, weight_initializer=None,
                 bias_initializer=None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.weight_initializer = weight_initializer
        self.reset_parameters()

    def reset_parameters(self):
        if self.weight_initializer == "glorot":
            a = math.sqrt(6.0 / (self.weight.size(-2) + self.weight.size(-1)))
            with torch.no_grad():
                self.weight.uniform_(-a, a)
        else:
            nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)


class PygBatchNorm(nn.Module):
    def __init__(self, in_channels, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True):
        super().__init__()
        self.module = nn.BatchNorm1d(in_channels, eps, momentum, affine, track_running_stats)

    def forward(self, x):
        return self.module(x)


class PygSequential(nn.Module):
    def __init__(self, input_args, modules):
        super().__init__()
        self.inputs = [s.strip() for s in input_args.split(",")]
        self.routes = []
        for i, (fn, desc) in enumerate(modules):
            ins, outs = re.split(r"\s*->\s*", desc)
            self.routes.append(([s.strip() for s in ins.split(",")],
                                [s.strip() for s in outs.split(",")]))
            if isinstance(fn, nn.Module):
                self.add_module(f"module_{i}", fn)
            else:
                object.__setattr__(self, f"module_{i}", fn)

    def forward(self, *args):
        env = dict(zip(self.inputs, args))
        out = None
        for i, (ins, outs) in enumerate(self.routes):
            out = getattr(self, f"module_{i}")(*[env[n] for n in ins])
            if len(outs) == 1:
                env[outs[0]] = out
            else:
                env.update(zip(outs, out))
        return out


def degree(index, num_nodes=None, dtype=None):
    n = int(index.max()) + 1 if num_nodes is None else num_nodes
    out = torch.zeros(n, dtype=dtype or torch.get_default_dtype())
    return out.scatter_add_(0, index, torch.ones(index.size(0), dtype=out.dtype))


def dense_to_sparse(adj):
    idx = adj.nonzero().t()
    return idx, adj[idx[0], idx[1]]


def scatter_add(src, index, dim=0, dim_size=None):
    n = int(index.max()) + 1 if dim_size is None else dim_size
    out = torch.zeros((n,) + tuple(src.shape[1:]), dtype=src.dtype)
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return out.scatter_add_(0, idx, src)


def scatter_mean(src, index, dim=0, dim_size=None):
    index = index.view(-1)
    s = scatter_add(src, index, 0, dim_size)
    c = scatter_add(torch.ones(index.numel(), dtype=src.dtype), index, 0, s.size(0))
    return s / c.clamp(min=1).view(-1, *([1] * (src.dim() - 1)))


def global_mean_pool(x, batch, size=None):
    return scatter_mean(x, batch, 0, size)


class SparseTensor:
    def __init__(self, row=None, col=None, value=None, sparse_sizes=None, **kw):
        n = sparse_sizes or (int(row.max()) + 1, int(col.max()) + 1)
        key = row * max(int(n[1]), 1) + col  # row-major (CSR) order
        perm = torch.argsort(key, stable=True)
        self.row, self.col = row[perm], col[perm]
        self.value = value[perm] if value is not None else None
        self.sizes = (int(n[0]), int(n[1]))

    def t(self):
        return SparseTensor(row=self.col, col=self.row, value=self.value,
                            sparse_sizes=(self.sizes[1], self.sizes[0]))

    def coo(self):
        return self.row, self.col, self.value


def sparse_matmul(src, other, reduce="sum"):
    assert reduce in ("sum", "add")
    msg = other.index_select(0, src.col)
    if src.value is not None:
        msg = src.value.view(-1, *([1] * (other.dim() - 1))) * msg
    out = torch.zeros((src.sizes[0],) + tuple(other.shape[1:]), dtype=msg.dtype)
    return out.index_add_(0, src.row, msg)


def to_undirected(edge_index, edge_attr=None, num_nodes=None, reduce="add"):
    """torch_geometric.utils.to_undirected (documented semantics): both
    directions, coalesced (sorted by row * N + col), duplicate attributes
    reduced by `reduce`; returns (edge_index, edge_attr) when edge_attr is
    given, else edge_index."""
    n = int(edge_index.max()) + 1 if num_nodes is None else int(num_nodes)
    row = torch.cat([edge_index[0], edge_index[1]])
    col = torch.cat([edge_index[1], edge_index[0]])
    key = row * n + col
    uniq, inv = torch.unique(key, sorted=True, return_inverse=True)
    ei = torch.stack([uniq // n, uniq % n])
    if edge_attr is None:
        return ei
    a = torch.cat([edge_attr, edge_attr])
    out = torch.zeros((uniq.numel(),) + tuple(a.shape[1:]), dtype=a.dtype)
    if reduce == "min":
        out = out.fill_(float("inf")).scatter_reduce(0, inv, a, "amin", include_self=True)
    elif reduce == "mean":
        out = out.scatter_reduce(0, inv, a, "mean", include_self=False)
    else:
        out = out.index_add(0, inv, a)
    return ei, out


def install():
    tg = _mod("torch_geometric")
    tg.__path__ = []
    nnm = _mod("torch_geometric.nn")
    nnm.__path__ = []
    tg.nn = nnm
    conv = _mod("torch_geometric.nn.conv")
    conv.MessagePassing = MessagePassing
    dense = _mod("torch_geometric.nn.dense")
    dense.__path__ = []
    lin = _mod("torch_geometric.nn.dense.linear")
    lin.Linear = PygLinear
    inits = _mod("torch_geometric.nn.inits")
    inits.zeros = lambda t: t.data.zero_() if t is not None else None
    pool = _mod("torch_geometric.nn.pool")
    pool.graclus = pool.max_pool = _Placeholder
    nnm.Sequential = PygSequential
    nnm.BatchNorm = PygBatchNorm
    nnm.global_mean_pool = global_mean_pool
    nnm.global_max_pool = _Placeholder
    typing_ = _mod("torch_geometric.typing")
    typing_.OptTensor = object
    typing_.SparseTensor = SparseTensor
    tsp = _mod("torch_sparse")
    tsp.SparseTensor = SparseTensor
    tsp.matmul = sparse_matmul
    data = _mod("torch_geometric.data")

    class Data:
        def __init__(self, **kw):
            for k, v in kw.items():
                setattr(self, k, v)

        def __inc__(self, key, value, *args, **kwargs):
            return 0

    data.Data = Data
    data.Batch = data.Dataset = data.InMemoryDataset = Data
    data.download_url = data.extract_zip = _Placeholder
    tg.data = data
    ds = _mod("torch_geometric.datasets")
    ds.GNNBenchmarkDataset = ds.ZINC = _Placeholder
    loader = _mod("torch_geometric.loader")
    loader.DataLoader = _Placeholder
    utils = _mod("torch_geometric.utils")
    utils.__path__ = []
    utils.to_undirected = to_undirected
    for name in ("add_self_loops", "coalesce", "to_scipy_sparse_matrix",
                 "subgraph", "unbatch_edge_index", "softmax", "unbatch",
                 "remove_isolated_nodes"):
        setattr(utils, name, _Placeholder)
    utils.degree = degree
    utils.dense_to_sparse = dense_to_sparse
    tg.utils = utils
    nn_ = _mod("torch_geometric.utils.num_nodes")
    nn_.maybe_num_nodes = lambda ei, n=None: n if n is not None else int(ei.max()) + 1
    ts = _mod("torch_scatter")
    ts.scatter = _Placeholder
    ts.scatter_add = scatter_add
    ts.scatter_mean = scatter_mean
    ts.scatter_max = _Placeholder
    tc = _mod("torch_cluster")
    tc.graclus_cluster = _Placeholder
    tm = _mod("torchmetrics")
    tm.__path__ = []
    tm.F1Score = _Placeholder
    tmc = _mod("torchmetrics.classification")
    tmc.BinaryF1Score = _Placeholder
