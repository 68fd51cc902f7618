"""ORACLE (test infrastructure only; never imported by the product).

PyTorch-CPU restatement of the HL-HGAT hot path, following the reference
(deepika090/HL-HGAT) operation by operation so the arithmetic order matches:

  propagate            PyG MessagePassing, message = norm*x_j, aggr='add'
                       (lib/Hodge_Cheb_Conv.py:442-443, 518-519, 455)
  laguerre_conv        lib/Hodge_Cheb_Conv.py:480-515
  laguerre_fast_conv_demo  HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:542-574 (bug kept)
  cheb_conv            lib/Hodge_Cheb_Conv.py:394-439
  adj2par1             lib/Hodge_Dataset.py:169-191
  node_edge_int        lib/Hodge_Cheb_Conv.py:293-309
  scatter_mean / global_mean_pool   torch_scatter / PyG semantics
  Ref* modules         same parameter names as the reference modules, so one
                       state_dict drives the oracle and the HIP product
  RefZincModel         lib/Hodge_ST_Model.py:544-646
"""
from __future__ import annotations

import math
import re
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import Dropout, Linear


# ----------------------------------------------------------------------------
# functional restatement
# ----------------------------------------------------------------------------
def propagate(x: torch.Tensor, edge_index: torch.Tensor,
              edge_weight: Optional[torch.Tensor]) -> torch.Tensor:
    """out[ei[1][e]] += w[e] * x[ei[0][e]] (source_to_target, dim_size = x.size(0))."""
    x_j = x.index_select(0, edge_index[0])
    msg = x_j if edge_weight is None else edge_weight.view(-1, 1) * x_j
    return torch.zeros_like(x).index_add_(0, edge_index[1], msg)


def laguerre_conv(x, edge_index, edge_weight, weights, bias):
    """lib/Hodge_Cheb_Conv.py:480-515 (2-D and 3-D x)."""
    K = len(weights)
    Tx_0 = x
    Tx_1 = x
    out = F.linear(Tx_0, weights[0])
    xshape = x.shape
    k = 1
    if K > 1:
        xv = x.reshape(xshape[0], -1)
        Tx_1 = xv - propagate(xv, edge_index, edge_weight)                # :494
        if len(xshape) >= 3:
            Tx_1 = Tx_1.view(xshape[0], xshape[1], -1)
        out = out + F.linear(Tx_1, weights[1])                            # :497
    for w in weights[2:]:
        inshape = Tx_1.shape
        Tx_1 = Tx_1.reshape(inshape[0], -1)
        Tx_2 = propagate(Tx_1, edge_index, edge_weight)                   # :502
        if len(xshape) >= 3:
            Tx_2 = Tx_2.view(inshape[0], inshape[1], -1)
            Tx_1 = Tx_1.view(xshape[0], xshape[1], -1)
        Tx_2 = (-Tx_2 + (2 * k + 1) * Tx_1 - k * Tx_0) / (k + 1)          # :507
        k += 1
        out = out + F.linear(Tx_2, w)                                     # :509
        Tx_0, Tx_1 = Tx_1, Tx_2
    if bias is not None:
        out = out + bias                                                  # :512-513
    return out


def laguerre_fast_conv_demo(x, edge_index, edge_weight, weights, bias):
    """HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:542-574 (HodgeLaguerreFastConv) AS
    PUBLISHED: the k >= 2 terms propagate the layer input x, not Tx_1 (:561).
    torch_sparse.matmul(adj_t, x, reduce='add') with adj_t = A^T of
    SparseTensor(row=ei[0], col=ei[1], value=w) (:179-180, :577-578) is the
    same sum as propagate."""
    K = len(weights)
    Tx_0 = x
    Tx_1 = x
    out = F.linear(Tx_0, weights[0])
    xshape = x.shape
    k = 1
    xv = x
    if K > 1:
        xv = x.reshape(xshape[0], -1)
        Tx_1 = xv - propagate(xv, edge_index, edge_weight)                # :554
        if len(xshape) >= 3:
            Tx_1 = Tx_1.view(xshape[0], xshape[1], -1)
        out = out + F.linear(Tx_1, weights[1])
    for w in weights[2:]:
        inshape = Tx_1.shape
        Tx_1 = Tx_1.reshape(inshape[0], -1)
        Tx_2 = propagate(xv, edge_index, edge_weight)                     # :561 (x, not Tx_1)
        if len(xshape) >= 3:
            Tx_2 = Tx_2.view(inshape[0], inshape[1], -1)
            Tx_1 = Tx_1.view(xshape[0], xshape[1], -1)
        Tx_2 = (-Tx_2 + (2 * k + 1) * Tx_1 - k * Tx_0) / (k + 1)          # :566
        k += 1
        out = out + F.linear(Tx_2, w)
        Tx_0, Tx_1 = Tx_1, Tx_2
    if bias is not None:
        out = out + bias
    return out


def cheb_conv(x, edge_index, edge_weight, weights, bias):
    """lib/Hodge_Cheb_Conv.py:394-439 (2-D x; the 3-D path only permutes
    features inside each propagated row)."""
    Tx_0 = x
    Tx_1 = x
    out = F.linear(Tx_0, weights[0])
    if len(weights) > 1:
        Tx_1 = propagate(x, edge_index, edge_weight)                      # :416
        out = out + F.linear(Tx_1, weights[1])
    for w in weights[2:]:
        Tx_2 = propagate(Tx_1, edge_index, edge_weight)                   # :430
        Tx_2 = 2. * Tx_2 - Tx_0                                           # :432
        out = out + F.linear(Tx_2, w)
        Tx_0, Tx_1 = Tx_1, Tx_2
    if bias is not None:
        out = out + bias
    return out


def adj2par1(edge_index, num_node, num_edge):
    """lib/Hodge_Dataset.py:169-191 (uncoalesced torch sparse COO B1)."""
    E = edge_index.shape[1]
    col_idx = torch.cat([torch.arange(E), torch.arange(E)], dim=-1)
    row_idx = torch.cat([edge_index[0], edge_index[1]], dim=-1)
    val = torch.cat([edge_index[0].new_full(edge_index[0].shape, -1),
                     edge_index[0].new_full(edge_index[0].shape, 1)], dim=-1).to(torch.float)
    return torch.sparse_coo_tensor(torch.cat([row_idx, col_idx], dim=-1).view(2, -1), val,
                                   torch.Size([num_node, num_edge]))


def degree(index, num_nodes=None):
    n = int(index.max()) + 1 if num_nodes is None else num_nodes
    out = torch.zeros(n)
    return out.scatter_add_(0, index, torch.ones(index.numel()))


def boundary_mix(x_t, x_s, par, D):
    """x_s2t, x_t2s of lib/Hodge_Cheb_Conv.py:294-295."""
    par = par if par.dtype == x_s.dtype else par.to(x_s.dtype)  # (fp64 noise studies)
    x_s2t = (1 / D).view(-1, 1) * torch.sparse.mm(par.abs(), x_s)
    x_t2s = torch.sparse.mm(par.abs().transpose(0, 1), x_t) / 2
    return x_s2t, x_t2s


def att_score(q_cross, q_self, k, lam, dk, sigma):
    """lib/Hodge_Cheb_Conv.py:299-304 for one side."""
    return sigma(((1 - lam) * (q_cross * k).sum(dim=1, keepdim=True)
                  + lam * (q_self * k).sum(dim=1, keepdim=True)) / np.sqrt(dk))


def scatter_mean(x, index, dim_size=None):
    """torch_scatter.scatter_mean(x, index, dim=0): sum / clamp(count, 1)."""
    index = index.view(-1).to(torch.long)
    n = int(index.max()) + 1 if dim_size is None else dim_size
    s = torch.zeros(n, x.size(1), dtype=x.dtype).index_add_(0, index, x)
    c = torch.zeros(n, dtype=x.dtype).index_add_(0, index, torch.ones(index.numel(), dtype=x.dtype))
    return s / c.clamp(min=1).view(-1, 1)


def global_mean_pool(x, batch):
    return scatter_mean(x, batch)


# ----------------------------------------------------------------------------
# reference-named modules (state_dict compatible with the product modules)
# ----------------------------------------------------------------------------
def glorot(t):
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class RefPygLinear(nn.Module):
    """torch_geometric Linear(bias=False, weight_initializer='glorot')."""

    def __init__(self, cin, cout):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cout, cin))
        glorot(self.weight)

    def forward(self, x):
        return F.linear(x, self.weight)


class RefHodgeConv(nn.Module):
    def __init__(self, cin, cout, K, bias=True, kind="laguerre"):
        super().__init__()
        assert K > 0
        self.kind = kind
        self.lins = nn.ModuleList([RefPygLinear(cin, cout) for _ in range(K)])
        if bias:
            self.bias = nn.Parameter(torch.zeros(cout))
        else:
            self.register_parameter("bias", None)

    def forward(self, x, edge_index, edge_weight=None, batch=None):
        fn = laguerre_conv if self.kind == "laguerre" else cheb_conv
        return fn(x, edge_index, edge_weight, [l.weight for l in self.lins], self.bias)


class RefBatchNorm(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.module = nn.BatchNorm1d(c)

    def forward(self, x):
        return self.module(x)


class RefSequential(nn.Module):
    """torch_geometric.nn.Sequential routing; entry i is module_{i}."""

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


class RefNodeEdgeInt(nn.Module):
    """lib/Hodge_Cheb_Conv.py:255-309."""

    def __init__(self, d=64, dk=32, dv=64, dl=64, only_att=False, sigma=nn.Sigmoid(), l=0.9):
        super().__init__()
        dl = dv
        self.sigma = sigma
        self.dk = dk
        self.only_att = only_att
        if only_att:
            self.WQ_Node = nn.Linear(d, dk)
            self.WK_Node = nn.Linear(d, dk)
            self.WQ_Edge = nn.Linear(d, dk)
            self.WK_Edge = nn.Linear(d, dk)
        else:
            self.WV_Node = nn.Sequential(nn.Linear(d * 2, dl), nn.BatchNorm1d(dl), nn.ReLU(),
                                         nn.Linear(dl, dv), nn.BatchNorm1d(dv), nn.ReLU())
            self.WV_Edge = nn.Sequential(nn.Linear(d * 2, dl), nn.BatchNorm1d(dl), nn.ReLU(),
                                         nn.Linear(dl, dv), nn.BatchNorm1d(dv), nn.ReLU())
        self.lambda_Node = l
        self.lambda_Edge = l

    def forward(self, x_t, x_s, par, D):
        x_s2t, x_t2s = boundary_mix(x_t, x_s, par, D)
        if self.only_att:
            a_t = att_score(self.WQ_Edge(x_s2t), self.WQ_Node(x_t), self.WK_Node(x_t),
                            self.lambda_Node, self.dk, self.sigma)
            a_s = att_score(self.WQ_Node(x_t2s), self.WQ_Edge(x_s), self.WK_Edge(x_s),
                            self.lambda_Edge, self.dk, self.sigma)
            return a_t, a_s
        x_t1 = self.WV_Node(torch.cat([x_s2t, x_t], dim=-1))
        x_s1 = self.WV_Edge(torch.cat([x_t2s, x_s], dim=-1))
        return x_t1, x_s1


def _ref_block(cin_t, cin_s, cout, K, dropout_ratio=0.0):
    layers = [(RefHodgeConv(cin_t, cout, K), "x_t, edge_index_t, edge_weight_t -> x_t"),
              (RefBatchNorm(cout), "x_t -> x_t"),
              (nn.ReLU(), "x_t -> x_t"),
              (Dropout(p=dropout_ratio), "x_t -> x_t"),
              (RefHodgeConv(cin_s, cout, K), "x_s, edge_index_s, edge_weight_s -> x_s"),
              (RefBatchNorm(cout), "x_s -> x_s"),
              (nn.ReLU(), "x_s -> x_s"),
              (Dropout(p=dropout_ratio), "x_s -> x_s"),
              (lambda x1, x2: [x1, x2], "x_t, x_s -> x")]
    return RefSequential("x_t, edge_index_t, edge_weight_t, x_s, edge_index_s, edge_weight_s",
                         layers)


class RefZincModel(nn.Module):
    """lib/Hodge_ST_Model.py:544-646 (HL_HGCNN_zinc_dense_int3_pyr)."""

    def __init__(self, channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[], K=2,
                 node_dim=21, edge_dim=3, num_classes=1, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, keig=7):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        node_dim = node_dim + keig
        edge_dim = edge_dim + keig
        c0 = filters[0]
        self.HL_init_conv = _ref_block(node_dim, edge_dim, c0, K, dropout_ratio)
        gin = c0
        for i, gout in enumerate(filters):
            for j in range(channels[i]):
                setattr(self, f"NEInt{i}{j}", RefNodeEdgeInt(d=gin, dv=gout))
                setattr(self, f"NEConv{i}{j}", _ref_block(gout, gout, gout, K, dropout_ratio))
                gin = gout + gin
        mlp_in = filters[-1] * 2
        for i, mo in enumerate(mlp_channels):
            setattr(self, f"mlp{i}", nn.Sequential(Linear(mlp_in, mo), nn.BatchNorm1d(mo),
                                                   nn.ReLU(), nn.Dropout(dropout_ratio_mlp)))
            mlp_in = mo
        self.out = Linear(mlp_in, num_classes)

    def forward(self, data):
        n_batch = torch.cat([torch.tensor([i] * int(nn_)) for i, nn_ in enumerate(data.num_node1)])
        s_batch = torch.cat([torch.tensor([i] * int(nn_)) for i, nn_ in enumerate(data.num_edge1)])
        x_t, x_s = self.HL_init_conv(data.x_t, data.edge_index_t, data.edge_weight_t,
                                     data.x_s, data.edge_index_s, data.edge_weight_s)
        x_s0, x_t0 = x_s, x_t
        for i, _ in enumerate(self.channels):
            par_1 = adj2par1(data.edge_index, x_t.shape[0], x_s.shape[0])
            D = degree(data.edge_index.reshape(-1))
            for j in range(self.channels[i]):
                x_t, x_s = getattr(self, f"NEInt{i}{j}")(x_t0, x_s0, par_1, D)
                x_t, x_s = getattr(self, f"NEConv{i}{j}")(
                    x_t, data.edge_index_t, data.edge_weight_t, x_s, data.edge_index_s,
                    data.edge_weight_s)
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
        x = torch.cat((global_mean_pool(x_s, s_batch), global_mean_pool(x_t, n_batch)), -1)
        for i, _ in enumerate(self.mlp_channels):
            x = getattr(self, f"mlp{i}")(x)
        return self.out(x)
