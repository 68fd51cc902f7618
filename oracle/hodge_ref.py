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
  RefTSPModel          lib/Hodge_ST_Model.py:756-855 (config 5 head)
  RefCifarAttPool      lib/Hodge_ST_Model.py:958-1091 (config 3 head)
  RefPepfuncAttPool    main_pepfunc_HL_HGCNN_dense_int3_attpool.py:36-168 (config 4)
  RefHLFilter          lib/Hodge_Cheb_Conv.py:117-188
  RefSAPool            lib/Hodge_Cheb_Conv.py:36-59
  graclus              torch_cluster 1.6.0 graclus_cluster (absent; parity
                       unpinned), called at lib/Hodge_Dataset.py:252, :311
  mlgc_map             lib/Hodge_Dataset.py:254-275 (MLGC's per-edge loop)
  to_undirected_mean   PyG to_undirected(reduce='mean'), lib/Hodge_Dataset.py:310
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


def _prop_ntc(x, edge_index, edge_weight):
    """The 3-D branch of lib/Hodge_Cheb_Conv.py:409-414 / :421-425: [N, T, C]
    transposed to [N, C, T], flattened per row, propagated, and back.  (The
    reference flattens with .view(), which raises unless T == 1 or C == 1;
    .reshape() gives the same rows wherever .view() succeeds.)"""
    if x.dim() != 3:
        return propagate(x, edge_index, edge_weight)
    n, t, c = x.shape
    y = propagate(x.transpose(1, 2).reshape(n, -1), edge_index, edge_weight)
    return y.view(n, c, -1).transpose(1, 2)


def cheb_conv(x, edge_index, edge_weight, weights, bias):
    """lib/Hodge_Cheb_Conv.py:394-439 (2-D and 3-D x)."""
    Tx_0 = x
    Tx_1 = x
    out = F.linear(Tx_0, weights[0])
    if len(weights) > 1:
        Tx_1 = _prop_ntc(x, edge_index, edge_weight)                      # :409-416
        out = out + F.linear(Tx_1, weights[1])
    for w in weights[2:]:
        Tx_2 = _prop_ntc(Tx_1, edge_index, edge_weight)                   # :421-430
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


def _ref_block(cin_t, cin_s, cout, K, dropout_ratio=0.0, act=nn.ReLU):
    layers = [(RefHodgeConv(cin_t, cout, K), "x_t, edge_index_t, edge_weight_t -> x_t"),
              (RefBatchNorm(cout), "x_t -> x_t"),
              (act(), "x_t -> x_t"),
              (Dropout(p=dropout_ratio), "x_t -> x_t"),
              (RefHodgeConv(cin_s, cout, K), "x_s, edge_index_s, edge_weight_s -> x_s"),
              (RefBatchNorm(cout), "x_s -> x_s"),
              (act(), "x_s -> x_s"),
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


def _batch_vec(counts):
    """torch.cat([torch.tensor([i] * n) for i, n in enumerate(counts)])
    (lib/Hodge_ST_Model.py:824-828, :1031-1034)."""
    return torch.cat([torch.full((int(c),), i, dtype=torch.long) for i, c in enumerate(counts)])


class Abs(nn.Module):
    """x.abs() as a module: the readout's |B1^T x_t| (:848), replaceable by a
    frozen-sign multiplication in the gradient gates (like nn.ReLU's masks)."""

    def forward(self, x):
        return x.abs()


class RefTSPModel(nn.Module):
    """lib/Hodge_ST_Model.py:756-855 (HL_HGCNN_TSP_dense_int3_pyr): no keig
    columns (:764-765), edge mask in x_s[:, 1:], readout |B1^T x_t| / 2 (:848),
    K=1 conv MLP and output conv over L1; returns (logits * mask, s_batch)."""

    def __init__(self, channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[], K=2,
                 node_dim=2, edge_dim=1, num_classes=1, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, keig=20):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        c0 = filters[0]
        self.HL_init_conv = _ref_block(node_dim, edge_dim, c0, K, dropout_ratio)
        gin = c0
        for i, gout in enumerate(filters):
            for j in range(channels[i]):
                setattr(self, f"NEInt{i}{j}", RefNodeEdgeInt(d=gin, dv=gout))
                setattr(self, f"NEConv{i}{j}", _ref_block(gout, gout, gout, K, dropout_ratio))
                gin = gout + gin
        mlp_in = gout * 2                                                      # :806
        if len(mlp_channels) == 1:                                             # :807-815
            self.mlp = RefSequential("x_t, edge_index_t, edge_weight_t", [
                (RefHodgeConv(mlp_in, mlp_channels[0], 1),
                 "x_t, edge_index_t, edge_weight_t -> x_t"),
                (RefBatchNorm(mlp_channels[0]), "x_t -> x_t"),
                (nn.ReLU(), "x_t -> x_t"),
                (Dropout(p=dropout_ratio), "x_t -> x_t")])
            mlp_in = mlp_channels[0]
        self.out = RefSequential("x_t, edge_index_t, edge_weight_t", [
            (RefHodgeConv(mlp_in, num_classes, 1), "x_t, edge_index_t, edge_weight_t -> x_t")])
        self.readout_abs = Abs()

    def forward(self, data):
        s_batch = _batch_vec(data.num_edge1)
        x_s, ei_s, ew_s = data.x_s[:, :1], data.edge_index_s, data.edge_weight_s  # :829
        edge_mask = data.x_s[:, 1:]
        x_t, ei_t, ew_t = data.x_t, data.edge_index_t, data.edge_weight_t
        x_t, x_s = self.HL_init_conv(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
        x_s0, x_t0 = x_s, x_t
        par_1 = adj2par1(data.edge_index, x_t.shape[0], x_s.shape[0])            # :835
        D = degree(data.edge_index.reshape(-1), num_nodes=x_t.shape[0]) + 1e-6    # :836
        for i, _ in enumerate(self.channels):
            for j in range(self.channels[i]):
                x_t, x_s = getattr(self, f"NEInt{i}{j}")(x_t0, x_s0, par_1, D)
                x_t, x_s = getattr(self, f"NEConv{i}{j}")(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
        par_x = par_1 if par_1.dtype == x_t.dtype else par_1.to(x_t.dtype)  # (fp64 studies)
        x_t2s = self.readout_abs(torch.sparse.mm(par_x.transpose(0, 1), x_t)) / 2  # :848
        x_s = torch.cat([x_s, x_t2s], dim=-1)
        if len(self.mlp_channels) == 1:
            x_s = self.mlp(x_s, ei_s, ew_s)
        return self.out(x_s, ei_s, ew_s) * edge_mask, s_batch


def _pos(datas, device=None):
    """pos_ts / pos_ss of the attpool heads (lib/Hodge_ST_Model.py:1029-1038):
    fine row -> global coarse index (float; inf for an edge MLGC dropped)."""
    n_batch = _batch_vec(datas[0].num_node1)
    s_batch = _batch_vec(datas[0].num_edge1)
    n_ahead = torch.cumsum(torch.cat([torch.zeros(1), torch.as_tensor(datas[1].num_node1,
                                                                      dtype=torch.float)]),
                           dim=0, dtype=torch.long)[:-1]
    s_ahead = torch.cumsum(torch.cat([torch.zeros(1), torch.as_tensor(datas[1].num_edge1,
                                                                      dtype=torch.float)]),
                           dim=0, dtype=torch.long)[:-1]
    pos_t = (datas[0].x_t[:, 0] + n_ahead[n_batch]).view(-1, 1)
    pos_s = (datas[0].x_s[:, 0] + s_ahead[s_batch]).view(-1, 1)
    return [pos_t], [pos_s]


def _pool(x_t0, x_s0, pos_t, pos_s):
    """structural pooling (lib/Hodge_ST_Model.py:1065-1069): scatter_mean by
    cluster, edges assigned inf dropped first."""
    x_t0 = scatter_mean(x_t0, pos_t.to(torch.long))
    keep = ~torch.isinf(pos_s).view(-1)
    x_s0 = scatter_mean(x_s0[keep], pos_s[keep].to(torch.long))
    return x_t0, x_s0


class _RefAttPool(nn.Module):
    """Shared constructor of the two attention-pooling heads."""

    def __init__(self, channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                 dropout_ratio, dropout_ratio_mlp, pool_loc, keig, l, every_level):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        self.pool_loc = pool_loc
        c0 = filters[0]
        self.HL_init_conv = _ref_block(node_dim + keig, edge_dim + keig, c0, 1, dropout_ratio)
        gin = c0
        for i, gout in enumerate(filters):
            for j in range(channels[i]):
                setattr(self, f"NEInt{i}{j}", RefNodeEdgeInt(d=gin, dv=gout))
                setattr(self, f"NEConv{i}{j}", _ref_block(gout, gout, gout, K, dropout_ratio))
                gin = gin + gout
            if every_level:   # main_pepfunc...:86-87
                setattr(self, f"NEAtt{i}", RefNodeEdgeInt(d=gin, dv=gout, only_att=True, l=0.5))
            elif i == pool_loc:  # lib/Hodge_ST_Model.py:1007-1010
                setattr(self, f"NEAtt{i}", RefNodeEdgeInt(d=gout, dv=gout, only_att=True,
                                                          sigma=nn.ReLU(), l=l))
        mlp_in = filters[-1] * 2
        for i, mo in enumerate(mlp_channels):
            setattr(self, f"mlp{i}", nn.Sequential(Linear(mlp_in, mo), nn.BatchNorm1d(mo),
                                                   nn.ReLU(), nn.Dropout(dropout_ratio_mlp)))
            mlp_in = mo
        self.out = Linear(mlp_in, num_classes)

    def _readout(self, x_s, x_t, datas, i):
        d = datas[min(i, 1)]                                                   # :1077-1081
        x = torch.cat((global_mean_pool(x_s, _batch_vec(d.num_edge1)),
                       global_mean_pool(x_t, _batch_vec(d.num_node1))), -1)
        for m in range(len(self.mlp_channels)):
            x = getattr(self, f"mlp{m}")(x)
        return self.out(x)


class RefCifarAttPool(_RefAttPool):
    """lib/Hodge_ST_Model.py:958-1091 (HL_HGCNN_CIFAR10SP_dense_int3_attpool)."""

    def __init__(self, channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[], K=2,
                 node_dim=5, l=0.5, edge_dim=4, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, pool_loc=0, keig=10):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, pool_loc, keig, l, False)

    def forward(self, datas):
        data = datas[0]
        pos_ts, pos_ss = _pos(datas)
        x_s, ei_s, ew_s = data.x_s[:, 1:], data.edge_index_s, data.edge_weight_s
        x_t, ei_t, ew_t = data.x_t[:, 1:], data.edge_index_t, data.edge_weight_t
        x_t, x_s = self.HL_init_conv(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
        x_s0, x_t0 = x_s, x_t
        k = 0
        par_1 = adj2par1(datas[k].edge_index, x_t0.shape[0], x_s0.shape[0])
        D = degree(datas[k].edge_index.reshape(-1), num_nodes=x_t0.shape[0]) + 1e-6
        for i, _ in enumerate(self.channels):
            for j in range(self.channels[i]):
                x_t, x_s = getattr(self, f"NEInt{i}{j}")(x_t0, x_s0, par_1, D)
                x_t, x_s = getattr(self, f"NEConv{i}{j}")(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
            if i == self.pool_loc:                                             # :1058-1074
                att_t, att_s = getattr(self, f"NEAtt{i}")(x_t, x_s, par_1, D)
                att_t = att_t / att_t.max()
                att_s = att_s / att_s.max()
                x_t = x_t * att_t
                x_s = x_s * att_s
                x_t0, x_s0 = _pool(x_t0, x_s0, pos_ts[k], pos_ss[k])
                ei_s, ew_s = datas[k + 1].edge_index_s, datas[k + 1].edge_weight_s
                ei_t, ew_t = datas[k + 1].edge_index_t, datas[k + 1].edge_weight_t
                k = 1
                par_1 = adj2par1(datas[k].edge_index, x_t0.shape[0], x_s0.shape[0])
                D = degree(datas[k].edge_index.reshape(-1), num_nodes=x_t0.shape[0]) + 1e-6
        return self._readout(x_s, x_t, datas, i)


class RefPepfuncAttPool(_RefAttPool):
    """main_pepfunc_HL_HGCNN_dense_int3_attpool.py:36-168: NEAtt (sigmoid,
    l = 0.5) on the dense concatenation after every level (:133-136)."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=9, edge_dim=3, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, pool_loc=0, keig=20):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, pool_loc, keig, 0.5, True)

    def forward(self, datas):
        data = datas[0]
        pos_ts, pos_ss = _pos(datas)
        x_s, ei_s, ew_s = data.x_s[:, 1:], data.edge_index_s, data.edge_weight_s
        x_t, ei_t, ew_t = data.x_t[:, 1:], data.edge_index_t, data.edge_weight_t
        x_t, x_s = self.HL_init_conv(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
        x_s0, x_t0 = x_s, x_t
        k = 0
        par_1 = adj2par1(datas[k].edge_index, x_t0.shape[0], x_s0.shape[0])
        D = degree(datas[k].edge_index.reshape(-1), num_nodes=x_t0.shape[0]) + 1e-6
        for i, _ in enumerate(self.channels):
            for j in range(self.channels[i]):
                x_t, x_s = getattr(self, f"NEInt{i}{j}")(x_t0, x_s0, par_1, D)
                x_t, x_s = getattr(self, f"NEConv{i}{j}")(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
            att_t, att_s = getattr(self, f"NEAtt{i}")(x_t0, x_s0, par_1, D)     # :133-136
            x_t0 = x_t0 * att_t
            x_s0 = x_s0 * att_s
            if i == self.pool_loc:                                             # :139-149
                x_t0, x_s0 = _pool(x_t0, x_s0, pos_ts[k], pos_ss[k])
                ei_s, ew_s = datas[k + 1].edge_index_s, datas[k + 1].edge_weight_s
                ei_t, ew_t = datas[k + 1].edge_index_t, datas[k + 1].edge_weight_t
                k = 1
                par_1 = adj2par1(datas[k].edge_index, x_t0.shape[0], x_s0.shape[0])
                D = degree(datas[k].edge_index.reshape(-1), num_nodes=x_t0.shape[0]) + 1e-6
        return self._readout(x_s, x_t, datas, i)


class RefHLFilter(nn.Module):
    """lib/Hodge_Cheb_Conv.py:117-188 (HL_filter): MSI + HL block per channel
    with dense concatenation (if_dense) or plain stacking; LeakyReLU."""

    def __init__(self, channels=2, filters=32, K=4, node_dim=64, edge_dim=64,
                 dropout_ratio=0.0, leaky_slope=0.1, if_dense=True):
        super().__init__()
        self.channels = channels
        self.if_dense = if_dense
        t_in, s_in = node_dim, edge_dim
        act = lambda: nn.LeakyReLU(negative_slope=leaky_slope)  # noqa: E731
        for j in range(channels):
            if if_dense:
                setattr(self, f"MSI{j}", RefNodeEdgeInt(d=t_in, dv=filters))
                setattr(self, f"NEConv{j}", _ref_block(filters, filters, filters, K,
                                                       dropout_ratio, act))
                t_in, s_in = t_in + filters, s_in + filters
            else:
                setattr(self, f"NEConv{j}", _ref_block(t_in, s_in, filters, K, dropout_ratio,
                                                       act))
                t_in = s_in = filters

    def forward(self, x_t0, ei_t, ew_t, x_s0, ei_s, ew_s, par_1=None, D=None):
        for j in range(self.channels):
            if self.if_dense:
                x_t, x_s = getattr(self, f"MSI{j}")(x_t0, x_s0, par_1, D)
                x_t, x_s = getattr(self, f"NEConv{j}")(x_t, ei_t, ew_t, x_s, ei_s, ew_s)
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
            else:
                x_t0, x_s0 = getattr(self, f"NEConv{j}")(x_t0, ei_t, ew_t, x_s0, ei_s, ew_s)
        return x_t0, x_s0


class RefSAPool(nn.Module):
    """lib/Hodge_Cheb_Conv.py:36-59 (SAPool): sigmoid attention on the dense
    features, then structural pooling to level k+1."""

    def __init__(self, d=64, dk=32):
        super().__init__()
        self.NEAtt = RefNodeEdgeInt(d=d, dk=dk, only_att=True, sigma=nn.Sigmoid())

    def forward(self, x_t0, x_s0, par_1, D, datas, pos_ts, pos_ss, k):
        att_t, att_s = self.NEAtt(x_t0, x_s0, par_1, D)
        x_t0 = x_t0 * att_t
        x_s0 = x_s0 * att_s
        x_t0, x_s0 = _pool(x_t0, x_s0, pos_ts[k], pos_ss[k])
        ei_s, ew_s = datas[k + 1].edge_index_s, datas[k + 1].edge_weight_s
        ei_t, ew_t = datas[k + 1].edge_index_t, datas[k + 1].edge_weight_t
        k += 1
        par_1 = adj2par1(datas[k].edge_index, x_t0.shape[0], x_s0.shape[0])
        D = degree(datas[k].edge_index.reshape(-1), num_nodes=x_t0.shape[0]) + 1e-6
        return x_t0, x_s0, par_1, D, k, ei_t, ew_t, ei_s, ew_s, att_t, att_s


# ----------------------------------------------------------------------------
# MLGC (dataset preprocessing for the attention-pooling heads)
# ----------------------------------------------------------------------------
def graclus(edge_index, n: int, weight=None, perm=None) -> np.ndarray:
    """Greedy graclus matching, torch_cluster 1.6.0 graclus_cluster (the
    reference's dependency, absent here; called at lib/Hodge_Dataset.py:252
    and :311, both times WITH a weight -- ones_like for MLGC -- so its
    weighted branch): self-loops dropped, neighbours in CSR order (row-sorted
    COO, columns ascending), nodes visited in `perm` (the reference draws
    torch.randperm); an unmatched node u scans its unmatched neighbours and
    keeps the last one whose weight is >= the best so far (best starts at 0:
    ties go to the LAST neighbour, zero weights match), then u and that
    neighbour get id min(u, v); with no unmatched neighbour u keeps id u.
    Restated from torch_cluster's published graclus_cpu; no copy of it is in
    the reference tree and no fixture holds its output: parity unpinned.
    Returns int64 [n]."""
    ei = np.asarray(edge_index)
    keep = ei[0] != ei[1]
    r, c = ei[0][keep], ei[1][keep]
    w = np.ones(r.size) if weight is None else np.asarray(weight, dtype=np.float64)[keep]
    o = np.lexsort((c, r))
    r, c, w = r[o], c[o], w[o]
    ptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=ptr[1:])
    out = -np.ones(n, dtype=np.int64)
    for u in (range(n) if perm is None else perm):
        if out[u] >= 0:
            continue
        best, wbest = u, 0.0
        for e in range(ptr[u], ptr[u + 1]):
            v = c[e]
            if out[v] >= 0:
                continue
            if w[e] >= wbest:
                best, wbest = v, w[e]
        out[u] = out[best] = min(u, best)
    return out


def mlgc_map(cluster, edge_index):
    """The per-edge loop of MLGC (lib/Hodge_Dataset.py:254-275, :312-333):
    cluster ids renumbered by ascending id; an edge inside one cluster gets
    inf, the others the coarse edge (min, max) in first-seen order.  Keys are
    (min, max) tuples where the reference uses imax + 1e-4 * imin (equal
    below 10^4 coarse nodes).  Returns (c_node int64 [n], c_edge float32 [E],
    coarse edge_index int64 [2, E1], n1)."""
    lab = np.asarray(cluster)
    uniq = np.unique(lab)
    rank = {int(v): i for i, v in enumerate(uniq)}
    c_node = np.array([rank[int(v)] for v in lab], dtype=np.int64)
    ei = np.asarray(edge_index)
    c_edge = np.zeros(ei.shape[1], dtype=np.float32)
    key, e1 = {}, [[], []]
    for i in range(ei.shape[1]):
        a, b = int(c_node[ei[0][i]]), int(c_node[ei[1][i]])
        if a == b:
            c_edge[i] = np.inf
            continue
        lo, hi = min(a, b), max(a, b)
        if (hi, lo) not in key:
            key[(hi, lo)] = len(e1[0])
            e1[0].append(lo)
            e1[1].append(hi)
        c_edge[i] = key[(hi, lo)]
    return c_node, c_edge, np.array(e1, dtype=np.int64).reshape(2, -1), int(uniq.size)


def to_undirected_mean(edge_index, weight, n: int):
    """PyG to_undirected(edge_index, edge_weight, reduce='mean')
    (lib/Hodge_Dataset.py:310): both directions, coalesced in (row, col)
    order, duplicate weights averaged."""
    ei = np.asarray(edge_index)
    w = np.asarray(weight, dtype=np.float32)
    r = np.concatenate([ei[0], ei[1]])
    c = np.concatenate([ei[1], ei[0]])
    ww = np.concatenate([w, w])
    key = r.astype(np.int64) * n + c
    uk, inv = np.unique(key, return_inverse=True)
    s = np.zeros(uk.size, dtype=np.float32)
    np.add.at(s, inv, ww)
    cnt = np.bincount(inv, minlength=uk.size).astype(np.float32)
    return np.stack([uk // n, uk % n]), s / cnt
