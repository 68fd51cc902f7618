"""The HL-HGAT hot-path layers, MI355X-native, with the reference's interface.

Same class names, constructor arguments, attributes, forward signatures and
state_dict keys as lib/Hodge_Cheb_Conv.py of deepika090/HL-HGAT; the
arithmetic runs in the HIP kernels of libhlhgat.so (see ops.py):

  HodgeLaguerreConv  (:452-523)  fused basis + one MFMA projection, adjoint bwd
  HodgeChebConv      (:366-448)  same kernels, Chebyshev recurrence
  NodeEdgeInt / MSI  (:255-309 / :61-115)  incidence gathers, split-K Linear,
                                           fused attention score
  HL_filter          (:117-188)  block composition
  SAPool             (:36-59)    attention-scaled cluster pooling
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor
from torch.nn import Dropout, Parameter

from . import nn as _nn
from . import ops
from .hodge_dataset import BoundaryOperator, adj2par1, boundary_from_sparse, degree
from .nn import BatchNorm, Linear, Sequential, run_sequential

__all__ = ["HodgeLaguerreConv", "HodgeChebConv", "NodeEdgeInt", "MSI", "HL_filter", "SAPool",
           "HodgeLaguerreFastConv"]


class _HodgePolyConv(nn.Module):
    _kind = ops.POLY_LAGUERRE

    def __init__(self, in_channels: int, out_channels: int, K: int, bias: bool = True,
                 **kwargs):
        super().__init__()
        aggr = kwargs.pop("aggr", "add")
        if aggr != "add":
            raise ValueError("HodgeConv: only aggr='add' is supported (as in the reference)")
        assert K > 0
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lins = nn.ModuleList([
            Linear(in_channels, out_channels, bias=False, weight_initializer="glorot")
            for _ in range(K)
        ])
        if bias:
            self.bias = Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        for lin in self.lins:
            lin.reset_parameters()
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x: Tensor, edge_index: Tensor, edge_weight: Optional[Tensor] = None,
                batch: Optional[Tensor] = None) -> Tensor:
        op = ops.hodge_operator(edge_index, edge_weight, x.size(0))
        out, self._hlhgat_out = getattr(self, "_hlhgat_out", None), None
        return ops.hodge_poly_conv(x, op, [lin.weight for lin in self.lins], self.bias,
                                   self._kind, out=out)

    def forward_bn(self, x: Tensor, edge_index: Tensor, edge_weight: Optional[Tensor],
                   bn: nn.BatchNorm1d, relu: bool) -> Tensor:
        """forward -> bn -> (ReLU) as one fused C++ autograd node (the tail of
        every HL block, lib/Hodge_ST_Model.py:556-566); same result as the
        three modules applied in turn."""
        op = ops.hodge_operator(edge_index, edge_weight, x.size(0))
        # one-shot output destination set by the caller (a DenseConcat sink)
        out, self._hlhgat_out = getattr(self, "_hlhgat_out", None), None
        return ops.hodge_poly_conv(x, op, [lin.weight for lin in self.lins], self.bias,
                                   self._kind, bn=bn, relu=relu, out=out)

    def __repr__(self) -> str:
        return (f"{self.__class__.__name__}({self.in_channels}, "
                f"{self.out_channels}, K={len(self.lins)})")


class HodgeLaguerreConv(_HodgePolyConv):
    """Laguerre-polynomial Hodge filter (lib/Hodge_Cheb_Conv.py:452-523):
    T_0 = x, T_1 = x - L x, T_{k+1} = (-L T_k + (2k+1) T_k - k T_{k-1})/(k+1),
    out = sum_k lins[k](T_k) + bias."""
    _kind = ops.POLY_LAGUERRE


class HodgeChebConv(_HodgePolyConv):
    """Chebyshev-polynomial Hodge filter (lib/Hodge_Cheb_Conv.py:366-448):
    T_1 = L x, T_{k+1} = 2 L T_k - T_{k-1}."""
    _kind = ops.POLY_CHEB


class HodgeLaguerreFastConv(HodgeLaguerreConv):
    """DEMO fork's torch_sparse variant (HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:519-582),
    ``forward(x, adj_t)``.

    As published, its k >= 2 terms propagate the layer INPUT x instead of
    Tx_1 (:561):  T_{k+1} = (-L x + (2k+1) T_k - k T_{k-1}) / (k+1).  That is
    what models trained with the DEMO (HL-HGAT-DEMO/weights/HL_HGAT_Brain.pt)
    compute, so it is the default here (``demo_recurrence=True``, HIP kind
    HLHGAT_POLY_LAGUERRE_DEMO); ``demo_recurrence=False`` gives the corrected
    Laguerre recurrence of lib/Hodge_Cheb_Conv.py:502-507.  K = 1, 2 agree.

    ``adj_t`` is any of: a torch_sparse-style object with ``.coo() -> (row,
    col, value)`` (the DEMO's ``SparseTensor(row=ei[0], col=ei[1],
    value=w).t()``, :179-180), a torch sparse COO/CSR tensor holding that
    transpose (``adj_t[j, i] = w_ij``), or an ``(edge_index, edge_weight)``
    pair in the ``propagate`` convention."""

    def __init__(self, in_channels: int, out_channels: int, K: int, bias: bool = True,
                 demo_recurrence: bool = True, **kwargs):
        super().__init__(in_channels, out_channels, K, bias=bias, **kwargs)
        self.demo_recurrence = demo_recurrence
        self._kind = ops.POLY_LAGUERRE_DEMO if demo_recurrence else ops.POLY_LAGUERRE

    @staticmethod
    def adj_to_edge_index(adj_t):
        """(edge_index, edge_weight) in the propagate convention (messages
        flow edge_index[0] -> edge_index[1]) for adj_t = A^T."""
        if isinstance(adj_t, (tuple, list)):
            return adj_t[0], (adj_t[1] if len(adj_t) > 1 else None)
        if hasattr(adj_t, "coo"):  # torch_sparse.SparseTensor
            row, col, val = adj_t.coo()
        elif torch.is_tensor(adj_t) and adj_t.layout in (torch.sparse_coo, torch.sparse_csr):
            coo = adj_t.to_sparse_coo().coalesce()
            (row, col), val = coo.indices(), coo.values()
        else:
            raise TypeError("HodgeLaguerreFastConv: adj_t must be a SparseTensor, a torch "
                            "sparse tensor or (edge_index, edge_weight)")
        # adj_t[r, c] = w  <=>  message c -> r; row-major order = target-sorted
        return torch.stack([col, row]), val

    def forward(self, x: Tensor, adj_t, *args, **kwargs) -> Tensor:  # type: ignore[override]
        edge_index, edge_weight = self.adj_to_edge_index(adj_t)
        return super().forward(x, edge_index, edge_weight)


def _sigma_code(sigma: nn.Module) -> int:
    if isinstance(sigma, nn.Sigmoid):
        return ops.SIGMA_SIGMOID
    if isinstance(sigma, nn.ReLU):
        return ops.SIGMA_RELU
    raise NotImplementedError(f"NodeEdgeInt: sigma {type(sigma).__name__} has no HIP kernel "
                              f"(supported: nn.Sigmoid, nn.ReLU)")


def _as_boundary(par, n_nodes: int, n_edges: int) -> BoundaryOperator:
    if isinstance(par, BoundaryOperator):
        if par.transposed:
            raise ValueError("NodeEdgeInt: par must be B1 [N_t, N_s] (adj2par1), not B1^T")
        return par  # |B1| or B1: the value / attention paths use |B1| either way
    if torch.is_tensor(par) and par.is_sparse:
        return boundary_from_sparse(par)
    raise TypeError("NodeEdgeInt: par must come from adj2par1")


def _value_mlp(seq: nn.Sequential, blocks) -> Tensor:
    """WV_* on cat(blocks): one fused C++ node for the reference structure
    Linear->BN->ReLU->Linear->BN->ReLU in training mode, module-by-module on
    the HIP ops otherwise."""
    m = list(seq)
    if (len(m) == 6 and isinstance(m[0], nn.Linear) and isinstance(m[1], nn.BatchNorm1d)
            and isinstance(m[2], nn.ReLU) and isinstance(m[3], nn.Linear)
            and isinstance(m[4], nn.BatchNorm1d) and isinstance(m[5], nn.ReLU)
            and all(b.training or not b.track_running_stats for b in (m[1], m[4]))
            and all(ops.sync_bn_group(b) is None for b in (m[1], m[4]))):
        return ops.mlp2(blocks, seq)
    return run_sequential(seq, blocks)


class NodeEdgeInt(nn.Module):
    """Node<->edge interaction through the boundary operator
    (lib/Hodge_Cheb_Conv.py:255-309)."""

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
            self.WV_Node = nn.Sequential(
                nn.Linear(d * 2, dl), nn.BatchNorm1d(dl), nn.ReLU(),
                nn.Linear(dl, dv), nn.BatchNorm1d(dv), nn.ReLU())
            self.WV_Edge = nn.Sequential(
                nn.Linear(d * 2, dl), nn.BatchNorm1d(dl), nn.ReLU(),
                nn.Linear(dl, dv), nn.BatchNorm1d(dv), nn.ReLU())
        self.lambda_Node = l
        self.lambda_Edge = l

    def interact(self, x_t: Tensor, x_s: Tensor, par, D: Tensor):
        """x_s2t = (1/D)·|B1| x_s and x_t2s = |B1|^T x_t / 2 (:294-295)."""
        bop = _as_boundary(par, x_t.size(0), x_s.size(0))
        inc = bop.incidence()
        rD = ops.reciprocal(D)
        x_s2t = ops.node_from_edges(x_s, inc, rD)
        x_t2s = ops.edge_from_nodes(x_t, inc)
        return x_s2t, x_t2s

    def forward(self, x_t: Tensor, x_s: Tensor, par, D: Tensor):
        if not self.only_att and x_t.is_cuda and x_t.dim() == 2:
            bop = _as_boundary(par, x_t.size(0), x_s.size(0))
            # one-shot gradient sinks set by the caller (DenseConcat.grad_sink)
            gsink, self._hlhgat_gsink = getattr(self, "_hlhgat_gsink", (None, None)), (None, None)
            # one-shot weight pack built for the whole forward (ops.nei_prepack)
            packed = ops.take_pack(self)
            tapping = _nn.TAP is not None
            if tapping:
                ops._ext.set_tap(True)
            r = ops.nei_value(x_t, x_s, bop.incidence(), ops.reciprocal(D), self.WV_Node,
                              self.WV_Edge, bop.valid_t, bop.valid_s, gsink=gsink, packed=packed)
            if tapping:
                hidden = ops._ext.take_tap()
                ops._ext.set_tap(False)
                if r is not None:  # hidden ReLUs (inside the node), then the outputs
                    for mod, y in zip((self.WV_Node[2], self.WV_Edge[2], self.WV_Node[5],
                                       self.WV_Edge[5]), list(hidden) + list(r)):
                        _nn.tap(mod, y)
            if r is not None:
                return r
        if (not self.only_att and getattr(par, "valid_t", None) is not None
                and any(isinstance(m, nn.BatchNorm1d) and ops._bn_uses_batch_stats(m)
                        for m in list(self.WV_Node) + list(self.WV_Edge))):
            # the unfused value path's batch-statistics BatchNorms would count
            # the padding rows (eval mode, on running statistics, is row-wise)
            raise RuntimeError("hlhgat: static-shape (padded) batches need the fused "
                               "NodeEdgeInt value path (training-mode WV_* MLPs)")
        ch = ops.active_chains(x_t.device) if x_t.is_cuda else None
        if ch is not None and ch.on:
            # the unfused path (eval mode, SyncBatchNorm, attention) runs on the
            # current (node-chain) stream: x_s comes from the edge chain, and
            # both outputs go back to it -- a full exchange with the edge chain
            # (the fused path exchanges only the first-layer GEMM results)
            ch.main.wait_stream(ch.side)
            x_s.record_stream(ch.main)
            r = self._unfused(x_t, x_s, par, D)
            ch.sync_side()
            for t in r:
                t.record_stream(ch.side)
            return r
        return self._unfused(x_t, x_s, par, D)

    def _unfused(self, x_t: Tensor, x_s: Tensor, par, D: Tensor):
        x_s2t, x_t2s = self.interact(x_t, x_s, par, D)
        if self.only_att:
            code = _sigma_code(self.sigma)
            dk = self.dk
            sq = float(np.sqrt(dk))
            # node side: K = WK_Node(x_t), Q_self = WQ_Node(x_t) in one GEMM
            # (the K|Q packs of the whole forward: ops.att_prepack, one launch)
            pk = ops.take_att_pack(self) if x_t.is_cuda else None
            if pk is not None:
                w_t, b_t, w_s, b_s = pk
            else:
                w_t = torch.cat([self.WK_Node.weight, self.WQ_Node.weight], 0)
                b_t = torch.cat([self.WK_Node.bias, self.WQ_Node.bias], 0)
                w_s = torch.cat([self.WK_Edge.weight, self.WQ_Edge.weight], 0)
                b_s = torch.cat([self.WK_Edge.bias, self.WQ_Edge.bias], 0)
            kq_t = ops.linear_blocks([x_t], w_t, b_t)
            qc_t = ops.linear_blocks([x_s2t], self.WQ_Edge.weight, self.WQ_Edge.bias)
            a_t = ops.att_score_kq(qc_t, kq_t, 1 - self.lambda_Node, self.lambda_Node, sq, code)
            kq_s = ops.linear_blocks([x_s], w_s, b_s)
            qc_s = ops.linear_blocks([x_t2s], self.WQ_Node.weight, self.WQ_Node.bias)
            a_s = ops.att_score_kq(qc_s, kq_s, 1 - self.lambda_Edge, self.lambda_Edge, sq, code)
            if isinstance(self.sigma, nn.ReLU):
                _nn.tap(self.sigma, a_t)
                _nn.tap(self.sigma, a_s)
            return a_t, a_s
        # node and edge MLPs are independent: edge side on the side stream
        return ops.fork(lambda: _value_mlp(self.WV_Node, [x_s2t, x_t]),
                        lambda: _value_mlp(self.WV_Edge, [x_t2s, x_s]),
                        side_inputs=(x_t2s, x_s), device=x_t.device)


class MSI(NodeEdgeInt):
    """Identical twin of NodeEdgeInt (lib/Hodge_Cheb_Conv.py:61-115)."""


class HL_filter(nn.Module):
    """Stack of HL-filtering blocks (lib/Hodge_Cheb_Conv.py:117-188)."""

    def __init__(self, channels=2, filters=32, K=4, node_dim=64, edge_dim=64,
                 dropout_ratio=0.0, leaky_slope=0.1, if_dense=True):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.node_dim = node_dim
        self.edge_dim = edge_dim
        self.if_dense = if_dense
        gcn_outsize = self.filters
        t_insize = self.node_dim
        s_insize = self.edge_dim
        for j in range(self.channels):
            if self.if_dense:
                setattr(self, "MSI{}".format(j), MSI(d=t_insize, dv=gcn_outsize))
                cin_t = cin_s = gcn_outsize
            else:
                cin_t, cin_s = t_insize, s_insize
            layers = [(HodgeLaguerreConv(cin_t, gcn_outsize, K=K),
                       "x_t, edge_index_t, edge_weight_t -> x_t"),
                      (BatchNorm(gcn_outsize), "x_t -> x_t"),
                      (nn.LeakyReLU(negative_slope=leaky_slope), "x_t -> x_t"),
                      (Dropout(p=dropout_ratio), "x_t -> x_t"),
                      (HodgeLaguerreConv(cin_s, gcn_outsize, K=K),
                       "x_s, edge_index_s, edge_weight_s -> x_s"),
                      (BatchNorm(gcn_outsize), "x_s -> x_s"),
                      (nn.LeakyReLU(negative_slope=leaky_slope), "x_s -> x_s"),
                      (Dropout(p=dropout_ratio), "x_s -> x_s"),
                      (lambda x1, x2: [x1, x2], "x_t, x_s -> x")]
            setattr(self, "NEConv{}".format(j),
                    Sequential("x_t, edge_index_t, edge_weight_t, x_s, edge_index_s, "
                               "edge_weight_s", layers))
            if self.if_dense:
                t_insize = t_insize + gcn_outsize
                s_insize = s_insize + gcn_outsize
            else:
                t_insize = gcn_outsize
                s_insize = gcn_outsize

    def forward(self, x_t0, edge_index_t, edge_weight_t, x_s0, edge_index_s, edge_weight_s,
                par_1=None, D=None):
        for j in range(self.channels):
            if self.if_dense:
                x_t, x_s = getattr(self, "MSI{}".format(j))(x_t0, x_s0, par_1, D)
                x_t, x_s = getattr(self, "NEConv{}".format(j))(
                    x_t, edge_index_t, edge_weight_t, x_s, edge_index_s, edge_weight_s)
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
            else:
                x_t0, x_s0 = getattr(self, "NEConv{}".format(j))(
                    x_t0, edge_index_t, edge_weight_t, x_s0, edge_index_s, edge_weight_s)
        return x_t0, x_s0


def cluster_mean(x: Tensor, assign: Tensor, n_seg: Optional[int] = None) -> Tensor:
    """torch_scatter.scatter_mean(x, assign, dim=0) on the HIP segment-mean
    kernel; members are grouped per cluster (stable) by the CSR builder.
    Members assigned inf (an edge dropped by MLGC, lib/Hodge_Dataset.py:262)
    are left out, as the reference's x[~isinf(pos)] filter does, without a
    host sync.  n_seg (the number of clusters, e.g. the coarse level's row
    count) avoids the max() sync; default max(assign) + 1."""
    n = x.size(0)
    a = assign.view(-1)
    if n_seg is None:
        fin = a[~torch.isinf(a)] if a.is_floating_point() else a
        n_seg = int(fin.max().item()) + 1 if fin.numel() else 0
    if a.is_floating_point():
        a = torch.where(torch.isinf(a), torch.full_like(a, float(n_seg)), a)
    idx = a.to(torch.long)
    ar = torch.arange(n, device=x.device)
    csr = ops._csr_general(idx, ar, None, n_seg + 1, max(n, 1))
    return ops.segment_mean(x, csr.rowptr, n_seg, csr.col)


class SAPool(nn.Module):
    """Attention-scaled structural pooling (lib/Hodge_Cheb_Conv.py:36-59)."""

    def __init__(self, d=64, dk=32):
        super().__init__()
        self.NEAtt = MSI(d=d, dk=dk, only_att=True, sigma=nn.Sigmoid())

    def forward(self, x_t0, x_s0, par_1, D, datas, pos_ts, pos_ss, k, device="cuda:0"):
        att_t, att_s = self.NEAtt(x_t0, x_s0, par_1, D)
        x_t0 = x_t0 * att_t
        x_s0 = x_s0 * att_s
        pos_t, pos_s = pos_ts[k], pos_ss[k]
        x_t0 = cluster_mean(x_t0, pos_t, datas[k + 1].x_t.shape[0])
        x_s0 = cluster_mean(x_s0, pos_s, datas[k + 1].x_s.shape[0])  # inf members dropped
        edge_index_s = datas[k + 1].edge_index_s.to(device)
        edge_weight_s = datas[k + 1].edge_weight_s.to(device)
        edge_index_t = datas[k + 1].edge_index_t.to(device)
        edge_weight_t = datas[k + 1].edge_weight_t.to(device)
        k += 1
        par_1 = adj2par1(datas[k].edge_index.to(device), x_t0.shape[0], x_s0.shape[0])
        D = degree(datas[k].edge_index.view(-1).to(device), num_nodes=x_t0.shape[0]) + 1e-6
        return (x_t0, x_s0, par_1, D, k, edge_index_t, edge_weight_t, edge_index_s,
                edge_weight_s, att_t, att_s)
