"""HL-HGAT task heads (callers of the hot path), reference names and keys.

Mirrors lib/Hodge_ST_Model.py; the per-step host work of the reference
(Python loops building batch vectors, :611-615) is replaced by device-side
segment pointers built from num_node1 / num_edge1.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn
from torch.nn import Dropout, Linear

from . import ops
from .hodge_cheb_conv import HodgeLaguerreConv, NodeEdgeInt, cluster_mean
from .distributed import global_max
from .hodge_dataset import adj2par1, degree
from . import nn as _nn
from .nn import Abs, BatchNorm, Sequential, run_mlp_stack

__all__ = ["HL_HGCNN_zinc_dense_int3_pyr", "HL_HGCNN_pepfunc_dense_int3_pyr",
           "HL_HGCNN_CIFAR10SP_dense_int3_pyr", "HL_HGCNN_zinc_dense_poolint3_pyr",
           "HL_HGCNN_TSP_dense_int3_pyr", "HL_HGCNN_CIFAR10SP_dense_int3_attpool",
           "HL_HGCNN_zinc_dense_int3_attpool", "HL_HGCNN_pepfunc_dense_int3_attpool",
           "segment_ptr", "mean_pool_sorted"]


def segment_ptr(counts: torch.Tensor, device) -> torch.Tensor:
    """int32 [B+1] offsets of graph-contiguous rows (PairData batching)."""
    counts = counts.to(device)
    ptr = torch.zeros(counts.numel() + 1, dtype=torch.int32, device=device)
    ptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return ptr


def mean_pool_sorted(x: torch.Tensor, counts: torch.Tensor,
                     ptr: torch.Tensor = None) -> torch.Tensor:
    """global_mean_pool(x, batch) for a graph-contiguous batch vector
    (lib/Hodge_ST_Model.py:636) on the HIP segment-mean kernel; ``ptr`` =
    the batch's precomputed int32 offsets (collate: seg_ptr_t / seg_ptr_s)."""
    if ptr is None or ptr.device != x.device or ptr.numel() != counts.numel() + 1:
        ptr = segment_ptr(counts, x.device)
    return ops.segment_mean(x, ptr, counts.numel())


READOUT_ON_CHAIN = True  # A/B hook: False = the edge readout on the main stream
# A/B hook: True = the edge chain waits for the main stream after HL_init_conv
# even when the batch carries its incidence / degree tables (nothing to wait for)
SYNC_SIDE_ALWAYS = False


def mean_pool_cat(parts, side=None) -> torch.Tensor:
    """torch.cat([mean_pool_sorted(x, counts, ptr) ...], -1) as one output
    written block by block (ops.segment_mean_cat): the readout of
    lib/Hodge_ST_Model.py:636 without the cat launch.  side: the edge chain's
    stream for the first part (ops.Chains)."""
    ptrs = []
    for x, counts, ptr in parts:
        if ptr is None or ptr.device != x.device or ptr.numel() != counts.numel() + 1:
            ptr = segment_ptr(counts, x.device)
        ptrs.append(ptr)
    return ops.segment_mean_cat([x for x, _, _ in parts], ptrs, parts[0][1].numel(), side=side)


def _hl_block(cin_t, cin_s, cout, K, dropout_ratio, act=nn.ReLU):
    layers = [(HodgeLaguerreConv(cin_t, cout, K=K), "x_t, edge_index_t, edge_weight_t -> x_t"),
              (BatchNorm(cout), "x_t -> x_t"),
              (act(), "x_t -> x_t"),
              (Dropout(p=dropout_ratio), "x_t -> x_t"),
              (HodgeLaguerreConv(cin_s, cout, K=K), "x_s, edge_index_s, edge_weight_s -> x_s"),
              (BatchNorm(cout), "x_s -> x_s"),
              (act(), "x_s -> x_s"),
              (Dropout(p=dropout_ratio), "x_s -> x_s"),
              (lambda x1, x2: [x1, x2], "x_t, x_s -> x")]
    return Sequential("x_t, edge_index_t, edge_weight_t, x_s, edge_index_s, edge_weight_s", layers)


def _sink(block, dt, ds, width):
    """Point the node / edge convs of an HL block (module_0 on L0, module_4 on
    L1, see _hl_block) at the next column blocks of the dense slabs."""
    block.module_0._hlhgat_out = dt.sink(width)
    block.module_4._hlhgat_out = ds.sink(width)


class _PyrHead(nn.Module):
    """The dense pyramid heads without pooling (lib/Hodge_ST_Model.py:307-407
    pepfunc, :544-646 ZINC, :858-955 CIFAR10SP): HL_init_conv, then per block
    NEInt{i}{j} (NodeEdgeInt on the dense concatenation) and NEConv{i}{j}
    (Laguerre on L0 and L1), mean readout, MLP.  They differ only in the
    initial convs' order (init_K: K, or 1 for CIFAR10SP :870-875), the degree
    (deg_eps: degree + 1e-6 in pepfunc :385 and CIFAR10SP :935, the bare
    degree in ZINC :624) and NodeEdgeInt's attention mix l (unused by its value
    path; CIFAR10SP :889)."""

    def __init__(self, channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                 dropout_ratio, dropout_ratio_mlp, keig, init_K, deg_eps, nei_l=0.9):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        self.node_dim = node_dim + keig
        self.edge_dim = edge_dim + keig
        self.initial_channel = self.filters[0]
        self._deg_eps = deg_eps
        self.HL_init_conv = _hl_block(self.node_dim, self.edge_dim, self.initial_channel, init_K,
                                      dropout_ratio)
        gcn_insize = self.initial_channel
        for i, gcn_outsize in enumerate(self.filters):
            for j in range(self.channels[i]):
                setattr(self, "NEInt{}{}".format(i, j),
                        NodeEdgeInt(d=gcn_insize, dv=gcn_outsize, l=nei_l))
                setattr(self, "NEConv{}{}".format(i, j),
                        _hl_block(gcn_outsize, gcn_outsize, gcn_outsize, K, dropout_ratio))
                gcn_insize = gcn_outsize + gcn_insize
        mlp_insize = self.filters[-1] * 2
        for i, mlp_outsize in enumerate(mlp_channels):
            setattr(self, "mlp%d" % i, nn.Sequential(
                Linear(mlp_insize, mlp_outsize), nn.BatchNorm1d(mlp_outsize), nn.ReLU(),
                nn.Dropout(dropout_ratio_mlp)))
            mlp_insize = mlp_outsize
        self.out = Linear(mlp_insize, num_classes)

    def forward(self, data, device="cuda:0", if_final_layer=False):
        x_s, edge_index_s, edge_weight_s = data.x_s, data.edge_index_s, data.edge_weight_s
        x_t, edge_index_t, edge_weight_t = data.x_t, data.edge_index_t, data.edge_weight_t
        # the dense concatenations x_t0 / x_s0 (:631-632) live in one slab per
        # side; every block's conv writes its output into its column block
        width = self.initial_channel + sum(c * f for c, f in zip(self.channels, self.filters))
        dense = x_t.is_cuda and x_t.dim() == 2 and ops.DENSE_SLAB
        if dense:
            dt = ops.DenseConcat(x_t.size(0), width, x_t)
            ds = ops.DenseConcat(x_s.size(0), width, x_s)
            _sink(self.HL_init_conv, dt, ds, self.initial_channel)
        n_t, n_s = x_t.shape[0], x_s.shape[0]
        valid_t = getattr(data, "valid_mask_t", None)
        if dense:  # every NodeEdgeInt's first-Linear pack in one launch
            ops.nei_prepack([getattr(self, "NEInt{}{}".format(i, j))
                             for i, _ in enumerate(self.channels) for j in range(self.channels[i])])

        def boundary():
            # the reference rebuilds par_1 and D for every block group (:623-624)
            # from the same edge_index, so the values are identical: build them
            # once.  reference: degree(edge_index.view(-1)) sized max(index)+1
            # (:624); that equals N_t whenever it does not crash (1/D broadcast
            # over x_t rows), so size it by N_t and skip the host sync of max()
            p1 = adj2par1(data.edge_index, n_t, n_s)
            d = getattr(data, "deg_t", None)  # built at collate (padding rows: 1)
            # device work issued here (degree / incidence builds on the main
            # stream) must be ordered before the edge chain uses it; batches
            # from collate carry both tables and issue none
            launched = d is None or d.device != x_t.device or d.numel() != n_t
            if launched:
                d = degree(data.edge_index.view(-1), num_nodes=n_t)
                if valid_t is not None:  # static-shape padding rows: unit degree, no 1/0
                    d = d.masked_fill(~valid_t, 1.0)
            if self._deg_eps:
                d = d + self._deg_eps
            if not x_t.is_cuda:
                return p1, d, False
            launched = launched or getattr(data.edge_index, "_hlhgat_incidence", None) is None
            p1.incidence()  # built here (or taken from collate), cached for every NodeEdgeInt
            return p1, d, launched

        # the incidence build (sort + CSR of |B1|) after HL_init_conv (building it
        # on a third stream beside the conv measured 1.4 % slower: its sort
        # kernels slow the two conv chains more than the overlap saves)
        # the node and edge chains of the block section on two streams with one
        # cross-stream exchange per block (ops.Chains) where the fused paths run
        # (not in SyncBatchNorm mode: its statistics all-reduce inside the
        # cross-block edge chain made hipStreamEndCapture segfault under RCCL,
        # while per-block fork / join captured bitwise the same step,
        # tools/probes/syncbn_capture_probe.py)
        chains = (ops.Chains(x_t.device, enabled=not ops.has_sync_bn(self) or ops.SYNCBN_CHAINS)
                  if dense else contextlib.nullcontext())
        with chains as ch:
            x_t, x_s = self.HL_init_conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                         edge_weight_s)
            par_1, D, launched = boundary()
            if dense:
                if launched or SYNC_SIDE_ALWAYS:
                    ch.sync_side()  # tables built on main feed the edge chain
                dt.append(x_t)
                with ch.side_context():  # a copy (no sink: eval, SyncBN) on x_s's chain
                    ds.append(x_s)
            x_s0, x_t0 = x_s, x_t
            for i, _ in enumerate(self.channels):
                for j in range(self.channels[i]):
                    neint = getattr(self, "NEInt{}{}".format(i, j))
                    if dense:
                        x_t0 = dt.view()
                        gs_t = dt.grad_sink()
                        with ch.side_context():  # the edge slab's view / gradient: edge chain
                            x_s0 = ds.view()
                            gs_s = ds.grad_sink()
                        # its input gradients go straight into the slab's gradient
                        neint._hlhgat_gsink = (gs_t, gs_s)
                    x_t, x_s = neint(x_t0, x_s0, par_1, D)
                    conv = getattr(self, "NEConv{}{}".format(i, j))
                    if dense:
                        _sink(conv, dt, ds, self.filters[i])
                    x_t, x_s = conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                    edge_weight_s)
                    if dense:
                        dt.append(x_t)
                        with ch.side_context():  # x_s was produced on the edge chain
                            ds.append(x_s)
                    else:
                        x_t0 = torch.cat([x_t0, x_t], dim=-1)
                        x_s0 = torch.cat([x_s0, x_s], dim=-1)
            # the readout; x_s's mean on the edge chain (joined when the chains end)
            x = mean_pool_cat([(x_s, data.num_edge1, getattr(data, "seg_ptr_s", None)),
                               (x_t, data.num_node1, getattr(data, "seg_ptr_t", None))],
                              side=ch.side if (dense and ch.on and READOUT_ON_CHAIN) else None)
        x = run_mlp_stack([getattr(self, "mlp%d" % i) for i in range(len(self.mlp_channels))],
                          [x])
        y = ops.linear_blocks([x], self.out.weight, self.out.bias)
        if if_final_layer:
            return x, y
        return y


class HL_HGCNN_zinc_dense_int3_pyr(_PyrHead):
    """ZINC regression head (lib/Hodge_ST_Model.py:544-646; BASELINE configs
    1-2): degree without the 1e-6 (:624)."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=21, edge_dim=3, num_classes=1, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, keig=7):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, keig, init_K=K, deg_eps=0.0)


class HL_HGCNN_pepfunc_dense_int3_pyr(_PyrHead):
    """Peptides-func pyramid head (lib/Hodge_ST_Model.py:307-407): the ZINC
    structure with peptides widths and degree + 1e-6 (:385)."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=9, edge_dim=3, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, keig=20):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, keig, init_K=K, deg_eps=1e-6)


class HL_HGCNN_CIFAR10SP_dense_int3_pyr(_PyrHead):
    """CIFAR10 superpixel pyramid head (lib/Hodge_ST_Model.py:858-955): K=1
    initial convs (:870-875), NodeEdgeInt(l=l) (:889), degree + 1e-6 (:935)."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=5, edge_dim=4, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, l=0.9, keig=10):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, keig, init_K=1, deg_eps=1e-6,
                         nei_l=l)


class HL_HGCNN_zinc_dense_poolint3_pyr(nn.Module):
    """ZINC head with the interaction AFTER the convs of a level
    (lib/Hodge_ST_Model.py:649-749): per level i, NEConv{i}{j} runs the
    Laguerre convs on the dense concatenation itself (width gcn_insize ->
    gcn_outsize) and appends its outputs, then ONE NEInt{i} mixes the whole
    concatenation and appends its outputs too; readout of the last NEInt's
    outputs.  Degree without the 1e-6 (:729)."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=21, edge_dim=3, num_classes=1, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, keig=7):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        self.node_dim = node_dim + keig
        self.edge_dim = edge_dim + keig
        self.initial_channel = self.filters[0]
        self.HL_init_conv = _hl_block(self.node_dim, self.edge_dim, self.initial_channel, K,
                                      dropout_ratio)
        gcn_insize = self.initial_channel
        for i, gcn_outsize in enumerate(self.filters):
            for j in range(self.channels[i]):
                setattr(self, "NEConv{}{}".format(i, j),
                        _hl_block(gcn_insize, gcn_insize, gcn_outsize, K, dropout_ratio))
                gcn_insize = gcn_outsize + gcn_insize
            setattr(self, "NEInt{}".format(i), NodeEdgeInt(d=gcn_insize, dv=gcn_outsize))
            gcn_insize = gcn_outsize + gcn_insize
        mlp_insize = self.filters[-1] * 2
        for i, mlp_outsize in enumerate(mlp_channels):
            setattr(self, "mlp%d" % i, nn.Sequential(
                Linear(mlp_insize, mlp_outsize), nn.BatchNorm1d(mlp_outsize), nn.ReLU(),
                nn.Dropout(dropout_ratio_mlp)))
            mlp_insize = mlp_outsize
        self.out = Linear(mlp_insize, num_classes)

    def forward(self, data, device="cuda:0"):
        x_s, edge_index_s, edge_weight_s = data.x_s, data.edge_index_s, data.edge_weight_s
        x_t, edge_index_t, edge_weight_t = data.x_t, data.edge_index_t, data.edge_weight_t
        width = self.initial_channel + sum((c + 1) * f for c, f in zip(self.channels, self.filters))
        dense = x_t.is_cuda and x_t.dim() == 2 and ops.DENSE_SLAB
        if dense:
            dt = ops.DenseConcat(x_t.size(0), width, x_t)
            ds = ops.DenseConcat(x_s.size(0), width, x_s)
            _sink(self.HL_init_conv, dt, ds, self.initial_channel)
        n_t, n_s = x_t.shape[0], x_s.shape[0]
        x_t, x_s = self.HL_init_conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                     edge_weight_s)
        if dense:
            dt.append(x_t)
            ds.append(x_s)
        x_s0, x_t0 = x_s, x_t
        # par_1 and D from the same edge_index at every level (:728-729): once;
        # degree sized by N_t (the reference's max(index)+1 equals it whenever
        # its 1/D broadcast over x_t rows does not fail)
        par_1 = adj2par1(data.edge_index, n_t, n_s)
        D = getattr(data, "deg_t", None)
        if D is None or D.device != x_t.device or D.numel() != n_t:
            D = degree(data.edge_index.view(-1), num_nodes=n_t)
            valid_t = getattr(data, "valid_mask_t", None)
            if valid_t is not None:
                D = D.masked_fill(~valid_t, 1.0)
        for i, _ in enumerate(self.channels):
            for j in range(self.channels[i]):
                conv = getattr(self, "NEConv{}{}".format(i, j))
                if dense:
                    x_t0, x_s0 = dt.view(), ds.view()
                    _sink(conv, dt, ds, self.filters[i])
                x_t, x_s = conv(x_t0, edge_index_t, edge_weight_t, x_s0, edge_index_s,
                                edge_weight_s)
                if dense:
                    dt.append(x_t)
                    ds.append(x_s)
                else:
                    x_t0 = torch.cat([x_t0, x_t], dim=-1)
                    x_s0 = torch.cat([x_s0, x_s], dim=-1)
            neint = getattr(self, "NEInt{}".format(i))
            if dense:
                x_t0, x_s0 = dt.view(), ds.view()
                neint._hlhgat_gsink = (dt.grad_sink(), ds.grad_sink())
            x_t, x_s = neint(x_t0, x_s0, par_1, D)
            if dense:
                dt.append(x_t)
                ds.append(x_s)
            else:
                x_t0 = torch.cat([x_t0, x_t], dim=-1)
                x_s0 = torch.cat([x_s0, x_s], dim=-1)
        x = mean_pool_cat([(x_s, data.num_edge1, getattr(data, "seg_ptr_s", None)),
                           (x_t, data.num_node1, getattr(data, "seg_ptr_t", None))])
        x = run_mlp_stack([getattr(self, "mlp%d" % i) for i in range(len(self.mlp_channels))],
                          [x])
        return ops.linear_blocks([x], self.out.weight, self.out.bias)


class HL_HGCNN_TSP_dense_int3_pyr(nn.Module):
    """TSP edge-classification head (lib/Hodge_ST_Model.py:756-855, BASELINE
    config 5): HL_init_conv on node coordinates and edge lengths, dense HL
    blocks, readout per edge = [x_s, |B1^T x_t| / 2] -> K=1 HL conv MLP ->
    K=1 HL conv, masked by the edge mask column of x_s.  Returns
    (logits * mask, s_batch) like the reference."""

    def __init__(self, channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[], K=2,
                 node_dim=2, edge_dim=1, num_classes=1, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, keig=20):
        super().__init__()
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        self.node_dim = node_dim
        self.edge_dim = edge_dim
        self.initial_channel = self.filters[0]
        self.HL_init_conv = _hl_block(self.node_dim, self.edge_dim, self.initial_channel, K,
                                      dropout_ratio)
        gcn_insize = self.initial_channel
        for i, gcn_outsize in enumerate(self.filters):
            for j in range(self.channels[i]):
                setattr(self, "NEInt{}{}".format(i, j), NodeEdgeInt(d=gcn_insize, dv=gcn_outsize))
                setattr(self, "NEConv{}{}".format(i, j),
                        _hl_block(gcn_outsize, gcn_outsize, gcn_outsize, K, dropout_ratio))
                gcn_insize = gcn_outsize + gcn_insize
        mlp_insize = self.filters[-1] * 2
        if len(self.mlp_channels) == 1:
            self.mlp = Sequential("x_t, edge_index_t, edge_weight_t", [
                (HodgeLaguerreConv(mlp_insize, self.mlp_channels[0], K=1),
                 "x_t, edge_index_t, edge_weight_t -> x_t"),
                (BatchNorm(self.mlp_channels[0]), "x_t -> x_t"),
                (nn.ReLU(), "x_t -> x_t"),
                (Dropout(p=dropout_ratio), "x_t -> x_t")])
            mlp_insize = self.mlp_channels[0]
        self.out = Sequential("x_t, edge_index_t, edge_weight_t", [
            (HodgeLaguerreConv(mlp_insize, num_classes, K=1),
             "x_t, edge_index_t, edge_weight_t -> x_t")])
        self.readout_abs = Abs()  # |B1^T x_t| (:848); a module so the gates can freeze its signs

    def forward(self, data, device="cuda:0"):
        dev = data.x_s.device
        # output_size given: no host sync (the step can be captured)
        s_batch = _per_row(torch.arange(data.num_edge1.numel(), device=dev), data.num_edge1,
                           data.x_s.size(0), fill=data.num_edge1.numel())  # padding: no graph
        x_s, edge_index_s, edge_weight_s = data.x_s[:, :1], data.edge_index_s, data.edge_weight_s
        edge_mask = data.x_s[:, 1:]
        x_t, edge_index_t, edge_weight_t = data.x_t, data.edge_index_t, data.edge_weight_t
        width = self.initial_channel + sum(c * f for c, f in zip(self.channels, self.filters))
        dense = x_t.is_cuda and x_t.dim() == 2 and ops.DENSE_SLAB
        # the readout's |B1^T x_t| / 2 in the edge slab's last columns, right
        # after the last block's x_s: cat([x_s, x_t2s]) is a window of the slab
        # (unless the Abs is observed: a tap or hooks see the unfused path)
        fused_ro = dense and _nn.TAP is None and not (self.readout_abs._forward_hooks or
                                                       self.readout_abs._forward_pre_hooks)
        if dense:
            dt = ops.DenseConcat(x_t.size(0), width, x_t)
            ds = ops.DenseConcat(x_s.size(0), width + (self.filters[-1] if fused_ro else 0), x_s)
            _sink(self.HL_init_conv, dt, ds, self.initial_channel)
        x_t, x_s = self.HL_init_conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                     edge_weight_s)
        if dense:
            dt.append(x_t)
            ds.append(x_s)
        x_s0, x_t0 = x_s, x_t
        par_1 = adj2par1(data.edge_index, x_t.shape[0], x_s.shape[0])
        D = _node_degree(data, x_t.shape[0], x_t.device) + 1e-6  # (:823)
        for i, _ in enumerate(self.channels):
            for j in range(self.channels[i]):
                neint = getattr(self, "NEInt{}{}".format(i, j))
                if dense:
                    x_t0, x_s0 = dt.view(), ds.view()
                    # its input gradients go straight into the slab's gradient
                    neint._hlhgat_gsink = (dt.grad_sink(), ds.grad_sink())
                x_t, x_s = neint(x_t0, x_s0, par_1, D)
                conv = getattr(self, "NEConv{}{}".format(i, j))
                if dense:
                    _sink(conv, dt, ds, self.filters[i])
                x_t, x_s = conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                edge_weight_s)
                if dense:
                    dt.append(x_t)
                    ds.append(x_s)
                else:
                    x_t0 = torch.cat([x_t0, x_t], dim=-1)
                    x_s0 = torch.cat([x_s0, x_s], dim=-1)
        # readout (:846-851): x_t2s = |B1^T x_t| / 2 per edge
        if fused_ro:
            c0, c1 = ds.cols[-1]
            x_s = ops.tsp_readout(x_s, x_t, par_1.incidence(), ds.S[:, c0:c1 + x_t.size(1)])
        else:
            x_t2s = self.readout_abs(ops.boundary_t(x_t, par_1.incidence())) / 2
            x_s = torch.cat([x_s, x_t2s], dim=-1)
        if len(self.mlp_channels) == 1:
            x_s = self.mlp(x_s, edge_index_s, edge_weight_s)
        return self.out(x_s, edge_index_s, edge_weight_s) * edge_mask, s_batch


def _has_pool_tables(d0, device) -> bool:
    return all(torch.is_tensor(getattr(d0, k, None)) and getattr(d0, k).device == device
               for k in ("pool_rowptr_t", "pool_rows_t", "pool_rowptr_s", "pool_rows_s"))


def _pool(x: torch.Tensor, pos, d0, side: str, n_seg: int, out=None, gsink=None) -> torch.Tensor:
    """cluster_mean(x, pos, n_seg) -- from the level list's collate-time
    cluster CSR when it carries one (hodge_dataset.pool_tables: the CSR
    cluster_mean would sort on the device, so the same bits; written into
    ``out``, a DenseConcat sink, when given; x's gradient into ``gsink``, the
    gradient slab of x = DenseConcat.view(), when given), else on the device
    from pos."""
    if pos is None:
        rp, rows = getattr(d0, "pool_rowptr_" + side), getattr(d0, "pool_rows_" + side)
        if rp.numel() != n_seg + 2 or rows.numel() != x.size(0):
            raise RuntimeError(f"hlhgat: pool tables ({rp.numel() - 2} clusters, {rows.numel()} "
                               f"rows) do not match ({n_seg}, {x.size(0)})")
        return ops.segment_mean(x, rp, n_seg, rows, out=out, covering=True, gsink=gsink)
    return cluster_mean(x, pos, n_seg)


def _node_degree(data, n: int, device) -> torch.Tensor:
    """degree(edge_index.view(-1), n) (lib/Hodge_Cheb_Conv.py:359): the
    collate-time deg_t when the batch carries it (no device work in the step;
    static-shape padding nodes get 1 there instead of 0 -- they belong to no
    edge of a real simplex, so no real row changes), else computed here."""
    d = getattr(data, "deg_t", None)
    if torch.is_tensor(d) and d.device == device and d.numel() == n:
        return d
    return degree(data.edge_index.view(-1), num_nodes=n)


def _per_row(vals: torch.Tensor, counts: torch.Tensor, rows: int, fill=0) -> torch.Tensor:
    """repeat_interleave(vals, counts) over `rows` rows without a host sync:
    rows beyond sum(counts) (static-shape padding rows, in no graph) get
    `fill` -- the count of that tail is computed on the device, so the output
    is fully written whatever the padding (never an uninitialised tail)."""
    dev = vals.device
    counts = counts.to(dev).to(torch.int64)
    tail = (rows - counts.sum()).clamp(min=0).reshape(1)
    v = torch.cat([vals, torch.full((1,), fill, dtype=vals.dtype, device=dev)])
    return torch.repeat_interleave(v, torch.cat([counts, tail]), output_size=rows)


def _level_offsets(counts_next: torch.Tensor, counts: torch.Tensor, device,
                   rows: int) -> torch.Tensor:
    """n_ahead[n_batch] of the attpool heads (lib/Hodge_ST_Model.py:1031-1036):
    for every row of the fine level (`rows` of them: no host sync), the first
    coarse row of its graph; padding rows get 0 (their cluster id is inf)."""
    ahead = torch.zeros(counts_next.numel(), dtype=torch.float32, device=device)
    ahead[1:] = torch.cumsum(counts_next.to(device), 0)[:-1].to(torch.float32)
    return _per_row(ahead, counts, rows)


def _valid_rows(x: torch.Tensor, n_valid) -> torch.Tensor:
    """x with its static-shape padding rows (>= n_valid, a device int32 [1])
    set to -inf, so a max over it is the max over the real rows."""
    if n_valid is None:
        return x
    keep = torch.arange(x.size(0), device=x.device) < n_valid.to(x.device)
    return x.masked_fill(~keep.view(-1, *([1] * (x.dim() - 1))), float("-inf"))


class _AttPoolHead(nn.Module):
    """Shared body of the attention-pooling heads (two MLGC levels, ``datas``
    = [fine batch with the cluster of each node / edge in feature column 0,
    coarse batch]).  att_mode:
      "every": NEAtt{i} (sigmoid) after every level on the dense
        concatenation, which it scales (main_pepfunc...:133-137);
      "concat": one NEAtt at pool_loc (sigmoid) on the dense concatenation,
        which it scales before pooling (lib/Hodge_ST_Model.py:223-226,276-280);
      "block": one NEAtt at pool_loc (ReLU) on the level's last block output,
        which it scales (the dense concatenation is pooled unscaled), divided
        by its batch max when att_max_norm (CIFAR10SP :1058-1064; ZINC
        :462-465,515-519 does not divide).
    init_K: the initial convs' order (1, or K for ZINC :425-430); deg_eps: the
    1e-6 added to the degree (0 for ZINC :504)."""

    # the reference builds NEAtt{i} for every level but uses only the pool_loc
    # one in this mode: those parameters get no gradient, so DDP must look for
    # unused parameters (hlhgat.distributed.wrap_ddp reads this flag)
    ddp_find_unused_parameters = True

    @property
    def forward_collectives(self) -> bool:
        """The pool_loc attention is divided by its batch max over every rank
        (distributed.global_max)."""
        return self.att_mode == "block" and self.att_max_norm

    def __init__(self, channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                 dropout_ratio, dropout_ratio_mlp, pool_loc, keig, l, att_mode,
                 att_max_norm=True, init_K=1, deg_eps=1e-6):
        super().__init__()
        assert att_mode in ("every", "concat", "block")
        self.channels = channels
        self.filters = filters
        self.mlp_channels = mlp_channels
        self.node_dim = node_dim + keig
        self.edge_dim = edge_dim + keig
        self.initial_channel = self.filters[0]
        self.pool_loc = pool_loc
        self.att_mode = att_mode
        self.att_every_level = att_mode == "every"
        self.att_max_norm = att_max_norm
        self._deg_eps = deg_eps
        self.HL_init_conv = _hl_block(self.node_dim, self.edge_dim, self.initial_channel, init_K,
                                      dropout_ratio)
        gcn_insize = self.initial_channel
        for i, gcn_outsize in enumerate(self.filters):
            for j in range(self.channels[i]):
                setattr(self, "NEInt{}{}".format(i, j), NodeEdgeInt(d=gcn_insize, dv=gcn_outsize))
                setattr(self, "NEConv{}{}".format(i, j),
                        _hl_block(gcn_outsize, gcn_outsize, gcn_outsize, K, dropout_ratio))
                gcn_insize = gcn_insize + gcn_outsize
            if att_mode == "every" or (att_mode == "concat" and i == self.pool_loc):
                setattr(self, "NEAtt{}".format(i),
                        NodeEdgeInt(d=gcn_insize, dv=gcn_outsize, only_att=True, l=l))
            elif att_mode == "block" and i == self.pool_loc:
                setattr(self, "NEAtt{}".format(i),
                        NodeEdgeInt(d=gcn_outsize, dv=gcn_outsize, only_att=True,
                                    sigma=nn.ReLU(), l=l))
        mlp_insize = self.filters[-1] * 2
        for i, mlp_outsize in enumerate(mlp_channels):
            setattr(self, "mlp%d" % i, nn.Sequential(
                Linear(mlp_insize, mlp_outsize), nn.BatchNorm1d(mlp_outsize), nn.ReLU(),
                nn.Dropout(dropout_ratio_mlp)))
            mlp_insize = mlp_outsize
        self.out = Linear(mlp_insize, num_classes)

    def _slab_ends(self, i: int) -> bool:
        """Level i ends by scaling (att) or pooling x0: the next level starts
        a new dense slab."""
        return (self.att_mode == "every" or i == self.pool_loc
                or i == len(self.channels) - 1)

    def _run_width(self, i: int) -> int:
        """Columns the blocks of levels i..(the end of i's slab run) add."""
        w = 0
        for q in range(i, len(self.channels)):
            w += self.channels[q] * self.filters[q]
            if self._slab_ends(q):
                break
        return w

    def forward(self, datas, device="cuda:0", if_final_layer=False, if_att=False):
        d0 = datas[0]
        dev = d0.x_t.device
        # global coarse index of every fine node / edge (pos_ts / pos_ss);
        # not needed when the level list carries its cluster CSR (pool_tables)
        pos_t = pos_s = None
        if not _has_pool_tables(d0, dev):
            pos_t = d0.x_t[:, 0] + _level_offsets(datas[1].num_node1, d0.num_node1, dev,
                                                     d0.x_t.size(0))
            pos_s = d0.x_s[:, 0] + _level_offsets(datas[1].num_edge1, d0.num_edge1, dev,
                                                     d0.x_s.size(0))
        x_s, edge_index_s, edge_weight_s = d0.x_s[:, 1:], d0.edge_index_s, d0.edge_weight_s
        x_t, edge_index_t, edge_weight_t = d0.x_t[:, 1:], d0.edge_index_t, d0.edge_weight_t
        x_t, x_s = self.HL_init_conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                     edge_weight_s)
        x_t0, x_s0 = x_t, x_s
        k = 0
        par_1 = adj2par1(d0.edge_index, x_t0.shape[0], x_s0.shape[0])
        D = _node_degree(d0, x_t0.shape[0], x_t0.device) + self._deg_eps
        att_t = att_s = None
        dense = x_t.is_cuda and ops.DENSE_SLAB
        nxt = None  # the next run's slabs, already holding the pooled x0
        last = len(self.channels) - 1
        if x_t.is_cuda:
            # every NodeEdgeInt's first-Linear pack and the K|Q packs of the
            # NEAtts this forward uses: one launch each
            ops.nei_prepack([getattr(self, "NEInt{}{}".format(i, j))
                             for i, _ in enumerate(self.channels)
                             for j in range(self.channels[i])])
            ops.att_prepack([getattr(self, "NEAtt%d" % i) for i in range(len(self.channels))
                             if hasattr(self, "NEAtt%d" % i)
                             and (self.att_mode == "every" or i == self.pool_loc)])
        for i, _ in enumerate(self.channels):
            # one dense slab per run of levels: x0 (scaled / pooled) then the
            # blocks of every level up to the next scale or pool of x0 (levels
            # whose x0 passes unchanged continue the same slab: no re-copy)
            if dense and (i == 0 or self._slab_ends(i - 1)):
                if nxt is not None:
                    dt, ds = nxt
                    nxt = None
                else:
                    w = x_t0.size(1) + self._run_width(i)
                    dt = ops.DenseConcat(x_t0.size(0), w, x_t0)
                    ds = ops.DenseConcat(x_s0.size(0), w, x_s0)
                    dt.append(x_t0)
                    ds.append(x_s0)
            for j in range(self.channels[i]):
                neint = getattr(self, "NEInt{}{}".format(i, j))
                if dense:
                    x_t0, x_s0 = dt.view(), ds.view()
                    # its input gradients go straight into the slab's gradient
                    neint._hlhgat_gsink = (dt.grad_sink(), ds.grad_sink())
                x_t, x_s = neint(x_t0, x_s0, par_1, D)
                conv = getattr(self, "NEConv{}{}".format(i, j))
                if dense:
                    _sink(conv, dt, ds, self.filters[i])
                x_t, x_s = conv(x_t, edge_index_t, edge_weight_t, x_s, edge_index_s,
                                edge_weight_s)
                if dense:
                    dt.append(x_t)
                    ds.append(x_s)
                else:
                    x_t0 = torch.cat([x_t0, x_t], dim=-1)
                    x_s0 = torch.cat([x_s0, x_s], dim=-1)
            if dense and self._slab_ends(i):
                # (a continuing slab takes no view here: the first view taken
                # after a part is appended hands that part its gradient, so it
                # must be one the next level's NodeEdgeInt consumes)
                x_t0, x_s0 = dt.view(), ds.view()
            if self.att_mode == "every" or (self.att_mode == "concat" and i == self.pool_loc):
                att_t, att_s = getattr(self, "NEAtt%d" % i)(x_t0, x_s0, par_1, D)
                if i == last:
                    pass  # x0 is not part of the readout: the product is never read
                elif dense:
                    out_t = out_s = None
                    if i != self.pool_loc:
                        # the scaled x0 lands in the first columns of the next slabs
                        w = x_t0.size(1) + self._run_width(i + 1)
                        nt = ops.DenseConcat(x_t0.size(0), w, x_t0)
                        ns = ops.DenseConcat(x_s0.size(0), w, x_s0)
                        out_t, out_s = nt.sink(x_t0.size(1)), ns.sink(x_s0.size(1))
                    # fresh views, consumed by the product alone: its input
                    # gradient is written into the slab's gradient in place
                    x_t0 = ops.row_scale(dt.view(), att_t, out_t, dt.grad_sink())
                    x_s0 = ops.row_scale(ds.view(), att_s, out_s, ds.grad_sink())
                    if out_t is not None:
                        nt.append(x_t0)
                        ns.append(x_s0)
                        nxt = (nt, ns)
                else:
                    x_t0 = x_t0 * att_t
                    x_s0 = x_s0 * att_s
            if i == self.pool_loc:
                if self.att_mode == "block":
                    att_t, att_s = getattr(self, "NEAtt%d" % i)(x_t, x_s, par_1, D)
                    if self.att_max_norm:
                        # batch-global max (all ranks under data parallelism) over
                        # the real rows (padding rows of a static-shape level excluded)
                        dk = datas[k]
                        att_t = att_t / global_max(_valid_rows(att_t,
                                                               getattr(dk, "n_valid_t", None)))
                        att_s = att_s / global_max(_valid_rows(att_s,
                                                               getattr(dk, "n_valid_s", None)))
                    if i == last:
                        # below the last level the scaled block output is never
                        # read (the next level's first NEConv replaces x_t): the
                        # reference's product is dead there, att is still returned
                        x_t = x_t * att_t
                        x_s = x_s * att_s
                d1 = datas[k + 1]
                out_t = out_s = None
                if dense and i < last and pos_t is None:
                    # the pooled x0 lands in the first columns of the next run's slabs
                    w = x_t0.size(1) + self._run_width(i + 1)
                    nt = ops.DenseConcat(d1.x_t.shape[0], w, x_t0)
                    ns = ops.DenseConcat(d1.x_s.shape[0], w, x_s0)
                    out_t, out_s = nt.sink(x_t0.size(1)), ns.sink(x_s0.size(1))
                # block mode pools the slab view itself: its gradient goes
                # straight into the slab's gradient
                gk_t = gk_s = None
                if dense and self.att_mode == "block":
                    gk_t, gk_s = dt.grad_sink(), ds.grad_sink()
                x_t0 = _pool(x_t0, pos_t, d0, "t", d1.x_t.shape[0], out_t, gk_t)
                x_s0 = _pool(x_s0, pos_s, d0, "s", d1.x_s.shape[0], out_s, gk_s)  # inf dropped
                if out_t is not None:
                    nt.append(x_t0)
                    ns.append(x_s0)
                    nxt = (nt, ns)
                edge_index_s, edge_weight_s = d1.edge_index_s, d1.edge_weight_s
                edge_index_t, edge_weight_t = d1.edge_index_t, d1.edge_weight_t
                k = 1
                par_1 = adj2par1(d1.edge_index, x_t0.shape[0], x_s0.shape[0])
                D = _node_degree(d1, x_t0.shape[0], x_t0.device) + self._deg_eps
        dr = datas[min(len(self.channels) - 1, 1)]
        if x_t.size(0) != dr.x_t.size(0) or x_s.size(0) != dr.x_s.size(0):
            # the reference's readout (lib/Hodge_ST_Model.py:1076-1080) pools the
            # last block's rows by datas[min(i, 1)]'s graph sizes: a pool at the
            # last level (or none with >1 level) leaves them mismatched
            raise RuntimeError(
                f"hlhgat: attpool readout rows ({x_t.size(0)}, {x_s.size(0)}) do not match "
                f"level {min(len(self.channels) - 1, 1)}'s ({dr.x_t.size(0)}, {dr.x_s.size(0)}): "
                f"pool_loc={self.pool_loc} must be below the last of {len(self.channels)} levels")
        x = mean_pool_cat([(x_s, dr.num_edge1, getattr(dr, "seg_ptr_s", None)),
                           (x_t, dr.num_node1, getattr(dr, "seg_ptr_t", None))])
        x = run_mlp_stack([getattr(self, "mlp%d" % i) for i in range(len(self.mlp_channels))],
                          [x])
        y = ops.linear_blocks([x], self.out.weight, self.out.bias)
        if if_final_layer:
            return x, y
        if if_att:
            return y, att_t, att_s
        return y


class HL_HGCNN_CIFAR10SP_dense_int3_attpool(_AttPoolHead):
    """CIFAR10 superpixel classification head with attention pooling
    (lib/Hodge_ST_Model.py:958-1091; BASELINE config 3 runs it with
    channels=[2,2,2], filters=[64,128,256], mlp=[256], K=4, keig=10,
    pool_loc=1, l=0.5, main_cifar10SP...:186-187)."""

    def __init__(self, channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[], K=2,
                 node_dim=5, l=0.5, edge_dim=4, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, pool_loc=0, keig=10):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, pool_loc, keig, l, att_mode="block")


class HL_HGCNN_zinc_dense_int3_attpool(_AttPoolHead):
    """ZINC head with attention pooling (lib/Hodge_ST_Model.py:412-541): K-order
    initial convs, NEAtt (ReLU, l=0.9) at pool_loc on the level's last block
    output WITHOUT the batch-max division, degree without the 1e-6."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=21, edge_dim=3, num_classes=1, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, pool_loc=0, keig=7):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, pool_loc, keig, 0.9,
                         att_mode="block", att_max_norm=False, init_K=K, deg_eps=0.0)

    def forward(self, datas, device="cuda:0"):
        return super().forward(datas, device)


class HL_HGCNN_pepfunc_dense_int3_attpool(_AttPoolHead):
    """Peptides-func head of lib/Hodge_ST_Model.py:173-304: NEAtt (sigmoid,
    l=0.9) only at pool_loc, on the dense concatenation, which it scales
    before pooling.  The training script main_pepfunc_HL_HGCNN_dense_int3_attpool.py
    redefines a class of this name (NEAtt after every level, l=0.5; BASELINE
    config 4): hlhgat.main_pepfunc.HL_HGCNN_pepfunc_dense_int3_attpool, which
    is also what ``hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool`` names."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=9, edge_dim=3, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, pool_loc=0, keig=20):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, pool_loc, keig, 0.9,
                         att_mode="concat")

    def forward(self, datas, device="cuda:0"):
        return super().forward(datas, device)
