"""Torch-facing wrappers and autograd Functions over the HIP C-ABI.

Every op here runs a kernel from libhlhgat.so on the caller's current HIP
stream; there is no CPU or eager-PyTorch fallback (tensors must live on a ROCm
device, fp32, with the documented layouts).  The reference semantics each op
reproduces are cited per function (paths relative to deepika090/HL-HGAT).
"""
from __future__ import annotations

import ctypes as C
import math
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import _lib
from ._lib import LIB, check

__all__ = [
    "SparseCSR", "HodgeOperator", "Incidence", "hodge_operator", "incidence",
    "mark_hodge", "spmm", "poly_basis", "hodge_poly_conv", "linear_blocks",
    "node_from_edges", "edge_from_nodes", "att_score", "segment_mean",
    "POLY_LAGUERRE", "POLY_CHEB", "SIGMA_SIGMOID", "SIGMA_RELU",
]

POLY_LAGUERRE, POLY_CHEB = _lib.POLY_LAGUERRE, _lib.POLY_CHEB
SIGMA_SIGMOID, SIGMA_RELU = _lib.SIGMA_SIGMOID, _lib.SIGMA_RELU


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------
def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _req_dev(t: torch.Tensor, name: str, dtype=torch.float32) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"hlhgat: {name} must be on a ROCm device (got {t.device}); "
                           f"the HIP path has no CPU fallback")
    if t.dtype != dtype:
        raise RuntimeError(f"hlhgat: {name} must be {dtype} (got {t.dtype})")


def _rows2d(t: torch.Tensor, name: str) -> torch.Tensor:
    """Row-major 2-D view with unit inner stride (copy only if needed)."""
    if t.dim() != 2:
        raise RuntimeError(f"hlhgat: {name} must be 2-D (got {tuple(t.shape)})")
    if t.stride(1) != 1 or t.stride(0) < t.size(1):
        t = t.contiguous()
    return t


def _ld(t: torch.Tensor) -> int:
    return max(t.stride(0), t.size(1), 1)


def _arr(ctype, vals):
    return (ctype * len(vals))(*vals)


# ----------------------------------------------------------------------------
# sparse operators (CSR) and their per-batch cache
# ----------------------------------------------------------------------------
@dataclass
class SparseCSR:
    rowptr: torch.Tensor  # int32 [n_rows+1]
    col: torch.Tensor     # int32 [nnz]
    val: Optional[torch.Tensor]  # fp32 [nnz] or None (= ones)
    n_rows: int
    n_cols: int
    nnz: int


@dataclass
class HodgeOperator:
    """A Laplacian as used by propagate: fwd = CSR keyed by edge_index[1]
    (Y[t] = sum w * X[s]), bwd = its transpose (keyed by edge_index[0])."""
    fwd: SparseCSR
    bwd: SparseCSR


@dataclass
class Incidence:
    """|B1| of adj2par1 (lib/Hodge_Dataset.py:169-191) for edge_index [2, E]:
    per-node CSR over incident edge ids (ascending) plus the edge list."""
    rowptr: torch.Tensor    # int32 [n_nodes+1]
    edge_ids: torch.Tensor  # int32 [2E]
    edge_index: torch.Tensor  # int64 [2, E] contiguous
    n_nodes: int
    n_edges: int


class _IdCache:
    """Cache keyed on a tensor object's identity + version (entries die with
    the tensor), so a freed-and-reused allocation can never hit stale CSR."""

    def __init__(self):
        self._d = {}

    def get(self, key_tensors: Sequence[torch.Tensor], extra):
        k = (tuple(id(t) for t in key_tensors), extra)
        hit = self._d.get(k)
        if hit is None:
            return None
        versions, value = hit
        if versions != tuple(t._version for t in key_tensors):
            return None
        return value

    def put(self, key_tensors: Sequence[torch.Tensor], extra, value):
        k = (tuple(id(t) for t in key_tensors), extra)
        self._d[k] = (tuple(t._version for t in key_tensors), value)
        for t in key_tensors:
            weakref.finalize(t, self._d.pop, k, None)
        return value

    def clear(self):
        self._d.clear()


_HODGE_CACHE = _IdCache()
_INC_CACHE = _IdCache()


def clear_caches() -> None:
    _HODGE_CACHE.clear()
    _INC_CACHE.clear()


def mark_hodge(edge_index: torch.Tensor) -> torch.Tensor:
    """Declare that edge_index/edge_weight describe a symmetric operator whose
    COO is sorted by (row, col) — true for every Laplacian the Hodge builder
    emits via dense_to_sparse (lib/Hodge_Dataset.py:455-456,467-468) and for
    PairData batches of them (block-diagonal, offsets :40-48).  Enables the
    sort-free CSR build and reuse of one CSR for forward and adjoint."""
    edge_index._hlhgat_sorted_symmetric = True  # type: ignore[attr-defined]
    return edge_index


def _csr_sorted(row: torch.Tensor, col: torch.Tensor, w: Optional[torch.Tensor],
                n_rows: int, n_cols: int) -> SparseCSR:
    nnz = row.numel()
    dev = row.device
    rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    col32 = torch.empty(nnz, dtype=torch.int32, device=dev)
    val = torch.empty(nnz, dtype=torch.float32, device=dev) if w is not None else None
    check(LIB.hlhgat_csr_from_sorted_coo(row.data_ptr(), col.data_ptr(), _ptr(w), nnz,
                                         n_rows, rowptr.data_ptr(), col32.data_ptr(),
                                         _ptr(val), _stream(row)),
          "csr_from_sorted_coo")
    return SparseCSR(rowptr, col32, val, n_rows, n_cols, nnz)


def _csr_general(row: torch.Tensor, col: torch.Tensor, w: Optional[torch.Tensor],
                 n_rows: int, n_cols: int) -> SparseCSR:
    nnz = row.numel()
    dev = row.device
    rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    col32 = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
    val = (torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)[:nnz]
           if w is not None else None)
    ws_bytes = int(LIB.hlhgat_csr_workspace_bytes(nnz))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    check(LIB.hlhgat_csr_from_coo(row.data_ptr() if nnz else None,
                                  col.data_ptr() if nnz else None, _ptr(w), nnz, n_rows,
                                  max(n_cols, 1), rowptr.data_ptr(),
                                  col32.data_ptr() if nnz else None, _ptr(val) if nnz else None,
                                  None, ws.data_ptr(), ws_bytes, _stream(row)),
          "csr_from_coo")
    return SparseCSR(rowptr, col32, val, n_rows, n_cols, nnz)


def hodge_operator(edge_index: torch.Tensor, edge_weight: Optional[torch.Tensor],
                   n: int) -> HodgeOperator:
    """CSR pair for PyG propagate over (edge_index, edge_weight) on n nodes.

    propagate (source_to_target, aggr='add', message = norm*x_j,
    lib/Hodge_Cheb_Conv.py:518-519) computes Y[ei[1][e]] += w[e] * X[ei[0][e]],
    i.e. Y = A X with A keyed by ei[1]; its adjoint is keyed by ei[0]."""
    _req_dev(edge_index, "edge_index", torch.int64)
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise RuntimeError(f"hlhgat: edge_index must be [2, nnz] (got {tuple(edge_index.shape)})")
    if edge_weight is not None:
        _req_dev(edge_weight, "edge_weight")
        if edge_weight.numel() != edge_index.size(1):
            raise RuntimeError("hlhgat: edge_weight must have one entry per edge")
    keys = [edge_index] + ([edge_weight] if edge_weight is not None else [])
    hit = _HODGE_CACHE.get(keys, n)
    if hit is not None:
        return hit
    ei = edge_index.contiguous()
    w = edge_weight.contiguous() if edge_weight is not None else None
    if getattr(edge_index, "_hlhgat_sorted_symmetric", False):
        a = _csr_sorted(ei[0], ei[1], w, n, n)
        op = HodgeOperator(a, a)
    else:
        fwd = _csr_general(ei[1], ei[0], w, n, n)
        bwd = _csr_general(ei[0], ei[1], w, n, n)
        op = HodgeOperator(fwd, bwd)
    return _HODGE_CACHE.put(keys, n, op)


def incidence(edge_index: torch.Tensor, n_nodes: int) -> Incidence:
    """Incidence CSR of |B1| built from the undirected edge list (i<j)."""
    _req_dev(edge_index, "edge_index", torch.int64)
    hit = _INC_CACHE.get([edge_index], n_nodes)
    if hit is not None:
        return hit
    ei = edge_index.contiguous()
    E = ei.size(1)
    dev = ei.device
    rowptr = torch.empty(n_nodes + 1, dtype=torch.int32, device=dev)
    eids = torch.empty(max(2 * E, 1), dtype=torch.int32, device=dev)[:2 * E]
    ws_bytes = int(LIB.hlhgat_csr_workspace_bytes(2 * E))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    check(LIB.hlhgat_incidence_csr(ei.data_ptr() if E else None, E, n_nodes,
                                   rowptr.data_ptr(), eids.data_ptr() if E else None,
                                   ws.data_ptr(), ws_bytes, _stream(ei)),
          "incidence_csr")
    return _INC_CACHE.put([edge_index], n_nodes, Incidence(rowptr, eids, ei, n_nodes, E))


# ----------------------------------------------------------------------------
# raw launches
# ----------------------------------------------------------------------------
def _poly_step(A: SparseCSR, X: torch.Tensor, Y: torch.Tensor, *, rs=None, Z=None, P=None,
               Q=None, alpha=1.0, beta=0.0, gamma=0.0, div=1.0, p=0.0, q=0.0) -> None:
    d = X.size(1)
    check(LIB.hlhgat_poly_step(
        A.rowptr.data_ptr(), A.col.data_ptr() if A.nnz else None, _ptr(A.val) if A.nnz else None,
        _ptr(rs), A.n_rows, A.nnz, X.data_ptr(), _ld(X), d,
        _ptr(Z), _ld(Z) if Z is not None else 0, _ptr(P), _ld(P) if P is not None else 0,
        _ptr(Q), _ld(Q) if Q is not None else 0, alpha, beta, gamma, div, p, q,
        Y.data_ptr(), _ld(Y), _stream(X)), "poly_step")


def spmm(A: SparseCSR, X: torch.Tensor) -> torch.Tensor:
    """Y = A X (no autograd); PyG propagate when A = hodge_operator(...).fwd."""
    _req_dev(X, "X")
    X = _rows2d(X, "X")
    Y = torch.empty(A.n_rows, X.size(1), device=X.device, dtype=X.dtype)
    if A.n_rows:
        check(LIB.hlhgat_spmm(A.rowptr.data_ptr(), A.col.data_ptr() if A.nnz else None,
                              _ptr(A.val) if A.nnz else None, A.n_rows, A.nnz,
                              X.data_ptr(), _ld(X), X.size(1), Y.data_ptr(), _ld(Y),
                              _stream(X)), "spmm")
    return Y


def poly_basis(op: HodgeOperator, X: torch.Tensor, K: int, kind: int) -> torch.Tensor:
    """T_1..T_{K-1} as a [K-1, n, F] slab (no autograd)."""
    n, F = X.size(0), X.size(1)
    T = torch.empty(max(K - 1, 0), n, F, device=X.device, dtype=X.dtype)
    if K > 1 and n > 0:
        A = op.fwd
        check(LIB.hlhgat_poly_basis_fwd(kind, A.rowptr.data_ptr(),
                                        A.col.data_ptr() if A.nnz else None,
                                        _ptr(A.val) if A.nnz else None, n, A.nnz,
                                        X.data_ptr(), _ld(X), F, K, T.data_ptr(),
                                        _stream(X)), "poly_basis_fwd")
    return T


def _proj_fwd(As: List[torch.Tensor], Ws: List[torch.Tensor], M: int, N: int,
              bias: Optional[torch.Tensor], out: torch.Tensor, accumulate=False) -> None:
    nb = len(As)
    check(LIB.hlhgat_proj_fwd(
        nb, _arr(C.c_void_p, [a.data_ptr() for a in As]), _arr(C.c_int64, [_ld(a) for a in As]),
        _arr(C.c_void_p, [w.data_ptr() for w in Ws]), _arr(C.c_int64, [w.stride(0) for w in Ws]),
        _arr(C.c_int64, [a.size(1) for a in As]), M, N, _ptr(bias), out.data_ptr(), _ld(out),
        int(accumulate), _stream(out)), "proj_fwd")


def _proj_bwd_data(G: torch.Tensor, Ws: List[torch.Tensor], kbs: List[int],
                   dAs: List[torch.Tensor], accumulate=False) -> None:
    nb = len(Ws)
    check(LIB.hlhgat_proj_bwd_data(
        nb, G.data_ptr(), _ld(G), _arr(C.c_void_p, [w.data_ptr() for w in Ws]),
        _arr(C.c_int64, [w.stride(0) for w in Ws]), _arr(C.c_int64, kbs), G.size(0), G.size(1),
        _arr(C.c_void_p, [d.data_ptr() for d in dAs]), _arr(C.c_int64, [_ld(d) for d in dAs]),
        int(accumulate), _stream(G)), "proj_bwd_data")


def _proj_bwd_weight(G: torch.Tensor, As: List[torch.Tensor], dWs: List[torch.Tensor],
                     dbias: Optional[torch.Tensor]) -> None:
    nb = len(As)
    kb = _arr(C.c_int64, [a.size(1) for a in As])
    M, N = G.size(0), G.size(1)
    wsf = int(LIB.hlhgat_proj_bwd_weight_workspace_floats(nb, kb, M, N, int(dbias is not None)))
    ws = torch.empty(max(wsf, 1), device=G.device, dtype=torch.float32)
    check(LIB.hlhgat_proj_bwd_weight(
        nb, G.data_ptr(), _ld(G), _arr(C.c_void_p, [a.data_ptr() for a in As]),
        _arr(C.c_int64, [_ld(a) for a in As]), kb, M, N,
        _arr(C.c_void_p, [d.data_ptr() for d in dWs]), _arr(C.c_int64, [d.stride(0) for d in dWs]),
        _ptr(dbias), 0, ws.data_ptr(), wsf, _stream(G)), "proj_bwd_weight")


# ----------------------------------------------------------------------------
# HodgeLaguerreConv / HodgeChebConv fused forward + hand-written backward
# ----------------------------------------------------------------------------
class _HodgePolyConvFn(torch.autograd.Function):
    """out = sum_k T_k W_k^T + bias with T_k the Laguerre / Chebyshev basis of
    x over L (lib/Hodge_Cheb_Conv.py:480-515 / :394-439).  x may be [N, C] or
    [N, T, C] (3-D inputs propagate over [N, T*C] rows, :493-505)."""

    @staticmethod
    def forward(ctx, x, op, kind, bias, *weights):
        K = len(weights)
        N = x.size(0)
        C_in = x.size(-1)
        xf = x.reshape(N, -1)
        if xf.stride(-1) != 1:
            xf = xf.contiguous()
        F = xf.size(1)
        T = poly_basis(op, xf, K, kind)  # [K-1, N, F]
        M = xf.numel() // C_in if N else 0
        dout = weights[0].size(0)
        out = torch.empty(M, dout, device=x.device, dtype=x.dtype)
        As = [xf.reshape(M, C_in)] + [T[k].view(M, C_in) for k in range(K - 1)]
        if M > 0:
            _proj_fwd(As, list(weights), M, dout, bias, out)
        elif bias is not None:
            out.copy_(bias.expand_as(out))
        ctx.op, ctx.kind, ctx.K = op, kind, K
        ctx.shape = (x.shape, N, F, M, C_in, dout)
        ctx.has_bias = bias is not None
        ctx.save_for_backward(xf, T, *weights)
        return out.view(*x.shape[:-1], dout)

    @staticmethod
    def backward(ctx, gout):
        xf, T, *weights = ctx.saved_tensors
        xshape, N, F, M, C_in, dout = ctx.shape
        K = ctx.K
        G = gout.reshape(M, dout)
        if G.stride(-1) != 1 or G.stride(0) != dout:
            G = G.contiguous()
        need_x = ctx.needs_input_grad[0]
        need_b = ctx.has_bias and ctx.needs_input_grad[3]
        need_w = any(ctx.needs_input_grad[4:])
        gx = gb = None
        gws = [None] * K
        As = [xf.reshape(M, C_in)] + [T[k].view(M, C_in) for k in range(K - 1)]
        if (need_w or need_b) and M > 0:
            dWs = [torch.empty_like(w) for w in weights]
            gb = torch.empty(dout, device=G.device, dtype=G.dtype) if need_b else None
            _proj_bwd_weight(G, As, dWs, gb)
            gws = dWs if need_w else gws
        elif need_w or need_b:
            gws = [torch.zeros_like(w) for w in weights]
            gb = torch.zeros(dout, device=G.device, dtype=G.dtype) if need_b else None
        if need_x:
            Gs = torch.empty(K, N, F, device=G.device, dtype=G.dtype)
            if M > 0:
                _proj_bwd_data(G, list(weights), [C_in] * K,
                               [Gs[k].view(M, C_in) for k in range(K)])
                if K > 1:
                    B = ctx.op.bwd
                    check(LIB.hlhgat_poly_basis_bwd(
                        ctx.kind, B.rowptr.data_ptr(), B.col.data_ptr() if B.nnz else None,
                        _ptr(B.val) if B.nnz else None, N, B.nnz, F, K, Gs.data_ptr(),
                        _stream(G)), "poly_basis_bwd")
            else:
                Gs.zero_()
            gx = Gs[0].view(xshape)
        return (gx, None, None, gb, *gws)


def hodge_poly_conv(x: torch.Tensor, op: HodgeOperator, weights: Sequence[torch.Tensor],
                    bias: Optional[torch.Tensor], kind: int = POLY_LAGUERRE) -> torch.Tensor:
    _req_dev(x, "x")
    for w in weights:
        _req_dev(w, "lins[k].weight")
        if w.stride(-1) != 1:
            raise RuntimeError("hlhgat: weights must have unit inner stride")
    if bias is not None:
        _req_dev(bias, "bias")
    if x.size(0) != op.fwd.n_rows:
        raise RuntimeError(f"hlhgat: x has {x.size(0)} rows but the operator has "
                           f"{op.fwd.n_rows}")
    return _HodgePolyConvFn.apply(x, op, kind, bias, *weights)


# ----------------------------------------------------------------------------
# Linear over a split reduction axis (Linear(cat[a, b]) without the cat)
# ----------------------------------------------------------------------------
class _LinearBlocksFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, bias, *As):
        M = As[0].size(0)
        N = weight.size(0)
        offs, Ws = [], []
        o = 0
        for a in As:
            offs.append(o)
            Ws.append(weight[:, o:o + a.size(1)])
            o += a.size(1)
        if o != weight.size(1):
            raise RuntimeError(f"hlhgat: Linear expects {weight.size(1)} input features, "
                               f"got {o}")
        out = torch.empty(M, N, device=weight.device, dtype=weight.dtype)
        if M > 0:
            _proj_fwd(list(As), Ws, M, N, bias, out)
        ctx.has_bias = bias is not None
        ctx.save_for_backward(weight, *As)
        return out

    @staticmethod
    def backward(ctx, gout):
        weight, *As = ctx.saved_tensors
        G = gout if (gout.stride(-1) == 1 and gout.stride(0) == gout.size(1)) else gout.contiguous()
        M, N = G.size(0), G.size(1)
        kbs = [a.size(1) for a in As]
        Ws, o = [], 0
        for k in kbs:
            Ws.append(weight[:, o:o + k])
            o += k
        gw = gb = None
        need_b = ctx.has_bias and ctx.needs_input_grad[1]
        if ctx.needs_input_grad[0] or need_b:
            if M > 0:
                gw = torch.empty_like(weight)
                dWs, o = [], 0
                for k in kbs:
                    dWs.append(gw[:, o:o + k])
                    o += k
                gb = torch.empty(N, device=G.device, dtype=G.dtype) if need_b else None
                _proj_bwd_weight(G, list(As), dWs, gb)
            else:
                gw = torch.zeros_like(weight)
                gb = torch.zeros(N, device=G.device, dtype=G.dtype) if need_b else None
            if not ctx.needs_input_grad[0]:
                gw = None
        gAs = [None] * len(As)
        need_a = [ctx.needs_input_grad[2 + i] for i in range(len(As))]
        if any(need_a) and M > 0:
            idx = [i for i in range(len(As)) if need_a[i]]
            outs = [torch.empty(M, kbs[i], device=G.device, dtype=G.dtype) for i in idx]
            _proj_bwd_data(G, [Ws[i] for i in idx], [kbs[i] for i in idx], outs)
            for i, t in zip(idx, outs):
                gAs[i] = t
        elif any(need_a):
            gAs = [torch.zeros_like(a) if n else None for a, n in zip(As, need_a)]
        return (gw, gb, *gAs)


def linear_blocks(As: Sequence[torch.Tensor], weight: torch.Tensor,
                  bias: Optional[torch.Tensor]) -> torch.Tensor:
    """F.linear(cat(As, -1), weight, bias) with the concatenation folded into
    the MFMA GEMM's reduction axis (lib/Hodge_Cheb_Conv.py:307-308)."""
    if len(As) > _lib.MAX_BLOCKS:
        raise RuntimeError(f"hlhgat: at most {_lib.MAX_BLOCKS} operand blocks")
    _req_dev(weight, "weight")
    if weight.stride(-1) != 1:
        weight = weight.contiguous()
    fixed = []
    for a in As:
        _req_dev(a, "input")
        fixed.append(_rows2d(a, "input"))
    return _LinearBlocksFn.apply(weight, bias, *fixed)


# ----------------------------------------------------------------------------
# boundary operator: x_s2t = (1/D) |B1| x_s ; x_t2s = |B1|^T x_t / 2
# ----------------------------------------------------------------------------
class _NodeFromEdgesFn(torch.autograd.Function):
    """x_s2t = (1/D).view(-1,1) * (|B1| @ x_s)   (lib/Hodge_Cheb_Conv.py:294)."""

    @staticmethod
    def forward(ctx, x_s, inc, rD):
        out = torch.empty(inc.n_nodes, x_s.size(1), device=x_s.device, dtype=x_s.dtype)
        A = SparseCSR(inc.rowptr, inc.edge_ids, None, inc.n_nodes, inc.n_edges, 2 * inc.n_edges)
        if inc.n_nodes:
            _poly_step(A, x_s, out, rs=rD)
        ctx.inc = inc
        ctx.save_for_backward(rD)
        return out

    @staticmethod
    def backward(ctx, g):
        (rD,) = ctx.saved_tensors
        inc = ctx.inc
        g = _rows2d(g, "grad")
        gx = torch.empty(inc.n_edges, g.size(1), device=g.device, dtype=g.dtype)
        if inc.n_edges:
            # d x_s[e] = rD[i] g[i] + rD[j] g[j]
            check(LIB.hlhgat_edge_gather2(inc.edge_index.data_ptr(), inc.n_edges, g.data_ptr(),
                                          _ld(g), g.size(1), rD.data_ptr(), rD.data_ptr(),
                                          1.0, 1.0, gx.data_ptr(), _ld(gx), 0, _stream(g)),
                  "edge_gather2")
        return gx, None, None


class _EdgeFromNodesFn(torch.autograd.Function):
    """x_t2s = (|B1|^T @ x_t) / 2   (lib/Hodge_Cheb_Conv.py:295)."""

    @staticmethod
    def forward(ctx, x_t, inc):
        out = torch.empty(inc.n_edges, x_t.size(1), device=x_t.device, dtype=x_t.dtype)
        if inc.n_edges:
            check(LIB.hlhgat_edge_gather2(inc.edge_index.data_ptr(), inc.n_edges, x_t.data_ptr(),
                                          _ld(x_t), x_t.size(1), None, None, 0.5, 0.5,
                                          out.data_ptr(), _ld(out), 0, _stream(x_t)),
                  "edge_gather2")
        ctx.inc = inc
        return out

    @staticmethod
    def backward(ctx, g):
        inc = ctx.inc
        g = _rows2d(g, "grad")
        gx = torch.empty(inc.n_nodes, g.size(1), device=g.device, dtype=g.dtype)
        A = SparseCSR(inc.rowptr, inc.edge_ids, None, inc.n_nodes, inc.n_edges, 2 * inc.n_edges)
        if inc.n_nodes:
            _poly_step(A, g, gx, alpha=0.5)
        return gx, None


def node_from_edges(x_s: torch.Tensor, inc: Incidence, rD: torch.Tensor) -> torch.Tensor:
    _req_dev(x_s, "x_s")
    _req_dev(rD, "1/D")
    if x_s.size(0) != inc.n_edges:
        raise RuntimeError(f"hlhgat: x_s has {x_s.size(0)} rows, |B1| has {inc.n_edges} edges")
    if rD.numel() != inc.n_nodes:
        raise RuntimeError(f"hlhgat: D has {rD.numel()} entries, |B1| has {inc.n_nodes} nodes")
    return _NodeFromEdgesFn.apply(_rows2d(x_s, "x_s"), inc, rD.contiguous().view(-1))


def edge_from_nodes(x_t: torch.Tensor, inc: Incidence) -> torch.Tensor:
    _req_dev(x_t, "x_t")
    if x_t.size(0) != inc.n_nodes:
        raise RuntimeError(f"hlhgat: x_t has {x_t.size(0)} rows, |B1| has {inc.n_nodes} nodes")
    return _EdgeFromNodesFn.apply(_rows2d(x_t, "x_t"), inc)


# ----------------------------------------------------------------------------
# only_att score
# ----------------------------------------------------------------------------
class _AttScoreFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Qc, Qs, Kr, w_cross, w_self, sqrt_dk, sigma):
        n, dk = Kr.size(0), Kr.size(1)
        a = torch.empty(n, 1, device=Kr.device, dtype=Kr.dtype)
        check(LIB.hlhgat_att_score_fwd(n, dk, Qc.data_ptr(), _ld(Qc), Qs.data_ptr(), _ld(Qs),
                                       Kr.data_ptr(), _ld(Kr), w_cross, w_self, sqrt_dk, sigma,
                                       a.data_ptr(), _stream(Kr)), "att_score_fwd")
        ctx.consts = (w_cross, w_self, sqrt_dk, sigma)
        ctx.save_for_backward(Qc, Qs, Kr, a)
        return a

    @staticmethod
    def backward(ctx, ga):
        Qc, Qs, Kr, a = ctx.saved_tensors
        w_cross, w_self, sqrt_dk, sigma = ctx.consts
        n, dk = Kr.size(0), Kr.size(1)
        ga = ga.contiguous()
        g = torch.empty(3, n, dk, device=Kr.device, dtype=Kr.dtype)
        check(LIB.hlhgat_att_score_bwd(n, dk, Qc.data_ptr(), _ld(Qc), Qs.data_ptr(), _ld(Qs),
                                       Kr.data_ptr(), _ld(Kr), w_cross, w_self, sqrt_dk, sigma,
                                       a.data_ptr(), ga.data_ptr(), g[0].data_ptr(),
                                       g[1].data_ptr(), g[2].data_ptr(), dk, _stream(Kr)),
              "att_score_bwd")
        return g[0], g[1], g[2], None, None, None, None


def att_score(Qc, Qs, Kr, w_cross: float, w_self: float, sqrt_dk: float,
              sigma: int) -> torch.Tensor:
    """sigma((w_cross<Qc,K> + w_self<Qs,K>)/sqrt_dk) per row -> [n, 1]
    (lib/Hodge_Cheb_Conv.py:299-304)."""
    for t, nm in ((Qc, "Qc"), (Qs, "Qs"), (Kr, "K")):
        _req_dev(t, nm)
    return _AttScoreFn.apply(_rows2d(Qc, "Qc"), _rows2d(Qs, "Qs"), _rows2d(Kr, "K"),
                             float(w_cross), float(w_self), float(sqrt_dk), int(sigma))


# ----------------------------------------------------------------------------
# segment mean (global_mean_pool / scatter_mean over sorted or listed members)
# ----------------------------------------------------------------------------
class _SegmentMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seg_ptr, seg_rows, n_seg):
        d = x.size(1)
        out = torch.empty(n_seg, d, device=x.device, dtype=x.dtype)
        check(LIB.hlhgat_segment_mean_fwd(seg_ptr.data_ptr(), _ptr(seg_rows), n_seg,
                                          x.data_ptr(), _ld(x), d, out.data_ptr(), _ld(out),
                                          _stream(x)), "segment_mean_fwd")
        ctx.meta = (x.size(0), n_seg, seg_rows is not None)
        ctx.save_for_backward(seg_ptr, seg_rows if seg_rows is not None else seg_ptr)
        return out

    @staticmethod
    def backward(ctx, g):
        seg_ptr, seg_rows = ctx.saved_tensors
        n_rows, n_seg, listed = ctx.meta
        g = _rows2d(g, "grad")
        gx = (torch.zeros if listed else torch.empty)(n_rows, g.size(1), device=g.device,
                                                      dtype=g.dtype)
        check(LIB.hlhgat_segment_mean_bwd(seg_ptr.data_ptr(), _ptr(seg_rows) if listed else None,
                                          n_seg, g.data_ptr(), _ld(g), g.size(1), gx.data_ptr(),
                                          _ld(gx), _stream(g)), "segment_mean_bwd")
        return gx, None, None, None


def segment_mean(x: torch.Tensor, seg_ptr: torch.Tensor, n_seg: int,
                 seg_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Mean of x rows per segment.  seg_ptr int32 [n_seg+1]; members are the
    contiguous rows seg_ptr[s]..seg_ptr[s+1] (global_mean_pool over a sorted
    batch vector) or seg_rows[seg_ptr[s]:seg_ptr[s+1]] (scatter_mean)."""
    _req_dev(x, "x")
    _req_dev(seg_ptr, "seg_ptr", torch.int32)
    if seg_rows is not None:
        _req_dev(seg_rows, "seg_rows", torch.int32)
    return _SegmentMeanFn.apply(_rows2d(x, "x"), seg_ptr, seg_rows, int(n_seg))


# ----------------------------------------------------------------------------
# BatchNorm1d (training statistics) + optional fused ReLU
# ----------------------------------------------------------------------------
_BN_WS = {}


def _bn_workspace(device: torch.device, n: int, C: int) -> torch.Tensor:
    """Persistent zero-initialised scratch per device (the kernels leave their
    arrival counters at zero, so it is reused by every BN launch on the
    stream)."""
    need = int(LIB.hlhgat_bn_workspace_bytes(n, C))
    key = (device.type, device.index)
    ws = _BN_WS.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.zeros(max(need, 1 << 20), dtype=torch.uint8, device=device)
        _BN_WS[key] = ws
    return ws


class _BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum, eps, relu):
        n, C = x.shape
        y = torch.empty(n, C, device=x.device, dtype=x.dtype)
        mean = torch.empty(C, device=x.device, dtype=torch.float32)
        invstd = torch.empty(C, device=x.device, dtype=torch.float32)
        ws = _bn_workspace(x.device, n, C)
        check(LIB.hlhgat_bn_fwd_train(x.data_ptr(), _ld(x), n, C, _ptr(weight), _ptr(bias),
                                      _ptr(running_mean), _ptr(running_var), _ptr(nbt),
                                      momentum, eps, int(relu), y.data_ptr(), _ld(y),
                                      mean.data_ptr(), invstd.data_ptr(), ws.data_ptr(),
                                      ws.numel(), _stream(x)), "bn_fwd_train")
        ctx.relu = relu
        ctx.save_for_backward(x, y if relu else None, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, mean, invstd = ctx.saved_tensors
        dy = _rows2d(dy, "grad")
        n, C = x.shape
        dx = torch.empty(n, C, device=x.device, dtype=x.dtype)
        need_w = weight is not None and ctx.needs_input_grad[1]
        need_b = ctx.needs_input_grad[2]
        dw = torch.empty(C, device=x.device, dtype=x.dtype) if need_w else None
        db = torch.empty(C, device=x.device, dtype=x.dtype) if need_b else None
        ws = _bn_workspace(x.device, n, C)
        check(LIB.hlhgat_bn_bwd_train(x.data_ptr(), _ld(x), _ptr(y), _ld(y) if y is not None else 0,
                                      dy.data_ptr(), _ld(dy), n, C, _ptr(weight), mean.data_ptr(),
                                      invstd.data_ptr(), dx.data_ptr(), _ld(dx), _ptr(dw),
                                      _ptr(db), ws.data_ptr(), ws.numel(), _stream(x)),
              "bn_bwd_train")
        return dx, dw, db, None, None, None, None, None, None


def batch_norm_act(x: torch.Tensor, bn: torch.nn.BatchNorm1d, relu: bool = False) -> torch.Tensor:
    """bn(x) followed by ReLU when ``relu``; training mode (or no running
    stats) uses the HIP batch-statistics kernels, eval mode the running
    statistics (ATen's fused eval kernel)."""
    _req_dev(x, "x")
    if x.dim() != 2:
        raise RuntimeError("hlhgat: batch_norm_act expects [N, C] input")
    use_batch = bn.training or not bn.track_running_stats
    if not use_batch:
        y = torch.nn.functional.batch_norm(x, bn.running_mean, bn.running_var, bn.weight,
                                           bn.bias, False, 0.0, bn.eps)
        return torch.relu(y) if relu else y
    if x.size(0) < 2 and bn.training:
        raise ValueError(f"Expected more than 1 value per channel when training, got input "
                         f"size {tuple(x.shape)}")
    track = bn.training and bn.track_running_stats and bn.running_mean is not None
    if track and bn.momentum is None:
        momentum = 1.0 / float(bn.num_batches_tracked.item() + 1)
    else:
        momentum = float(bn.momentum) if bn.momentum is not None else 0.0
    return _BatchNormActFn.apply(
        _rows2d(x, "x"), bn.weight, bn.bias, bn.running_mean if track else None,
        bn.running_var if track else None, bn.num_batches_tracked if track else None,
        momentum, float(bn.eps), bool(relu))


# ----------------------------------------------------------------------------
# live kernel timing (bench.py)
# ----------------------------------------------------------------------------
def prof_enable(kernel_class: int, enable: bool = True) -> None:
    check(LIB.hlhgat_prof_enable(kernel_class, int(enable)), "prof_enable")


def prof_reset() -> None:
    check(LIB.hlhgat_prof_reset(), "prof_reset")


def prof_read(kernel_class: int):
    n = C.c_int64()
    ms, b, f = C.c_double(), C.c_double(), C.c_double()
    check(LIB.hlhgat_prof_read(kernel_class, C.byref(n), C.byref(ms), C.byref(b), C.byref(f)),
          "prof_read")
    return {"launches": n.value, "ms": ms.value, "bytes": b.value, "flops": f.value}
