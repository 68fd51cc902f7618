"""Simplex-graph layout (PairData), PyG-free batching and the boundary operator.

Mirrors lib/Hodge_Dataset.py of the reference:
  * PairData and its batching offsets (:27-48): x_t [N_t, F_t], x_s [N_s, F_s],
    edge_index_t / edge_weight_t = COO of L0, edge_index_s / edge_weight_s = COO
    of L1 (diagonal included, row-major sorted), edge_index = B1 columns (i<j),
    num_node1 / num_edge1 / num_nodes, y.  On collation edge_index_s is
    shifted by N_s, edge_index_t and edge_index by N_t.
  * adj2par1 (:169-191) -> BoundaryOperator (|B1| as a lazily built incidence
    CSR instead of an uncoalesced torch sparse COO).
  * the Hodge builder of the ZINC process() (:447-470): L0 = 2 B1 B1^T / lmax,
    L1 = 2 B1^T B1 / lmax, dense_to_sparse row-major COO.
Host-side code (numpy / torch CPU), run once per graph outside the hot loop.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import os

import numpy as np
import torch

__all__ = ["PairData", "Batch", "collate", "adj2par1", "BoundaryOperator", "degree",
           "hodge_laplacians", "dense_to_sparse", "is_sorted_symmetric", "locality_order",
           "static_caps", "pad_batch", "level_caps", "pad_levels", "PackedGraphs", "halo_tiles", "graclus", "mlgc", "mlgc_weighted", "mlgc_map", "to_undirected_mean",
           "hodge_factor_ok", "hodge_coo_from_boundary"]

_INC_KEYS = ("edge_index_s", "edge_index_t", "edge_index", "row_order_s", "row_order_t")
_HODGE_KEYS = ("edge_index_s", "edge_index_t")


class PairData:
    """One simplex graph (lib/Hodge_Dataset.py:27-38)."""

    def __init__(self, edge_index_s=None, x_s=None, edge_index_t=None, x_t=None,
                 edge_weight_s=None, edge_weight_t=None, edge_index=None, y=None, **kw):
        self.edge_index_s = edge_index_s
        self.x_s = x_s
        self.edge_index_t = edge_index_t
        self.x_t = x_t
        self.edge_weight_s = edge_weight_s
        self.edge_weight_t = edge_weight_t
        self.edge_index = edge_index
        self.y = y
        for k, v in kw.items():
            setattr(self, k, v)

    def __inc__(self, key: str, value=None) -> int:
        """Batching offset per key (lib/Hodge_Dataset.py:40-48)."""
        if key in ("edge_index_s", "row_order_s"):
            return self.x_s.size(0)
        if key in ("edge_index", "edge_index_t", "row_order_t"):
            return self.x_t.size(0)
        return 0

    def keys(self) -> List[str]:
        return [k for k, v in self.__dict__.items() if v is not None and not k.startswith("_")]

    def to(self, device):
        for k in self.keys():
            v = getattr(self, k)
            if torch.is_tensor(v):
                setattr(self, k, v.to(device))
        return self

    def __repr__(self) -> str:
        parts = []
        for k in self.keys():
            v = getattr(self, k)
            parts.append(f"{k}={list(v.shape)}" if torch.is_tensor(v) else f"{k}={v}")
        return f"PairData({', '.join(parts)})"


class Batch(PairData):
    """A collated mini-batch of PairData graphs.

    Per-graph scalars (num_node1, num_edge1) become int64 tensors [B] as PyG
    collation does; ``hodge_sorted`` records which Laplacian COO blocks are
    row-major sorted and symmetric so the device path can build CSR without a
    sort (ops.mark_hodge)."""

    num_graphs: int
    hodge_sorted: Dict[str, bool]

    def to(self, device, non_blocking: bool = False):
        self._check_counts()
        for k in self.keys():
            v = getattr(self, k)
            if torch.is_tensor(v):
                setattr(self, k, v.to(device, non_blocking=non_blocking))
        self._mark()
        return self

    def _check_counts(self) -> None:
        """Per-graph row counts must not exceed the row count: the forward's
        repeat_interleave(..., output_size=rows) (no host sync, capturable)
        trusts it, and a larger sum would write past the output.  Checked on
        the host copy only (never a device sync); rows beyond the sum are
        padding and are allowed."""
        for kc, kx in (("num_node1", "x_t"), ("num_edge1", "x_s")):
            c, x = getattr(self, kc, None), getattr(self, kx, None)
            if torch.is_tensor(c) and torch.is_tensor(x) and not c.is_cuda:
                tot = int(c.sum())
                if tot > x.shape[0]:
                    raise ValueError(f"Batch.{kc} sums to {tot} but {kx} has "
                                     f"{x.shape[0]} rows")

    def _mark(self) -> None:
        from . import ops
        from .ops import mark_hodge, set_halo, set_row_order, set_valid
        for k, ok in (getattr(self, "hodge_sorted", None) or {}).items():
            t = getattr(self, k, None)
            if ok and torch.is_tensor(t) and t.is_cuda:
                mark_hodge(t)
        for k, ko, kv in (("edge_index_s", "row_order_s", "n_valid_s"),
                          ("edge_index_t", "row_order_t", "n_valid_t")):
            t, o = getattr(self, k, None), getattr(self, ko, None)
            nv = getattr(self, kv, None)
            if torch.is_tensor(t) and t.is_cuda and torch.is_tensor(o):
                set_row_order(t, o)
            if torch.is_tensor(t) and t.is_cuda and torch.is_tensor(nv):
                set_valid(t, nv)
            side = k[-1]
            hk = {h: getattr(self, h + "_" + side, None) for h in _HALO_KEYS + ("halo_bounds",)}
            if (torch.is_tensor(t) and t.is_cuda and all(torch.is_tensor(v) for v in hk.values())
                    and self.hodge_sorted.get(k, False)):
                set_halo(t, hk)
        ei = getattr(self, "edge_index", None)
        eis = getattr(self, "edge_index_s", None)
        if (getattr(self, "l1_factor", False) and torch.is_tensor(ei) and ei.is_cuda
                and torch.is_tensor(eis) and eis.is_cuda):
            tabs = tuple(getattr(self, k, None) for k in ("fac_alpha", "fac_sign", "fac_ends"))
            tabs = tabs if all(torch.is_tensor(t) and t.is_cuda for t in tabs) else None
            ops.set_hodge_factor(eis, ei, self.x_t.size(0), getattr(self, "row_order_t", None),
                                 tables=tabs)
            if tabs is not None:
                # the factor's signed B1 values are the incidence CSR's signs
                # (ops._incidence_signs) -- not rebuilt on the device per step
                ei._hlhgat_inc_signs = tabs[1]
        for side in ("t", "s"):
            k = "edge_index_" + side
            t = getattr(self, k, None)
            rp, col = getattr(self, "csr_rowptr_" + side, None), getattr(self, "csr_col_" + side, None)
            if (torch.is_tensor(t) and t.is_cuda and torch.is_tensor(rp) and torch.is_tensor(col)
                    and self.hodge_sorted.get(k, False)):
                ops.set_csr(t, rp, col)
        ip, ie = getattr(self, "inc_rowptr", None), getattr(self, "inc_eids", None)
        if torch.is_tensor(ei) and ei.is_cuda and torch.is_tensor(ip) and torch.is_tensor(ie):
            ops.set_incidence(ei, ip, ie)
        dg, rdg = getattr(self, "deg_t", None), getattr(self, "inv_deg_t", None)
        if torch.is_tensor(dg) and dg.is_cuda and torch.is_tensor(rdg):
            dg._hlhgat_rcp = rdg  # ops.reciprocal(deg_t) without a launch
        if torch.is_tensor(ei) and ei.is_cuda:
            for kv in ("n_valid_t", "n_valid_s"):
                nv = getattr(self, kv, None)
                if torch.is_tensor(nv):
                    set_valid(ei, nv, "_hlhgat_valid_" + kv[-1])

    @property
    def batch_t(self) -> torch.Tensor:
        return torch.repeat_interleave(torch.arange(self.num_graphs, device=self.x_t.device),
                                       self.num_node1.to(self.x_t.device))

    @property
    def batch_s(self) -> torch.Tensor:
        return torch.repeat_interleave(torch.arange(self.num_graphs, device=self.x_s.device),
                                       self.num_edge1.to(self.x_s.device))


def locality_order(edge_index, n: int) -> torch.Tensor:
    """Row schedule for the SpMM of a large Laplacian: reverse Cuthill-McKee
    order of its sparsity pattern (int64 permutation of range(n)).

    Rows visited in this order share most of their neighbours with the rows
    visited just before them, so each XCD's L2 (the kernel walks one
    contiguous range of the schedule per XCD) serves the gathers that a
    natural order would send to the Infinity Cache.  A schedule only: results
    are bitwise those of the natural order (hlhgat_spmm, row_order).  Built
    once per graph with the Hodge Laplacians (host side, like
    lib/Hodge_Dataset.py:451-468)."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    ei = np.asarray(edge_index)
    A = sp.csr_matrix((np.ones(ei.shape[1], dtype=np.int8), (ei[0], ei[1])), shape=(n, n))
    return torch.from_numpy(reverse_cuthill_mckee(A, symmetric_mode=True).astype(np.int64))


# Halo-tile bounds: measured on the config-5 L1 (tools/tsp_spmm.py,
# profiles/r01_g_tsp_spmm.log) small tiles win -- 24 rows, <= 160 halo rows
# (a 20 KB LDS image at 32 floats) and <= 768 entries: 256-thread workgroups,
# several per CU, whose load latency overlaps; 128-row / 256-halo tiles reuse
# more (5.4x vs 3.6x) but leave too few workgroups in flight.
HALO_MAX = 160        # distinct neighbour rows per halo tile
HALO_ROWS = 24        # rows per halo tile
HALO_NNZ = 768        # Laplacian entries per halo tile
_HALO_KEYS = ("halo_tile_ptr", "halo_ptr", "halo", "halo_srp", "halo_lcol", "halo_eperm",
              "halo_hdr")


def halo_tiles(edge_index, n: int, order=None, max_rows: int = HALO_ROWS,
               max_halo: int = HALO_MAX, max_nnz: int = HALO_NNZ
               ) -> Optional[Dict[str, torch.Tensor]]:
    """Halo tiles of a sorted symmetric Laplacian COO (the CSR the device path
    builds from it: rows = edge_index[0], entries in COO order) for the
    LDS-staged SpMM, visiting rows in `order` (e.g. locality_order).  Host
    side, once per graph, like the row schedule; runs the library's native
    builder (hlhgat_halo_tiles).  Returns int32 tensors halo_tile_ptr /
    halo_ptr / halo / halo_srp / halo_eperm, int16 halo_lcol (holding uint16)
    and halo_bounds, or None if one row exceeds a bound."""
    import ctypes as C
    from ._lib import LIB
    ei = np.asarray(edge_index)
    nnz = ei.shape[1]
    rowptr = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(np.bincount(ei[0], minlength=n), out=rowptr[1:])
    col = np.ascontiguousarray(ei[1], dtype=np.int32)
    ordr = None if order is None else np.ascontiguousarray(np.asarray(order), dtype=np.int32)
    tile_ptr = np.zeros(n + 1, dtype=np.int32)
    halo_ptr = np.zeros(n + 1, dtype=np.int32)
    srp = np.zeros(n + 1, dtype=np.int32)
    halo = np.zeros(max(nnz, 1), dtype=np.int32)
    lcol = np.zeros(max(nnz, 1), dtype=np.uint16)
    eperm = np.zeros(max(nnz, 1), dtype=np.int32)
    hdr = np.zeros((max(n, 1), 8), dtype=np.int32)
    nt, nh = C.c_int64(0), C.c_int64(0)
    vp = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    rc = LIB.hlhgat_halo_tiles(vp(rowptr), vp(col), n, n, vp(ordr), max_rows, max_nnz, max_halo,
                               vp(tile_ptr), vp(halo_ptr), vp(halo), vp(srp), vp(lcol), vp(eperm),
                               vp(hdr), C.byref(nt), C.byref(nh))
    if rc != 0:
        return None
    t, h = nt.value, nh.value
    return {"halo_tile_ptr": torch.from_numpy(tile_ptr[:t + 1].copy()),
            "halo_ptr": torch.from_numpy(halo_ptr[:t + 1].copy()),
            "halo": torch.from_numpy(halo[:h].copy()),
            "halo_srp": torch.from_numpy(srp),
            "halo_lcol": torch.from_numpy(lcol[:nnz].view(np.int16).copy()),
            "halo_eperm": torch.from_numpy(eperm[:nnz].copy()),
            "halo_hdr": torch.from_numpy(hdr[:t].copy()),
            "halo_bounds": torch.tensor([max_halo, max_rows, max_nnz], dtype=torch.int64)}


def _collate_halo(b: "Batch", graphs: Sequence["PairData"], side: str) -> None:
    """Concatenate per-graph halo tiles: schedule positions and halo ids shift
    by the graph's row offset, halo offsets by the halo entries before it,
    schedule-order entry offsets and eperm by the entries before it; lcol is
    tile-local and unchanged.  All graphs must share the bounds."""
    keys = [k + "_" + side for k in _HALO_KEYS]
    bk = "halo_bounds_" + side
    if not all(getattr(g, k, None) is not None for g in graphs for k in keys + [bk]):
        return
    bounds = np.asarray(getattr(graphs[0], bk))
    if not all(np.array_equal(np.asarray(getattr(g, bk)), bounds) for g in graphs):
        return
    xk, ek = "x_" + side, "edge_index_" + side
    z = [np.zeros(1, np.int32)]
    tp, hp, srp, hc, lc, ep, hd = list(z), list(z), list(z), [], [], [], []
    roff = hoff = eoff = 0
    for g in graphs:
        gtp, ghp, ghc, gsrp, glc, gep, ghd = (np.asarray(getattr(g, k)) for k in keys)
        hd.append(ghd + np.array([roff, 0, hoff, 0, eoff, 0, 0, 0], dtype=np.int32))
        tp.append(gtp[1:] + roff)
        hp.append(ghp[1:] + hoff)
        srp.append(gsrp[1:] + eoff)
        hc.append(ghc + roff)
        lc.append(glc)
        ep.append(gep + eoff)
        roff += getattr(g, xk).size(0)
        hoff += int(ghp[-1])
        eoff += int(np.asarray(getattr(g, ek)).shape[1])
    for k, parts in zip(keys, (tp, hp, hc, srp, lc, ep, hd)):
        setattr(b, k, torch.from_numpy(np.ascontiguousarray(np.concatenate(parts))))
    setattr(b, bk, torch.from_numpy(bounds.copy()))


def is_sorted_symmetric(ei: np.ndarray, w: Optional[np.ndarray]) -> bool:
    """True if COO (ei, w) is sorted by (row, col) and equals its transpose."""
    if ei.shape[1] == 0:
        return True
    r, c = ei[0], ei[1]
    if np.any((r[1:] < r[:-1]) | ((r[1:] == r[:-1]) & (c[1:] < c[:-1]))):
        return False
    order = np.lexsort((r, c))  # sort the transpose by (col, row)
    if not (np.array_equal(c[order], r) and np.array_equal(r[order], c)):
        return False
    if w is not None and not np.array_equal(w[order], w):
        return False
    return True


def incidence_csr(edge_index, n_nodes: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Host build of the incidence CSR of |B1| for the edge list [2, E]
    (adj2par1, lib/Hodge_Dataset.py:169-191: edge e is incident to
    edge_index[0][e] and edge_index[1][e]): int32 rowptr [n_nodes+1] and
    edge ids [2E], ascending within a node; a self-edge (padding) appears
    twice.  The same CSR hlhgat_incidence_csr sorts on the device."""
    ei = np.asarray(edge_index, dtype=np.int64).reshape(2, -1)
    E = ei.shape[1]
    if E and (ei.min() < 0 or ei.max() >= n_nodes):
        raise ValueError(f"incidence_csr: node index out of range [0, {n_nodes})")
    e = np.arange(E, dtype=np.int64)
    keys = np.sort(np.concatenate([ei[0] * E + e, ei[1] * E + e]), kind="stable")
    rowptr = np.zeros(n_nodes + 1, dtype=np.int32)
    if E:
        np.cumsum(np.bincount(keys // E, minlength=n_nodes), out=rowptr[1:])
    return (torch.from_numpy(rowptr),
            torch.from_numpy((keys % E if E else keys).astype(np.int32)))


def laplacian_csr(edge_index, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """CSR of a row-sorted Laplacian COO (rows edge_index[0]): int32 rowptr
    [n+1] and int32 columns -- what hlhgat_csr_from_sorted_coo builds on the
    device; built here by the data loader instead."""
    ei = np.asarray(edge_index, dtype=np.int64).reshape(2, -1)
    rowptr = np.zeros(n + 1, dtype=np.int32)
    if ei.shape[1]:
        np.cumsum(np.bincount(ei[0], minlength=n)[:n], out=rowptr[1:])
    return torch.from_numpy(rowptr), torch.from_numpy(ei[1].astype(np.int32))


def _attach_csr(b, sides=("t", "s")) -> None:
    for side in sides:
        k = "edge_index_" + side
        ei, x = getattr(b, k, None), getattr(b, "x_" + side, None)
        if torch.is_tensor(ei) and torch.is_tensor(x) and (getattr(b, "hodge_sorted", None)
                                                            or {}).get(k, False):
            rp, col = laplacian_csr(ei, x.size(0))
            setattr(b, "csr_rowptr_" + side, rp)
            setattr(b, "csr_col_" + side, col)


# HLHGAT_FACTOR_TABLES=0: leave the factored L1's tables to the device build
# inside the step (A/B)
FACTOR_TABLES = os.environ.get("HLHGAT_FACTOR_TABLES", "1") != "0"


def factor_tables(b) -> None:
    """The factored L1's per-batch tables (hlhgat_hodge_factor_t), built on
    the host at collate time so the training step does not rebuild them on
    the device (in a captured step: every replay): alpha_e = L1[e, e] / 2
    (fp32, the diagonal's weight times 0.5), the signed B1 values in
    incidence-CSR order (-1 tail, +1 head: adj2par1, lib/Hodge_Dataset.py:
    169-191) and the edge ends as int32 [E, 2].  The same values as
    ops._build_factor's device build (tests/test_host.py)."""
    ei_s = np.asarray(b.edge_index_s, dtype=np.int64)
    w = np.asarray(b.edge_weight_s, dtype=np.float32)
    E = int(b.x_s.shape[0])
    diag = ei_s[0] == ei_s[1]
    alpha = np.zeros(E, dtype=np.float32)
    np.add.at(alpha, ei_s[0][diag], w[diag] * np.float32(0.5))
    rp = np.asarray(b.inc_rowptr, dtype=np.int64)
    eids = np.asarray(b.inc_eids, dtype=np.int64)
    ei = np.asarray(b.edge_index, dtype=np.int64).reshape(2, -1)
    node = np.repeat(np.arange(rp.size - 1, dtype=np.int64), np.diff(rp))
    sign = np.where(ei[1][eids] == node, np.float32(1.0), np.float32(-1.0)).astype(np.float32)
    b.fac_alpha = torch.from_numpy(alpha)
    b.fac_sign = torch.from_numpy(np.ascontiguousarray(sign))
    b.fac_ends = torch.from_numpy(np.ascontiguousarray(ei.T.astype(np.int32)))


def node_degree(inc_rowptr: torch.Tensor, valid: Optional[int] = None
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    """degree(edge_index.view(-1), N_t) (lib/Hodge_Cheb_Conv.py:359, the D of
    NodeEdgeInt) from the incidence CSR, and its fp32 reciprocal (1/0 = inf
    as on the device); rows >= valid (padding) get degree 1."""
    rp = np.asarray(inc_rowptr, dtype=np.int64)
    d = (rp[1:] - rp[:-1]).astype(np.float32)
    if valid is not None:
        d[valid:] = 1.0
    with np.errstate(divide="ignore"):
        r = np.float32(1.0) / d
    return torch.from_numpy(d), torch.from_numpy(r.astype(np.float32))


def collate(graphs: Sequence[PairData], check_hodge: bool = True) -> Batch:
    """PyG-free equivalent of DataLoader collation for PairData
    (offsets from PairData.__inc__, lib/Hodge_Dataset.py:40-48)."""
    b = Batch()
    B = len(graphs)
    b.num_graphs = B
    first = graphs[0]
    keys = first.keys()
    for k in keys:
        if k.rsplit("_", 1)[0] in _HALO_KEYS + ("halo_bounds",):
            continue  # _collate_halo
        vals = [getattr(g, k) for g in graphs]
        v0 = vals[0]
        if k in _INC_KEYS:
            incs = np.array([g.__inc__(k) for g in graphs], dtype=np.int64)
            off = np.concatenate([[0], np.cumsum(incs)[:-1]])
            cat = np.concatenate([np.asarray(v) + o for v, o in zip(vals, off)], axis=-1)
            setattr(b, k, torch.from_numpy(np.ascontiguousarray(cat)))
        elif torch.is_tensor(v0):
            if v0.dim() == 0:
                setattr(b, k, torch.stack(vals))
            else:
                setattr(b, k, torch.cat(vals, dim=0))
        elif isinstance(v0, (int, np.integer, float)):
            setattr(b, k, torch.tensor(vals))
        else:
            setattr(b, k, vals)
    b.num_nodes = int(sum(g.x_t.size(0) for g in graphs))
    hs = {}
    for k, wk in (("edge_index_s", "edge_weight_s"), ("edge_index_t", "edge_weight_t")):
        if getattr(b, k, None) is None:
            continue
        if check_hodge:
            ok = all(is_sorted_symmetric(np.asarray(getattr(g, k)),
                                         None if getattr(g, wk, None) is None
                                         else np.asarray(getattr(g, wk)))
                     for g in graphs)
        else:
            ok = all(getattr(g, "_hodge_sorted", False) for g in graphs)
        hs[k] = ok
    b.hodge_sorted = hs
    # factored L1 for large high-degree edge Laplacians (hlhgat.h, hodge factor)
    b.l1_factor = bool(hs.get("edge_index_s")) and _factor_wanted(graphs)
    for side in ("s", "t"):
        _collate_halo(b, graphs, side)
    # Laplacian CSR (rowptr / int32 columns) for the sorted symmetric blocks
    _attach_csr(b)
    # incidence CSR of |B1| (adj2par1) for the NodeEdgeInt gathers, built
    # here instead of by a device radix sort in every step
    ei = getattr(b, "edge_index", None)
    if torch.is_tensor(ei) and torch.is_tensor(getattr(b, "x_t", None)):
        b.inc_rowptr, b.inc_eids = incidence_csr(ei, b.x_t.size(0))
        b.deg_t, b.inv_deg_t = node_degree(b.inc_rowptr)
        if b.l1_factor and FACTOR_TABLES:
            factor_tables(b)
    # graph segment offsets of the readout (global_mean_pool over the
    # graph-contiguous rows, lib/Hodge_ST_Model.py:636), built here once
    # instead of by four small device ops per pool in every step
    for key, ck in (("seg_ptr_t", "num_node1"), ("seg_ptr_s", "num_edge1")):
        c = getattr(b, ck, None)
        if torch.is_tensor(c) and c.dim() == 1 and not c.is_floating_point():
            ptr = torch.zeros(c.numel() + 1, dtype=torch.int32)
            ptr[1:] = torch.cumsum(c, 0).to(torch.int32)
            setattr(b, key, ptr)
    return b


FACTOR_MIN_ROW = 8.0  # L1 entries per row from which the factored L1 pays (hlhgat.h)


def hodge_factor_ok(edge_index, n_nodes: int, edge_index_s, edge_weight_s) -> bool:
    """True iff the L1 COO (edge_index_s, edge_weight_s) is EXACTLY
    alpha_e * B1^T B1 for the boundary B1 of edge_index ([2, E], i < j;
    adj2par1, lib/Hodge_Dataset.py:169-191), alpha_e = L1[e,e] / 2 -- the form
    of every L1 the reference builds (2 B1^T B1 / lmax in fp32,
    lib/Hodge_Dataset.py:451-456): diagonal 2 alpha, +alpha for two edges
    sharing their tail or their head, -alpha for tail-to-head, every pair of
    edges sharing a node present once, nothing else."""
    ei = np.asarray(edge_index)
    eis = np.asarray(edge_index_s)
    w = np.asarray(edge_weight_s, dtype=np.float32).reshape(-1)
    E = ei.shape[1] if ei.ndim == 2 else 0
    if E == 0 or eis.shape[1] != w.size or np.any(ei[0] >= ei[1]):
        return False
    r, c = eis[0], eis[1]
    if r.min() < 0 or max(r.max(), c.max()) >= E:
        return False
    diag = r == c
    if int(diag.sum()) != E or not np.array_equal(np.sort(r[diag]), np.arange(E)):
        return False
    alpha = np.zeros(E, dtype=np.float32)
    alpha[r[diag]] = w[diag] * np.float32(0.5)
    a, b, p, q = ei[0][r], ei[1][r], ei[0][c], ei[1][c]
    if np.any(~diag & (a == p) & (b == q)):
        return False  # parallel edges
    v = np.where(diag, 2, np.where((a == p) | (b == q), 1, np.where((a == q) | (b == p), -1, 0)))
    if np.any(v == 0) or not np.array_equal(w, alpha[r] * v.astype(np.float32)):
        return False
    deg = np.bincount(ei.reshape(-1), minlength=int(n_nodes)).astype(np.int64)
    if eis.shape[1] != E + int((deg * (deg - 1)).sum()):
        return False
    key = r.astype(np.int64) * E + c
    return np.unique(key).size == key.size


def _factor_wanted(graphs) -> bool:
    """Collate-time choice of the factored L1: every graph's L1 is its
    alpha B1^T B1 and the batch averages >= FACTOR_MIN_ROW entries per row
    (ZINC ~4: the CSR path; CIFAR superpixels ~18, TSP ~20: factored)."""
    E = sum(int(np.asarray(g.edge_index_s).shape[1]) for g in graphs)
    rows = sum(int(g.x_s.shape[0]) for g in graphs)
    if rows == 0 or E < FACTOR_MIN_ROW * rows:
        return False
    for g in graphs:
        ok = getattr(g, "_l1_factor_ok", None)
        if ok is None:
            if getattr(g, "edge_index", None) is None or getattr(g, "edge_weight_s", None) is None:
                return False
            ok = hodge_factor_ok(g.edge_index, g.x_t.shape[0], g.edge_index_s, g.edge_weight_s)
            g._l1_factor_ok = ok
        if not ok:
            return False
    return True


PAD_MIN_ROWS = 64  # padding rows share the padding entries: keep every padding row short


def _spread(n_items: int, n_bins: int) -> np.ndarray:
    """Items per bin for n_items spread evenly over n_bins (first bins +1)."""
    base, extra = divmod(int(n_items), int(n_bins))
    return np.full(n_bins, base, dtype=np.int64) + (np.arange(n_bins) < extra)


def _roundup(v: int, q: int) -> int:
    return (int(v) + q - 1) // q * q


def static_caps(b: "Batch", quantum: int = 512) -> Dict[str, int]:
    """Capacity bucket of a collated batch for hipGraph replay: node / edge
    rows rounded up to `quantum` (at least PAD_MIN_ROWS padding rows),
    Laplacian entries to 4*quantum.  Batches with equal caps share one
    captured training step."""
    rows_t = _roundup(b.x_t.size(0) + PAD_MIN_ROWS, quantum)
    rows_s = _roundup(b.x_s.size(0) + PAD_MIN_ROWS, quantum)
    caps = {"rows_t": rows_t, "rows_s": rows_s,
            "nnz_t": _roundup(b.edge_index_t.size(1) + 1, 4 * quantum),
            "nnz_s": _roundup(b.edge_index_s.size(1) + 1, 4 * quantum)}
    return caps


def pool_tables(datas: Sequence["Batch"]) -> None:
    """The attpool heads' MLGC cluster CSR per side, built on the host once
    per level list instead of inside every step (lib/Hodge_ST_Model.py:
    1029-1038, 1067-1069): fine row r of datas[0] belongs to coarse cluster
    x[r, 0] + (first coarse row of its graph); rows whose cluster is inf
    (edges MLGC dropped, static-shape padding) go to a trailing bucket that
    the mean leaves out.  datas[0].pool_rowptr_{t,s} (int32 [n_coarse + 2])
    and pool_rows_{t,s} (int32 [n_fine], the fine rows grouped by cluster,
    ascending within one) are the CSR hodge_cheb_conv.cluster_mean sorts on
    the device -- the same members in the same order."""
    d0, d1 = datas[0], datas[1]
    for side, cnt in (("t", "num_node1"), ("s", "num_edge1")):
        x0 = np.asarray(getattr(d0, "x_" + side)[:, 0], dtype=np.float32)
        n = x0.size
        n_seg = int(getattr(d1, "x_" + side).shape[0])
        counts = np.asarray(getattr(d0, cnt), dtype=np.int64)
        ahead = np.zeros(counts.size, dtype=np.float32)
        ahead[1:] = np.cumsum(np.asarray(getattr(d1, cnt), dtype=np.int64))[:-1]
        per_row = np.zeros(n, dtype=np.float32)
        k = min(int(counts.sum()), n)
        per_row[:k] = np.repeat(ahead, counts)[:k]
        pos = x0 + per_row  # float32, as the device forward adds them
        idx = np.where(np.isinf(pos), n_seg, pos).astype(np.int64)
        if idx.size and (idx.min() < 0 or idx.max() > n_seg):
            raise ValueError(f"pool_tables: cluster ids outside [0, {n_seg}] on side {side}")
        order = np.argsort(idx, kind="stable")
        rowptr = np.zeros(n_seg + 2, dtype=np.int32)
        rowptr[1:] = np.cumsum(np.bincount(idx, minlength=n_seg + 1)).astype(np.int32)
        setattr(d0, "pool_rowptr_" + side, torch.from_numpy(rowptr))
        setattr(d0, "pool_rows_" + side, torch.from_numpy(order.astype(np.int32)))


def level_caps(levels: Sequence[Sequence["Batch"]], quantum: int = 512) -> List[Dict[str, int]]:
    """static_caps per MLGC level, the max over several level-batch lists
    (the attpool heads' `datas`): one capacity bucket for all of them."""
    out = []
    for lv in zip(*levels):
        cs = [static_caps(b, quantum) for b in lv]
        out.append({k: max(c[k] for c in cs) for k in cs[0]})
    return out


def pad_levels(datas: Sequence["Batch"], caps: Sequence[Dict[str, int]]) -> List["Batch"]:
    """Static-shape copy of an attpool level-batch list (datas = [fine level
    with the MLGC cluster of each node / edge in feature column 0, coarse
    level], lib/Hodge_ST_Model.py:1029-1038, main_pepfunc...:111-118): every
    level padded by pad_batch to its caps, and the fine level's padding rows
    put in NO cluster -- their column 0 (the cluster id the heads add the
    graph offsets to) is inf, so cluster_mean drops them as it drops the edges
    MLGC removed (lib/Hodge_ST_Model.py:1067-1069).  Real rows, the pooled
    features and every gradient equal the unpadded list's
    (tests/test_train_step.py)."""
    if len(datas) != len(caps):
        raise ValueError("pad_levels: one caps dict per level")
    out = [pad_batch(b, c) for b, c in zip(datas, caps)]
    p0, b0 = out[0], datas[0]
    for key in ("x_t", "x_s"):
        x = getattr(p0, key).clone()
        x[getattr(b0, key).size(0):, 0] = float("inf")
        setattr(p0, key, x)
    if getattr(b0, "pool_rowptr_t", None) is not None and p0.x_t.device.type == "cpu":
        pool_tables(out)  # the padded rows (inf) in the dropped bucket
    else:
        for k in ("pool_rowptr_t", "pool_rows_t", "pool_rowptr_s", "pool_rows_s"):
            if hasattr(p0, k):
                delattr(p0, k)
    return out


def _h2d(a: np.ndarray, dev: torch.device) -> torch.Tensor:
    """A host array on dev without blocking the host: staged through pinned
    memory and copied asynchronously on the current stream (a pageable copy
    would wait for the stream's queued kernels -- on a loader thread, for its
    own device work of the batch)."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if torch.device(dev).type != "cuda":
        return t
    return t.pin_memory().to(dev, non_blocking=True)


def pad_batch(b: "Batch", caps: Dict[str, int]) -> "Batch":
    """Static-shape copy of a collated host batch (hlhgat.train replays one
    hipGraph for every batch of the same caps).

    Padding rows are isolated simplices that belong to no graph:
      * x_t / x_s get zero rows; num_node1 / num_edge1 are unchanged, so the
        per-graph readouts never see them;
      * each Laplacian gets zero-weight self-loops spread evenly over its
        padding rows (COO stays row-sorted and symmetric; real rows keep
        their entries; no padding row is long);
      * the B1 edge list gets self-edges spread over the padding nodes;
      * n_valid_t / n_valid_s (int32 [1]) and valid_mask_t tell the BatchNorm
        kernels and the degree normalisation which rows are real.
    The real rows' values, gradients and statistics are those of the
    unpadded batch (tests/test_train_step.py)."""
    nt, ns = b.x_t.size(0), b.x_s.size(0)
    Rt, Rs = caps["rows_t"], caps["rows_s"]
    dev = b.x_t.device  # a device batch (e.g. SuperpixelPipeline's) is padded on the device
    if Rt <= nt or Rs <= ns:
        raise ValueError(f"pad_batch: caps ({Rt}, {Rs}) must exceed the rows ({nt}, {ns})")
    out = Batch()
    for k, v in vars(b).items():
        setattr(out, k, v)
    # Factored L1 (alpha_e B1^T B1) stays valid: a padding edge is a B1
    # self-edge, a zero column of B1, and its L1 row holds only zero-weight
    # self-loops, so alpha_e = 0 -- its row of alpha B1^T B1 is zero like its CSR
    # row, and the real edges' incidence never reaches the padding nodes.
    out.l1_factor = getattr(b, "l1_factor", False)
    for k in list(vars(out)):
        if k.startswith(tuple(_HALO_KEYS)) or k.startswith("halo_bounds"):
            delattr(out, k)  # halo tiles describe the unpadded CSR: plain schedule here

    def pad_rows(x, R):
        return torch.cat([x, x.new_zeros((R - x.size(0),) + tuple(x.shape[1:]))], 0)

    def pad_coo(ei, w, n, R, Z):
        extra = Z - ei.size(1)
        if extra < 0:
            raise ValueError(f"pad_batch: {ei.size(1)} Laplacian entries exceed the cap {Z}")
        per_row = _spread(extra, R - n)
        rows = _h2d(np.repeat(np.arange(n, R), per_row).astype(np.int64), ei.device).to(ei.dtype)
        return (torch.cat([ei, torch.stack([rows, rows])], 1),
                torch.cat([w, w.new_zeros(extra)]), per_row)

    out.x_t, out.x_s = pad_rows(b.x_t, Rt), pad_rows(b.x_s, Rs)
    y = getattr(b, "y", None)
    if torch.is_tensor(y) and y.dim() >= 1 and getattr(b, "num_graphs", None) != y.size(0):
        # per-simplex labels (TSP: one per edge, main_TSP...:316-321): zero rows
        if y.size(0) == ns:
            out.y = pad_rows(y, Rs)
        elif y.size(0) == nt:
            out.y = pad_rows(y, Rt)
    out.edge_index_t, out.edge_weight_t, _ = pad_coo(b.edge_index_t, b.edge_weight_t, nt, Rt,
                                                        caps["nnz_t"])
    out.edge_index_s, out.edge_weight_s, _ = pad_coo(b.edge_index_s, b.edge_weight_s, ns, Rs,
                                                        caps["nnz_s"])
    if getattr(b, "csr_rowptr_t", None) is not None or getattr(b, "csr_rowptr_s", None) is not None:
        _attach_csr(out)  # the padded COO (zero-weight self-loops on padding rows)
    if getattr(b, "edge_index", None) is not None:
        nodes = _h2d((nt + np.arange(Rs - ns) % (Rt - nt)).astype(np.int64),
                     b.edge_index.device).to(b.edge_index.dtype)
        out.edge_index = torch.cat([b.edge_index, torch.stack([nodes, nodes])], 1)
        if getattr(b, "inc_rowptr", None) is not None:
            out.inc_rowptr, out.inc_eids = incidence_csr(out.edge_index, Rt)
            # padding nodes: unit degree (the model's masked_fill, no 1/0)
            out.deg_t, out.inv_deg_t = node_degree(out.inc_rowptr, valid=nt)
            if out.l1_factor and getattr(b, "fac_alpha", None) is not None:
                factor_tables(out)  # padding edges: alpha 0, self-edge signs +1
    for side, n, R in (("t", nt, Rt), ("s", ns, Rs)):
        o = getattr(b, "row_order_" + side, None)
        if o is not None:
            setattr(out, "row_order_" + side,
                    torch.cat([o, torch.arange(n, R, dtype=o.dtype, device=o.device)]))
        setattr(out, "n_valid_" + side, torch.full((1,), n, dtype=torch.int32, device=dev))
    out.valid_mask_t = torch.arange(Rt, device=dev) < nt
    out.num_nodes = Rt
    if dev.type == "cuda":
        out._mark()  # the device-side declarations Batch.to makes (sorted, valid rows, factor)
    return out


ARENA_ALIGN = 256


def arena_alloc(shapes: Dict[str, tuple], pin: bool = False, device=None):
    """One uint8 buffer holding tensors of the given {name: (shape, dtype)}
    back to back (ARENA_ALIGN-byte aligned, in the dict's order); returns
    (arena, {name: view}).  The same shapes give the same layout, so two
    arenas of one batch shape copy into each other whole."""
    offs, off = {}, 0
    for k, (shape, dt) in shapes.items():
        nb = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
        offs[k] = (off, nb)
        off += (nb + ARENA_ALIGN - 1) // ARENA_ALIGN * ARENA_ALIGN
    arena = torch.empty(max(off, 1), dtype=torch.uint8, pin_memory=pin, device=device)
    views = {k: arena[o:o + nb].view(shapes[k][1]).view(shapes[k][0])
             for k, (o, nb) in offs.items()}
    return arena, views


class PackedGraphs:
    """A dataset of PairData simplex graphs packed back to back (the
    InMemoryDataset storage the reference's Hodge_Dataset keeps,
    lib/Hodge_Dataset.py:27-48): per-graph slices of x_t, x_s, the L0 / L1
    COO (graph-local, row-sorted, symmetric), the B1 edge list and y.

    ``collate(idx, caps)`` builds the batch of graphs ``idx`` in ONE native
    call (hlhgat_collate, csrc/collate.hip): bitwise the Batch of
    ``pad_batch(collate([self.graphs[i] for i in idx]), caps)`` (or of
    ``collate`` alone when caps is None), tables included, with no Python
    work per graph.  ``pin=True`` allocates the batch in pinned host memory
    (asynchronous copy-in)."""

    _KEYS = ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
             "edge_index")

    def __init__(self, graphs: Sequence[PairData], check_hodge: bool = True):
        from . import _lib
        self._lib = _lib
        G = len(graphs)
        if G == 0:
            raise ValueError("PackedGraphs: no graphs")
        for g in graphs:
            for k in self._KEYS:
                if getattr(g, k, None) is None:
                    raise ValueError(f"PackedGraphs: graph without {k}")
        a = lambda v, dt: np.ascontiguousarray(np.asarray(v), dtype=dt)  # noqa: E731
        self.f_t = int(graphs[0].x_t.shape[1])
        self.f_s = int(graphs[0].x_s.shape[1])
        if any(g.x_t.shape[1] != self.f_t or g.x_s.shape[1] != self.f_s for g in graphs):
            raise ValueError("PackedGraphs: feature widths differ between graphs")
        cnt = lambda f: np.concatenate([[0], np.cumsum([f(g) for g in graphs])]).astype(np.int64)  # noqa: E731
        self.node_ptr = cnt(lambda g: g.x_t.shape[0])
        self.edge_ptr = cnt(lambda g: g.x_s.shape[0])
        self.lt_ptr = cnt(lambda g: np.asarray(g.edge_index_t).shape[1])
        self.ls_ptr = cnt(lambda g: np.asarray(g.edge_index_s).shape[1])
        for g in graphs:
            if np.asarray(g.edge_index).shape[1] != g.x_s.shape[0]:
                raise ValueError("PackedGraphs: edge_index must have one column per x_s row")
        self.x_t = np.concatenate([a(g.x_t, np.float32) for g in graphs])
        self.x_s = np.concatenate([a(g.x_s, np.float32) for g in graphs])
        cat = lambda k, i, dt: np.concatenate([a(getattr(g, k), np.int64)[i].astype(dt)  # noqa: E731
                                               for g in graphs])
        self.lt_row, self.lt_col = cat("edge_index_t", 0, np.int32), cat("edge_index_t", 1, np.int32)
        self.ls_row, self.ls_col = cat("edge_index_s", 0, np.int32), cat("edge_index_s", 1, np.int32)
        self.b1_src, self.b1_dst = cat("edge_index", 0, np.int32), cat("edge_index", 1, np.int32)
        self.lt_w = np.concatenate([a(g.edge_weight_t, np.float32).reshape(-1) for g in graphs])
        self.ls_w = np.concatenate([a(g.edge_weight_s, np.float32).reshape(-1) for g in graphs])
        ys = [getattr(g, "y", None) for g in graphs]
        if all(y is not None for y in ys):
            self.y = np.stack([a(y, np.float32).reshape(-1) for y in ys])
            self.y_dim = int(self.y.shape[1])
            self._y_dtype = torch.as_tensor(ys[0]).dtype
        else:
            self.y, self.y_dim, self._y_dtype = np.zeros((G, 0), np.float32), 0, None
        if self._y_dtype is not None and self._y_dtype != torch.float32:
            raise ValueError("PackedGraphs: y must be float32")
        if check_hodge:
            sorted_sym = {k: all(is_sorted_symmetric(np.asarray(getattr(g, k)),
                                                     np.asarray(getattr(g, w)))
                                 for g in graphs)
                          for k, w in (("edge_index_s", "edge_weight_s"),
                                       ("edge_index_t", "edge_weight_t"))}
        else:
            ok = all(getattr(g, "_hodge_sorted", False) for g in graphs)
            sorted_sym = {"edge_index_s": ok, "edge_index_t": ok}
        if not all(sorted_sym.values()):
            raise ValueError("PackedGraphs: every Laplacian COO must be row-sorted and symmetric "
                             "(the Hodge builder's dense_to_sparse output)")
        self.hodge_sorted = sorted_sym
        self.n_graphs = G
        self._desc = _lib.PackedGraphsDesc(
            G, self.node_ptr.ctypes.data, self.edge_ptr.ctypes.data, self.lt_ptr.ctypes.data,
            self.ls_ptr.ctypes.data, self.x_t.ctypes.data, self.f_t, self.x_s.ctypes.data,
            self.f_s, self.lt_row.ctypes.data, self.lt_col.ctypes.data, self.lt_w.ctypes.data,
            self.ls_row.ctypes.data, self.ls_col.ctypes.data, self.ls_w.ctypes.data,
            self.b1_src.ctypes.data, self.b1_dst.ctypes.data, self.y.ctypes.data, self.y_dim)

    def __len__(self) -> int:
        return self.n_graphs

    def graph(self, i: int) -> PairData:
        """Graph i as a PairData (views of the packed arrays)."""
        n0, n1 = self.node_ptr[i], self.node_ptr[i + 1]
        e0, e1 = self.edge_ptr[i], self.edge_ptr[i + 1]
        t0, t1 = self.lt_ptr[i], self.lt_ptr[i + 1]
        s0, s1 = self.ls_ptr[i], self.ls_ptr[i + 1]
        T = lambda v: torch.from_numpy(np.ascontiguousarray(v))  # noqa: E731
        ei = lambda r, c: T(np.stack([r, c]).astype(np.int64))  # noqa: E731
        return PairData(edge_index_s=ei(self.ls_row[s0:s1], self.ls_col[s0:s1]),
                        x_s=T(self.x_s[e0:e1]), edge_index_t=ei(self.lt_row[t0:t1],
                                                               self.lt_col[t0:t1]),
                        x_t=T(self.x_t[n0:n1]), edge_weight_s=T(self.ls_w[s0:s1]),
                        edge_weight_t=T(self.lt_w[t0:t1]),
                        edge_index=ei(self.b1_src[e0:e1], self.b1_dst[e0:e1]),
                        y=T(self.y[i]) if self.y_dim else None)

    def _factor_ok(self, i: int) -> bool:
        cache = self.__dict__.setdefault("_fac", {})
        if i not in cache:
            g = self.graph(i)
            cache[i] = hodge_factor_ok(g.edge_index, g.x_t.shape[0], g.edge_index_s,
                                       g.edge_weight_s)
        return cache[i]

    def sizes(self, idx) -> Tuple[int, int, int, int]:
        """(nodes, edges, L0 entries, L1 entries) of the graphs idx."""
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        out = np.zeros(4, dtype=np.int64)
        self._lib.check(self._lib.LIB.hlhgat_collate_sizes(C_ref(self._desc), idx.ctypes.data,
                                                           idx.size, out.ctypes.data),
                        "collate_sizes")
        return tuple(int(v) for v in out)

    def caps_for(self, idx, quantum: int = 512) -> Dict[str, int]:
        """static_caps of the batch of graphs idx (without building it)."""
        n_t, n_s, z_t, z_s = self.sizes(idx)
        return {"rows_t": _roundup(n_t + PAD_MIN_ROWS, quantum),
                "rows_s": _roundup(n_s + PAD_MIN_ROWS, quantum),
                "nnz_t": _roundup(z_t + 1, 4 * quantum), "nnz_s": _roundup(z_s + 1, 4 * quantum)}

    def collate(self, idx, caps: Optional[Dict[str, int]] = None, pin: bool = False) -> "Batch":
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        B = int(idx.size)
        n_t, n_s, z_t, z_s = self.sizes(idx)
        padded = caps is not None
        Rt, Rs = (caps["rows_t"], caps["rows_s"]) if padded else (n_t, n_s)
        Zt, Zs = (caps["nnz_t"], caps["nnz_s"]) if padded else (z_t, z_s)
        if padded and (Rt <= n_t or Rs <= n_s):
            raise ValueError(f"PackedGraphs.collate: caps ({Rt}, {Rs}) must exceed the rows "
                             f"({n_t}, {n_s})")
        if padded and (Zt < z_t or Zs < z_s):
            raise ValueError(f"PackedGraphs.collate: {z_t} / {z_s} Laplacian entries exceed "
                             f"the caps {Zt} / {Zs}")
        f32, i32, i64 = torch.float32, torch.int32, torch.int64
        # every tensor of the batch is a view of ONE host arena (pinned when
        # asked): hlhgat.train.TrainStep.stage uploads it in one copy into a
        # device arena of the same layout (the static buffers of a graph)
        shapes = {"x_t": ((Rt, self.f_t), f32), "x_s": ((Rs, self.f_s), f32),
                  "edge_index_t": ((2, Zt), i64), "edge_weight_t": ((Zt,), f32),
                  "edge_index_s": ((2, Zs), i64), "edge_weight_s": ((Zs,), f32),
                  "edge_index": ((2, Rs), i64), "y": ((B * self.y_dim,), f32),
                  "num_node1": ((B,), i64), "num_edge1": ((B,), i64),
                  "csr_rowptr_t": ((Rt + 1,), i32), "csr_col_t": ((Zt,), i32),
                  "csr_rowptr_s": ((Rs + 1,), i32), "csr_col_s": ((Zs,), i32),
                  "inc_rowptr": ((Rt + 1,), i32), "inc_eids": ((2 * Rs,), i32),
                  "deg_t": ((Rt,), f32), "inv_deg_t": ((Rt,), f32),
                  "seg_ptr_t": ((B + 1,), i32), "seg_ptr_s": ((B + 1,), i32),
                  "valid_mask_t": ((Rt,), torch.bool),
                  "n_valid_t": ((1,), i32), "n_valid_s": ((1,), i32)}
        arena, t = arena_alloc(shapes, pin)
        o = self._lib.CollatedDesc(Rt, Rs, Zt, Zs, *[t[k].data_ptr() for k in (
            "x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
            "edge_index", "y", "num_node1", "num_edge1", "csr_rowptr_t", "csr_col_t",
            "csr_rowptr_s", "csr_col_s", "inc_rowptr", "inc_eids", "deg_t", "inv_deg_t",
            "seg_ptr_t", "seg_ptr_s", "valid_mask_t")], 0, 0)
        self._lib.check(self._lib.LIB.hlhgat_collate(C_ref(self._desc), idx.ctypes.data, B,
                                                     C_ref(o)), "collate")
        b = Batch()
        b.num_graphs = B
        for k in self._KEYS:
            setattr(b, k, t[k])
        if self.y_dim:
            b.y = t["y"]
        b.num_node1, b.num_edge1 = t["num_node1"], t["num_edge1"]
        b.num_nodes = Rt
        b.hodge_sorted = dict(self.hodge_sorted)
        # factored L1 as collate decides it (never for padded batches: pad_batch)
        b.l1_factor = (not padded and z_s >= FACTOR_MIN_ROW * n_s and n_s > 0
                       and all(self._factor_ok(int(i)) for i in idx))
        for k in ("csr_rowptr_t", "csr_col_t", "csr_rowptr_s", "csr_col_s", "inc_rowptr",
                  "inc_eids", "deg_t", "inv_deg_t", "seg_ptr_t", "seg_ptr_s"):
            setattr(b, k, t[k])
        if padded:
            t["n_valid_t"][0] = n_t
            t["n_valid_s"][0] = n_s
            b.n_valid_t = t["n_valid_t"]
            b.n_valid_s = t["n_valid_s"]
            b.valid_mask_t = t["valid_mask_t"]
        b._arena = arena
        return b


def C_ref(struct):
    import ctypes
    return ctypes.byref(struct)


class BoundaryOperator:
    """B1 of adj2par1 for the undirected edge list edge_index [2, E] (column
    e: -1 at edge_index[0][e], +1 at edge_index[1][e]), or a view of it:
    ``.abs()`` (|B1|), ``.t()`` / ``.transpose(0, 1)`` (B1^T).

    It stands in for the reference's torch sparse COO: ``torch.sparse.mm(P,
    x)``, ``torch.mm``, ``torch.matmul`` and ``P @ x`` with P any of those
    views run the HIP incidence kernels (ops.incidence_mm; bitwise the
    coalesced sparse product, with autograd), so reference lines such as
    ``torch.sparse.mm(par_1.transpose(0,1), x_t).abs()/2``
    (lib/Hodge_ST_Model.py:848) and ``torch.sparse.mm(par.abs(), x_s)``
    (lib/Hodge_Cheb_Conv.py:294) work unchanged.  The incidence CSR is built
    once and shared by every view and every NodeEdgeInt of a block group.
    ``to_sparse_coo`` returns the reference's exact torch sparse tensor."""

    _MM = None  # the torch functions that mean "sparse @ dense" (set on first use)

    def __init__(self, edge_index: torch.Tensor, num_node: int, num_edge: int,
                 _transposed: bool = False, _absolute: bool = False, _base=None):
        self.edge_index = edge_index
        self.num_node = int(num_node)
        self.num_edge = int(num_edge)
        if edge_index.size(1) != self.num_edge:
            raise ValueError(f"adj2par1: edge_index has {edge_index.size(1)} edges, "
                             f"num_edge={num_edge}")
        self.transposed = bool(_transposed)
        self.absolute = bool(_absolute)
        self._base = _base  # views share the base operator's incidence CSR
        self._inc = None
        # static-shape batches: valid node / edge row counts (pad_batch)
        self.valid_t = getattr(edge_index, "_hlhgat_valid_t", None)
        self.valid_s = getattr(edge_index, "_hlhgat_valid_s", None)

    # -- tensor-like surface ---------------------------------------------------
    @property
    def shape(self):
        return (torch.Size([self.num_edge, self.num_node]) if self.transposed
                else torch.Size([self.num_node, self.num_edge]))

    def size(self, dim: Optional[int] = None):
        return self.shape if dim is None else self.shape[dim]

    def dim(self) -> int:
        return 2

    is_sparse = True
    layout = torch.sparse_coo
    dtype = torch.float32

    @property
    def device(self):
        return self.edge_index.device

    def _view(self, transposed: bool, absolute: bool) -> "BoundaryOperator":
        return BoundaryOperator(self.edge_index, self.num_node, self.num_edge, transposed,
                                absolute, self._base or self)

    def abs(self) -> "BoundaryOperator":
        return self._view(self.transposed, True)

    def t(self) -> "BoundaryOperator":
        return self._view(not self.transposed, self.absolute)

    def transpose(self, dim0: int, dim1: int) -> "BoundaryOperator":
        if sorted((dim0 % 2, dim1 % 2)) != [0, 1]:
            raise ValueError("BoundaryOperator.transpose: only (0, 1)")
        return self.t()

    @property
    def T(self) -> "BoundaryOperator":
        return self.t()

    def coalesce(self) -> "BoundaryOperator":
        return self

    def is_coalesced(self) -> bool:
        return True

    def to(self, device=None, *args, **kwargs) -> "BoundaryOperator":
        if device is None or torch.device(device) == self.edge_index.device:
            return self
        return BoundaryOperator(self.edge_index.to(device), self.num_node, self.num_edge,
                                self.transposed, self.absolute)

    def incidence(self):
        if self._base is not None:
            return self._base.incidence()
        if self._inc is None:
            from .ops import incidence
            self._inc = incidence(self.edge_index, self.num_node)
        return self._inc

    # -- products (HIP) --------------------------------------------------------
    def matmul(self, x: torch.Tensor) -> torch.Tensor:
        from .ops import incidence_mm
        if not (torch.is_tensor(x) and x.is_cuda):
            raise RuntimeError("hlhgat: BoundaryOperator products run on the ROCm device only "
                               "(use .to_sparse_coo() for a CPU torch sparse tensor)")
        if x.dim() != 2:
            raise RuntimeError(f"hlhgat: BoundaryOperator @ x needs a 2-D x, got {x.dim()}-D")
        return incidence_mm(x, self.incidence(), self.transposed, not self.absolute)

    __matmul__ = matmul
    mm = matmul

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        if cls._MM is None:
            cls._MM = {torch.sparse.mm, torch.mm, torch.matmul, torch.Tensor.mm,
                       torch.Tensor.matmul, torch.Tensor.__matmul__}
        kwargs = kwargs or {}
        if func in cls._MM and len(args) == 2 and isinstance(args[0], BoundaryOperator) \
                and torch.is_tensor(args[1]) and not kwargs:
            return args[0].matmul(args[1])
        return NotImplemented

    def to_sparse_coo(self) -> torch.Tensor:
        ei = self.edge_index
        E = ei.shape[1]
        col_idx = torch.cat([torch.arange(E), torch.arange(E)]).to(ei.device)
        row_idx = torch.cat([ei[0], ei[1]])
        val = torch.cat([ei[0].new_full(ei[0].shape, -1), ei[0].new_full(ei[0].shape, 1)]).float()
        P = torch.sparse_coo_tensor(torch.stack([row_idx, col_idx]), val,
                                    (self.num_node, self.num_edge))
        if self.absolute:
            P = P.abs()
        return P.t() if self.transposed else P

    def to_dense(self) -> torch.Tensor:
        return self.to_sparse_coo().to_dense()

    def __repr__(self) -> str:
        v = ("|B1|" if self.absolute else "B1") + ("^T" if self.transposed else "")
        return f"BoundaryOperator({v}, shape={tuple(self.shape)}, device={self.device})"


def adj2par1(edge_index: torch.Tensor, num_node: int, num_edge: int) -> BoundaryOperator:
    """First boundary operator of the undirected adjacency
    (lib/Hodge_Dataset.py:169-191)."""
    return BoundaryOperator(edge_index, num_node, num_edge)


def boundary_from_sparse(par: torch.Tensor) -> BoundaryOperator:
    """Recover the edge list from a reference-built torch sparse B1."""
    par = par.coalesce()
    idx, val = par.indices(), par.values()
    E = par.shape[1]
    ei = torch.empty(2, E, dtype=torch.int64, device=idx.device)
    neg = val < 0
    ei[0, idx[1][neg]] = idx[0][neg]
    ei[1, idx[1][~neg]] = idx[0][~neg]
    return BoundaryOperator(ei, par.shape[0], E)


def degree(index: torch.Tensor, num_nodes: Optional[int] = None,
           dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """torch_geometric.utils.degree: occurrences of each index (float)."""
    n = num_nodes if num_nodes is not None else (int(index.max()) + 1 if index.numel() else 0)
    out = torch.zeros(n, dtype=dtype or torch.get_default_dtype(), device=index.device)
    return out.scatter_add_(0, index, torch.ones_like(index, dtype=out.dtype))


def dense_to_sparse(a: torch.Tensor):
    """torch_geometric.utils.dense_to_sparse for one 2-D matrix: row-major
    indices of the nonzero entries and their values."""
    idx = a.nonzero().t().contiguous()
    return idx, a[idx[0], idx[1]]


def hodge_laplacians(edge_index: np.ndarray, n: int):
    """(L0, L1, maxeig, B1) of an undirected simple graph (edges i<j), computed
    exactly as the ZINC process() does in float32 torch
    (lib/Hodge_Dataset.py:451-456)."""
    ei = torch.as_tensor(np.asarray(edge_index), dtype=torch.int64)
    E = ei.shape[1]
    par1 = torch.zeros(n, E)
    ar = torch.arange(E)
    par1[ei[0], ar] = -1.0
    par1[ei[1], ar] = 1.0
    L0 = torch.matmul(par1, par1.T)
    lam = torch.linalg.eigh(L0)[0]
    maxeig = lam.max()
    L0 = 2 * torch.matmul(par1, par1.T) / maxeig
    L1 = 2 * torch.matmul(par1.T, par1) / maxeig
    return L0, L1, maxeig, par1


def hodge_coo_from_boundary(edge_index, n: int, lmax: float):
    """Sparse (row-major sorted) COO of L0 = 2 B1 B1^T / lmax and
    L1 = 2 B1^T B1 / lmax from the edge list (i<j) and a given lmax, with the
    entries the reference's dense float32 construction produces
    (lib/Hodge_Dataset.py:451-456: fl(fl(2 v) / lmax), v the integer entry of
    B1 B1^T / B1^T B1; zeros dropped as dense_to_sparse does) -- without the
    dense [E, E] L1 (1.37 M entries for the DEMO brain skeleton, ~10 GB dense
    at BASELINE config 5).  Returns (ei_t, w_t, ei_s, w_s) as torch tensors."""
    import scipy.sparse as sp
    ei = np.asarray(edge_index, dtype=np.int64)
    E = ei.shape[1]
    B = sp.csr_matrix((np.concatenate([-np.ones(E), np.ones(E)]).astype(np.int64),
                       (np.concatenate([ei[0], ei[1]]), np.concatenate([np.arange(E)] * 2))),
                      shape=(n, E))
    lam = np.float32(lmax)

    def coo(M):
        M = M.tocoo()
        M.sum_duplicates()
        o = np.lexsort((M.col, M.row))
        r, c, v = M.row[o], M.col[o], M.data[o]
        keep = v != 0
        w = (np.float32(2.0) * v[keep].astype(np.float32)) / lam
        return (torch.from_numpy(np.stack([r[keep], c[keep]]).astype(np.int64)),
                torch.from_numpy(w.astype(np.float32)))

    ei_t, w_t = coo(B @ B.T)
    ei_s, w_s = coo(B.T @ B)
    return ei_t, w_t, ei_s, w_s


# ----------------------------------------------------------------------------
# multi-level graph coarsening (MLGC) for the attention-pooling heads
# ----------------------------------------------------------------------------
def graclus(edge_index, n: int, weight=None, seed: int = 0, perm=None) -> np.ndarray:
    """Greedy graclus matching (torch_cluster 1.6.0 graclus_cluster, the
    reference's dependency, absent here; called at lib/Hodge_Dataset.py:252,
    :311), run by the library's native host builder (hlhgat_graclus):
    self-loops dropped, nodes visited in a random order (torch_cluster draws
    a torch.randperm; here a seeded numpy permutation), each unmatched node
    paired with the LAST of its unmatched neighbours (ascending column order)
    whose weight is >= the best so far, from 0 -- torch_cluster's weighted
    branch, which the reference always takes (MLGC passes ones_like) -- both
    get cluster id min(u, v); a node with no unmatched neighbour stays alone
    (id u).  Parity unpinned (no torch_cluster output exists here).
    perm: an explicit node order (replaces the seeded permutation).
    Returns int64 [n] cluster ids."""
    from ._lib import LIB, check
    ei = np.ascontiguousarray(np.asarray(edge_index, dtype=np.int64).reshape(2, -1))
    w = None if weight is None else np.ascontiguousarray(np.asarray(weight, dtype=np.float64))
    if perm is None:
        perm = np.random.default_rng(seed).permutation(n)
    perm = np.ascontiguousarray(np.asarray(perm, dtype=np.int64))
    if perm.shape != (n,):
        raise ValueError(f"graclus: perm must have {n} entries")
    out = np.empty(n, dtype=np.int64)
    check(LIB.hlhgat_graclus(ei.ctypes.data, None if w is None else w.ctypes.data,
                             ei.shape[1], n, perm.ctypes.data, out.ctypes.data), "graclus")
    return out


def mlgc_map(cluster, edge_index):
    """Fine -> coarse assignment of one MLGC level (lib/Hodge_Dataset.py:
    254-275) by the native host builder (hlhgat_mlgc_map): cluster ids
    renumbered by ascending id; an edge inside one cluster gets inf, the
    others the coarse edge (min, max) numbered in first-seen edge order.
    Returns (c_node int64 [n], c_edge float32 [E], coarse edge_index int64
    [2, E1], n1)."""
    import ctypes as C
    from ._lib import LIB, check
    lab = np.ascontiguousarray(np.asarray(cluster, dtype=np.int64))
    ei = np.ascontiguousarray(np.asarray(edge_index, dtype=np.int64).reshape(2, -1))
    n, E = lab.size, ei.shape[1]
    c_node = np.empty(n, dtype=np.int64)
    c_edge = np.empty(E, dtype=np.float32)
    e1 = np.empty((2, max(E, 1)), dtype=np.int64)
    n1, ne = C.c_int64(0), C.c_int64(0)
    check(LIB.hlhgat_mlgc_map(lab.ctypes.data, n, ei.ctypes.data, E, c_node.ctypes.data,
                              c_edge.ctypes.data, e1.ctypes.data, C.byref(n1), C.byref(ne)),
          "mlgc_map")
    if E == 0:
        e1 = e1[:, :0]
    return c_node, c_edge, np.ascontiguousarray(e1.reshape(2, -1)[:, :ne.value]) if E else e1, \
        int(n1.value)


class MLGCBatch:
    """hlhgat_mlgc_batch's flat outputs for G graphs: c_node [N] and c_edge
    [E] (per graph, concatenated), ce [2, E] holding graph g's coarse edges
    (local coarse ids) at the head of its edge slot edge_ptr[g] ..
    edge_ptr[g] + cm[g], cn [G] coarse node counts, cm [G] coarse edge
    counts."""

    def __init__(self, node_ptr, edge_ptr, c_node, c_edge, ce, cn, cm):
        self.node_ptr, self.edge_ptr = node_ptr, edge_ptr
        self.c_node, self.c_edge, self.ce, self.cn, self.cm = c_node, c_edge, ce, cn, cm

    def per_graph(self):
        """[(c_node, c_edge, coarse edge_index, n1)] per graph, like mlgc_map."""
        out = []
        for g in range(self.cn.size):
            n0, n1_ = self.node_ptr[g], self.node_ptr[g + 1]
            e0, e1 = self.edge_ptr[g], self.edge_ptr[g + 1]
            out.append((self.c_node[n0:n1_], self.c_edge[e0:e1],
                        np.ascontiguousarray(self.ce[:, e0:e0 + self.cm[g]]), int(self.cn[g])))
        return out


def mlgc_batch_flat(edges, edge_counts, ns, perm, threads: int = 0) -> MLGCBatch:
    """One MLGC level for a batch of graphs by one native call
    (hlhgat_mlgc_batch) on flat arrays: edges int64 [2, E] (each graph's i<j
    edges in local node ids, graph after graph), edge_counts [G], ns [G],
    perm [N] (graph g's graclus node order, local ids, in its node slot).
    Per graph: graclus over the edges taken both ways with unit weights, then
    mlgc_map -- the same results as mlgc_map(graclus(both, n, ones, perm=p),
    ei) graph by graph, on host threads."""
    from ._lib import LIB, check
    ns = np.asarray(ns, np.int64)
    G = ns.size
    node_ptr = np.zeros(G + 1, np.int64)
    node_ptr[1:] = np.cumsum(ns)
    edge_ptr = np.zeros(G + 1, np.int64)
    edge_ptr[1:] = np.cumsum(np.asarray(edge_counts, np.int64))
    E = int(edge_ptr[-1])
    edges = np.ascontiguousarray(np.asarray(edges, np.int64).reshape(2, E))
    perm = np.ascontiguousarray(np.asarray(perm, np.int64).reshape(-1))
    if perm.size != node_ptr[-1]:
        raise ValueError("mlgc_batch: one permutation of each graph's nodes expected")
    c_node = np.empty(int(node_ptr[-1]), np.int64)
    c_edge = np.empty(E, np.float32)
    ce = np.empty((2, max(E, 1)), np.int64)
    cn = np.empty(G, np.int64)
    cm = np.empty(G, np.int64)
    threads = threads or min(8, os.cpu_count() or 1)
    check(LIB.hlhgat_mlgc_batch(G, node_ptr.ctypes.data, edge_ptr.ctypes.data, edges.ctypes.data,
                                perm.ctypes.data, threads, c_node.ctypes.data, c_edge.ctypes.data,
                                ce.ctypes.data, cn.ctypes.data, cm.ctypes.data), "mlgc_batch")
    return MLGCBatch(node_ptr, edge_ptr, c_node, c_edge, ce.reshape(2, -1)[:, :E], cn, cm)


def mlgc_batch(edge_lists, ns, perms, threads: int = 0):
    """mlgc_batch_flat over per-graph lists: edge_lists[g] int64 [2, E_g],
    perms[g] a permutation of graph g's nodes.  Returns [(c_node, c_edge,
    coarse edge_index, n1)] per graph, like mlgc_map."""
    G = len(ns)
    edges = (np.concatenate([np.asarray(e, np.int64).reshape(2, -1) for e in edge_lists], axis=1)
             if G else np.zeros((2, 0), np.int64))
    perm = (np.concatenate([np.asarray(p, np.int64) for p in perms]) if G
            else np.zeros(0, np.int64))
    counts = [int(np.asarray(e).reshape(2, -1).shape[1]) for e in edge_lists]
    return mlgc_batch_flat(edges, counts, ns, perm, threads).per_graph()


def to_undirected_mean(edge_index, weight, n: int):
    """PyG to_undirected(edge_index, edge_weight, reduce='mean') as used by
    MLGC_weighted (lib/Hodge_Dataset.py:310): both directions, coalesced in
    (row, col) order, duplicate weights averaged.  Returns (int64 [2, E'],
    float32 [E'])."""
    ei = np.asarray(edge_index, dtype=np.int64)
    w = np.asarray(weight, dtype=np.float32)
    r = np.concatenate([ei[0], ei[1]])
    c = np.concatenate([ei[1], ei[0]])
    ww = np.concatenate([w, w])
    o = np.lexsort((c, r))
    r, c, ww = r[o], c[o], ww[o]
    first = np.ones(r.size, dtype=bool)
    first[1:] = (r[1:] != r[:-1]) | (c[1:] != c[:-1])
    starts = np.flatnonzero(first)
    seg = torch.from_numpy(np.cumsum(first) - 1)
    # PyG's scatter mean: scatter_add in entry order, then / count
    s = torch.zeros(starts.size).scatter_add_(0, seg, torch.from_numpy(ww))
    cnt = torch.bincount(seg, minlength=starts.size).to(torch.float32)
    return np.stack([r[starts], c[starts]]), (s / cnt).numpy()


def _mlgc_level(ei1: np.ndarray, n1: int) -> "PairData":
    """The coarse graph of one MLGC level (lib/Hodge_Dataset.py:275-294):
    Hodge Laplacians built as the reference does (dense eigh,
    2 B1 B1^T / lmax) and unit features."""
    L0, L1, _, _ = hodge_laplacians(ei1, n1)
    eit, ewt = dense_to_sparse(L0)
    eis, ews = dense_to_sparse(L1)
    c = PairData(x_s=torch.ones(ei1.shape[1], 1), edge_index_s=eis, edge_weight_s=ews,
                 x_t=torch.ones(n1, 1), edge_index_t=eit, edge_weight_t=ewt)
    c.edge_index = torch.from_numpy(ei1)
    c.num_node1 = n1
    c.num_edge1 = int(ei1.shape[1])
    c.num_nodes = n1
    c._hodge_sorted = True
    return c


def mlgc(g: "PairData", seed: int = 0):
    """One level of MLGC (lib/Hodge_Dataset.py:241-295): graclus on L0's
    pattern with unit weights, then the fine -> coarse map (mlgc_map) and the
    coarse graph's Hodge Laplacians.
    Returns (coarse PairData, c_node [n, 1] float, c_edge [E, 1] float)."""
    n = int(g.num_node1)
    lab = graclus(np.asarray(g.edge_index_t), n, seed=seed)
    c_node, c_edge, ei1, n1 = mlgc_map(lab, np.asarray(g.edge_index))
    return (_mlgc_level(ei1, n1), torch.from_numpy(c_node.astype(np.float32)).view(-1, 1),
            torch.from_numpy(c_edge).view(-1, 1))


def mlgc_weighted(g: "PairData", seed: int = 0):
    """MLGC_weighted (lib/Hodge_Dataset.py:298-353): graclus on the graph's
    own edges made undirected, weighted by exp(-x_s[:, 0]^2) (duplicates
    averaged), then the same map and coarse graph as mlgc."""
    n = int(g.num_node1)
    xs = np.asarray(g.x_s, dtype=np.float32)[:, 0]
    ei_u, w_u = to_undirected_mean(np.asarray(g.edge_index), np.exp(-(xs * xs)), n)
    lab = graclus(ei_u, n, weight=w_u, seed=seed)
    c_node, c_edge, ei1, n1 = mlgc_map(lab, np.asarray(g.edge_index))
    return (_mlgc_level(ei1, n1), torch.from_numpy(c_node.astype(np.float32)).view(-1, 1),
            torch.from_numpy(c_edge).view(-1, 1))
