"""Torch-facing wrappers and autograd Functions over the HIP C-ABI.

Every op here runs a kernel from libhlhgat.so on the caller's current HIP
stream; there is no CPU or eager-PyTorch fallback (tensors must live on a ROCm
device, fp32, with the documented layouts).  The reference semantics each op
reproduces are cited per function (paths relative to deepika090/HL-HGAT).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import math
import os
import weakref
from dataclasses import dataclass
from typing import Tuple, List, Optional, Sequence

import torch

from . import _lib
from ._lib import LIB, check

try:  # C++ autograd nodes over the same C-ABI (hl-hgat_amd/csrc/torch_ext.cpp)
    from . import _hlhgat_ext as _ext
except ImportError as e:  # pragma: no cover - the build always produces it
    raise ImportError(f"hlhgat: torch extension _hlhgat_ext missing ({e}); run the build "
                      f"(make -C hl-hgat_amd/csrc)") from e

__all__ = [
    "SparseCSR", "HodgeOperator", "Incidence", "hodge_operator", "incidence",
    "mark_hodge", "spmm", "poly_basis", "hodge_poly_conv", "linear_blocks", "mlp2", "nei_value",
    "batch_norm_act", "check_device_errors", "clear_device_errors", "device_errors",
    "node_from_edges", "edge_from_nodes", "incidence_mm", "att_score", "segment_mean",
    "POLY_LAGUERRE", "POLY_CHEB", "POLY_LAGUERRE_DEMO", "SIGMA_SIGMOID", "SIGMA_RELU",
]

POLY_LAGUERRE, POLY_CHEB = _lib.POLY_LAGUERRE, _lib.POLY_CHEB
POLY_LAGUERRE_DEMO = _lib.POLY_LAGUERRE_DEMO
SIGMA_SIGMOID, SIGMA_RELU = _lib.SIGMA_SIGMOID, _lib.SIGMA_RELU


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------
def _stream(t: torch.Tensor) -> int:
    return torch._C._cuda_getCurrentRawStream(t.device.index)


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
# node / edge chain concurrency
# ----------------------------------------------------------------------------
# Every HL block runs two independent chains — the node side on L0 and the edge
# side on L1 (lib/Hodge_ST_Model.py:556-566, lib/Hodge_Cheb_Conv.py:307-308).
# At ZINC scale each launch is latency-bound and fills a fraction of the 256
# CUs, so the edge chain is issued on a second HIP stream and the two overlap.
# Autograd replays each node's backward on the stream its forward used, so the
# backward chains overlap too; captured into a hipGraph the fork/join becomes
# two graph branches.
_SIDE_STREAMS = {}
# HLHGAT_STREAM_FORK=0: every chain on one stream (diagnosis / A-B)
_FORK_ENABLED = os.environ.get("HLHGAT_STREAM_FORK", "1") != "0"


def set_stream_fork(enabled: bool) -> None:
    """Enable / disable issuing the edge chain on a second stream."""
    global _FORK_ENABLED
    _FORK_ENABLED = bool(enabled)


_OWN_STREAMS = {}


def own_stream(device, role: str, cu_mask=None, priority: int = 0) -> torch.cuda.Stream:
    """A HIP stream of this library's own for `role` on `device` (created
    once, non-blocking, never from torch's stream pool).  torch.cuda.Stream()
    hands out its 32 pool streams round-robin, so two unrelated users can get
    the same stream -- e.g. a user's copy stream and a side stream that has
    joined a graph capture, whose uploads would then be captured.  The capture,
    copy and side streams of TrainStep / StagedFeed / the chains are these.
    Created by libhlhgat (hlhgat_stream_create), i.e. by the HIP runtime torch
    loaded.  cu_mask (a list of 32-bit words, bit c = CU c): the stream runs on
    those CUs only (the first call for a role fixes its mask); priority: HIP
    stream priority (lower = higher; 0 = default)."""
    idx = device.index if getattr(device, "index", None) is not None else (
        device if isinstance(device, int) else torch.cuda.current_device())
    s = _OWN_STREAMS.get((idx, role))
    if s is None:
        import ctypes
        h = ctypes.c_void_p()
        if cu_mask:
            words = (ctypes.c_uint32 * len(cu_mask))(*[int(w) & 0xffffffff for w in cu_mask])
            check(LIB.hlhgat_stream_create(idx, 1, 0, words, len(cu_mask), ctypes.byref(h)),
                  "stream_create")
        else:
            check(LIB.hlhgat_stream_create(idx, 1, int(priority), None, 0, ctypes.byref(h)),
                  "stream_create")
        s = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
        _OWN_STREAMS[(idx, role)] = s
    return s


def cu_mask_high(n_on: int, n_cu: int):
    """A CU mask (32-bit words covering n_cu CUs) with the n_on
    highest-numbered CUs set."""
    words = (n_cu + 31) // 32
    mask = [0] * words
    for c in range(n_cu - n_on, n_cu):
        mask[c // 32] |= 1 << (c % 32)
    return mask


def stream_cu_mask(stream, words: int = 8):
    """The CU mask `stream` runs on (a list of 32-bit words)."""
    import ctypes
    buf = (ctypes.c_uint32 * words)()
    check(LIB.hlhgat_stream_cu_mask(stream.cuda_stream, buf, words), "stream_cu_mask")
    return list(buf)


def side_stream(device: torch.device, slot: int = 0) -> torch.cuda.Stream:
    """Side stream `slot` of the device (0: the edge chains; 1: batch
    preparation that overlaps the first conv)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE_STREAMS.get((idx, slot))
    if s is None:
        s = own_stream(idx, f"side{slot}")
        _SIDE_STREAMS[(idx, slot)] = s
    return s


def join_capture_streams(device: torch.device) -> int:
    """Make the capturing current stream wait for every side stream (the C++
    fork's and ops.side_stream's) that joined its capture -- the last
    operation of a hipGraph capture (hlhgat.train.TrainStep)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    extra = [s.cuda_stream for (d, _), s in _SIDE_STREAMS.items() if d == idx]
    return int(_ext.join_capture_streams(idx, extra))


def side_streams_capturing(device: torch.device) -> List[int]:
    """raw handles of the side streams still part of an active capture"""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    cand = [s.cuda_stream for (d, _), s in _SIDE_STREAMS.items() if d == idx]
    cand.append(int(_ext.fork_side_stream(idx)))
    return [h for h in cand if _ext.stream_capturing(h)]


def _tensors(x):
    if torch.is_tensor(x):
        yield x
    elif isinstance(x, (list, tuple)):
        for v in x:
            yield from _tensors(v)


_CHAIN = None  # the active Chains, or None
CHAINS_ENABLED = True  # A/B hook: False = a fork / join per HL block


class Chains:
    """The node and edge chains of a model's HL blocks on two streams for the
    whole block section of a forward, instead of a fork / join per block
    (lib/Hodge_ST_Model.py:608-633: each block's node and edge convs are
    independent; only NodeEdgeInt exchanges features between them).

    Inside ``with Chains(device) as ch:`` a two-chain Sequential (an HL block)
    runs its edge half on the side stream without waiting for the main stream
    and without a join, and the fused NodeEdgeInt keeps its edge MLP on the
    side stream (torch_ext.cpp chain mode): the exchange of the two
    first-layer GEMM results is the only cross-stream dependency per block.
    Entering makes the side stream wait for the main stream (the batch, the
    slabs, the weight packs); ``ch.sync_side()`` does so again (e.g. after
    tables built on the main stream); leaving joins the side stream into the
    main stream.  Values are unchanged (the same kernels in the same order on
    each stream).  A cross-stream hazard of a hipGraph capture is caught the
    same way as for ``fork``: the side stream is joined before capture end."""

    def __init__(self, device, enabled: bool = True):
        self.device = device
        self.on = (enabled and CHAINS_ENABLED and _FORK_ENABLED and device is not None
                   and device.type == "cuda" and _ext is not None)

    def __enter__(self):
        global _CHAIN
        if self.on:
            if _CHAIN is not None:
                raise RuntimeError("hlhgat: Chains do not nest")
            self.main = torch.cuda.current_stream(self.device)
            # the C++ fork's side stream: the fused NodeEdgeInt's edge half runs
            # there, so the edge convs must too (one edge stream, no syncs between)
            idx = (self.device.index if self.device.index is not None
                   else torch.cuda.current_device())
            self.side = torch.cuda.ExternalStream(int(_ext.fork_side_stream(idx)),
                                                  device=self.device)
            self.side.wait_stream(self.main)
            _CHAIN = self
            _ext.set_chain(True)
        return self

    def sync_side(self) -> None:
        if self.on:
            self.side.wait_stream(self.main)

    def side_context(self):
        """Issue (and record for autograd) on the edge chain's stream."""
        return torch.cuda.stream(self.side) if self.on else contextlib.nullcontext()

    def to_main(self, *ts):
        """Side-chain tensors handed to the main stream after the join."""
        if self.on:
            for t in _tensors(ts):
                t.record_stream(self.main)
        return ts if len(ts) != 1 else ts[0]

    def __exit__(self, *exc):
        global _CHAIN
        if self.on:
            _ext.set_chain(False)
            _CHAIN = None
            self.main.wait_stream(self.side)
        return False


def active_chains(device):
    """The active Chains on `device`, or None."""
    ch = _CHAIN
    if ch is None or device is None or ch.device != device:
        return None
    return ch


def fork(fn_main, fn_side, side_inputs=(), device=None, slot=0):
    """Run fn_main() on the current stream and fn_side() on the side stream
    concurrently; returns (fn_main(), fn_side()) with the side results ordered
    before anything issued next on the current stream.  Tensors in
    side_inputs (produced on the current stream) are kept alive for the side
    stream's use."""
    if not _FORK_ENABLED or device is None or device.type != "cuda":
        return fn_main(), fn_side()
    main = torch.cuda.current_stream(device)
    side = side_stream(device, slot)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        for t in _tensors(side_inputs):
            t.record_stream(side)
        out_side = fn_side()
    out_main = fn_main()
    main.wait_stream(side)
    for t in _tensors(out_side):
        t.record_stream(main)
    return out_main, out_side


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
    order: Optional[torch.Tensor] = None  # int32 [n_rows] row schedule (locality_order)
    valid: Optional[torch.Tensor] = None  # int32 [1]: rows >= valid are static-shape padding
    # halo tiles (tile_ptr, halo_ptr, halo, lcol, max_halo) for the LDS-staged
    # SpMM of large Laplacians (hodge_dataset.halo_tiles; hlhgat_halo_t)
    halo: Optional[tuple] = None


@dataclass
class HodgeOperator:
    """A Laplacian as used by propagate: fwd = CSR keyed by edge_index[1]
    (Y[t] = sum w * X[s]), bwd = its transpose (keyed by edge_index[0]).
    ``factor`` (an L1 = alpha B1^T B1 declared by set_hodge_factor): the 7
    tensors of hlhgat_hodge_factor_t and the node count; the polynomial
    bases then run factored (hlhgat_poly_basis_*_factored)."""
    fwd: SparseCSR
    bwd: SparseCSR
    factor: Optional[tuple] = None
    factor_nodes: int = 0


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
_RCP_CACHE = _IdCache()


def clear_caches() -> None:
    _HODGE_CACHE.clear()
    _INC_CACHE.clear()
    _RCP_CACHE.clear()


def reciprocal(D: torch.Tensor) -> torch.Tensor:
    """(1 / D).view(-1) (lib/Hodge_Cheb_Conv.py:294), computed once per D
    tensor: every NodeEdgeInt of a block group divides by the same degrees.
    Gradients do not flow into D (the reference's D is an integer count)."""
    if D.requires_grad:
        return (1 / D).view(-1)
    pre = getattr(D, "_hlhgat_rcp", None)  # built with the batch (hodge_dataset.node_degree)
    if pre is not None and pre.shape == D.shape and pre.device == D.device:
        return pre.view(-1)
    hit = _RCP_CACHE.get([D], None)
    if hit is not None:
        return hit
    return _RCP_CACHE.put([D], None, (1 / D).view(-1))


def mark_hodge(edge_index: torch.Tensor) -> torch.Tensor:
    """Declare that edge_index/edge_weight describe a symmetric operator whose
    COO is sorted by (row, col) — true for every Laplacian the Hodge builder
    emits via dense_to_sparse (lib/Hodge_Dataset.py:455-456,467-468) and for
    PairData batches of them (block-diagonal, offsets :40-48).  Enables the
    sort-free CSR build and reuse of one CSR for forward and adjoint."""
    edge_index._hlhgat_sorted_symmetric = True  # type: ignore[attr-defined]
    return edge_index


def set_row_order(edge_index: torch.Tensor, order: torch.Tensor) -> torch.Tensor:
    """Attach a row schedule (a permutation of the operator's rows, e.g.
    hodge_dataset.locality_order) to a Laplacian's edge_index: every SpMM /
    polynomial-basis launch over the operator built from it visits rows in
    that order (same results, better L2 locality on large graphs)."""
    edge_index._hlhgat_row_order = order.to(device=edge_index.device,  # type: ignore
                                            dtype=torch.int32).contiguous()
    return edge_index


def set_valid(edge_index: torch.Tensor, n_valid: torch.Tensor, attr: str = "_hlhgat_valid"
              ) -> torch.Tensor:
    """Declare the rows >= n_valid (device int32 [1]) of the operator built
    from edge_index as static-shape padding (hodge_dataset.pad_batch): the
    BatchNorm statistics of its layers use the valid rows only."""
    setattr(edge_index, attr, n_valid.to(device=edge_index.device, dtype=torch.int32).view(1))
    return edge_index


def set_halo(edge_index: torch.Tensor, ht: dict) -> torch.Tensor:
    """Attach halo tiles (hodge_dataset.halo_tiles, built for this operator's
    CSR and row schedule) to a sorted symmetric Laplacian's edge_index: its
    SpMM / polynomial steps then stage each tile's entries and neighbour rows
    in LDS (k_poly_halo; bitwise the same results)."""
    dev = edge_index.device
    i32 = lambda k: ht[k].to(dev, torch.int32).contiguous()  # noqa: E731
    edge_index._hlhgat_halo = (  # type: ignore[attr-defined]
        i32("halo_tile_ptr"), i32("halo_ptr"), i32("halo"), i32("halo_srp"),
        ht["halo_lcol"].to(dev, torch.int16).contiguous(), i32("halo_eperm"),
        [int(v) for v in ht["halo_bounds"]], i32("halo_hdr"))
    return edge_index


# Factored L1 (hlhgat_hodge_factor_t): on for the operators collate declares
# (hodge_dataset.hodge_factor_ok: exact identity, >= FACTOR_MIN_ROW entries per
# row); HLHGAT_FACTOR=0 keeps the bitwise CSR path everywhere.
FACTOR_ENABLED = os.environ.get("HLHGAT_FACTOR", "1") != "0"


def set_hodge_factor(edge_index_s: torch.Tensor, edge_index: torch.Tensor, n_nodes: int,
                     node_order: Optional[torch.Tensor] = None,
                     tables: Optional[tuple] = None) -> torch.Tensor:
    """Declare that the L1 built from (edge_index_s, edge_weight_s) equals
    alpha_e * B1^T B1 with B1 the boundary of ``edge_index`` ([2, E], i < j,
    adj2par1 lib/Hodge_Dataset.py:169-191) on n_nodes nodes -- exactly, as
    every L1 of the Hodge builder is (lib/Hodge_Dataset.py:451-456); the
    caller has checked it (hodge_dataset.hodge_factor_ok).  Polynomial bases
    over it then gather ~4 rows per edge instead of nnz/E (hlhgat.h).
    ``tables`` = (alpha [E] f32, signs [2E] f32 in incidence-CSR order,
    ends [E, 2] int32) built at collate time (hodge_dataset.factor_tables):
    the operator then takes them instead of building them on the device (in
    a captured step, every replay)."""
    edge_index_s._hlhgat_factor = (edge_index, int(n_nodes), node_order,  # type: ignore
                                   tables)
    return edge_index_s


def has_hodge_factor(edge_index_s: torch.Tensor) -> bool:
    """Whether set_hodge_factor declared this L1 (its polynomial bases then
    take the factored path when FACTOR_ENABLED)."""
    return getattr(edge_index_s, "_hlhgat_factor", None) is not None


def _build_factor(op: "HodgeOperator", ei_s: torch.Tensor, w: torch.Tensor, decl) -> None:
    """The device tensors of hlhgat_hodge_factor_t for op (no host sync)."""
    edge_index, n_nodes, node_order, tables = decl
    E = op.fwd.n_rows
    if edge_index.size(1) != E:
        raise RuntimeError(f"hlhgat: hodge factor: B1 has {edge_index.size(1)} edges, "
                           f"L1 has {E} rows")
    inc = incidence(edge_index, n_nodes)
    dev = ei_s.device
    if tables is not None:  # collate-time tables: no device work here
        alpha, signs, ends = tables
        if (alpha.numel() != E or signs.numel() != 2 * E or tuple(ends.shape) != (E, 2)
                or alpha.device != dev or signs.device != dev or ends.device != dev):
            raise RuntimeError("hlhgat: hodge factor tables do not match the operator "
                               f"({alpha.numel()}, {signs.numel()}, {tuple(ends.shape)}; E={E})")
    else:
        diag = ei_s[0] == ei_s[1]
        alpha = torch.zeros(E, device=dev, dtype=torch.float32)
        alpha.index_put_((ei_s[0],), torch.where(diag, w * 0.5, torch.zeros_like(w)),
                         accumulate=True)
        signs = _incidence_signs(inc)
        ends = edge_index.t().to(torch.int32).contiguous()
    none_i = torch.empty(0, dtype=torch.int32, device=dev)
    no = (node_order.to(dev, torch.int32).contiguous() if node_order is not None else none_i)
    eo = op.fwd.order if op.fwd.order is not None else none_i
    op.factor = (inc.rowptr, inc.edge_ids, signs, no, ends, alpha, eo)
    op.factor_nodes = int(n_nodes)


def _attach_halo(a: "SparseCSR", halo) -> None:
    """A.halo = (tile_ptr, halo_ptr, halo, srp, lcol, sval, bounds); sval =
    the CSR values in schedule order, gathered on device once per operator."""
    tp, hp, hc, srp, lcol, eperm, bounds, hdr = halo
    if lcol.numel() != a.nnz:
        raise RuntimeError("hlhgat: halo tiles were built for a different operator")
    sval = None
    if a.val is not None and a.nnz:
        sval = torch.empty_like(a.val)
        check(LIB.hlhgat_gather_f32(a.val.data_ptr(), eperm.data_ptr(), a.nnz,
                                    sval.data_ptr(), _stream(a.val)), "gather_f32")
    a.halo = (tp, hp, hc, srp, lcol, sval, bounds, hdr)


def _halo_desc(A: "SparseCSR"):
    """ctypes pointer to an hlhgat_halo_t for A, or None."""
    if A.halo is None:
        return None
    tp, hp, hc, srp, lc, sval, (mh, mr, mn), hdr = A.halo
    d = _lib.HaloDesc(hdr.data_ptr(), tp.data_ptr(), hp.data_ptr(), hc.data_ptr(), srp.data_ptr(),
                      lc.data_ptr(), _ptr(sval), tp.numel() - 1, mh, mr, mn)
    return C.pointer(d)


def _halo_args(A: "SparseCSR"):
    """The halo arguments of the C++ conv node (Nones when A has none)."""
    if A.halo is None:
        return (None, None, None, None, None, None, [0, 0, 0], None)
    return A.halo


_CHECK_SIZES = os.environ.get("HLHGAT_CHECK_SIZES", "0") == "1"


def hodge_build(edge_index: torch.Tensor, node_counts, lmax: Optional[torch.Tensor] = None,
                steps: int = 64, sizes=None):
    """Hodge Laplacians of a block-diagonal batch ON DEVICE (hlhgat_hodge_*):
    edge_index int64 [2, E] (i < j, PairData offsets), node_counts per graph.
    lmax per graph: given (float, as the reference's eigh result) or computed
    by the on-device Lanczos (fp64).  Returns (ei_t, w_t, ei_s, w_s, lmax) with
    the COO in the reference's dense_to_sparse order (row-major, zeros
    dropped) and entries fl(fl(2 v) / lmax) (lib/Hodge_Dataset.py:451-468).
    sizes = (N, nnz(L0), nnz(L1)) when the caller knows them (nnz(L0) = the
    non-isolated nodes + 2 E, nnz(L1) = sum deg^2 - E): then nothing here
    waits on the device (HLHGAT_CHECK_SIZES=1 compares them with the device's
    own row sizes).  Sizes that do not fit the graph never write past the
    buffers: the build kernels raise HLHGAT_DEVERR_HODGE_SIZE instead
    (check_device_errors reports it)."""
    _req_dev(edge_index, "edge_index", torch.int64)
    dev = edge_index.device
    counts = torch.as_tensor(node_counts, dtype=torch.int64).to(dev)
    B = counts.numel()
    node_ptr = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    node_ptr[1:] = torch.cumsum(counts, 0)
    N = int(sizes[0]) if sizes is not None else int(node_ptr[-1].item())
    ei = edge_index.contiguous()
    E = ei.size(1)
    inc = incidence(ei, N)
    st = _stream(ei)
    if lmax is None:
        wsb = int(LIB.hlhgat_hodge_lmax_workspace_bytes(N, steps))
        ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=dev)
        lam64 = torch.empty(B, dtype=torch.float64, device=dev)
        check(LIB.hlhgat_hodge_lmax(inc.rowptr.data_ptr(), inc.edge_ids.data_ptr() if E else None,
                                    ei.data_ptr() if E else None, E, N, node_ptr.data_ptr(), B,
                                    steps, lam64.data_ptr(), ws.data_ptr(), wsb, st), "hodge_lmax")
        lam = lam64.to(torch.float32)
    else:
        lam = torch.as_tensor(lmax, dtype=torch.float32).to(dev).reshape(B)
    lam_node = torch.repeat_interleave(lam, counts, output_size=N).contiguous()
    sz0 = torch.empty(N, dtype=torch.int32, device=dev)
    sz1 = torch.empty(E, dtype=torch.int32, device=dev)
    check(LIB.hlhgat_hodge_row_sizes(inc.rowptr.data_ptr(), _ptr(ei) if E else None, E, N,
                                     sz0.data_ptr(), sz1.data_ptr(), st), "hodge_row_sizes")
    rp0 = torch.zeros(N + 1, dtype=torch.int32, device=dev)
    rp1 = torch.zeros(E + 1, dtype=torch.int32, device=dev)
    rp0[1:] = torch.cumsum(sz0, 0)
    rp1[1:] = torch.cumsum(sz1, 0)
    if sizes is not None:
        nnz0, nnz1 = int(sizes[1]), int(sizes[2])
        if _CHECK_SIZES:
            got = (int(node_ptr[-1].item()), int(rp0[-1].item()), int(rp1[-1].item()))
            if got != (N, nnz0, nnz1):
                raise RuntimeError(f"hlhgat: hodge_build sizes {tuple(sizes)} != device {got}")
    else:
        nnz0, nnz1 = int(rp0[-1].item()), int(rp1[-1].item())
    # caller's sizes: zero-filled, so entries past the device's rows (sizes
    # too large: HLHGAT_DEVERR_HODGE_SIZE) hold in-range column 0, never garbage
    alloc = torch.empty if sizes is None else torch.zeros
    c0 = alloc(max(nnz0, 1), dtype=torch.int32, device=dev)
    v0 = alloc(max(nnz0, 1), dtype=torch.float32, device=dev)
    c1 = alloc(max(nnz1, 1), dtype=torch.int32, device=dev)
    v1 = alloc(max(nnz1, 1), dtype=torch.float32, device=dev)
    # the kernels check every row against these capacities (a caller's sizes
    # that do not fit the graph raise HLHGAT_DEVERR_HODGE_SIZE, nothing past
    # the buffers is written)
    check(LIB.hlhgat_hodge_build(inc.rowptr.data_ptr(), inc.edge_ids.data_ptr() if E else None,
                                 _ptr(ei) if E else None, E, N, lam_node.data_ptr(), rp0.data_ptr(),
                                 c0.data_ptr(), v0.data_ptr(), nnz0,
                                 rp1.data_ptr(), c1.data_ptr(), v1.data_ptr(),
                                 nnz1, st), "hodge_build")

    def coo(rp, c, v, n, nnz):
        if sizes is not None:
            # a caller's nnz may not match the device's rows (then the build
            # raised HLHGAT_DEVERR_HODGE_SIZE): the row of entry k by binary
            # search over the clamped row pointers -- repeat_interleave with an
            # output_size other than the sum of the repeats trips torch's
            # device-side assert, a GPU exception that ends the process's context
            rp = rp.clamp(max=nnz)
            k = torch.arange(nnz, device=dev, dtype=torch.int32)
            rows = torch.searchsorted(rp[1:], k, right=True).clamp_(max=max(n - 1, 0))
        else:
            rows = torch.repeat_interleave(torch.arange(n, device=dev), (rp[1:] - rp[:-1]).long(),
                                           output_size=nnz)
        return torch.stack([rows, c[:nnz].long()]), v[:nnz]

    ei_t, w_t = coo(rp0, c0, v0, N, nnz0)
    ei_s, w_s = coo(rp1, c1, v1, E, nnz1)
    return ei_t, w_t, ei_s, w_s, lam


def eig_pe(edge_index: torch.Tensor, node_counts, k: int, max_nodes: Optional[int] = None,
           n_nodes: Optional[int] = None):
    """Eigenvector PE of every graph of a block-diagonal batch and its
    lambda_max, on the device in one launch (hlhgat_eig_pe; the reference's
    per-sample eig_pe(L0) and eigh(L0).max(), lib/Hodge_Dataset.py:97-112,
    :782): edge_index int64 [2, E] (i < j, PairData offsets), node_counts per
    graph (a host sequence, or a device tensor with max_nodes given; n_nodes,
    their sum, spares a device read).
    Returns (pe float32 [N, k - 1]: eigenvectors 1 .. k-1 of each graph's L0,
    ascending, zero columns past a graph's own size; lmax float64 [B])."""
    _req_dev(edge_index, "edge_index", torch.int64)
    dev = edge_index.device
    if torch.is_tensor(node_counts) and node_counts.is_cuda:
        if max_nodes is None:
            raise ValueError("eig_pe: max_nodes is required with device node counts")
        counts = node_counts.to(torch.int64)
        N = None if n_nodes is None else int(n_nodes)
    else:
        host = [int(c) for c in node_counts]
        mx = max(host) if host else 0
        if max_nodes is not None and int(max_nodes) < mx:
            raise ValueError(f"eig_pe: max_nodes {max_nodes} < largest graph {mx}")
        max_nodes = mx if max_nodes is None else int(max_nodes)
        counts = torch.tensor(host, dtype=torch.int64).to(dev)
        N = sum(host)
    B = counts.numel()
    node_ptr = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    node_ptr[1:] = torch.cumsum(counts, 0)
    if N is None:
        N = int(node_ptr[-1].item())
    ei = edge_index.contiguous()
    E = ei.size(1)
    inc = incidence(ei, N)
    pe = torch.empty(N, k - 1, dtype=torch.float32, device=dev)
    lmax = torch.empty(B, dtype=torch.float64, device=dev)
    wsb = int(LIB.hlhgat_eig_pe_workspace_bytes(B, int(max_nodes), k))
    ws = torch.empty(max(wsb, 8), dtype=torch.uint8, device=dev)
    check(LIB.hlhgat_eig_pe(inc.rowptr.data_ptr(), inc.edge_ids.data_ptr() if E else None,
                            ei.data_ptr() if E else None, E, N, node_ptr.data_ptr(), B,
                            int(max_nodes), k, pe.data_ptr(), k - 1, lmax.data_ptr(), ws.data_ptr(),
                            wsb, _stream(ei)), "eig_pe")
    return pe, lmax


def copy_words_batched(srcs: Sequence[torch.Tensor], dsts: Sequence[torch.Tensor]) -> None:
    """dst.copy_(src) for contiguous same-size tensors whose byte size is a
    multiple of 4, up to HLHGAT_MAX_COPY_BLOCKS per launch
    (hlhgat_copy2d_batched over 4-byte words), on the current stream."""
    n = len(srcs)
    for i in range(0, n, _lib.MAX_COPY_BLOCKS):
        ss, ds = srcs[i:i + _lib.MAX_COPY_BLOCKS], dsts[i:i + _lib.MAX_COPY_BLOCKS]
        words = [t.numel() * t.element_size() // 4 for t in ss]
        m = len(ss)
        check(LIB.hlhgat_copy2d_batched(
            m, _arr(C.c_void_p, [t.data_ptr() for t in ss]), _arr(C.c_int64, words),
            _arr(C.c_void_p, [t.data_ptr() for t in ds]), _arr(C.c_int64, words),
            _arr(C.c_int64, [1] * m), _arr(C.c_int64, words), _stream(ds[0])), "copy2d_batched")


def _factor_args(op: "HodgeOperator"):
    """The factor arguments of the C++ conv node ([] = CSR path)."""
    if op.factor is None:
        return ([], 0)
    return (list(op.factor), op.factor_nodes)


def _factor_desc(op: "HodgeOperator"):
    nr, ne, ns, no, ends, alpha, eo = op.factor
    return C.pointer(_lib.HodgeFactorDesc(
        nr.data_ptr(), ne.data_ptr() if ne.numel() else None, ns.data_ptr() if ns.numel() else None,
        no.data_ptr() if no.numel() else None, op.factor_nodes, ends.data_ptr(),
        alpha.data_ptr(), eo.data_ptr() if eo.numel() else None, op.fwd.n_rows))


def hodge_spmm(op: "HodgeOperator", X: torch.Tensor) -> torch.Tensor:
    """Y = L1 X through the factorisation (op must carry one; no autograd)."""
    if op.factor is None:
        raise RuntimeError("hlhgat: hodge_spmm needs a factored operator (set_hodge_factor)")
    X = _rows2d(X, "X")
    Y = torch.empty(op.fwd.n_rows, X.size(1), device=X.device, dtype=X.dtype)
    work = torch.empty(int(LIB.hlhgat_hodge_factor_work_floats(op.factor_nodes, X.size(1))),
                       device=X.device)
    check(LIB.hlhgat_hodge_spmm(_factor_desc(op), X.data_ptr(), _ld(X), X.size(1), Y.data_ptr(),
                                _ld(Y), work.data_ptr(), _stream(X)), "hodge_spmm")
    return Y


def _hodge_step(op: "HodgeOperator", X: torch.Tensor, Y: torch.Tensor, *, Z=None, P=None,
                Q=None, alpha=1.0, beta=0.0, gamma=0.0, div=1.0, p=0.0, q=0.0,
                work: Optional[torch.Tensor] = None) -> None:
    """_poly_step with the factored L1 of op (hlhgat_hodge_poly_step)."""
    if work is None:
        work = torch.empty(int(LIB.hlhgat_hodge_factor_work_floats(op.factor_nodes, X.size(1))),
                           device=X.device)
    check(LIB.hlhgat_hodge_poly_step(
        _factor_desc(op), X.data_ptr(), _ld(X), X.size(1), _ptr(Z), _ld(Z) if Z is not None else 0,
        _ptr(P), _ld(P) if P is not None else 0, _ptr(Q), _ld(Q) if Q is not None else 0, alpha,
        beta, gamma, div, p, q, Y.data_ptr(), _ld(Y), work.data_ptr(), _stream(X)),
        "hodge_poly_step")


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
    order = getattr(edge_index, "_hlhgat_row_order", None)
    if order is not None and order.numel() != n:
        raise RuntimeError(f"hlhgat: row schedule has {order.numel()} entries, operator {n} rows")
    valid = getattr(edge_index, "_hlhgat_valid", None)
    if getattr(edge_index, "_hlhgat_sorted_symmetric", False):
        pre = getattr(edge_index, "_hlhgat_csr", None)  # built at collate (set_csr)
        if pre is not None and pre[0].numel() == n + 1 and pre[1].numel() == ei.size(1):
            a = SparseCSR(pre[0], pre[1], w, n, n, ei.size(1))
        else:
            a = _csr_sorted(ei[0], ei[1], w, n, n)
        a.order = order
        a.valid = valid
        halo = getattr(edge_index, "_hlhgat_halo", None)
        if halo is not None:  # built for the COO order = this CSR's entry order
            _attach_halo(a, halo)
        op = HodgeOperator(a, a)
        decl = getattr(edge_index, "_hlhgat_factor", None)
        if decl is not None and FACTOR_ENABLED and w is not None:
            _build_factor(op, ei, w, decl)
    else:
        fwd = _csr_general(ei[1], ei[0], w, n, n)
        bwd = _csr_general(ei[0], ei[1], w, n, n)
        for c in (fwd, bwd):
            c.order = order
            c.valid = valid
        op = HodgeOperator(fwd, bwd)
    return _HODGE_CACHE.put(keys, n, op)


def set_csr(edge_index: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor) -> torch.Tensor:
    """Attach the CSR of a sorted symmetric Laplacian COO built with the batch
    (hodge_dataset.laplacian_csr, at collate): int32 rowptr over edge_index[0]
    and int32 columns; the values are edge_weight itself.  hodge_operator then
    uses it instead of hlhgat_csr_from_sorted_coo (the same arrays, bitwise)."""
    edge_index._hlhgat_csr = (  # type: ignore[attr-defined]
        rowptr.to(device=edge_index.device, dtype=torch.int32).contiguous(),
        col.to(device=edge_index.device, dtype=torch.int32).contiguous())
    return edge_index


def set_incidence(edge_index: torch.Tensor, rowptr: torch.Tensor,
                  edge_ids: torch.Tensor) -> torch.Tensor:
    """Attach the incidence CSR of |B1| built with the batch
    (hodge_dataset.incidence_csr, at collate): ``incidence`` then uses it
    instead of sorting on the device.  It must be the CSR hlhgat_incidence_csr
    builds (rows = nodes, incident edge ids ascending; tests check bitwise)."""
    edge_index._hlhgat_incidence = (  # type: ignore[attr-defined]
        rowptr.to(device=edge_index.device, dtype=torch.int32).contiguous(),
        edge_ids.to(device=edge_index.device, dtype=torch.int32).contiguous())
    return edge_index


def incidence(edge_index: torch.Tensor, n_nodes: int) -> Incidence:
    """Incidence CSR of |B1| built from the undirected edge list (i<j)."""
    _req_dev(edge_index, "edge_index", torch.int64)
    hit = _INC_CACHE.get([edge_index], n_nodes)
    if hit is not None:
        return hit
    ei = edge_index.contiguous()
    E = ei.size(1)
    dev = ei.device
    pre = getattr(edge_index, "_hlhgat_incidence", None)
    if pre is not None:
        rowptr, eids = pre
        if rowptr.numel() != n_nodes + 1 or eids.numel() != 2 * E:
            raise RuntimeError(f"hlhgat: attached incidence CSR has {rowptr.numel() - 1} rows / "
                               f"{eids.numel()} entries, expected {n_nodes} / {2 * E}")
        inc = Incidence(rowptr, eids, ei, n_nodes, E)
        signs = getattr(edge_index, "_hlhgat_inc_signs", None)  # collate-time (factor tables)
        if torch.is_tensor(signs) and signs.numel() == 2 * E and signs.device == dev:
            inc._signs = signs  # type: ignore[attr-defined]
        return _INC_CACHE.put([edge_index], n_nodes, inc)
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
        _ptr(rs), A.n_rows, A.nnz, _ptr(A.order), _halo_desc(A), X.data_ptr(), _ld(X), d,
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
                              _ptr(A.order), _halo_desc(A), X.data_ptr(), _ld(X), X.size(1),
                              Y.data_ptr(),
                              _ld(Y),
                              _stream(X)), "spmm")
    return Y


def poly_basis(op: HodgeOperator, X: torch.Tensor, K: int, kind: int) -> torch.Tensor:
    """T_1..T_{K-1} as a [K-1, n, F] slab (no autograd)."""
    n, F = X.size(0), X.size(1)
    T = torch.empty(max(K - 1, 0), n, F, device=X.device, dtype=X.dtype)
    if K > 1 and n > 0 and op.factor is not None:
        work = torch.empty(int(LIB.hlhgat_hodge_factor_work_floats(op.factor_nodes, F)),
                           device=X.device)
        check(LIB.hlhgat_poly_basis_fwd_factored(kind, _factor_desc(op), X.data_ptr(), _ld(X), F,
                                                 K, T.data_ptr(), work.data_ptr(), _stream(X)),
              "poly_basis_fwd_factored")
    elif K > 1 and n > 0:
        A = op.fwd
        check(LIB.hlhgat_poly_basis_fwd(kind, A.rowptr.data_ptr(),
                                        A.col.data_ptr() if A.nnz else None,
                                        _ptr(A.val) if A.nnz else None, n, A.nnz,
                                        _ptr(A.order), _halo_desc(A), X.data_ptr(), _ld(X), F,
                                        K, T.data_ptr(),
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
def _bn_args(bn: Optional[torch.nn.BatchNorm1d]):
    """(weight, bias, running_mean, running_var, num_batches_tracked, momentum,
    eps) for a training-mode BatchNorm1d, torch semantics."""
    track = bn.training and bn.track_running_stats and bn.running_mean is not None
    if track and bn.momentum is None:
        momentum = 1.0 / float(bn.num_batches_tracked.item() + 1)
    else:
        momentum = float(bn.momentum) if bn.momentum is not None else 0.0
    return (bn.weight, bn.bias, bn.running_mean if track else None,
            bn.running_var if track else None, bn.num_batches_tracked if track else None,
            momentum, float(bn.eps))


def _bn_uses_batch_stats(bn) -> bool:
    return bn.training or not bn.track_running_stats


def hodge_poly_conv(x: torch.Tensor, op: HodgeOperator, weights: Sequence[torch.Tensor],
                    bias: Optional[torch.Tensor], kind: int = POLY_LAGUERRE,
                    bn: Optional[torch.nn.BatchNorm1d] = None, relu: bool = False,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = sum_k T_k W_k^T + bias with T_k the Laguerre / Chebyshev basis of
    x over L (lib/Hodge_Cheb_Conv.py:480-515 / :394-439); x may be [N, C] or
    [N, T, C] (3-D inputs propagate over [N, T*C] rows, :493-505).  With
    ``bn`` the following BatchNorm (and ReLU) of the HL block runs inside the
    same C++ autograd node (lib/Hodge_ST_Model.py:556-566).  ``out`` (a
    DenseConcat sink) receives the final output when the conv, BN and ReLU run
    as one node; otherwise it is ignored and the caller copies."""
    _req_dev(x, "x")
    if x.size(0) != op.fwd.n_rows:
        raise RuntimeError(f"hlhgat: x has {x.size(0)} rows but the operator has "
                           f"{op.fwd.n_rows}")
    A, At = op.fwd, op.bwd
    ws = list(weights)
    if bn is not None and x.dim() == 2 and _bn_uses_batch_stats(bn) and sync_bn_group(bn) is None:
        if x.size(0) < 2 and bn.training:
            raise ValueError("Expected more than 1 value per channel when training")
        return _ext.conv_bn(x, A.rowptr, A.col, A.val, At.rowptr, At.col, At.val, A.nnz, kind,
                            ws, bias, *_bn_args(bn), 2 if relu else 1, out, A.order, At.order,
                            A.valid, *_halo_args(A), *_factor_args(op))
    sink = out if (bn is None and not relu and x.dim() == 2) else None
    y = _ext.conv_bn(x, A.rowptr, A.col, A.val, At.rowptr, At.col, At.val, A.nnz, kind, ws,
                     bias, None, None, None, None, None, 0.0, 0.0, 0, sink, A.order, At.order,
                     A.valid, *_halo_args(A), *_factor_args(op))
    if bn is not None:
        y = batch_norm_act(y, bn, relu, valid=A.valid)
    elif relu:
        y = torch.relu(y)
    return y


# ----------------------------------------------------------------------------
# Dense concatenation of the HL blocks in one slab
# ----------------------------------------------------------------------------
DENSE_SLAB = True   # tests set False: the torch.cat concatenation
GRAD_SINK = True


class DenseConcat:
    """The running concatenation x0 = cat[y_0, y_1, ...] of the dense HL
    blocks (lib/Hodge_ST_Model.py:631-632: x_t0 = torch.cat([x_t0, x_t], -1))
    held in ONE preallocated [rows, width] slab.

    Each block output is written straight into its column block (``sink``
    hands the conv a destination; ``append`` copies only when the producer
    could not write there), and ``view()`` returns x0 as a column prefix of the
    slab: no O(depth^2) re-copies in the forward.  In the backward, every
    view's gradient is accumulated into one gradient slab and each block's
    output gradient is handed out as a column block of it, so the per-block
    slice / add / copy kernels of torch.cat's backward disappear too.  Forward
    values are identical to the torch.cat formulation; gradients are the same
    fp32 sums, accumulated in view order (tests: tolerance of the model)."""

    def __init__(self, rows: int, width: int, like: torch.Tensor):
        self.S = torch.empty(rows, width, dtype=torch.float32, device=like.device)
        self.width = width
        # backward-side state shared by the views; it holds no reference to the
        # parts, so the autograd graph and this object do not form a cycle
        self._state = _DenseGrad(self.S)
        self.parts: List[torch.Tensor] = []
        self.cols: List[Tuple[int, int]] = []
        self.owned: List[bool] = []  # part's gradient already handed to a view

    @property
    def used(self) -> int:
        return self.cols[-1][1] if self.cols else 0

    def sink(self, w: int) -> torch.Tensor:
        c0 = self.used
        if c0 + w > self.width:
            raise RuntimeError(f"hlhgat: DenseConcat overflow ({c0}+{w} > {self.width})")
        return self.S[:, c0:c0 + w]

    def append(self, y: torch.Tensor) -> None:
        if y.dim() != 2 or y.size(0) != self.S.size(0):
            raise RuntimeError(f"hlhgat: DenseConcat rows {self.S.size(0)}, got {tuple(y.shape)}")
        c0 = self.used
        c1 = c0 + y.size(1)
        if c1 > self.width:
            raise RuntimeError(f"hlhgat: DenseConcat overflow ({c1} > {self.width})")
        if y.data_ptr() != self.S.data_ptr() + 4 * c0 or y.stride(0) != self.S.stride(0):
            # through .data (its own version counter): columns [c0, c1) are
            # outside every view handed out so far, and a tracked in-place
            # copy would bump the version counter those views share with S
            self.S.data[:, c0:c1].copy_(y.detach())
        self.parts.append(y)
        self.cols.append((c0, c1))
        self.owned.append(False)

    def grad_sink(self) -> Optional[torch.Tensor]:
        """The gradient slab's view of the current x0 = view() (columns
        [0, used)): a consumer whose backward ADDS its input gradient into
        this view (NodeEdgeInt, accumulate_d of hlhgat_proj_bwd) spares the
        view's backward its add.  Returns (view, flag): the host int32 flag
        says whether a gradient has landed in the slab yet -- the first
        writer overwrites, the later ones add, so the slab is never zeroed."""
        if (not GRAD_SINK or not torch.is_grad_enabled()
                or not any(p.requires_grad for p in self.parts)):
            return None
        if self._state.G is None:
            # not zero-filled: the first gradient to land overwrites (flag)
            self._state.G = torch.empty_like(self.S)
            self._state.sink = True
        return self._state.G[:, :self.used], self._state.written

    def view(self) -> torch.Tensor:
        w = self.used
        if not torch.is_grad_enabled() or not any(p.requires_grad for p in self.parts):
            return self.S[:, :w]
        # the first view created after a part was appended is the last of the
        # views to run backward that covers it: it hands out that part's gradient
        ranges = [(c0, c1, not o) for (c0, c1), o in zip(self.cols, self.owned)]
        self.owned = [True] * len(self.owned)
        return _DenseViewFn.apply(self._state, ranges, w, *self.parts)


class _DenseGrad:
    def __init__(self, S: torch.Tensor):
        self.S = S
        self.G: Optional[torch.Tensor] = None
        self.sink = False  # G was handed out as a gradient sink (grad_sink)
        self.written = torch.zeros(1, dtype=torch.int32)  # host flag: G holds a gradient


class _DenseViewFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, state, ranges, w, *parts):
        ctx.state, ctx.ranges, ctx.w = state, ranges, w
        return state.S[:, :w]

    @staticmethod
    def backward(ctx, g):
        st, w = ctx.state, ctx.w
        if st.G is None:
            # first view to run backward = the widest (created last): it
            # initialises every column the narrower views accumulate into
            st.G = torch.empty_like(st.S)
            st.G[:, :w].copy_(g)
        elif (st.sink and g.data_ptr() == st.G.data_ptr() and g.shape == (st.G.size(0), w)
              and g.stride() == st.G[:, :w].stride()):
            pass  # the consumer already added its gradient into the slab (grad_sink)
        elif st.sink and int(st.written[0]) == 0:
            st.G[:, :w].copy_(g)  # first gradient into a sink slab: overwrite
            st.written[0] = 1
        else:
            st.G[:, :w].add_(g)
        grads = [st.G[:, c0:c1] if own else None for c0, c1, own in ctx.ranges]
        return (None, None, None, *grads)


# ----------------------------------------------------------------------------
# Linear over a split reduction axis (Linear(cat[a, b]) without the cat)
# ----------------------------------------------------------------------------
def linear_blocks(As: Sequence[torch.Tensor], weight: torch.Tensor,
                  bias: Optional[torch.Tensor]) -> torch.Tensor:
    """F.linear(cat(As, -1), weight, bias) with the concatenation folded into
    the MFMA GEMM's reduction axis (lib/Hodge_Cheb_Conv.py:307-308)."""
    if len(As) > _lib.MAX_BLOCKS:
        raise RuntimeError(f"hlhgat: at most {_lib.MAX_BLOCKS} operand blocks")
    _req_dev(weight, "weight")
    return _ext.linear(list(As), weight, bias)


def mlp2(blocks: Sequence[torch.Tensor], seq: torch.nn.Sequential) -> torch.Tensor:
    """NodeEdgeInt WV_* (Linear(2d, dl) -> BN -> ReLU -> Linear(dl, dv) -> BN ->
    ReLU, lib/Hodge_Cheb_Conv.py:276-289) on cat(blocks) as one C++ node."""
    lin0, bn1, _, lin3, bn4, _ = list(seq)
    return _ext.mlp2(list(blocks), lin0.weight, lin0.bias, *_bn_args(bn1)[:5], lin3.weight,
                     lin3.bias, *_bn_args(bn4)[:5], _bn_args(bn1)[5], float(bn1.eps),
                     _bn_args(bn4)[5], float(bn4.eps))


def _mlp2_params(seq: torch.nn.Sequential):
    """The 14 tensors of a reference WV_* MLP (Linear, BN, ReLU, Linear, BN,
    ReLU) in training mode with affine, tracked BN and biased Linears, or
    None when the module differs from that structure."""
    m = list(seq)
    if not (len(m) == 6 and isinstance(m[0], torch.nn.Linear)
            and isinstance(m[1], torch.nn.BatchNorm1d) and isinstance(m[2], torch.nn.ReLU)
            and isinstance(m[3], torch.nn.Linear) and isinstance(m[4], torch.nn.BatchNorm1d)
            and isinstance(m[5], torch.nn.ReLU)):
        return None
    l0, b1, _, l3, b4, _ = m
    for b in (b1, b4):
        if not (b.training and b.affine and b.track_running_stats and b.momentum is not None
                and b.running_mean is not None) or sync_bn_group(b) is not None:
            return None
    if l0.bias is None or l3.bias is None:
        return None
    return ([l0.weight, l0.bias, b1.weight, b1.bias, b1.running_mean, b1.running_var,
             b1.num_batches_tracked, l3.weight, l3.bias, b4.weight, b4.bias, b4.running_mean,
             b4.running_var, b4.num_batches_tracked],
            [float(b1.momentum), float(b1.eps), float(b4.momentum), float(b4.eps)])


def nei_prepack(neints) -> None:
    """Pack the first-Linear weights / biases of every NodeEdgeInt value path
    in `neints` (hodge_cheb_conv.NodeEdgeInt modules) in ONE launch at the
    start of the forward, instead of one pack launch inside each NodeEdgeInt
    on the critical stream; each module consumes its pack once (nei_value)."""
    mods, groups = [], []
    for m in (neints if PREPACK else []):
        pn, pe = _mlp2_params(m.WV_Node), _mlp2_params(m.WV_Edge)
        if pn is None or pe is None or not pn[0][0].is_cuda:
            continue
        mods.append(m)
        groups.append([pn[0][0], pn[0][1], pe[0][0], pe[0][1]])
    global _PACK_EPOCH
    _PACK_EPOCH += 1
    if not mods:
        return
    for m, packed in zip(mods, _ext.nei_prepack(groups)):
        m._hlhgat_packed = (_PACK_EPOCH, packed)


_PACK_EPOCH = 0  # a pack is only used by the forward that built it
# PREPACK = False (tests; HLHGAT_PREPACK=0 for A/B): each NodeEdgeInt packs its
# own weights, each only_att NodeEdgeInt concatenates its K|Q (same results)
PREPACK = os.environ.get("HLHGAT_PREPACK", "1") != "0"


class _AttPackFn(torch.autograd.Function):
    """The only_att NodeEdgeInts' concatenated projections
    (cat[WK_Node; WQ_Node] and cat[WK_Edge; WQ_Edge], weights and biases) of
    a whole forward in ONE batched copy instead of four torch.cat launches
    per module; the backward hands each parameter its rows of the packed
    gradients (views, as torch.cat's backward does)."""

    @staticmethod
    def forward(ctx, n_mod, *params):
        outs, srcs, dsts = [], [], []
        for i in range(n_mod):
            wkn, wqn, bkn, bqn, wke, wqe, bke, bqe = params[8 * i:8 * i + 8]
            for a, b in ((wkn, wqn), (bkn, bqn), (wke, wqe), (bke, bqe)):
                o = torch.empty((a.size(0) + b.size(0),) + tuple(a.shape[1:]), device=a.device,
                                dtype=a.dtype)
                srcs += [a.detach(), b.detach()]
                dsts += [o[:a.size(0)], o[a.size(0):]]
                outs.append(o)
        copy_words_batched(srcs, dsts)
        ctx.n_mod = n_mod
        ctx.rows = [p.size(0) for p in params]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        out = [None]
        for i in range(ctx.n_mod):
            r = ctx.rows[8 * i:8 * i + 8]
            for q, g in enumerate(grads[4 * i:4 * i + 4]):
                k = r[2 * q]  # rows of the pair's first parameter
                if g is None:
                    out += [None, None]
                else:
                    out += [g[:k], g[k:]]
        # params order: wkn, wqn, bkn, bqn, wke, wqe, bke, bqe per module
        return tuple(out)


def att_prepack(neatts) -> None:
    """Pack the K|Q projections of every only_att NodeEdgeInt in `neatts`
    in one launch at the start of the forward (NodeEdgeInt._unfused takes
    its pack once, take_pack's epoch rule)."""
    mods = [m for m in (neatts if PREPACK else [])
            if m.only_att and m.WK_Node.weight.is_cuda and m.WK_Node.bias is not None]
    if not mods:
        return
    params = []
    for m in mods:
        params += [m.WK_Node.weight, m.WQ_Node.weight, m.WK_Node.bias, m.WQ_Node.bias,
                   m.WK_Edge.weight, m.WQ_Edge.weight, m.WK_Edge.bias, m.WQ_Edge.bias]
    global _ATT_EPOCH
    _ATT_EPOCH += 1
    outs = _AttPackFn.apply(len(mods), *params)
    for i, m in enumerate(mods):
        m._hlhgat_att_packed = (outs[4 * i:4 * i + 4], _att_versions(m), _ATT_EPOCH)


_ATT_EPOCH = 0  # the latest att_prepack (a pack is only used until the next one)


def _att_versions(m):
    return tuple(t._version for t in (m.WK_Node.weight, m.WQ_Node.weight, m.WK_Node.bias,
                                      m.WQ_Node.bias, m.WK_Edge.weight, m.WQ_Edge.weight,
                                      m.WK_Edge.bias, m.WQ_Edge.bias))


def take_att_pack(m):
    """The module's (w_t, b_t, w_s, b_s) from the latest att_prepack,
    consumed; None when there is none, a later att_prepack ran, or a
    parameter's version counter moved since (an in-place update)."""
    p, m._hlhgat_att_packed = getattr(m, "_hlhgat_att_packed", None), None
    if p is None or p[2] != _ATT_EPOCH or p[1] != _att_versions(m):
        return None
    if (torch.is_grad_enabled() and m.WK_Node.weight.requires_grad
            and not p[0][0].requires_grad):
        return None  # packed under no_grad, used with gradients
    return p[0]


def take_pack(m) -> Optional[torch.Tensor]:
    """The module's pack from the current forward's nei_prepack, consumed."""
    p, m._hlhgat_packed = getattr(m, "_hlhgat_packed", None), None
    return p[1] if p is not None and p[0] == _PACK_EPOCH else None


def nei_value(x_t: torch.Tensor, x_s: torch.Tensor, inc: "Incidence", rD: torch.Tensor,
              wv_node: torch.nn.Sequential, wv_edge: torch.nn.Sequential,
              valid_t: Optional[torch.Tensor] = None, valid_s: Optional[torch.Tensor] = None,
              gsink=(None, None), packed: Optional[torch.Tensor] = None):
    """NodeEdgeInt value path (lib/Hodge_Cheb_Conv.py:293-295,307-308) as one
    C++ node, first Linear projected before the |B1| gathers (torch_ext.cpp,
    NEIntValueFn); returns (x_t1, x_s1), or None when the WV_* modules are not
    the reference training-mode structure (caller falls back)."""
    pn, pe = _mlp2_params(wv_node), _mlp2_params(wv_edge)
    if pn is None or pe is None:
        return None
    _req_dev(x_t, "x_t")
    _req_dev(x_s, "x_s")
    if x_s.size(0) != inc.n_edges or x_t.size(0) != inc.n_nodes:
        raise RuntimeError(f"hlhgat: x_t/x_s rows ({x_t.size(0)}, {x_s.size(0)}) do not match "
                           f"|B1| ({inc.n_nodes}, {inc.n_edges})")
    if rD.numel() != inc.n_nodes:
        raise RuntimeError(f"hlhgat: D has {rD.numel()} entries, |B1| has {inc.n_nodes} nodes")
    # gsink: the DenseConcat gradient-slab views of x_t / x_s (DenseConcat.grad_sink):
    # their gradients are added straight into the slab by the Linear backward
    (gt, ft), (gs, fs) = [g if g is not None else (None, None) for g in gsink]
    if gt is not None and (gt.shape != x_t.shape or gt.data_ptr() == x_t.data_ptr()):
        gt = ft = None
    if gs is not None and (gs.shape != x_s.shape or gs.data_ptr() == x_s.data_ptr()):
        gs = fs = None
    r = _ext.nei_value(x_t, x_s, inc.rowptr, inc.edge_ids, inc.edge_index,
                       rD.contiguous().view(-1), pn[0], pe[0], *pn[1], *pe[1], valid_t, valid_s,
                       gt, gs, ft, fs, packed)
    return r[0], r[1]


# ----------------------------------------------------------------------------
# boundary operator: x_s2t = (1/D) |B1| x_s ; x_t2s = |B1|^T x_t / 2
# ----------------------------------------------------------------------------
def node_from_edges(x_s: torch.Tensor, inc: Incidence, rD: torch.Tensor) -> torch.Tensor:
    _req_dev(x_s, "x_s")
    _req_dev(rD, "1/D")
    if x_s.size(0) != inc.n_edges:
        raise RuntimeError(f"hlhgat: x_s has {x_s.size(0)} rows, |B1| has {inc.n_edges} edges")
    if rD.numel() != inc.n_nodes:
        raise RuntimeError(f"hlhgat: D has {rD.numel()} entries, |B1| has {inc.n_nodes} nodes")
    return _ext.node_from_edges(x_s, inc.rowptr, inc.edge_ids, inc.edge_index,
                                rD.contiguous().view(-1), inc.n_nodes)


def _incidence_signs(inc: Incidence) -> torch.Tensor:
    """Signed B1 values in incidence-CSR order: for node v's slot of edge e,
    -1 if v = edge_index[0][e] (tail), +1 if v = edge_index[1][e] (head)
    (adj2par1, lib/Hodge_Dataset.py:169-191).  Cached on the Incidence."""
    s = getattr(inc, "_signs", None)
    if s is None:
        dev = inc.rowptr.device
        counts = (inc.rowptr[1:] - inc.rowptr[:-1]).long()
        node = torch.repeat_interleave(torch.arange(inc.n_nodes, device=dev), counts,
                                       output_size=2 * inc.n_edges)
        head = inc.edge_index[1][inc.edge_ids.long()]
        s = torch.where(head == node, 1.0, -1.0).to(torch.float32).contiguous()
        inc._signs = s  # type: ignore[attr-defined]
    return s


class _BoundaryTFn(torch.autograd.Function):
    """y = B1^T x_t (y[e] = x_t[j] - x_t[i]); backward dx = B1 dy."""

    @staticmethod
    def forward(ctx, x_t, inc):
        ctx.inc = inc
        E, d = inc.n_edges, x_t.size(1)
        y = torch.empty(E, d, device=x_t.device, dtype=x_t.dtype)
        if E:
            check(LIB.hlhgat_edge_gather2(inc.edge_index.data_ptr(), E, x_t.data_ptr(), _ld(x_t),
                                          d, None, None, -1.0, 1.0, None, 0, y.data_ptr(),
                                          _ld(y), 0, _stream(x_t)), "edge_gather2(B1^T)")
        return y

    @staticmethod
    def backward(ctx, g):
        inc = ctx.inc
        g = _rows2d(g.contiguous(), "grad")
        A = SparseCSR(inc.rowptr, inc.edge_ids, _incidence_signs(inc), inc.n_nodes,
                      inc.n_edges, 2 * inc.n_edges)
        dx = torch.empty(inc.n_nodes, g.size(1), device=g.device, dtype=g.dtype)
        if inc.n_nodes:
            _poly_step(A, g, dx)
        return dx, None


class _TspReadoutFn(torch.autograd.Function):
    """R = cat([x_s, |B1^T x_t| / 2], -1) where R is a column window of a
    dense slab whose first columns already hold x_s (its last part): only the
    x_t2s half is computed, in one pass; the backward hands x_s its half of
    dR as a view and x_t B1 ((dR2 / 2) * sgn(B1^T x_t))."""

    @staticmethod
    def forward(ctx, x_s, x_t, inc, R):
        cs, E, d = x_s.size(1), inc.n_edges, x_t.size(1)
        ctx.inc, ctx.cs = inc, cs
        ctx.save_for_backward(x_t)
        check(LIB.hlhgat_edge_absdiff(inc.edge_index.data_ptr(), E, x_t.data_ptr(), _ld(x_t), d,
                                      None, 0, R.data_ptr() + 4 * cs, _ld(R), _stream(x_t)),
              "edge_absdiff")
        return R

    @staticmethod
    def backward(ctx, g):
        (x_t,) = ctx.saved_tensors
        inc, cs = ctx.inc, ctx.cs
        g = _rows2d(g, "grad")
        E, d = inc.n_edges, x_t.size(1)
        ge = torch.empty(E, d, device=g.device, dtype=g.dtype)
        check(LIB.hlhgat_edge_absdiff(inc.edge_index.data_ptr(), E, x_t.data_ptr(), _ld(x_t), d,
                                      g.data_ptr() + 4 * cs, _ld(g), ge.data_ptr(), d,
                                      _stream(g)), "edge_absdiff backward")
        A = SparseCSR(inc.rowptr, inc.edge_ids, _incidence_signs(inc), inc.n_nodes,
                      inc.n_edges, 2 * inc.n_edges)
        dx = torch.empty(inc.n_nodes, d, device=g.device, dtype=g.dtype)
        if inc.n_nodes:
            _poly_step(A, ge, dx)
        return g[:, :cs], dx, None, None


def tsp_readout(x_s: torch.Tensor, x_t: torch.Tensor, inc: Incidence,
                R: torch.Tensor) -> torch.Tensor:
    """The TSP head's readout input cat([x_s, |B1^T x_t| / 2], -1)
    (lib/Hodge_ST_Model.py:846-849) into R, a [n_edges, C_s + C_t] window of
    the edge slab whose first C_s columns hold x_s already: bitwise the
    unfused boundary_t / abs / div / cat and their gradients."""
    _req_dev(x_t, "x_t")
    x_t = _rows2d(x_t, "x_t")
    E = inc.n_edges
    if x_t.size(0) != inc.n_nodes or x_s.size(0) != E:
        raise RuntimeError(f"hlhgat: tsp_readout rows ({x_t.size(0)}, {x_s.size(0)}) vs |B1| "
                           f"({inc.n_nodes}, {E})")
    if tuple(R.shape) != (E, x_s.size(1) + x_t.size(1)) or R.stride(1) != 1:
        raise RuntimeError(f"hlhgat: tsp_readout window {tuple(R.shape)} does not fit")
    return _TspReadoutFn.apply(x_s, x_t, inc, R)


def boundary_t(x_t: torch.Tensor, inc: Incidence) -> torch.Tensor:
    """torch.sparse.mm(par_1.transpose(0, 1), x_t) for par_1 = adj2par1(...)
    (lib/Hodge_ST_Model.py:846): per edge (i, j), x_t[j] - x_t[i], summed in
    the coalesced order of the sparse product (tail entry first)."""
    _req_dev(x_t, "x_t")
    x_t = _rows2d(x_t, "x_t")
    if x_t.size(0) != inc.n_nodes:
        raise RuntimeError(f"hlhgat: x_t has {x_t.size(0)} rows, |B1| has {inc.n_nodes} nodes")
    return _BoundaryTFn.apply(x_t, inc)


class _IncidenceMMFn(torch.autograd.Function):
    """One of the four products with B1 of adj2par1 (lib/Hodge_Dataset.py:
    169-191) that torch.sparse.mm forms in the reference: B1 y, |B1| y (node
    rows: incidence CSR, edges ascending = the coalesced order) and B1^T x,
    |B1|^T x (edge rows: tail entry first).  The backward of each is the
    transposed product."""

    @staticmethod
    def forward(ctx, x, inc, transposed, signed):
        ctx.inc, ctx.transposed, ctx.signed = inc, transposed, signed
        return _incidence_mm(x, inc, transposed, signed)

    @staticmethod
    def backward(ctx, g):
        g = _rows2d(g.contiguous(), "grad")
        return _incidence_mm(g, ctx.inc, not ctx.transposed, ctx.signed), None, None, None


def _incidence_mm(x: torch.Tensor, inc: Incidence, transposed: bool, signed: bool):
    d = x.size(1)
    if transposed:  # edge rows: y[e] = c_i x[i] + x[j]
        y = torch.empty(inc.n_edges, d, device=x.device, dtype=x.dtype)
        if inc.n_edges:
            check(LIB.hlhgat_edge_gather2(inc.edge_index.data_ptr(), inc.n_edges, x.data_ptr(),
                                          _ld(x), d, None, None, -1.0 if signed else 1.0, 1.0,
                                          None, 0, y.data_ptr(), _ld(y), 0, _stream(x)),
                  "edge_gather2(B1^T)")
        return y
    A = SparseCSR(inc.rowptr, inc.edge_ids, _incidence_signs(inc) if signed else None,
                  inc.n_nodes, inc.n_edges, 2 * inc.n_edges)
    y = torch.empty(inc.n_nodes, d, device=x.device, dtype=x.dtype)
    if inc.n_nodes:
        _poly_step(A, x, y)
    return y


def incidence_mm(x: torch.Tensor, inc: Incidence, transposed: bool = False,
                 signed: bool = True) -> torch.Tensor:
    """torch.sparse.mm(P, x) for P = adj2par1(...) (signed) or its .abs(), or
    their transposes: bitwise the coalesced sparse product (autograd)."""
    _req_dev(x, "x")
    x = _rows2d(x, "x")
    rows = inc.n_nodes if transposed else inc.n_edges
    if x.size(0) != rows:
        raise RuntimeError(f"hlhgat: B1{'^T' if transposed else ''} product: x has {x.size(0)} "
                           f"rows, expected {rows}")
    return _IncidenceMMFn.apply(x, inc, bool(transposed), bool(signed))


def edge_from_nodes(x_t: torch.Tensor, inc: Incidence) -> torch.Tensor:
    _req_dev(x_t, "x_t")
    if x_t.size(0) != inc.n_nodes:
        raise RuntimeError(f"hlhgat: x_t has {x_t.size(0)} rows, |B1| has {inc.n_nodes} nodes")
    return _ext.edge_from_nodes(x_t, inc.rowptr, inc.edge_ids, inc.edge_index)


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


class _AttScoreKQFn(torch.autograd.Function):
    """_AttScoreFn with K = kq[:, :dk] and Qs = kq[:, dk:2dk] (one GEMM's
    output): the backward returns kq's gradient as ONE [n, 2dk] block, no
    per-slice zero fill + copy + add."""

    @staticmethod
    def forward(ctx, Qc, kq, w_cross, w_self, sqrt_dk, sigma):
        n, dk = kq.size(0), Qc.size(1)
        a = torch.empty(n, 1, device=kq.device, dtype=kq.dtype)
        check(LIB.hlhgat_att_score_fwd(n, dk, Qc.data_ptr(), _ld(Qc), kq.data_ptr() + 4 * dk,
                                       _ld(kq), kq.data_ptr(), _ld(kq), w_cross, w_self, sqrt_dk,
                                       sigma, a.data_ptr(), _stream(kq)), "att_score_fwd")
        ctx.consts = (w_cross, w_self, sqrt_dk, sigma)
        ctx.save_for_backward(Qc, kq, a)
        return a

    @staticmethod
    def backward(ctx, ga):
        Qc, kq, a = ctx.saved_tensors
        w_cross, w_self, sqrt_dk, sigma = ctx.consts
        n, dk = kq.size(0), Qc.size(1)
        ga = ga.contiguous()
        # columns [0, dk) dK, [dk, 2dk) dQs (= d kq), [2dk, 3dk) dQc
        g = torch.empty(n, 3 * dk, device=kq.device, dtype=kq.dtype)
        p = g.data_ptr()
        check(LIB.hlhgat_att_score_bwd(n, dk, Qc.data_ptr(), _ld(Qc), kq.data_ptr() + 4 * dk,
                                       _ld(kq), kq.data_ptr(), _ld(kq), w_cross, w_self, sqrt_dk,
                                       sigma, a.data_ptr(), ga.data_ptr(), p + 8 * dk,
                                       p + 4 * dk, p, 3 * dk, _stream(kq)), "att_score_bwd")
        return g[:, 2 * dk:], g[:, :2 * dk], None, None, None, None


def att_score_kq(Qc, kq, w_cross: float, w_self: float, sqrt_dk: float,
                 sigma: int) -> torch.Tensor:
    """att_score(Qc, kq[:, dk:], kq[:, :dk], ...) with dk = Qc.size(1): the
    key and the self query as the two column halves of one [n, 2dk] GEMM
    output (lib/Hodge_Cheb_Conv.py:299-304)."""
    _req_dev(Qc, "Qc")
    _req_dev(kq, "kq")
    Qc, kq = _rows2d(Qc, "Qc"), _rows2d(kq, "kq")
    if kq.size(1) != 2 * Qc.size(1) or kq.size(0) != Qc.size(0):
        raise RuntimeError(f"hlhgat: att_score_kq: kq {tuple(kq.shape)} vs Qc {tuple(Qc.shape)}")
    return _AttScoreKQFn.apply(Qc, kq, float(w_cross), float(w_self), float(sqrt_dk), int(sigma))


class _RowScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a, out, gsink):
        n, d = x.size(0), x.size(1)
        y = out if out is not None else torch.empty(n, d, device=x.device, dtype=x.dtype)
        check(LIB.hlhgat_row_scale_fwd(n, d, x.data_ptr(), _ld(x), a.data_ptr(), y.data_ptr(),
                                       _ld(y), _stream(x)), "row_scale_fwd")
        ctx.gsink = gsink
        ctx.save_for_backward(x, a)
        return y

    @staticmethod
    def backward(ctx, g):
        x, a = ctx.saved_tensors
        n, d = x.size(0), x.size(1)
        g = _rows2d(g, "grad")
        sink, flag = ctx.gsink if ctx.gsink is not None else (None, None)
        if sink is not None and int(flag[0]) == 0:
            gx = sink  # the first gradient into x's slab: written in place
            flag[0] = 1
        else:
            gx = torch.empty(n, d, device=x.device, dtype=x.dtype)
        ga = torch.empty(n, 1, device=x.device, dtype=x.dtype)
        check(LIB.hlhgat_row_scale_bwd(n, d, x.data_ptr(), _ld(x), a.data_ptr(), g.data_ptr(),
                                       _ld(g), gx.data_ptr(), _ld(gx), ga.data_ptr(),
                                       _stream(x)), "row_scale_bwd")
        return gx, ga, None, None


def row_scale(x: torch.Tensor, a: torch.Tensor, out: Optional[torch.Tensor] = None,
              gsink=None) -> torch.Tensor:
    """x * a for a per-row score a [n, 1] (the NEAtt product, main_pepfunc...:
    134-136): bitwise ATen's product; the backward's da = rowsum(dy * x) is
    one fused pass (fp32, its own summation order).  out: a DenseConcat sink
    for y; gsink: DenseConcat.grad_sink() of x = view(), written in place
    when x's gradient lands there first -- x must then have no other
    consumer (take a fresh view())."""
    _req_dev(x, "x")
    _req_dev(a, "a")
    x = _rows2d(x, "x")
    if a.numel() != x.size(0):
        raise RuntimeError(f"hlhgat: row_scale: a has {a.numel()} entries for {x.size(0)} rows")
    a = a.contiguous()
    if out is not None and (tuple(out.shape) != tuple(x.shape) or out.stride(1) != 1):
        raise RuntimeError(f"hlhgat: row_scale out {tuple(out.shape)} vs x {tuple(x.shape)}")
    if gsink is not None and (gsink[0] is None or gsink[0].shape != x.shape):
        gsink = None
    return _RowScaleFn.apply(x, a, out, gsink)


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
    def forward(ctx, x, seg_ptr, seg_rows, n_seg, out, covering, gsink):
        d = x.size(1)
        if out is None:
            out = torch.empty(n_seg, d, device=x.device, dtype=x.dtype)
        check(LIB.hlhgat_segment_mean_fwd(seg_ptr.data_ptr(), _ptr(seg_rows), n_seg,
                                          x.data_ptr(), _ld(x), d, out.data_ptr(), _ld(out),
                                          _stream(x)), "segment_mean_fwd")
        ctx.meta = (x.size(0), n_seg, seg_rows is not None, covering)
        ctx.gsink = gsink
        ctx.save_for_backward(seg_ptr, seg_rows if seg_rows is not None else seg_ptr)
        return out

    @staticmethod
    def backward(ctx, g):
        seg_ptr, seg_rows = ctx.saved_tensors
        n_rows, n_seg, listed, covering = ctx.meta
        g = _rows2d(g, "grad")
        if covering:
            # every row is listed (the trailing bucket: rows in no cluster,
            # written as zeros): no zero fill; into the slab's gradient when
            # this is the first gradient to land there (DenseConcat.grad_sink)
            sink, flag = ctx.gsink if ctx.gsink is not None else (None, None)
            if sink is not None and int(flag[0]) == 0 and sink.shape == (n_rows, g.size(1)):
                gx = sink
                flag[0] = 1
            else:
                gx = torch.empty(n_rows, g.size(1), device=g.device, dtype=g.dtype)
            check(LIB.hlhgat_pool_mean_bwd(seg_ptr.data_ptr(), seg_rows.data_ptr(), n_seg,
                                           g.data_ptr(), _ld(g), g.size(1), gx.data_ptr(),
                                           _ld(gx), n_rows, _stream(g)), "pool_mean_bwd")
            return gx, None, None, None, None, None, None
        gx = (torch.zeros if listed else torch.empty)(n_rows, g.size(1), device=g.device,
                                                      dtype=g.dtype)
        check(LIB.hlhgat_segment_mean_bwd(seg_ptr.data_ptr(), _ptr(seg_rows) if listed else None,
                                          n_seg, g.data_ptr(), _ld(g), g.size(1), gx.data_ptr(),
                                          _ld(gx), n_rows, _stream(g)), "segment_mean_bwd")
        return gx, None, None, None, None, None, None


class _SegmentMeanCatFn(torch.autograd.Function):
    """cat([segment_mean(x_i, ptr_i) for i], -1) with each mean written
    straight into its column block (no cat launch); contiguous segments."""

    @staticmethod
    def forward(ctx, n_seg, ptrs, side, *xs):
        # side: the edge chain's stream (ops.Chains) for part 0, whose input
        # was produced there and whose gradient is consumed there
        widths = [x.size(1) for x in xs]
        out = torch.empty(n_seg, sum(widths), device=xs[0].device, dtype=xs[0].dtype)
        if side is not None:
            # `out` comes from the main stream's pool: a block main freed may
            # still be read by main's queued kernels, so the side stream's write
            # waits for main
            side.wait_stream(torch.cuda.current_stream(xs[0].device))
            out.record_stream(side)
        c0 = 0
        for i, (x, p, w) in enumerate(zip(xs, ptrs, widths)):
            st = side.cuda_stream if (side is not None and i == 0) else _stream(x)
            check(LIB.hlhgat_segment_mean_fwd(p.data_ptr(), None, n_seg, x.data_ptr(), _ld(x), w,
                                              out.data_ptr() + 4 * c0, _ld(out), st),
                  "segment_mean_fwd")
            c0 += w
        ctx.meta = (n_seg, widths, [x.size(0) for x in xs])
        ctx.side = side
        ctx.save_for_backward(*ptrs)
        return out

    @staticmethod
    def backward(ctx, g):
        n_seg, widths, rows = ctx.meta
        g = _rows2d(g, "grad").contiguous()
        side = ctx.side
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(g.device))
            g.record_stream(side)
        gx, c0 = [], 0
        for i, (p, w, n) in enumerate(zip(ctx.saved_tensors, widths, rows)):
            on_side = side is not None and i == 0
            with (torch.cuda.stream(side) if on_side else contextlib.nullcontext()):
                t = torch.empty(n, w, device=g.device, dtype=g.dtype)
                check(LIB.hlhgat_segment_mean_bwd(p.data_ptr(), None, n_seg,
                                                  g.data_ptr() + 4 * c0, _ld(g), w, t.data_ptr(),
                                                  _ld(t), n, _stream(t)),
                      "segment_mean_bwd")
            if on_side:
                t.record_stream(torch.cuda.current_stream(g.device))
            gx.append(t)
            c0 += w
        return (None, None, None, *gx)


def segment_mean_cat(xs: Sequence[torch.Tensor], seg_ptrs: Sequence[torch.Tensor],
                     n_seg: int, side=None) -> torch.Tensor:
    """torch.cat([segment_mean(x, p, n_seg) for x, p in zip(xs, seg_ptrs)], -1)
    (the readout x = cat(mean_pool(x_s), mean_pool(x_t)),
    lib/Hodge_ST_Model.py:636) without the cat: bitwise the same values."""
    xs = [_rows2d(x, "x") for x in xs]
    for x in xs:
        _req_dev(x, "x")
    for p in seg_ptrs:
        _req_dev(p, "seg_ptr", torch.int32)
        if p.numel() != n_seg + 1:
            raise RuntimeError(f"hlhgat: segment_mean_cat: seg_ptr has {p.numel()} entries, "
                               f"expected {n_seg + 1}")
    return _SegmentMeanCatFn.apply(int(n_seg), list(seg_ptrs), side, *xs)


def segment_mean(x: torch.Tensor, seg_ptr: torch.Tensor, n_seg: int,
                 seg_rows: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                 covering: bool = False, gsink=None) -> torch.Tensor:
    """Mean of x rows per segment.  seg_ptr int32 [n_seg+1]; members are the
    contiguous rows seg_ptr[s]..seg_ptr[s+1] (global_mean_pool over a sorted
    batch vector) or seg_rows[seg_ptr[s]:seg_ptr[s+1]] (scatter_mean).
    covering: seg_ptr has n_seg+2 entries and the extra segment lists the
    rows in no segment, so seg_rows is a permutation of x's rows (the pool
    tables of hodge_dataset.pool_tables); the backward then writes every row
    (zeros for that bucket) without a zero fill, into ``gsink`` (a
    DenseConcat.grad_sink of x) when it is the first gradient there.  out: a
    [n_seg, d] destination (a DenseConcat sink) instead of a new tensor."""
    _req_dev(x, "x")
    _req_dev(seg_ptr, "seg_ptr", torch.int32)
    if seg_rows is not None:
        _req_dev(seg_rows, "seg_rows", torch.int32)
    x = _rows2d(x, "x")
    if covering and (seg_rows is None or seg_ptr.numel() != n_seg + 2
                     or seg_rows.numel() != x.size(0)):
        raise RuntimeError("hlhgat: segment_mean(covering=True) needs seg_ptr [n_seg+2] and "
                           "seg_rows listing every row of x")
    if out is not None and (tuple(out.shape) != (n_seg, x.size(1)) or out.stride(1) != 1
                            or out.device != x.device or out.dtype != x.dtype):
        raise RuntimeError(f"hlhgat: segment_mean out {tuple(out.shape)} does not match "
                           f"({n_seg}, {x.size(1)})")
    if gsink is not None and (gsink[0] is None or gsink[0].shape != x.shape):
        gsink = None
    return _SegmentMeanFn.apply(x, seg_ptr, seg_rows, int(n_seg), out, bool(covering), gsink)


# ----------------------------------------------------------------------------
# BatchNorm1d (training statistics) + optional fused ReLU
# ----------------------------------------------------------------------------
def batch_norm_act(x: torch.Tensor, bn: torch.nn.BatchNorm1d, relu: bool = False,
                   valid: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bn(x) followed by ReLU when ``relu``; training mode (or no running
    stats) uses the HIP batch-statistics kernels; eval mode the running
    statistics: inference (nothing to differentiate) in one HIP launch
    (hlhgat_bn_apply_running, the ReLU fused), an eval-mode BatchNorm inside
    a differentiated graph through ATen's eval kernel (its autograd)."""
    _req_dev(x, "x")
    if x.dim() != 2:
        raise RuntimeError("hlhgat: batch_norm_act expects [N, C] input")
    use_batch = bn.training or not bn.track_running_stats
    if not use_batch:
        grads = torch.is_grad_enabled() and (
            x.requires_grad or any(t is not None and t.requires_grad
                                   for t in (bn.weight, bn.bias)))
        if not grads and x.size(0) > 0:
            x = _rows2d(x, "x")
            y = torch.empty(x.shape, device=x.device, dtype=x.dtype)
            check(LIB.hlhgat_bn_apply_running(
                x.data_ptr(), _ld(x), x.size(0), x.size(1), _ptr(bn.weight), _ptr(bn.bias),
                bn.running_mean.data_ptr(), bn.running_var.data_ptr(), float(bn.eps),
                1 if relu else 0, y.data_ptr(), _ld(y), _stream(x)), "bn_apply_running")
            return y
        y = torch.nn.functional.batch_norm(x, bn.running_mean, bn.running_var, bn.weight,
                                           bn.bias, False, 0.0, bn.eps)
        return torch.relu(y) if relu else y
    if x.size(0) < 2 and bn.training:
        raise ValueError(f"Expected more than 1 value per channel when training, got input "
                         f"size {tuple(x.shape)}")
    if sync_bn_group(bn) is not None:
        return _SyncBatchNormFn.apply(x, bn.weight, bn.bias, bool(relu), valid,
                                      sync_bn_group(bn), _bn_args(bn))
    return _ext.bn_act(x, *_bn_args(bn), bool(relu), valid)


# ----------------------------------------------------------------------------
# SyncBatchNorm (hlhgat.distributed.convert_sync_batchnorm): batch statistics
# over every rank's rows -- the single-process statistics of the whole
# data-parallel batch (parity caveat 1).
# ----------------------------------------------------------------------------
class _SyncGroup:
    """Marker held by a BatchNorm1d in SyncBatchNorm mode: its process group
    (None = the default group)."""

    def __init__(self, group=None):
        self.group = group


def sync_bn_group(bn) -> Optional[_SyncGroup]:
    """The _SyncGroup of a BatchNorm1d in SyncBatchNorm mode (training-mode
    batch statistics only), else None."""
    g = getattr(bn, "_hlhgat_sync", None)
    if g is None or not _bn_uses_batch_stats(bn):
        return None
    return g


def has_sync_bn(module: torch.nn.Module) -> bool:
    """True when a BatchNorm1d of ``module`` normalises in SyncBatchNorm mode
    now (hlhgat.distributed.convert_sync_batchnorm, training mode)."""
    return any(isinstance(m, torch.nn.BatchNorm1d) and sync_bn_group(m) is not None
               for m in module.modules())


_SYNC_WS = {}
_SYNC_WS_RETIRED = []
# SYNCBN_CHAINS (probe only): run SyncBatchNorm models with the persistent
# node / edge chains (ops.Chains) instead of a fork / join per block -- their
# capture under RCCL segfaults in hipStreamEndCapture (round 5; issuing the
# statistics all-reduces from one dedicated stream does not change that,
# round 6: tools/probes/syncbn_capture_probe.py, profiles/r06/)
SYNCBN_CHAINS = os.environ.get("HLHGAT_SYNCBN_CHAINS", "0") == "1"


def _sync_workspace(x: torch.Tensor, n: int, Cc: int) -> torch.Tensor:
    """Zeroed BatchNorm workspace per (device, stream); outgrown ones are
    retired, not freed (a captured graph may still hold the address)."""
    key = (x.device.index, _stream(x))
    need = int(LIB.hlhgat_bn_workspace_bytes(n, Cc))
    ws = _SYNC_WS.get(key)
    if ws is None or ws.numel() < need:
        if ws is not None:
            _SYNC_WS_RETIRED.append(ws)
        ws = torch.zeros(max(need, 1 << 20, 2 * (ws.numel() if ws is not None else 0)),
                         dtype=torch.uint8, device=x.device)
        _SYNC_WS[key] = ws
    return ws


def _sum_over_ranks(t: torch.Tensor, group) -> torch.Tensor:
    """[1, len(t)]: the fp64 sums of every rank, added by an all-reduce (SUM)
    -- RCCL under nccl, which a hipGraph capture records like the attention
    max's all-reduce (an all_gather_into_tensor of the same vector did not
    capture: hipStreamEndCapture segfaulted, ProcessGroupNCCL's watchdog then
    queried an event of the capturing stream; round 4).  Every rank receives
    the same bits; one rank (or no process group) returns t itself, so the
    statistics are bitwise the single-process BatchNorm's."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return t.view(1, -1)
    from .distributed import collectives_on
    if not collectives_on(group):
        return t.view(1, -1)
    out = t.clone()
    # on the current stream (a SyncBatchNorm model's block section runs with
    # per-block fork / join, not ops.Chains: see _PyrHead.forward)
    dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
    return out.view(1, -1)


class _SyncBatchNormFn(torch.autograd.Function):
    """BatchNorm1d (+ ReLU) with statistics over all ranks: local fp64 sums
    (hlhgat_bn_sums_fwd) -> all-reduce (SUM) -> apply with the totals
    (hlhgat_bn_sync_fwd_apply, one gathered row).  Backward as torch.nn.SyncBatchNorm: global
    sum g / sum g (x - mean) for dx, local dweight / dbias (DDP averages
    them)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu, valid, sg, bn_args):
        _, _, rm, rv, nbt, momentum, eps = bn_args
        x = _rows2d(x, "x")
        n, Cc = x.shape
        y = torch.empty(n, Cc, device=x.device, dtype=x.dtype)
        ws = _sync_workspace(x, n, Cc)
        L = int(LIB.hlhgat_bn_sums_len(Cc))
        sums = torch.empty(L, dtype=torch.float64, device=x.device)
        check(LIB.hlhgat_bn_sums_fwd(x.data_ptr(), _ld(x), y.data_ptr(), _ld(y), n, _ptr(valid),
                                     Cc, sums.data_ptr(), ws.data_ptr(), ws.numel(), _stream(x)),
              "bn_sums_fwd")
        gathered = _sum_over_ranks(sums, sg.group).contiguous()
        mean = torch.empty(Cc, device=x.device, dtype=x.dtype)
        invstd = torch.empty(Cc, device=x.device, dtype=x.dtype)
        check(LIB.hlhgat_bn_sync_fwd_apply(
            x.data_ptr(), _ld(x), n, _ptr(valid), Cc, gathered.data_ptr(), gathered.size(0),
            _ptr(weight), _ptr(bias), _ptr(rm), _ptr(rv), _ptr(nbt), float(momentum), float(eps),
            int(relu), y.data_ptr(), _ld(y), mean.data_ptr(), invstd.data_ptr(), _stream(x)),
            "bn_sync_fwd_apply")
        ctx.save_for_backward(x, y if relu else None, weight, mean, invstd, valid)
        ctx.sg = sg
        ctx.has_b = bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, weight, mean, invstd, valid = ctx.saved_tensors
        gy = _rows2d(gy, "dy")
        n, Cc = x.shape
        dx = torch.empty_like(x)
        need_w = weight is not None and ctx.needs_input_grad[1]
        need_b = ctx.has_b and ctx.needs_input_grad[2]
        dw = torch.empty(Cc, device=x.device, dtype=x.dtype) if need_w else None
        db = torch.empty(Cc, device=x.device, dtype=x.dtype) if need_b else None
        ws = _sync_workspace(x, n, Cc)
        sums = torch.empty(int(LIB.hlhgat_bn_sums_len(Cc)), dtype=torch.float64, device=x.device)
        check(LIB.hlhgat_bn_sums_bwd(
            x.data_ptr(), _ld(x), _ptr(y), _ld(y) if y is not None else 0, gy.data_ptr(), _ld(gy),
            dx.data_ptr(), _ld(dx), n, _ptr(valid), Cc, mean.data_ptr(), invstd.data_ptr(),
            sums.data_ptr(), _ptr(dw), _ptr(db), ws.data_ptr(), ws.numel(), _stream(x)),
            "bn_sums_bwd")
        gathered = _sum_over_ranks(sums, ctx.sg.group).contiguous()
        check(LIB.hlhgat_bn_sync_bwd_apply(
            x.data_ptr(), _ld(x), _ptr(y), _ld(y) if y is not None else 0, gy.data_ptr(), _ld(gy),
            n, _ptr(valid), Cc, _ptr(weight), mean.data_ptr(), invstd.data_ptr(),
            gathered.data_ptr(), gathered.size(0), dx.data_ptr(), _ld(dx), _stream(x)),
            "bn_sync_bwd_apply")
        return dx, dw, db, None, None, None, None


# ----------------------------------------------------------------------------
# Adam on a flat parameter buffer (hlhgat_adam_flat; hlhgat.train.TrainStep)
# ----------------------------------------------------------------------------
def adam_prepare(grad: torch.Tensor, step: torch.Tensor) -> None:
    """Zero the flat gradient buffer and increment the device step count in
    one launch (hlhgat_adam_prepare); adam_flat(..., prepared=True) then
    uses that count."""
    _req_dev(grad, "grad")
    _req_dev(step, "step")
    if not grad.is_contiguous():
        raise RuntimeError("hlhgat: adam_prepare: grad must be contiguous")
    check(LIB.hlhgat_adam_prepare(grad.data_ptr(), grad.numel(), step.data_ptr(), _stream(grad)),
          "adam_prepare")


def adam_flat(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor,
              exp_avg_sq: torch.Tensor, step: torch.Tensor, lr: float, betas, eps: float,
              weight_decay: float, prepared: bool = False) -> None:
    """One torch.optim.Adam (fused, capturable) update of a flat fp32 buffer;
    `step` the fp32 step count on device (incremented; prepared=True: already
    incremented by adam_prepare)."""
    for t, name in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"),
                    (exp_avg_sq, "exp_avg_sq"), (step, "step")):
        _req_dev(t, name)
        if not t.is_contiguous():
            raise RuntimeError(f"hlhgat: adam_flat: {name} must be contiguous")
    n = param.numel()
    if not (grad.numel() == exp_avg.numel() == exp_avg_sq.numel() == n):
        raise RuntimeError("hlhgat: adam_flat: buffer sizes differ")
    fn = LIB.hlhgat_adam_flat_prepared if prepared else LIB.hlhgat_adam_flat
    check(fn(param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), n,
             step.data_ptr(), float(lr), float(betas[0]), float(betas[1]), float(eps),
             float(weight_decay), _stream(param)), "adam_flat")


class _L1LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        check(LIB.hlhgat_l1_loss_fwd(x.data_ptr(), y.data_ptr(), x.numel(), loss.data_ptr(),
                                     _stream(x)), "l1_loss_fwd")
        ctx.save_for_backward(x, y)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        g = g.contiguous()
        dx = torch.empty_like(x)
        check(LIB.hlhgat_l1_loss_bwd(x.data_ptr(), y.data_ptr(), x.numel(), g.data_ptr(),
                                     dx.data_ptr(), _stream(x)), "l1_loss_bwd")
        return dx, None


def l1_loss(input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """torch.nn.functional.l1_loss(input, target) (mean) in one launch each way
    (hlhgat_l1_loss_fwd / _bwd): the same input gradient bit for bit; the
    loss value is the fp32 mean summed in a fixed order.  No gradient flows
    into target (the regression labels)."""
    _req_dev(input, "input")
    if input.shape != target.shape:
        raise RuntimeError(f"hlhgat: l1_loss shapes differ: {tuple(input.shape)} vs "
                           f"{tuple(target.shape)}")
    if target.requires_grad:
        raise RuntimeError("hlhgat: l1_loss: target must not require grad")
    if input.numel() == 0:
        raise RuntimeError("hlhgat: l1_loss of an empty tensor")
    x = input.contiguous()
    return _L1LossFn.apply(x, target.to(torch.float32).contiguous())


class _BCELogitsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, div):
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        check(LIB.hlhgat_bce_logits_fwd(x.data_ptr(), y.data_ptr(), x.numel(), div,
                                        loss.data_ptr(), _stream(x)), "bce_logits_fwd")
        ctx.div = div
        ctx.save_for_backward(x, y)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        g = g.contiguous()
        dx = torch.empty_like(x)
        check(LIB.hlhgat_bce_logits_bwd(x.data_ptr(), y.data_ptr(), x.numel(), ctx.div,
                                        g.data_ptr(), dx.data_ptr(), _stream(x)),
              "bce_logits_bwd")
        return dx, None, None


def bce_with_logits(input: torch.Tensor, target: torch.Tensor,
                    reduction: str = "mean") -> torch.Tensor:
    """F.binary_cross_entropy_with_logits(input, target, reduction=...) for
    "mean" / "sum" without weights, one launch each way
    (hlhgat_bce_logits_fwd / _bwd); the loss value is the fp32 sum in a fixed
    order.  No gradient flows into target (the labels)."""
    _req_dev(input, "input")
    if input.shape != target.shape:
        raise RuntimeError(f"hlhgat: bce_with_logits shapes differ: {tuple(input.shape)} vs "
                           f"{tuple(target.shape)}")
    if target.requires_grad:
        raise RuntimeError("hlhgat: bce_with_logits: target must not require grad")
    if input.numel() == 0:
        raise RuntimeError("hlhgat: bce_with_logits of an empty tensor")
    if reduction not in ("mean", "sum"):
        raise ValueError(f"hlhgat: bce_with_logits reduction {reduction!r}")
    div = float(input.numel()) if reduction == "mean" else 1.0
    return _BCELogitsFn.apply(input.contiguous(), target.to(torch.float32).contiguous(), div)


# ----------------------------------------------------------------------------
# device error word (include/hlhgat.h: hlhgat_device_errors)
# ----------------------------------------------------------------------------
_DEVERR_TEXT = {
    _lib.DEVERR_HODGE_SIZE: "hodge_build: a Laplacian row would end past the buffers sized "
                            "from the caller's sizes= (duplicate edges or self-loops?); the "
                            "row was not written",
    _lib.DEVERR_BN_STATE: "BatchNorm: an arrival counter was found beyond its total (the "
                          "workspace was written by something else or shared by concurrent "
                          "launches); that launch's statistics are not trusted",
}


def device_errors() -> int:
    """The device error word as kernels that have COMPLETED so far left it
    (no synchronisation)."""
    w = C.c_uint32(0)
    check(LIB.hlhgat_device_errors(C.byref(w)), "device_errors")
    return int(w.value)


def clear_device_errors() -> None:
    check(LIB.hlhgat_clear_device_errors(), "clear_device_errors")


def check_device_errors(sync: bool = True) -> None:
    """Raise RuntimeError if a kernel reported results that must not be used
    (sync=True first waits for all queued work on every stream)."""
    if sync and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    w = device_errors()
    if w:
        what = _DEVERR_TEXT.get(w, f"device error code {w}")
        raise RuntimeError(f"hlhgat: {what}; results since the last clear_device_errors() are "
                           f"invalid")


def bn_giveups() -> dict:
    """Give-ups of the one-launch BatchNorm barrier since the last
    bn_giveups_reset(): a workgroup whose wait for its tile's statistics ran
    out (hlhgat_set_bn_wait_us) and handed its rows to the finalising
    workgroup.  Correct results either way; this is where the time went.
    Synchronises the device."""
    n = C.c_uint32(0)
    check(LIB.hlhgat_bn_wait_timeouts(C.byref(n)), "bn_wait_timeouts")
    recs = (_lib.BnGiveup * _lib.BN_LOG_MAX)()
    logged = C.c_int32(0)
    check(LIB.hlhgat_bn_giveup_log(recs, _lib.BN_LOG_MAX, C.byref(logged)), "bn_giveup_log")
    k = min(int(logged.value), _lib.BN_LOG_MAX)
    log = [{f: int(getattr(recs[i], f)) for f, _ in _lib.BnGiveup._fields_} for i in range(k)]
    return {"count": int(n.value), "log": log}


def bn_giveups_reset() -> None:
    check(LIB.hlhgat_bn_giveup_reset(), "bn_giveup_reset")


# ----------------------------------------------------------------------------
# captured-graph introspection (include/hlhgat.h: hlhgat_graph_kernel_count)
# ----------------------------------------------------------------------------
def graph_kernel_count(graph_handle: int, name_part: str) -> Tuple[int, int]:
    """(kernel nodes, kernel nodes whose name contains name_part) of a
    captured hipGraph (e.g. torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph())."""
    k, m = C.c_int64(), C.c_int64()
    check(LIB.hlhgat_graph_kernel_count(C.c_void_p(int(graph_handle)), name_part.encode(),
                                        C.byref(k), C.byref(m)), "graph_kernel_count")
    return int(k.value), int(m.value)


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
