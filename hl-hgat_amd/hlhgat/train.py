"""Training-step runtime: flat parameters, one-bucket gradient all-reduce and
whole-step hipGraph replay.

The reference trains with a plain eager loop (main_zinc_*.py: forward, L1
loss, backward, Adam step per DataLoader batch, 'cuda:0').  At ZINC scale
one such step is ~600 short kernels, so on MI355X the step is bound by launch
issue and inter-kernel gaps, not by the kernels' bytes.  TrainStep keeps the
reference's semantics (same model, loss, Adam with L2 weight decay) and
executes the step MI355X-first:

  * parameters and gradients live in two flat fp32 buffers (the model's
    Parameters become views), so Adam is ONE fused multi-tensor launch over
    one tensor and the data-parallel gradient exchange is ONE all-reduce of
    one contiguous bucket over RCCL/xGMI (2.6 MB for cfg2);
  * forward + loss + backward (+ Adam on one GPU) are captured into a
    hipGraph per distinct batch shape and replayed; the node / edge chains
    of every HL block are two graph branches (ops.fork);
  * a batch is copied into the graph's static device buffers (D2D, inside the
    step), so any batch of a captured shape reuses its graph.

The first step of a new shape runs eagerly (that step IS the training step)
and the capture happens right after it; capture records work without
executing it, so no batch is trained twice.
"""
from __future__ import annotations

import contextlib
import gc
import os
import threading
import time
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

from . import ops
from .distributed import collectives_on

__all__ = ["Staged", "TrainStep", "InferStep", "batch_key", "forward_collectives"]

# HIP_ADAM = False: torch's fused Adam instead of hlhgat_adam_flat
HIP_ADAM = True
# DEFER_REDUCE = False (tests): every Linear backward launches its own split
# reduction instead of handing it to the next one on its stream (same bits)
DEFER_REDUCE = True
# Gradient exchange for world > 1 (DDP's job in the reference-side drop-in,
# SURVEY §8e; the reference itself is single-GPU): the flat gradient buffer is
# cut into buckets of about BUCKET_MB, last parameters first (the order the
# backward finishes them), and each bucket's all-reduce is issued from a
# post-accumulate-grad hook as soon as its last gradient has landed, so it
# runs beside the rest of the backward.  OVERLAP: "auto" (default) = only when
# that makes at least two buckets (configs 3-5: 10-16 MB of gradients; config
# 2's 2.6 MB stays one all-reduce after the backward), "1" = always (tests),
# "0" = never.
BUCKET_MB = float(os.environ.get("HLHGAT_BUCKET_MB", "4"))
OVERLAP = os.environ.get("HLHGAT_OVERLAP", "auto")
# KEEP_GRAPHS = True (tests, introspection): captures keep their hipGraph_t
# (torch.cuda.CUDAGraph(keep_graph=True), then instantiate), so
# ops.graph_kernel_count can inspect a captured step
KEEP_GRAPHS = False


def forward_collectives(model: torch.nn.Module) -> bool:
    """True when the model's training forward exchanges data between ranks:
    SyncBatchNorm layers (hlhgat.distributed.convert_sync_batchnorm) or a
    head that declares ``forward_collectives`` (the CIFAR attpool head's
    batch-global max, hodge_st_model._AttPoolHead)."""
    if getattr(model, "forward_collectives", False):
        return True
    return any(ops.sync_bn_group(m) is not None for m in model.modules()
               if isinstance(m, torch.nn.modules.batchnorm._BatchNorm))


def _tensor_items(batch):
    return [(k, v) for k, v in sorted(vars(batch).items())
            if torch.is_tensor(v) and not k.startswith("_")]


def _parts(batch):
    """The batch objects of one step: a Batch, or the list of per-level
    batches the attention-pooling heads take (`datas`)."""
    return list(batch) if isinstance(batch, (list, tuple)) else [batch]


def _clone_batch(batch):
    static = type(batch).__new__(type(batch))
    arena = getattr(batch, "_arena", None)
    if arena is not None and arena.is_cuda and _in_arena(batch, arena):
        # keep the one-arena layout (TrainStep.stage then refills it in one copy)
        da = arena.clone()
        for k, v in vars(batch).items():
            if k == "_arena":
                continue
            if torch.is_tensor(v):
                o = v.data_ptr() - arena.data_ptr()
                nb = v.numel() * v.element_size()
                setattr(static, k, da[o:o + nb].view(v.dtype).view(v.shape))
            else:
                setattr(static, k, v)
        static._arena = da
        if hasattr(static, "_mark"):
            static._mark()
        return static
    for k, v in vars(batch).items():
        if k == "_arena":
            continue
        setattr(static, k, v.clone() if torch.is_tensor(v) else v)
    if hasattr(static, "_mark"):
        static._mark()  # sorted/symmetric Laplacian flags on the static tensors
    return static


def batch_key(batch) -> Tuple:
    """Shape signature of a batch: every tensor attribute's (name, shape,
    dtype) plus the scalar attributes that change the launch sequence; for a
    list of level batches, the tuple of their signatures."""
    if isinstance(batch, (list, tuple)):
        return ("levels",) + tuple(batch_key(b) for b in batch)
    key = [(k, tuple(v.shape), str(v.dtype)) for k, v in _tensor_items(batch)]
    key.append(("num_graphs", getattr(batch, "num_graphs", None)))
    hs = getattr(batch, "hodge_sorted", None)
    if hs:
        key.append(("hodge_sorted", tuple(sorted(hs.items()))))
    return tuple(key)


BN_RESERVE_CHANNELS = 2048  # BatchNorm workspace reserved per capture stream


def _in_arena(b, arena) -> bool:
    """Every tensor attribute of b is a contiguous view inside arena."""
    lo, hi = arena.data_ptr(), arena.data_ptr() + arena.numel()
    for _, v in _tensor_items(b):
        p = v.data_ptr()
        if not v.is_contiguous() or p < lo or p + v.numel() * v.element_size() > hi:
            return False
    return True


def _same_layout(b, ha, sb, da) -> bool:
    """b's tensors sit in host arena ha at the offsets sb's sit in device
    arena da (same shapes: then one arena copy updates every static tensor)."""
    if ha.numel() != da.numel():
        return False
    for k, v in _tensor_items(b):
        w = getattr(sb, k, None)
        if (w is None or w.shape != v.shape or w.dtype != v.dtype
                or w.data_ptr() - da.data_ptr() != v.data_ptr() - ha.data_ptr()):
            return False
    return True


@contextlib.contextmanager
def _no_gc():
    """No cyclic garbage collection while a graph is being captured: a
    collection that frees another capture's graph, pool or event then calls
    HIP APIs the global capture mode refuses, and the destructor aborts the
    process (measured: a collection inside a capture's forward).  Pending
    garbage is collected first, outside the capture."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


# Events of TrainStep.stage live as long as the process: an event destroyed
# by the garbage collector while ANOTHER stream is capturing (global capture
# mode) aborts the process (hipEventDestroy is refused during a capture), so
# every staging event comes from a per-TrainStep ring kept here.
_EVENTS_KEEP = []


def _event():
    ev = torch.cuda.Event()
    _EVENTS_KEEP.append(ev)
    return ev


class _Captured:
    def __init__(self, graph, static_batch, loss):
        self.graph = graph
        self.batch = static_batch
        self.loss = loss
        self.slots = [self]  # TrainStep.stage: the graphs of this shape, used in turn
        self.free = None     # event after this graph's last replay (its buffers reusable)
        self.pending = 0     # staged uploads into this graph's buffers not yet stepped

    def released(self, stream):
        if self.free is None:
            self.free = _event()
        self.free.record(stream)

    def load(self, batch):
        """Copy a batch into the graph's static buffers: every contiguous
        same-device tensor goes into batched-copy launches (up to 8 tensors
        per launch, hlhgat_copy2d_batched) instead of one copy launch each
        (15 at the ZINC shape, ~75 us of serial copy kernels per step)."""
        pend = []
        items = [(getattr(sb, k), v) for b, sb in zip(_parts(batch), _parts(self.batch))
                 for k, v in _tensor_items(b)]
        for dst, v in items:
            if dst.data_ptr() == v.data_ptr():
                continue
            if (v.is_cuda and dst.device == v.device and v.is_contiguous() and dst.is_contiguous()
                    and v.dtype == dst.dtype and v.numel() == dst.numel()
                    and (v.numel() * v.element_size()) % 4 == 0):
                pend.append((v, dst))
            else:
                dst.copy_(v, non_blocking=True)
        if pend:
            ops.copy_words_batched([p[0] for p in pend], [p[1] for p in pend])


STAGE_SLOTS = 2  # default captured graphs per batch shape TrainStep.stage fills in turn
STAGE_RING = 8   # staged batches that may be outstanding (uploaded, not yet stepped)
# how an upload into a captured graph's buffers waits for that graph's previous
# replay to release them: "host" (the staging thread waits for the release
# event, then enqueues the copy with no cross-stream dependency) or "device"
# (the copy stream waits on the event).  "host" by default: with the
# device-side wait the runtime blocks the enqueueing thread inside the copy
# until the event has completed anyway (tools/probes/h2d_probe.py) and the
# loader-fed loop measured 0.92 of device-resident steps; with the host-side
# wait 0.96-0.98 (same-box A/B)
STAGE_WAIT = os.environ.get("HLHGAT_STAGE_WAIT", "host")


class Staged:
    """A batch uploaded for a coming step by TrainStep.stage: either already
    in the static buffers of the captured graph `slot`, or in fresh device
    tensors (`batch`); `event` marks the end of the upload."""
    __slots__ = ("batch", "event", "slot", "key", "done")

    def __init__(self, batch, event, slot, key):
        self.batch, self.event, self.slot, self.key = batch, event, slot, key
        self.done = False  # stepped, or given back by TrainStep.unstage


def _quiesce_collectives() -> None:
    """Before a capture: every collective issued so far has completed and left
    its process group's watchdog list (ProcessGroup._wait_for_pending_works),
    so no watchdog query of an eager collective's events overlaps the capture
    (the SyncBatchNorm step's capture_end segfaulted intermittently after eager
    steps full of statistics all-reduces, round 5)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    torch.cuda.synchronize()
    from torch.distributed import distributed_c10d as c10d
    for pg in list(getattr(c10d._world, "pg_map", {}).keys()):
        wait = getattr(pg, "_wait_for_pending_works", None)
        if wait is not None:
            try:
                wait()
            except (RuntimeError, NotImplementedError):  # a backend without it (gloo)
                pass


class TrainStep:
    """step(batch) -> loss: forward, loss_fn(out, batch), backward, gradient
    all-reduce (mean over ranks, as DDP) and Adam (L2 weight decay, as
    torch.optim.Adam).

    graphs=True replays a captured hipGraph per batch shape (requires a ROCm
    device); graphs=False runs the same step eagerly (any device)."""

    def __init__(self, model: torch.nn.Module, loss_fn: Callable, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 graphs: bool = True, max_graphs: int = 32, stage_slots: int = STAGE_SLOTS,
                 overlap: Optional[bool] = None, bucket_mb: Optional[float] = None):
        if isinstance(model, torch.nn.parallel.DistributedDataParallel):
            # DDP would all-reduce the gradients in its hooks and TrainStep again in
            # its bucket (two reductions, and DDP's gradient_as_bucket_view fights the
            # flat gradient views): TrainStep IS the data-parallel wrapper
            raise ValueError("TrainStep: pass the bare module, not a DistributedDataParallel "
                             "wrapper -- TrainStep reduces the gradients itself (one bucket)")
        self.model = model
        self.loss_fn = loss_fn
        # stage(): graphs per batch shape filled in turn (a feeder staging d
        # batches ahead of the step needs d + 1), and the lock that lets a
        # feeder thread stage while this thread replays (slot choice, pending
        # counts and the slot lists are shared)
        if not 1 <= stage_slots <= STAGE_RING:
            raise ValueError(f"TrainStep: stage_slots must be in [1, {STAGE_RING}]")
        self.stage_slots = int(stage_slots)
        self._stage_lock = threading.RLock()
        self._outstanding = 0
        self.stage_timing = dict.fromkeys(("lock", "wait", "copy", "record", "total", "n"), 0.0)
        params = [p for p in model.parameters() if p.requires_grad]
        if not params:
            raise ValueError("TrainStep: model has no trainable parameters")
        dev = params[0].device
        self.device = dev
        self.graphs = bool(graphs) and dev.type == "cuda"
        n = sum(p.numel() for p in params)
        self.flat = torch.empty(n, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        self._offsets = []
        with torch.no_grad():
            for p in params:
                if p.dtype != torch.float32:
                    raise ValueError("TrainStep: fp32 parameters expected")
                k = p.numel()
                self.flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + k].view_as(p)
                p.grad = self.flat_grad[off:off + k].view_as(p)
                self._offsets.append(off)
                off += k
        self.params = params
        # HIP autograd nodes write parameter gradients straight into flat_grad
        # (torch_ext.cpp, "Gradient bucket"): no per-parameter add / copy
        self._ext = None
        if dev.type == "cuda":
            self._ext = ops._ext
            self._ext.grad_bucket_set(params, self.flat_grad, self._offsets)
        self.master = torch.nn.Parameter(self.flat)  # shares storage with the model
        self.master.grad = self.flat_grad
        kw = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        if dev.type == "cuda":
            kw.update(fused=True, capturable=self.graphs)
        self.opt = torch.optim.Adam([self.master], **kw)
        self._hip_adam = dev.type == "cuda" and HIP_ADAM
        if self._hip_adam:
            # the optimiser state torch's fused Adam would create, updated by
            # ONE hlhgat_adam_flat launch (torch's multi-tensor kernel runs a
            # single 65536-element chunk per workgroup on this one flat
            # tensor: ~10 workgroups, 0.1 ms per step at the ZINC size)
            self.opt.state[self.master] = {
                "step": torch.zeros((), dtype=torch.float32, device=dev),
                "exp_avg": torch.zeros_like(self.flat),
                "exp_avg_sq": torch.zeros_like(self.flat)}
            self._hyper = (lr, betas, eps, weight_decay)
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        # the gradient exchange runs (world > 1, or a one-rank group in the
        # tests' COLLECTIVES_AT_WORLD_1 mode)
        self._exchange = collectives_on()
        # under RCCL the all-reduce, the 1/W scale and Adam are captured into
        # the step's graph; under gloo (host collectives) they run after it
        self._exchange_in_graph = (self.graphs and self._exchange
                                   and dist.get_backend() == "nccl")
        self.graphs_off = None
        # (SyncBatchNorm's statistics exchange is an RCCL all-reduce, which
        # captures; round 4's all-gather made hipStreamEndCapture segfault and
        # ProcessGroupNCCL's watchdog query an event of the capturing stream)
        if self.graphs and self._exchange and dist.get_backend() != "nccl" \
                and forward_collectives(model):
            # a collective inside the forward (SyncBatchNorm statistics, the
            # attpool heads' batch-global max) runs on the host under gloo and
            # cannot be captured: this step runs eagerly (RCCL ones can)
            self.graphs = False
            self.graphs_off = "forward collectives under a host (gloo) backend"
        self.max_graphs = max_graphs
        self._graphs: Dict[Tuple, _Captured] = {}
        self._pool = None
        self._stream = ops.own_stream(dev, "capture") if self.graphs else None
        self._setup_buckets(overlap, bucket_mb)
        self.stats = {"eager": 0, "replay": 0, "captures": 0}
        self._fwd_bwd_calls = 0
        self._ones = {}

    # -- the step ---------------------------------------------------------
    def _prepare(self) -> bool:
        """Start of a step: zero the gradient bucket.  With the HIP Adam the
        step count is incremented in the same launch (hlhgat_adam_prepare);
        returns whether it was (the update then must not count again)."""
        if self._hip_adam:
            ops.adam_prepare(self.flat_grad, self.opt.state[self.master]["step"])
            return True
        self.flat_grad.zero_()
        return False

    def _fwd_bwd(self, batch, zeroed: bool = False) -> torch.Tensor:
        if not zeroed:
            self.flat_grad.zero_()
        # deferred split reductions (torch_ext.cpp): not in the first step,
        # which finds the parameters used twice (those are never deferred)
        defer = self._ext is not None and DEFER_REDUCE and self._fwd_bwd_calls > 0
        self._fwd_bwd_calls += 1
        if self._ext is not None:
            for p in self.params:
                p.grad = None
            self._ext.grad_bucket_begin()
        dests = []
        if defer:
            self._ext.reduce_defer(True)
        ov = self._overlap_begin(defer)
        try:
            out = self.model(batch)
            loss = self.loss_fn(out, batch)
            # the seed gradient from a cached ones tensor (no fill launch)
            key = (loss.dtype, loss.device)
            one = self._ones.get(key)
            if one is None:
                one = self._ones[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
            loss.backward(one if loss.dim() == 0 else None)
        finally:
            if ov is not None:
                self._ov = None  # hooks idle again (also after an exception)
            if self._ext is not None and self._fwd_bwd_calls == 1:
                # first step: only a parameter whose .grad IS its bucket view
                # (ONE contribution, a HIP node's view that AccumulateGrad
                # adopted unread) may have its reduction deferred; a summed,
                # cloned or torch-produced gradient is never deferred (with the
                # overlap, a bucket's launch re-points .grad at its view: the
                # hook recorded what AccumulateGrad had left there)
                base = self.flat_grad.data_ptr()
                self._ext.grad_bucket_no_defer(
                    [p for i, (p, off) in enumerate(zip(self.params, self._offsets))
                     if (ov is not None and i in ov["not_adopted"]) or p.grad is None
                     or p.grad.data_ptr() != base + 4 * off])
            if defer:
                # the last reduction of each stream, before anything reads the bucket
                dests = self._ext.reduce_flush(self._dev_index())
                self._ext.reduce_defer(False)
        if ov is not None:
            dests = list(dests) + ov["dests"]
        if self._ext is not None:
            self._adopt_grads(set(dests))
        if ov is not None:
            # buckets whose hooks did not all fire (unused parameters; a
            # gradient that never reached AccumulateGrad): now, after the flush
            late = 0
            for b in range(len(self._buckets)):
                if not ov["launched"][b]:
                    self._launch_bucket(ov, b, flush=False)
                    late += 1
            self._ov_works = ov["works"]
            self.overlap_stats["in_backward"] += len(self._buckets) - late
            self.overlap_stats["after_backward"] += late
        return loss.detach()

    # -- the gradient exchange, bucketed and overlapped with the backward --
    def _dev_index(self) -> int:
        return self.device.index if self.device.index is not None else torch.cuda.current_device()

    def _setup_buckets(self, overlap: Optional[bool], bucket_mb: Optional[float]) -> None:
        """Buckets of the flat gradient buffer (contiguous ranges, last
        parameters first, each >= bucket_mb unless it is the first) and a
        post-accumulate-grad hook per parameter that counts its bucket down."""
        self._ov = None
        self._ov_works = []
        self._buckets = []
        self.overlap = False
        # bucket all-reduces issued from the backward's hooks / after it
        self.overlap_stats = {"in_backward": 0, "after_backward": 0}
        if not self._exchange:
            return
        mb = BUCKET_MB if bucket_mb is None else float(bucket_mb)
        lim = max(1, int(mb * (1 << 20) / 4))
        cur, size = [], 0
        for i in reversed(range(len(self.params))):
            cur.append(i)
            size += self.params[i].numel()
            if size >= lim:
                self._buckets.append(cur)
                cur, size = [], 0
        if cur:
            self._buckets.append(cur)
        want = OVERLAP if overlap is None else ("1" if overlap else "0")
        on = want == "1" or (want == "auto" and len(self._buckets) >= 2)
        # replayed gloo steps exchange after the replay (host collectives are
        # not captured): nothing to overlap with there
        on = on and (not self.graphs or self._exchange_in_graph)
        if not on:
            self._buckets = []
            return
        self.overlap = True
        self._bucket_of = {}
        for b, idx in enumerate(self._buckets):
            for i in idx:
                self._bucket_of[i] = b
        self._ranges = []
        for idx in self._buckets:
            lo = min(self._offsets[i] for i in idx)
            hi = max(self._offsets[i] + self.params[i].numel() for i in idx)
            self._ranges.append((lo, hi))
        for i, p in enumerate(self.params):
            p.register_post_accumulate_grad_hook(self._grad_hook(i))

    def _grad_hook(self, i: int):
        def hook(p):
            ov = self._ov
            if ov is None:
                return
            off = self._offsets[i]
            if p.grad is None or p.grad.data_ptr() != self.flat_grad.data_ptr() + 4 * off:
                ov["not_adopted"].add(i)
            b = self._bucket_of[i]
            ov["left"][b] -= 1
            if ov["left"][b] == 0 and not ov["launched"][b]:
                self._launch_bucket(ov, b, flush=True)
        return hook

    def _overlap_begin(self, defer: bool):
        if not self.overlap:
            return None
        self._ov_works = []
        self._ov = {"left": [len(idx) for idx in self._buckets],
                    "launched": [False] * len(self._buckets), "works": [], "dests": [],
                    "not_adopted": set(), "defer": defer,
                    "main": torch.cuda.current_stream(self.device)
                    if self.device.type == "cuda" else None}
        return self._ov

    def _launch_bucket(self, ov, b: int, flush: bool) -> None:
        """All-reduce bucket b now: on the step's main stream, after every
        stream that produced gradients so far (the chains' and fork's side
        streams that are part of the step), after the deferred split
        reductions pending so far (hlhgat reduce_flush: a deferred gradient is
        written by a later launch on its stream), with each gradient
        AccumulateGrad did not adopt copied into the bucket view first."""
        ov["launched"][b] = True
        main = ov["main"]
        ctx = torch.cuda.stream(main) if main is not None else contextlib.nullcontext()
        with ctx:
            if main is not None and self._ext is not None:
                self._ext.join_capture_streams(self._dev_index(), self._side_handles()) \
                    if torch.cuda.is_current_stream_capturing() else self._join_sides(main)
            if flush and ov["defer"]:
                ov["dests"].extend(self._ext.reduce_flush(self._dev_index()))
            deferred = set(ov["dests"])
            base = self.flat_grad.data_ptr()
            for i in self._buckets[b]:
                p, off = self.params[i], self._offsets[i]
                view = self.flat_grad[off:off + p.numel()].view_as(p)
                g = p.grad
                if g is not None and g.data_ptr() != base + 4 * off:
                    if base + 4 * off not in deferred:
                        view.copy_(g)
                    p.grad = view
            lo, hi = self._ranges[b]
            ov["works"].append(dist.all_reduce(self.flat_grad[lo:hi], async_op=True))

    def _side_handles(self):
        idx = self._dev_index()
        return [ops.side_stream(self.device, k).cuda_stream for k in (0, 1)] + \
            [int(self._ext.fork_side_stream(idx))]

    def _join_sides(self, main) -> None:
        # eager: the main stream waits for every side stream and for the
        # stream this hook runs on (autograd's, for the node that finished)
        cur = torch.cuda.current_stream(self.device)
        for h in self._side_handles():
            main.wait_stream(torch.cuda.ExternalStream(h, device=self.device))
        if cur.cuda_stream != main.cuda_stream:
            main.wait_stream(cur)

    def _adopt_grads(self, deferred=frozenset()) -> None:
        """Every p.grad must be its flat_grad view: gradients produced outside
        the bucket (torch ops) are copied in; missing ones stay zero."""
        base = self.flat_grad.data_ptr()
        for p, off in zip(self.params, self._offsets):
            g = p.grad
            view = self.flat_grad[off:off + p.numel()].view_as(p)
            if g is None:
                p.grad = view
            elif g.data_ptr() != base + 4 * off:
                if base + 4 * off not in deferred:
                    view.copy_(g)
                # else: AccumulateGrad cloned the view before its deferred
                # reduction ran; the bucket region itself holds the gradient
                p.grad = view

    def _opt_step(self, prepared: bool = False) -> None:
        if not self._hip_adam:
            self.opt.step()
            return
        st = self.opt.state[self.master]
        lr, betas, eps, wd = self._hyper
        ops.adam_flat(self.flat, self.flat_grad, st["exp_avg"], st["exp_avg_sq"], st["step"],
                      lr, betas, eps, wd, prepared=prepared)

    def _exchange_and_update(self, prepared: bool = False) -> None:
        if self._exchange:
            if self.overlap and self._ov_works:
                # the buckets' all-reduces were issued during the backward
                works, self._ov_works = self._ov_works, []
                for w in works:
                    w.wait()
            else:
                dist.all_reduce(self.flat_grad)  # one contiguous bucket
            self.flat_grad.div_(self.world)  # mean over ranks, as DDP
        self._opt_step(prepared)

    def _eager(self, batch) -> torch.Tensor:
        ops.clear_caches()
        prepared = self._prepare()
        loss = self._fwd_bwd(batch, zeroed=True)
        self._exchange_and_update(prepared)
        ops.clear_caches()
        self.stats["eager"] += 1
        return loss

    def _capture(self, batch, key, slot_of: Optional[_Captured] = None) -> _Captured:
        if slot_of is not None:  # a staged device batch becomes the new slot's buffers
            static = batch
            for b in _parts(static):
                if hasattr(b, "_mark"):
                    b._mark()
        else:
            static = ([_clone_batch(b) for b in batch] if isinstance(batch, (list, tuple))
                      else _clone_batch(batch))
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph(keep_graph=KEEP_GRAPHS)
        s = self._stream
        if self._ext is not None and BN_RESERVE_CHANNELS:
            # BatchNorm workspaces of every stream the capture uses, made (and
            # zeroed) outside the capture: no zero fill recorded into the graph
            idx = self.device.index if self.device.index is not None else \
                torch.cuda.current_device()
            for h in [s.cuda_stream, int(self._ext.fork_side_stream(idx))] + \
                    [ops.side_stream(self.device, k).cuda_stream for k in (0, 1)]:
                self._ext.bn_workspace_reserve(int(h), idx, BN_RESERVE_CHANNELS)
        s.wait_stream(torch.cuda.current_stream(self.device))
        ops.clear_caches()
        _quiesce_collectives()
        # thread-local capture: the data loader's collation threads and a
        # StagedFeed thread keep running beside it (pinned allocations, copies
        # on other streams are legal there; a global-mode capture turns them
        # into hipErrorStreamCaptureUnsupported); the stage lock keeps the
        # feeder's uploads out of the capture window altogether
        with self._stage_lock, _no_gc(), torch.cuda.graph(g, pool=self._pool, stream=s,
                                                          capture_error_mode="thread_local"):
            prepared = self._prepare()
            loss = self._fwd_bwd(static, zeroed=True)
            if self._exchange_in_graph:
                self._exchange_and_update(prepared)  # RCCL all-reduce + scale + Adam, captured
            elif not self._exchange:
                self._opt_step(prepared)
            # every stream forked from the capture (the node / edge side streams,
            # forks inside autograd backward nodes, which run on autograd's
            # device thread) rejoins it before hipStreamEndCapture: an unjoined
            # fork is what crashed capture_end in round 1
            if self._ext is not None:
                ops.join_capture_streams(self.device)
        left = ops.side_streams_capturing(self.device) if self._ext is not None else []
        if left:
            raise RuntimeError(f"TrainStep: {len(left)} side stream(s) still capturing after the "
                               f"graph capture ended (unjoined fork); refusing the graph")
        ops.clear_caches()
        torch.cuda.current_stream(self.device).wait_stream(s)
        if KEEP_GRAPHS:
            g.instantiate()
        ent = _Captured(g, static, loss)
        self.stats["captures"] += 1
        if slot_of is not None:
            with self._stage_lock:
                slot_of.slots.append(ent)
            return ent
        if len(self._graphs) >= self.max_graphs:
            self._graphs.pop(next(iter(self._graphs)))
        self._graphs[key] = ent
        return ent

    def stage(self, batch, stream: Optional["torch.cuda.Stream"] = None) -> Staged:
        """Upload a host batch (pinned CPU tensors, e.g. hlhgat.loader.
        GraphLoader's) for a coming step, on `stream` (default: a copy stream
        of this TrainStep), and return the handle to pass to step(...).  Once
        the batch shape has STAGE_SLOTS captured graphs, the tensors go
        straight into the static buffers of the graph that replays next, after
        its previous replay has released them (double buffering): the step
        then replays with no copy-in at all.  Until then (first steps of a
        shape) the batch goes to fresh device tensors, which the step adopts
        as the next graph's static buffers."""
        if not self.graphs:
            raise RuntimeError("TrainStep.stage needs graphs=True (a ROCm device)")
        if stream is None:
            if getattr(self, "_copy_stream", None) is None:
                self._copy_stream = ops.own_stream(self.device, "copy")
            stream = self._copy_stream
        key = batch_key(batch)
        # the stream the replays run on (stage may be called from a feeder
        # thread, whose current stream is not the training loop's)
        main = getattr(self, "_replay_stream", None) or torch.cuda.current_stream(self.device)
        self._staging = True
        # only the bookkeeping holds the lock (slot choice, pending count, ring
        # event): the uploads themselves are enqueued after it is released, so
        # the training thread's replay bookkeeping never waits for a feeder's
        # copies (round 5: holding it for the whole body put 1.5 ms of the
        # feeder's stage() into every step call).  A capture may then run
        # beside an upload: thread-local capture mode allows that, the copy is
        # on another stream and into a slot no capture touches.
        clock = time.perf_counter
        t0 = clock()
        with self._stage_lock:
            t1 = clock()
            ev, slot, free = self._stage_plan(key)
        try:
            st = self._stage_copy(batch, stream, key, main, ev, slot, free)
        except BaseException:
            self._release(slot)  # the plan counted this batch: give the counts back
            raise
        # host time per stage() part (diagnostics: bench.py's loader leg)
        tm = self.stage_timing
        tm["lock"] += t1 - t0
        tm["total"] += clock() - t0
        tm["n"] += 1
        return st

    def _stage_plan(self, key):
        # a ring of events (kept for the process, see _EVENTS_KEEP): at most
        # STAGE_RING staged batches may be outstanding (a ring event is
        # re-recorded only once its batch has been stepped)
        if self._outstanding >= STAGE_RING:
            raise RuntimeError(f"TrainStep.stage: more than {STAGE_RING} staged batches "
                               f"outstanding (step them before staging more)")
        ring = getattr(self, "_stage_ring", None)
        if ring is None:
            ring = self._stage_ring = [_event() for _ in range(STAGE_RING)]
            self._stage_next = 0
        ev = ring[self._stage_next]
        self._stage_next = (self._stage_next + 1) % STAGE_RING
        self._outstanding += 1
        ent = self._graphs.get(key)
        slot = None
        if ent is not None and len(ent.slots) >= self.stage_slots:
            # the next graph of the shape in turn whose buffers no staged
            # batch is waiting in (a slot with one pending would be
            # overwritten before its batch is stepped)
            n = len(ent.slots)
            k0 = getattr(ent, "next_slot", 0)
            for d in range(n):
                cand = ent.slots[(k0 + d) % n]
                if cand.pending == 0:
                    slot = cand
                    ent.next_slot = (k0 + d + 1) % n
                    break
        free = None
        if slot is not None:
            slot.pending += 1
            free = slot.free
        return ev, slot, free

    def _release(self, slot) -> None:
        """Undo one staged batch's bookkeeping: its slot's pending count (the
        slot may be staged into again) and the outstanding count."""
        with self._stage_lock:
            if slot is not None:
                slot.pending -= 1
            self._outstanding -= 1

    def unstage(self, st: Staged) -> None:
        """Give back a staged batch that will not be stepped (a feed closed
        early: a break, an exception, StagedFeed.close()).  Its upload may
        still be in flight; a later stage() into the same slot waits for the
        slot's release as always, and the copy stream is in order.  A handle
        already stepped or given back is ignored."""
        if st.done:
            return
        st.done = True
        self._release(st.slot)

    def _stage_copy(self, batch, stream, key, main, ev, slot, free) -> Staged:
        if slot is None:  # fresh device tensors (first steps of a shape, or every slot taken)
            with torch.cuda.stream(stream):
                dev = [self._upload(b) for b in _parts(batch)]
                if not isinstance(batch, (list, tuple)):
                    dev = dev[0]
                ev.record(stream)
            for b in _parts(dev):
                for _, v in _tensor_items(b):
                    v.record_stream(main)
            return Staged(dev, ev, None, key)
        clock = time.perf_counter
        t0 = clock()
        if free is not None:
            if STAGE_WAIT == "host":
                free.synchronize()
            else:
                stream.wait_event(free)
        else:  # replayed before staging began (no release event): after all of main
            stream.wait_stream(main)
        t1 = clock()
        with torch.cuda.stream(stream):
            for b, sb in zip(_parts(batch), _parts(slot.batch)):
                ha, da = getattr(b, "_arena", None), getattr(sb, "_arena", None)
                if (ha is not None and da is not None and _in_arena(b, ha)
                        and _same_layout(b, ha, sb, da)):
                    da.copy_(ha, non_blocking=True)  # the whole batch in one copy
                    continue
                for name, v in _tensor_items(b):
                    getattr(sb, name).copy_(v, non_blocking=True)
            t2 = clock()
            ev.record(stream)
        tm = self.stage_timing
        tm["wait"] += t1 - t0
        tm["copy"] += t2 - t1
        tm["record"] += clock() - t2
        return Staged(None, ev, slot, key)

    def _upload(self, b):
        """A device copy of batch object b that shares no storage with it
        (it may become a graph's static buffers, which later uploads
        overwrite).  A batch whose tensors all live in one host arena
        (PackedGraphs.collate) goes up in one copy, as views of a device
        arena with the same layout."""
        out = type(b).__new__(type(b))
        arena = getattr(b, "_arena", None)
        if arena is not None and not arena.is_cuda and _in_arena(b, arena):
            da = arena.to(self.device, non_blocking=True)
            base = arena.data_ptr()
            for k, v in vars(b).items():
                if k == "_arena":
                    continue
                if torch.is_tensor(v):
                    o = v.data_ptr() - base
                    nb = v.numel() * v.element_size()
                    setattr(out, k, da[o:o + nb].view(v.dtype).view(v.shape))
                else:
                    setattr(out, k, v)
            out._arena = da
        else:
            for k, v in vars(b).items():
                if k == "_arena":
                    continue
                if torch.is_tensor(v):
                    d = v.to(self.device, non_blocking=True)
                    setattr(out, k, d.clone() if d.data_ptr() == v.data_ptr() else d)
                else:
                    setattr(out, k, v)
        if hasattr(out, "_mark"):
            out._mark()
        return out

    def _replay(self, ent: _Captured) -> torch.Tensor:
        self._replay_stream = torch.cuda.current_stream(self.device)
        ent.graph.replay()
        if getattr(self, "_staging", False):  # stage() waits for the slot's release
            ent.released(torch.cuda.current_stream(self.device))
        if self._exchange and not self._exchange_in_graph:
            # the graph began with _prepare (the step counted when HIP Adam)
            self._exchange_and_update(prepared=self._hip_adam)
        self.stats["replay"] += 1
        return ent.loss

    def _call_staged(self, st: Staged) -> torch.Tensor:
        if st.done:
            raise RuntimeError("TrainStep: this staged batch was already stepped or unstaged")
        st.done = True
        torch.cuda.current_stream(self.device).wait_event(st.event)
        try:
            if st.slot is not None:
                try:
                    return self._replay(st.slot)  # records the slot's release event
                finally:
                    with self._stage_lock:  # only now may a feeder stage into it again
                        st.slot.pending -= 1
            ent = self._graphs.get(st.key)
            if ent is None:
                return self(st.batch)
            if len(ent.slots) >= self.stage_slots:
                with self._stage_lock:
                    free = [sl for sl in ent.slots if sl.pending == 0]
                    if free:  # taken, so a feeder does not stage into it meanwhile
                        free[0].pending += 1
                if free:  # copy-in into a graph no staged upload is waiting for
                    try:
                        free[0].load(st.batch)
                        return self._replay(free[0])
                    finally:
                        with self._stage_lock:
                            free[0].pending -= 1
            # one more slot for this shape: the staged tensors are its static
            # buffers; capturing does not run the step, the first replay does
            return self._replay(self._capture(st.batch, st.key, slot_of=ent))
        finally:
            with self._stage_lock:
                self._outstanding -= 1

    def __call__(self, batch) -> torch.Tensor:
        # a kernel of an earlier step that reported unusable results (the
        # device error word, read without synchronising) stops training here
        if self._ext is not None:
            ops.check_device_errors(sync=False)
        if isinstance(batch, Staged):
            return self._call_staged(batch)
        if not self.graphs:
            return self._eager(batch)
        key = batch_key(batch)
        ent = self._graphs.get(key)
        if ent is None:
            loss = self._eager(batch)
            self._capture(batch, key)
            return loss
        with self._stage_lock:
            free = [sl for sl in ent.slots if sl.pending == 0]
            if free:
                free[0].pending += 1
        if not free:  # every graph of the shape awaits a staged batch: one more
            return self._replay(self._capture(self._upload(batch), key, slot_of=ent))
        try:
            free[0].load(batch)
            return self._replay(free[0])
        finally:
            with self._stage_lock:
                free[0].pending -= 1

    def state_dict(self):
        return {"model": self.model.state_dict(), "opt": self.opt.state_dict()}


class InferStep:
    """Evaluation / serving: the reference's test() loop body
    (main_zinc_HL_HGCNN_dense_int3_pyr.py:165-177, main_pepfunc...:201-225):
    model.eval() and ``out = model(data)`` under torch.no_grad(), one batch
    per call.  graphs=True captures the eval forward into a hipGraph per batch
    shape (the first call of a shape runs eagerly, then captures) and replays
    it; the returned output is the graph's static
    buffer, valid until the next call with a batch of the same shape (clone
    it to keep it)."""

    def __init__(self, model: torch.nn.Module, graphs: bool = True, max_graphs: int = 32):
        self.model = model
        params = list(model.parameters())
        dev = params[0].device if params else torch.device("cpu")
        self.device = dev
        self.graphs = bool(graphs) and dev.type == "cuda"
        self.max_graphs = max_graphs
        self._graphs: Dict[Tuple, _Captured] = {}
        self._pool = None
        self._stream = ops.own_stream(dev, "capture") if self.graphs else None
        self.stats = {"eager": 0, "replay": 0, "captures": 0}

    def _forward(self, batch):
        was = self.model.training
        self.model.eval()
        try:
            with torch.no_grad():
                return self.model(batch)
        finally:
            self.model.train(was)

    def _capture(self, batch, key):
        static = ([_clone_batch(b) for b in batch] if isinstance(batch, (list, tuple))
                  else _clone_batch(batch))
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph(keep_graph=KEEP_GRAPHS)
        s = self._stream
        s.wait_stream(torch.cuda.current_stream(self.device))
        ops.clear_caches()
        _quiesce_collectives()
        with _no_gc(), torch.cuda.graph(g, pool=self._pool, stream=s,
                                        capture_error_mode="thread_local"):
            out = self._forward(static)
            ops.join_capture_streams(self.device)
        left = ops.side_streams_capturing(self.device)
        if left:
            raise RuntimeError(f"InferStep: {len(left)} side stream(s) still capturing after the "
                               f"graph capture ended (unjoined fork); refusing the graph")
        ops.clear_caches()
        torch.cuda.current_stream(self.device).wait_stream(s)
        if KEEP_GRAPHS:
            g.instantiate()
        if len(self._graphs) >= self.max_graphs:
            self._graphs.pop(next(iter(self._graphs)))
        ent = _Captured(g, static, out)
        self._graphs[key] = ent
        self.stats["captures"] += 1
        return ent

    def __call__(self, batch):
        if ops._ext is not None:
            ops.check_device_errors(sync=False)
        if not self.graphs:
            self.stats["eager"] += 1
            return self._forward(batch)
        key = batch_key(batch)
        ent = self._graphs.get(key)
        if ent is None:
            out = self._forward(batch)
            self.stats["eager"] += 1
            self._capture(batch, key)
            return out
        ent.load(batch)
        ent.graph.replay()
        self.stats["replay"] += 1
        return ent.loss  # the captured forward's output
