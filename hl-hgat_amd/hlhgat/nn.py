"""PyG-free building blocks with the reference's module names and semantics.

The reference composes its layers with torch_geometric ``Sequential``,
``BatchNorm`` and ``Linear`` (e.g. lib/Hodge_ST_Model.py:556-567,
lib/Hodge_Cheb_Conv.py:462-465); its checkpoints therefore carry keys such as
``HL_init_conv.module_0.lins.0.weight`` and ``.module_1.module.running_mean``
(verified against HL-HGAT-DEMO/weights/HL_HGAT_Brain.pt).  These classes
reproduce those names so reference state_dicts load unchanged.
"""
from __future__ import annotations

import math
import re
from typing import Callable, List, Sequence, Tuple, Union

import torch
import torch.nn as tnn

__all__ = ["Sequential", "BatchNorm", "Linear", "L1Loss", "BCEWithLogitsLoss", "glorot",
           "global_mean_pool"]


def glorot(t: torch.Tensor) -> None:
    """torch_geometric.nn.inits.glorot: U(-a, a), a = sqrt(6/(fan_in+fan_out))."""
    if t is not None:
        a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
        with torch.no_grad():
            t.uniform_(-a, a)


class Linear(tnn.Module):
    """torch_geometric.nn.dense.linear.Linear (weight [out, in]); the convs only
    use ``.weight`` (bias=False, weight_initializer='glorot',
    lib/Hodge_Cheb_Conv.py:462-465)."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True,
                 weight_initializer: str = "glorot", bias_initializer=None):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight_initializer = weight_initializer
        self.weight = tnn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = tnn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        if self.weight_initializer == "glorot":
            glorot(self.weight)
        else:
            tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .ops import linear_blocks
        shp = x.shape
        y = linear_blocks([x.reshape(-1, shp[-1])], self.weight, self.bias)
        return y.view(*shp[:-1], self.out_channels)

    def __repr__(self) -> str:
        return (f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, "
                f"bias={self.bias is not None})")


class BatchNorm(tnn.Module):
    """torch_geometric.nn.BatchNorm: BatchNorm1d held as ``.module``."""

    def __init__(self, in_channels: int, eps: float = 1e-5, momentum: float = 0.1,
                 affine: bool = True, track_running_stats: bool = True):
        super().__init__()
        self.in_channels = in_channels
        self.module = tnn.BatchNorm1d(in_channels, eps, momentum, affine, track_running_stats)

    def reset_parameters(self) -> None:
        self.module.reset_parameters()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from .ops import batch_norm_act
        return batch_norm_act(x, self.module, relu=False)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels})"


_ARROW = re.compile(r"\s*->\s*")

# Activation tap (test infrastructure): while TAP is a dict, every ReLU site
# -- fused into a conv / BatchNorm node or not -- records a copy of its output
# under the nn.ReLU module it stands for, one entry per call in call order.
# The frozen-mask gradient checks (tests/test_frozen_mask_grads.py) rebuild
# the ReLU masks of the HIP forward from it.
TAP = None


def tap(mod, y) -> None:
    if TAP is not None and torch.is_tensor(y):
        TAP.setdefault(mod, []).append(y.detach().clone())


class Abs(tnn.Module):
    """x.abs() as a module (the TSP readout's |B1^T x_t|, lib/Hodge_ST_Model.py:
    848): under TAP its input is recorded, so the gradient gates can freeze
    the signs the HIP forward saw (tests/test_frozen_mask_grads.py)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        tap(self, x)
        return x.abs()


class L1Loss(tnn.L1Loss):
    """torch.nn.L1Loss (the ZINC training loss) whose mean reduction on ROCm
    tensors runs as one HIP launch each way (ops.l1_loss: the same input
    gradient bit for bit).  CPU tensors and other reductions go to torch."""

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if (self.reduction == "mean" and input.is_cuda and input.dtype == torch.float32
                and input.shape == target.shape and not target.requires_grad
                and input.numel() > 0):
            from . import ops
            return ops.l1_loss(input, target)
        return super().forward(input, target)


class BCEWithLogitsLoss(tnn.BCEWithLogitsLoss):
    """torch.nn.BCEWithLogitsLoss (the peptides-func and TSP training losses)
    whose unweighted "mean" / "sum" reductions on ROCm fp32 tensors run as one
    HIP launch each way (ops.bce_with_logits; the input gradient in ATen's
    arithmetic) up to FUSED_MAX elements: the forward's fixed-order sum is one
    workgroup, which for a per-edge loss (config 5: 207k logits) waits on
    ~800 dependent loads per lane and loses to ATen's grid reduction
    (measured +0.3 ms per config-5 step).  Weights, pos_weight, CPU tensors,
    "none" and larger inputs go to torch."""

    FUSED_MAX = 16384

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if (self.weight is None and self.pos_weight is None
                and self.reduction in ("mean", "sum") and input.is_cuda
                and input.dtype == torch.float32 and input.shape == target.shape
                and not target.requires_grad and 0 < input.numel() <= self.FUSED_MAX):
            from . import ops
            return ops.bce_with_logits(input, target, self.reduction)
        return super().forward(input, target)


def _names(s: str) -> List[str]:
    return [t.strip() for t in s.split(",") if t.strip()]


class Sequential(tnn.Module):
    """torch_geometric.nn.Sequential(input_args, [(callable, 'a, b -> c'), ...]).

    Entry i is registered as ``module_{i}`` (modules and plain callables
    alike), arguments are routed by name, and the value of the last entry is
    returned — e.g. the ``lambda x1, x2: [x1, x2]`` tail of every HL block
    (lib/Hodge_ST_Model.py:566)."""

    def __init__(self, input_args: str,
                 modules: Sequence[Union[Tuple[Callable, str], Callable]]):
        super().__init__()
        self.input_args = _names(input_args)
        self._routes: List[Tuple[List[str], List[str]]] = []
        prev_out = list(self.input_args)
        for i, entry in enumerate(modules):
            if isinstance(entry, (tuple, list)):
                fn, desc = entry
                parts = _ARROW.split(desc)
                ins = _names(parts[0])
                outs = _names(parts[1]) if len(parts) > 1 else list(ins)
            else:
                fn, ins, outs = entry, list(prev_out), list(prev_out[:1])
            if isinstance(fn, tnn.Module):
                self.add_module(f"module_{i}", fn)
            else:
                object.__setattr__(self, f"module_{i}", fn)
            self._routes.append((ins, outs))
            prev_out = outs
        self._n = len(modules)
        # Fusions (same result as the modules in turn):
        #  HodgeConv -> BatchNorm [-> ReLU] on one variable: one C++ node
        #  BatchNorm -> ReLU: one fused HIP BN+ReLU op
        self._fuse = [None] * self._n  # (kind, n_entries_consumed)
        i = 0
        while i < self._n:
            m0 = getattr(self, f"module_{i}")
            r0 = self._routes[i]

            def same_var(j):
                return (j < self._n and len(r0[1]) == 1
                        and self._routes[j][0] == r0[1] and self._routes[j][1] == r0[1])

            if hasattr(m0, "forward_bn") and same_var(i + 1) and isinstance(
                    getattr(self, f"module_{i + 1}"), BatchNorm):
                relu = same_var(i + 2) and isinstance(getattr(self, f"module_{i + 2}"), tnn.ReLU)
                self._fuse[i] = ("conv_bn_relu" if relu else "conv_bn", 3 if relu else 2)
            elif isinstance(m0, BatchNorm) and same_var(i + 1) and isinstance(
                    getattr(self, f"module_{i + 1}"), tnn.ReLU):
                self._fuse[i] = ("bn_relu", 2)
            i += self._fuse[i][1] if self._fuse[i] else 1
        self._split = self._two_chains()

    def _two_chains(self):
        """Index s such that entries [0, s) and [s, n-1) touch disjoint
        variables and entry n-1 joins them (the node / edge chains of every
        HL block, lib/Hodge_ST_Model.py:556-566), else None."""
        if self._n < 3:
            return None
        for s in range(1, self._n - 1):
            if any(self._fuse[j] and j + self._fuse[j][1] > s for j in range(s)):
                continue
            a = set().union(*[set(r[0]) | set(r[1]) for r in self._routes[:s]])
            b = set().union(*[set(r[0]) | set(r[1]) for r in self._routes[s:self._n - 1]])
            if not (a & b):
                last_in = set(self._routes[-1][0])
                if last_in & a and last_in & b:
                    return s
        return None

    def _run(self, env, lo, hi):
        out = None
        i = lo
        while i < hi:
            ins, outs = self._routes[i]
            fn = getattr(self, f"module_{i}")
            fuse = self._fuse[i]
            if fuse is None:
                if isinstance(fn, tnn.Dropout) and (fn.p == 0.0 or not fn.training):
                    out = env[ins[0]]  # identity: no copy kernel
                else:
                    out = fn(*[env[n] for n in ins])
                    if isinstance(fn, tnn.ReLU):
                        tap(fn, out)
                i += 1
            elif fuse[0] == "bn_relu":
                from .ops import batch_norm_act
                out = batch_norm_act(env[ins[0]], fn.module, relu=True)
                tap(getattr(self, f"module_{i + 1}"), out)
                i += 2
            else:
                bn = getattr(self, f"module_{i + 1}").module
                out = fn.forward_bn(*[env[n] for n in ins], bn=bn,
                                    relu=fuse[0] == "conv_bn_relu")
                if fuse[0] == "conv_bn_relu":
                    tap(getattr(self, f"module_{i + 2}"), out)
                i += fuse[1]
            if len(outs) == 1:
                env[outs[0]] = out
            else:
                for n, v in zip(outs, out):
                    env[n] = v
        return out

    def forward(self, *args):
        if len(args) != len(self.input_args):
            raise TypeError(f"Sequential expects {len(self.input_args)} inputs "
                            f"({', '.join(self.input_args)}), got {len(args)}")
        env = dict(zip(self.input_args, args))
        s = self._split
        dev = next((a.device for a in args if torch.is_tensor(a)), None)
        if s is None or dev is None:
            return self._run(env, 0, self._n)
        from .ops import active_chains, fork
        side_env = dict(env)
        ch = active_chains(dev)
        if ch is not None:
            # the block section's two chains (ops.Chains): the edge half on the
            # side stream, no fork wait and no join
            with torch.cuda.stream(ch.side):
                self._run(side_env, s, self._n - 1)
            self._run(env, 0, s)
            for r in self._routes[s:self._n - 1]:
                for k in r[1]:
                    env[k] = side_env[k]
            return self._run(env, self._n - 1, self._n)
        # node chain on the current stream, edge chain on the side stream
        side_in = [env[n] for r in self._routes[s:self._n - 1] for n in r[0]
                   if n in env and torch.is_tensor(env[n])]
        fork(lambda: self._run(env, 0, s), lambda: self._run(side_env, s, self._n - 1),
             side_inputs=side_in, device=dev)
        for r in self._routes[s:self._n - 1]:
            for k in r[1]:
                env[k] = side_env[k]
        return self._run(env, self._n - 1, self._n)

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i: int):
        return getattr(self, f"module_{i}")


def run_sequential(seq: tnn.Sequential, blocks) -> torch.Tensor:
    """Run an nn.Sequential of Linear / BatchNorm1d / ReLU / Dropout modules on
    the HIP ops: the first Linear consumes ``blocks`` (a list of tensors whose
    concatenation is its input, e.g. cat[x_s2t, x_t] of NodeEdgeInt,
    lib/Hodge_Cheb_Conv.py:307-308) without materialising the cat, and each
    BatchNorm1d followed by ReLU runs as one fused op."""
    from .ops import batch_norm_act, linear_blocks
    mods = list(seq)
    h = None
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, tnn.Linear):
            h = linear_blocks(blocks if h is None else [h], m.weight, m.bias)
        elif isinstance(m, tnn.BatchNorm1d):
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], tnn.ReLU)
            h = batch_norm_act(h, m, relu=relu)
            if relu:
                tap(mods[i + 1], h)
            i += relu
        elif isinstance(m, tnn.Dropout) and (m.p == 0.0 or not m.training):
            pass
        else:
            h = m(h if h is not None else torch.cat(list(blocks), -1))
            if isinstance(m, tnn.ReLU):
                tap(m, h)
        i += 1
    return h


def _bn_relu_layer(mods, i):
    """mods[i:i+3] is Linear -> training-mode BatchNorm1d -> ReLU."""
    from .ops import sync_bn_group
    return (i + 3 <= len(mods) and isinstance(mods[i], tnn.Linear)
            and isinstance(mods[i + 1], tnn.BatchNorm1d) and isinstance(mods[i + 2], tnn.ReLU)
            and (mods[i + 1].training or not mods[i + 1].track_running_stats)
            and sync_bn_group(mods[i + 1]) is None)


MLP_PAIRS = True  # A/B hook: False = run_mlp_stack runs module by module


def run_mlp_stack(seqs, blocks) -> torch.Tensor:
    """The readout MLP of the heads (consecutive nn.Sequential layers Linear ->
    BatchNorm1d -> ReLU -> Dropout, lib/Hodge_ST_Model.py:589-597): identity
    dropouts dropped, every two consecutive Linear -> BN -> ReLU layers run as
    ONE fused node (ops.mlp2: each Linear + BatchNorm in one launch), the rest
    module by module (run_sequential).  The same arithmetic as running the
    layers one by one."""
    from . import ops
    mods = [m for seq in seqs for m in seq
            if not (isinstance(m, tnn.Dropout) and (m.p == 0.0 or not m.training))]
    h, i = None, 0
    while i < len(mods):
        if MLP_PAIRS and _bn_relu_layer(mods, i) and _bn_relu_layer(mods, i + 3):
            tapping = TAP is not None
            if tapping:
                ops._ext.set_tap(True)
            h = ops.mlp2(blocks if h is None else [h], mods[i:i + 6])
            if tapping:
                hidden = ops._ext.take_tap()
                ops._ext.set_tap(False)
                tap(mods[i + 2], hidden[0])
                tap(mods[i + 5], h)
            i += 6
        else:
            j = i + 1
            while j < len(mods) and not (MLP_PAIRS and _bn_relu_layer(mods, j)
                                         and _bn_relu_layer(mods, j + 3)):
                j += 1
            h = run_sequential(tnn.Sequential(*mods[i:j]), blocks if h is None else [h])
            i = j
    return h


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor, size: int = None) -> torch.Tensor:
    """torch_geometric.nn.global_mean_pool over a sorted batch vector
    (PairData batches are graph-contiguous), on the HIP segment-mean kernel."""
    from .ops import segment_mean
    if size is None:
        size = int(batch.max().item()) + 1 if batch.numel() else 0
    counts = torch.bincount(batch, minlength=size)
    ptr = torch.zeros(size + 1, dtype=torch.int32, device=x.device)
    ptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return segment_mean(x, ptr, size)
