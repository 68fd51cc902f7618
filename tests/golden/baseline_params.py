"""Deterministic parameters for the BASELINE-hyperparameter fixtures.

The config 3/4/5 heads have 2.5-4.1 M parameters; storing their state dicts
(and every gradient) would make 10+ MB fixtures.  Instead the generator
(make_golden_baseline.py, run against the reference) and the tests (run on the
product and the oracle) both overwrite every parameter by this function of
(seed, parameter name, shape), so the three models hold identical values
without shipping them.  Shared test infrastructure, no reference code.
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch

GRAD_FULL_MAX = 2048   # gradients up to this many entries are stored whole
GRAD_SAMPLES = 256     # larger ones: this many sampled entries + sum / max


def _gen(seed: int, name: str) -> torch.Generator:
    return torch.Generator().manual_seed(seed * 1_000_003 + zlib.crc32(name.encode()) % 1_000_003)


def fill_params(model: torch.nn.Module, seed: int) -> None:
    """Glorot-uniform matrices, BatchNorm weight U(0.8, 1.2) / bias
    U(-0.1, 0.1), every other vector U(-0.1, 0.1); running statistics reset."""
    bn = set()
    for mname, mod in model.named_modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            for pname, _ in mod.named_parameters(recurse=False):
                bn.add(f"{mname}.{pname}" if mname else pname)
            mod.reset_running_stats()
    with torch.no_grad():
        for name, p in model.named_parameters():
            g = _gen(seed, name)
            u = torch.rand(p.shape, generator=g, dtype=torch.float64)
            if p.dim() >= 2:
                a = math.sqrt(6.0 / (p.shape[-1] + p.shape[-2]))
                v = (2 * u - 1) * a
            elif name in bn and name.endswith("weight"):
                v = 0.8 + 0.4 * u
            else:
                v = (2 * u - 1) * 0.1
            p.copy_(v.to(p.dtype))


def sample_index(name: str, numel: int) -> np.ndarray:
    g = _gen(7, "sample/" + name)
    return torch.randint(0, numel, (GRAD_SAMPLES,), generator=g).numpy()


def grad_record(name: str, grad: torch.Tensor) -> dict:
    """The stored form of one parameter gradient."""
    g = grad.detach().reshape(-1).cpu()
    if g.numel() <= GRAD_FULL_MAX:
        return {f"grad/{name}": g.numpy()}
    idx = sample_index(name, g.numel())
    return {f"gidx/{name}": idx, f"gval/{name}": g[idx].numpy(),
            f"gmax/{name}": np.float64(g.abs().max()),
            f"gsum/{name}": np.float64(g.double().sum())}


def grad_view(g: dict, name: str, grad: torch.Tensor):
    """(stored reference values, the same entries of `grad`, scale): the
    comparison of one parameter gradient against a fixture."""
    flat = grad.detach().reshape(-1).cpu().double()
    if f"grad/{name}" in g:
        ref = torch.from_numpy(np.asarray(g[f"grad/{name}"])).double()
        return ref, flat, max(1.0, float(ref.abs().max()))
    idx = torch.from_numpy(np.asarray(g[f"gidx/{name}"])).long()
    ref = torch.from_numpy(np.asarray(g[f"gval/{name}"])).double()
    return ref, flat[idx], max(1.0, float(g[f"gmax/{name}"]))
