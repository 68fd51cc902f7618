"""Whole-model gradients held to 1e-4 with the ReLU masks frozen (-m gpu).

Why: the heads stack 6-12 dense blocks of batch-statistics BatchNorm + ReLU.
Pre-activations within fp32 rounding of 0 make the HIP path (fp32, MFMA
summation order) and an fp64 evaluation disagree on a few ReLU masks, and a
flipped mask moves deep-layer gradients by up to ~18 % (relative, max-norm;
tests/test_baseline_configs.py measures it as `cond`).  That gate therefore
bounds the HIP gradient by 3x the conditioning.  Here the conditioning is
taken out instead:

  1. the HIP forward runs with hlhgat.nn.TAP on: every ReLU site (fused into a
     conv / BatchNorm / NodeEdgeInt node or not) records its output, so the
     masks the HIP forward actually applied are known (y > 0);
  2. the fp64 oracle (oracle/hodge_ref.py, pinned to the reference by the
     golden fixtures) runs with each nn.ReLU replaced by multiplication with
     the HIP mask of the same module and call;
  3. both backward passes use the same upstream gradient.

In exact arithmetic the two now compute the same function, so every
parameter gradient must match to 1e-4 relative (max|hip - fp64| <=
1e-4 * max(1, max|fp64|)) -- or, where fp32 arithmetic itself cannot reach
that, to 3x the error of the fp32 oracle run with the SAME frozen masks (the
reference's own fp32 rounding floor; small-batch BatchNorm stacks at the
config 3-5 fixtures' 1-2 graphs amplify rounding, not mask flips).  Each
parameter's bound and both errors are written to
gpurun_out/grad_gates/frozen_<case>.json; the tests also print how many
parameters needed the fp32-floor bound.  Biases that feed a training-mode
BatchNorm have an analytically zero gradient and are checked to be noise
(<= 1e-3 of the gradient scale).
"""
import json
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn as tnn

from conftest import REPO, close, load_golden
from oracle import hodge_ref as R

import test_baseline_configs as TB  # noqa: E402  (fixtures' helpers and settings)

sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from baseline_params import fill_params  # noqa: E402

pytestmark = pytest.mark.gpu
T = torch.from_numpy
TOL = 1e-4


class MaskedReLU(tnn.Module):
    """ReLU (or Abs) with the mask (signs) of a recorded forward: x * [y_hip > 0]
    (x * sign(x_hip)), call by call."""

    def __init__(self, masks):
        super().__init__()
        self.masks = masks
        self.i = 0

    def forward(self, x):
        assert self.i < len(self.masks), "more ReLU calls than the HIP forward made"
        m = self.masks[self.i]
        self.i += 1
        assert tuple(m.shape) == tuple(x.shape), (m.shape, x.shape)
        return x * m.to(x.dtype)


def _run_tapped(fn):
    from hlhgat import nn as hnn
    hnn.TAP = {}
    try:
        out = fn()
        taps = hnn.TAP
    finally:
        hnn.TAP = None
    return out, taps


def _freeze(ref, m_hip, taps):
    """Replace every nn.ReLU of the oracle `ref` by the HIP forward's masks,
    and every Abs (the TSP readout's |B1^T x_t|, lib/Hodge_ST_Model.py:848) by
    multiplication with the signs of the HIP forward's input: sign flips of
    values within rounding of 0 are the same non-smooth points as ReLU's."""
    names = {id(mod): n for n, mod in m_hip.named_modules()}
    raw = {names[id(mod)]: ys for mod, ys in taps.items()}
    masked = []
    for name, mod in list(ref.named_modules()):
        if isinstance(mod, tnn.ReLU):
            assert name in raw, f"HIP forward recorded no ReLU output for {name}"
            mm = MaskedReLU([(y > 0).cpu() for y in raw[name]])
        elif isinstance(mod, R.Abs):
            assert name in raw, f"HIP forward recorded no Abs input for {name}"
            mm = MaskedReLU([torch.sign(y).cpu() for y in raw[name]])
        else:
            continue
        parent = ref.get_submodule(name.rsplit(".", 1)[0]) if "." in name else ref
        setattr(parent, name.rsplit(".", 1)[-1], mm)
        masked.append(mm)
    return masked


def _check(case, m_hip, ref64, masked, ref32=None, cond=None):
    for mm in masked:
        assert mm.i == len(mm.masks), "fewer ReLU calls than the HIP forward made"
    p64 = dict(ref64.named_parameters())
    p32 = dict(ref32.named_parameters()) if ref32 is not None else {}
    rows, bad = [], []
    for k, p in m_hip.named_parameters():
        e = p64[k].grad
        if p.grad is None or e is None:
            assert (p.grad is None or float(p.grad.abs().max()) == 0.0) and \
                (e is None or float(e.abs().max()) == 0.0), k
            continue
        scale = max(1.0, float(e.abs().max()))
        err = float((p.grad.detach().cpu().double() - e).abs().max()) / scale
        if TB._bn_fed_bias(k):
            # analytically zero: noise no larger than 3x the fp32 oracle's (frozen masks)
            noise32 = float(p32[k].grad.abs().max()) / scale if k in p32 else 0.0
            nb = max(1e-3, 3 * noise32)
            rows.append({"param": k, "err": err, "bound": nb, "kind": "bn-fed bias (noise)"})
            if err > nb:
                bad.append((k, err, noise32))
            continue
        err32 = (float((p32[k].grad.double() - e).abs().max()) / scale) if k in p32 else 0.0
        # the fp64 conditioning probe is logged, not gated: the
        # bound is 1e-4 or 3x the fp32 oracle's own error with the same masks
        c = (cond or {}).get(k, 0.0)
        bound = max(TOL, 3 * err32)
        floor = "1e-4" if bound == TOL else "3x fp32 (frozen)"
        rows.append({"param": k, "err": err, "bound": bound, "err_fp32_frozen": err32,
                     "cond_fp64_frozen": c, "scale": scale, "floor": floor})
        if err > bound:
            bad.append((k, err, err32))
    out_dir = os.path.join(REPO, "gpurun_out", "grad_gates")
    os.makedirs(out_dir, exist_ok=True)
    tight = [r for r in rows if "err_fp32_frozen" in r]
    n_floor = sum(r["floor"] != "1e-4" for r in tight)
    n_cond = sum(r["cond_fp64_frozen"] > r["err_fp32_frozen"] for r in tight)
    worst = max((r["err"], r["param"]) for r in tight)
    worst32 = max(r["err_fp32_frozen"] for r in tight)
    with open(os.path.join(out_dir, f"frozen_{case}.json"), "w") as f:
        json.dump({"case": case, "tol": TOL, "n_masks": sum(len(m.masks) for m in masked),
                   "worst_hip": worst[0], "worst_fp32_oracle_frozen": worst32,
                   "params_at_fp32_floor": n_floor,
                   "params_where_fp64_conditioning_exceeds_fp32_error": n_cond,
                   "params": rows}, f, indent=1)
    print(f"[frozen-mask] {case}: {len(tight)} params, worst HIP {worst[0]:.2e} ({worst[1]}), "
          f"worst fp32 oracle {worst32:.2e}; {n_floor} params bounded by the fp32 floor")
    assert not bad, bad


def _d64(b):
    d = TB._D()
    for k in TB.KEYS:
        v = getattr(b, k)
        setattr(d, k, v.double() if torch.is_tensor(v) and v.is_floating_point() else v)
    return d


@pytest.mark.parametrize("case,kw", [
    # config 1 at its exact hyperparameters (main_zinc_HL_HGCNN_dense_int3_pyr.py:151-177):
    # one level of 2 blocks
    ("cfg1_zinc_200", dict(channels=[2], filters=[64], mlp_channels=[256, 256], K=3, keig=15)),
    ("cfg2_zinc_200", dict(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256],
                           K=3, keig=15))])
def test_frozen_mask_grads_zinc_200(cuda, case, kw):
    """Configs 1 (2 blocks) and 2 (6 blocks), K=3 d=64, mlp [256, 256], on 200
    ZINC-like graphs."""
    import hlhgat
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(200, seed=21)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**kw)
    ref64 = R.RefZincModel(**kw).double()
    ref64.load_state_dict({k: v.double() if v.is_floating_point() else v
                           for k, v in m.state_dict().items()})
    ref32 = R.RefZincModel(**kw)
    ref32.load_state_dict(m.state_dict())
    m = m.to(cuda).train()
    bd = zinc_like_batch(200, seed=21).to(cuda)
    out, taps = _run_tapped(lambda: m(bd))
    Rg = torch.randn(out.shape, generator=torch.Generator().manual_seed(5))
    (out * Rg.to(cuda)).sum().backward()
    masked = _freeze(ref64, m, taps)
    out64 = ref64.train()(_d64(b))
    close(out.detach().cpu(), out64.detach(), 1e-4, "out vs fp64 oracle (frozen masks)")
    (out64 * Rg.double()).sum().backward()
    _freeze(ref32, m, taps)
    (ref32.train()(b) * Rg).sum().backward()
    _check(case, m, ref64, masked, ref32)


@pytest.mark.parametrize("name,factored", [("baseline_cfg3_cifar", False),
                                           ("baseline_cfg3_cifar", True),
                                           ("baseline_cfg4_pepfunc", False),
                                           ("baseline_cfg5_tsp", False),
                                           ("baseline_cfg5_tsp", True)])
def test_frozen_mask_grads_heads_at_baseline(cuda, name, factored):
    """Configs 3 / 4 / 5 at their own hyperparameters on the reference
    fixtures' inputs (tests/golden/make_golden_baseline.py)."""
    import hlhgat
    from hlhgat import ops
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g = load_golden(name)
    cls_ref, cls_name, kw = TB.HEADS[name]
    m = getattr(hlhgat, cls_name)(**kw)
    fill_params(m, int(g["seed"]))
    m = m.to(cuda).train()
    ops.clear_caches()
    if "tsp" in name:
        b = TB._product_batch(g, "", cuda, factored)
        (out, _), taps = _run_tapped(lambda: m(b))
    else:
        datas = [TB._product_batch(g, "l0/", cuda, factored),
                 TB._product_batch(g, "l1/", cuda, False)]
        out, taps = _run_tapped(lambda: m(datas))
    (out * T(g["R"]).to(cuda)).sum().backward()
    ref64 = getattr(R, cls_ref)(**kw)
    fill_params(ref64, int(g["seed"]))
    ref64 = ref64.double().train()
    masked = _freeze(ref64, m, taps)
    ref32 = getattr(R, cls_ref)(**kw)
    fill_params(ref32, int(g["seed"]))
    ref32.train()
    _freeze(ref32, m, taps)
    outs = []
    for ref, dt in ((ref64, torch.float64), (ref32, torch.float32)):
        if "tsp" in name:
            o, _ = ref(TB._data(g, "", dt))
        else:
            o = ref([TB._data(g, "l0/", dt), TB._data(g, "l1/", dt)])
        (o * T(g["R"]).to(dt)).sum().backward()
        outs.append(o)
    close(out.detach().cpu(), outs[0].detach(), 1e-4, "out vs fp64 oracle (frozen masks)")
    _check(f"{name}{'_factored' if factored else ''}", m, ref64, masked, ref32)
    ops.check_device_errors()


def _realistic(kind):
    """Realistic per-GPU batches (verdict r3): 16 CIFAR superpixel graphs, 16
    peptides, 4 TSP graphs of 2500 nodes -- at these sizes every BatchNorm
    normalises over thousands of rows, as at the configs' own batch sizes.
    Built from the deterministic synthetic generators (seeded), collated with
    the same host code as the fixtures (the oracle itself is pinned to the
    reference by the small fixtures, tests/test_baseline_configs.py)."""
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import cifar_like_graphs, peptides_like_graphs, tsp_like_graph
    if kind == "tsp":
        return collate([tsp_like_graph(910 + s, n=2500, k=9, row_order=False)
                        for s in range(4)], check_hodge=False)
    make = cifar_like_graphs if kind == "cifar" else peptides_like_graphs
    pairs = [make(900 + s) for s in range(16)]
    return [collate([p[0] for p in pairs], check_hodge=False),
            collate([p[1] for p in pairs], check_hodge=False)]


def _as_d(b, dtype):
    d = TB._D()
    for k in TB.KEYS:
        v = torch.as_tensor(getattr(b, k))
        setattr(d, k, v.to(dtype) if v.is_floating_point() else v)
    return d


def _to_dev(b, cuda, factored):
    import copy
    from hlhgat import ops
    bd = copy.copy(b)  # Batch.to moves in place: keep the host batch for the oracle
    # Batch.to declares the Hodge factor of L1 whenever collate set l1_factor:
    # the CSR variant must not carry that flag (the _csr case had
    # silently run the factored path)
    bd.l1_factor = bool(factored) and bool(getattr(b, "l1_factor", False))
    bd = bd.to(cuda)
    ops.mark_hodge(bd.edge_index_t)
    ops.mark_hodge(bd.edge_index_s)
    if factored:
        ops.set_hodge_factor(bd.edge_index_s, bd.edge_index, bd.x_t.shape[0])
    assert ops.has_hodge_factor(bd.edge_index_s) == bool(factored)
    return bd


_HIP_GRADS = {}  # case -> HIP parameter gradients (the CSR / factored pair compared)


@pytest.mark.parametrize("name,kind,factored", [("cfg3_cifar_16", "cifar", True),
                                                ("cfg4_pepfunc_16", "peptides", False),
                                                ("cfg5_tsp_4x2500", "tsp", True),
                                                ("cfg5_tsp_4x2500_csr", "tsp", False)])
def test_frozen_mask_grads_heads_realistic_batches(cuda, name, kind, factored):
    """Configs 3 / 4 / 5 at their own hyperparameters on realistic batches:
    every parameter gradient within 1e-4 of the fp64 oracle (frozen masks),
    or within 3x the fp32 oracle's own error where that is larger (each such
    parameter named in the gate log with its fp32 error).  TSP (12 blocks of
    batch-statistics BatchNorm over 10k nodes / 52k edges) is ill-conditioned
    in fp32 itself (the fp32 oracle is up to ~1e-2 from fp64); the fp64
    gradient's own change under two 1e-6 relative parameter perturbations
    WITH THE SAME frozen masks (a conditioning probe with no mask flip) is
    logged per parameter for information, not used in the bound."""
    import hlhgat
    from hlhgat import ops
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    key = {"cifar": "baseline_cfg3_cifar", "peptides": "baseline_cfg4_pepfunc",
           "tsp": "baseline_cfg5_tsp"}[kind]
    cls_ref, cls_name, kw = TB.HEADS[key]
    seed = 41
    raw = _realistic(kind)
    m = getattr(hlhgat, cls_name)(**kw)
    fill_params(m, seed)
    m = m.to(cuda).train()
    ops.clear_caches()
    if kind == "tsp":
        b = _to_dev(raw, cuda, factored)
        (out, _), taps = _run_tapped(lambda: m(b))
    else:
        datas = [_to_dev(raw[0], cuda, factored), _to_dev(raw[1], cuda, False)]
        out, taps = _run_tapped(lambda: m(datas))
    Rg = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed))
    (out * Rg.to(cuda)).sum().backward()
    ref64 = getattr(R, cls_ref)(**kw)
    fill_params(ref64, seed)
    ref64 = ref64.double().train()
    masked = _freeze(ref64, m, taps)
    ref32 = getattr(R, cls_ref)(**kw)
    fill_params(ref32, seed)
    ref32.train()
    _freeze(ref32, m, taps)
    outs = []
    for ref, dt in ((ref64, torch.float64), (ref32, torch.float32)):
        if kind == "tsp":
            o, _ = ref(_as_d(raw, dt))
        else:
            o = ref([_as_d(raw[0], dt), _as_d(raw[1], dt)])
        (o * Rg.to(dt)).sum().backward()
        outs.append(o)
    close(out.detach().cpu(), outs[0].detach(), 1e-4, "out vs fp64 oracle (frozen masks)")
    cond = None
    if kind == "tsp":
        cond = {}
        base = dict(ref64.named_parameters())
        for ps in (0, 1):
            rp = getattr(R, cls_ref)(**kw)
            fill_params(rp, seed)
            rp = rp.double().train()
            TB._perturb(rp, 1e-6, ps)
            _freeze(rp, m, taps)
            o, _ = rp(_as_d(raw, torch.float64))
            (o * Rg.double()).sum().backward()
            for k, p in rp.named_parameters():
                if p.grad is None or base[k].grad is None:
                    continue
                sc = max(1.0, float(base[k].grad.abs().max()))
                cond[k] = max(cond.get(k, 0.0), float((p.grad - base[k].grad).abs().max()) / sc)
    _HIP_GRADS[name] = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()
                        if p.grad is not None}
    if name == "cfg5_tsp_4x2500_csr" and "cfg5_tsp_4x2500" in _HIP_GRADS:
        # the two variants run different kernels (CSR SpMM vs the factored L1,
        # not bitwise the same arithmetic): their gradients must differ
        other = _HIP_GRADS["cfg5_tsp_4x2500"]
        assert any(not torch.equal(v, other[k]) for k, v in _HIP_GRADS[name].items())
    _check(name, m, ref64, masked, ref32, cond)
    ops.check_device_errors()


@pytest.mark.parametrize("factored", [True, False])
def test_one_block_gate_cfg5_widths(cuda, factored):
    """One dense HL block at config-5 widths (d=128, K=4; Laguerre conv on L0
    and L1, BatchNorm, ReLU -- lib/Hodge_ST_Model.py:22-34 HL_block) on 4 TSP
    graphs of 2500 nodes, against the fp64 oracle (oracle/hodge_ref.py
    _ref_block) with the HIP forward's ReLU masks frozen.  One block has no
    depth to amplify rounding, so this isolates the kernels' own error from the
    12-block model's conditioning: every parameter and input
    gradient within 1e-5 of fp64 (max|hip - fp64| <= 1e-5 * max(1, max|fp64|)),
    the fp32 oracle's own error logged beside it."""
    from hlhgat import ops
    from hlhgat.hodge_st_model import _hl_block
    tol = 1e-5
    raw = _realistic("tsp")
    n0, n1 = raw.x_t.shape[0], raw.x_s.shape[0]
    d, K = 128, 4
    gen = torch.Generator().manual_seed(7)
    xt = torch.randn(n0, d, generator=gen)
    xs = torch.randn(n1, d, generator=gen)
    Rt = torch.randn(n0, d, generator=gen)
    Rs = torch.randn(n1, d, generator=gen)
    torch.manual_seed(3)
    blk = _hl_block(d, d, d, K, 0.0)
    for mod in blk.modules():  # non-trivial affine BatchNorm parameters
        if isinstance(mod, tnn.BatchNorm1d):
            with torch.no_grad():
                mod.weight.uniform_(0.5, 1.5, generator=gen)
                mod.bias.uniform_(-0.5, 0.5, generator=gen)
    sd = blk.state_dict()
    blk = blk.to(cuda).train()
    ops.clear_caches()
    bd = _to_dev(raw, cuda, factored)
    xt_d = xt.to(cuda).requires_grad_(True)
    xs_d = xs.to(cuda).requires_grad_(True)
    (ot, os_), taps = _run_tapped(lambda: blk(xt_d, bd.edge_index_t, bd.edge_weight_t, xs_d,
                                              bd.edge_index_s, bd.edge_weight_s))
    ((ot * Rt.to(cuda)).sum() + (os_ * Rs.to(cuda)).sum()).backward()
    torch.cuda.synchronize()
    errs = {}
    for dt in (torch.float64, torch.float32):
        ref = R._ref_block(d, d, d, K, 0.0)
        ref.load_state_dict({k: v.to(dt) if v.is_floating_point() else v for k, v in sd.items()})
        ref = ref.to(dt).train()
        _freeze(ref, blk, taps)
        a = _as_d(raw, dt)
        xr, sr = xt.to(dt).requires_grad_(True), xs.to(dt).requires_grad_(True)
        rt, rs = ref(xr, a.edge_index_t, a.edge_weight_t, sr, a.edge_index_s, a.edge_weight_s)
        ((rt * Rt.to(dt)).sum() + (rs * Rs.to(dt)).sum()).backward()
        grads = {k: p.grad for k, p in ref.named_parameters()}
        grads.update({"input.x_t": xr.grad, "input.x_s": sr.grad})
        if dt == torch.float64:
            g64, o64 = grads, (rt.detach(), rs.detach())
            close(ot.detach().cpu(), o64[0], tol, "x_t out vs fp64")
            close(os_.detach().cpu(), o64[1], tol, "x_s out vs fp64")
        else:
            g32 = grads
    hip = {k: p.grad for k, p in blk.named_parameters()}
    hip.update({"input.x_t": xt_d.grad, "input.x_s": xs_d.grad})
    rows, bad = [], []
    for k, e in g64.items():
        h = hip[k]
        scale = max(1.0, float(e.abs().max()))
        err = float((h.detach().cpu().double() - e).abs().max()) / scale
        err32 = float((g32[k].double() - e).abs().max()) / scale
        if TB._bn_fed_bias(k):  # analytically zero (bias before a training BatchNorm):
            # noise no larger than 3x the fp32 oracle's, as in _check
            noise32 = float(g32[k].abs().max()) / scale
            nb = max(1e-3, 3 * noise32)
            rows.append({"param": k, "err": err, "bound": nb, "kind": "bn-fed bias (noise)"})
            if err > nb:
                bad.append((k, err, err32))
            continue
        rows.append({"param": k, "err": err, "err_fp32_oracle": err32, "bound": tol,
                     "scale": scale})
        if err > tol:
            bad.append((k, err, err32))
    case = f"one_block_cfg5_{'factored' if factored else 'csr'}"
    out_dir = os.path.join(REPO, "gpurun_out", "grad_gates")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, f"{case}.json"), "w") as f:
        json.dump({"case": case, "tol": tol, "params": rows}, f, indent=1)
    worst = max((r["err"], r["param"]) for r in rows if "err_fp32_oracle" in r)
    worst32 = max(r["err_fp32_oracle"] for r in rows if "err_fp32_oracle" in r)
    print(f"[one-block] {case}: worst HIP {worst[0]:.2e} ({worst[1]}), worst fp32 oracle "
          f"{worst32:.2e}")
    assert ops.has_hodge_factor(bd.edge_index_s) == factored
    assert not bad, bad
    ops.check_device_errors()
