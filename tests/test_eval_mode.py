"""Evaluation mode: model.eval() under torch.no_grad() (the reference's test()
loop, main_zinc_HL_HGCNN_dense_int3_pyr.py:165-177; main_pepfunc...:171-225).

Fixtures: tests/golden/make_golden_eval.py ran the REFERENCE's heads (config 2
ZINC, config 3 CIFAR attpool, config 4 peptides attpool, config 5 TSP) with
baseline_params.fill_params parameters: a few training-mode forwards under
no_grad (running statistics move, momentum 0.1), then eval() + no_grad.  They
hold every BatchNorm buffer after the training passes and the eval output.

* CPU: the oracle reproduces buffers (1e-6) and eval outputs (1e-5).
* GPU: the HIP heads
  - update the running statistics in their training passes like the
    reference: running_mean / running_var within 1e-5 relative (max-norm,
    scale max(1, max|ref|)), num_batches_tracked exact;
  - with the reference's buffers loaded, give the reference's eval output
    within 1e-5 relative.
"""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, close, load_golden
from oracle import hodge_ref as R

sys.path.insert(0, GOLDEN)
from baseline_params import fill_params  # noqa: E402

T = torch.from_numpy
KEYS = ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
        "edge_index", "num_node1", "num_edge1")
CFG2 = dict(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256], K=3, keig=15)
CFG3 = dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256], K=4, keig=10,
            pool_loc=1, l=0.5)
CFG4 = dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256], K=6, pool_loc=1)
CFG5 = dict(channels=[4, 4, 4], filters=[32, 64, 128], mlp_channels=[256], K=4)
# fixture -> (oracle class, product class, kwargs, inputs fixture)
CASES = {"eval_cfg2_zinc": ("RefZincModel", "HL_HGCNN_zinc_dense_int3_pyr", CFG2, None),
         "eval_cfg3_cifar": ("RefCifarAttPool", "HL_HGCNN_CIFAR10SP_dense_int3_attpool", CFG3,
                             "baseline_cfg3_cifar"),
         "eval_cfg4_pepfunc": ("RefPepfuncAttPool", "HL_HGCNN_pepfunc_dense_int3_attpool", CFG4,
                               "baseline_cfg4_pepfunc"),
         "eval_cfg5_tsp": ("RefTSPModel", "HL_HGCNN_TSP_dense_int3_pyr", CFG5, "baseline_cfg5_tsp")}


class _D:
    pass


def _oracle_data(g, prefix):
    d = _D()
    for k in KEYS:
        setattr(d, k, T(g[prefix + k]))
    return d


def _product_data(g, prefix, cuda):
    from hlhgat import ops
    from hlhgat.hodge_dataset import Batch
    b = Batch()
    for k in KEYS:
        setattr(b, k, T(g[prefix + k]).to(cuda))
    ops.mark_hodge(b.edge_index_t)  # fixture COO: collate(check_hodge=True) output
    ops.mark_hodge(b.edge_index_s)
    return b


def _inputs(name, make):
    """(training-pass inputs, eval inputs) in the model's call form."""
    g = load_golden(name)
    src = CASES[name][3]
    if src is None:  # ZINC: stored batches
        train = [make(g, f"train{i}/") for i in range(int(g["n_train"]))]
        return g, train, make(g, "eval/")
    gi = load_golden(src)
    if "tsp" in name:
        d = make(gi, "")
    else:
        d = [make(gi, "l0/"), make(gi, "l1/")]
    return g, [d] * int(g["n_train"]), d


def _call(m, d):
    out = m(d)
    return out[0] if isinstance(out, tuple) else out


def _buffers(m):
    return {k: v for k, v in m.state_dict().items()
            if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_eval_matches_reference(name):
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        g, train, ev = _inputs(name, _oracle_data)
        m = getattr(R, CASES[name][0])(**CASES[name][2])
        fill_params(m, int(g["seed"]))
        m.train()
        with torch.no_grad():
            for d in train:
                _call(m, d)
        bufs = _buffers(m)
        assert len(bufs) == sum(1 for k in g if k.startswith("buf/")) > 10
        for k, v in bufs.items():
            close(v, g["buf/" + k], 1e-6, k)
        m.eval()
        with torch.no_grad():
            out = _call(m, ev)
    finally:
        torch.set_num_threads(nt)
    close(out, g["out"], 1e-5, "eval out")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_hip_eval_matches_reference(cuda, name):
    import hlhgat
    from hlhgat import ops
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ops.clear_caches()
    g, train, ev = _inputs(name, lambda gg, p: _product_data(gg, p, cuda))
    m = getattr(hlhgat, CASES[name][1])(**CASES[name][2])
    fill_params(m, int(g["seed"]))
    m = m.to(cuda).train()
    # training passes on the HIP path move the running statistics like the reference's
    with torch.no_grad():
        for d in train:
            _call(m, d)
    bufs = _buffers(m)
    assert len(bufs) == sum(1 for k in g if k.startswith("buf/")) > 10
    worst = 0.0
    for k, v in bufs.items():
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(g["buf/" + k]), k
        else:
            worst = max(worst, close(v.cpu(), g["buf/" + k], 1e-5, k))
    # eval with the reference's buffers: the running-statistics route alone
    m.load_state_dict({k: T(np.asarray(g["buf/" + k])) for k in bufs}, strict=False)
    m.eval()
    with torch.no_grad():
        out = _call(m, ev)
    err = close(out.cpu(), g["out"], 1e-5, "eval out")
    ops.check_device_errors()
    print(f"[eval] {name}: running stats max err {worst:.2e}, eval out max err {err:.2e}")


@pytest.mark.gpu
def test_eval_chains_bitwise_one_stream(cuda):
    """Eval mode with the node / edge chains on two streams (ops.Chains):
    BatchNorm on running statistics does not write into the dense slab's sink,
    so DenseConcat copies each edge block; the copy runs on the edge chain
    (where the block was produced).  Outputs equal the one-stream run bit for
    bit, repeated with the allocator churned between runs."""
    import hlhgat
    from hlhgat import ops
    g, train, ev = _inputs("eval_cfg2_zinc", lambda gg, p: _product_data(gg, p, cuda))
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**CASES["eval_cfg2_zinc"][2])
    fill_params(m, int(g["seed"]))
    m = m.to(cuda).eval()
    outs = {}
    prev = ops.CHAINS_ENABLED
    try:
        for on in (False, True, True):
            ops.CHAINS_ENABLED = on
            ops.clear_caches()
            with torch.no_grad():
                junk = [torch.full((1 << 20,), float(i), device=cuda) for i in range(8)]
                del junk  # freed main-stream blocks, reused by the next forward
                outs.setdefault(on, []).append(_call(m, ev).cpu())
    finally:
        ops.CHAINS_ENABLED = prev
    torch.cuda.synchronize()
    for o in outs[True]:
        assert torch.equal(o, outs[False][0])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["eval_cfg2_zinc", "eval_cfg4_pepfunc"])
def test_infer_step_replay_matches_eager_and_reference(cuda, name):
    """hlhgat.train.InferStep (the reference's test() loop body, captured per
    batch shape and replayed): replayed outputs equal the eager eval forward
    bit for bit, and the reference's eval output within 1e-5."""
    import hlhgat
    from hlhgat.train import InferStep
    g, _, ev = _inputs(name, lambda gg, p: _product_data(gg, p, cuda))
    bufs = {k[4:]: T(np.asarray(g[k])) for k in g if k.startswith("buf/")}
    m = getattr(hlhgat, CASES[name][1])(**CASES[name][2])
    fill_params(m, int(g["seed"]))
    m.load_state_dict(bufs, strict=False)
    m = m.to(cuda).train()
    inf = InferStep(m)
    outs = [_call_out(inf(ev)).clone() for _ in range(4)]
    torch.cuda.synchronize()
    assert inf.stats["captures"] == 1 and inf.stats["replay"] == 3, inf.stats
    assert m.training  # InferStep restores the mode it found
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    close(outs[0].cpu(), g["out"], 1e-5, "eval out (InferStep)")


def _call_out(out):
    return out[0] if isinstance(out, tuple) else out


@pytest.mark.gpu
def test_infer_step_padded_batch_equals_unpadded(cuda):
    """Eval on a static-shape (padded) batch: the NodeEdgeInt value path runs
    unfused in eval mode (BatchNorm on running statistics is row-wise, so the
    padding rows change nothing); InferStep's replayed outputs on the padded
    batch equal the eager eval forward on the unpadded one."""
    import hlhgat
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    from hlhgat.train import InferStep
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**CFG2)
    m = m.to(cuda).train()
    with torch.no_grad():  # move the running statistics off their initial values
        for s in (1, 2):
            m(zinc_like_batch(60, seed=s).to(cuda))
    raw = zinc_like_batch(50, seed=7)
    padded = pad_batch(raw, static_caps(raw, 512))
    m.eval()
    with torch.no_grad():
        ref = m(zinc_like_batch(50, seed=7).to(cuda)).cpu()
    m.train()
    inf = InferStep(m)
    pb = padded.to(cuda)
    outs = [inf(pb).clone().cpu() for _ in range(3)]
    assert inf.stats["replay"] == 2, inf.stats
    for o in outs:
        assert o.shape == ref.shape
        close(o, ref.numpy(), 1e-5, "padded eval vs unpadded")


@pytest.mark.gpu
@pytest.mark.parametrize("n,C,relu,affine", [(23157, 64, True, True), (4097, 6, False, True),
                                             (1000, 256, True, False), (700, 128, False, False)])
def test_eval_batch_norm_hip_matches_torch(cuda, n, C, relu, affine):
    """Eval-mode BatchNorm (+ ReLU) in inference runs in one HIP launch from
    the running statistics (hlhgat_bn_apply_running; unaligned C takes the
    scalar path) and equals torch's eval batch_norm (+ relu) to 1e-6; with
    gradients wanted it stays on ATen's autograd (same values)."""
    from hlhgat import ops
    torch.manual_seed(n + C)
    bn = torch.nn.BatchNorm1d(C, affine=affine).to(cuda)
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.2, 3.0)
        if affine:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
    bn.eval()
    x = torch.randn(n, C, device=cuda) * 2 + 0.3
    with torch.no_grad():
        ref = torch.nn.functional.batch_norm(x, bn.running_mean, bn.running_var, bn.weight,
                                             bn.bias, False, 0.0, bn.eps)
        if relu:
            ref = torch.relu(ref)
    with torch.no_grad():
        y = ops.batch_norm_act(x, bn, relu=relu)
    torch.cuda.synchronize()
    ops.check_device_errors()
    close(y.cpu(), ref.cpu(), 1e-6, "eval bn")
    xg = x.clone().requires_grad_(True)
    yg = ops.batch_norm_act(xg, bn, relu=relu)  # differentiated: ATen's path
    yg.sum().backward()
    close(yg.detach().cpu(), ref.cpu(), 1e-6, "eval bn (autograd path)")
    assert xg.grad is not None
