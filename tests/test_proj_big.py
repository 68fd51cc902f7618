"""Large-tile projection kernels (csrc/proj_big.h) against an fp64 reference
and against the 64x64-tile kernels they replace at the config 3-5 shapes
(-m gpu).

The projections are the Linear layers of HodgeLaguerreConv (sum_k lins[k](T_k)
+ bias, lib/Hodge_Cheb_Conv.py:487-513) and NodeEdgeInt (Linear(cat[a, b]),
:307-308); their torch fp32 reference is F.linear.  Both kernel families are
fp32 MFMA chains in different orders, so the gate is: the large-tile result's
error against fp64 is at most 2x the small-tile family's own error on the same
data (plus an absolute floor of 1e-6 of the products' magnitude |A| |W|^T),
for every output of the forward, the data gradient and the weight / bias
gradients -- ragged M, reduction widths that are not multiples of the 32-wide
LDS stage, N = 32 / 64 / 96 / 128 / 256, several operand blocks, accumulate.
hlhgat_set_gemm_big(1) forces the large tiles at these small sizes;
hlhgat_set_gemm_big(0) forces the small ones.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # M, N, reduction widths of the blocks
    (1000, 128, [128, 128, 128, 128]),
    (777, 64, [36, 100]),
    (3001, 32, [64, 64, 64]),
    (513, 256, [448, 448]),
    (4099, 96, [52]),
    (2500, 128, [800, 800]),
]


def _mode(mode):
    from hlhgat import _lib
    _lib.check(_lib.LIB.hlhgat_set_gemm_big(mode, 0), "set_gemm_big")


@pytest.fixture(autouse=True)
def _restore_mode():
    yield
    _mode(-1)


def _data(M, N, kbs, seed):
    g = torch.Generator().manual_seed(seed)
    As = [torch.randn(M, k, generator=g) for k in kbs]
    W = torch.randn(N, sum(kbs), generator=g) / sum(kbs) ** 0.5
    bias = torch.randn(N, generator=g)
    G = torch.randn(M, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    return As, W, bias, G, C0


def _split(W, kbs):
    out, o = [], 0
    for k in kbs:
        out.append(W[:, o:o + k])
        o += k
    return out


def _err(x, ref, mag):
    return float(((x.double().cpu() - ref).abs() - 1e-6 * mag).max())


def _run(cuda, mode, As, W, bias, G, C0, kbs):
    from hlhgat import ops
    _mode(mode)
    M, N = G.shape
    Ad = [a.to(cuda) for a in As]
    Wd = W.to(cuda)
    Ws = _split(Wd, kbs)
    out = torch.empty(M, N, device=cuda)
    ops._proj_fwd(Ad, Ws, M, N, bias.to(cuda), out)
    acc = C0.to(cuda).clone()
    ops._proj_fwd(Ad, Ws, M, N, None, acc, accumulate=True)
    Gd = G.to(cuda)
    dAs = [torch.empty(M, k, device=cuda) for k in kbs]
    ops._proj_bwd_data(Gd, Ws, kbs, dAs)
    dW = torch.empty_like(Wd)
    db = torch.empty(N, device=cuda)
    ops._proj_bwd_weight(Gd, Ad, _split(dW, kbs), db)
    # the fused autograd path (hlhgat_proj_bwd: weight + data in one call)
    Ar = [a.clone().requires_grad_(True) for a in Ad]
    Wr = Wd.clone().requires_grad_(True)
    br = bias.to(cuda).clone().requires_grad_(True)
    y = ops.linear_blocks(Ar, Wr, br)
    y.backward(Gd)
    torch.cuda.synchronize()
    ops.check_device_errors()
    return dict(out=out.cpu(), acc=acc.cpu(), dA=[d.cpu() for d in dAs], dW=dW.cpu(),
                db=db.cpu(), y=y.detach().cpu(), fdA=[a.grad.cpu() for a in Ar],
                fdW=Wr.grad.cpu(), fdb=br.grad.cpu())


@pytest.mark.parametrize("M,N,kbs", SHAPES)
def test_large_tiles_vs_fp64_and_small_tiles(cuda, M, N, kbs):
    As, W, bias, G, C0 = _data(M, N, kbs, seed=M + N)
    A64 = torch.cat(As, 1).double()
    W64, G64 = W.double(), G.double()
    ref = dict(out=A64 @ W64.t() + bias.double(), acc=C0.double() + A64 @ W64.t(),
               dA=list((G64 @ W64).split(kbs, 1)), dW=G64.t() @ A64, db=G64.sum(0))
    mag = dict(out=A64.abs() @ W64.abs().t(), dA=list((G64.abs() @ W64.abs()).split(kbs, 1)),
               dW=G64.abs().t() @ A64.abs(), db=G64.abs().sum(0))
    mag["acc"] = mag["out"]
    small = _run(cuda, 0, As, W, bias, G, C0, kbs)
    big = _run(cuda, 1, As, W, bias, G, C0, kbs)
    rows = []
    for k in ("out", "acc", "dW", "db"):
        eb, es = _err(big[k], ref[k], mag[k]), _err(small[k], ref[k], mag[k])
        rows.append((k, eb, es))
        assert eb <= max(2 * es, 0.0), (k, eb, es)
    for b in range(len(kbs)):
        eb, es = _err(big["dA"][b], ref["dA"][b], mag["dA"][b]), \
            _err(small["dA"][b], ref["dA"][b], mag["dA"][b])
        rows.append((f"dA{b}", eb, es))
        assert eb <= max(2 * es, 0.0), (b, eb, es)
    # the fused autograd path runs the same large-tile kernels: the same bits
    assert torch.equal(big["y"], big["out"])
    assert torch.equal(big["fdW"], big["dW"]) and torch.equal(big["fdb"], big["db"])
    for x, y in zip(big["fdA"], big["dA"]):
        assert torch.equal(x, y)
    print(f"[large tiles] M={M} N={N} kb={kbs}: " +
          ", ".join(f"{k} {eb:.1e}/{es:.1e}" for k, eb, es in rows))


def test_large_tiles_auto_by_shape(cuda):
    """Mode -1 picks the large-tile forward for config-5 edge rows (M >= 65538,
    N >= 128, a reduction >= 224): the result is bitwise the forced-large one,
    and differs from the small tiles."""
    from hlhgat import ops
    M, N, kbs = 131072, 128, [128] * 4
    As, W, bias, G, C0 = _data(M, N, kbs, seed=5)
    Ad = [a.to(cuda) for a in As]
    Ws = _split(W.to(cuda), kbs)
    outs = {}
    for mode in (-1, 1, 0):
        _mode(mode)
        out = torch.empty(M, N, device=cuda)
        ops._proj_fwd(Ad, Ws, M, N, None, out)
        outs[mode] = out.cpu()
    assert torch.equal(outs[-1], outs[1])
    assert not torch.equal(outs[1], outs[0])


def test_mixed_large_weight_small_data_fused_equals_separate(cuda):
    """Mode -1 at a config-5 conv shape where the rules differ per part (weight
    gradient large tiles, data gradient small, M = 131072, N = 64, K = 4 x 64):
    the fused backward (one hlhgat_proj_bwd call) gives the bits of the
    separate weight / data calls."""
    from hlhgat import ops
    _mode(-1)
    M, N, kbs = 131072, 64, [64] * 4
    As, W, bias, G, _ = _data(M, N, kbs, seed=9)
    Ad = [a.to(cuda) for a in As]
    Wd = W.to(cuda)
    Gd = G.to(cuda)
    dAs = [torch.empty(M, k, device=cuda) for k in kbs]
    ops._proj_bwd_data(Gd, _split(Wd, kbs), kbs, dAs)
    dW = torch.empty_like(Wd)
    db = torch.empty(N, device=cuda)
    ops._proj_bwd_weight(Gd, Ad, _split(dW, kbs), db)
    Ar = [a.clone().requires_grad_(True) for a in Ad]
    Wr = Wd.clone().requires_grad_(True)
    br = bias.to(cuda).clone().requires_grad_(True)
    ops.linear_blocks(Ar, Wr, br).backward(Gd)
    torch.cuda.synchronize()
    assert torch.equal(Wr.grad, dW) and torch.equal(br.grad, db)
    for x, y in zip(Ar, dAs):
        assert torch.equal(x.grad, y)
    ops.check_device_errors()
