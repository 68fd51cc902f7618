"""torch.ops.hlhgat: the dispatcher-registered op boundary.

CPU: every schema is registered, the Meta kernels give the right shapes, and
autograd runs through the Meta kernels (what FakeTensor / torch.compile
tracing exercises).  GPU: each op equals the C-ABI path it wraps (bitwise
where the kernels are the same), its gradient equals the oracle's, and
torch.library.opcheck passes (schema, autograd registration, fake tensors).
"""
import numpy as np
import pytest
import torch

from conftest import close
from oracle import hodge_ref as R

OPS = ("spmm", "poly_basis", "poly_basis_backward", "proj", "proj_backward", "att_score",
       "att_score_backward", "segment_mean", "segment_mean_backward", "csr_from_coo")


def _ops():
    from hlhgat import ops  # noqa: F401  (loads _hlhgat_ext: registers torch.ops.hlhgat)
    return torch.ops.hlhgat


def test_schemas_registered():
    h = _ops()
    for name in OPS:
        schema = str(getattr(h, name).default._schema)
        assert schema.startswith(f"hlhgat::{name}("), schema


def _csr_meta(n, nnz):
    m = torch.device("meta")
    return (torch.empty(n + 1, dtype=torch.int32, device=m),
            torch.empty(nnz, dtype=torch.int32, device=m),
            torch.empty(nnz, dtype=torch.float32, device=m))


def test_meta_shapes_and_autograd():
    h = _ops()
    m = torch.device("meta")
    rp, col, val = _csr_meta(100, 700)
    x = torch.empty(100, 64, device=m, requires_grad=True)
    y = h.spmm(rp, col, val, x)
    assert y.shape == (100, 64) and y.device.type == "meta"
    T = h.poly_basis(rp, col, val, x, 4, 0)
    assert T.shape == (3, 100, 64)
    (y.sum() + T.sum()).backward()
    assert x.grad.shape == x.shape
    A = [torch.empty(50, 24, device=m, requires_grad=True),
         torch.empty(50, 40, device=m, requires_grad=True)]
    W = torch.empty(32, 64, device=m, requires_grad=True)
    b = torch.empty(32, device=m, requires_grad=True)
    out = h.proj(A, W, b)
    assert out.shape == (50, 32)
    out.sum().backward()
    assert W.grad.shape == W.shape and b.grad.shape == b.shape and A[1].grad.shape == (50, 40)
    q = [torch.empty(70, 32, device=m, requires_grad=True) for _ in range(3)]
    a = h.att_score(q[0], q[1], q[2], 0.5, 0.5, 32 ** 0.5, 0)
    assert a.shape == (70, 1)
    a.sum().backward()
    assert all(t.grad.shape == (70, 32) for t in q)
    xs = torch.empty(90, 16, device=m, requires_grad=True)
    sp = torch.empty(6, dtype=torch.int32, device=m)
    s = h.segment_mean(xs, sp, None, 5)
    assert s.shape == (5, 16)
    s.sum().backward()
    assert xs.grad.shape == xs.shape
    r = torch.empty(700, dtype=torch.int64, device=m)
    rp2, c2, v2 = h.csr_from_coo(r, r, torch.empty(700, device=m), 100, True)
    assert rp2.shape == (101,) and rp2.dtype == torch.int32 and c2.shape == (700,) \
        and v2.shape == (700,)


def test_fake_tensor_propagation():
    """FakeTensorMode (the tracer torch.compile uses) propagates the ops."""
    from torch._subclasses.fake_tensor import FakeTensorMode
    h = _ops()
    with FakeTensorMode():
        rp = torch.empty(33, dtype=torch.int32)
        col = torch.empty(200, dtype=torch.int32)
        x = torch.empty(32, 8)
        y = h.spmm(rp, col, None, x)
        assert y.shape == (32, 8)
        out = h.proj([x], torch.empty(5, 8), None)
        assert out.shape == (32, 5)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
def _graph(n_graphs=12, seed=3):
    from hlhgat.synthetic import zinc_like_batch
    return zinc_like_batch(n_graphs, seed=seed)


@pytest.mark.gpu
def test_spmm_and_basis_match_c_abi_and_oracle(cuda):
    from hlhgat import ops
    h = _ops()
    b = _graph()
    n = b.x_s.shape[0]
    ei, w = b.edge_index_s, b.edge_weight_s
    rp, col, val = h.csr_from_coo(ei[1].to(cuda), ei[0].to(cuda), w.to(cuda), n, False)
    op = ops.hodge_operator(ei.to(cuda), w.to(cuda), n)
    assert torch.equal(rp, op.fwd.rowptr) and torch.equal(col, op.fwd.col)
    assert torch.equal(val, op.fwd.val)
    x = torch.randn(n, 24, generator=torch.Generator().manual_seed(1))
    xd = x.to(cuda).requires_grad_(True)
    y = h.spmm(rp, col, val, xd)
    assert torch.equal(y.detach().cpu(), R.propagate(x, ei, w))  # bit-exact
    T = h.poly_basis(rp, col, val, xd, 4, 0)
    assert torch.equal(T.detach(), ops.poly_basis(op, xd.detach(), 4, ops.POLY_LAGUERRE))
    Rg = torch.randn(T.shape, generator=torch.Generator().manual_seed(2))
    (T * Rg.to(cuda)).sum().backward()
    xr = x.double().requires_grad_(True)
    Ws = [torch.zeros(24, 24, dtype=torch.float64)] + \
        [torch.eye(24, dtype=torch.float64) for _ in range(3)]
    # sum_k <T_k, R_k> through the oracle's Laguerre recurrence: a conv whose
    # projections are identity blocks, contracted with R
    outs = []
    Tx0, Tx1 = xr, xr - R.propagate(xr, ei, w.double())
    outs.append(Tx1)
    for k in (1, 2):
        Tx2 = (-R.propagate(Tx1, ei, w.double()) + (2 * k + 1) * Tx1 - k * Tx0) / (k + 1)
        outs.append(Tx2)
        Tx0, Tx1 = Tx1, Tx2
    sum((o * Rg[i].double()).sum() for i, o in enumerate(outs)).backward()
    del Ws
    close(xd.grad.cpu(), xr.grad, 1e-5, "poly_basis grad")


@pytest.mark.gpu
def test_proj_att_segment_match_torch(cuda):
    h = _ops()
    g = torch.Generator().manual_seed(5)
    A = [torch.randn(300, k, generator=g) for k in (64, 8, 36)]
    W = torch.randn(48, 108, generator=g)
    bias = torch.randn(48, generator=g)
    Ad = [a.to(cuda).requires_grad_(True) for a in A]
    Wd, bd = W.to(cuda).requires_grad_(True), bias.to(cuda).requires_grad_(True)
    out = h.proj(Ad, Wd, bd)
    Ar = [a.double().requires_grad_(True) for a in A]
    Wr, br = W.double().requires_grad_(True), bias.double().requires_grad_(True)
    ref = torch.nn.functional.linear(torch.cat(Ar, 1), Wr, br)
    close(out.detach().cpu(), ref.detach(), 1e-5, "proj")
    Rg = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (out * Rg.float().to(cuda)).sum().backward()
    (ref * Rg).sum().backward()
    for a, r in zip(Ad + [Wd, bd], Ar + [Wr, br]):
        close(a.grad.cpu(), r.grad, 1e-4, "proj grad")
    q = [torch.randn(200, 32, generator=g) for _ in range(3)]
    qd = [t.to(cuda).requires_grad_(True) for t in q]
    a = h.att_score(qd[0], qd[1], qd[2], 0.5, 0.5, float(np.sqrt(32)), 0)
    qr = [t.double().requires_grad_(True) for t in q]
    ar = R.att_score(qr[0], qr[1], qr[2], 0.5, 32, torch.nn.Sigmoid())
    close(a.detach().cpu(), ar.detach(), 1e-5, "att")
    a.sum().backward()
    ar.sum().backward()
    for t, r in zip(qd, qr):
        close(t.grad.cpu(), r.grad, 1e-5, "att grad")
    x = torch.randn(90, 16, generator=g)
    ptr = torch.tensor([0, 10, 10, 40, 77, 90], dtype=torch.int32)
    xd = x.to(cuda).requires_grad_(True)
    s = h.segment_mean(xd, ptr.to(cuda), None, 5)
    batch = torch.repeat_interleave(torch.arange(5), (ptr[1:] - ptr[:-1]).long())
    xr = x.double().requires_grad_(True)
    sr = R.scatter_mean(xr, batch, 5)
    close(s.detach().cpu(), sr.detach(), 1e-6, "segment_mean")
    s.sum().backward()
    sr.sum().backward()
    close(xd.grad.cpu(), xr.grad, 1e-6, "segment_mean grad")


@pytest.mark.gpu
def test_opcheck(cuda):
    """torch.library.opcheck: schema, autograd registration, fake-tensor
    (Meta) kernels agree with the HIP kernels."""
    h = _ops()
    b = _graph(4, seed=9)
    n = b.x_t.shape[0]
    ei, w = b.edge_index_t.to(cuda), b.edge_weight_t.to(cuda)
    rp, col, val = h.csr_from_coo(ei[1], ei[0], w, n, False)
    x = torch.randn(n, 16, device=cuda, requires_grad=True)
    tests = ("test_schema", "test_autograd_registration", "test_faketensor")
    torch.library.opcheck(h.spmm.default, (rp, col, val, x), test_utils=tests)
    torch.library.opcheck(h.poly_basis.default, (rp, col, val, x, 3, 0), test_utils=tests)
    A = [torch.randn(n, 16, device=cuda, requires_grad=True)]
    torch.library.opcheck(h.proj.default, (A, torch.randn(8, 16, device=cuda, requires_grad=True),
                                           None), test_utils=tests)
    q = [torch.randn(n, 8, device=cuda, requires_grad=True) for _ in range(3)]
    torch.library.opcheck(h.att_score.default, (*q, 0.1, 0.9, 8 ** 0.5, 1), test_utils=tests)
    ptr = torch.tensor([0, n // 2, n], dtype=torch.int32, device=cuda)
    torch.library.opcheck(h.segment_mean.default, (x, ptr, None, 2), test_utils=tests)


@pytest.mark.gpu
def test_row_scale_att_kq_pool_bwd_match_torch(cuda):
    """The attention-pooling heads' glue kernels: ops.row_scale (x0 * att,
    main_pepfunc...:134-136) against ATen's broadcast product (forward and dx
    bitwise, da to fp32 rounding); att_score_kq against att_score on the two
    column halves (bitwise); segment_mean(covering=True) (the pool tables'
    backward, zero bucket written by the kernel) against the zero-filled
    scatter_mean backward (bitwise), also into a strided slab column block."""
    from hlhgat import ops
    g = torch.Generator().manual_seed(11)
    for n, d in ((517, 448), (300, 192), (64, 3)):
        x = torch.randn(n, d + 5, generator=g)[:, :d].to(cuda)  # strided rows
        a = torch.rand(n, 1, generator=g).to(cuda)
        xd, ad = x.clone().requires_grad_(True), a.clone().requires_grad_(True)
        y = ops.row_scale(xd, ad)
        xr, ar = x.clone().requires_grad_(True), a.clone().requires_grad_(True)
        yr = xr * ar
        assert torch.equal(y, yr)
        R_ = torch.randn(n, d, generator=g).to(cuda)
        (y * R_).sum().backward()
        (yr * R_).sum().backward()
        assert torch.equal(xd.grad, xr.grad)
        close(ad.grad.cpu(), ar.grad.cpu(), 1e-5, "row_scale da")
        slab = torch.zeros(n, d + 64, device=cuda)
        y2 = ops.row_scale(x, a, out=slab[:, :d])
        assert y2.data_ptr() == slab.data_ptr() and torch.equal(slab[:, :d], yr.detach())
        assert not slab[:, d:].any()
    dk = 32
    qc = torch.randn(200, dk, generator=g).to(cuda)
    kq = torch.randn(200, 2 * dk, generator=g).to(cuda)
    q1, k1 = qc.clone().requires_grad_(True), kq.clone().requires_grad_(True)
    q2, k2 = qc.clone().requires_grad_(True), kq.clone().requires_grad_(True)
    for code in (ops.SIGMA_SIGMOID, ops.SIGMA_RELU):
        a1 = ops.att_score_kq(q1, k1, 0.1, 0.9, float(np.sqrt(dk)), code)
        a2 = ops.att_score(q2, k2[:, dk:], k2[:, :dk], 0.1, 0.9, float(np.sqrt(dk)), code)
        assert torch.equal(a1, a2)
        w = torch.randn(200, 1, generator=g).to(cuda)
        (a1 * w).sum().backward()
        (a2 * w).sum().backward()
        assert torch.equal(q1.grad, q2.grad) and torch.equal(k1.grad, k2.grad)
    # covering pool tables: 4 clusters, rows 3, 7, 11 in no cluster (bucket 4)
    n, d, n_seg = 13, 24, 4
    assign = torch.tensor([0, 1, 1, -1, 2, 0, 3, -1, 2, 2, 1, -1, 0])
    order = torch.argsort(torch.where(assign < 0, n_seg, assign), stable=True)
    counts = torch.bincount(torch.where(assign < 0, n_seg, assign), minlength=n_seg + 1)
    rp = torch.zeros(n_seg + 2, dtype=torch.int32)
    rp[1:] = torch.cumsum(counts, 0).to(torch.int32)
    rows = order.to(torch.int32)
    x = torch.randn(n, d, generator=g).to(cuda)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    s1 = ops.segment_mean(x1, rp.to(cuda), n_seg, rows.to(cuda), covering=True)
    s2 = ops.segment_mean(x2, rp[:n_seg + 1].to(cuda), n_seg, rows[:int(rp[n_seg])].to(cuda))
    assert torch.equal(s1, s2)
    gr = torch.randn(n_seg, d, generator=g).to(cuda)
    (s1 * gr).sum().backward()
    (s2 * gr).sum().backward()
    assert torch.equal(x1.grad, x2.grad) and not x1.grad[assign < 0].any()
    # into a strided destination + the gradient sink of a DenseConcat-style slab
    G = torch.full((n, d + 8), float("nan"), device=cuda)
    flag = torch.zeros(1, dtype=torch.int32)
    out = torch.zeros(n_seg, d + 4, device=cuda)
    x3 = x.clone().requires_grad_(True)
    s3 = ops.segment_mean(x3, rp.to(cuda), n_seg, rows.to(cuda), out=out[:, :d], covering=True,
                          gsink=(G[:, :d], flag))
    assert s3.data_ptr() == out.data_ptr() and torch.equal(out[:, :d], s2.detach())
    (s3 * gr).sum().backward()
    assert int(flag[0]) == 1 and torch.equal(G[:, :d], x2.grad)
    assert torch.isnan(G[:, d:]).all()


@pytest.mark.gpu
def test_tsp_readout_bitwise_unfused(cuda):
    """ops.tsp_readout (cat([x_s, |B1^T x_t| / 2]) in a slab window, one pass
    each way) against boundary_t / abs / div / cat: bitwise values and
    gradients (lib/Hodge_ST_Model.py:846-849)."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import adj2par1
    from hlhgat.synthetic import tsp_like_graph
    from hlhgat.hodge_dataset import collate
    b = collate([tsp_like_graph(1), tsp_like_graph(2)], check_hodge=False).to(cuda)
    nt, ne = b.x_t.size(0), b.x_s.size(0)
    inc = adj2par1(b.edge_index, nt, ne).incidence()
    g = torch.Generator().manual_seed(4)
    ct, cs = 64, 48
    xt = torch.randn(nt, ct, generator=g).to(cuda)
    xt[:5] = 0.0  # zero differences: sgn 0 in the backward
    xs = torch.randn(ne, cs, generator=g).to(cuda)
    S = torch.full((ne, 16 + cs + ct), float("nan"), device=cuda)
    S[:, 16:16 + cs] = xs
    x1, s1 = xt.clone().requires_grad_(True), xs.clone().requires_grad_(True)
    R = ops.tsp_readout(s1, x1, inc, S[:, 16:])
    x2, s2 = xt.clone().requires_grad_(True), xs.clone().requires_grad_(True)
    R2 = torch.cat([s2, ops.boundary_t(x2, inc).abs() / 2], dim=-1)
    assert R.data_ptr() == S.data_ptr() + 4 * 16 and torch.equal(R, R2)
    W = torch.randn(ne, cs + ct, generator=g).to(cuda)
    (R * W).sum().backward()
    (R2 * W).sum().backward()
    assert torch.equal(x1.grad, x2.grad) and torch.equal(s1.grad, s2.grad)


@pytest.mark.gpu
def test_bce_with_logits_matches_torch(cuda):
    """hlhgat.nn.BCEWithLogitsLoss (one HIP launch each way) against torch's:
    loss to fp32 summation order, input gradient to 1 ulp-scale tolerance;
    weighted, CPU and large inputs go to torch."""
    import hlhgat
    g = torch.Generator().manual_seed(8)
    for shape, red in (((64, 10), "mean"), ((16001,), "sum"), ((3, 5), "mean")):
        x = (torch.randn(shape, generator=g) * 6).to(cuda)
        x.view(-1)[:3] = torch.tensor([0.0, -0.0, 30.0])
        t = (torch.rand(shape, generator=g) > 0.5).float().to(cuda)
        x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
        l1 = hlhgat.nn.BCEWithLogitsLoss(reduction=red)(x1, t)
        l2 = torch.nn.BCEWithLogitsLoss(reduction=red)(x2, t)
        close(l1.detach().cpu(), l2.detach().cpu(), 1e-5, f"bce {red} loss")
        (l1 * 1.7).backward()
        (l2 * 1.7).backward()
        close(x1.grad.cpu(), x2.grad.cpu(), 1e-6, f"bce {red} grad")
    w = torch.rand(4, 3).to(cuda)
    x = torch.randn(4, 3).to(cuda)
    t = torch.ones(4, 3).to(cuda)
    assert torch.equal(hlhgat.nn.BCEWithLogitsLoss(weight=w)(x, t),
                       torch.nn.BCEWithLogitsLoss(weight=w)(x, t))
