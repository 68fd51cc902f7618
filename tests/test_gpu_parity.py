"""HIP path vs the oracle / the reference's golden vectors (MI355X only).

Tolerances, written per assertion:
  * SpMM, Laguerre/Chebyshev basis, incidence gathers: BIT-EXACT vs the oracle
    (same operation order, -ffp-contract=off);
  * outputs through the MFMA projection: max|d| <= 1e-5 * max(1, max|ref|);
  * gradients: 1e-4 relative;  whole model after BN: 1e-4 relative.
"""
import os

import numpy as np
import pytest
import torch

from conftest import close, golden_names, load_golden
from oracle import hodge_ref as R

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T = torch.from_numpy


def dev(a, d="cuda:0"):
    return (T(a) if isinstance(a, np.ndarray) else a).to(d)


def rand_graph(n, nnz, seed, sym=False, sort=True):
    g = torch.Generator().manual_seed(seed)
    r = torch.randint(0, max(n, 1), (nnz,), generator=g)
    c = torch.randint(0, max(n, 1), (nnz,), generator=g)
    w = torch.randn(nnz, generator=g)
    if sym:
        r, c = torch.cat([r, c]), torch.cat([c, r])
        w = torch.cat([w, w])
    ei = torch.stack([r, c])
    if sort:
        key = ei[0] * max(n, 1) + ei[1]
        o = torch.argsort(key, stable=True)
        ei, w = ei[:, o], w[o]
    return ei.contiguous(), w.contiguous()


# ---------------------------------------------------------------------------
# SpMM / propagate
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("d", [1, 2, 3, 18, 36, 64, 128, 300])
@pytest.mark.parametrize("mode", ["general", "general_unsorted"])
def test_spmm_bitexact_vs_propagate(cuda, d, mode):
    from hlhgat import ops
    n = 517
    ei, w = rand_graph(n, 3000, seed=d, sort=(mode == "general"))
    x = torch.randn(n, d, generator=torch.Generator().manual_seed(1))
    ref = R.propagate(x, ei, w)
    op = ops.hodge_operator(dev(ei), dev(w), n)
    y = ops.spmm(op.fwd, dev(x)).cpu()
    # CSR keeps COO order within a row only for sorted input; unsorted input is
    # reordered by (row, col) like torch coalesce -> compare with tolerance
    if mode == "general":
        assert torch.equal(y, ref), (y - ref).abs().max()
    else:
        close(y, ref, 1e-5, "spmm unsorted")


def test_spmm_hodge_fast_path_bitexact(cuda):
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(40, seed=3)
    for side in ("t", "s"):
        ei = getattr(b, "edge_index_" + side)
        w = getattr(b, "edge_weight_" + side)
        n = getattr(b, "x_" + side).shape[0]
        x = torch.randn(n, 64, generator=torch.Generator().manual_seed(2))
        ref = R.propagate(x, ei, w)
        ei_d = ops.mark_hodge(dev(ei))
        op = ops.hodge_operator(ei_d, dev(w), n)
        assert op.fwd is op.bwd  # symmetric fast path: one CSR
        y = ops.spmm(op.fwd, dev(x)).cpu()
        assert torch.equal(y, ref)


def test_spmm_empty_rows_and_empty_matrix(cuda):
    from hlhgat import ops
    n = 50
    ei = torch.tensor([[3, 3, 7], [1, 9, 7]])  # rows 0..2, 4..6, 8.. are empty
    w = torch.tensor([1.5, -2.0, 0.25])
    x = torch.randn(n, 64)
    op = ops.hodge_operator(dev(ei), dev(w), n)
    assert torch.equal(ops.spmm(op.fwd, dev(x)).cpu(), R.propagate(x, ei, w))
    op0 = ops.hodge_operator(dev(torch.zeros(2, 0, dtype=torch.long)),
                             dev(torch.zeros(0)), n)
    assert torch.equal(ops.spmm(op0.fwd, dev(x)).cpu(), torch.zeros(n, 64))


def test_spmm_skewed_rows(cuda):
    """A hub row with thousands of entries next to rows with one (L1-style skew)."""
    from hlhgat import ops
    n = 3000
    hub = torch.stack([torch.zeros(n, dtype=torch.long), torch.arange(n)])
    diag = torch.stack([torch.arange(n), torch.arange(n)])
    ei = torch.cat([hub, diag], 1)
    key = ei[0] * n + ei[1]
    o = torch.argsort(key, stable=True)
    ei = ei[:, o].contiguous()
    w = torch.randn(ei.size(1))
    x = torch.randn(n, 64)
    op = ops.hodge_operator(dev(ei), dev(w), n)
    close(ops.spmm(op.fwd, dev(x)).cpu(), R.propagate(x, ei, w), 1e-6, "skew")


@pytest.mark.parametrize("d", [3, 64, 128])
def test_poly_step_ragged_rows_bitexact(cuda, d):
    """Rows of 0..40 entries (every tail length of the batched gathers: a
    chunk of <= 8 entries in one batch, 4-wide batches and a < 4 tail above,
    chunks of 16 staged entries): the Laguerre basis equals the oracle's
    recurrence over propagate bit for bit."""
    from hlhgat import ops
    gen = torch.Generator().manual_seed(3)
    n = 400
    deg = torch.arange(n) % 41
    rows = torch.repeat_interleave(torch.arange(n), deg)
    cols = torch.randint(0, n, (rows.numel(),), generator=gen)
    o = torch.argsort(rows * n + cols, stable=True)
    ei = torch.stack([rows[o], cols[o]]).contiguous()
    w = torch.randn(ei.size(1), generator=gen)
    x = torch.randn(n, d, generator=gen)
    ref = _ref_basis(x, ei, w, 3, "laguerre")
    op = ops.hodge_operator(dev(ei), dev(w), n)
    T = ops.poly_basis(op, dev(x), 3, ops.POLY_LAGUERRE).cpu()
    for k in range(2):
        assert torch.equal(T[k], ref[k]), k
    assert torch.equal(ops.spmm(op.fwd, dev(x)).cpu(), R.propagate(x, ei, w))


# ---------------------------------------------------------------------------
# polynomial basis (bit-exact) and full conv vs golden
# ---------------------------------------------------------------------------
def _ref_basis(x, ei, w, K, kind):
    Ts = [x]
    if K > 1:
        p = R.propagate(x, ei, w)
        Ts.append(x - p if kind == "laguerre" else p)
    for k in range(1, K - 1):
        p = R.propagate(Ts[k], ei, w)
        if kind == "laguerre":
            Ts.append((-p + (2 * k + 1) * Ts[k] - k * Ts[k - 1]) / (k + 1))
        else:
            Ts.append(2. * p - Ts[k - 1])
    return Ts[1:]


@pytest.mark.parametrize("kind", ["laguerre", "cheb"])
@pytest.mark.parametrize("K", [2, 3, 4, 6])
def test_poly_basis_bitexact(cuda, kind, K):
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(20, seed=K)
    ei, w, n = b.edge_index_s, b.edge_weight_s, b.x_s.shape[0]
    x = torch.randn(n, 64, generator=torch.Generator().manual_seed(K))
    op = ops.hodge_operator(ops.mark_hodge(dev(ei)), dev(w), n)
    code = ops.POLY_LAGUERRE if kind == "laguerre" else ops.POLY_CHEB
    Tdev = ops.poly_basis(op, dev(x), K, code).cpu()
    for k, Tr in enumerate(_ref_basis(x, ei, w, K, kind)):
        assert torch.equal(Tdev[k], Tr), (kind, K, k, (Tdev[k] - Tr).abs().max())


@pytest.mark.parametrize("name", golden_names("conv_"))
def test_conv_vs_reference_golden(cuda, name):
    import hlhgat
    g = load_golden(name)
    K = int(g["K"])
    cls = hlhgat.HodgeChebConv if "cheb" in name else hlhgat.HodgeLaguerreConv
    conv = cls(g["w0"].shape[1], g["w0"].shape[0], K=K).to(cuda)
    sd = {"bias": T(g["bias"])}
    sd.update({f"lins.{k}.weight": T(g[f"w{k}"]) for k in range(K)})
    conv.load_state_dict(sd)
    x = dev(g["x"]).requires_grad_(True)
    out = conv(x, dev(g["edge_index"]), dev(g["edge_weight"]))
    close(out.detach().cpu(), g["out"], 1e-5, "out")
    (out * dev(g["R"])).sum().backward()
    close(x.grad.cpu(), g["grad_x"], 1e-4, "grad_x")
    close(conv.bias.grad.cpu(), g["grad_bias"], 1e-4, "grad_bias")
    for k in range(K):
        close(conv.lins[k].weight.grad.cpu(), g[f"grad_w{k}"], 1e-4, f"grad_w{k}")


@pytest.mark.parametrize("name", golden_names("demo_fastconv_"))
def test_demo_fastconv_vs_reference_golden(cuda, name):
    """HL-HGAT-DEMO HodgeLaguerreFastConv (published :561 recurrence) on the
    HIP kind HLHGAT_POLY_LAGUERRE_DEMO, adj_t in the DEMO's transpose form."""
    import hlhgat
    g = load_golden(name)
    K = int(g["K"])
    conv = hlhgat.HodgeLaguerreFastConv(g["w0"].shape[1], g["w0"].shape[0], K=K).to(cuda)
    sd = {"bias": T(g["bias"])}
    sd.update({f"lins.{k}.weight": T(g[f"w{k}"]) for k in range(K)})
    conv.load_state_dict(sd)
    ei, w = T(g["edge_index"]), T(g["edge_weight"])
    n = g["x"].shape[0]
    adj_t = torch.sparse_coo_tensor(torch.stack([ei[1], ei[0]]), w, (n, n)).to(cuda)
    x = dev(g["x"]).requires_grad_(True)
    out = conv(x, adj_t)
    close(out.detach().cpu(), g["out"], 1e-5, "out")
    (out * dev(g["R"])).sum().backward()
    close(x.grad.cpu(), g["grad_x"], 1e-4, "grad_x")
    close(conv.bias.grad.cpu(), g["grad_bias"], 1e-4, "grad_bias")
    for k in range(K):
        close(conv.lins[k].weight.grad.cpu(), g[f"grad_w{k}"], 1e-4, f"grad_w{k}")


@pytest.mark.parametrize("K", [3, 5])
def test_demo_basis_bitexact(cuda, K):
    """Forward DEMO basis equals the oracle's operation order bit for bit."""
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(20, seed=K + 40)
    ei, w, n = b.edge_index_t, b.edge_weight_t, b.x_t.shape[0]
    x = torch.randn(n, 32, generator=torch.Generator().manual_seed(K))
    op = ops.hodge_operator(ops.mark_hodge(dev(ei)), dev(w), n)
    Tdev = ops.poly_basis(op, dev(x), K, ops.POLY_LAGUERRE_DEMO).cpu()
    p = R.propagate(x, ei, w)
    Ts = [x, x - p]
    for k in range(1, K - 1):
        Ts.append((-p + (2 * k + 1) * Ts[k] - k * Ts[k - 1]) / (k + 1))
    for k in range(1, K):
        assert torch.equal(Tdev[k - 1], Ts[k]), (K, k, (Tdev[k - 1] - Ts[k]).abs().max())


def test_conv_unsorted_nonsymmetric_operator(cuda):
    """General (sorting) CSR path incl. the transposed adjoint for a
    non-symmetric operator: gradient w.r.t. x must use L^T."""
    import hlhgat
    n, cin, cout, K = 300, 24, 32, 4
    ei, w = rand_graph(n, 2000, seed=5, sort=False)
    torch.manual_seed(0)
    conv = hlhgat.HodgeLaguerreConv(cin, cout, K=K).to(cuda)
    ref = R.RefHodgeConv(cin, cout, K)
    ref.load_state_dict({k: v.cpu() for k, v in conv.state_dict().items()})
    x = torch.randn(n, cin)
    xd = dev(x).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    out = conv(xd, dev(ei), dev(w))
    outr = ref(xr, ei, w)
    close(out.detach().cpu(), outr.detach(), 1e-5, "out")
    Rg = torch.randn(out.shape)
    (out * dev(Rg)).sum().backward()
    (outr * Rg).sum().backward()
    close(xd.grad.cpu(), xr.grad, 1e-4, "grad_x")


def test_conv_K1_is_linear(cuda):
    import hlhgat
    conv = hlhgat.HodgeLaguerreConv(8, 5, K=1).to(cuda)
    x = torch.randn(10, 8, device=cuda)
    ei = torch.zeros(2, 0, dtype=torch.long, device=cuda)
    out = conv(x, ei, torch.zeros(0, device=cuda))
    close(out.detach().cpu(), (x @ conv.lins[0].weight.t() + conv.bias).detach().cpu(), 1e-5, "K=1")


# ---------------------------------------------------------------------------
# MFMA projection GEMMs vs a plain fp32 torch reference
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("M,N,kbs", [(1, 1, [1]), (17, 16, [4]), (1000, 64, [64, 64, 64]),
                                     (5000, 64, [384, 384]), (333, 33, [18, 7]),
                                     (4097, 130, [36]), (2048, 256, [128, 128]),
                                     (70000, 64, [64]), (23001, 64, [36, 36, 36]),
                                     (999, 32, [20, 12, 4]), (513, 16, [8, 40]),
                                     (3000, 64, [384, 384, 128])])
def test_linear_blocks_fwd_bwd(cuda, M, N, kbs):
    from hlhgat import ops
    g = torch.Generator().manual_seed(M + N)
    As = [torch.randn(M, k, generator=g) for k in kbs]
    W = torch.randn(N, sum(kbs), generator=g) * 0.1
    b = torch.randn(N, generator=g)
    Ad = [dev(a).requires_grad_(True) for a in As]
    Wd = dev(W).requires_grad_(True)
    bd = dev(b).requires_grad_(True)
    out = ops.linear_blocks(Ad, Wd, bd)
    Ar = [a.clone().double().requires_grad_(True) for a in As]
    Wr = W.clone().double().requires_grad_(True)
    br = b.clone().double().requires_grad_(True)
    outr = torch.cat(Ar, 1) @ Wr.t() + br
    close(out.detach().cpu(), outr.detach(), 1e-5, "fwd")
    Rg = torch.randn(M, N, generator=g)
    (out * dev(Rg)).sum().backward()
    (outr * Rg.double()).sum().backward()
    for i in range(len(kbs)):
        close(Ad[i].grad.cpu(), Ar[i].grad, 1e-5, f"dA{i}")
    close(Wd.grad.cpu(), Wr.grad, 1e-4, "dW")
    close(bd.grad.cpu(), br.grad, 1e-4, "db")


def test_linear_blocks_strided_views(cuda):
    """Operands that are column slices of wider tensors (ld > width)."""
    from hlhgat import ops
    A = torch.randn(500, 96, device=cuda)
    W = torch.randn(40, 64, device=cuda)
    out = ops.linear_blocks([A[:, 8:40], A[:, 64:96]], W, None)
    exp = torch.cat([A[:, 8:40], A[:, 64:96]], 1) @ W.t()
    close(out.cpu(), exp.cpu(), 1e-5, "strided")


# ---------------------------------------------------------------------------
# boundary operator, attention, pooling
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["nei_value", "nei_att_sigmoid", "nei_att_relu"])
def test_node_edge_int_vs_reference_golden(cuda, name):
    import hlhgat
    g = load_golden(name)
    sd = {k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")}
    if name == "nei_value":
        m = hlhgat.NodeEdgeInt(d=sd["WV_Node.0.weight"].shape[1] // 2,
                               dv=sd["WV_Node.3.weight"].shape[0])
    else:
        sig = torch.nn.Sigmoid() if "sigmoid" in name else torch.nn.ReLU()
        m = hlhgat.NodeEdgeInt(d=sd["WQ_Node.weight"].shape[1], dk=sd["WQ_Node.weight"].shape[0],
                               only_att=True, sigma=sig, l=0.9 if "sigmoid" in name else 0.5)
    m.load_state_dict(sd)
    m = m.to(cuda).train()
    x_t = dev(g["x_t"]).requires_grad_(True)
    x_s = dev(g["x_s"]).requires_grad_(True)
    par = hlhgat.adj2par1(dev(g["edge_index"]), x_t.shape[0], x_s.shape[0])
    a, c = m(x_t, x_s, par, dev(g["D"]))
    close(a.detach().cpu(), g["out_t"], 1e-5, "out_t")
    close(c.detach().cpu(), g["out_s"], 1e-5, "out_s")
    ((a * dev(g["R_t"])).sum() + (c * dev(g["R_s"])).sum()).backward()
    close(x_t.grad.cpu(), g["grad_x_t"], 1e-4, "grad_x_t")
    close(x_s.grad.cpu(), g["grad_x_s"], 1e-4, "grad_x_s")
    for k, p in m.named_parameters():
        close(p.grad.cpu(), g["grad/" + k], 1e-4, "grad " + k)


def test_poly_step_call_site_census(cuda):
    """Each k_poly_step call site is stamped under its own hlhgat_prof class
    (the bench's per-call-site census): a Laguerre conv's forward basis under
    PROF_POLY and its backward under PROF_POLY_ADJ; NodeEdgeInt's |B1| node
    gathers under PROF_INCIDENCE (counted with the n_src rows they read) and
    its edge gathers under PROF_GATHER2, none under PROF_POLY."""
    import hlhgat
    from hlhgat import _lib, ops
    classes = (_lib.PROF_POLY, _lib.PROF_POLY_ADJ, _lib.PROF_INCIDENCE, _lib.PROF_GATHER2)

    def census(fn):
        torch.cuda.synchronize()
        ops.prof_reset()
        for c in classes:
            ops.prof_enable(c, True)
        fn()
        torch.cuda.synchronize()
        for c in classes:
            ops.prof_enable(c, False)
        return {c: ops.prof_read(c) for c in classes}

    ei, w = rand_graph(300, 2000, seed=5, sort=True)
    conv = hlhgat.HodgeLaguerreConv(24, 32, K=4).to(cuda)
    xd = torch.randn(300, 24, device=cuda, requires_grad=True)
    got = census(lambda: conv(xd, dev(ei), dev(w)).sum().backward())
    assert got[_lib.PROF_POLY]["launches"] > 0 and got[_lib.PROF_POLY_ADJ]["launches"] > 0, got
    assert got[_lib.PROF_INCIDENCE]["launches"] == 0 and got[_lib.PROF_GATHER2]["launches"] == 0

    g = load_golden("nei_value")
    sd = {k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")}
    m = hlhgat.NodeEdgeInt(d=sd["WV_Node.0.weight"].shape[1] // 2,
                           dv=sd["WV_Node.3.weight"].shape[0])
    m.load_state_dict(sd)
    m = m.to(cuda).train()
    x_t = dev(g["x_t"]).requires_grad_(True)
    x_s = dev(g["x_s"]).requires_grad_(True)
    par = hlhgat.adj2par1(dev(g["edge_index"]), x_t.shape[0], x_s.shape[0])

    def nei():
        a, c = m(x_t, x_s, par, dev(g["D"]))
        (a.sum() + c.sum()).backward()
    got = census(nei)
    inc = got[_lib.PROF_INCIDENCE]
    assert inc["launches"] >= 2 and got[_lib.PROF_GATHER2]["launches"] >= 1, got
    assert got[_lib.PROF_POLY]["launches"] == 0 and got[_lib.PROF_POLY_ADJ]["launches"] == 0
    # the gathered operand is the edge side: at least 4 n_edges d bytes a launch
    E = x_s.shape[0]
    assert inc["bytes"] / inc["launches"] >= 4.0 * E * 1, inc
    ops.check_device_errors()


def test_incidence_gathers_bitexact(cuda):
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(30, seed=8)
    ei = b.edge_index
    N_t, N_s = b.x_t.shape[0], b.x_s.shape[0]
    D = R.degree(ei.reshape(-1), N_t) + 1e-6
    x_t, x_s = torch.randn(N_t, 40), torch.randn(N_s, 40)
    par = R.adj2par1(ei, N_t, N_s)
    s2t, t2s = R.boundary_mix(x_t, x_s, par, D)
    inc = ops.incidence(dev(ei), N_t)
    s2t_d = ops.node_from_edges(dev(x_s), inc, dev(1 / D)).cpu()
    t2s_d = ops.edge_from_nodes(dev(x_t), inc).cpu()
    assert torch.equal(t2s_d, t2s)
    assert torch.equal(s2t_d, s2t)


def test_collate_incidence_equals_device_build(cuda):
    """The incidence CSR built at collate (plain and padded batches) is the
    one hlhgat_incidence_csr sorts on the device, bit for bit, and the batch
    path uses it (no device build)."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(40, seed=9)
    for host in (b, pad_batch(b, static_caps(b, 256))):
        n = host.x_t.shape[0]
        built = ops.incidence(dev(host.edge_index), n)
        bd = host.to(cuda)
        inc = ops.incidence(bd.edge_index, n)
        assert inc.rowptr.data_ptr() == bd.inc_rowptr.data_ptr()
        assert torch.equal(inc.rowptr, built.rowptr) and torch.equal(inc.edge_ids, built.edge_ids)
        # the degree D and its reciprocal built with the batch: the device ops' bits
        from hlhgat.hodge_dataset import degree
        d = degree(bd.edge_index.view(-1), num_nodes=n)
        vm = getattr(bd, "valid_mask_t", None)
        if vm is not None:
            d = d.masked_fill(~vm, 1.0)
        assert torch.equal(bd.deg_t, d)
        assert torch.equal(ops.reciprocal(bd.deg_t), (1 / d).view(-1))
        assert ops.reciprocal(bd.deg_t).data_ptr() == bd.inv_deg_t.data_ptr()
        # the Laplacian CSRs built with the batch: the device build's arrays
        for side in ("t", "s"):
            ei, w = getattr(bd, "edge_index_" + side), getattr(bd, "edge_weight_" + side)
            rows = getattr(bd, "x_" + side).shape[0]
            ref = ops._csr_sorted(ei[0], ei[1], w, rows, rows)
            got = ops.hodge_operator(ei, w, rows).fwd
            assert got.rowptr.data_ptr() == getattr(bd, "csr_rowptr_" + side).data_ptr()
            assert torch.equal(got.rowptr, ref.rowptr) and torch.equal(got.col, ref.col)
            assert torch.equal(got.val, ref.val)


def test_segment_mean_cat_equals_cat(cuda):
    """The readout's cat(mean_pool(x_s), mean_pool(x_t)) written block by
    block (ops.segment_mean_cat): the values and both input gradients of the
    torch.cat of two segment means, bit for bit."""
    from hlhgat import ops
    g = torch.Generator().manual_seed(12)
    counts = [torch.randint(1, 9, (50,), generator=g) for _ in range(2)]
    ptrs = [dev(torch.cat([torch.zeros(1, dtype=torch.int32), c.cumsum(0).to(torch.int32)]))
            for c in counts]
    xs = [dev(torch.randn(int(c.sum()), 24, generator=g)) for c in counts]
    gy = dev(torch.randn(50, 48, generator=g))
    res = []
    for fused in (False, True):
        xr = [x.clone().requires_grad_(True) for x in xs]
        if fused:
            y = ops.segment_mean_cat(xr, ptrs, 50)
        else:
            y = torch.cat([ops.segment_mean(x, p, 50) for x, p in zip(xr, ptrs)], -1)
        y.backward(gy)
        res.append([y.detach(), xr[0].grad, xr[1].grad])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def _poison(cuda, n):
    """Leave NaN in the caching allocator's next blocks, so a torch.empty
    that is not fully written shows up."""
    for _ in range(4):
        t = torch.full((n,), float("nan"), device=cuda)
        del t


@pytest.mark.parametrize("lead,tail", [(0, 0), (0, 300), (7, 0), (7, 300)])
def test_segment_mean_bwd_zeroes_uncovered_rows(cuda, lead, tail):
    """global_mean_pool's adjoint is 0 on rows no segment covers
    (lib/Hodge_ST_Model.py:636): the backward of segment_mean /
    segment_mean_cat / the hlhgat::segment_mean_backward op writes exact zeros
    into rows [0, ptr[0]) and [ptr[n_seg], n) (padding rows of a padded batch)
    and dout[s] / |s| (bitwise torch's division) into the member rows."""
    from hlhgat import ops
    import hlhgat  # noqa: F401  (registers torch.ops.hlhgat)
    g = torch.Generator().manual_seed(13 + lead + tail)
    counts = torch.randint(0, 9, (40,), generator=g)  # empty segments too
    S = int(counts.sum())
    ptr = dev(lead + torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)]).to(torch.int32))
    n = lead + S + tail
    x = torch.randn(n, 24, generator=g)
    gy = torch.randn(40, 24, generator=g)
    exp = torch.zeros(n, 24)
    exp[lead:lead + S] = torch.repeat_interleave(gy / counts.clamp(min=1).float().unsqueeze(1),
                                                 counts, dim=0)
    for how in ("mean", "cat", "op"):
        _poison(cuda, 4 * n * 24)
        if how == "op":
            gx = torch.ops.hlhgat.segment_mean_backward(dev(gy), ptr, None, n)
        else:
            xr = dev(x).requires_grad_(True)
            y = ops.segment_mean_cat([xr], [ptr], 40) if how == "cat" else ops.segment_mean(xr, ptr, 40)
            y.backward(dev(gy))
            gx = xr.grad
        assert torch.equal(gx.cpu(), exp), how
    # no segments at all: every row is uncovered
    _poison(cuda, 4 * n * 24)
    gx = torch.ops.hlhgat.segment_mean_backward(dev(torch.zeros(0, 24)), ptr[:1], None, n)
    assert torch.equal(gx.cpu(), torch.zeros(n, 24))


def test_padded_batch_readout_grad_padding_rows_exactly_zero(cuda, monkeypatch):
    """In a capacity-padded ZINC batch (hodge_dataset.pad_batch) the readout's
    input gradients are exactly 0.0 on the padding rows (finite and zero, not
    merely masked later by the BatchNorm backward)."""
    import hlhgat
    from hlhgat import hodge_st_model, ops
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(37, seed=21)
    pb = pad_batch(b, static_caps(b, 256)).to(cuda)
    n_t, n_s = b.x_t.shape[0], b.x_s.shape[0]
    assert pb.x_t.shape[0] > n_t and pb.x_s.shape[0] > n_s
    seen = {}
    real = ops.segment_mean_cat

    def spy(xs, ptrs, n_seg, side=None):
        for i, x in enumerate(xs):
            x.register_hook(lambda gr, i=i: seen.__setitem__(i, gr.detach().clone()))
        return real(xs, ptrs, n_seg, side=side)

    monkeypatch.setattr(hodge_st_model.ops, "segment_mean_cat", spy)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[1, 1], filters=[32, 32], mlp_channels=[64],
                                            K=3, keig=15).to(cuda).train()
    _poison(cuda, 4 * pb.x_s.shape[0] * 64)
    m(pb).sum().backward()
    gs, gt = seen[0], seen[1]  # readout order: (x_s, x_t)
    assert torch.isfinite(gs).all() and torch.isfinite(gt).all()
    assert torch.equal(gs[n_s:], torch.zeros_like(gs[n_s:]))
    assert torch.equal(gt[n_t:], torch.zeros_like(gt[n_t:]))
    assert gs[:n_s].abs().sum() > 0 and gt[:n_t].abs().sum() > 0


def test_segment_and_cluster_mean(cuda):
    from hlhgat import ops
    from hlhgat.hodge_cheb_conv import cluster_mean
    g = torch.Generator().manual_seed(4)
    x = torch.randn(1000, 48, generator=g)
    assign = torch.randint(0, 77, (1000,), generator=g)
    xd = dev(x).requires_grad_(True)
    out = cluster_mean(xd, dev(assign))
    xr = x.clone().requires_grad_(True)
    outr = R.scatter_mean(xr, assign)
    close(out.detach().cpu(), outr.detach(), 1e-6, "scatter_mean")
    Rg = torch.randn(outr.shape, generator=g)
    (out * dev(Rg)).sum().backward()
    (outr * Rg).sum().backward()
    close(xd.grad.cpu(), xr.grad, 1e-6, "scatter_mean grad")


# ---------------------------------------------------------------------------
# whole model (lib/Hodge_ST_Model.py:544-646)
# ---------------------------------------------------------------------------
def test_zinc_model_vs_reference_golden(cuda):
    import hlhgat
    from hlhgat.hodge_dataset import Batch
    g = load_golden("zinc_model_small")
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[1, 1], filters=[16, 16],
                                            mlp_channels=[32], K=3, keig=15)
    m.load_state_dict({k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")})
    m = m.to(cuda).train()
    b = Batch()
    for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
              "edge_index", "num_node1", "num_edge1"):
        setattr(b, k, dev(g[k]))
    out = m(b)
    close(out.detach().cpu(), g["out"], 1e-4, "out")
    (out * dev(g["R"])).sum().backward()
    for k, p in m.named_parameters():
        close(p.grad.cpu(), g["grad/" + k], 1e-4, "grad " + k)


def test_tsp_model_vs_reference_golden(cuda):
    """HL_HGCNN_TSP_dense_int3_pyr (lib/Hodge_ST_Model.py:756-855, config 5
    head) against the reference's own forward / backward on two small
    TSP-like graphs (tests/golden/make_golden.py tsp_case): reference state
    dict loaded unchanged, masked edge logits and every parameter gradient
    within 1e-4 relative."""
    import hlhgat
    from hlhgat.hodge_dataset import Batch
    g = load_golden("tsp_model_small")
    m = hlhgat.HL_HGCNN_TSP_dense_int3_pyr(channels=[1, 1], filters=[16, 16],
                                           mlp_channels=[32], K=3)
    m.load_state_dict({k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")})
    m = m.to(cuda).train()
    b = Batch()
    for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
              "edge_index", "num_node1", "num_edge1"):
        setattr(b, k, dev(g[k]))
    out, s_batch = m(b)
    assert torch.equal(s_batch.cpu(), T(g["s_batch"]))
    close(out.detach().cpu(), g["out"], 1e-4, "out")
    (out * dev(g["R"])).sum().backward()
    import re
    for k, p in m.named_parameters():
        if re.search(r"module_[04]\.bias$", k) and not k.startswith("out."):
            # bias of a conv/linear that feeds a training-mode BatchNorm: its gradient
            # is analytically 0 (BN removes any per-channel shift); both sides
            # hold only fp32 rounding noise, compared as such
            assert float(p.grad.abs().max()) < 1e-3 and float(np.abs(g["grad/" + k]).max()) < 1e-3
            continue
        close(p.grad.cpu(), g["grad/" + k], 1e-4, "grad " + k)


def test_boundary_transpose_matches_sparse_mm(cuda):
    """ops.boundary_t == torch.sparse.mm(adj2par1(...).T, x) bitwise, and its
    adjoint == B1 @ g (reference readout, lib/Hodge_ST_Model.py:846)."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import adj2par1
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(20, seed=4)
    par = adj2par1(b.edge_index, b.x_t.shape[0], b.x_s.shape[0])
    B1 = par.to_sparse_coo()
    x = torch.randn(b.x_t.shape[0], 24, generator=torch.Generator().manual_seed(1))
    ref = torch.sparse.mm(B1.t().coalesce(), x)
    pard = adj2par1(dev(b.edge_index), b.x_t.shape[0], b.x_s.shape[0])
    xd = dev(x).requires_grad_(True)
    y = ops.boundary_t(xd, pard.incidence())
    assert torch.equal(y.detach().cpu(), ref)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(2))
    y.backward(dev(gy))
    assert torch.equal(xd.grad.cpu(), torch.sparse.mm(B1.coalesce(), gy))


def test_zinc_model_cfg2_vs_oracle(cuda):
    """BASELINE config 2 model at a 200-graph batch: HIP product vs oracle.

    Tolerance: forward output 1e-4 relative.  Gradients pass through 6 blocks of
    batch-statistics BN + ReLU, where they are ill-conditioned: the fp32 oracle
    itself deviates from an fp64 evaluation by up to ~3e-2 (relative, max-norm)
    on deep-layer weight gradients, and a 1e-6 relative change of the weights
    moves the fp64 gradients by as much (pre-ReLU values within rounding of 0
    flip masks).  So each parameter gradient of the HIP path must be within 3x
    the larger of the fp32 oracle's distance to fp64 and that conditioning
    (two perturbed fp64 runs), floor 1e-4 relative (tests/test_baseline_configs.py
    applies the same gate to configs 3-5)."""
    import hlhgat
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(200, seed=21)
    kw = dict(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256], K=3, keig=15)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**kw)
    ref = R.RefZincModel(**kw)
    ref.load_state_dict(m.state_dict())
    ref64 = R.RefZincModel(**kw).double()
    ref64.load_state_dict({k: v.double() if v.is_floating_point() else v
                           for k, v in m.state_dict().items()})
    m, ref, ref64 = m.to(cuda).train(), ref.train(), ref64.train()

    class _D:
        pass

    b64 = _D()
    for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
              "edge_index", "num_node1", "num_edge1"):
        v = getattr(b, k)
        setattr(b64, k, v.double() if v.is_floating_point() else v)
    out_r = ref(b)
    out_64 = ref64(b64)
    pert = []
    for ps in (0, 1):  # conditioning probe: fp64 at weights * (1 + 1e-6 N(0,1))
        mp = R.RefZincModel(**kw).double()
        mp.load_state_dict(ref64.state_dict())
        gen = torch.Generator().manual_seed(ps)
        with torch.no_grad():
            for p in mp.parameters():
                p.mul_(1 + 1e-6 * torch.randn(p.shape, generator=gen, dtype=torch.float64))
        pert.append((mp.train(), mp(b64)))
    bd = zinc_like_batch(200, seed=21).to(cuda)
    out = m(bd)
    close(out.detach().cpu(), out_r.detach(), 1e-4, "out")
    Rg = torch.randn(out_r.shape)
    (out * dev(Rg)).sum().backward()
    (out_r * Rg).sum().backward()
    (out_64 * Rg.double()).sum().backward()
    for mp, op in pert:
        (op * Rg.double()).sum().backward()
    rp = dict(ref.named_parameters())
    r64 = dict(ref64.named_parameters())
    pp = [dict(mp.named_parameters()) for mp, _ in pert]
    from test_baseline_configs import write_gate_log
    rows = []
    for k, p in m.named_parameters():
        e = r64[k].grad
        scale = max(1.0, e.abs().max().item())
        err_ref = (rp[k].grad.double() - e).abs().max().item() / scale
        cond = max((q[k].grad - e).abs().max().item() / scale for q in pp)
        err_hip = (p.grad.cpu().double() - e).abs().max().item() / scale
        rows.append({"param": k, "err": err_hip, "bound": max(3 * max(err_ref, cond), 1e-4),
                     "err_fp32_oracle": err_ref, "cond": cond})
    write_gate_log("cond_cfg2_zinc_200", rows)
    for r in rows:
        assert r["err"] <= r["bound"], r


# ---------------------------------------------------------------------------
# fused BatchNorm1d (+ReLU), training statistics
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n,C,relu", [(2, 1, False), (23000, 64, True), (1000, 256, True),
                                      (4097, 18, False), (777, 130, True), (50, 384, False)])
def test_batch_norm_act_vs_torch(cuda, n, C, relu):
    from hlhgat import ops
    g = torch.Generator().manual_seed(n + C)
    x = torch.randn(n, C, generator=g) * 3 + 1.5
    bn_ref = torch.nn.BatchNorm1d(C)
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.5, 0.5)
        bn_ref.running_mean.uniform_(-1, 1)
        bn_ref.running_var.uniform_(0.5, 2)
    bn = torch.nn.BatchNorm1d(C).to(cuda)
    bn.load_state_dict(bn_ref.state_dict())
    bn.train()
    bn_ref.train()
    xr = x.clone().requires_grad_(True)
    yr = bn_ref(xr)
    if relu:
        yr = torch.relu(yr)
    xd = dev(x).requires_grad_(True)
    y = ops.batch_norm_act(xd, bn, relu=relu)
    close(y.detach().cpu(), yr.detach(), 1e-5, "y")
    Rg = torch.randn(n, C, generator=g)
    (yr * Rg).sum().backward()
    (y * dev(Rg)).sum().backward()
    close(xd.grad.cpu(), xr.grad, 1e-4, "dx")
    close(bn.weight.grad.cpu(), bn_ref.weight.grad, 1e-4, "dw")
    close(bn.bias.grad.cpu(), bn_ref.bias.grad, 1e-4, "db")
    close(bn.running_mean.cpu(), bn_ref.running_mean, 1e-5, "running_mean")
    close(bn.running_var.cpu(), bn_ref.running_var, 1e-5, "running_var")
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    # a second call reuses the (self-resetting) workspace counters
    with torch.no_grad():
        y2 = ops.batch_norm_act(xd.detach(), bn, relu=relu)
    close(y2.cpu(), y.detach().cpu(), 1e-6, "repeat")


@pytest.mark.parametrize("d,dv", [(64, 64), (96, 64), (40, 24)])
def test_nei_value_projected_first_matches_gather_first(cuda, d, dv, monkeypatch):
    """NEIntValueFn (first Linear projected before the |B1| gathers) against
    the gather-then-Linear path of the reference's operation order: outputs
    1e-5, gradients 1e-4 relative, BN running statistics 1e-5."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(60, seed=21)
    N_t, N_s = b.x_t.shape[0], b.x_s.shape[0]
    g = torch.Generator().manual_seed(d)
    xt0, xs0 = torch.randn(N_t, d, generator=g), torch.randn(N_s, d, generator=g)
    Rt, Rs = torch.randn(N_t, dv, generator=g), torch.randn(N_s, dv, generator=g)
    D = R.degree(b.edge_index.reshape(-1), N_t)
    torch.manual_seed(3)
    m0 = hlhgat.NodeEdgeInt(d=d, dv=dv)
    sd0 = {k: v.clone() for k, v in m0.state_dict().items()}

    def run(fused):
        m = hlhgat.NodeEdgeInt(d=d, dv=dv)
        m.load_state_dict(sd0)
        m = m.to(cuda).train()
        if not fused:
            monkeypatch.setattr(ops, "nei_value", lambda *a, **k: None)
        x_t = dev(xt0).requires_grad_(True)
        x_s = dev(xs0).requires_grad_(True)
        par = hlhgat.adj2par1(dev(b.edge_index), N_t, N_s)
        a, c = m(x_t, x_s, par, dev(D))
        ((a * dev(Rt)).sum() + (c * dev(Rs)).sum()).backward()
        monkeypatch.undo()
        res = {"out_t": a, "out_s": c, "gx_t": x_t.grad, "gx_s": x_s.grad}
        res.update({"grad/" + k: p.grad for k, p in m.named_parameters()})
        res.update({"buf/" + k: v for k, v in m.state_dict().items() if "running" in k})
        return {k: v.detach().cpu() for k, v in res.items()}

    ref, new = run(False), run(True)
    for k in ref:
        close(new[k], ref[k], 1e-4 if k.startswith(("g", "grad")) else 1e-5, k)


class _BnWait:
    """hlhgat_set_bn_wait_us for the duration of a with-block (0 forces every
    waiting one-launch BatchNorm workgroup to hand its rows to the finaliser
    unless the statistics are already final), restoring the default after."""

    def __init__(self, us):
        self.us = us

    def __enter__(self):
        from hlhgat import _lib
        _lib.check(_lib.LIB.hlhgat_set_bn_wait_us(self.us), "set_bn_wait_us")

    def __exit__(self, *exc):
        from hlhgat import _lib
        _lib.LIB.hlhgat_set_bn_wait_us(1000)


@pytest.mark.parametrize("d,dv", [(64, 64), (96, 64), (40, 24)])
def test_nei_bn_handover_bitwise(cuda, d, dv):
    """NodeEdgeInt (its two one-launch BatchNorms per side) with every waiting
    BatchNorm workgroup handing its rows to the finaliser (wait bound 0) ==
    the default, bit for bit: outputs, input gradients, every parameter
    gradient and the running statistics (dv = 24: the unaligned width takes
    the two-launch BatchNorm either way)."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(60, seed=23)
    N_t, N_s = b.x_t.shape[0], b.x_s.shape[0]
    g = torch.Generator().manual_seed(d)
    xt0, xs0 = torch.randn(N_t, d, generator=g), torch.randn(N_s, d, generator=g)
    Rt, Rs = torch.randn(N_t, dv, generator=g), torch.randn(N_s, dv, generator=g)
    D = R.degree(b.edge_index.reshape(-1), N_t)
    torch.manual_seed(5)
    sd0 = {k: v.clone() for k, v in hlhgat.NodeEdgeInt(d=d, dv=dv).state_dict().items()}

    def run():
        m = hlhgat.NodeEdgeInt(d=d, dv=dv)
        m.load_state_dict(sd0)
        m = m.to(cuda).train()
        x_t = dev(xt0).requires_grad_(True)
        x_s = dev(xs0).requires_grad_(True)
        par = hlhgat.adj2par1(dev(b.edge_index), N_t, N_s)
        a, c = m(x_t, x_s, par, dev(D))
        ((a * dev(Rt)).sum() + (c * dev(Rs)).sum()).backward()
        res = {"out_t": a, "out_s": c, "gx_t": x_t.grad, "gx_s": x_s.grad}
        res.update({"grad/" + k: p.grad for k, p in m.named_parameters()})
        res.update({"buf/" + k: v for k, v in m.state_dict().items() if "running" in k})
        return {k: v.detach().cpu() for k, v in res.items()}

    base = run()
    ops.bn_giveups_reset()
    with _BnWait(0):
        handed = run()
    gu = ops.bn_giveups()
    ops.check_device_errors()
    for k in base:
        assert torch.equal(base[k], handed[k]), k
    if dv % 4 == 0:
        assert gu["count"] > 0  # the hand-over path did run


# ---------------------------------------------------------------------------
# row schedules (locality_order) and XCD-aware slots never change results
# ---------------------------------------------------------------------------
def test_row_schedule_is_bitwise_neutral(cuda):
    from hlhgat import ops
    from hlhgat.hodge_dataset import locality_order
    from hlhgat.synthetic import tsp_like_graph
    g = tsp_like_graph(1, n=2000, k=6)
    ei, w, n = g.edge_index_s, g.edge_weight_s, g.x_s.shape[0]
    x = torch.randn(n, 64, generator=torch.Generator().manual_seed(0))
    ref = R.propagate(x, ei, w)
    ei_d = ops.mark_hodge(dev(ei))
    op = ops.hodge_operator(ei_d, dev(w), n)
    y0 = ops.spmm(op.fwd, dev(x))
    for order in (locality_order(ei.numpy(), n), torch.randperm(n)):
        ei_o = ops.set_row_order(ops.mark_hodge(dev(ei)), order)
        op_o = ops.hodge_operator(ei_o, dev(w), n)
        assert op_o.fwd.order is not None
        y = ops.spmm(op_o.fwd, dev(x))
        assert torch.equal(y, y0)
        assert torch.equal(y.cpu(), ref)
        T0 = ops.poly_basis(op, dev(x), 4, ops.POLY_LAGUERRE)
        T1 = ops.poly_basis(op_o, dev(x), 4, ops.POLY_LAGUERRE)
        assert torch.equal(T0, T1)


def test_conv_with_row_schedule_matches(cuda):
    """HodgeLaguerreConv forward + backward with a scheduled operator equal
    the natural-order results bitwise (TSP-like graph, config 5 shape)."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.synthetic import tsp_like_graph
    g = tsp_like_graph(2, n=1500, k=6)
    n = g.x_s.shape[0]
    torch.manual_seed(0)
    conv = hlhgat.HodgeLaguerreConv(32, 32, K=4).to(cuda)
    x = torch.randn(n, 32, device=cuda)
    outs = []
    for sched in (False, True):
        ei = ops.mark_hodge(dev(g.edge_index_s))
        if sched:
            ops.set_row_order(ei, g.row_order_s)
        xx = x.clone().requires_grad_(True)
        y = conv(xx, ei, dev(g.edge_weight_s))
        (y * y).sum().backward()
        outs.append((y.detach(), xx.grad.clone(), conv.lins[2].weight.grad.clone()))
        conv.zero_grad()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


# ---------------------------------------------------------------------------
# LDS-staged halo-tile SpMM (k_poly_halo) == plain SpMM, bitwise
# ---------------------------------------------------------------------------
def _halo_ops(g, side, max_rows, max_halo):
    from hlhgat import ops
    from hlhgat.hodge_dataset import halo_tiles
    ei, w = getattr(g, "edge_index_" + side), getattr(g, "edge_weight_" + side)
    n = getattr(g, "x_" + side).shape[0]
    order = getattr(g, "row_order_" + side)
    plain = ops.hodge_operator(ops.set_row_order(ops.mark_hodge(dev(ei)), order), dev(w), n)
    ht = halo_tiles(ei.numpy(), n, order.numpy(), max_rows=max_rows, max_halo=max_halo)
    ei_h = ops.set_row_order(ops.mark_hodge(dev(ei)), order)
    ops.set_halo(ei_h, ht)
    halo = ops.hodge_operator(ei_h, dev(w), n)
    assert halo.fwd.halo is not None and plain.fwd.halo is None
    return ei, w, n, plain, halo, ei_h


@pytest.mark.parametrize("d", [1, 6, 32, 64, 128, 200])
@pytest.mark.parametrize("tiles", [(128, 256), (7, 48)])
def test_halo_spmm_bitwise_equals_plain(cuda, d, tiles):
    from hlhgat import ops
    from hlhgat.synthetic import tsp_like_graph
    g = tsp_like_graph(6, n=1200, k=7, halo=False)
    for side in ("s", "t"):
        ei, w, n, plain, halo, _ = _halo_ops(g, side, *tiles)
        x = torch.randn(n, d, generator=torch.Generator().manual_seed(d))
        y0 = ops.spmm(plain.fwd, dev(x))
        y1 = ops.spmm(halo.fwd, dev(x))
        assert torch.equal(y0, y1), (side, d, (y0 - y1).abs().max())
        assert torch.equal(y1.cpu(), R.propagate(x, ei, w))
        for kind in (ops.POLY_LAGUERRE, ops.POLY_CHEB, ops.POLY_LAGUERRE_DEMO):
            assert torch.equal(ops.poly_basis(plain, dev(x), 4, kind),
                               ops.poly_basis(halo, dev(x), 4, kind))


def test_halo_conv_fwd_bwd_bitwise(cuda):
    """HodgeLaguerreConv (+BN+ReLU node) forward and adjoint over halo tiles
    equal the plain path bitwise; batch of two TSP-like graphs via collate."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph
    b = collate([tsp_like_graph(7, n=900, k=7), tsp_like_graph(8, n=700, k=7)],
                check_hodge=False)
    n = b.x_s.shape[0]
    torch.manual_seed(0)
    conv = hlhgat.HodgeLaguerreConv(64, 64, K=4).to(cuda)
    bn = torch.nn.BatchNorm1d(64).to(cuda)
    x = torch.randn(n, 64, device=cuda)
    outs = []
    for use_halo in (False, True):
        bd = collate([tsp_like_graph(7, n=900, k=7), tsp_like_graph(8, n=700, k=7)],
                     check_hodge=False).to(cuda)
        if use_halo:
            assert getattr(bd.edge_index_s, "_hlhgat_halo", None) is not None
        else:
            bd.edge_index_s._hlhgat_halo = None
        op = ops.hodge_operator(bd.edge_index_s, bd.edge_weight_s, n)
        assert (op.fwd.halo is not None) == use_halo
        xx = x.clone().requires_grad_(True)
        y = conv.forward_bn(xx, bd.edge_index_s, bd.edge_weight_s, bn, relu=True)
        (y * y).sum().backward()
        outs.append((y.detach(), xx.grad.clone(), conv.lins[3].weight.grad.clone()))
        conv.zero_grad()
    for a, c in zip(*outs):
        assert torch.equal(a, c)


def _attpool_case(cuda, name, cls, **kw):
    import re
    from hlhgat.hodge_dataset import Batch
    g = load_golden(name)
    m = cls(**kw)
    m.load_state_dict({k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")})
    m = m.to(cuda).train()
    datas = []
    for lv in range(2):
        b = Batch()
        for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s",
                  "edge_weight_s", "edge_index", "num_node1", "num_edge1"):
            setattr(b, k, dev(g[f"l{lv}/{k}"]))
        datas.append(b)
    out = m(datas)
    close(out.detach().cpu(), g["out"], 1e-4, "out")
    (out * dev(g["R"])).sum().backward()
    for k, p in m.named_parameters():
        if "nograd/" + k in g:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
            continue
        if re.search(r"module_[04]\.bias$", k) or re.search(r"mlp\d+\.0\.bias$", k) or \
                re.search(r"WV_(Node|Edge)\.[03]\.bias$", k):
            # bias feeding a training-mode BatchNorm: analytically zero gradient
            assert float(p.grad.abs().max()) < 1e-3 and float(np.abs(g["grad/" + k]).max()) < 1e-3
            continue
        close(p.grad.cpu(), g["grad/" + k], 1e-4, "grad " + k)


def test_attpool_cifar_model_vs_reference_golden(cuda):
    """HL_HGCNN_CIFAR10SP_dense_int3_attpool (lib/Hodge_ST_Model.py:958-1091,
    config 3 head): two MLGC levels, NEAtt(ReLU) / batch max at pool_loc,
    inf-masked cluster means, level switch, readout; reference forward and
    every parameter gradient within 1e-4 relative."""
    import hlhgat
    _attpool_case(cuda, "attpool_cifar_small", hlhgat.HL_HGCNN_CIFAR10SP_dense_int3_attpool,
                  channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10,
                  pool_loc=0, l=0.5)


def test_attpool_pepfunc_model_vs_reference_golden(cuda):
    """HL_HGCNN_pepfunc_dense_int3_attpool (main_pepfunc...:36-168, config 4
    head): NEAtt(sigmoid, l=0.5) on the dense concatenation after every level."""
    import hlhgat
    _attpool_case(cuda, "attpool_pepfunc_small", hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool,
                  channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)


def test_attpool_zinc_model_vs_reference_golden(cuda):
    """HL_HGCNN_zinc_dense_int3_attpool (lib/Hodge_ST_Model.py:412-541): K-order
    initial convs, NEAtt(ReLU) on the block output without the batch-max
    division, bare degree; reference forward and every gradient (its NEAtt
    gets none: the scaled block output is overwritten by the next level)."""
    import hlhgat
    _attpool_case(cuda, "head_zinc_attpool_small", hlhgat.HL_HGCNN_zinc_dense_int3_attpool,
                  channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, node_dim=5,
                  edge_dim=4, keig=10, pool_loc=0)


def test_attpool_pepfunc_lib_model_vs_reference_golden(cuda):
    """The library's HL_HGCNN_pepfunc_dense_int3_attpool (lib/Hodge_ST_Model.py:
    173-304: NEAtt only at pool_loc, on the dense concatenation, l=0.9; the
    training script shadows it with hlhgat.main_pepfunc's)."""
    from hlhgat import hodge_st_model
    _attpool_case(cuda, "head_pepfunc_attpool_lib_small",
                  hodge_st_model.HL_HGCNN_pepfunc_dense_int3_attpool,
                  channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)


def _pyr_case(cuda, name, cls, **kw):
    import re
    from hlhgat.hodge_dataset import Batch
    g = load_golden(name)
    m = cls(**kw)
    m.load_state_dict({k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")})
    m = m.to(cuda).train()
    b = Batch()
    for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
              "edge_index", "num_node1", "num_edge1"):
        setattr(b, k, dev(g[k]))
    out = m(b)
    close(out.detach().cpu(), g["out"], 1e-4, "out")
    (out * dev(g["R"])).sum().backward()
    for k, p in m.named_parameters():
        if re.search(r"module_[04]\.bias$", k) or re.search(r"mlp\d+\.0\.bias$", k):
            # bias feeding a training-mode BatchNorm: analytically zero gradient
            assert float(p.grad.abs().max()) < 1e-3 and float(np.abs(g["grad/" + k]).max()) < 1e-3
            continue
        close(p.grad.cpu(), g["grad/" + k], 1e-4, "grad " + k)


@pytest.mark.parametrize("name,cls,kw", [
    ("head_pepfunc_pyr_small", "HL_HGCNN_pepfunc_dense_int3_pyr",
     dict(channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, node_dim=21, edge_dim=3,
          keig=15)),
    ("head_cifar_pyr_small", "HL_HGCNN_CIFAR10SP_dense_int3_pyr",
     dict(channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, node_dim=21, edge_dim=3,
          keig=15, l=0.5)),
    ("head_zinc_poolint3_small", "HL_HGCNN_zinc_dense_poolint3_pyr",
     dict(channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, keig=15))])
def test_pyr_heads_vs_reference_golden(cuda, name, cls, kw):
    """The pyramid heads of lib/Hodge_ST_Model.py beside the ZINC one:
    pepfunc (:307-407, degree + 1e-6), CIFAR10SP (:858-955, K=1 initial convs)
    and ZINC poolint3 (:649-749, the interaction after the convs of a level):
    the reference's forward and every parameter gradient, its state_dict
    loaded unchanged, within 1e-4 relative."""
    import hlhgat
    _pyr_case(cuda, name, getattr(hlhgat, cls), **kw)


# ---------------------------------------------------------------------------
# Hodge-factored L1 (L1 = alpha B1^T B1, hlhgat_hodge_factor_t): same
# real-arithmetic operator, different fp32 rounding -- 1e-5 relative, not bitwise
# ---------------------------------------------------------------------------
def _factored_pair(g, node_order=None, edge_order=None):
    from hlhgat import ops
    n = g.x_s.shape[0]
    ei_c = ops.mark_hodge(dev(g.edge_index_s))
    ei_f = ops.mark_hodge(dev(g.edge_index_s))
    if edge_order is not None:
        ops.set_row_order(ei_f, edge_order)
    ops.set_hodge_factor(ei_f, dev(g.edge_index), g.x_t.shape[0], node_order)
    w = dev(g.edge_weight_s)
    op_c = ops.hodge_operator(ei_c, w, n)
    op_f = ops.hodge_operator(ei_f, w, n)
    assert op_c.factor is None and op_f.factor is not None
    return op_c, op_f, ei_c, ei_f, w


@pytest.mark.parametrize("d", [1, 3, 32, 64, 128])
@pytest.mark.parametrize("sched", [False, True])
def test_hodge_factored_spmm_matches_csr(cuda, d, sched):
    """alpha B1^T (B1 X) == the CSR SpMM of L1 == the oracle's propagate
    (TSP-like graph, config 5 structure; RCM schedules on both factors)."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import hodge_factor_ok
    from hlhgat.synthetic import tsp_like_graph
    g = tsp_like_graph(5, n=3000, k=9)
    assert hodge_factor_ok(g.edge_index, g.x_t.shape[0], g.edge_index_s, g.edge_weight_s)
    op_c, op_f, *_ = _factored_pair(g, g.row_order_t if sched else None,
                                    g.row_order_s if sched else None)
    x = torch.randn(g.x_s.shape[0], d, generator=torch.Generator().manual_seed(d))
    ref = R.propagate(x, g.edge_index_s, g.edge_weight_s)
    y = ops.hodge_spmm(op_f, dev(x)).cpu()
    assert torch.equal(ops.spmm(op_c.fwd, dev(x)).cpu(), ref)
    close(y, ref, 1e-5, "factored spmm")


@pytest.mark.parametrize("kind,K", [("lag", 2), ("lag", 4), ("cheb", 4), ("demo", 4)])
def test_hodge_factored_basis_matches_csr(cuda, kind, K):
    from hlhgat import ops
    from hlhgat.synthetic import tsp_like_graph
    kd = {"lag": ops.POLY_LAGUERRE, "cheb": ops.POLY_CHEB, "demo": ops.POLY_LAGUERRE_DEMO}[kind]
    g = tsp_like_graph(6, n=2000, k=8)
    op_c, op_f, *_ = _factored_pair(g, g.row_order_t, g.row_order_s)
    x = dev(torch.randn(g.x_s.shape[0], 48, generator=torch.Generator().manual_seed(1)))
    Tc = ops.poly_basis(op_c, x, K, kd).cpu()
    Tf = ops.poly_basis(op_f, x, K, kd).cpu()
    for k in range(K - 1):
        close(Tf[k], Tc[k], 1e-5, f"T_{k + 1}")


@pytest.mark.parametrize("kind", ["lag", "cheb"])
def test_hodge_factored_conv_bn_fwd_bwd(cuda, kind):
    """HodgeLaguerreConv / HodgeChebConv -> BN -> ReLU (one C++ node) on a
    factored L1: output, dX and every parameter gradient vs the CSR operator."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.synthetic import cifar_like_graphs
    from hlhgat.hodge_dataset import collate
    b = collate([cifar_like_graphs(60 + s)[0] for s in range(4)])
    assert b.l1_factor
    cls = hlhgat.HodgeLaguerreConv if kind == "lag" else hlhgat.HodgeChebConv
    torch.manual_seed(0)
    conv = cls(32, 32, K=4).to(cuda)
    bn = torch.nn.BatchNorm1d(32).to(cuda)
    x = torch.randn(b.x_s.shape[0], 32, device=cuda)
    res = []
    for factored in (False, True):
        ei = ops.mark_hodge(dev(b.edge_index_s))
        if factored:
            ops.set_hodge_factor(ei, dev(b.edge_index), b.x_t.shape[0])
        op = ops.hodge_operator(ei, dev(b.edge_weight_s), b.x_s.shape[0])
        assert (op.factor is not None) == factored
        xx = x.clone().requires_grad_(True)
        y = ops.hodge_poly_conv(xx, op, [l.weight for l in conv.lins], conv.bias,
                                ops.POLY_LAGUERRE if kind == "lag" else ops.POLY_CHEB,
                                bn=bn, relu=True)
        (y * torch.linspace(-1, 1, y.numel(), device=cuda).view_as(y)).sum().backward()
        res.append([y.detach().cpu(), xx.grad.cpu()] +
                   [l.weight.grad.cpu().clone() for l in conv.lins] + [bn.weight.grad.cpu().clone()])
        conv.zero_grad()
        bn.zero_grad()
    for i, (a, c) in enumerate(zip(res[1], res[0])):
        close(a, c, 1e-5 if i == 0 else 1e-4, f"item {i}")


def test_tsp_model_factored_vs_reference_golden(cuda):
    """The config-5 head with its L1 factored (set_hodge_factor) against the
    reference's own forward / backward (tsp_model_small): 1e-4 relative."""
    import re
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import Batch, hodge_factor_ok
    g = load_golden("tsp_model_small")
    assert hodge_factor_ok(g["edge_index"], g["x_t"].shape[0], g["edge_index_s"],
                           g["edge_weight_s"])
    m = hlhgat.HL_HGCNN_TSP_dense_int3_pyr(channels=[1, 1], filters=[16, 16],
                                           mlp_channels=[32], K=3)
    m.load_state_dict({k[3:]: T(v) for k, v in g.items() if k.startswith("sd/")})
    m = m.to(cuda).train()
    b = Batch()
    for k in ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
              "edge_index", "num_node1", "num_edge1"):
        setattr(b, k, dev(g[k]))
    ops.mark_hodge(b.edge_index_s)
    ops.set_hodge_factor(b.edge_index_s, b.edge_index, b.x_t.shape[0])
    out, _ = m(b)
    assert ops.hodge_operator(b.edge_index_s, b.edge_weight_s, b.x_s.shape[0]).factor is not None
    close(out.detach().cpu(), g["out"], 1e-4, "out")
    (out * dev(g["R"])).sum().backward()
    for k, p in m.named_parameters():
        if re.search(r"module_[04]\.bias$", k) and not k.startswith("out."):
            assert float(p.grad.abs().max()) < 1e-3 and float(np.abs(g["grad/" + k]).max()) < 1e-3
            continue
        close(p.grad.cpu(), g["grad/" + k], 1e-4, "grad " + k)


@pytest.mark.parametrize("side,factored", [("t", False), ("s", False), ("s", True)])
def test_brain_skeleton_conv_vs_reference_golden(cuda, side, factored):
    """HodgeLaguerreConv(8, 8, K=3) on the reference's brain skeleton
    (HL-HGAT-DEMO data: 268 nodes, 8997 edges, nnz(L1) 1.37 M, 152 entries
    per L1 row; L0 / L1 rebuilt bitwise by hodge_coo_from_boundary) against
    the reference's forward and gradients: CSR operator and factored L1."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import hodge_coo_from_boundary
    g = load_golden("brain_skeleton")
    n = int(g["n_nodes"])
    ei_t, w_t, ei_s, w_s = hodge_coo_from_boundary(g["edge_index"], n, float(g["lmax"]))
    e, w = (ei_t, w_t) if side == "t" else (ei_s, w_s)
    e = ops.mark_hodge(dev(e))
    if factored:
        ops.set_hodge_factor(e, dev(g["edge_index"]), n)
    conv = hlhgat.HodgeLaguerreConv(8, 8, K=3).to(cuda)
    with torch.no_grad():
        for k, lin in enumerate(conv.lins):
            lin.weight.copy_(dev(g[f"{side}/w{k}"]))
        conv.bias.copy_(dev(g[f"{side}/bias"]))
    x = dev(g[f"{side}/x"]).requires_grad_(True)
    out = conv(x, e, dev(w))
    assert (ops.hodge_operator(e, dev(w), x.shape[0]).factor is not None) == factored
    close(out.detach().cpu(), g[f"{side}/out"], 1e-5, "out")
    (out * dev(g[f"{side}/R"])).sum().backward()
    close(x.grad.cpu(), g[f"{side}/gx"], 1e-4, "dx")
    close(conv.bias.grad.cpu(), g[f"{side}/gbias"], 1e-4, "dbias")
    for k, lin in enumerate(conv.lins):
        close(lin.weight.grad.cpu(), g[f"{side}/gw{k}"], 1e-4, f"dW{k}")


def test_hodge_factored_edge_cases(cuda):
    """Factored L1 on a batch with isolated nodes (empty incidence rows), a
    single-edge graph, a star (one node in every edge) and a triangle: equals
    the CSR SpMM / basis; hodge_factor_ok holds for each graph."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import PairData, collate, hodge_coo_from_boundary, hodge_factor_ok
    graphs = []
    for ei, n in ((np.array([[0], [1]]), 2), (np.array([[0, 0, 0, 0], [1, 2, 3, 4]]), 6),
                  (np.array([[0, 0, 1], [1, 2, 2]]), 3), (np.array([[1, 2], [2, 4]]), 7)):
        ei_t, w_t, ei_s, w_s = hodge_coo_from_boundary(ei, n, 3.0)
        assert hodge_factor_ok(ei, n, ei_s.numpy(), w_s.numpy())
        g = PairData(x_s=torch.randn(ei.shape[1], 4), edge_index_s=ei_s, edge_weight_s=w_s,
                     x_t=torch.randn(n, 4), edge_index_t=ei_t, edge_weight_t=w_t)
        g.edge_index = torch.from_numpy(ei)
        g.num_node1, g.num_edge1, g.num_nodes = n, ei.shape[1], n
        g._hodge_sorted = True
        graphs.append(g)
    b = collate(graphs)
    E = b.x_s.shape[0]
    op_c = ops.hodge_operator(ops.mark_hodge(dev(b.edge_index_s)), dev(b.edge_weight_s), E)
    e = ops.mark_hodge(dev(b.edge_index_s))
    ops.set_hodge_factor(e, dev(b.edge_index), b.x_t.shape[0])
    op_f = ops.hodge_operator(e, dev(b.edge_weight_s), E)
    for d in (1, 4, 64):
        x = dev(torch.randn(E, d, generator=torch.Generator().manual_seed(d)))
        close(ops.hodge_spmm(op_f, x).cpu(), ops.spmm(op_c.fwd, x).cpu(), 1e-5, f"spmm d={d}")
        Tf = ops.poly_basis(op_f, x, 4, ops.POLY_LAGUERRE).cpu()
        Tc = ops.poly_basis(op_c, x, 4, ops.POLY_LAGUERRE).cpu()
        close(Tf, Tc, 1e-5, f"basis d={d}")


def test_device_hodge_builder_matches_reference(cuda):
    """On-device Hodge builder (hlhgat_hodge_lmax / _build) on the reference's
    brain skeleton and a batch of ZINC-like molecules: with the reference's
    lmax the COO equals the reference construction bitwise (brain: sampled
    entries + checksums from the reference; molecules: the host dense
    restatement); the on-device Lanczos lmax equals float32 eigh to 2e-6
    relative; a conv on the device-built L1 matches the golden output."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate, hodge_laplacians, dense_to_sparse
    from hlhgat.synthetic import zinc_like_graph
    g = load_golden("brain_skeleton")
    n = int(g["n_nodes"])
    ei = dev(g["edge_index"])
    ei_t, w_t, ei_s, w_s, lam = ops.hodge_build(ei, [n], torch.tensor([float(g["lmax"])]))
    for side, (e, w) in {"t": (ei_t, w_t), "s": (ei_s, w_s)}.items():
        e, w = e.cpu().numpy(), w.cpu().numpy()
        assert e.shape[1] == int(g[f"nnz_{side}"])
        idx = g[f"{side}/coo_idx"]
        assert np.array_equal(e[:, idx], g[f"{side}/coo_rc"])
        assert np.array_equal(w[idx], g[f"{side}/coo_w"])
        assert float(np.asarray(w, np.float64).sum()) == float(g[f"{side}/w_sum64"])
    *_, lam_dev = ops.hodge_build(ei, [n])
    assert abs(float(lam_dev[0]) - float(g["lmax"])) <= 2e-6 * float(g["lmax"])
    # molecules: batch of 6 graphs, reference dense construction per graph
    gs = [zinc_like_graph(700 + i) for i in range(6)]
    b = collate(gs)
    lams = [float(hodge_laplacians(gg.edge_index.numpy(), gg.x_t.shape[0])[2]) for gg in gs]
    ei_t, w_t, ei_s, w_s, _ = ops.hodge_build(dev(b.edge_index), b.num_node1.tolist(),
                                              torch.tensor(lams))
    assert torch.equal(ei_t.cpu(), b.edge_index_t) and torch.equal(w_t.cpu(), b.edge_weight_t)
    assert torch.equal(ei_s.cpu(), b.edge_index_s) and torch.equal(w_s.cpu(), b.edge_weight_s)
    *_, lam_d = ops.hodge_build(dev(b.edge_index), b.num_node1.tolist())
    close(lam_d.cpu(), torch.tensor(lams), 2e-6, "lanczos lmax")


def test_hodge_build_undersized_raises(cuda):
    """sizes= smaller (a caller's simple-graph formula given other
    input) or larger than the graph's Laplacians: the build
    kernels write nothing past the buffers and raise HLHGAT_DEVERR_HODGE_SIZE;
    exact sizes stay
    clean and bitwise the sizes=None build."""
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import zinc_like_graph
    b = collate([zinc_like_graph(720 + i) for i in range(4)])
    ei = dev(b.edge_index)
    N = int(b.num_node1.sum())
    lam = torch.ones(4)
    ops.check_device_errors()
    ref = ops.hodge_build(ei, b.num_node1.tolist(), lam)
    nnz0, nnz1 = ref[0].shape[1], ref[2].shape[1]
    got = ops.hodge_build(ei, b.num_node1.tolist(), lam, sizes=(N, nnz0, nnz1))
    for x, y in zip(got[:4], ref[:4]):
        assert torch.equal(x, y)
    ops.check_device_errors()
    # undersized, and oversized: a total past the device's rows
    # would leave the tail of col / val unwritten
    for short in ((N, nnz0 - 5, nnz1), (N, nnz0, nnz1 - 7), (N, 0, 0),
                  (N, nnz0 + 5, nnz1), (N, nnz0, nnz1 + 7)):
        ops.hodge_build(ei, b.num_node1.tolist(), lam, sizes=short)
        with pytest.raises(RuntimeError, match="hodge_build"):
            ops.check_device_errors()
        ops.clear_device_errors()
    ops.check_device_errors()


def _grads_with_fused_bwd(fused, run):
    from hlhgat import ops
    try:
        ops._ext.set_fused_bwd(fused)
        return run()
    finally:
        ops._ext.set_fused_bwd(True)


@pytest.mark.parametrize("M", [37, 5000, 70000])
def test_fused_linear_backward_bitwise(cuda, M):
    """hlhgat_proj_bwd (weight / bias split partials and the data gradient in
    one launch, then the split reduction) == the separate weight / reduce /
    data launches, bit for bit: three input blocks (concatenated
    Linear input, lib/Hodge_Cheb_Conv.py:307-308), one of them 4-unaligned
    (the fallback), and the aligned case."""
    from hlhgat import ops
    g = torch.Generator(device="cpu").manual_seed(M)
    for widths in ([64, 128, 8], [64, 6, 32]):
        blocks = [torch.randn(M, k, generator=g).to(cuda) for k in widths]
        W = torch.randn(96, sum(widths), generator=g).to(cuda) * 0.1
        b = torch.randn(96, generator=g).to(cuda)
        R = torch.randn(M, 96, generator=g).to(cuda)

        def run():
            xs = [t.clone().requires_grad_(True) for t in blocks]
            Wv, bv = W.clone().requires_grad_(True), b.clone().requires_grad_(True)
            (ops.linear_blocks(xs, Wv, bv) * R).sum().backward()
            return [Wv.grad, bv.grad] + [x.grad for x in xs]
        a = _grads_with_fused_bwd(True, run)
        c = _grads_with_fused_bwd(False, run)
        ref = [R.t() @ torch.cat(blocks, 1), R.sum(0)] + list((R @ W).split(widths, 1))
        for u, v, r in zip(a, c, ref):
            assert torch.equal(u, v)
            close(u.cpu(), r.cpu(), 1e-4, "linear grad vs torch")


@pytest.mark.parametrize("M", [9000, 25000])
@pytest.mark.parametrize("widths,N", [([64, 64, 64], 64), ([384, 384], 64), ([36, 36, 36], 32),
                                      ([128], 48)])
def test_fused_linear_backward_row_blocks_bitwise(cuda, M, widths, N):
    """The fused Linear backward's data gradient with one workgroup per row
    block covering every column tile (N <= 64, hlhgat_set_proj_bwd_rows) ==
    one workgroup per (row block, column tile), bit for bit, and both against
    torch: the conv (K = 3, d = 64), NodeEdgeInt Linear(768, 64) and
    narrower shapes."""
    from hlhgat import _lib, ops
    g = torch.Generator(device="cpu").manual_seed(M + N)
    blocks = [torch.randn(M, k, generator=g).to(cuda) for k in widths]
    W = torch.randn(N, sum(widths), generator=g).to(cuda) * 0.1
    b = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda)

    def run():
        xs = [t.clone().requires_grad_(True) for t in blocks]
        Wv, bv = W.clone().requires_grad_(True), b.clone().requires_grad_(True)
        (ops.linear_blocks(xs, Wv, bv) * R).sum().backward()
        return [Wv.grad, bv.grad] + [x.grad for x in xs]
    res = []
    for rows in (1, 0):
        _lib.check(_lib.LIB.hlhgat_set_proj_bwd_rows(rows), "set_proj_bwd_rows")
        try:
            res.append(run())
        finally:
            _lib.LIB.hlhgat_set_proj_bwd_rows(1)
    ref = [R.t() @ torch.cat(blocks, 1), R.sum(0)] + list((R @ W).split(widths, 1))
    for u, v, r in zip(res[0], res[1], ref):
        assert torch.equal(u, v)
        close(u.cpu(), r.cpu(), 1e-4, "linear grad vs torch")


@pytest.mark.parametrize("padded", [False, True])
def test_fused_backward_zinc_model_bitwise(cuda, padded):
    """Every parameter gradient of the ZINC head (conv projections, NodeEdgeInt
    MLPs, readout MLP) is bitwise the same with the fused Linear backward as
    with the separate launches; padded: static-shape capacity rows (n_valid)."""
    import hlhgat
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(48, seed=5)
    if padded:
        b = pad_batch(b, static_caps(b, 128))
    b = b.to(cuda)

    def run():
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[2, 2, 2], filters=[64, 64, 64],
                                                mlp_channels=[256, 256], K=3,
                                                keig=15).to(cuda).train()
        torch.nn.functional.l1_loss(m(b).view(-1), b.y.view(-1)).backward()
        return {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    a = _grads_with_fused_bwd(True, run)
    c = _grads_with_fused_bwd(False, run)
    assert a.keys() == c.keys() and len(a) > 100
    for k in a:
        assert torch.equal(a[k], c[k]), k


@pytest.mark.parametrize("padded", [False, True])
def test_bn_handover_zinc_model_bitwise(cuda, padded):
    """The config-2 ZINC head with every waiting one-launch BatchNorm workgroup
    (k_bn_fwd_grid, k_proj_bn_fwd) handing its rows to its tile's finaliser
    (wait bound 0) == the default, bit for bit: the output, every parameter
    gradient and running statistic, padded (n_valid) or not."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(200, seed=6)
    if padded:
        b = pad_batch(b, static_caps(b, 128))
    b = b.to(cuda)

    def run():
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[2, 2, 2], filters=[64, 64, 64],
                                                mlp_channels=[256, 256], K=3,
                                                keig=15).to(cuda).train()
        out = m(b)
        torch.nn.functional.l1_loss(out.view(-1), b.y.view(-1)).backward()
        g = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
        g.update({k: v.clone() for k, v in m.state_dict().items() if "running" in k})
        g["out"] = out.detach().clone()
        return g
    a = run()
    ops.bn_giveups_reset()
    with _BnWait(0):
        c = run()
    gu = ops.bn_giveups()
    ops.check_device_errors()
    assert a.keys() == c.keys() and len(a) > 100
    for k in a:
        assert torch.equal(a[k], c[k]), k
    assert gu["count"] > 0


@pytest.mark.parametrize("n,C,relu,pad", [(700, 64, True, 0), (25600, 64, True, 333),
                                          (25600, 256, False, 0), (4097, 6, True, 5),
                                          (200000, 64, True, 0)])
def test_bn_one_launch_bitwise(cuda, n, C, relu, pad):
    """BatchNorm forward in one launch (k_bn_train_fused: statistics, a tile-
    wide wait for the finalising workgroup, normalisation) == the statistics +
    apply launches bit for bit: output, batch mean / invstd, running stats and
    the backward through it; padded rows (n_valid) and an unaligned C (the
    vector path off) included; n = 200000 exceeds the one-launch grid cap and
    takes the two launches either way."""
    from hlhgat import _lib, ops
    g = torch.Generator(device="cpu").manual_seed(n + C)
    x0 = (torch.randn(n, C, generator=g) * 3 + 1).to(cuda)
    R = torch.randn(n, C, generator=g).to(cuda)
    valid = torch.tensor([n - pad], dtype=torch.int32, device=cuda) if pad else None
    outs = []
    ops.bn_giveups_reset()
    prior = int(_lib.LIB.hlhgat_get_bn_one_launch())
    try:
        for one in (1, 0):
            _lib.check(_lib.LIB.hlhgat_set_bn_one_launch(one), "set_bn_one_launch")
            torch.manual_seed(0)
            bn = torch.nn.BatchNorm1d(C).to(cuda).train()
            with torch.no_grad():
                bn.weight.uniform_(0.5, 1.5)
                bn.bias.uniform_(-0.5, 0.5)
            x = x0.clone().requires_grad_(True)
            y = ops.batch_norm_act(x, bn, relu=relu, valid=valid)
            (y * R).sum().backward()
            outs.append([y.detach(), x.grad, bn.weight.grad, bn.bias.grad, bn.running_mean,
                         bn.running_var])
    finally:
        _lib.LIB.hlhgat_set_bn_one_launch(prior)
    ops.check_device_errors()
    import ctypes
    t = ctypes.c_uint(7)
    _lib.check(_lib.LIB.hlhgat_bn_wait_timeouts(ctypes.addressof(t)), "bn_wait_timeouts")
    assert t.value == 0
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    nv = n - pad
    ref = torch.nn.functional.batch_norm(x0[:nv].double(), None, None, training=True, eps=1e-5)
    ref = ref * bn.weight.detach().double() + bn.bias.detach().double()
    if relu:
        ref = ref.clamp_min(0)
    close(outs[0][0][:nv].cpu(), ref.float().cpu(), 1e-5, "bn forward vs fp64")
    assert not outs[0][0][nv:].any()


def test_bn_one_launch_handover_bitwise(cuda):
    """A one-launch BatchNorm (k_bn_fwd_grid) whose waiting workgroups all
    give up at once (wait bound 0) hands their rows to the finalising
    workgroup, which normalises them from x: the output and the running
    statistics are bitwise those of the two-launch path, no device error is
    raised, and the give-ups are counted and logged (tile, total,
    generations)."""
    from hlhgat import _lib, ops
    ops.check_device_errors()
    x = torch.randn(25600, 64, device=cuda) * 2 + 1
    outs = []
    for one, wait in ((0, 1000), (1, 0)):
        prior = int(_lib.LIB.hlhgat_get_bn_one_launch())
        try:
            _lib.check(_lib.LIB.hlhgat_set_bn_one_launch(one), "set_bn_one_launch")
            ops.bn_giveups_reset()
            with _BnWait(wait):
                torch.manual_seed(0)
                bn = torch.nn.BatchNorm1d(64).to(cuda).train()
                y = ops.batch_norm_act(x, bn, relu=True)
                torch.cuda.synchronize()
            outs.append((y, bn.running_mean.clone(), bn.running_var.clone(), ops.bn_giveups()))
        finally:
            _lib.LIB.hlhgat_set_bn_one_launch(prior)
    ops.check_device_errors()
    (y2, rm2, rv2, _), (y1, rm1, rv1, gu) = outs
    assert torch.equal(y1, y2) and torch.equal(rm1, rm2) and torch.equal(rv1, rv2)
    assert gu["count"] > 0
    for r in gu["log"]:
        assert r["kernel"] == 1 and r["total"] == 128 and r["outcome"] in (1, 2)
        assert r["arrivals"] <= r["total"]


_HOG = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from hlhgat import _lib
cus = torch.cuda.get_device_properties(0).multi_processor_count
s = torch.cuda.Stream()
_lib.check(_lib.LIB.hlhgat_test_occupy(cus, cus - 64, 140 * 1024, int(sys.argv[2]),
                                       s.cuda_stream), "test_occupy")
print("hog launched", flush=True)
s.synchronize()
print("hog done", flush=True)
"""


@pytest.mark.parametrize("wait_us", [1000, 0])
def test_bn_one_launch_beside_cu_hog(cuda, wait_us):
    """The one-launch BatchNorm kernels launched while ANOTHER PROCESS's kernel
    holds the LDS of all but 64 CUs for 0.6 s (hlhgat_test_occupy; a second
    process gets hardware queues of its own): the launches complete long
    before the hog ends, with the bits of the undisturbed launches and no
    device error -- at the default wait, and with wait_us = 0, where every
    workgroup that finds the statistics not yet final hands its rows to the
    finaliser while the other kernel runs (hand-overs counted > 0).
    (tools/probes/hog_probe.py, round 5: with only 16 CUs free the launch was
    not started before the hog ended -- no wait, no hand-over; the queue, not
    the barrier, held it.)"""
    import subprocess
    import sys
    import time
    from hlhgat import ops
    ops.check_device_errors()
    g = torch.Generator(device="cpu").manual_seed(11)
    x = (torch.randn(25600, 64, generator=g) * 3 + 1).to(cuda)
    As = [torch.randn(25600, 64, generator=g).to(cuda) for _ in range(3)]
    W = (torch.randn(64, 192, generator=g) / 192 ** 0.5).to(cuda)
    bns = []

    def launches():
        torch.manual_seed(0)
        bn = torch.nn.BatchNorm1d(64).to(cuda).train()
        bn2 = torch.nn.BatchNorm1d(64).to(cuda).train()
        bns.append((bn, bn2))
        torch.cuda.synchronize()  # parameters in place before the timed launches
        t0 = time.perf_counter()
        y = ops.batch_norm_act(x, bn, relu=True)
        _, y2, _, _ = _proj_bn_call_nosync(cuda, As, W, None, bn2, None, True)
        torch.cuda.synchronize()
        return (y, y2, bn.running_var, bn2.running_var), time.perf_counter() - t0

    ref, _ = launches()
    ref = [t.clone() for t in ref]
    ops.bn_giveups_reset()
    usec = 600000
    pkg = os.path.join(REPO, "hl-hgat_amd")
    hog = subprocess.Popen([sys.executable, "-c", _HOG, pkg, str(usec)], stdout=subprocess.PIPE,
                           text=True)
    try:
        assert hog.stdout.readline().strip() == "hog launched"
        time.sleep(0.1)  # the hog's workgroups are resident
        with _BnWait(wait_us):
            got, dt = launches()
        gu = ops.bn_giveups()
    finally:
        rest = hog.communicate(timeout=60)[0]
    assert hog.returncode == 0 and "hog done" in rest
    ops.check_device_errors()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    print(f"beside the hog (wait {wait_us} us): {dt * 1e3:.1f} ms, hand-overs {gu['count']}, "
          f"log {gu['log'][:4]}")
    assert dt < 0.5 * usec * 1e-6, dt  # ran beside the hog, did not wait for it to end
    if wait_us == 0:
        assert gu["count"] > 0


def test_boundary_operator_reference_lines_verbatim(cuda):
    """The reference's own sparse products run unchanged on hlhgat.adj2par1:
    torch.sparse.mm(par_1.transpose(0,1), x_t).abs()/2 (lib/Hodge_ST_Model.py:
    848), torch.sparse.mm(par.abs(), x_s) and torch.sparse.mm(par.abs().
    transpose(0,1), x_t) (lib/Hodge_Cheb_Conv.py:294-295), B1 @ y -- bitwise
    the coalesced torch.sparse.mm of the reference's COO, gradients included."""
    from hlhgat.hodge_dataset import adj2par1
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(30, seed=8)
    N, E = b.x_t.shape[0], b.x_s.shape[0]
    ref_P = R.adj2par1(b.edge_index, N, E).coalesce()
    par_1 = adj2par1(dev(b.edge_index), N, E)
    gen = torch.Generator().manual_seed(3)
    x_t = torch.randn(N, 20, generator=gen)
    x_s = torch.randn(E, 20, generator=gen)
    cases = [
        (lambda P, xt, xs: torch.sparse.mm(P.transpose(0, 1), xt).abs() / 2, "readout :848"),
        (lambda P, xt, xs: torch.sparse.mm(P.abs(), xs), "|B1| x_s :294"),
        (lambda P, xt, xs: torch.sparse.mm(P.abs().transpose(0, 1), xt) / 2, "|B1|^T x_t :295"),
        (lambda P, xt, xs: torch.mm(P, xs), "B1 x_s"),
        (lambda P, xt, xs: P.t() @ xt, "B1^T @ x_t"),
    ]
    for fn, what in cases:
        xt_r, xs_r = x_t.clone().requires_grad_(True), x_s.clone().requires_grad_(True)
        y_r = fn(ref_P, xt_r, xs_r)
        xt_d, xs_d = dev(x_t).requires_grad_(True), dev(x_s).requires_grad_(True)
        y_d = fn(par_1, xt_d, xs_d)
        assert torch.equal(y_d.detach().cpu(), y_r.detach()), what
        Rg = torch.randn(y_r.shape, generator=gen)
        (y_r * Rg).sum().backward()
        (y_d * dev(Rg)).sum().backward()
        for a, r in ((xt_d, xt_r), (xs_d, xs_r)):
            if r.grad is None:
                assert a.grad is None or not a.grad.any(), what
            else:
                close(a.grad.cpu(), r.grad, 1e-6, what + " grad")


def _proj_bn_call(cuda, As, W, bias, bn, valid, relu, fused):
    """hlhgat_proj_bn_fwd through the C-ABI: returns x, y, mean, invstd."""
    from hlhgat import _lib
    _lib.check(_lib.LIB.hlhgat_set_proj_bn_fused(1 if fused else 0), "set_proj_bn_fused")
    try:
        out = _proj_bn_call_nosync(cuda, As, W, bias, bn, valid, relu)
    finally:
        _lib.LIB.hlhgat_set_proj_bn_fused(1)
    torch.cuda.synchronize()
    return out


def _proj_bn_call_nosync(cuda, As, W, bias, bn, valid, relu):
    """hlhgat_proj_bn_fwd on the current stream, not synchronised."""
    import ctypes
    from hlhgat import _lib
    L = _lib.LIB
    M, N, nb = As[0].shape[0], W.shape[0], len(As)
    kb = [a.shape[1] for a in As]
    offs = [sum(kb[:i]) for i in range(nb)]
    A_p = (ctypes.c_void_p * nb)(*[a.data_ptr() for a in As])
    lda = (ctypes.c_int64 * nb)(*[a.stride(0) for a in As])
    W_p = (ctypes.c_void_p * nb)(*[W.data_ptr() + 4 * o for o in offs])
    ldw = (ctypes.c_int64 * nb)(*([W.stride(0)] * nb))
    kbs = (ctypes.c_int64 * nb)(*kb)
    x = torch.empty(M, N, device=cuda)
    y = torch.empty(M, N, device=cuda)
    mean = torch.empty(N, device=cuda)
    invstd = torch.empty(N, device=cuda)
    ws = torch.zeros(int(L.hlhgat_bn_workspace_bytes(M, N)), dtype=torch.uint8, device=cuda)
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(L.hlhgat_proj_bn_fwd(
        nb, A_p, lda, W_p, ldw, kbs, M, N, bias.data_ptr() if bias is not None else None,
        x.data_ptr(), N, valid.data_ptr() if valid is not None else None,
        bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
        bn.running_var.data_ptr(), bn.num_batches_tracked.data_ptr(), 0.1, 1e-5,
        1 if relu else 0, y.data_ptr(), N, mean.data_ptr(), invstd.data_ptr(),
        ws.data_ptr(), ws.numel(), s), "proj_bn_fwd")
    _keep.append(ws)
    return x, y, mean, invstd


_keep = []  # workspaces of unsynchronised calls (freed only at exit)


@pytest.mark.parametrize("M,N,kb,pad,relu,expect_fused", [
    (23157, 64, [64, 64, 64], 0, True, True),       # cfg2 node conv K=3
    (25600, 64, [384, 384], 333, True, True),      # NodeEdgeInt Linear(768, 64), padded rows
    (9728, 128, [128, 128], 0, True, True),        # heads: 128 columns = two BN tiles
    (700, 256, [256], 0, False, True),             # readout-sized, no ReLU
    (4097, 64, [36, 36, 36], 5, True, True),       # init conv widths
    (40000, 64, [64, 64, 64], 0, True, False),     # > 512 row blocks: two calls
    (3000, 32, [32], 0, True, False)])             # N % 64 != 0: two calls
def test_proj_bn_fused_matches_two_calls(cuda, M, N, kb, pad, relu, expect_fused):
    """hlhgat_proj_bn_fwd (k_proj_bn_fwd: projection + BatchNorm + ReLU in one
    launch, statistics by a last-arriver tree) against its two-call path
    (hlhgat_proj_fwd, hlhgat_bn_fwd_train): x bitwise, y / batch statistics /
    running statistics within 1e-6 (fp64 sums in another order), padded rows 0,
    fused launches deterministic run to run, both against an fp64 evaluation
    (1e-5)."""
    import ctypes
    from hlhgat import _lib, ops
    cap = ctypes.c_int64(0)
    _lib.check(_lib.LIB.hlhgat_proj_bn_fused_capacity(ctypes.byref(cap)), "capacity")
    assert cap.value >= 400  # the cfg2 shapes (<= 400 row blocks) take the fused launch
    g = torch.Generator(device="cpu").manual_seed(M + N)
    As = [torch.randn(M, k, generator=g).to(cuda) for k in kb]
    W = (torch.randn(N, sum(kb), generator=g) / sum(kb) ** 0.5).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    valid = torch.tensor([M - pad], dtype=torch.int32, device=cuda) if pad else None
    res = []
    for fused in (True, True, False):
        torch.manual_seed(0)
        bn = torch.nn.BatchNorm1d(N).to(cuda).train()
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        ops.prof_reset()
        ops.prof_enable(_lib.PROF_PROJ_BN, True)
        out = _proj_bn_call(cuda, As, W, bias, bn, valid, relu, fused)
        ops.prof_enable(_lib.PROF_PROJ_BN, False)
        launches = ops.prof_read(_lib.PROF_PROJ_BN)["launches"]
        assert launches == (1 if (fused and expect_fused) else 0), launches
        res.append(list(out) + [bn.running_mean.clone(), bn.running_var.clone(),
                                bn.num_batches_tracked.clone()])
    ops.check_device_errors()
    (f1, f2, two) = res
    for a, b in zip(f1, f2):
        assert torch.equal(a, b)  # deterministic
    assert torch.equal(f1[0], two[0])  # x: the same GEMM arithmetic
    for i, nm in ((1, "y"), (2, "mean"), (3, "invstd"), (4, "running_mean"), (5, "running_var")):
        close(f1[i].cpu(), two[i].cpu(), 1e-6, nm)
    assert torch.equal(f1[6], two[6])
    nv = M - pad
    xr = sum(a.double() @ W[:, o:o + a.shape[1]].double().T
             for a, o in zip(As, [sum(kb[:i]) for i in range(len(kb))])) + bias.double()
    ref = torch.nn.functional.batch_norm(xr[:nv], None, None, training=True, eps=1e-5)
    ref = ref * bn.weight.detach().double() + bn.bias.detach().double()
    if relu:
        ref = ref.clamp_min(0)
    close(f1[1][:nv].cpu(), ref.float().cpu(), 1e-5, "y vs fp64")
    assert not f1[1][nv:].any()


def test_proj_bn_handover_bitwise(cuda):
    """k_proj_bn_fwd with every waiting workgroup handing its 64-row tile to
    the finaliser (wait bound 0), which normalises it from the x the owner
    stored: x, y and the statistics bitwise those of the default launch, no
    device error."""
    from hlhgat import ops
    ops.check_device_errors()
    g = torch.Generator(device="cpu").manual_seed(3)
    As = [torch.randn(25600, 64, generator=g).to(cuda) for _ in range(3)]
    W = (torch.randn(64, 192, generator=g) / 192 ** 0.5).to(cuda)
    bias = torch.randn(64, generator=g).to(cuda)
    valid = torch.tensor([25600 - 77], dtype=torch.int32, device=cuda)
    res = []
    for wait in (1000, 0):
        torch.manual_seed(0)
        bn = torch.nn.BatchNorm1d(64).to(cuda).train()
        ops.bn_giveups_reset()
        with _BnWait(wait):
            out = _proj_bn_call(cuda, As, W, bias, bn, valid, True, True)
        res.append(list(out) + [bn.running_mean.clone(), bn.running_var.clone(),
                                ops.bn_giveups()])
    ops.check_device_errors()
    for a, b in zip(res[0][:6], res[1][:6]):
        assert torch.equal(a, b)
    gu = res[1][6]
    assert gu["count"] > 0 and all(r["kernel"] == 2 for r in gu["log"])


def test_proj_bn_phase_stamps(cuda):
    """hlhgat_set_proj_bn_stamps (diagnostics, tools/probes/proj_bn_phases.py):
    the stamped instantiation of k_proj_bn_fwd gives the same x / y as the
    product one, and every workgroup's phases are in order, with exactly one
    finaliser; the stamps are off again afterwards."""
    from hlhgat import _lib
    M, kb = 23157, [64, 64, 64]
    g = torch.Generator(device="cpu").manual_seed(5)
    As = [torch.randn(M, k, generator=g).to(cuda) for k in kb]
    W = (torch.randn(64, 192, generator=g) / 192 ** 0.5).to(cuda)
    bias = torch.randn(64, generator=g).to(cuda)
    gx = (M + 63) // 64
    st = torch.zeros(gx * 8, dtype=torch.int64, device=cuda)
    res = []
    for stamps in (False, True):
        torch.manual_seed(0)
        bn = torch.nn.BatchNorm1d(64).to(cuda).train()
        if stamps:
            _lib.check(_lib.LIB.hlhgat_set_proj_bn_stamps(st.data_ptr(), st.numel()), "stamps")
        try:
            res.append(_proj_bn_call(cuda, As, W, bias, bn, None, True, True))
        finally:
            _lib.LIB.hlhgat_set_proj_bn_stamps(None, 0)
    for a, b in zip(*res):
        assert torch.equal(a, b)
    t = st.view(gx, 8).cpu()
    assert int(((t[:, 6] & 2) != 0).sum()) == 1
    for k in range(5):
        assert bool((t[:, k + 1] >= t[:, k]).all()), k
    assert bool((t[:, 0] > 0).all())


@pytest.mark.parametrize("M,N,kb,pad", [(23157, 64, [64, 64, 64], 0), (25600, 64, [384, 384], 333),
                                        (9728, 128, [128, 128], 0)])
def test_proj_bn_split_bitwise(cuda, M, N, kb, pad):
    """hlhgat_set_proj_bn_split(1): the projection with the BatchNorm
    statistics in its epilogue (no workgroup waits), then k_bn_apply == the
    one launch whose workgroups wait for the statistics: x, y, the batch and
    running statistics bit for bit."""
    from hlhgat import _lib
    g = torch.Generator(device="cpu").manual_seed(M + 7)
    As = [torch.randn(M, k, generator=g).to(cuda) for k in kb]
    W = (torch.randn(N, sum(kb), generator=g) / sum(kb) ** 0.5).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    valid = torch.tensor([M - pad], dtype=torch.int32, device=cuda) if pad else None
    res = []
    for split in (0, 1):
        torch.manual_seed(0)
        bn = torch.nn.BatchNorm1d(N).to(cuda).train()
        _lib.check(_lib.LIB.hlhgat_set_proj_bn_split(split), "set_proj_bn_split")
        try:
            out = _proj_bn_call(cuda, As, W, bias, bn, valid, True, True)
        finally:
            _lib.LIB.hlhgat_set_proj_bn_split(0)
        res.append(list(out) + [bn.running_mean.clone(), bn.running_var.clone(),
                                bn.num_batches_tracked.clone()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_factor_tables_from_collate_bitwise_device_build(cuda):
    """A factored L1 whose batch carries the collate-time tables
    (hodge_dataset.factor_tables: alpha, signs, ends) builds the same
    hlhgat_hodge_factor_t as the device build without them, and the factored
    SpMM and a Laguerre conv over it give the same bits -- padded batch."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate, pad_batch, static_caps
    from hlhgat.synthetic import cifar_like_graphs
    cb = collate([cifar_like_graphs(s)[0] for s in range(3)])
    pb = pad_batch(cb, static_caps(cb))
    assert pb.l1_factor and pb.fac_alpha is not None
    torch.manual_seed(0)
    conv = hlhgat.HodgeLaguerreConv(16, 24, K=4).to(cuda)
    X = torch.randn(pb.x_s.shape[0], 16, device=cuda)
    res = []
    for keep in (True, False):
        b = pb.__class__.__new__(pb.__class__)
        for k, v in vars(pb).items():
            if keep or not k.startswith("fac_"):
                setattr(b, k, v)
        d = b.to(cuda)
        op = ops.hodge_operator(d.edge_index_s, d.edge_weight_s, d.x_s.shape[0])
        assert op.factor is not None and ops.has_hodge_factor(d.edge_index_s)
        xr = X.clone().requires_grad_(True)
        y = conv(xr, d.edge_index_s, d.edge_weight_s)
        y.square().sum().backward()
        res.append([t.clone() for t in op.factor] + [ops.hodge_spmm(op, X), y.detach(),
                                                     xr.grad])
    ops.check_device_errors()
    for a, b in zip(*res):
        assert torch.equal(a, b)
