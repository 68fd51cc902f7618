"""Config 5 at its FULL per-GPU size (BASELINE configs[4]: 4 TSP-like graphs of
10k nodes, k = 9 nearest neighbours; L1 with n = 207k rows, nnz = 4.1M), the
operator the bench's `spmm_cfg5` leg measures.  Only small cases are compared
with the oracle elsewhere; here the full operator is checked:

* the CSR SpMM as the product runs it (RCM row schedule + LDS halo tiles) is
  bit-exact against the oracle's propagate (torch CPU index_add_, the
  reference's scatter-add order);
* the Hodge-factored SpMM and Laguerre basis (the config-5 default) agree with
  the CSR path / an fp64 oracle to 1e-5 relative;
* size-independent properties of the Hodge Laplacian: symmetry
  <L X, Y> = <X, L Y> and linearity, in fp64 sums of the fp32 results.
"""
import pytest
import torch

from conftest import close
from oracle import hodge_ref as R


@pytest.fixture(scope="module")
def cfg5(cuda):
    from hlhgat import ops
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph
    b = collate([tsp_like_graph(s) for s in range(4)], check_hodge=False)
    n = b.x_s.shape[0]
    ei, w = b.edge_index_s, b.edge_weight_s
    assert n > 200_000 and ei.shape[1] > 4_000_000
    bd = collate([tsp_like_graph(s) for s in range(4)], check_hodge=False).to(cuda)
    op = ops.hodge_operator(bd.edge_index_s, bd.edge_weight_s, n)
    assert op.fwd.halo is not None and op.factor is not None
    return dict(n=n, ei=ei, w=w, op=op, dev=cuda)


def _rand(n, d, seed):
    return torch.randn(n, d, generator=torch.Generator().manual_seed(seed))


@pytest.mark.gpu
def test_cfg5_csr_spmm_bit_exact_full_size(cfg5):
    from hlhgat import ops
    torch.set_num_threads(1)  # the oracle's scatter-add in index order
    x = _rand(cfg5["n"], 8, 1)
    ref = R.propagate(x, cfg5["ei"], cfg5["w"])
    y = ops.spmm(cfg5["op"].fwd, x.to(cfg5["dev"])).cpu()
    assert torch.equal(y, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("d", [8, 64])
def test_cfg5_factored_spmm_full_size(cfg5, d):
    from hlhgat import ops
    x = _rand(cfg5["n"], d, 2).to(cfg5["dev"])
    yc = ops.spmm(cfg5["op"].fwd, x).cpu()
    yf = ops.hodge_spmm(cfg5["op"], x).cpu()
    close(yf, yc, 1e-5, "factored vs CSR SpMM, full config 5")


@pytest.mark.gpu
def test_cfg5_factored_laguerre_basis_vs_fp64_oracle(cfg5):
    """K = 4 Laguerre basis (config 5's K) through the factored operator vs
    the oracle's recurrence in fp64 (lib/Hodge_Cheb_Conv.py:494-507)."""
    from hlhgat import ops
    x = _rand(cfg5["n"], 16, 3)
    T = ops.poly_basis(cfg5["op"], x.to(cfg5["dev"]), 4, ops.POLY_LAGUERRE).cpu()
    ei, w = cfg5["ei"], cfg5["w"].double()
    xd = x.double()
    t0, t1 = xd, xd - R.propagate(xd, ei, w)
    ref = [t1]
    for k in (1, 2):
        t2 = (-R.propagate(t1, ei, w) + (2 * k + 1) * t1 - k * t0) / (k + 1)
        ref.append(t2)
        t0, t1 = t1, t2
    for k in range(3):
        close(T[k].double(), ref[k], 1e-5, f"T_{k + 1}")


@pytest.mark.gpu
def test_cfg5_symmetry_and_linearity(cfg5):
    """L1 is symmetric and linear: <L X, Y> = <X, L Y>, L(aX + bY) = aLX + bLY
    (fp64 sums of the fp32 kernel outputs; both paths)."""
    from hlhgat import ops
    dv = cfg5["dev"]
    X, Y = _rand(cfg5["n"], 16, 4).to(dv), _rand(cfg5["n"], 16, 5).to(dv)
    for name, apply in (("csr", lambda z: ops.spmm(cfg5["op"].fwd, z)),
                        ("factored", lambda z: ops.hodge_spmm(cfg5["op"], z))):
        LX, LY = apply(X), apply(Y)
        a = (LX.double() * Y.double()).sum()
        b = (X.double() * LY.double()).sum()
        assert abs(float(a - b)) <= 1e-5 * float(a.abs() + b.abs()), (name, float(a), float(b))
        Lc = apply(2.0 * X - 0.5 * Y)
        close(Lc.cpu(), (2.0 * LX - 0.5 * LY).cpu(), 1e-5, f"{name} linearity")
