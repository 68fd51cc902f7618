"""Launch groups (include/hlhgat.h hlhgat_group_*): the node (L0) and edge
(L1) convs of an HL block as one paired autograd node whose launches cover
both sides (ops.hodge_poly_conv_pair).  The paired path must give the bits of
the two single conv nodes: outputs, every gradient, the BatchNorm running
statistics -- for the ZINC shape, for the init conv (different input widths,
so some launches cannot pair), and for factored / halo-tiled operators.
"""
import pytest
import torch

from conftest import REPO  # noqa: F401


def _capi():
    from hlhgat import _lib
    return _lib.LIB


def test_group_api_errors_without_gpu():
    """Nesting and unmatched calls are refused with a message (no GPU)."""
    lib = _capi()
    assert lib.hlhgat_group_next() != 0
    assert lib.hlhgat_group_end(None, None) != 0
    assert lib.hlhgat_group_begin() == 0
    assert lib.hlhgat_group_begin() != 0
    assert b"already" in lib.hlhgat_last_error()
    assert lib.hlhgat_group_next() == 0
    assert lib.hlhgat_group_next() != 0
    assert lib.hlhgat_group_end(None, None) == 0  # nothing recorded: nothing issued
    assert lib.hlhgat_group_abort() == 0


def test_sequential_finds_the_pair():
    from hlhgat.hodge_st_model import _hl_block
    blk = _hl_block(16, 16, 16, 3, 0.0)
    assert blk._pair == (0, 4)


def _run_block(blk, batch, x_t, x_s, pair):
    from hlhgat import ops
    prev, ops.PAIR_CONV = ops.PAIR_CONV, pair
    try:
        xt = x_t.clone().requires_grad_(True)
        xs = x_s.clone().requires_grad_(True)
        yt, ys = blk(xt, batch.edge_index_t, batch.edge_weight_t, xs, batch.edge_index_s,
                     batch.edge_weight_s)
        g = torch.Generator(device="cpu").manual_seed(3)
        rt = torch.randn(yt.shape, generator=g).to(yt.device)
        rs = torch.randn(ys.shape, generator=g).to(ys.device)
        ((yt * rt).sum() + (ys * rs).sum()).backward()
        fn = type(yt.grad_fn).__name__ + str(yt.grad_fn.name())
        grads = [xt.grad, xs.grad] + [p.grad.clone() for p in blk.parameters()]
        bufs = [b.clone() for b in blk.buffers()]
        for p in blk.parameters():
            p.grad = None
        return [yt.detach(), ys.detach()] + grads + bufs, fn
    finally:
        ops.PAIR_CONV = prev


@pytest.mark.gpu
@pytest.mark.parametrize("cin_t,cin_s", [(64, 64), (36, 18)])
def test_conv_pair_bitwise_equal_to_two_nodes(cuda, cin_t, cin_s):
    from hlhgat.hodge_st_model import _hl_block
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(300, seed=5).to(cuda)
    torch.manual_seed(0)
    blk = _hl_block(cin_t, cin_s, 64, 3, 0.0).to(cuda).train()
    g = torch.Generator().manual_seed(1)
    x_t = torch.randn(b.x_t.shape[0], cin_t, generator=g).to(cuda)
    x_s = torch.randn(b.x_s.shape[0], cin_s, generator=g).to(cuda)
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    ref, fn_ref = _run_block(blk, b, x_t, x_s, False)
    blk.load_state_dict(state)
    got, fn_got = _run_block(blk, b, x_t, x_s, True)
    assert "Pair" in fn_got and "Pair" not in fn_ref, (fn_got, fn_ref)
    assert len(ref) == len(got)
    for i, (a, c) in enumerate(zip(ref, got)):
        assert torch.equal(a, c), i


@pytest.mark.gpu
def test_conv_pair_factored_and_halo_operators(cuda):
    """A TSP-like pair (L1 factored, L0 plain CSR): the launches that differ
    in kernel run one after the other inside the group, still bitwise."""
    from hlhgat.hodge_dataset import collate
    from hlhgat.hodge_st_model import _hl_block
    from hlhgat.synthetic import tsp_like_graph
    b = collate([tsp_like_graph(0, n=600)], check_hodge=False).to(cuda)
    torch.manual_seed(0)
    blk = _hl_block(32, 32, 32, 4, 0.0).to(cuda).train()
    g = torch.Generator().manual_seed(2)
    x_t = torch.randn(b.x_t.shape[0], 32, generator=g).to(cuda)
    x_s = torch.randn(b.x_s.shape[0], 32, generator=g).to(cuda)
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    ref, _ = _run_block(blk, b, x_t, x_s, False)
    blk.load_state_dict(state)
    got, fn = _run_block(blk, b, x_t, x_s, True)
    assert "Pair" in fn
    for i, (a, c) in enumerate(zip(ref, got)):
        assert torch.equal(a, c), i


@pytest.mark.gpu
def test_zinc_train_step_paired_equals_unpaired(cuda):
    """Graph-replayed ZINC training steps on padded batches (one capture)
    with and without the paired convs: bitwise the same losses, parameters
    and running statistics."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    from hlhgat.train import TrainStep
    raw = [zinc_like_batch(48, seed=s) for s in (1, 2, 3)]
    cs = [static_caps(b, 256) for b in raw]
    caps = {k: max(c[k] for c in cs) for k in cs[0]}
    batches = [pad_batch(b, caps).to(cuda) for b in raw]
    res = []
    prev = ops.PAIR_CONV
    for pair in (False, True):
        ops.PAIR_CONV = pair
        try:
            torch.manual_seed(0)
            m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[1, 1], filters=[64, 64],
                                                    mlp_channels=[64], K=3,
                                                    keig=15).to(cuda).train()
            crit = torch.nn.L1Loss()
            step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                             graphs=True)
            losses = [float(step(batches[i])) for i in (0, 1, 2, 0)]
            torch.cuda.synchronize()
            res.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
        finally:
            ops.PAIR_CONV = prev
    l0, s0 = res[0]
    for l1, s1 in res[1:]:
        assert l0 == l1
        for k in s0:
            assert torch.equal(s0[k], s1[k]), k


@pytest.mark.gpu
def test_dense_grad_sink_bitwise(cuda):
    """NodeEdgeInt adding its input gradients straight into the dense slab's
    gradient (DenseConcat.grad_sink, accumulate_d of hlhgat_proj_bwd) gives
    the bits of the view-by-view accumulation: every parameter gradient of
    the ZINC model."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(64, seed=11).to(cuda)
    res = []
    prev = ops.GRAD_SINK
    for sink in (False, True):
        ops.GRAD_SINK = sink
        try:
            torch.manual_seed(0)
            m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[2, 2], filters=[64, 64],
                                                    mlp_channels=[64], K=3,
                                                    keig=15).to(cuda).train()
            out = m(b)
            torch.nn.functional.l1_loss(out.view(-1), b.y.view(-1)).backward()
            res.append({k: p.grad.clone() for k, p in m.named_parameters()})
        finally:
            ops.GRAD_SINK = prev
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k
