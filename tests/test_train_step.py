"""hlhgat.train.TrainStep: flat parameters + fused Adam + one-bucket gradient
all-reduce, replayed as hipGraphs per batch shape.

CPU (gloo, not gpu): the eager step on a plain torch model equals the
reference training loop (torch.optim.Adam, DDP-style mean of gradients).
GPU: the hipGraph-replayed HL-HGAT step equals the eager step bit for bit,
and the two-stream node/edge fork changes no bit of the result."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(5, 7)
        self.b = torch.nn.Linear(7, 1)

    def forward(self, batch):
        return self.b(torch.relu(self.a(batch.x)))


class _B:
    def __init__(self, x, y):
        self.x, self.y = x, y


def _loss(out, b):
    return torch.nn.functional.l1_loss(out.view(-1), b.y.view(-1))


def _data(seed, n=16):
    g = torch.Generator().manual_seed(seed)
    return _B(torch.randn(n, 5, generator=g), torch.randn(n, generator=g))


def test_eager_step_matches_adam_loop():
    from hlhgat.train import TrainStep
    torch.manual_seed(0)
    m1 = _Tiny()
    m2 = _Tiny()
    m2.load_state_dict(m1.state_dict())
    step = TrainStep(m1, _loss, lr=1e-2, weight_decay=1e-3, graphs=False)
    opt = torch.optim.Adam(m2.parameters(), lr=1e-2, weight_decay=1e-3)
    for i in range(4):
        b = _data(i)
        l1 = step(b)
        opt.zero_grad()
        l2 = _loss(m2(b), b)
        l2.backward()
        opt.step()
        assert torch.allclose(l1, l2.detach(), rtol=1e-6, atol=1e-7)
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p1, p2, rtol=1e-6, atol=1e-7), k
    # parameters are views of the flat buffer
    assert m1.a.weight.data_ptr() == step.flat.data_ptr()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from hlhgat.distributed import init_distributed
    from hlhgat.train import TrainStep
    init_distributed("gloo")
    torch.manual_seed(0)
    m = _Tiny()
    step = TrainStep(m, _loss, lr=1e-2, graphs=False)
    for i in range(3):
        step(_data(10 * i + rank))
    q.put((rank, {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}))
    dist.destroy_process_group()


def test_two_rank_gloo_matches_mean_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    # single-process reference: Adam on the mean of the two shards' gradients
    torch.manual_seed(0)
    m = _Tiny()
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    for i in range(3):
        opt.zero_grad()
        for r in range(world):
            b = _data(10 * i + r)
            (_loss(m(b), b) / world).backward()
        opt.step()
    for k, v in m.state_dict().items():
        for r in range(world):
            assert torch.allclose(torch.from_numpy(res[r][k]), v, rtol=1e-5, atol=1e-6), (k, r)


# ---------------------------------------------------------------------------
# GPU: graph replay == eager, fork == no fork
# ---------------------------------------------------------------------------
KW = dict(channels=[1, 1], filters=[32, 32], mlp_channels=[64], K=3, keig=15)


def _check_errors():
    """No kernel raised the device error word during the run."""
    from hlhgat import ops
    assert ops.device_errors() == 0, ops.device_errors()


def _run(graphs, fork, batches, order):
    import hlhgat
    from hlhgat import ops
    from hlhgat.train import TrainStep
    ops.set_stream_fork(fork)
    try:
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to("cuda:0").train()
        crit = torch.nn.L1Loss()
        step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                         weight_decay=1e-3, graphs=graphs)
        ops.clear_device_errors()
        if os.environ.get("HLHGAT_TEST_VERBOSE"):
            losses = []
            import time
            for k, i in enumerate(order):
                t0 = time.perf_counter()
                lo = step(batches[i])
                th = (time.perf_counter() - t0) * 1e3
                losses.append(float(lo))
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3
                print(f"   host call {th:.1f} ms", flush=True)
                print(f"[_run graphs={graphs} fork={fork}] step {k} shape {i}: {dt:.1f} ms "
                      f"err {ops.device_errors()} stats {step.stats}", flush=True)
        else:
            losses = [float(step(batches[i])) for i in order]
        torch.cuda.synchronize()
        _check_errors()
        sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        return losses, sd, dict(step.stats)
    finally:
        ops.set_stream_fork(True)


@pytest.mark.gpu
def test_graph_replay_equals_eager(cuda):
    from hlhgat.synthetic import zinc_like_batch
    batches = [zinc_like_batch(40, seed=3).to(cuda), zinc_like_batch(33, seed=4).to(cuda),
               zinc_like_batch(40, seed=3).to(cuda)]  # [2] = same shape as [0], other tensors
    order = [0, 1, 0, 1, 2, 0]
    l_e, sd_e, _ = _run(False, True, batches, order)
    l_g, sd_g, st = _run(True, True, batches, order)
    assert st["captures"] == 2 and st["replay"] == 4, st
    assert l_e == l_g
    for k in sd_e:
        assert torch.equal(sd_e[k], sd_g[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_stream_fork_is_bitwise_neutral(cuda, graphs):
    """Two streams (the block section's node / edge chains, ops.Chains, and
    the NodeEdgeInt / backward forks) give the bits of one stream: eager and
    graph-replayed steps over two batch shapes (a missing cross-stream
    dependency shows up as a changed loss or parameter)."""
    from hlhgat.synthetic import zinc_like_batch
    batches = [zinc_like_batch(40, seed=7).to(cuda), zinc_like_batch(33, seed=8).to(cuda)]
    order = [0, 1, 0, 1, 1, 0]
    l0, sd0, _ = _run(graphs, False, batches, order)
    l1, sd1, _ = _run(graphs, True, batches, order)
    assert l0 == l1
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_deferred_split_reductions_bitwise(cuda, graphs):
    """Split reductions handed to the next Linear backward on the stream
    (hlhgat_proj_bwd_defer, TrainStep from its second step on) give the bits
    of the per-layer launches: losses and every parameter / running
    statistic after eager and graph-replayed steps, both streams."""
    from hlhgat import train
    from hlhgat.synthetic import zinc_like_batch
    batches = [zinc_like_batch(40, seed=3).to(cuda), zinc_like_batch(33, seed=4).to(cuda)]
    order = [0, 1, 0, 1, 0]
    res = []
    prev = train.DEFER_REDUCE
    for defer in (False, True):
        train.DEFER_REDUCE = defer
        try:
            res.append(_run(graphs, True, batches, order))
        finally:
            train.DEFER_REDUCE = prev
    (l0, sd0, _), (l1, sd1, _) = res
    assert l0 == l1
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k


@pytest.mark.gpu
def test_prepacked_neint_weights_bitwise(cuda):
    """Every NodeEdgeInt's weight pack built in one launch per forward
    (ops.nei_prepack) and the gradient unpack deferred to the flush give the
    bits of the per-module packs: graph-replayed steps."""
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    batches = [zinc_like_batch(40, seed=5).to(cuda), zinc_like_batch(33, seed=6).to(cuda)]
    res = []
    prev = ops.PREPACK
    for pre in (False, True):
        ops.PREPACK = pre
        try:
            res.append(_run(True, True, batches, [0, 1, 0, 1]))
        finally:
            ops.PREPACK = prev
    (l0, sd0, _), (l1, sd1, _) = res
    assert l0 == l1
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["peptides", "cifar", "tsp"])
def test_deferred_reductions_heads_bitwise(cuda, kind):
    """The config 3 / 4 / 5 heads (attention pooling, MLGC levels, parameters
    with torch-op gradients) under TrainStep with and without deferred split
    reductions: the same losses and parameters, bit for bit."""
    import hlhgat
    from hlhgat import train
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph, two_level_batch
    F = torch.nn.functional
    if kind == "tsp":
        raw = [collate([tsp_like_graph(s, n=300)], check_hodge=False) for s in (0, 1)]
        batches = [b.to(cuda) for b in raw]
        cls, kw = "HL_HGCNN_TSP_dense_int3_pyr", dict(channels=[2, 2, 2], filters=[16, 32, 32],
                                                      mlp_channels=[32], K=4)

        def loss_fn(o, d):
            return F.binary_cross_entropy_with_logits(o[0].view(-1), d.y.view(-1).float())
    else:
        raw = [two_level_batch(kind, 6, seed=s) for s in (0, 1)]
        batches = [[x.to(cuda) for x in b] for b in raw]
        kw = dict(channels=[1, 1, 1], filters=[16, 32, 32], mlp_channels=[32], pool_loc=1)
        if kind == "cifar":
            cls = "HL_HGCNN_CIFAR10SP_dense_int3_attpool"
            kw.update(K=3, keig=10, l=0.5)

            def loss_fn(o, d):
                return F.cross_entropy(o, d[0].y.view(-1).long())
        else:
            cls = "HL_HGCNN_pepfunc_dense_int3_attpool"
            kw.update(K=3)

            def loss_fn(o, d):
                return F.binary_cross_entropy_with_logits(o, d[0].y.view(o.shape).float())
    res = []
    prev = train.DEFER_REDUCE
    for defer in (False, True):
        train.DEFER_REDUCE = defer
        try:
            torch.manual_seed(0)
            m = getattr(hlhgat, cls)(**kw).to(cuda).train()
            st = train.TrainStep(m, loss_fn, lr=1e-3, graphs=False)
            losses = [float(st(batches[i % 2])) for i in range(4)]
            res.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
        finally:
            train.DEFER_REDUCE = prev
    assert res[0][0] == res[1][0], (res[0][0], res[1][0])
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["peptides", "cifar"])
@pytest.mark.parametrize("graphs", [False, True])
def test_prepacked_attpool_weights_bitwise(cuda, kind, graphs):
    """The attention-pooling heads with their NodeEdgeInt packs and NEAtt K|Q
    packs built in one launch each per forward (ops.nei_prepack,
    ops.att_prepack) equal the per-module packs / torch.cat: losses and every
    parameter after eager or graph-replayed steps, bit for bit."""
    import hlhgat
    from hlhgat import ops, train
    from hlhgat.synthetic import two_level_batch
    F = torch.nn.functional
    raw = [two_level_batch(kind, 6, seed=s) for s in (0, 1)]
    batches = [[x.to(cuda) for x in b] for b in raw]
    kw = dict(channels=[1, 1, 1], filters=[16, 32, 32], mlp_channels=[32], pool_loc=1, K=3)
    if kind == "cifar":
        cls = "HL_HGCNN_CIFAR10SP_dense_int3_attpool"
        kw.update(keig=10, l=0.5)

        def loss_fn(o, d):
            return F.cross_entropy(o, d[0].y.view(-1).long())
    else:
        cls = "HL_HGCNN_pepfunc_dense_int3_attpool"

        def loss_fn(o, d):
            return F.binary_cross_entropy_with_logits(o, d[0].y.view(o.shape).float())
    res = []
    prev = ops.PREPACK
    for pre in (False, True):
        ops.PREPACK = pre
        try:
            torch.manual_seed(0)
            m = getattr(hlhgat, cls)(**kw).to(cuda).train()
            st = train.TrainStep(m, loss_fn, lr=1e-3, graphs=graphs)
            losses = [float(st(batches[i % 2])) for i in range(4)]
            res.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
        finally:
            ops.PREPACK = prev
    assert res[0][0] == res[1][0], (res[0][0], res[1][0])
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k


class _Twice(torch.nn.Module):
    """One HIP Linear applied twice: its weight gets two gradients per step."""

    def __init__(self):
        super().__init__()
        import hlhgat
        self.a = hlhgat.nn.Linear(64, 64)
        self.b = hlhgat.nn.Linear(64, 1)

    def forward(self, batch):
        return self.b(torch.relu(self.a(torch.relu(self.a(batch.x)))))


@pytest.mark.gpu
def test_deferred_reduction_skips_parameters_used_twice(cuda):
    """A parameter used twice is never deferred (its second gradient adds into
    .grad): TrainStep with deferral equals TrainStep without it."""
    from hlhgat import train
    from hlhgat.train import TrainStep
    g = torch.Generator().manual_seed(2)
    xb = _B(torch.randn(3000, 64, generator=g).to(cuda), torch.randn(3000, 1, generator=g).to(cuda))
    res = []
    prev = train.DEFER_REDUCE
    for defer in (False, True):
        train.DEFER_REDUCE = defer
        try:
            torch.manual_seed(0)
            m = _Twice().to(cuda)
            step = TrainStep(m, lambda o, b: torch.nn.functional.mse_loss(o, b.y), lr=1e-3,
                             graphs=False)
            losses = [float(step(xb)) for _ in range(4)]
            res.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}))
        finally:
            train.DEFER_REDUCE = prev
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k


# ---------------------------------------------------------------------------
# GPU: static-shape (padded) batches
# ---------------------------------------------------------------------------
def _caps_for(batches, quantum=256):
    from hlhgat.hodge_dataset import static_caps
    cs = [static_caps(b, quantum) for b in batches]
    return {k: max(c[k] for c in cs) for k in cs[0]}


@pytest.mark.gpu
def test_padded_batch_matches_unpadded(cuda):
    """Capacity padding (hodge_dataset.pad_batch) leaves the real rows' forward
    values and every parameter gradient unchanged (BN statistics over the
    valid rows only, padding rows isolated)."""
    import hlhgat
    from hlhgat.hodge_dataset import pad_batch
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(37, seed=21)
    pb = pad_batch(b, _caps_for([b]))
    assert pb.x_t.shape[0] > b.x_t.shape[0] and pb.x_s.shape[0] > b.x_s.shape[0]
    res = []
    for batch in (b, pb):
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(cuda).train()
        d = batch.to(cuda)
        out = m(d)
        loss = torch.nn.functional.l1_loss(out.view(-1), d.y.view(-1))
        loss.backward()
        res.append((out.detach().cpu(), {k: p.grad.detach().cpu().clone()
                                         for k, p in m.named_parameters()},
                    {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}))
    (o0, g0, s0), (o1, g1, s1) = res
    assert torch.allclose(o0, o1, rtol=1e-5, atol=1e-6), (o0 - o1).abs().max()
    for k in g0:
        scale = g0[k].abs().max().clamp_min(1e-6)
        assert ((g0[k] - g1[k]).abs().max() / scale) < 1e-4, k
    for k in s0:  # running statistics of every BatchNorm
        if s0[k].dtype.is_floating_point:
            assert torch.allclose(s0[k], s1[k], rtol=1e-5, atol=1e-6), k


@pytest.mark.gpu
def test_padded_batches_share_one_graph(cuda):
    """Batches of different sizes padded to one capacity bucket replay ONE
    captured step; the replay equals the eager step on the same batches."""
    from hlhgat.hodge_dataset import pad_batch
    from hlhgat.synthetic import zinc_like_batch
    raw = [zinc_like_batch(40, seed=s) for s in (3, 4, 5)]
    caps = _caps_for(raw)
    batches = [pad_batch(b, caps).to(cuda) for b in raw]
    order = [0, 1, 2, 1, 0]
    l_e, sd_e, _ = _run(False, True, batches, order)
    l_g, sd_g, st = _run(True, True, batches, order)
    assert st["captures"] == 1 and st["replay"] == len(order) - 1, st
    assert l_e == l_g
    for k in sd_e:
        assert torch.equal(sd_e[k], sd_g[k]), k


class _SideEffectInBackward(torch.autograd.Function):
    """Identity whose backward also runs work on a side stream forked from the
    current (capture) stream and never joined back -- the shape of the round-1
    variant whose hipGraph capture crashed at capture_end."""
    buf = None

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        from hlhgat import ops
        side = ops.side_stream(g.device)
        side.wait_stream(torch.cuda.current_stream(g.device))
        with torch.cuda.stream(side):
            _SideEffectInBackward.buf.copy_(g.abs().sum().view(1))
        g.record_stream(side)
        return g


class _TinyFork(_Tiny):
    def forward(self, batch):
        return self.b(_SideEffectInBackward.apply(torch.relu(self.a(batch.x))))


@pytest.mark.gpu
def test_capture_rejoins_fork_left_open_in_backward(cuda):
    """TrainStep rejoins every side stream that joined the capture before
    hipStreamEndCapture (ops.join_capture_streams), so a fork left open inside
    a backward node neither breaks the capture nor loses its work: replayed
    steps equal eager steps bitwise, the side work runs in every replay, and
    no side stream is left capturing."""
    from hlhgat import ops
    from hlhgat.train import TrainStep
    res = []
    for graphs in (False, True):
        torch.manual_seed(0)
        m = _TinyFork().to(cuda)
        _SideEffectInBackward.buf = torch.zeros(1, device=cuda)
        step = TrainStep(m, _loss, lr=1e-2, graphs=graphs)
        bufs = []
        for i in range(4):
            b = _data(i)
            step(_B(b.x.to(cuda), b.y.to(cuda)))
            torch.cuda.synchronize()
            bufs.append(_SideEffectInBackward.buf.clone())
        if graphs:
            assert step.stats["captures"] == 1 and step.stats["replay"] >= 2
            assert ops.side_streams_capturing(cuda) == []
        res.append(([p.detach().clone() for p in m.parameters()], bufs))
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b)
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 1e-3])
def test_adam_flat_matches_torch_fused_adam(cuda, wd):
    """hlhgat_adam_flat (one launch over the flat parameter buffer) against
    torch.optim.Adam(fused=True, capturable=True) on the same tensor, 3 steps:
    the same arithmetic up to FMA contraction (torch's kernel is built with
    contraction on, hlhgat with -ffp-contract=off): a few ulp."""
    from hlhgat import ops
    n = 300_001
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g).to(cuda)
    grads = [torch.randn(n, generator=g).to(cuda) for _ in range(3)]
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([ref], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd,
                           fused=True, capturable=True)
    p = p0.clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    step = torch.zeros((), device=cuda)
    for gr in grads:
        ref.grad = gr.clone()
        opt.step()
        ops.adam_flat(p, gr, m, v, step, 1e-3, (0.9, 0.999), 1e-8, wd)
    st = opt.state[ref]
    assert float(step) == 3.0
    assert torch.allclose(p, ref.detach(), rtol=1e-6, atol=1e-7)
    assert torch.allclose(m, st["exp_avg"], rtol=1e-5, atol=1e-7)
    assert torch.allclose(v, st["exp_avg_sq"], rtol=1e-5, atol=1e-9)


@pytest.mark.gpu
def test_l1_loss_matches_torch(cuda):
    """hlhgat.nn.L1Loss (hlhgat_l1_loss_fwd / _bwd) against torch.nn.L1Loss:
    the input gradient bit for bit (zeros, ties and a NaN included), the
    loss to fp32 rounding."""
    import hlhgat
    g = torch.Generator().manual_seed(7)
    for n in (1, 5, 1000, 4099):
        x = torch.randn(n, 1, generator=g)
        y = torch.randn(n, 1, generator=g)
        if n >= 5:
            y[:2] = x[:2]  # |x - y| = 0: sgn 0
        xs = []
        for crit in (torch.nn.L1Loss(), hlhgat.nn.L1Loss()):
            xd = x.to(cuda).requires_grad_(True)
            loss = crit(xd, y.to(cuda))
            (loss * 3.0).backward()
            xs.append((loss.detach().cpu(), xd.grad.cpu()))
        (l0, g0), (l1, g1) = xs
        assert torch.equal(g0, g1), n
        assert abs(float(l0) - float(l1)) <= 1e-6 * abs(float(l0)) + 1e-7, (n, float(l0), float(l1))
    xn = torch.tensor([[float("nan")], [1.0]], device=cuda, requires_grad=True)
    hlhgat.nn.L1Loss()(xn, torch.zeros(2, 1, device=cuda)).backward()
    assert xn.grad.cpu().tolist() == [[0.0], [0.5]]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["peptides", "cifar", "tsp"])
def test_head_graph_replay_equals_eager(cuda, kind):
    """The config 3/4/5 heads (level-batch lists for the attpool heads) run
    as replayed hipGraphs through TrainStep, one graph per batch shape (no
    host sync left in their forward / backward): the losses and every
    parameter after eager and graph-replayed steps are bitwise equal."""
    import hlhgat
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph, two_level_batch
    from hlhgat.train import TrainStep
    F = torch.nn.functional
    if kind == "tsp":
        raw = [collate([tsp_like_graph(s, n=400, k=6)], check_hodge=False) for s in (1, 2)]
        batches = [b.to(cuda) for b in raw]
        mk = lambda: hlhgat.HL_HGCNN_TSP_dense_int3_pyr(  # noqa: E731
            channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3)
        loss = lambda o, d: F.binary_cross_entropy_with_logits(  # noqa: E731
            o[0].view(-1), d.y.view(-1).float())
    else:
        batches = [[x.to(cuda) for x in two_level_batch(kind, 6, seed=s)] for s in (1, 2)]
        if kind == "cifar":
            mk = lambda: hlhgat.HL_HGCNN_CIFAR10SP_dense_int3_attpool(  # noqa: E731
                channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0)
            loss = lambda o, d: F.cross_entropy(o, d[0].y.view(-1).long())  # noqa: E731
        else:
            mk = lambda: hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(  # noqa: E731
                channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)
            loss = lambda o, d: F.binary_cross_entropy_with_logits(  # noqa: E731
                o, d[0].y.view(o.shape).float())
    res = []
    for graphs in (False, True):
        torch.manual_seed(0)
        m = mk().to(cuda).train()
        st = TrainStep(m, loss, lr=1e-3, graphs=graphs)
        ls = [float(st(batches[i % 2]).detach()) for i in range(5)]
        res.append((ls, {k: v.detach().clone() for k, v in m.state_dict().items()}, st.stats))
    (l_e, sd_e, _), (l_g, sd_g, stg) = res
    assert stg["captures"] == 2 and stg["replay"] == 3, stg
    assert l_e == l_g
    for k in sd_e:
        assert torch.equal(sd_e[k], sd_g[k]), k


@pytest.mark.gpu
def test_attpool_rejects_pool_at_last_level(cuda):
    """Pooling at the last level leaves the readout's rows (fine level)
    mismatched with the coarse level's graph sizes it pools by (the
    reference's readout, lib/Hodge_ST_Model.py:1076-1080): a clear error, not
    a partial readout with uncovered rows."""
    import hlhgat
    from hlhgat.synthetic import two_level_batch
    b = [x.to(cuda) for x in two_level_batch("peptides", 3, seed=1)]
    m = hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(
        channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=1).to(cuda)
    with pytest.raises(RuntimeError, match="pool_loc=1 must be below the last"):
        m(b)


# ---------------------------------------------------------------------------
# GPU: static-shape level-batch lists (attpool heads) and TSP batches
# ---------------------------------------------------------------------------
def _head_case(kind):
    """(raw host batches [3], model factory, loss) of a small config 3/4/5 head."""
    import hlhgat
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import tsp_like_graph, two_level_batch
    F = torch.nn.functional
    if kind == "tsp":
        raw = [collate([tsp_like_graph(s, n=300 + 40 * s, k=6)], check_hodge=False)
               for s in (1, 2, 3)]
        mk = lambda: hlhgat.HL_HGCNN_TSP_dense_int3_pyr(  # noqa: E731
            channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3)
        # BCE over the real edges (padding edges: zero mask, zero label; the
        # mean taken over the real count so padding leaves the objective alone)
        loss = lambda o, d: F.binary_cross_entropy_with_logits(  # noqa: E731
            o[0].view(-1), d.y.view(-1).float(), weight=d.x_s[:, 1],
            reduction="sum") / d.num_edge1.sum()
        return raw, mk, loss
    # the same graph count, different graphs: a per-graph readout's shapes
    # (y, num_node1) depend on the count, so a partial tail batch is its own bucket
    raw = [two_level_batch(kind, 6, seed=s) for s in (1, 2, 3)]
    if kind == "cifar":
        mk = lambda: hlhgat.HL_HGCNN_CIFAR10SP_dense_int3_attpool(  # noqa: E731
            channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0)
        loss = lambda o, d: F.cross_entropy(o, d[0].y.view(-1).long())  # noqa: E731
    else:
        mk = lambda: hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(  # noqa: E731
            channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)
        loss = lambda o, d: F.binary_cross_entropy_with_logits(  # noqa: E731
            o, d[0].y.view(o.shape).float())
    return raw, mk, loss


def _pad_all(kind, raw, quantum=128):
    from hlhgat.hodge_dataset import level_caps, pad_batch, pad_levels
    if kind == "tsp":
        caps = _caps_for(raw, quantum)
        return [pad_batch(b, caps) for b in raw]
    caps = level_caps(raw, quantum)
    return [pad_levels(b, caps) for b in raw]


def _dev(b, cuda):
    return [x.to(cuda) for x in b] if isinstance(b, list) else b.to(cuda)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["peptides", "cifar", "tsp"])
def test_padded_levels_match_unpadded(cuda, kind):
    """Static-shape level-batch lists (hodge_dataset.pad_levels: padding rows
    in no MLGC cluster, pos = inf) and padded TSP batches: the head's outputs,
    every parameter gradient and the running statistics equal the unpadded
    batch's (BN statistics, the attention's batch max and the readout over
    real rows only)."""
    raw, mk, loss = _head_case(kind)
    padded = _pad_all(kind, raw)
    res = []
    for batch in (raw[0], padded[0]):
        torch.manual_seed(0)
        m = mk().to(cuda).train()
        d = _dev(batch, cuda)
        out = m(d)
        o = out[0] if isinstance(out, tuple) else out
        if kind == "tsp":  # per-edge logits: compare the real edges
            o = o[:raw[0].x_s.size(0)]
            loss(out, d).backward()
        else:
            loss(out, d).backward()
        res.append((o.detach().cpu(), {k: p.grad.detach().cpu().clone()
                                       for k, p in m.named_parameters() if p.grad is not None},
                    {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}))
    (o0, g0, s0), (o1, g1, s1) = res
    assert torch.allclose(o0, o1, rtol=1e-5, atol=1e-6), (o0 - o1).abs().max()
    assert set(g0) == set(g1)
    for k in g0:
        scale = g0[k].abs().max().clamp_min(1e-6)
        assert ((g0[k] - g1[k]).abs().max() / scale) < 1e-4, k
        assert torch.isfinite(g1[k]).all(), k
    for k in s0:
        if s0[k].dtype.is_floating_point:
            assert torch.allclose(s0[k], s1[k], rtol=1e-5, atol=1e-6), k


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["peptides", "cifar", "tsp"])
def test_padded_levels_share_one_graph(cuda, kind):
    """Three batches of different shapes padded to one bucket replay ONE
    captured step (the level-batch copy-in loads each batch's data: losses
    differ between batches), bitwise equal to eager steps."""
    raw, mk, loss = _head_case(kind)
    batches = [_dev(b, cuda) for b in _pad_all(kind, raw)]
    order = [0, 1, 2, 1, 0, 2]
    from hlhgat.train import TrainStep
    res = []
    for graphs in (False, True):
        torch.manual_seed(0)
        m = mk().to(cuda).train()
        st = TrainStep(m, loss, lr=1e-3, graphs=graphs)
        ls = [float(st(batches[i]).detach()) for i in order]
        res.append((ls, {k: v.detach().clone() for k, v in m.state_dict().items()}, st.stats))
    (l_e, sd_e, _), (l_g, sd_g, stg) = res
    assert stg["captures"] == 1 and stg["replay"] == len(order) - 1, stg
    assert len(set(l_g[:3])) == 3  # each replay ran on its own batch's data
    assert l_e == l_g
    for k in sd_e:
        assert torch.equal(sd_e[k], sd_g[k]), k


@pytest.mark.gpu
def test_staged_double_buffered_steps_bitwise(cuda):
    """TrainStep.stage (the loader-fed path: host batches uploaded on a copy
    stream straight into the static buffers of the graph that replays next,
    two captured graphs per shape used in turn, the next batch staged while
    the current step runs) gives the bits of step(device batch): losses and
    every parameter / running statistic, two shapes interleaved."""
    import hlhgat
    from hlhgat import ops
    from hlhgat.synthetic import zinc_like_batch
    from hlhgat.train import Staged, TrainStep
    import copy
    b2 = copy.copy(zinc_like_batch(40, seed=3))  # the shape of [0], other values
    g = torch.Generator().manual_seed(11)
    b2.x_t = b2.x_t + 0.25 * torch.randn(b2.x_t.shape, generator=g)
    b2.x_s = b2.x_s + 0.25 * torch.randn(b2.x_s.shape, generator=g)
    b2.y = b2.y + 0.5
    host = [zinc_like_batch(40, seed=3), zinc_like_batch(33, seed=4), b2]
    order = [0, 1, 0, 2, 1, 0, 2, 1, 1, 0, 2]
    l_ref, sd_ref, _ = _run(True, True, [copy.copy(b).to(cuda) for b in host], order)
    assert all(not b.x_t.is_cuda for b in host)  # Batch.to works in place: copies went
    ops.set_stream_fork(True)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(cuda).train()
    crit = torch.nn.L1Loss()
    step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                     weight_decay=1e-3, graphs=True)
    cs = torch.cuda.Stream(device=cuda)
    losses = []
    nxt = step.stage(host[order[0]], cs)
    slots_used = 0
    for k in range(len(order)):
        cur = nxt
        if k + 1 < len(order):
            nxt = step.stage(host[order[k + 1]], cs)
        assert isinstance(cur, Staged)
        slots_used += cur.slot is not None
        losses.append(float(step(cur)))
    torch.cuda.synchronize()
    _check_errors()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    assert losses == l_ref, (losses, l_ref)
    for key in sd_ref:
        assert torch.equal(sd_ref[key], sd[key]), key
    # two shapes x two slots captured; later steps went straight into a slot
    assert step.stats["captures"] == 4 and slots_used >= 5, (step.stats, slots_used)


@pytest.mark.gpu
def test_staged_arena_batches_single_copy_bitwise(cuda):
    """PackedGraphs.collate batches (pinned, every tensor a view of one host
    arena): TrainStep.stage uploads each into a graph's device arena of the
    same layout in ONE copy; losses and parameters equal those of
    step(device batch) with per-tensor copy-in, bit for bit."""
    import hlhgat
    import numpy as np
    from hlhgat.hodge_dataset import PackedGraphs
    from hlhgat.synthetic import zinc_like_graph
    from hlhgat.train import TrainStep
    ds = PackedGraphs([zinc_like_graph(500 + i) for i in range(60)], check_hodge=False)
    idx = [np.arange(k * 12, (k + 1) * 12) for k in range(5)]
    cs = [ds.caps_for(i, 128) for i in idx]
    caps = {k: max(c[k] for c in cs) for k in cs[0]}
    order = [0, 1, 2, 3, 4, 1, 0, 3]
    l_ref, sd_ref, _ = _run(True, True, [ds.collate(idx[i], caps).to(cuda) for i in range(5)],
                            order)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(cuda).train()
    crit = torch.nn.L1Loss()
    step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                     weight_decay=1e-3, graphs=True)
    cs_ = torch.cuda.Stream(device=cuda)
    host = [ds.collate(idx[i], caps, pin=True) for i in order]
    assert all(hasattr(b, "_arena") and b._arena.is_pinned() for b in host)
    losses, nxt = [], step.stage(host[0], cs_)
    single = 0
    for k in range(len(order)):
        cur = nxt
        if k + 1 < len(order):
            nxt = step.stage(host[k + 1], cs_)
        if cur.slot is not None:
            single += hasattr(cur.slot.batch, "_arena")
        losses.append(float(step(cur)))
    torch.cuda.synchronize()
    _check_errors()
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    assert losses == l_ref, (losses, l_ref)
    for key in sd_ref:
        assert torch.equal(sd_ref[key], sd[key]), key
    assert step.stats["captures"] == 2 and single >= 4, (step.stats, single)


@pytest.mark.gpu
def test_staged_three_ahead_bitwise(cuda):
    """Staging more batches ahead than a shape has captured graphs (three
    ahead, two graphs): a graph whose buffers still hold a staged batch is
    never picked again (the batch would be overwritten before its step and
    never trained); the extra batch goes to fresh device tensors.  Losses and
    parameters bitwise those of step(device batch) in the same order."""
    import copy
    import hlhgat
    from hlhgat.synthetic import zinc_like_batch
    from hlhgat.train import TrainStep
    g = torch.Generator().manual_seed(5)
    host = []
    for k in range(4):  # one shape, four value sets
        b = copy.copy(zinc_like_batch(36, seed=8))
        b.x_t = b.x_t + 0.3 * k * torch.randn(b.x_t.shape, generator=g)
        b.y = b.y + 0.1 * k
        host.append(b)
    order = [0, 1, 2, 3, 0, 2, 1, 3, 3, 0, 1, 2]
    l_ref, sd_ref, _ = _run(True, True, [copy.copy(b).to(cuda) for b in host], order)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(cuda).train()
    crit = torch.nn.L1Loss()
    step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                     weight_decay=1e-3, graphs=True)
    assert step.stage_slots == 2
    cs = torch.cuda.Stream(device=cuda)
    ahead = 3
    queue = [step.stage(host[order[k]], cs) for k in range(ahead)]
    losses = []
    for k in range(len(order)):
        cur = queue.pop(0)
        if k + ahead < len(order):
            queue.append(step.stage(host[order[k + ahead]], cs))
        pend = [sl.pending for sl in step._graphs[cur.key].slots] if cur.key in step._graphs \
            else []
        assert all(p <= 1 for p in pend), pend  # never two batches waiting in one graph
        losses.append(float(step(cur)))
    torch.cuda.synchronize()
    _check_errors()
    assert step._outstanding == 0
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    assert losses == l_ref, (losses, l_ref)
    for key in sd_ref:
        assert torch.equal(sd_ref[key], sd[key]), key


@pytest.mark.gpu
@pytest.mark.parametrize("wait,thread,slots", [("host", True, 4), ("device", True, 3),
                                               ("host", False, 4)])
def test_staged_feed_thread_bitwise(cuda, monkeypatch, wait, thread, slots):
    """hlhgat.loader.StagedFeed: a feeder thread (or, thread=False, this
    thread between its steps) stages GraphLoader batches (native collate on
    worker threads, pinned arenas) two ahead while this thread replays, and
    the shape's later graphs are captured meanwhile (the collation and feeder
    threads run beside a thread-local capture); the slot's release waited for
    on the host or by the copy stream (train.STAGE_WAIT); losses and
    parameters bitwise those of step(device batch) in order."""
    import hlhgat.train as train_mod
    monkeypatch.setattr(train_mod, "STAGE_WAIT", wait)
    import numpy as np
    import hlhgat
    from hlhgat.hodge_dataset import PackedGraphs
    from hlhgat.loader import GraphLoader, StagedFeed
    from hlhgat.synthetic import zinc_like_graph
    from hlhgat.train import TrainStep
    ds = PackedGraphs([zinc_like_graph(700 + i) for i in range(96)], check_hodge=False)
    ld = GraphLoader(ds, 12, caps=None, workers=3, prefetch=6, pin=True)
    idxs = ld.batch_indices(0)
    caps = ld.epoch_caps(idxs)
    ref_batches = [ds.collate(i, caps).to(cuda) for i in idxs]
    l_ref, sd_ref, _ = _run(True, True, ref_batches, list(range(len(idxs))))
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(cuda).train()
    crit = torch.nn.L1Loss()
    step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                     weight_decay=1e-3, graphs=True, stage_slots=slots)
    losses = []
    for st in StagedFeed(ld, step, depth=2, thread=thread):
        losses.append(float(step(st)))
    torch.cuda.synchronize()
    _check_errors()
    assert len(losses) == len(idxs) and step._outstanding == 0
    assert step.stats["captures"] == slots, step.stats
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    assert losses == l_ref, (losses, l_ref)
    for key in sd_ref:
        assert torch.equal(sd_ref[key], sd[key]), key
    assert np.isfinite(losses).all()


@pytest.mark.gpu
@pytest.mark.parametrize("thread", [True, False])
def test_staged_feed_early_close_then_stage_again(cuda, thread):
    """leaving StagedFeed(GraphLoader.stream(), ...) early gives
    back the batches it staged and nobody stepped (TrainStep.unstage): after
    several early exits the step's outstanding count is 0, every slot's
    pending count is 0, and staging / stepping goes on (it would raise
    'more than 8 staged batches outstanding' with the handles leaked)."""
    import hlhgat
    from hlhgat.hodge_dataset import PackedGraphs
    from hlhgat.loader import GraphLoader, StagedFeed
    from hlhgat.synthetic import zinc_like_graph
    from hlhgat.train import TrainStep
    ds = PackedGraphs([zinc_like_graph(900 + i) for i in range(48)], check_hodge=False)
    ld = GraphLoader(ds, 12, caps=None, workers=2, prefetch=4, pin=True)
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to(cuda).train()
    crit = torch.nn.L1Loss()
    step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                     graphs=True, stage_slots=4)
    n = 0
    for rnd in range(5):
        it = ld.stream()
        try:
            for k, st in enumerate(StagedFeed(it, step, depth=3, thread=thread)):
                if k == 2 and rnd % 2:
                    break  # left before stepping the handle
                step(st)
                n += 1
                if k == 2:
                    break
        finally:
            it.close()
        assert step._outstanding == 0, (rnd, step._outstanding)
        for ent in step._graphs.values():
            assert all(sl.pending == 0 for sl in ent.slots), rnd
    torch.cuda.synchronize()
    _check_errors()
    assert n == 3 * 3 + 2 * 2
    assert step.stats["replay"] >= 8


@pytest.mark.gpu
def test_own_streams_never_from_torch_pool(cuda):
    """Round 5's host segfault: torch's 32-stream round-robin pool handed a
    test's copy stream out again as a capture-joined side stream.  The
    library's capture, copy and side streams (Python roles and the C++
    fork's side stream) are its own: none of them is among 64 consecutive
    torch.cuda.Stream() handles, and each role keeps one stream."""
    from hlhgat import ops
    idx = cuda.index if cuda.index is not None else torch.cuda.current_device()
    ours = {ops.own_stream(cuda, r).cuda_stream for r in ("capture", "copy")}
    ours |= {ops.side_stream(cuda, k).cuda_stream for k in (0, 1)}
    ours.add(int(ops._ext.fork_side_stream(idx)))
    assert len(ours) == 5
    pool = {torch.cuda.Stream(device=cuda).cuda_stream for _ in range(64)}
    assert not (ours & pool), "a library stream came from torch's pool"
    assert ops.own_stream(cuda, "copy").cuda_stream in ours  # cached per role
    # unmasked streams run on every CU
    n_cu = torch.cuda.get_device_properties(cuda).multi_processor_count
    mask = ops.stream_cu_mask(ops.own_stream(cuda, "capture"), words=(n_cu + 31) // 32)
    assert sum(bin(w).count("1") for w in mask) == n_cu


@pytest.mark.gpu
def test_cu_masked_stream_runs_kernels(cuda):
    """hlhgat_stream_create with a CU mask (the config-3 producer's stream):
    the mask reads back as set, and library kernels launched on the stream
    give the same results as on the default stream."""
    from hlhgat import ops
    n_cu = torch.cuda.get_device_properties(cuda).multi_processor_count
    words = (n_cu + 31) // 32
    mask = [0] * words
    for c in range(0, n_cu, 8):  # one CU in eight: every XCD keeps some
        mask[c // 32] |= 1 << (c % 32)
    s = ops.own_stream(cuda, "test-masked", cu_mask=mask)
    got = ops.stream_cu_mask(s, words=words)
    assert got == mask, (got, mask)
    x = torch.randn(5000, 64, device=cuda)
    w = torch.randn(32, 64, device=cuda)
    ref = ops.linear_blocks([x], w, None)
    torch.cuda.synchronize()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out = ops.linear_blocks([x], w, None)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["peptides", "cifar"])
@pytest.mark.parametrize("padded", [False, True])
def test_pool_tables_bitwise_device_cluster_csr(cuda, kind, padded):
    """An attpool level list carrying its collate-time MLGC cluster CSR
    (hodge_dataset.pool_tables) gives the same outputs, gradients and running
    statistics, bit for bit, as the same list without it (the cluster CSR
    sorted on the device inside the step), padded or not."""
    from hlhgat.hodge_dataset import pool_tables
    raw, mk, loss = _head_case(kind)
    base = _pad_all(kind, raw)[0] if padded else raw[0]
    res = []
    for tables in (False, True):
        datas = []
        for b in base:
            c = b.__class__.__new__(b.__class__)
            for k, v in vars(b).items():
                if not k.startswith("pool_"):
                    setattr(c, k, v)
            datas.append(c)
        if tables:
            pool_tables(datas)
            assert datas[0].pool_rowptr_t is not None
        torch.manual_seed(0)
        m = mk().to(cuda).train()
        d = _dev(datas, cuda)
        out = m(d)
        loss(out, d).backward()
        res.append((out.detach().cpu(), {k: p.grad.detach().cpu().clone()
                                         for k, p in m.named_parameters() if p.grad is not None},
                    {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}))
    (o0, g0, s0), (o1, g1, s1) = res
    assert torch.equal(o0, o1)
    assert set(g0) == set(g1) and all(torch.equal(g0[k], g1[k]) for k in g0)
    assert all(torch.equal(s0[k], s1[k]) for k in s0)
