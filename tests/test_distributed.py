"""Data-parallel path on CPU: 2 gloo ranks, graphs sharded by rank, DDP
gradient all-reduce == mean of the per-shard gradients (the only exchange
step of the HL-HGAT data path)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


KW = dict(channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, keig=15)


def _shard_batch(rank, world, n_graphs=12):
    from hlhgat.distributed import shard_graphs
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import zinc_like_graph
    graphs = [zinc_like_graph(100 + i) for i in range(n_graphs)]
    return collate(shard_graphs(graphs, rank, world))


def _worker(rank, world, port, out_q):
    sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from hlhgat.distributed import init_distributed, max_over_ranks, wrap_ddp
    from oracle.hodge_ref import RefZincModel
    r, w, dev = init_distributed("gloo")
    torch.manual_seed(0)
    model = RefZincModel(**KW).train()
    ddp = wrap_ddp(model, dev)
    b = _shard_batch(r, w)
    out = ddp(b)
    loss = torch.nn.functional.l1_loss(out.view(-1), b.y.view(-1))
    loss.backward()
    grads = {k: p.grad.clone() for k, p in model.named_parameters()}
    t = max_over_ranks(float(r + 1))
    out_q.put((r, {k: v.numpy() for k, v in grads.items()}, t))
    dist.destroy_process_group()


def test_shard_range_balanced():
    from hlhgat.distributed import shard_by_weight, shard_range
    parts = [shard_range(10, r, 4) for r in range(4)]
    assert parts == [(0, 3), (3, 6), (6, 8), (8, 10)]
    groups = shard_by_weight([5, 1, 1, 1, 1, 1], 2)
    assert sorted(sum(groups, [])) == list(range(6))
    assert groups[0] == [0]


def test_ddp_gloo_two_ranks_matches_mean_of_shard_gradients():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, g, t = q.get(timeout=300)
        res[r] = (g, t)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # both ranks hold the same all-reduced gradient, and the timing reduce is a MAX
    g0, g1 = res[0][0], res[1][0]
    for k in g0:
        assert (abs(g0[k] - g1[k]).max() if g0[k].size else 0) < 1e-6, k
    assert res[0][1] == res[1][1] == 2.0
    # = mean over ranks of the per-shard gradients computed independently
    from oracle.hodge_ref import RefZincModel
    ref = {}
    for r in range(world):
        torch.manual_seed(0)
        m = RefZincModel(**KW).train()
        b = _shard_batch(r, world)
        out = m(b)
        torch.nn.functional.l1_loss(out.view(-1), b.y.view(-1)).backward()
        for k, p in m.named_parameters():
            ref[k] = ref.get(k, 0) + p.grad / world
    for k, v in ref.items():
        scale = max(1.0, float(v.abs().max()))
        assert float(abs(torch.from_numpy(g0[k]) - v).max()) <= 1e-5 * scale, k


def _gmax_worker(rank, world, port, out_q):
    sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from hlhgat.distributed import global_max, init_distributed
    init_distributed("gloo")
    x = torch.arange(5.0).mul(rank + 1).add(rank).requires_grad_(True)  # max on rank 1 only
    m = global_max(x)
    (3.0 * (rank + 1) * m).backward()  # a different upstream gradient per rank
    out_q.put((rank, float(m), x.grad.tolist()))
    dist.destroy_process_group()


def test_global_max_two_ranks_matches_single_process():
    """att / att.max() of the attpool heads (lib/Hodge_ST_Model.py:1061-1062)
    is a BATCH max: under graph sharding it must span every rank (SURVEY §8e
    caveat 2).  global_max over 2 gloo ranks == max of the concatenation, and
    its gradient is that of the data-parallel objective (1/W)·Σ_r L_r: each
    rank's x.grad, averaged over ranks as DDP averages parameter gradients,
    equals the single-process gradient of that objective."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gmax_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (m, g)) for r, m, g in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
    xs = [torch.arange(5.0).mul(r + 1).add(r).requires_grad_(True) for r in range(world)]
    m_ref = torch.cat(xs).max()
    sum(3.0 * (r + 1) * m_ref for r in range(world)).div(world).backward()
    for r in range(world):
        assert res[r][0] == float(m_ref)
        assert [v / world for v in res[r][1]] == xs[r].grad.tolist()
    assert any(v != 0 for v in res[1][1]) and not any(res[0][1])


class _PartlyUnused(torch.nn.Module):
    """Stand-in for the attpool heads: a parameter the forward never uses."""
    ddp_find_unused_parameters = True

    def __init__(self):
        super().__init__()
        self.used = torch.nn.Linear(3, 2)
        self.unused = torch.nn.Linear(3, 2)

    def forward(self, x):
        return self.used(x)


def _unused_worker(rank, world, port, out_q):
    sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from hlhgat.distributed import init_distributed, wrap_ddp
    _, _, dev = init_distributed("gloo")
    torch.manual_seed(0)
    m = _PartlyUnused()
    ddp = wrap_ddp(m, dev)
    ddp(torch.full((4, 3), float(rank + 1))).sum().backward()
    out_q.put((rank, m.used.weight.grad.tolist(), m.unused.weight.grad))
    dist.destroy_process_group()


def test_ddp_unused_parameters_flag_gives_the_mean_gradient():
    """wrap_ddp honours a model's ddp_find_unused_parameters flag: without it
    the bucket holding an unused parameter is never reduced and every gradient
    stays pre-scaled by 1/W (measured on the pepfunc head: tools/ddp_check.py)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_unused_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, gu)) for r, g, gu in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # d/dW sum(W x + b) over 4 rows of value v = 4 v per entry; mean over ranks v = 1, 2
    for r in range(world):
        assert res[r][0] == [[6.0] * 3] * 2
        assert res[r][1] is None


def _bench(argv, env_extra=None, timeout=240):
    import json
    import subprocess
    env = dict(os.environ)
    env.pop("RANK", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + argv, env=env,
                       capture_output=True, text=True, timeout=timeout, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_spawns_n_ranks(n):
    """`python bench.py --gpus N` (no torchrun env) starts N ranks itself and
    rank 0 reports n_gpus == N (gloo dry run of the same launcher)."""
    r, line = _bench(["--gpus", str(n), "--dry-run", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert line is not None and line["n_gpus"] == n and line["ranks_seen"] == n
    assert line["dry_run"] is True and line["steps"] == 2


@pytest.mark.parametrize("workload", ["cfg4", "cfg5"])
def test_bench_workload_dry_run(workload):
    """`--workload cfg4|cfg5` (BASELINE configs[3] peptides, configs[4] TSP:
    the 8-GPU configs) goes through the same launcher: 2 ranks, the head's
    own gradient bucket all-reduced on gloo."""
    r, line = _bench(["--gpus", "2", "--dry-run", "--workload", workload, "--steps", "2",
                      "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2 and line["workload"] == workload
    assert line["bucket_floats"] > 1_000_000


def test_bench_rank_count_mismatch_fails():
    """Under torchrun with 2 ranks, --gpus 3 must fail instead of reporting
    a wrong n_gpus."""
    import subprocess
    env = dict(os.environ)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "3", "--dry-run", "--steps", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode != 0
    assert "world size 2 != --gpus 3" in (r.stdout + r.stderr)
