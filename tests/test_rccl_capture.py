"""RCCL inside the captured step (one GPU, a world-size-1 `nccl` group).

Under RCCL, TrainStep captures the step's collectives into its hipGraph: the
forward ones (the CIFAR attpool head's batch-global attention max,
lib/Hodge_ST_Model.py:1061-1062; SyncBatchNorm's statistics all-reduce) and
the gradient all-reduce + 1/W scale + Adam after the backward.  A one-GPU box
cannot run two RCCL ranks, so the child process forms a one-rank nccl group
with distributed.COLLECTIVES_AT_WORLD_1 = True: every collective then really
executes (RCCL kernels on a one-rank communicator) and is captured.  The
replayed steps must give the bits of the eager steps (same collectives, run
eagerly) -- losses and every parameter / running statistic.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["cifar_global_max", "zinc_sync_bn", "zinc_overlap",
                                  "pepfunc_overlap"])
def test_rccl_collectives_captured_replay_equals_eager(cuda, case):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), case], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["losses_equal"] and not res["param_diffs"], res
    # SyncBatchNorm's statistics all-reduces (forward and backward) and the
    # attpool heads' attention max are captured with the step
    assert not res["graphs_off"], res
    assert res["captures"] == 2 and res["replay"] >= 3, res
    assert res["exchange_in_graph"] is True
    # RCCL's kernels inside the graphs (names resolved: ours are found by name)
    assert res["own_kernels_in_graphs"] > 0 and res["foreign_kernels_in_graphs"] > 0, res
    if case.endswith("_overlap"):
        # the gradient all-reduce in buckets issued from the backward's hooks
        # (deferred split reductions flushed per bucket, the chains' side
        # streams joined), captured; the same bits as the one-bucket step
        assert res["overlap"] and res["buckets"] >= 3, res
        assert res["overlap_stats"]["in_backward"] > 0, res
        assert res["one_bucket_equal"], res


def _child(case):
    import faulthandler
    faulthandler.enable()
    sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
    import torch
    import torch.distributed as dist
    import hlhgat
    from hlhgat import distributed as hd
    from hlhgat.train import TrainStep
    hd.COLLECTIVES_AT_WORLD_1 = True
    from hlhgat import train
    train.KEEP_GRAPHS = True  # the captured hipGraph_t stays inspectable

    def note(*a):
        print("[child]", *a, file=sys.stderr, flush=True)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    F = torch.nn.functional
    if case == "cifar_global_max":
        from hlhgat.synthetic import two_level_batch
        batches = [[x.to(dev) for x in two_level_batch("cifar", 6, seed=s)] for s in (1, 2)]

        def mk():
            return hlhgat.HL_HGCNN_CIFAR10SP_dense_int3_attpool(
                channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0)

        def loss(o, d):
            return F.cross_entropy(o, d[0].y.view(-1).long())
    elif case == "pepfunc_overlap":
        from hlhgat.synthetic import two_level_batch
        batches = [[x.to(dev) for x in two_level_batch("peptides", 6, seed=s)] for s in (1, 2)]

        def mk():
            return hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(
                channels=[1, 1], filters=[32, 64], mlp_channels=[64], K=3, pool_loc=0)

        def loss(o, d):
            return F.binary_cross_entropy_with_logits(o, d[0].y.view(o.shape).float())
    else:
        from hlhgat.synthetic import zinc_like_batch
        batches = [zinc_like_batch(40, seed=3).to(dev), zinc_like_batch(33, seed=4).to(dev)]

        def mk():
            m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[1, 1], filters=[32, 32],
                                                    mlp_channels=[64], K=3, keig=15)
            return m if case == "zinc_overlap" else hd.convert_sync_batchnorm(m)

        crit = torch.nn.L1Loss()

        def loss(o, d):
            return crit(o.view(-1, 1), d.y.view(-1, 1))
    order = [0, 1, 0, 1, 1, 0]
    ov = case.endswith("_overlap")
    # small buckets: several per step at these widths
    kw = dict(overlap=True, bucket_mb=0.02) if ov else {}
    res = []
    for graphs, kwr in ((False, kw), (True, kw)) + (((True, dict(overlap=False)),) if ov else ()):
        torch.manual_seed(0)
        m = mk().to(dev).train()
        st = TrainStep(m, loss, lr=1e-3, weight_decay=1e-3, graphs=graphs, **kwr)
        ls = []
        for k, i in enumerate(order):
            ls.append(float(st(batches[i]).detach()))
            note(f"graphs={graphs} {kwr} step {k}: {st.stats} {st.overlap_stats}")
        torch.cuda.synchronize()
        res.append((ls, {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}, st))
    (l_e, sd_e, _), (l_g, sd_g, st) = res[:2]
    one_equal = None
    if ov:
        l_1, sd_1, _ = res[2]
        one_equal = l_1 == l_g and all(torch.equal(sd_1[k], sd_g[k]) for k in sd_g)
    # kernels in the captured step graphs that are not this library's (k_*):
    # RCCL's (and torch's few elementwise ones, which the eager step has too)
    n_coll, n_ours = 0, 0
    for ent in st._graphs.values():
        k, ours = hlhgat.ops.graph_kernel_count(ent.graph.raw_cuda_graph(), "k_")
        n_coll += k - ours
        n_ours += ours
    hlhgat.ops.check_device_errors()
    print(json.dumps({"captures": st.stats["captures"], "replay": st.stats["replay"],
                      "exchange_in_graph": st._exchange_in_graph,
                      "foreign_kernels_in_graphs": n_coll, "own_kernels_in_graphs": n_ours,
                      "graphs_off": st.graphs_off, "overlap": st.overlap,
                      "buckets": len(st._buckets), "overlap_stats": st.overlap_stats,
                      "one_bucket_equal": one_equal,
                      "losses_equal": l_e == l_g, "losses": [l_e, l_g],
                      "param_diffs": [k for k in sd_e if not torch.equal(sd_e[k], sd_g[k])]}))
    dist.destroy_process_group()


if __name__ == "__main__":
    _child(sys.argv[1])
