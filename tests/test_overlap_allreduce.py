"""The data-parallel gradient exchange in buckets, each all-reduced as soon as
the backward has finished its gradients (hlhgat.train.TrainStep overlap;
SURVEY §8e: the reference-side drop-in replaces DDP, whose bucketed,
backward-overlapped all-reduce is the loop main_pepfunc_HL_HGCNN_dense_int3_
attpool.py:171-225 / main_TSP_HL_HGCNN_dense_int3_pyr.py:311-354 would get
under 8-GPU DDP).

CPU (gloo, world 2): a plain torch model through TrainStep with the overlap
and several buckets gives BITWISE the parameters of the one-bucket path (with
two ranks each element's sum is a + b whatever the bucketing); the buckets
cover the flat buffer exactly, last parameters first; unused parameters
still reach the exchange (their bucket launches after the backward).
GPU: the product heads over two gloo ranks sharing the card, overlapped vs
one bucket, bitwise; RCCL world 1 (captured): test_rccl_capture.py.
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist

from test_sync_bn import _env, _run_ranks

STEPS = 3


class _Net(torch.nn.Module):
    def __init__(self, unused=False):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(24, 64)
        self.b = torch.nn.Linear(64, 64)
        self.c = torch.nn.Linear(64, 8)
        self.dead = torch.nn.Linear(3, 3) if unused else None  # never used in forward

    def forward(self, batch):  # batch = (x, y), as TrainStep hands it over
        return self.c(torch.relu(self.b(torch.relu(self.a(batch[0])))))


def _data(rank, step):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(32, 24, generator=g), torch.randn(32, 8, generator=g)


def _worker(rank, world, port, q, overlap, bucket_mb, unused):
    _env(rank, world, port)
    from hlhgat.train import TrainStep
    dist.init_process_group("gloo")
    m = _Net(unused)
    mse = torch.nn.MSELoss()
    st = TrainStep(m, lambda o, b: mse(o, b[1]), lr=1e-2, weight_decay=1e-3, graphs=False,
                   overlap=overlap, bucket_mb=bucket_mb)
    info = dict(overlap=st.overlap, ranges=list(getattr(st, "_ranges", [])),
                offsets=list(st._offsets), numels=[p.numel() for p in st.params])
    for s in range(STEPS):
        x, y = _data(rank, s)
        st((x, y))
    q.put((rank, dict(flat=st.flat.detach().numpy().copy(), stats=dict(st.overlap_stats),
                      **info)))
    dist.destroy_process_group()


@pytest.mark.parametrize("unused", [False, True])
def test_overlapped_buckets_bitwise_one_bucket_gloo(unused):
    one = _run_ranks(_worker, 2, False, None, unused)
    many = _run_ranks(_worker, 2, True, 0.001, unused)  # 262 floats: one Linear per bucket
    assert not one[0]["overlap"] and many[0]["overlap"]
    ranges = many[0]["ranges"]
    assert len(ranges) >= 3, ranges
    # the buckets tile the flat buffer, last parameters first
    total = sum(many[0]["numels"])
    cov = sorted(ranges)
    assert cov[0][0] == 0 and cov[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(cov, cov[1:]))
    assert ranges[0][1] == total
    # issued from the backward's hooks; the bucket holding the unused
    # parameters (registered last: the first bucket) after the backward
    st = many[0]["stats"]
    assert st["after_backward"] == (STEPS if unused else 0), st
    assert st["in_backward"] == STEPS * len(ranges) - st["after_backward"], st
    for r in range(2):
        assert np.array_equal(one[r]["flat"], many[r]["flat"]), r
    assert np.array_equal(many[0]["flat"], many[1]["flat"])


def test_overlap_off_without_exchange():
    """One process (no process group): no buckets, no hooks at work."""
    from hlhgat.train import TrainStep
    m = torch.nn.Linear(4, 2)
    st = TrainStep(m, lambda o, b: o.sum(), graphs=False, overlap=True)
    assert not st.overlap and st._buckets == []
    st(torch.randn(3, 4))
