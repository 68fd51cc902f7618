"""Losses of TrainStep runs, eager vs graph-replayed, with / without the NEInt prepack."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
import torch  # noqa: E402
import hlhgat  # noqa: E402
from hlhgat import ops  # noqa: E402
from hlhgat.synthetic import zinc_like_batch  # noqa: E402
from hlhgat.train import TrainStep  # noqa: E402

KW = dict(channels=[1, 1], filters=[32, 32], mlp_channels=[64], K=3, keig=15)
batches = [zinc_like_batch(40, seed=3).to("cuda"), zinc_like_batch(33, seed=4).to("cuda"),
           zinc_like_batch(40, seed=3).to("cuda")]
order = [0, 1, 0, 1, 2, 0]
for pre in (False, True):
    for graphs in (False, True):
        ops.PREPACK = pre
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to("cuda").train()
        crit = torch.nn.L1Loss()
        step = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                         weight_decay=1e-3, graphs=graphs)
        losses = [round(float(step(batches[i])), 7) for i in order]
        print(f"prepack={pre} graphs={graphs} {losses}", flush=True)
