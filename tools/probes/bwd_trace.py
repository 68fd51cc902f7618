"""One eager config-2 training step (temporary probe for launch traces)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    sys.path.insert(0, p)
import torch
import bench, hlhgat
from hlhgat.train import TrainStep
dev = torch.device("cuda:0")
batches, caps, _, _, _ = bench.make_batches(1, 0, dev)
m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
crit = hlhgat.nn.L1Loss()
st = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
               weight_decay=1e-3, graphs=False)
st(batches[0]); torch.cuda.synchronize()
print("---- step 2", file=sys.stderr, flush=True)
st(batches[0]); torch.cuda.synchronize()
