"""Diagnose eager vs graph-replay differences of a small attpool head."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hl-hgat_amd")]
import torch  # noqa: E402
import hlhgat  # noqa: E402
from hlhgat.synthetic import two_level_batch  # noqa: E402
from hlhgat.train import TrainStep  # noqa: E402
from hlhgat import ops  # noqa: E402
F = torch.nn.functional
cuda = torch.device("cuda:0")
kind = sys.argv[1] if len(sys.argv) > 1 else "peptides"
bs = {s: [x.to(cuda) for x in two_level_batch(kind, 6, seed=s)] for s in (1, 2)}


def mk():
    if kind == "cifar":
        return hlhgat.HL_HGCNN_CIFAR10SP_dense_int3_attpool(
            channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0)
    return hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(
        channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)


def loss(o, d):
    if kind == "cifar":
        return F.cross_entropy(o, d[0].y.view(-1).long())
    return F.binary_cross_entropy_with_logits(o, d[0].y.view(o.shape).float())


if os.environ.get("NOFORK") == "1":
    ops.set_stream_fork(False)
GRAPHS = os.environ.get("GRAPHS", "01")


def run(graphs, order, n=5):
    torch.manual_seed(0)
    m = mk().to(cuda).train()
    st = TrainStep(m, loss, lr=1e-3, graphs=graphs)
    ls = [float(st(bs[order[i % len(order)]]).detach()) for i in range(n)]
    return ls


print(json.dumps({k: [tuple(x.x_t.shape) + tuple(x.x_s.shape) for x in v] for k, v in bs.items()}))
reps = int(os.environ.get("REPS", "1"))
for order in ([2], [1, 2]):
    es = [run(False, order) for _ in range(reps)]
    gs = [run(True, order) for _ in range(reps)] if "1" in GRAPHS else es
    print(json.dumps({"order": order, "eager_distinct": len({tuple(x) for x in es}),
                      "graph_distinct": len({tuple(x) for x in gs}),
                      "equal": all(x == es[0] for x in es + gs)}), flush=True)
