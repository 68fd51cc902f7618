"""Uninitialised-read probe for the attpool heads: before each eager step the
caching allocator's free blocks are filled with NaN (large and small pools);
forward / backward hooks then name the first module whose output or input
gradient holds a NaN."""
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
if os.environ.get("NOFORK") == "1":
    ops.set_stream_fork(False)
bs = {s: [x.to(cuda) for x in two_level_batch(kind, 6, seed=s)] for s in (1, 2)}
torch.manual_seed(0)
if kind == "cifar":
    m = hlhgat.HL_HGCNN_CIFAR10SP_dense_int3_attpool(
        channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0)
    loss = lambda o, d: F.cross_entropy(o, d[0].y.view(-1).long())  # noqa: E731
else:
    m = hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(
        channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)
    loss = lambda o, d: F.binary_cross_entropy_with_logits(o, d[0].y.view(o.shape).float())  # noqa: E731
m = m.to(cuda).train()
events = []


def bad(t):
    if isinstance(t, torch.Tensor):
        return t.is_floating_point() and bool(torch.isnan(t).any())
    if isinstance(t, (list, tuple)):
        return any(bad(x) for x in t)
    return False


for name, mod in m.named_modules():
    mod.register_forward_hook(lambda mo, i, o, n=name: events.append(("fwd", n)) if bad(o) else None)
    mod.register_full_backward_hook(
        lambda mo, gi, go, n=name: events.append(("bwd_in", n, bad(go))) if bad(gi) else None)


def poison():
    torch.cuda.synchronize()
    free = torch.cuda.mem_get_info()[0]
    big = torch.empty(int(min(free * 0.5, 8 << 30)) // 4, dtype=torch.float32, device=cuda)
    big.fill_(float("nan"))
    small = [torch.full((256 * 1024 // 4 * (1 + i % 4),), float("nan"), device=cuda)
             for i in range(2000)]
    torch.cuda.synchronize()
    del big, small


st = TrainStep(m, loss, lr=1e-3, graphs=False)
for i, s in enumerate([1, 2, 1, 2]):
    poison()
    events.clear()
    l = float(st(bs[s]).detach())
    torch.cuda.synchronize()
    pn = [n for n, p in m.named_parameters() if bad(p)]
    print(json.dumps({"step": i, "batch": s, "loss": l, "first_events": events[:12],
                      "nan_params": pn[:10]}), flush=True)
    if pn:
        break
