"""Run-to-run determinism bisect for the attpool heads: the same weights and
batch, forward + backward repeated R times (with other-shape steps between
them to vary memory reuse); reports the first module (in execution order)
whose forward output differs between repetitions, and which parameter
gradients differ."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hl-hgat_amd")]
import torch  # noqa: E402
import hlhgat  # noqa: E402
from hlhgat.synthetic import two_level_batch  # noqa: E402
from hlhgat import ops  # noqa: E402
F = torch.nn.functional
cuda = torch.device("cuda:0")
kind = sys.argv[1] if len(sys.argv) > 1 else "peptides"
if os.environ.get("NOFORK") == "1":
    ops.set_stream_fork(False)
bs = {s: [x.to(cuda) for x in two_level_batch(kind, 6, seed=s)] for s in (1, 2)}
torch.manual_seed(0)
m = hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool(
    channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0).to(cuda).train()
for mod in m.modules():  # BN running stats would change between repetitions
    if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
        mod.momentum = 0.0
rec = []


def flat(o):
    if isinstance(o, torch.Tensor):
        return [o.detach().clone()]
    if isinstance(o, (list, tuple)):
        return [t for x in o for t in flat(x)]
    return []


brec = []
for name, mod in m.named_modules():
    mod.register_forward_hook(lambda mo, i, o, n=name: rec.append((n, flat(o))))
    if name:
        mod.register_full_backward_hook(
            lambda mo, gi, go, n=name: brec.append((n, flat(go), flat(gi))))


def once(s):
    rec.clear()
    brec.clear()
    m.zero_grad(set_to_none=True)
    o = m(bs[s])
    F.binary_cross_entropy_with_logits(o, bs[s][0].y.view(o.shape).float()).backward()
    torch.cuda.synchronize()
    once.b = list(brec)
    return list(rec), {n: p.grad.detach().clone() for n, p in m.named_parameters()
                       if p.grad is not None}


runs, bruns = [], []
for r in range(int(os.environ.get("REPS", "6"))):
    runs.append(once(2))
    bruns.append(once.b)
    once(1)
bdiff = []
for br in bruns[1:]:
    for (n, go0, gi0), (n1, go1, gi1) in zip(bruns[0], br):
        dgo = any(not torch.equal(a, b) for a, b in zip(go0, go1))
        dgi = any(not torch.equal(a, b) for a, b in zip(gi0, gi1))
        if dgo or dgi:
            bdiff.append((n, "grad_out_differs" if dgo else "grad_out_same",
                          "grad_in_differs" if dgi else "grad_in_same"))
            break
f0, g0 = runs[0]
out = {"fwd_first_diff": None, "grad_diff": set(), "n_mods": len(f0)}
for fr, gr in runs[1:]:
    for (n, a), (n2, b) in zip(f0, fr):
        if any(not torch.equal(x, y) for x, y in zip(a, b)):
            if out["fwd_first_diff"] is None:
                out["fwd_first_diff"] = n
            break
    for n in g0:
        if n not in gr or not torch.equal(g0[n], gr[n]):
            out["grad_diff"].add(n)
out["bwd_order"] = [b[0] for b in bruns[0]]
out["bwd_first_diff"] = sorted(set(map(tuple, bdiff)))
out["grad_same"] = sorted(set(g0) - out["grad_diff"])
out["grad_diff"] = {n: float(max((g0[n] - gr[n]).abs().max() / (g0[n].abs().max() + 1e-30)
                                 for _, gr in runs[1:])) for n in sorted(out["grad_diff"])}
out["grad_diff"] = dict(sorted(out["grad_diff"].items(), key=lambda kv: kv[1])[:8])
print(json.dumps(out), flush=True)
