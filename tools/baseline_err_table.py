"""Per-parameter gradient error table of the HIP heads at the BASELINE
hyperparameters (tests/test_baseline_configs.py fixtures): HIP and the fp32
reference/oracle, each against the fp64 oracle (max-norm relative)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import test_baseline_configs as TB  # noqa: E402
from conftest import load_golden  # noqa: E402

torch.set_num_threads(16)
cuda = torch.device("cuda:0")
rows = {}
CASES = (("baseline_cfg3_cifar", False), ("baseline_cfg3_cifar", True),
         ("baseline_cfg4_pepfunc", False), ("baseline_cfg5_tsp", False),
         ("baseline_cfg5_tsp", True))
only = [a for a in sys.argv[1:] if not a.startswith("-")]
ALL = "--all" in sys.argv
for name, factored in CASES:
    if only and not any(o in name for o in only):
        continue
    import hlhgat
    from hlhgat import ops
    g = load_golden(name)
    _, cls_name, kw = TB.HEADS[name]
    m = getattr(hlhgat, cls_name)(**kw)
    TB.fill_params(m, int(g["seed"]))
    m = m.to(cuda).train()
    ops.clear_caches()
    if "tsp" in name:
        out, _ = m(TB._product_batch(g, "", cuda, factored))
    else:
        out = m([TB._product_batch(g, "l0/", cuda, factored),
                 TB._product_batch(g, "l1/", cuda, False)])
    (out * TB.T(g["R"]).to(cuda)).sum().backward()
    m32, o32, _ = TB._run_oracle(name, g, torch.float32)
    m64, o64, _ = TB._run_oracle(name, g, torch.float64)
    p32, p64 = dict(m32.named_parameters()), dict(m64.named_parameters())
    tab = []
    for k, p in m.named_parameters():
        if p.grad is None or p64[k].grad is None:
            continue
        e64 = p64[k].grad.double()
        sc = max(1.0, float(e64.abs().max()))
        tab.append((k, float((p.grad.cpu().double() - e64).abs().max()) / sc,
                    float((p32[k].grad.double() - e64).abs().max()) / sc, bool(TB._bn_fed_bias(k))))
    oerr = float((out.detach().cpu().double() - o64).abs().max()) / max(1, float(o64.abs().max()))
    o32err = float((o32.double() - o64).abs().max()) / max(1, float(o64.abs().max()))
    key = f"{name}{'_factored' if factored else ''}"
    ratios = [h / max(r, 1e-7) for _, h, r, bn in tab if not bn]
    rows[key] = {"out_err_hip": oerr, "out_err_fp32": o32err,
                 "max_err_hip": max(h for _, h, _, bn in tab if not bn),
                 "max_err_fp32": max(r for _, _, r, bn in tab if not bn),
                 "median_ratio": float(np.median(ratios)), "p90_ratio": float(np.percentile(ratios, 90)),
                 "worst": sorted(tab, key=lambda t: -t[1])[:6]}
    print(key, json.dumps({k: v for k, v in rows[key].items() if k != "worst"}), flush=True)
    for w in (sorted(tab, key=lambda t: -t[1] / max(t[2], 1e-7)) if ALL else rows[key]["worst"]):
        print("   ", w, flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(os.path.join(REPO, "gpurun_out", "baseline_err_table.json"), "w") as f:
    json.dump(rows, f, indent=1)
