"""Lane replay probe: small ZINC models under TrainStep(graphs=True) over two
batch shapes (two captures); after every replay synchronise, read the device
error word and every lane counter, and time the replay.

    python tools/probes/lane_probe.py [plan ...]
plan items: L (a TrainStep with lane replay), T (torch's replay of the whole
graph); each item builds a fresh model + TrainStep and runs 2 captures + 6
replays; e.g. `T L` = a torch-replayed step first, then a lane-replayed one."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

WD = float(os.environ.get("WD", "0"))
ORDER = [int(c) for c in os.environ.get("ORDER", "010110")]


def run(tag, mode, bs, keep):
    lanes = mode == "L"
    import hlhgat
    from hlhgat import ops, train
    from hlhgat.train import TrainStep, batch_key
    train.LANES = lanes
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[1, 1], filters=[32, 32], mlp_channels=[64],
                                            K=3, keig=15).to("cuda:0").train()
    crit = torch.nn.L1Loss()
    st = TrainStep(m, lambda o, d: crit(o.view(-1, 1), d.y.view(-1, 1)), lr=1e-3,
                   weight_decay=WD, graphs=mode != "E")
    keep.append(st)
    for b in bs[:2]:
        st(b)
    torch.cuda.synchronize()
    print(f"[{tag}] stats {st.stats} lanes_off {st.lanes_off}", flush=True)
    for i, j in enumerate(ORDER):
        ops.clear_device_errors()
        t0 = time.perf_counter()
        st(bs[j])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        err = ops.device_errors()
        cnt = {}
        if lanes:
            cnt = {k: st._graphs[batch_key(b)].lanes.counters()[0] for k, b in enumerate(bs[:2])}
        print(f"[{tag}] replay {i} (shape {j}): {dt:.2f} ms, device errors {err}, "
              f"counters {[(min(c), max(c)) for c in cnt.values()]}", flush=True)
        for k, c in cnt.items():
            if min(c) != max(c):
                print("   shape", k, c, flush=True)


def main():
    from hlhgat.synthetic import zinc_like_batch
    print("env:", {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_HIP", "DEBUG_CLR"))})
    dev = torch.device("cuda:0")
    bs = [zinc_like_batch(40, seed=3).to(dev), zinc_like_batch(33, seed=4).to(dev),
          zinc_like_batch(40, seed=3).to(dev)]
    keep = []
    plan = sys.argv[1:] or ["L"]
    for k, p in enumerate(plan):
        run(f"{k}{p}", p, bs, keep)
        if os.environ.get("DROP", "1") == "1":
            keep.clear()
            import gc
            gc.collect()


if __name__ == "__main__":
    main()
