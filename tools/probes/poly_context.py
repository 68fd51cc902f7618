"""k_poly_step in context: the bench's replayed config-2 step, with the node /
edge chains on two streams (default) or on one stream (HLHGAT_ONE_STREAM=1).
Run under `rocprofv3 --kernel-trace` (durations per launch) or `--pmc`
(counters; those serialise the dispatches, so they show data locality, not
concurrency), then tools/step_kernels.py / tools/pmc_kernel.py.

    python tools/probes/poly_context.py [--steps 12]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    args = ap.parse_args()
    import bench
    import hlhgat
    from hlhgat import ops
    from hlhgat.train import TrainStep
    if os.environ.get("HLHGAT_ONE_STREAM") == "1":
        ops.set_stream_fork(False)
    dev = torch.device("cuda:0")
    batches, _, _, _, _ = bench.make_batches(2, 0, dev)
    crit = hlhgat.nn.L1Loss()
    torch.manual_seed(0)
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
    st = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                   weight_decay=1e-3, graphs=True)
    for i in range(4 + args.steps):
        st(batches[i % 2])
    torch.cuda.synchronize()
    ops.check_device_errors()
    print(st.stats)
    print("bn give-ups", ops.bn_giveups())


if __name__ == "__main__":
    main()
