"""Host-side cost of one cfg2 training step: wall vs enqueue time, and the
torch.profiler CPU op table (where the Python/launch overhead goes)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    import hlhgat
    from hlhgat import ops
    dev = torch.device("cuda:0")
    batches = bench.make_batches(2, 0, dev)
    torch.manual_seed(0)
    model = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-3, fused=True)
    crit = torch.nn.L1Loss()

    def step(i):
        b = batches[i % 2]
        ops.clear_caches()
        out = model(b)
        loss = crit(out.view(-1, 1), b.y.view(-1, 1))
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    print(f"per step: enqueue {t_enq / n * 1e3:.2f} ms, wall {t_wall / n * 1e3:.2f} ms")
    # forward-only / backward-only host costs
    b = batches[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        ops.clear_caches()
        out = model(b)
    t_f = (time.perf_counter() - t0) / n
    loss = crit(out.view(-1, 1), b.y.view(-1, 1))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss.backward()
    t_b = time.perf_counter() - t0
    torch.cuda.synchronize()
    print(f"host enqueue: forward {t_f * 1e3:.2f} ms, backward {t_b * 1e3:.2f} ms")
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for i in range(3):
            step(i)
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))


if __name__ == "__main__":
    main()
