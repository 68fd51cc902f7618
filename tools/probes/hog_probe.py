"""Does a kernel of another process / stream run while a hog kernel holds
most CUs?  (tests/test_gpu_parity.py::test_bn_one_launch_beside_cu_hog)

    python tools/probes/hog_probe.py
Prints the host time of small launches issued while the hog runs.
"""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "hl-hgat_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

HOG = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from hlhgat import _lib
cus = torch.cuda.get_device_properties(0).multi_processor_count
s = torch.cuda.Stream()
_lib.check(_lib.LIB.hlhgat_test_occupy(int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]),
                                       int(sys.argv[2]), s.cuda_stream), "test_occupy")
print("hog launched", flush=True)
s.synchronize()
print("hog done", flush=True)
"""


def timed(fn):
    # this stream only: a device-wide synchronize would also wait for the
    # same-process hog on its own stream
    cs = torch.cuda.current_stream()
    cs.synchronize()
    t0 = time.perf_counter()
    fn()
    cs.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    from hlhgat import _lib, ops
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    x = torch.randn(25600, 64, device=dev)
    bn = torch.nn.BatchNorm1d(64).to(dev).train()
    tiny = torch.zeros(16, device=dev)
    work = {"tiny add": lambda: tiny.add_(1.0),
            "bn one launch": lambda: ops.batch_norm_act(x, bn, relu=True)}
    for k, f in work.items():
        timed(f)
        print(f"idle: {k} {timed(f):.2f} ms", flush=True)
    pkg = os.path.join(REPO, "hl-hgat_amd")
    usec = 300000
    for wgs, hold, lds in ((cus, cus - 16, 140 * 1024), (cus, cus - 64, 140 * 1024),
                           (cus // 2, cus // 2, 140 * 1024), (cus, cus - 16, 0)):
        for where in ("process", "stream"):
            ops.bn_giveups_reset()
            if where == "process":
                p = subprocess.Popen([sys.executable, "-c", HOG, pkg, str(usec), str(wgs),
                                      str(hold), str(lds)], stdout=subprocess.PIPE, text=True)
                assert p.stdout.readline().strip() == "hog launched"
            else:
                s = torch.cuda.Stream(priority=0)
                _lib.check(_lib.LIB.hlhgat_test_occupy(wgs, hold, lds, usec, s.cuda_stream), "occ")
            time.sleep(0.05)
            t = {k: timed(f) for k, f in work.items()}
            gu = ops.bn_giveups()["count"]
            if where == "process":
                p.communicate(timeout=60)
            torch.cuda.synchronize()
            print(f"hog wgs={wgs} hold={hold} lds={lds} in another {where}: "
                  + ", ".join(f"{k} {v:.1f} ms" for k, v in t.items()) + f", give-ups {gu}",
                  flush=True)


if __name__ == "__main__":
    main()
