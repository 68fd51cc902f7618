"""Which part of a SyncBatchNorm step breaks hipStreamEndCapture under RCCL?
(tests/test_rccl_capture.py::...[zinc_sync_bn] segfaulted in capture_end,
round 5.)  Each variant runs the test's child in its own process (a
one-rank nccl group, collectives executed) with one thing changed:

  base        as the test
  nofork      ops.set_stream_fork(False): every chain on the capture stream
  nochains    ops.CHAINS_ENABLED = False: a fork / join per HL block
  fwdonly     the backward's statistics all-reduce skipped (one rank: the
              same sums), so only the forward's collectives are captured
  bwdonly     the forward's skipped instead
  chains      the persistent chains forced on (ops.SYNCBN_CHAINS), all-reduce
              on the layer's stream (the round-5 crash)
  (round 6 also tried every statistics all-reduce issued from one dedicated
   collective stream, event-ordered with the layer's stream: the chains
   capture crashed the same way, profiles/r06/syncbn_capture_probe.log)

    python tools/probes/syncbn_capture_probe.py [variant ...]
"""
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def child(variant):
    sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "hl-hgat_amd")]
    from hlhgat import ops
    if variant.startswith("chains"):
        ops.SYNCBN_CHAINS = True
    if variant == "nofork":
        ops.set_stream_fork(False)
    elif variant == "nochains":
        ops.CHAINS_ENABLED = False
    elif variant in ("fwdonly", "bwdonly"):
        orig = ops._sum_over_ranks
        state = {"fwd": True}
        fwd_fn = ops._SyncBatchNormFn.forward
        bwd_fn = ops._SyncBatchNormFn.backward

        def fwd(ctx, *a, **k):
            state["fwd"] = True
            return fwd_fn(ctx, *a, **k)

        def bwd(ctx, *a, **k):
            state["fwd"] = False
            return bwd_fn(ctx, *a, **k)

        def sor(t, group):
            skip = (variant == "fwdonly") != state["fwd"]
            return t.view(1, -1) if skip else orig(t, group)
        ops._SyncBatchNormFn.forward = staticmethod(fwd)
        ops._SyncBatchNormFn.backward = staticmethod(bwd)
        ops._sum_over_ranks = sor
    import test_rccl_capture as T
    T._child("zinc_sync_bn")


def main():
    variants = sys.argv[1:] or ["base", "nofork", "nochains"]
    for v in variants:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0",
                   WORLD_SIZE="1", LOCAL_RANK="0")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", v], env=env,
                               cwd=REPO, capture_output=True, text=True, timeout=180)
            rc, out, err = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired:
            rc, out, err = "timeout", "", ""
        last = [ln for ln in out.splitlines() if ln.startswith("{")]
        tail = [ln for ln in err.splitlines() if "Fatal" in ln or "Error" in ln or "line" in ln]
        print(f"=== {v}: rc={rc} {last[-1][:300] if last else ''}", flush=True)
        for ln in tail[-6:]:
            print("   ", ln[:200], flush=True)
        if rc not in (0, 1):
            break  # a crash / time-out: nothing more on the GPU in this call


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
