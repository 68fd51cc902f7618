"""Host time of enqueueing one 10.75 MB H2D copy (the loader-fed loop's
per-batch upload) on a side stream, while the device is busy with other
work, by path: torch copy_(non_blocking) from a pinned torch tensor, the
same through hipMemcpyAsync directly, and from hipHostMalloc'd memory.
Prints host enqueue time and device time per copy (diagnostics for
DESIGN.md §18's loader analysis)."""
import ctypes
import time

import torch

NB = 10_901_884
REPS = 20


def main():
    dev = torch.device("cuda:0")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    cs = torch.cuda.Stream(device=dev)
    dst = torch.empty(NB, dtype=torch.uint8, device=dev)
    src_t = torch.empty(NB, dtype=torch.uint8, pin_memory=True)
    src_t.fill_(1)
    print("torch pinned:", src_t.is_pinned())
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), NB, 0) == 0
    ctypes.memset(p, 1, NB)
    big = torch.randn(4096, 4096, device=dev)

    def busy():
        for _ in range(8):
            big.mul_(1.0000001)  # keeps the device busy on the main stream

    def run(name, fn):
        host = 0.0
        busy()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(REPS):
            busy()
            if i == 0:
                e0.record(cs)
            t0 = time.perf_counter()
            fn()
            host += time.perf_counter() - t0
        e1.record(cs)
        torch.cuda.synchronize()
        print(f"{name:34s} host {host / REPS * 1e3:7.3f} ms/copy   device span {e0.elapsed_time(e1) / REPS:7.3f} ms/copy")

    def torch_copy():
        with torch.cuda.stream(cs):
            dst.copy_(src_t, non_blocking=True)

    def raw_torch_ptr():
        assert hip.hipMemcpyAsync(dst.data_ptr(), src_t.data_ptr(), NB, 1, cs.cuda_stream) == 0

    def raw_hostmalloc():
        assert hip.hipMemcpyAsync(dst.data_ptr(), p, NB, 1, cs.cuda_stream) == 0

    main = torch.cuda.current_stream(dev)
    gate = torch.cuda.Event()

    def dep_copy():  # the copy waits for the work queued so far on main
        gate.record(main)
        cs.wait_event(gate)
        assert hip.hipMemcpyAsync(dst.data_ptr(), src_t.data_ptr(), NB, 1, cs.cuda_stream) == 0

    def dep_done_copy():  # ... on an event that has completed
        cs.wait_event(done_ev)
        assert hip.hipMemcpyAsync(dst.data_ptr(), src_t.data_ptr(), NB, 1, cs.cuda_stream) == 0

    done_ev = torch.cuda.Event()
    done_ev.record(main)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    busy()
    torch.cuda.synchronize()
    print(f"busy() device time {(time.perf_counter() - t0) * 1e3:.3f} ms")
    for _ in range(2):
        run("copy after wait on main's queued work", dep_copy)
        run("copy after wait on a completed event", dep_done_copy)
        run("torch copy_ (pinned tensor)", torch_copy)
        run("hipMemcpyAsync (torch pinned ptr)", raw_torch_ptr)
        run("hipMemcpyAsync (hipHostMalloc ptr)", raw_hostmalloc)
    assert hip.hipHostFree(p) == 0


if __name__ == "__main__":
    main()
