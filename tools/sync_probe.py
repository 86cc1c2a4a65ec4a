"""How long the host waits, after the GPU's last write, to learn that a plan finished: round trips of
one tiny launch + (a) hipStreamSynchronize, (b) hipEventSynchronize, (c) a spin on a word of mapped
pinned host memory the launch writes (hipMemsetD32Async on its device alias). Usage:
python tools/sync_probe.py [iterations]"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    torch.cuda.init()
    x = torch.zeros(1, device="cuda:0")
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln)
    hip = ctypes.CDLL(path)
    hip.hipMemsetD32Async.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    stream = torch.cuda.current_stream()
    sh = ctypes.c_void_p(stream.cuda_stream)
    out = {}

    def bench(name, body):
        for _ in range(50):
            body(0)
        t0 = time.perf_counter()
        for i in range(n):
            body(i + 1)
        out[name + "_us"] = (time.perf_counter() - t0) / n * 1e6

    bench("launch+stream_sync", lambda i: (x.add_(1), stream.synchronize()))
    ev = ctypes.c_void_p()
    hip.hipEventCreateWithFlags(ctypes.byref(ev), 0x2 | 0x20000000)   # DisableTiming | DisableSystemFence
    bench("launch+event_sync", lambda i: (x.add_(1), hip.hipEventRecord(ev, sh), hip.hipEventSynchronize(ev)))
    stage = _lib.HostStaging(64)
    word = stage.array.view(np.int32)

    def spin(i):
        x.add_(1)
        hip.hipMemsetD32Async(stage.device, i + 7, 1, sh)
        while word[0] != i + 7:
            pass
    bench("launch+memset_to_mapped+spin", spin)

    def memset_sync(i):
        x.add_(1)
        hip.hipMemsetD32Async(stage.device, i + 7, 1, sh)
        stream.synchronize()
    bench("launch+memset_to_mapped+stream_sync", memset_sync)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
