"""Host wake-up latency after a long GPU wait: per iteration one ~N ms device-side sleep
(torch.cuda._sleep) then (a) stream.synchronize() (HIP's blocking wait) or (b) a spin on
stream.query(); reports wall minus the sleep's own event-timed duration. Usage:
python tools/wake_probe.py [ms] [iterations]"""
import json
import sys
import time

import numpy as np
import torch


def main():
    ms = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    torch.cuda.init()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); torch.cuda._sleep(1000000); b.record(); s.synchronize()
    cyc = int(1000000 * ms / a.elapsed_time(b))
    out = {"sleep_ms": ms}
    for mode in ("sync", "spin", "sync", "spin"):
        gaps = []
        for _ in range(n):
            a.record()
            torch.cuda._sleep(cyc)
            b.record()
            t0 = time.perf_counter()
            if mode == "sync":
                s.synchronize()
            else:
                while not s.query():
                    pass
            wall = time.perf_counter() - t0
            gaps.append(wall * 1e3 - a.elapsed_time(b))
        g = np.array(gaps) * 1e3
        out[mode] = out.get(mode, []) + [dict(mean_us=float(g.mean()), p50_us=float(np.median(g)),
                                              p90_us=float(np.percentile(g, 90)), max_us=float(g.max()))]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
