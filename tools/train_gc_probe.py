"""Diagnostic: the first long train_model call of a process runs slower per step than later ones. This
times 50-epoch calls in a fresh process with the garbage collector's pauses recorded (gc.callbacks),
then the same calls with the collector disabled, to tell host pauses from device effects.
Usage: python tools/train_gc_probe.py [calls]"""
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import train_bench  # noqa: E402
from mbrl_amd import models  # noqa: E402

pauses = []
_t = {}


def _cb(phase, info):
    if phase == "start":
        _t["t"] = time.perf_counter()
    else:
        pauses.append((info["generation"], (time.perf_counter() - _t["t"]) * 1e3))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    ds = train_bench.dataset()
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=512).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    np.random.seed(1)
    m.train_model(ds, opt, batch_size=512, num_epochs=10)
    torch.cuda.synchronize()
    gc.collect()
    gc.callbacks.append(_cb)
    steps = 50 * ((ds.num_transitions() + 511) // 512)

    def span():
        del pauses[:]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        m.train_model(ds, opt, batch_size=512, num_epochs=50)
        e1.record()
        torch.cuda.synchronize()
        return dict(us_per_step=round(e0.elapsed_time(e1) * 1e3 / steps, 2),
                    gc=[(g, round(ms, 2)) for g, ms in pauses])

    out = {"gc_on": [span() for _ in range(calls)]}
    gc.disable()
    out["gc_off"] = [span() for _ in range(calls)]
    gc.enable()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
