"""Where a training step's wall time goes on the GPU path: train_model's loop with
_GraphStep.run and AdamStep.step wrapped in perf_counter timers (host time of each call; the GPU
runs asynchronously behind them). Usage: python tools/train_turn.py [W]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import train_bench  # noqa: E402
from mbrl_amd import models, optim  # noqa: E402

ACC = {}


def timed(cls, name):
    fn = getattr(cls, name)

    def wrap(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[cls.__name__ + "." + name] = ACC.get(cls.__name__ + "." + name, 0.0) + time.perf_counter() - t
    setattr(cls, name, wrap)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    ds = train_bench.dataset()
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=W).to("cuda:0")
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    np.random.seed(1)
    m.train_model(ds, opt, batch_size=512, num_epochs=1)
    torch.cuda.synchronize()
    timed(models._GraphStep, "run")
    timed(models._NativeGrads, "run")
    timed(optim.AdamStep, "step")
    epochs = 10
    t0 = time.perf_counter()
    m.train_model(ds, opt, batch_size=512, num_epochs=epochs)
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = epochs * ((ds.num_transitions() + 511) // 512)
    print(json.dumps(dict(W=W, steps=steps, wall_us_per_step=wall / steps * 1e6, host_us_per_step=host / steps * 1e6,
                          **{k + "_us": v / steps * 1e6 for k, v in ACC.items()})))


if __name__ == "__main__":
    main()
