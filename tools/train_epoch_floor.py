"""Diagnostic: the device time of training epochs issued back to back with nothing between them (one
device row order reused, no side-stream copy, no event, no host draw) against train_model's own
epoch loop over the same epochs, both between two events; the difference is what the loop's per-epoch
plumbing costs the GPU. Usage: python tools/train_epoch_floor.py [epochs] [reps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import train_bench  # noqa: E402
from mbrl_amd import models  # noqa: E402
from mbrl_amd.optim import AdamStep  # noqa: E402


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    ds = train_bench.dataset()
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=512).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    np.random.seed(1)
    m.train_model(ds, opt, batch_size=512, num_epochs=10)
    torch.cuda.synchronize()
    n = ds.num_transitions()
    steps = epochs * ((n + 511) // 512)
    native = models._NATIVE_CACHE[m][1]
    fast = AdamStep.maybe(opt)
    order = torch.from_numpy(models._epoch_order(ds)).to(dev)

    def span(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / steps

    def bare():
        for _ in range(epochs):
            native.epoch(order, 512, fast)

    def loop():
        m.train_model(ds, opt, batch_size=512, num_epochs=epochs)

    out = {"bare_us_per_step": [], "train_model_us_per_step": []}
    for _ in range(reps):
        out["bare_us_per_step"].append(round(span(bare), 2))
        out["train_model_us_per_step"].append(round(span(loop), 2))
    out["epochs"], out["steps"] = epochs, steps
    print(json.dumps(out))


if __name__ == "__main__":
    main()
