"""A/B of the training step's launch structure: train_model (2 x W, batch 512, Adam,
cheetah-shaped data, 10k transitions) in the r05 two-launch step (F and O in one launch) against the
r04 three-launch step (MBRL_OPT_TRAIN_FO = 1) and the r03 five-launch layout (MBRL_OPT_TRAIN_SPLIT = 1),
interleaved on one GPU, with the trained parameters required equal bit for bit; wall-clock steps/s of whole epochs (the
step is GPU-bound: one host call per epoch). Usage: python tools/train_split_ab.py [W ...] [--epochs E]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, models  # noqa: E402
from train_bench import dataset  # noqa: E402


def run(W, epochs, ds, split, fo_split):
    with _lib.option("train_split", split), _lib.option("train_fo", fo_split):
        torch.manual_seed(0)
        m = models.Model(17, 6, hidden_units=W).to("cuda:0")
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        np.random.seed(1)
        m.train_model(ds, opt, batch_size=512, num_epochs=1)
        torch.cuda.synchronize()
        np.random.seed(2)
        t0 = time.perf_counter()
        m.train_model(ds, opt, batch_size=512, num_epochs=epochs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    steps = epochs * ((len(ds.transition_index()) + 511) // 512)
    return steps / dt, torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    epochs = 20
    if "--epochs" in sys.argv:
        epochs = int(sys.argv[sys.argv.index("--epochs") + 1])
        args = [a for a in args if a != str(epochs)]
    widths = [int(a) for a in args] or [512]
    ds = dataset()
    for W in widths:
        out = {"workload": f"train_model s=17 a=6 2x{W} batch 512, 10k transitions, Adam", "unit": "steps/s"}
        for _ in range(3):
            ref = None
            for name, split, fo in (("split5 (r03)", 1, 0), ("fused3 (r04)", 0, 1), ("fused2 (r05)", 0, 0)):
                rate, params = run(W, epochs, ds, split, fo)
                ref = params if ref is None else ref
                assert torch.equal(params, ref), f"{name}: parameters differ from the five-launch layout's"
                out.setdefault(name, []).append(round(rate, 1))
        out["us_per_step"] = {k: round(1e6 / float(np.median(v)), 2) for k, v in out.items() if isinstance(v, list)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
