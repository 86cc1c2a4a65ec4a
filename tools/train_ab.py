"""A/B of the training step's launch structure: train_model (2 x W, batch 512, Adam,
cheetah-shaped data) on one GPU with the r02 layout (32 x 32 backward tiles, the layer-0 weight
gradient in its own launch) and the r03 layout (64 x 32 tiles for the W x W products, the layer-0
gradient folded into the dH_0 launch), interleaved; GPU-time steps/s. Usage: python tools/train_ab.py [W] [epochs]"""
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


def run(W, epochs, ds, tile, no_fold):
    with _lib.option("train_tile", tile), _lib.option("train_no_fold", no_fold):
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
    return steps / dt


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ds = dataset()
    out = {"workload": f"train_model s=17 a=6 2x{W} batch 512, 10k transitions, Adam"}
    combos = {"tile32_nofold (r02)": (32, 1), "tile_auto_nofold": (0, 1), "tile32_fold": (32, 0),
              "tile_auto_fold (r03 default)": (0, 0)}
    for _ in range(3):
        for k, (tile, nf) in combos.items():
            out.setdefault(k, []).append(round(run(W, epochs, ds, tile, nf), 1))
    out["unit"] = "steps/s"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
