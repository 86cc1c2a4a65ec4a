"""A/B of MBRL_OPT_TRAIN_XCD (training launches' row-band tiles in XCD order, so each launch reads the
rows the previous one wrote on its own XCD): train_model 2 x W, batch 512, Adam, cheetah-shaped data,
steps/s over whole epochs, rounds interleaved; the trained parameters must be bit-identical.
Usage: python tools/train_xcd_ab.py [W] [epochs] [rounds]"""
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


def run(W, epochs, ds, xcd):
    with _lib.option("train_xcd", xcd):
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
    return steps / dt, torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ds = dataset()
    out = {"workload": f"train_model s=17 a=6 2x{W} batch 512, 10k transitions, Adam", "unit": "steps/s"}
    ref = None
    for _ in range(rounds):
        for xcd in (0, 1):
            sps, params = run(W, epochs, ds, xcd)
            if ref is None:
                ref = params
            assert torch.equal(params, ref), f"train_xcd={xcd}: parameters differ"
            out.setdefault(f"xcd{xcd}", []).append(round(sps, 1))
    out["bit_identical"] = True
    print(json.dumps(out))


if __name__ == "__main__":
    main()
