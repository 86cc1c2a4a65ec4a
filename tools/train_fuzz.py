"""Fuzz of the training step's launch layouts: random shapes the fused step accepts (two hidden
layers, s + a <= 64, J <= 32, W <= 512, batch rows in (64, 512]), each trained for two epochs (short
last batch included) under the five-launch layout, the three-launch step (F and O apart) and the
two-launch step; gradients of one batch and the parameters, Adam state and losses after the epochs
must agree bit for bit, and the status word stay clear. Usage: python tools/train_fuzz.py [cases] [seed]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, models  # noqa: E402
from test_gpu_train_native import _dataset, _model  # noqa: E402

LAYOUTS = (("split5", 1, 0), ("fused3", 0, 1), ("fused2", 0, 0))


def run_case(rng):
    kind = "reward" if rng.random() < 0.35 else "model"
    s = int(rng.integers(1, 31 if kind == "reward" else 32))
    a = int(rng.integers(1, 64 - s + 1))
    W = int(rng.integers(8, 513))
    H = int(rng.integers(1, 3))
    lo, hi = [(64, 128), (128, 255), (256, 512)][int(rng.integers(0, 3))]
    B = int(rng.integers(lo // H + 1, hi // H + 1))
    T = int(rng.integers(2 * B, 4 * B))
    ds = _dataset(s, a, H, T, seed=int(rng.integers(1 << 30)))
    _, ins, outs = ds.stacked("cuda:0")
    reward = kind == "reward"
    idx = torch.randperm(ds.num_transitions(), generator=torch.Generator().manual_seed(B))[:B].to("cuda:0")
    got = {}
    for name, split, fo in LAYOUTS:
        with _lib.option("train_split", split), _lib.option("train_fo", fo):
            m = _model(kind, s, a, W, 2, seed=W)
            nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
            loss, parts = nat.run(idx)
            torch.cuda.synchronize()
            nat.check_status()
            grads = [loss.clone(), parts[0].clone(), parts[1].clone()] + [p.grad.clone() for p in m.parameters()]
            m = _model(kind, s, a, W, 2, seed=W)
            opt = torch.optim.Adam(m.parameters(), lr=1e-3)
            np.random.seed(3)
            m.train_model(ds, opt, batch_size=B, num_epochs=2)
            torch.cuda.synchronize()
            trained = [p.detach().clone() for p in m.parameters()] + \
                      [t.clone() for st in opt.state.values() for t in (st["exp_avg"], st["exp_avg_sq"])]
            got[name] = grads + trained
    ok = all(torch.equal(x, y) for name in ("fused3", "fused2") for x, y in zip(got[name], got["split5"]))
    return dict(kind=kind, s=s, a=a, W=W, H=H, B=B, R=B * H, T=ds.num_transitions(), ok=ok)


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 11
    rng = np.random.default_rng(seed)
    bad = []
    for i in range(cases):
        r = run_case(rng)
        if not r["ok"]:
            bad.append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps(dict(cases=cases, failed=len(bad))))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
