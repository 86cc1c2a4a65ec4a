"""Dump of the trained parameters and Adam state after a few train_model epochs at several shapes
(two-hidden-layer models: the fused step, its dW_0 fold), for comparing two builds of the library bit
for bit (MBRL_AMD_LIB selects the build). Usage: python tools/train_bits_dump.py out.pt"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_train_native import _dataset, _model  # noqa: E402

CASES = [("model", 17, 6, 512, 1, 512, 700), ("model", 24, 6, 512, 1, 512, 1500), ("reward", 17, 6, 200, 1, 256, 700),
         ("model", 17, 6, 512, 2, 200, 900), ("model", 5, 1, 256, 1, 96, 500), ("model", 30, 20, 300, 1, 512, 1100)]


def main():
    out = {}
    for n, (kind, s, a, W, H, B, T) in enumerate(CASES):
        ds = _dataset(s, a, H, T, seed=n + 1)
        m = _model(kind, s, a, W, 2, seed=n)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        np.random.seed(n)
        m.train_model(ds, opt, batch_size=B, num_epochs=3)
        torch.cuda.synchronize()
        out[n] = [p.detach().cpu() for p in m.parameters()] + \
                 [t.cpu() for st in opt.state.values() for t in (st["exp_avg"], st["exp_avg_sq"])] + \
                 [p.grad.detach().cpu() for p in m.parameters()]
    torch.save(out, sys.argv[1])
    print("saved", len(out), "cases")


if __name__ == "__main__":
    main()
