"""Which of mbrl_adam_step's contraction patterns (csrc/mbrl_internal.h AdamArith bits) reproduces
torch.optim.Adam on this GPU, per hyper-parameter set. Usage: python tools/adam_arith.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import test_gpu_train_adam as t  # noqa: E402
from mbrl_amd import _lib  # noqa: E402

for kw in t.CONFIGS:
    ref_opt, ref_p = t._run(kw, 6, fused=False)
    ref = t._state(ref_opt, ref_p)
    res = {}
    for bits in range(16):
        with _lib.option("adam_arith", bits + 1):
            o, p = t._run(kw, 6, fused=True)
        got = t._state(o, p)
        res[bits] = [sum(int((a != b).sum()) for a, b in zip(x[:3], y[:3])) for x, y in zip(ref, got)]
    print(kw, "matching:", [b for b, v in res.items() if sum(v) == 0])
    print("   mismatches per pattern:", {b: sum(v) for b, v in res.items()})
