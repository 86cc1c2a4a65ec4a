"""Diagnostic: tests/test_gpu_train_native.py::test_epoch_call_equals_per_batch_calls under each
training launch layout (default, MBRL_OPT_TRAIN_FO = 1, MBRL_OPT_TRAIN_SPLIT = 1): which parameters
differ between the epoch call and per-batch calls, and by how much. Usage: python tools/epoch_eq_probe.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, models  # noqa: E402
from test_gpu_train_native import _dataset, _model  # noqa: E402


def train(kind, epoch_call, epochs, bs):
    ds = _dataset(17, 6, 2, 700, seed=9)
    m = _model(kind, 17, 6, 96, 2, seed=1)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4)
    saved = models._NativeGrads.epoch
    if not epoch_call:
        models._NativeGrads.epoch = lambda self, *a: None
    try:
        np.random.seed(2)
        m.train_model(ds, opt, batch_size=bs, num_epochs=epochs)
    finally:
        models._NativeGrads.epoch = saved
    torch.cuda.synchronize()
    return [p.detach().cpu() for p in m.parameters()]


def main():
    out = []
    for layout, opts in (("default", {}), ("fo_split", {"train_fo": 1}), ("split5", {"train_split": 1})):
        for epochs, bs in ((1, 128), (3, 128), (1, 512), (1, 64)):
            saved = {k: _lib.load().mbrl_set_option(_lib.OPTIONS[k], v) for k, v in opts.items()}
            try:
                a = train("model", True, epochs, bs)
                b = train("model", False, epochs, bs)
            finally:
                for k, v in saved.items():
                    _lib.load().mbrl_set_option(_lib.OPTIONS[k], v)
            diff = [float((x - y).abs().max()) for x, y in zip(a, b)]
            out.append(dict(layout=layout, epochs=epochs, batch=bs, max_abs_diff=diff))
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
