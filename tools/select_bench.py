"""Elite selection timing (select_reg_kernel through mbrl_select_elites): mean device time per call
from HIP events over 200 calls, per N and ensemble size, on plan-like returns (one binade).
Usage: python tools/select_bench.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import fused  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    out = []
    for E in (1, 5):
        for N in (1024, 4096, 16384, 32768):
            costs = torch.from_numpy(np.random.default_rng(N + E).uniform(130, 250, (E, N)).astype(np.float32)).to(dev)
            ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
            for _ in range(10):
                fused.select(costs, N // 10, workspace=ws)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(200):
                fused.select(costs, N // 10, workspace=ws)
            b.record()
            torch.cuda.synchronize()
            out.append(dict(E=E, N=N, us_per_call=a.elapsed_time(b) * 1e3 / 200))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
