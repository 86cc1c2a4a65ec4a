"""The fused per-iteration update (cem_update_kernel through mbrl_cem_update) at the sizes the plans run
it: mean device time per call from HIP events over 200 calls, and with the -DMBRL_STAMPS library
(--stamps) thread 0's phase times of one workgroup: selection (load, wide pass, list, passes,
compaction), refit (the elites' actions regenerated from the counter RNG, chunked sums), draw.
Usage: python tools/update_bench.py [--stamps] [N K H a draw_count] ..."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAMPS = "--stamps" in sys.argv
if STAMPS:
    os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so")
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, fused  # noqa: E402

CASES = [(16384, 1638, 30, 6, 2048), (16384, 1638, 30, 6, 16384), (4096, 409, 30, 6, 4096), (32768, 3276, 30, 6, 4096),
         (1024, 102, 20, 1, 1024)]


def main():
    args = [int(x) for x in sys.argv[1:] if not x.startswith("--")]
    cases = [tuple(args[i:i + 5]) for i in range(0, len(args), 5)] if args else CASES
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    buf = torch.zeros(16, dtype=torch.int64, device=dev)
    if STAMPS:
        lib.mbrl_diag_set_cem_stamps.argtypes = [ctypes.c_void_p]
        assert lib.mbrl_diag_set_cem_stamps(buf.data_ptr()) == 0
    out = []
    for N, K, H, a, D in cases:
        rng = np.random.default_rng(N)
        costs = torch.from_numpy(rng.uniform(130, 250, (1, N)).astype(np.float32)).to(dev)
        mu = torch.zeros((H, a), device=dev)
        sg = torch.full((H, a), 0.5, device=dev)
        mu_o, sg_o = torch.empty_like(mu), torch.empty_like(sg)
        nxt = torch.empty((H, D, a), device=dev)
        sp = fused.make_sampler(7, 1, mu, sg, -1.0, 1.0)
        for _ in range(10):
            fused.cem_update(costs, K, sp, H, a, 0.1, mu_o, sg_o, next_actions=nxt)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            fused.cem_update(costs, K, sp, H, a, 0.1, mu_o, sg_o, next_actions=nxt)
        e1.record()
        torch.cuda.synchronize()
        row = dict(N=N, K=K, H=H, a=a, draw=D, us_per_call=e0.elapsed_time(e1) * 1e3 / 200)
        if STAMPS:
            rows = []
            for _ in range(20):
                fused.cem_update(costs, K, sp, H, a, 0.1, mu_o, sg_o, next_actions=nxt)
                torch.cuda.synchronize()
                rows.append(buf.cpu().numpy().copy())
            st = np.array(rows[5:], dtype=np.float64)
            d = np.diff(st, axis=1).mean(0) / 100.0
            row["phases_us"] = dict(zip(["load+minmax", "wide", "list", "passes", "compaction", "select->refit",
                                         "refit"], [round(float(x), 2) for x in d]))
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
