"""Diagnostic: where one training step's launches spend their time, from the -DMBRL_STAMPS build's
s_memrealtime stamps (8 slots per launch: 4 from the first workgroup and 4 from a probe workgroup --
the first tile of a launch's second product, else the last workgroup). Two runs: mbrl_train_grads
(gradient only) and the last step of an mbrl_train_epoch over whole batches (Adam in the launches).
Usage: make -C mujoco-mbrl_amd diag && python tools/train_stamps.py [W] [split]

Stamp points: gemm launches (train_gemm_kernel): entry, K loop done, after the partial-sum barrier
(and a dW tile's arrival wait), exit.
Fused F: entry, input gathered, H_0 rows in LDS, exit. Fused O: entry, dY in LDS, dH_1 / dW_out
partials stored, ticket taken (last arriver's sum after)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("MBRL_AMD_LIB", os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import train_bench  # noqa: E402
from mbrl_amd import _lib, models, optim  # noqa: E402


def show(title, reps):
    st = np.median(np.stack(reps), axis=0)
    n = int((st[:, 0] > 0).sum())
    t0 = st[0, 0]
    print(title)
    print("launch  first-WG: s0      s1      s2      s3  | probe-WG: s0      s1      s2      s3   (us from launch 0 entry)")
    for k in range(n):
        r = st[k] - t0
        print(f"{k:5d}   {r[0]:8.2f} {r[1]:7.2f} {r[2]:7.2f} {r[3]:7.2f} | {r[4]:8.2f} {r[5]:7.2f} {r[6]:7.2f} {r[7]:7.2f}")


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    split = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    lib = _lib.load()
    lib.mbrl_set_option(_lib.OPTIONS["train_split"], split)
    ds = train_bench.dataset()
    m = models.Model(17, 6, hidden_units=W).to("cuda:0")
    _, ins, outs = ds.stacked("cuda:0")
    nat = models._NativeGrads(m, ins, outs, ds.horizon, 512, False)
    lib.mbrl_diag_set_train_stamps.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(8 * 16, dtype=torch.int64, device="cuda:0")
    idx = torch.randperm(ds.num_transitions())[:512].to("cuda:0")
    for _ in range(20):
        nat.run(idx)
    torch.cuda.synchronize()
    lib.mbrl_diag_set_train_stamps(ctypes.c_void_p(buf.data_ptr()))
    reps = []
    for _ in range(10):
        buf.zero_()
        nat.run(idx)
        torch.cuda.synchronize()
        reps.append(buf.cpu().numpy().reshape(16, 8).astype(np.float64) * 10.0 / 1000.0)   # us
    show(f"mbrl_train_grads 2x{W} batch 512 (split={split})", reps)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    fast = optim.AdamStep.maybe(opt)
    order = torch.randperm(ds.num_transitions())[:512 * 4].to("cuda:0")
    reps = []
    for i in range(12):
        buf.zero_()
        nat.epoch(order, 512, fast)
        torch.cuda.synchronize()
        if i >= 2:
            reps.append(buf.cpu().numpy().reshape(16, 8).astype(np.float64) * 10.0 / 1000.0)
    lib.mbrl_diag_set_train_stamps(ctypes.c_void_p(0))
    show(f"mbrl_train_epoch 2x{W} batch 512, last of 4 steps (split={split})", reps)


if __name__ == "__main__":
    main()
