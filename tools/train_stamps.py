"""Diagnostic: where one mbrl_train_grads launch sequence spends its time, from the -DMBRL_STAMPS
build's s_memrealtime stamps (first and last workgroup of each launch: entry, epilogue operands
issued, K loop done, exit). Usage: make -C mujoco-mbrl_amd diag && python tools/train_stamps.py [W]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so")
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import train_bench  # noqa: E402
from mbrl_amd import _lib, models  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    ds = train_bench.dataset()
    m = models.Model(17, 6, hidden_units=W).to("cuda:0")
    _, ins, outs = ds.stacked("cuda:0")
    nat = models._NativeGrads(m, ins, outs, ds.horizon, 512, False)
    lib = _lib.load()
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
    lib.mbrl_diag_set_train_stamps(ctypes.c_void_p(0))
    st = np.median(np.stack(reps), axis=0)
    n = int((st[:, 0] > 0).sum())
    t0 = st[0, 0]
    print("launch  first-WG: entry  epi-issued  kloop-done  exit | last-WG: entry  exit   (us from launch 0 entry)")
    for k in range(n):
        r = st[k] - t0
        print(f"{k:5d}   {r[0]:8.2f} {r[1]:10.2f} {r[2]:10.2f} {r[3]:8.2f} | {r[4]:8.2f} {r[7]:8.2f}")


if __name__ == "__main__":
    main()
