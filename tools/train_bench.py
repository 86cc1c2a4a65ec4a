"""Model-training throughput: train_model on synthetic rollouts, CPU (the
reference's arithmetic, torch threads = this process's CPU share) vs the MI355X.

    python tools/train_bench.py [W] [epochs]      -> one JSON line

Workload: cheetah-shaped data (s = 17, a = 6), 20 rollouts x 500 steps = 10k transitions, Model with
2 hidden layers of W units, Adam(1e-3), batch 512 (models.py:53-59 defaults), state_only mode."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import data, models  # noqa: E402


def dataset():
    rng = np.random.Generator(np.random.PCG64(5))
    rolls = []
    for _ in range(20):
        K = 500
        st = rng.standard_normal((K + 1, 17)).astype(np.float32)
        rolls.append(data.Rollout(states=list(torch.from_numpy(st)), observations=list(torch.from_numpy(st)),
                                  actions=list(torch.from_numpy(rng.uniform(-1, 1, (K, 6)).astype(np.float32))),
                                  rewards=list(torch.from_numpy(rng.standard_normal(K).astype(np.float32)))))
    ds = data.TransitionsDataset(rollouts=rolls)
    ds.set_data_mode("state_only")
    return ds


def run(device, W, epochs, ds):
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=W).to(device)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    np.random.seed(1)
    m.train_model(ds, opt, batch_size=512, num_epochs=1)      # warm-up (also stacks the data on device)
    if device != "cpu":
        torch.cuda.synchronize()
    np.random.seed(2)
    t0 = time.perf_counter()
    m.train_model(ds, opt, batch_size=512, num_epochs=epochs)
    if device != "cpu":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = epochs * ((len(ds.transition_index()) + 511) // 512)
    return dict(seconds=dt, steps=steps, steps_per_s=steps / dt, samples_per_s=steps * 512 / dt)


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    cores = len(os.sched_getaffinity(0))
    torch.set_num_threads(min(cores, 16))
    ds = dataset()
    out = dict(workload=f"train_model s=17 a=6 2x{W} batch 512, 10k transitions", epochs=epochs,
               cpu=run("cpu", W, max(1, epochs // 5), ds), cpu_threads=torch.get_num_threads())
    if torch.cuda.is_available():
        out["gpu"] = run("cuda:0", W, epochs, ds)
        out["speedup"] = out["gpu"]["steps_per_s"] / out["cpu"]["steps_per_s"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
