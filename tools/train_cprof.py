import cProfile, pstats, sys, os, time
sys.path[:0] = ['.', 'mujoco-mbrl_amd', 'tools']
import numpy as np, torch
import train_bench
from mbrl_amd import models
ds = train_bench.dataset()
torch.manual_seed(0)
m = models.Model(17, 6, hidden_units=512).to("cuda:0")
opt = torch.optim.Adam(m.parameters(), lr=1e-3)
np.random.seed(1)
m.train_model(ds, opt, batch_size=512, num_epochs=1)
torch.cuda.synchronize()
for rep in range(2):
    np.random.seed(2)
    pr = cProfile.Profile(); pr.enable()
    t0 = time.perf_counter()
    m.train_model(ds, opt, batch_size=512, num_epochs=10)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pr.disable()
    print("rep", rep, "wall ms", dt * 1e3)
    pstats.Stats(pr).sort_stats("cumtime").print_stats(22)
