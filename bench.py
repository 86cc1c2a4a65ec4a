"""Benchmark: CEM planning throughput (candidate-timesteps/s) on the BASELINE.json workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` without a launcher (no WORLD_SIZE in the environment) starts the N rank processes itself
(one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1) before this process touches
the GPU, waits for them and exits with their status; rank 0 prints the line.

A "step" is one CEMPlanner.plan() call (I iterations of proposal draw -> rollout ->
elite top-K -> refit, plus the final mean's rollout) on the cheetah-run config (BASELINE.json
configs[2]: N=4096, H=30, 17/6, 3x512 MLP, I=5, K=N/10) with synthetic random weights.
value = I * N_total * H * K_steps / (max over ranks of the timed wall clock).
With N GPUs each rank owns 4096 candidates (weak scaling: N_total = 4096 * N); one RCCL
all-gather of returns per CEM iteration. `--strong` splits the config's N over the GPUs instead
(e.g. `--config 4 --strong`: walker N=16384 over 8 GPUs, BASELINE.json configs[3]);
`--candidates` overrides N (per GPU, or in total with --strong).

Extra objects on the JSON line:
  roofline     -- the rollout kernel (dominant): algorithmic MLP FLOP per launch / average launch
                  time from fence-free HIP events recorded on the launch stream around the rollout
                  launch of CEM iteration MEASURED_IT in every timed plan (each record idles the GPU
                  ~4 us, so not all five); peak = fp32 MFMA dense 157.3 TFLOP/s (MI355X_MICROARCH.md).
  cpu_baseline -- the CPU oracle (NumPy restatement of the reference rollout + CEM refit), rank 0,
                  N=1 only, on a bounded sample; a reported baseline, not the target.
  cpu_baseline_torch -- the reference's own CPU arrangement beside it: torch on the host with
                  autograd on (planners.py:199-210), NumPy refit; same conditions.
  parity       -- iteration-0 returns of 256 sampled candidates re-computed by the CPU oracle.
  plan_gpu_ms  -- mean device span of a timed plan: fence-free HIP events recorded on the plan's stream
                  just before and just after the C call that enqueues it (so from the enqueue of its
                  first launch to the end of its last kernel); host_ms_per_plan = ms_per_step minus it:
                  the host's turn per plan (Python around the call, the result sync and copy-out).
  strong       -- BASELINE.json configs[3]: walker-walk N=16384 H=30 split over the ranks (strong
                  scaling, N/G candidates per GPU), same timing rules; at N=1 the single-GPU plan the
                  split is measured against.
  strong_headline -- the headline cheetah N=4096 split over the ranks (N/G per GPU; north_star's
                  ">= 6x at 8 GPUs" read as strong scaling), beside the weak-scaled line.
  variants     -- the same workload timed with the other rollout precisions (default headline: exact
                  fp32; variants: f16x6 and f16x3, fp32 emulated on the f16 matrix cores).
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mujoco-mbrl_amd"))
sys.path.insert(0, REPO)

PEAK_FP32_MFMA_TFLOPS = 157.3
L2_STREAM_TBPS = 32.4   # tools/ubench/l2stream.hip: every CU streaming one L2-resident weight set
ITERATIONS = 5
MEASURED_IT = 2     # the CEM iteration whose rollout launch bench.py brackets with events


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, help="SURVEY.md §8d config id (default: cheetah-run CEM)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0,
                    help="seconds of CPU oracle work the cpu_baseline sample may take (about half is used)")
    ap.add_argument("--precision", default="f32", choices=["f32", "f16x3", "f16x6"],
                    help="rollout matmul precision (include/mbrl_cem.h MBRL_PRECISION_*)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the second-precision measurement (rocprof runs: only the headline launches)")
    ap.add_argument("--candidates", type=int, default=None,
                    help="candidates per GPU (weak) or in total (--strong); default: the config's N")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the config's N split over the GPUs (default weak: N per GPU)")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per rollout launch from a rocprofv3 PMC pass (profiles/)")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the strong-scaling walker object (BASELINE.json configs[3])")
    ap.add_argument("--no-train", action="store_true",
                    help="skip the model-training object (SURVEY.md §8f rank 2)")
    return ap.parse_args()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, script=None, argv=None):
    """`bench.py --gpus N` run directly: start N rank processes (this same script, its argv) and wait.
    Nothing here touches the GPU (no torch.cuda call at all), so the children are plain fresh
    processes; if one fails the others are stopped and its exit status is returned."""
    import subprocess
    port = str(_free_port())
    script = os.path.abspath(__file__) if script is None else script
    argv = sys.argv[1:] if argv is None else argv
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for pr in list(live):
            code = pr.poll()
            if code is None:
                continue
            live.remove(pr)
            if code != 0 and rc == 0:
                rc = code
                for other in live:
                    other.terminate()
        time.sleep(0.05)
    return rc


class TimingEvent:
    """A HIP event for timing only: hipEventCreateWithFlags(hipEventDisableSystemFence). A
    torch.cuda.Event record ends in a system-scope fence (cache writeback and invalidate) that left
    the GPU idle ~5.5 us at every record, ~55 us of a cheetah plan with two records per rollout
    (hip_runtime_api.h documents the flag for exactly this use). Same interface as torch's event
    where bench.py and the planners use it: .cuda_event, .record(), .elapsed_time(end)."""
    _hip = None

    @classmethod
    def _lib(cls):
        if cls._hip is None:
            import ctypes
            # torch's own HIP runtime (the one its streams and our extension live in), by path
            path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln)
            lib = ctypes.CDLL(path)
            lib.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            lib.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            lib.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            lib.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._hip = lib
        return cls._hip

    def __init__(self):
        import ctypes
        h = ctypes.c_void_p()
        if self._lib().hipEventCreateWithFlags(ctypes.byref(h), 0x20000000) != 0:   # hipEventDisableSystemFence
            raise RuntimeError("hipEventCreateWithFlags failed")
        self.cuda_event = h.value

    def record(self):
        import ctypes
        if self._lib().hipEventRecord(ctypes.c_void_p(self.cuda_event),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end):
        import ctypes
        ms = ctypes.c_float()
        if self._lib().hipEventElapsedTime(ctypes.byref(ms), ctypes.c_void_p(self.cuda_event),
                                           ctypes.c_void_p(end.cuda_event)) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def __del__(self):
        import ctypes
        if self._hip is not None and getattr(self, "cuda_event", None):
            self._hip.hipEventDestroy(ctypes.c_void_p(self.cuda_event))


def host_cores():
    """(cores used, how they were counted): the CPUs this process may run on
    (len(os.sched_getaffinity(0))), capped by the cgroup CPU quota when one is set
    (cpu.max / cfs_quota_us) -- threads beyond the quota only get throttled."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / period
        except (OSError, ValueError):
            pass
    cores = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    how = f"sched_getaffinity {aff}" + ("" if quota is None else f", cgroup quota {quota:g} CPUs")
    return cores, how


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return "unknown"


def cpu_baseline(cfg_id, budget_s=20.0):
    """Time the CPU oracle (rank 0, N=1 only) on a bounded sample of the same workload, with its BLAS
    on every core this process may use (host_cores)."""
    from oracle import cem as ocem
    cores, how = host_cores()
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=cores)
    except Exception:  # pragma: no cover
        limiter = None
    try:
        p = ocem.synth_problem(cfg_id)
        cfg = p["cfg"]
        N, H = cfg["N"], cfg["H"]
        # sample: whole CEM plans at the full N and H while they fit the budget, else fewer candidates
        t0 = time.perf_counter()
        ocem.cem_plan(p, num_iterations=1, record=False)
        one_iter = time.perf_counter() - t0
        n_sample = N if one_iter * ITERATIONS <= budget_s else max(64, int(N * budget_s / (one_iter * ITERATIONS)))
        plans, elapsed = 0, 0.0
        while elapsed < budget_s / 2 and plans < 10:
            t0 = time.perf_counter()
            ocem.cem_plan(p, N=n_sample, num_iterations=ITERATIONS, record=False)
            elapsed += time.perf_counter() - t0
            plans += 1
    finally:
        if limiter is not None:
            limiter.unregister()
    value = ITERATIONS * n_sample * H * plans / elapsed
    return dict(value=value, unit="candidate-timesteps/s", cores=int(cores), cores_counted=how, kind="port",
                cpu=_cpu_model(),
                sample=f"{plans} full CEM plan(s) (I={ITERATIONS}, N={n_sample}, H={H}) of the NumPy oracle "
                       f"(oracle/cem.py), fp32, {elapsed:.1f} s")


def cpu_torch_baseline(prob, budget_s=20.0):
    """The reference's own CPU arrangement, timed beside the NumPy oracle: torch on the host with
    autograd ON, as RandomShootingPlanner._generate_trajectories runs it (planners.py:199-210: H
    model calls writing state_list slices, then one cost call, view(H, N).sum(0)); the model is
    mbrl_amd.models on CPU (the reference's DynamicsModel math). CEM proposal / select / refit in
    NumPy (stable argsort, population variance). A bounded sample of the same workload, on every core
    this process may use (host_cores), and the same again under torch.no_grad() (labelled
    value_no_grad; the reference never disables autograd)."""
    cfg = prob["cfg"]
    N, H, a, s = cfg["N"], cfg["H"], cfg["a"], cfg["s"]
    threads, how = host_cores()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    model, cost = prob["model"], prob["cost"]
    s0 = prob["s0"].reshape(1, s).float()

    def plan(n):
        mu = np.zeros((H, a), np.float32)
        sg = np.full((H, a), 0.5, np.float32)
        for _ in range(ITERATIONS):
            A = np.clip(mu[:, None, :] + sg[:, None, :] * rng.standard_normal((H, n, a), dtype=np.float32), -1.0, 1.0)
            action_list = torch.from_numpy(A.reshape(H * n, a))
            state_list = torch.zeros((H * n, s))
            states = s0.expand(n, s)
            for t in range(H):
                states = model(states, action_list[t * n:(t + 1) * n])
                state_list[t * n:(t + 1) * n] = states
            costs = cost(state_list, action_list).view(H, n).sum(0).detach().numpy()
            el = A[:, np.argsort(costs, kind="stable")[:max(1, n // 10)], :]
            mu = 0.1 * mu + 0.9 * el.mean(axis=1)
            sg = np.sqrt(0.1 * sg * sg + 0.9 * el.var(axis=1)).astype(np.float32)
        return mu

    def measure(budget):
        t0 = time.perf_counter()
        plan(max(64, N // 16))
        probe = (time.perf_counter() - t0) * 16
        n_sample = N if probe <= budget else max(64, int(N * budget / probe))
        plans, elapsed = 0, 0.0
        while elapsed < budget and plans < 10:
            t0 = time.perf_counter()
            plan(n_sample)
            elapsed += time.perf_counter() - t0
            plans += 1
        return ITERATIONS * n_sample * H * plans / elapsed, n_sample, plans, elapsed

    try:
        v, n_sample, plans, elapsed = measure(budget_s / 2)
        with torch.no_grad():
            v_ng, n_ng, plans_ng, el_ng = measure(budget_s / 4)
    finally:
        torch.set_num_threads(prev_threads)
    return dict(value=v, unit="candidate-timesteps/s", cores=threads, cores_counted=how, kind="port",
                autograd=True, value_no_grad=v_ng, cpu=_cpu_model(),
                sample=f"{plans} CEM plan(s) (I={ITERATIONS}, N={n_sample}, H={H}): torch on the host, autograd on, "
                       f"the reference's _generate_trajectories loop + NumPy refit, {elapsed:.1f} s; "
                       f"value_no_grad: {plans_ng} plan(s) at N={n_ng} under torch.no_grad(), {el_ng:.1f} s")


def train_line(dev, W=512, epochs=50):
    """the reference's train_model (models.py:53-93; Adam, experiment.py:55-62)
    for a 2 x W Model on 10k synthetic cheetah-shaped transitions (s = 17, a = 6), batch 512 -- on this
    GPU through mbrl_train_epoch (csrc/train.hip: the fused two-launch step, Adam in its launches).
    Warm-up calls of 10, `epochs` and `epochs` epochs, then a 10-epoch and an `epochs`-epoch call, each
    timed between two events on the training stream (GPU-bound: one host call per epoch; the call's own
    start-up -- the first epoch's shuffle, the checks before the first launch, the final status read --
    inside the span). 50 is the
    reference's num_epochs default, which its agent's training loop uses (agents.py:292); a 10-epoch
    call is timed beside it. FLOP per step: forward 2R(K0 W + W^2 + W s), the same for the weight
    gradients, 2R(W s + W^2) for the input gradients (R = 512 rows)."""
    from mbrl_amd import data, models
    rng = np.random.Generator(np.random.PCG64(5))
    rolls = []
    for _ in range(20):
        st = rng.standard_normal((501, 17)).astype(np.float32)
        rolls.append(data.Rollout(states=list(torch.from_numpy(st)), observations=list(torch.from_numpy(st)),
                                  actions=list(torch.from_numpy(rng.uniform(-1, 1, (500, 6)).astype(np.float32))),
                                  rewards=list(torch.from_numpy(rng.standard_normal(500).astype(np.float32)))))
    ds = data.TransitionsDataset(rollouts=rolls)
    ds.set_data_mode("state_only")
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=W).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    gc.collect()    # the set-up's garbage (tens of thousands of per-step tensors) before the warm-up
    np.random.seed(1)
    # warm-up: the ring rows, the copy stream, events -- and ~120 ms of back-to-back training, which the
    # GPU needs to reach its steady clock after the host-side set-up above left it idle (the first
    # 50-epoch call of a process measured 57.1 us per step, the third 54.8: tools/train_gc_probe.py)
    for n in (10, epochs, epochs):
        m.train_model(ds, opt, batch_size=512, num_epochs=n)
    torch.cuda.synchronize(dev)
    def timed(n_epochs):
        np.random.seed(2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        m.train_model(ds, opt, batch_size=512, num_epochs=n_epochs)
        e1.record()
        torch.cuda.synchronize(dev)
        steps = n_epochs * ((ds.num_transitions() + 511) // 512)
        return steps, time.perf_counter() - t0, e0.elapsed_time(e1) * 1e3 / steps

    steps10, _, gpu_us10 = timed(10)
    steps, wall, gpu_us = timed(epochs)
    R, K0, s = 512, 23, 17
    flop = 2 * (2 * R * (K0 * W + W * W + W * s)) + 2 * R * (W * s + W * W)
    return dict(workload=f"train_model Model(17, 6) 2x{W}, batch 512, Adam, 10k synthetic transitions "
                         f"(SURVEY.md §8f rank 2)", steps_per_s=steps / wall, us_per_step=wall / steps * 1e6,
                gpu_us_per_step=gpu_us, gpu_us_per_step_10_epochs=gpu_us10, launches_per_step=2,
                status="the fused step's sticky status word (bounded in-launch waits) is read at the end of "
                       "every train_model call, which raises if it is set: clear for every call here",
                flop_per_step=flop, frac=flop / (gpu_us * 1e-6) / 1e12 / PEAK_FP32_MFMA_TFLOPS, epochs=epochs,
                steps=steps)


def rank_projection(dev, cfg_id, world, n_total, plans, warmup, allowances_us=(10.0, 25.0, 40.0)):
    """One rank's real share of a `world`-GPU plan, timed on this GPU: under
    the library's timing emulation (MBRL_OPT_SHARD_EMULATE = 2) mbrl_cem_plan_sharded runs exactly rank
    world-1's work -- its shard's rollout, the update over ALL n_total candidates with K = n_total/10,
    its own draw, the trajectory -- and fills the other ranks' slots of the all-gather from the costs a
    mode-1 plan kept (one launch per iteration). The result is checked bit-identical to the single-GPU
    plan first. The all-gather itself cannot run on one GPU: its time is an assumption, reported at
    each value of `allowances_us` per iteration."""
    from mbrl_amd import CEMPlanner, _lib, fused, planners, synthetic
    p = synthetic.make_problem(cfg_id)
    cfg = p["cfg"]
    md, cd = fused.describe(p["model"], p["cost"], dev)
    prob = fused.device_problem(md, cd, dev)
    kw = dict(num_candidates=n_total, num_elites=n_total // 10, num_iterations=ITERATIONS, seed=p["rng_seed"],
              device=dev)
    st = CEMPlanner._settings(p["sample_action"], cfg["H"], kw)
    st_rec = CEMPlanner._settings(p["sample_action"], cfg["H"], dict(kw, record=True))
    s0 = p["s0"].cpu().float()
    rank = world - 1
    ref = planners._cem_fused_single(prob, s0.to(dev), st_rec)
    with _lib.option("shard_emulate", 1):
        planners._cem_sharded_native(prob, s0.to(dev), st_rec, world, 0, comm=None)
    with _lib.option("shard_emulate", 2):
        got = planners._cem_sharded_native(prob, s0.to(dev), st_rec, world, rank, comm=None)
        same = all(torch.equal(torch.as_tensor(got[k]).cpu(), torch.as_tensor(ref[k]).cpu())
                   for k in ("elites", "mu", "sigma", "actions", "states"))
        for _ in range(warmup):
            planners._cem_sharded_native(prob, s0, st, world, rank, comm=None)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(plans):
            planners._cem_sharded_native(prob, s0, st, world, rank, comm=None)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / plans * 1e3
    return dict(gpus=world, rank=rank, candidates_total=n_total, candidates_per_rank=n_total // world,
                elites=n_total // 10, rank_ms_per_plan=ms, bit_identical_to_single_gpu_plan=same,
                allgather_us_assumed=list(allowances_us),
                rank_ms_with_allgather={f"{a:g}us": ms + ITERATIONS * a / 1e3 for a in allowances_us})


def parity_sample(prob, res, n=256):
    from oracle import cem as ocem
    from oracle.philox import cem_actions
    p = ocem.synth_problem(prob["cfg_id"])
    cfg = p["cfg"]
    H, a = cfg["H"], cfg["a"]
    idx = np.sort(np.random.default_rng(0).choice(res["returns"].shape[1], size=n, replace=False))
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1.0, 1.0, p["rng_seed"], 0, idx)
    ref = ocem.ensemble_returns(ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A)).astype(np.float64)
    got = res["returns"][0].cpu().numpy()[idx].astype(np.float64)
    return dict(return_mae=float(np.mean(np.abs(got - ref))),
                return_max_rel_err=float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0))),
                sample=f"iteration-0 returns of {n} candidates vs CPU oracle")


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; on a box with fewer GPUs than ranks (a gloo rehearsal, MBRL_DIST_BACKEND=gloo)
    # ranks share devices round-robin
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("MBRL_DIST_BACKEND", "nccl")     # nccl == RCCL over xGMI on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    from mbrl_amd import CEMPlanner, _lib, synthetic
    prob = synthetic.make_problem(args.config)
    prob["cfg_id"] = args.config
    cfg = prob["cfg"]
    H, E = cfg["H"], cfg["E"]
    n_cfg = args.candidates if args.candidates is not None else cfg["N"]
    if args.strong:
        if n_cfg % world:
            raise SystemExit(f"--strong: {n_cfg} candidates do not split over {world} GPUs")
        N, n_local = n_cfg, n_cfg // world
    else:
        n_local = n_cfg
        N = n_local * world
    K = N // 10
    kw = dict(num_candidates=N, num_elites=K, num_iterations=ITERATIONS, alpha=0.1, seed=prob["rng_seed"],
              distributed=world > 1, device=dev, precision=args.precision)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def timed(precision, problem=None, plan_kw=None):
        """W warm-up plans, then K timed plans between barriers; (max-over-ranks seconds, mean rollout
        launch seconds from HIP events on the launch stream, the first plan's record)."""
        pr = prob if problem is None else problem
        pkw = kw if plan_kw is None else plan_kw

        def plan(**extra):
            return CEMPlanner.plan_detailed(pr["s0"], pr["model"], pr["cost"], pr["sample_action"], pr["cfg"]["H"],
                                            **dict(pkw, precision=precision), **extra)
        first = plan(record=True)           # also warms the weight pack / workspaces
        for _ in range(max(0, args.warmup - 1)):
            plan()
        try:
            make_event = TimingEvent
            make_event()
        except (StopIteration, OSError, AttributeError, RuntimeError):   # no libamdhip64 mapping found
            def make_event():
                return torch.cuda.Event(enable_timing=True)
        # one bracketed rollout per plan (iteration MEASURED_IT of every timed plan): an event record
        # leaves the GPU idle ~4 us, so bracketing all five would cost the plan ~40 us
        events = [[(make_event(), make_event()) if it == MEASURED_IT else None for it in range(ITERATIONS)]
                  for _ in range(args.steps)]
        # one pair per plan around the C call that enqueues it: the plan's device span
        spans = [(make_event(), make_event()) for _ in range(args.steps)]
        for ev in events + [[sp] for sp in spans]:   # torch creates its events lazily: record once so
            for pair in ev:                          # the C ABI gets live handles
                if pair is not None:
                    pair[0].record()
                    pair[1].record()
        barrier()
        gc_acc = [0.0, 0, None]          # the Python garbage collector's pauses inside the timed region

        def gc_cb(phase, info):
            if phase == "start":
                gc_acc[2] = time.perf_counter()
            elif gc_acc[2] is not None:
                gc_acc[0] += time.perf_counter() - gc_acc[2]
                gc_acc[1] += 1
        gc.callbacks.append(gc_cb)
        stamps = [0.0] * (args.steps + 1)
        t0 = time.perf_counter()
        for k in range(args.steps):
            stamps[k] = time.perf_counter()
            plan(rollout_events=events[k], plan_events=spans[k])
        stamps[args.steps] = time.perf_counter()
        barrier()
        elapsed = time.perf_counter() - t0
        gc.callbacks.remove(gc_cb)
        timed.gc = dict(ms=gc_acc[0] * 1e3, collections=gc_acc[1])
        walls = np.diff(np.array(stamps)) * 1e3     # host wall time of each timed plan call
        timed.walls = dict(median=float(np.median(walls)), p90=float(np.percentile(walls, 90)),
                           max=float(walls.max()), min=float(walls.min()))
        if dist is not None:
            t = torch.tensor([elapsed], dtype=torch.float64,
                             device="cpu" if dist.get_backend() == "gloo" else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        rollout_ms = [pair[0].elapsed_time(pair[1]) for ev in events for pair in ev if pair is not None]
        span_ms = [sp[0].elapsed_time(sp[1]) for sp in spans]
        if dist is not None:   # the slowest rank's device span, as elapsed is the slowest rank's wall time
            t = torch.tensor([float(np.mean(span_ms))], dtype=torch.float64,
                             device="cpu" if dist.get_backend() == "gloo" else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            span_ms = [float(t.item())]
        timed.plan_gpu_ms = float(np.mean(span_ms))
        return elapsed, float(np.mean(rollout_ms)) / 1e3, first

    elapsed, avg_rollout_s, first = timed(args.precision)
    plan_gpu_ms = timed.plan_gpu_ms
    gc_stats = timed.gc
    wall_stats = timed.walls
    cand_steps = ITERATIONS * N * H * args.steps
    value = cand_steps / elapsed
    flop_launch = n_local * H * synthetic.flop_per_candidate_step(cfg)
    achieved = flop_launch / avg_rollout_s / 1e12
    traffic = args.traffic_bytes
    if traffic is None:
        prof = os.path.join(REPO, "profiles", "rollout_traffic.json")
        if os.path.exists(prof):
            try:
                traffic = json.load(open(prof)).get(cfg["name"])
            except Exception:  # pragma: no cover
                traffic = None
    out = {
        "metric": "candidate-timesteps/sec (CEM NxH rollout)",
        "value": value,
        "unit": "candidate-timesteps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "plan_gpu_ms": plan_gpu_ms,
        "host_ms_per_plan": elapsed / args.steps * 1e3 - plan_gpu_ms,
        "host_gc_in_timed_region": gc_stats,
        "plan_wall_ms": wall_stats,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": {"f32": "f32", "f16x3": "f32 (f16x3 split MFMA: fp32 emulated, 22-bit operands)",
                  "f16x6": "f32 (f16x6 split MFMA: fp32 emulated, 33-bit operands, fp32 accumulation)"}[args.precision],
        "data": "synthetic (random nn.Linear-law weights, PCG64 seed 1000+config; Philox proposals)",
        "config": {"workload": f"{cfg['name']} CEM N={N} H={H} s={cfg['s']} a={cfg['a']} "
                               f"{cfg['L']}x{cfg['W']} MLP E={E} I={ITERATIONS} K={K}",
                   "candidates_per_gpu": n_local, "horizon": H, "iterations": ITERATIONS, "elites": K,
                   "parallelism": f"candidates sharded x{world}" if world > 1 else "single GPU",
                   "world_size": world,
                   "backend": (dist.get_backend() if dist is not None else None),
                   "precision": args.precision},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP32_MFMA_TFLOPS, "traffic": traffic,
                     "kernel": "rollout_kernel", "avg_launch_ms": avg_rollout_s * 1e3,
                     "flop_per_launch": flop_launch},
    }
    built, same = _lib.build_info()
    out["build"] = {"library": "mujoco-mbrl_amd/mbrl_amd/libmbrl_cem.so", "source_digest": built,
                    "matches_tree": same}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["parity"] = parity_sample(prob, first)
    if not args.no_variants:
        # the same workload with the other matmul precisions (include/mbrl_cem.h MBRL_PRECISION_*)
        notes = {"f32": "exact fp32 MFMA",
                 "f16x3": "fp32 emulated on the f16 matrix cores: operands split into two f16 pieces (22 "
                          "significant bits), 3 partial products, fp32 accumulation; same parity bars "
                          "(tests/test_gpu_f16x3.py); bound by the L2 weight stream",
                 "f16x6": "fp32 emulated on the f16 matrix cores: operands split into three f16 pieces (33 "
                          "significant bits), the 6 partial products x_i w_j with i + j < 3 (exact), fp32 "
                          "accumulation; same parity bars (tests/test_gpu_f16x3.py)"}
        out["variants"] = []
        # the split kernels serve goal-state costs only (include/mbrl_cem.h); a reward-head model
        # would run fp32 under every precision, so it has no variants
        others = [] if cfg.get("reward") else [p for p in ("f32", "f16x6", "f16x3") if p != args.precision]
        for other in others:
            v_elapsed, v_rollout_s, v_first = timed(other)
            var = dict(precision=other, value=cand_steps / v_elapsed, ms_per_step=v_elapsed / args.steps * 1e3,
                       plan_gpu_ms=timed.plan_gpu_ms, rollout_avg_launch_ms=v_rollout_s * 1e3,
                       rollout_tflops_fp32_equivalent=flop_launch / v_rollout_s / 1e12, note=notes[other])
            if other != "f32":
                # the split kernels are bound by the per-CU L2 weight stream: algorithmic bytes = every
                # workgroup's weight stream for H steps; peak = tools/ubench/l2stream.hip's
                # measured 32.4 TB/s for this access pattern (MI355X_MICROARCH.md: 34.5 nominal)
                R = 2 if n_local >= 256 * 32 else 1
                wgs = -(-n_local // (16 * R)) * E
                l2 = wgs * H * synthetic.split_stream_bytes_per_step(cfg, 3 if other == "f16x6" else 2)
                var["roofline"] = {"bound": "l2", "achieved": l2 / v_rollout_s / 1e12, "peak": L2_STREAM_TBPS,
                                   "unit": "TB/s", "frac": l2 / v_rollout_s / 1e12 / L2_STREAM_TBPS,
                                   "kernel": "rollout_split_kernel", "algorithmic_bytes_per_launch": l2,
                                   "pmc": "profiles/r01_split_rollout_pmc.json"}
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                var["parity"] = parity_sample(prob, v_first)
            out["variants"].append(var)
    if not args.no_strong and not args.strong:
        # BASELINE.json configs[3]: walker-walk N=16384 H=30 split over the ranks (strong scaling)
        wprob = synthetic.make_problem(4)
        wcfg = wprob["cfg"]
        Nw = wcfg["N"]
        if Nw % world == 0:
            wkw = dict(num_candidates=Nw, num_elites=Nw // 10, num_iterations=ITERATIONS, alpha=0.1,
                       seed=wprob["rng_seed"], distributed=world > 1, device=dev)
            w_elapsed, w_rollout_s, _ = timed("f32", wprob, wkw)
            w_flop = Nw // world * wcfg["H"] * synthetic.flop_per_candidate_step(wcfg)
            out["strong"] = dict(
                workload=f"{wcfg['name']} CEM N={Nw} H={wcfg['H']} s={wcfg['s']} a={wcfg['a']} "
                         f"{wcfg['L']}x{wcfg['W']} MLP I={ITERATIONS} K={Nw // 10} (BASELINE.json configs[3])",
                scaling="strong", candidates_per_gpu=Nw // world, n_gpus=world,
                value=ITERATIONS * Nw * wcfg["H"] * args.steps / w_elapsed, unit="candidate-timesteps/s",
                ms_per_step=w_elapsed / args.steps * 1e3, plan_gpu_ms=timed.plan_gpu_ms,
                rollout_avg_launch_ms=w_rollout_s * 1e3,
                rollout_frac=w_flop / w_rollout_s / 1e12 / PEAK_FP32_MFMA_TFLOPS)
    if not args.no_strong and not args.strong and cfg["N"] % world == 0:
        # the headline workload itself split over the ranks: N = 4096 in total, N/G per GPU
        Nh = cfg["N"]
        hkw = dict(kw, num_candidates=Nh, num_elites=Nh // 10)
        h_elapsed, h_rollout_s, _ = timed(args.precision, prob, hkw) if world > 1 else (elapsed, avg_rollout_s, None)
        h_flop = Nh // world * H * synthetic.flop_per_candidate_step(cfg)
        out["strong_headline"] = dict(
            workload=f"{cfg['name']} CEM N={Nh} H={H} (the headline workload split over the ranks)",
            scaling="strong", candidates_per_gpu=Nh // world, n_gpus=world,
            value=ITERATIONS * Nh * H * args.steps / h_elapsed, unit="candidate-timesteps/s",
            ms_per_step=h_elapsed / args.steps * 1e3,
            plan_gpu_ms=timed.plan_gpu_ms if world > 1 else plan_gpu_ms,
            rollout_avg_launch_ms=h_rollout_s * 1e3,
            rollout_frac=h_flop / h_rollout_s / 1e12 / PEAK_FP32_MFMA_TFLOPS)
    if rank == 0 and world == 1 and not args.no_strong and not args.strong and args.config == 3:
        # the 8-GPU figures projected from one GPU: one rank's real work timed under the library's timing
        # emulation, with an assumed all-gather time (rank_projection): walker N=16384 split over 8
        # (strong, BASELINE configs[3]) against the walker single-GPU plan of `strong`, and the headline
        # weak-scaled to 8 GPUs (4096 per GPU, N = 32768, K = 3276 on every rank) against this line
        proj = {}
        wk = rank_projection(dev, 4, 8, 16384, plans=args.steps, warmup=args.warmup)
        t1 = out["strong"]["ms_per_step"]
        wk["single_gpu_ms_per_plan"] = t1
        wk["projected_speedup"] = {k: t1 / v for k, v in wk["rank_ms_with_allgather"].items()}
        proj["walker_strong_8"] = wk
        hw = rank_projection(dev, 3, 8, 8 * cfg["N"], plans=args.steps, warmup=args.warmup)
        t1 = out["ms_per_step"]
        hw["single_gpu_ms_per_plan"] = t1
        hw["projected_weak_efficiency"] = {k: t1 / v for k, v in hw["rank_ms_with_allgather"].items()}
        hw["projected_value_8gpu"] = {k: ITERATIONS * 8 * cfg["N"] * H / (v * 1e-3)
                                      for k, v in hw["rank_ms_with_allgather"].items()}
        proj["cheetah_weak_8"] = hw
        proj["note"] = ("projections on ONE GPU: a rank's own work under MBRL_OPT_SHARD_EMULATE=2 (DESIGN.md §5), "
                        "the all-gather's time assumed; the measured multi-GPU line is the driver's SCALE run")
        out["projection_8gpu"] = proj
    if rank == 0 and world == 1 and not args.no_train:   # (single-GPU runs only: no rank waits on it)
        out["train"] = train_line(dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.config, budget_s=args.cpu_budget)
        out["cpu_baseline_torch"] = cpu_torch_baseline(prob, budget_s=args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
