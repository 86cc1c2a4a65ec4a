"""Planners with the reference's static `plan()` API (/root/reference/src/mbrl/planners.py:14-25).

    plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs)
        -> (states [H, s], actions [H, a])

The class itself (not an instance) is what agents pass around (experiment.py:15-26, agents.py:48),
kwargs are read as kwargs.get(name, Cls.defaults[name]) (planners.py:141,153-155), and
`initial_trajectory` is accepted and ignored exactly as the reference's random-shooting planner
ignores it (planners.py:166-187).

RandomShootingPlanner -- the reference's planner (planners.py:140-216), same sampling call and
    argmin semantics, rollout + cost + argmin on the GPU.
CEMPlanner            -- the CEM hot path of BASELINE.json: I iterations of
    Philox proposal -> persistent MFMA rollout -> stable top-K -> alpha-smoothed Gaussian refit.
    With torch.distributed initialised and distributed=True, candidates are sharded over ranks:
    one RCCL all-gather of the per-candidate returns per iteration; every rank then runs the same
    deterministic selection and refit (the refit regenerates elite actions from the counter RNG,
    so no moment collective is needed and the result is bit-identical for any rank count).

Both take the fused path when fused.describe_* recognise the model / cost closures; otherwise the
user's callables run on device tensors (reference semantics, planners.py:199-210) and selection /
refit still run in the HIP extension.
"""
import contextlib
import threading
import warnings

import numpy as np
import torch

from . import _lib, fused


class ModelPlanner:
    """planners.py:14-25."""

    @staticmethod
    def plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs):
        raise NotImplementedError


def _device(kwargs):
    dev = kwargs.get("device")
    if dev is None:
        if not torch.cuda.is_available():
            raise RuntimeError("mbrl_amd planners need a ROCm GPU (torch.cuda.is_available() is False)")
        dev = torch.device("cuda", torch.cuda.current_device())
    return torch.device(dev)


_NULL_CTX = contextlib.nullcontext()


def _on_device(dev):
    """torch.cuda.device(dev), or a no-op when dev is already the current device (the common case:
    the context manager's enter and exit are a few microseconds of every plan's host turn)."""
    if dev.index is not None and torch._C._cuda_getDevice() == dev.index:
        return _NULL_CTX
    return torch.cuda.device(dev)


def _to_host(x, keep_device):
    return x if keep_device else x.cpu()


def _generic_costs(model, cost, s0, actions, H, N):
    """planners.py:199-210 with the caller's callables. actions [H, N, a] on the GPU.

    The callables are opaque: they run on GPU tensors when they accept them, else (their own
    parameters live on the host, e.g. a cost closing over CPU goal tensors as the reference's
    agents build them) on host copies of the inputs. Returns costs [1, N] (sequential sum over t)
    and states [H, N, s] on the GPU; selection and refit stay in the HIP extension."""
    dev = actions.device
    s = s0.shape[0]

    def call(fn, *args):
        try:
            return fn(*args).to(dev)
        except RuntimeError as e:
            if "device" not in str(e):
                raise
            return fn(*[x.cpu() for x in args]).to(dev)

    states = torch.empty((H, N, s), dtype=torch.float32, device=dev)
    cur = s0.unsqueeze(0).repeat_interleave(N, dim=0)
    with torch.no_grad():
        for t in range(H):
            cur = call(model, cur, actions[t])
            states[t] = cur
        c = call(cost, states.reshape(H * N, s), actions.reshape(H * N, -1)).reshape(H, N)
        total = c[0].clone()
        for t in range(1, H):
            total = total + c[t]
    return total.reshape(1, N).contiguous(), states


class GradientDescentPlanner(ModelPlanner):
    """planners.py:28-137: Adam(lr=0.01) on one action sequence through the learned dynamics, on the
    GPU for recognised closures (mbrl_amd/gd.py), else the reference's loop on the given callables.
    Returns lists of H+1 states [1, s] and H actions [1, a], as the reference does."""
    defaults = dict(num_iterations=40, stop_condition=0.002)
    # plans start from the previous plan of the same episode (MPCPolicy's initial_trajectory,
    # agents.py:40-55): the planner service passes those to plan_batch (parallel._answer)
    warm_starts = True

    @staticmethod
    def plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs):
        from . import gd
        num_iterations = int(kwargs.get("num_iterations", GradientDescentPlanner.defaults["num_iterations"]))
        stop_condition = float(kwargs.get("stop_condition", GradientDescentPlanner.defaults["stop_condition"]))
        H = int(horizon)
        mdesc = None
        if torch.cuda.is_available():
            dev = _device(kwargs)
            mdesc, cdesc = gd.describe(model, cost, dev)
        if mdesc is not None:
            if initial_trajectory is None:
                # planners.py:94: the nominal sequence (its states are not used for a deterministic model)
                action_list = list(sample_action(batch_size=H).split(1, dim=0))
            else:
                action_list = initial_trajectory[1]
            with torch.cuda.device(dev):
                states, actions = gd.plan_device(initial_state, mdesc, cdesc, action_list, H, num_iterations,
                                                 stop_condition, dev)
        else:
            states, actions = gd.plan_generic(initial_state, model, cost, sample_action, H, initial_trajectory,
                                              num_iterations, stop_condition)
        keep = kwargs.get("return_device", False)
        states, actions = _to_host(states, keep), _to_host(actions, keep)
        return list(states.split(1, 0)), list(actions.split(1, 0))

    @staticmethod
    def plan_batch(initial_states, model, cost, sample_action, horizon, initial_trajectories=None, **kwargs):
        """B independent plans, one per row of initial_states [B, s] (parallel environments), each
        what plan() returns for that row. Row b starts from initial_trajectories[b][1] or, where that
        (or the whole list) is None, from sample_action(batch_size=horizon), drawn in row order (as
        B plan() calls would draw). Recognised closures run in shared launches (mbrl_gd_plan_batch: the
        cooperative grids of up to 256 / (Wpad / 16) plans at once); others run plan() per row.
        Returns (states [B, H+1, s], actions [B, H, a])."""
        from . import gd
        num_iterations = int(kwargs.get("num_iterations", GradientDescentPlanner.defaults["num_iterations"]))
        stop_condition = float(kwargs.get("stop_condition", GradientDescentPlanner.defaults["stop_condition"]))
        H, B = int(horizon), int(initial_states.shape[0])
        inits = [None if initial_trajectories is None else initial_trajectories[b] for b in range(B)]
        keep = kwargs.get("return_device", False)
        mdesc = cdesc = None
        if torch.cuda.is_available():
            dev = _device(kwargs)
            mdesc, cdesc = gd.describe(model, cost, dev)
        if mdesc is not None and gd.fused_supported(mdesc, cdesc, dev) and num_iterations > 0:
            starts = [torch.cat(list(sample_action(batch_size=H).split(1, dim=0)), 0) if init is None
                      else torch.cat([x.reshape(1, -1) for x in init[1]], 0) for init in inits]
            with torch.cuda.device(dev):
                states, actions, _ = gd.plan_fused_batch(initial_states, mdesc, cdesc, torch.stack(starts), H,
                                                         num_iterations, stop_condition, dev)
            return _to_host(states, keep), _to_host(actions, keep)
        # per row, in row order; a row without a warm start draws its sequence inside its own plan(),
        # so a model that uses torch's RNG sees exactly the stream of B plan() calls
        outs = [GradientDescentPlanner.plan(initial_states[b], model, cost, sample_action, H,
                                            initial_trajectory=None if inits[b] is None else (None, list(inits[b][1])),
                                            **dict(kwargs, return_device=True)) for b in range(B)]
        states = torch.stack([torch.cat(o[0], 0).reshape(H + 1, -1) for o in outs])
        actions = torch.stack([torch.cat(o[1], 0).reshape(H, -1) for o in outs])
        return _to_host(states, keep), _to_host(actions, keep)


def _rs_host(initial_state, model, cost, sample_action, H, N):
    """RandomShootingPlanner on a host without a GPU (BASELINE configs[0]: the reference's own CPU
    random-shooting path): the reference's a2 loop on the caller's callables, as written
    (/root/reference/src/mbrl/planners.py:189-216: one sample_action(N * H) draw, time-major rows
    t * N + n, H model calls, one cost call, view(H, N).sum(0)), then np.argmin (first index on ties,
    :184). Returns (states [H, s], actions [H, a]) of the chosen candidate."""
    s = initial_state.shape[0]
    with torch.no_grad():
        state_list = torch.zeros((N * H, s))
        action_list = sample_action(batch_size=N * H)
        for t in range(H):
            states = (initial_state.unsqueeze(dim=0).repeat_interleave(N, dim=0) if t == 0
                      else state_list[(t - 1) * N:t * N])
            state_list[t * N:(t + 1) * N] = model(states, action_list[t * N:(t + 1) * N])
        costs = cost(state_list, action_list).view(H, N).sum(0).detach().numpy()
    i = int(np.argmin(costs))
    return state_list.view(H, N, -1)[:, i], action_list.view(H, N, -1)[:, i]


class RandomShootingPlanner(ModelPlanner):
    """planners.py:140-216 on the GPU; on a host without one (torch.cuda.is_available() False), the
    reference's own CPU loop on the given callables (_rs_host: BASELINE configs[0] is this planner on
    CPU). With a GPU the HIP path always runs (and raises if the extension is missing)."""
    defaults = dict(num_trajectories=1000)

    @staticmethod
    def plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs):
        kw = dict(kwargs)
        num_trajectories = kw.pop("num_trajectories", RandomShootingPlanner.defaults["num_trajectories"])
        return RandomShootingPlanner._plan(initial_state, model, cost, sample_action, horizon, initial_trajectory,
                                           num_trajectories, **kw)

    @staticmethod
    def _plan(initial_state, model, cost, sample_action, horizon, initial_trajectory, num_trajectories, **kwargs):
        N, H = int(num_trajectories), int(horizon)
        if kwargs.get("device") is None and not torch.cuda.is_available():
            return _rs_host(initial_state, model, cost, sample_action, H, N)
        dev = _device(kwargs)
        # planners.py:200: one draw of N*H actions from the caller's sampler (host RNG), time-major
        action_list = sample_action(batch_size=N * H)
        a = action_list.shape[1]
        with torch.cuda.device(dev):
            acts = action_list.to(device=dev, dtype=torch.float32).reshape(H, N, a).contiguous()
            s0 = initial_state.to(device=dev, dtype=torch.float32).contiguous()
            mdesc, cdesc, prob = fused.describe_problem(model, cost, dev,
                                                        _lib.precision_code(kwargs.get("precision", "f32")))
            if mdesc is not None and cdesc is not None and mdesc["E"] == 1 and mdesc["a"] == a:
                states = torch.empty((1, H, N, mdesc["s"]), dtype=torch.float32, device=dev)
                costs = fused.rollout(prob, s0, N, H, actions=acts, states_out=states)
                states = states[0]
            else:
                costs, states = _generic_costs(model, cost, s0, acts, H, N)
            idx = fused.select(costs, 1, nan_policy=_lib.MBRL_NAN_FIRST)   # np.argmin, planners.py:184
            i = idx[0]
            out_states = states[:, i]
            out_actions = acts[:, i]
            keep = kwargs.get("return_device", False)
            return _to_host(out_states, keep), _to_host(out_actions, keep)


    @staticmethod
    def plan_batch(initial_states, model, cost, sample_action, horizon, **kwargs):
        """B plans, one per row of initial_states [B, s] (parallel environments), each what plan()
        returns for that row: row b's N x H proposals are the b-th sample_action(batch_size=N*H)
        draw (row order, as B plan() calls would draw). Recognised closures roll all B*N candidates
        out in one launch (per-candidate start states), then take each row's np.argmin.
        Returns (states [B, H, s], actions [B, H, a])."""
        kw = dict(kwargs)
        N = int(kw.pop("num_trajectories", RandomShootingPlanner.defaults["num_trajectories"]))
        H, B = int(horizon), int(initial_states.shape[0])
        keep = kw.get("return_device", False)
        dev = _device(kw)
        with torch.cuda.device(dev):
            mdesc, cdesc = fused.describe(model, cost, dev)
            fusable = mdesc is not None and cdesc is not None and mdesc["E"] == 1
            # recognised closures use no RNG, so all B draws can come first; unrecognised ones (a model
            # may draw from torch's RNG) interleave each row's draw with its plan, as B plan() calls do
            draws = [sample_action(batch_size=N * H) for _ in range(B)] if fusable else None
            if not fusable or mdesc["a"] != draws[0].shape[1]:
                outs = []
                for b in range(B):
                    sampler = sample_action
                    if draws is not None:
                        it = iter([draws[b]])
                        sampler = lambda batch_size, it=it: next(it)  # noqa: E731
                    outs.append(RandomShootingPlanner._plan(initial_states[b], model, cost, sampler, H, None, N,
                                                            **dict(kw, return_device=True)))
                return (_to_host(torch.stack([o[0] for o in outs]), keep),
                        _to_host(torch.stack([o[1] for o in outs]), keep))
            a = draws[0].shape[1]
            prob = fused.device_problem(mdesc, cdesc, dev, _lib.precision_code(kw.get("precision", "f32")))
            acts = torch.cat([d.to(device=dev, dtype=torch.float32).reshape(H, N, a) for d in draws], 1).contiguous()
            s0 = initial_states.to(device=dev, dtype=torch.float32).reshape(B, 1, -1).expand(B, N, -1)
            s0 = s0.reshape(B * N, -1).contiguous()
            states = torch.empty((1, H, B * N, mdesc["s"]), dtype=torch.float32, device=dev)
            costs = fused.rollout(prob, s0, B * N, H, actions=acts, s0_per_candidate=True, states_out=states)
            best = torch.stack([fused.select(costs[:, b * N:(b + 1) * N].contiguous(), 1,
                                             nan_policy=_lib.MBRL_NAN_FIRST)[0] for b in range(B)])  # np.argmin
            cols = best + torch.arange(B, device=dev) * N
            out_states = states[0][:, cols].transpose(0, 1)
            out_actions = acts[:, cols].transpose(0, 1)
            return _to_host(out_states.contiguous(), keep), _to_host(out_actions.contiguous(), keep)


class CEMPlanner(ModelPlanner):
    """Cross-entropy method over action sequences (not in the reference).

    kwargs (defaults): num_candidates (1000), num_elites (None -> num_candidates // 10),
    num_iterations (5), alpha (0.1), seed (None -> drawn from the global NumPy RNG, like the
    reference's sampler), init_std (None -> (hi - lo) / 4), action_bounds (None -> from
    sample_action's action_spec, else (-1, 1)), distributed (False), return_device (False),
    precision ("f32": exact fp32 MFMA; "f16x6" / "f16x3": fp32 emulated on the f16 matrix cores
    with 33 / 22 significant operand bits, see include/mbrl_cem.h). Timing hooks (bench.py):
    rollout_events (per-iteration event pairs around the rollout launch), plan_events (one pair
    recorded on the plan's stream just before and just after the C call that enqueues the plan).
    Returns the final Gaussian mean (clipped) and its predicted states (ensemble mean)."""
    defaults = dict(num_candidates=1000, num_elites=None, num_iterations=5, alpha=0.1, seed=None, init_std=None,
                    action_bounds=None, distributed=False, return_device=False, precision="f32")

    @staticmethod
    def plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs):
        res = CEMPlanner.plan_detailed(initial_state, model, cost, sample_action, horizon, initial_trajectory,
                                       **kwargs)
        return res["states"], res["actions"]

    @staticmethod
    def plan_batch(initial_states, model, cost, sample_action, horizon, **kwargs):
        """B plans at once, one per row of initial_states [B, s] (see cem_plan_batch)."""
        return cem_plan_batch(initial_states, model, cost, sample_action, horizon, **kwargs)

    _SETTINGS = {}
    _HOOKS = ("rollout_events", "plan_events")

    @staticmethod
    def _settings(sample_action, horizon, kwargs):
        """The plan's settings; with an explicit seed the dict is built once per (sampler, horizon,
        kwargs) and reused (part of every plan's host turn). The timing hooks (fresh lists per plan in
        bench.py) stay out of the key and are set on a copy."""
        if kwargs.get("seed") is not None:
            try:
                key = (id(sample_action), horizon,
                       tuple((k, v) for k, v in kwargs.items() if k not in CEMPlanner._HOOKS))
                hit = CEMPlanner._SETTINGS.get(key)
            except TypeError:          # an unhashable kwargs value: no caching
                key, hit = None, None
            if hit is None or hit[0] is not sample_action:
                hit = (sample_action, CEMPlanner._settings_build(sample_action, horizon, kwargs))
                if key is not None:
                    if len(CEMPlanner._SETTINGS) > 64:
                        CEMPlanner._SETTINGS.clear()
                    CEMPlanner._SETTINGS[key] = hit
            st = hit[1]
            ev, pev = kwargs.get("rollout_events"), kwargs.get("plan_events")
            if ev is not st["events"] or pev is not st["plan_events"]:
                st = dict(st, events=ev, plan_events=pev)
            return st
        return CEMPlanner._settings_build(sample_action, horizon, kwargs)

    @staticmethod
    def _settings_build(sample_action, horizon, kwargs):
        d = CEMPlanner.defaults
        g = lambda k: kwargs.get(k, d[k])  # noqa: E731
        N = int(g("num_candidates"))
        K = g("num_elites")
        K = max(1, N // 10) if K is None else int(K)
        bounds = g("action_bounds")
        sdesc = fused.describe_sampler(sample_action) if sample_action is not None else None
        if bounds is None:
            bounds = (sdesc[0], sdesc[1]) if sdesc is not None else (-1.0, 1.0)
        lo, hi = float(bounds[0]), float(bounds[1])
        init_std = g("init_std")
        init_std = float(np.float32(hi - lo) / np.float32(4.0)) if init_std is None else float(init_std)
        seed = g("seed")
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 62, dtype=np.int64))
        if not 1 <= K <= N:
            raise ValueError(f"need 1 <= num_elites ({K}) <= num_candidates ({N})")
        return dict(N=N, K=K, H=int(horizon), I=int(g("num_iterations")), alpha=float(g("alpha")), lo=lo, hi=hi,
                    init_std=init_std, seed=seed, distributed=bool(g("distributed")),
                    keep=bool(g("return_device")), record=bool(kwargs.get("record", False)),
                    events=kwargs.get("rollout_events"), plan_events=kwargs.get("plan_events"),
                    adim=sdesc[2] if sdesc else None,
                    precision=_lib.precision_code(g("precision")))

    @staticmethod
    def plan_detailed(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs):
        """plan() plus diagnostics: dict(states, actions, mu, sigma[, costs, returns, elites per iteration])."""
        dev = _device(kwargs)
        st = CEMPlanner._settings(sample_action, horizon, kwargs)
        with _on_device(dev):
            mdesc, cdesc, prob = fused.describe_problem(model, cost, dev, st["precision"])
            ws = None
            if st["distributed"] and torch.distributed.is_available() and torch.distributed.is_initialized() \
                    and torch.distributed.get_world_size() > 1:
                ws = torch.distributed.get_world_size()
            if mdesc is not None and cdesc is not None:
                if ws is None:
                    res = _cem_fused_single(prob, initial_state, st)
                    if res.pop("_host", False):
                        return res
                else:
                    res = _cem_fused_sharded(prob, initial_state, st, ws)
                    if res.pop("_host", False):
                        return res
            else:
                a = st["adim"]
                if a is None:
                    a = sample_action(batch_size=1).shape[1]
                res = _cem_generic(model, cost, initial_state.to(device=dev, dtype=torch.float32).contiguous(), st,
                                   a, dev)
            both = res.pop("_both", None)
            if both is not None and not st["keep"]:
                host = both.cpu()              # one device-to-host copy for states and actions
                H, s = res["states"].shape
                res["states"] = host[:H * s].view(H, s)
                res["actions"] = host[H * s:].view(H, -1)
            else:
                res["states"] = _to_host(res["states"], st["keep"])
                res["actions"] = _to_host(res["actions"], st["keep"])
            return res


def cem_plan_batch(initial_states, model, cost, sample_action, horizon, **kwargs):
    """B independent CEM plans in shared launches (mbrl_cem_plan_batch): one per row of
    initial_states [B, s], e.g. the observations of B parallel environments (parallel.py:20-52
    runs one planner per worker process; here one GPU serves them all). kwargs as CEMPlanner.plan;
    num_candidates / num_elites are per problem. Problem b draws its proposals as candidates
    [b*N, (b+1)*N) of one Philox stream. Returns (states [B, H, s], actions [B, H, a]).

    Closures the fused path does not recognise fall back to one CEMPlanner.plan per row."""
    dev = _device(kwargs)
    st = CEMPlanner._settings(sample_action, horizon, kwargs)
    B = int(initial_states.shape[0])
    with torch.cuda.device(dev):
        mdesc, cdesc, prob = fused.describe_problem(model, cost, dev, st["precision"])
        if mdesc is None or cdesc is None:
            outs = [CEMPlanner.plan(initial_states[b], model, cost, sample_action, horizon,
                                    **dict(kwargs, seed=st["seed"], return_device=True)) for b in range(B)]
            states, actions = torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs])
        else:
            lib = _lib.load()
            N, K, H, I = st["N"], st["K"], st["H"], st["I"]
            a, s = mdesc["a"], mdesc["s"]
            params = _lib.CemParams(N, H, K, I, st["alpha"], st["lo"], st["hi"], 0.0, st["init_std"], 0,
                                    int(st["seed"]) & 0xFFFFFFFFFFFFFFFF)
            need = lib.mbrl_cem_plan_batch_workspace_bytes(fused.ctypes_ref(prob.shape), fused.ctypes_ref(params), B)
            ws = _workspace(("cem_batch", str(dev)), need, dev)
            s0 = initial_states.to(device=dev, dtype=torch.float32).reshape(B, s).contiguous()
            actions = torch.empty((B, H, a), dtype=torch.float32, device=dev)
            states = torch.empty((B, H, s), dtype=torch.float32, device=dev)
            _lib.check(lib.mbrl_cem_plan_batch(fused.ctypes_ref(prob.shape), _lib.ptr(prob.packed),
                                               fused.ctypes_ref(prob.norm), fused.ctypes_ref(prob.cost), _lib.ptr(s0),
                                               B, fused.ctypes_ref(params), None, None, _lib.ptr(actions),
                                               _lib.ptr(states), _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev)),
                       "mbrl_cem_plan_batch")
        keep = st["keep"]
        return _to_host(states, keep), _to_host(actions, keep)


_WS = threading.local()


def _workspace(key, nbytes, device):
    """Scratch for `key` owned by this thread and the current stream of `device`. A plan enqueues on
    the current stream and reuses its scratch in stream order; another thread, or this thread on
    another stream, gets a buffer of its own, so plans in flight never share scratch (the flags,
    epochs and proposals of one plan are not overwritten by another's launches)."""
    bufs = getattr(_WS, "bufs", None)
    if bufs is None:
        bufs = _WS.bufs = {}
    idx = device.index if device.index is not None else torch.cuda.current_device()
    k = key + (torch._C._cuda_getCurrentRawStream(idx),)
    buf = bufs.get(k)
    if buf is None or buf.numel() < nbytes or buf.device != device:
        if buf is None and len(bufs) > 16:
            bufs.clear()
        buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        bufs[k] = buf
    return buf


_STAGING = threading.local()
# plan() with host inputs / outputs goes through mapped pinned staging (_cem_plan_host); False: the
# device-buffer path with a host-to-device copy of s0 and a device-to-host copy of the results (A/B)
HOST_STAGING = True


def _staging(dev, n):
    """This thread's mapped pinned host buffer of >= n floats for plans on `dev` (_lib.HostStaging)."""
    bufs = getattr(_STAGING, "bufs", None)
    if bufs is None:
        bufs = _STAGING.bufs = {}
    buf = bufs.get(str(dev))
    if buf is None or buf.n < n:
        buf = bufs[str(dev)] = _lib.HostStaging(max(n, 256))
    return buf


def _cem_plan_host(lib, prob, initial_state, st, params, ws, pref):
    """mbrl_cem_plan with host staging (_lib.HostStaging): the plan's first launch reads the initial
    state from mapped host memory and its last launches write states, actions, mu and sigma there, so
    no copy launch precedes or follows the plan; one stream sync, then host tensors."""
    dev = prob.device
    md = prob.mdesc
    H, a, s = st["H"], md["a"], md["s"]
    stage = _staging(dev, H * (s + 3 * a) + s)
    arr = stage.array
    o_s0 = H * (s + 3 * a)
    x = initial_state.detach() if initial_state.requires_grad else initial_state
    arr[o_s0:o_s0 + s] = x.numpy().reshape(-1) if x.dtype == torch.float32 else x.reshape(-1).to(torch.float32).numpy()
    o_act, o_mu, o_sg = H * s, H * (s + a), H * (s + 2 * a)
    at = stage.cached_at((H, s, a), (o_s0, o_mu, o_sg, o_act, 0))
    pev = st["plan_events"]
    if pev is not None:
        pev[0].record()
    _lib.check(lib.mbrl_cem_plan(*prob.refs, at[0], pref, at[1], at[2], at[3], at[4], None, None, None,
                                 _events(st, params.iterations), _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev)),
               "mbrl_cem_plan")
    if pev is not None:
        pev[1].record()
    torch.cuda.current_stream(dev).synchronize()
    x = arr[:o_s0].copy()                 # (NumPy views wrapped once each: ~2.4x cheaper than torch views)
    return dict(states=torch.from_numpy(x[:o_act].reshape(H, s)), actions=torch.from_numpy(x[o_act:o_mu].reshape(H, a)),
                mu=torch.from_numpy(x[o_mu:o_sg].reshape(H, a)), sigma=torch.from_numpy(x[o_sg:].reshape(H, a)),
                _host=True)


_EVENT_ARRAYS = {}


def _events(st, I):
    events = st["events"]
    if events is None:
        return None
    handles = tuple((e.cuda_event if pair is not None else None) for pair in events for e in (pair or (None, None)))
    arr = _EVENT_ARRAYS.get(handles)
    if arr is None:
        if len(_EVENT_ARRAYS) > 16:
            _EVENT_ARRAYS.clear()
        arr = _EVENT_ARRAYS[handles] = (_lib.c_void_p * (2 * I))(*handles)
    return arr


def _cem_fused_single(prob, initial_state, st):
    """One C-ABI call: mbrl_cem_plan (every iteration stream-ordered, no host sync)."""
    lib = _lib.load()
    dev = prob.device
    md = prob.mdesc
    N, K, H, I = st["N"], st["K"], st["H"], st["I"]
    a, s, E = md["a"], md["s"], md["E"]
    # the params struct and the workspace size per settings, built once per problem (host turn)
    pkey = (N, H, K, I, st["alpha"], st["lo"], st["hi"], st["init_std"], int(st["seed"]) & 0xFFFFFFFFFFFFFFFF)
    hit = prob.plan_cache.get(pkey)
    if hit is None:
        params = _lib.CemParams(N, H, K, I, st["alpha"], st["lo"], st["hi"], 0.0, st["init_std"], 0, pkey[-1])
        need = lib.mbrl_cem_workspace_bytes(fused.ctypes_ref(prob.shape), fused.ctypes_ref(params))
        if len(prob.plan_cache) > 64:
            prob.plan_cache.clear()
        hit = prob.plan_cache[pkey] = (params, fused.ctypes_ref(params), need)
    params, pref, need = hit
    ws = _workspace(("cem", str(dev)), need, dev)
    if HOST_STAGING and not st["keep"] and not st["record"] and not initial_state.is_cuda:
        return _cem_plan_host(lib, prob, initial_state, st, params, ws, pref)
    s0 = initial_state.to(device=dev, dtype=torch.float32).contiguous()
    # one allocation for the outputs; states and actions side by side, so that plan() hands both
    # back to the host in ONE copy
    buf = torch.empty(H * (s + 3 * a), dtype=torch.float32, device=dev)
    both = buf[:H * (s + a)]
    states = both[:H * s].view(H, s)
    actions = both[H * s:].view(H, a)
    mu = buf[H * (s + a):H * (s + 2 * a)].view(H, a)
    sigma = buf[H * (s + 2 * a):].view(H, a)
    rec = st["record"]
    cost_hist = torch.empty((I, E, N), dtype=torch.float32, device=dev) if rec else None
    ret_hist = torch.empty((I, N), dtype=torch.float32, device=dev) if rec else None
    elite_hist = torch.empty((I, K), dtype=torch.int64, device=dev) if rec else None
    ev_arr = _events(st, I)
    pev = st["plan_events"]
    if pev is not None:
        pev[0].record()
    _lib.check(lib.mbrl_cem_plan(fused.ctypes_ref(prob.shape), _lib.ptr(prob.packed), fused.ctypes_ref(prob.norm),
                                 fused.ctypes_ref(prob.cost), _lib.ptr(s0), fused.ctypes_ref(params), _lib.ptr(mu),
                                 _lib.ptr(sigma), _lib.ptr(actions), _lib.ptr(states), _lib.ptr(cost_hist),
                                 _lib.ptr(ret_hist), _lib.ptr(elite_hist), ev_arr, _lib.ptr(ws), ws.numel(),
                                 _lib.stream_handle(dev)), "mbrl_cem_plan")
    if pev is not None:
        pev[1].record()
    out = dict(states=states, actions=actions, mu=mu, sigma=sigma, _both=both)
    if rec:
        out.update(costs=cost_hist, returns=ret_hist, elites=elite_hist)
    return out


def cem_sharded_protocol(ops, st, world, rank):
    """Host protocol of the sharded CEM plan, independent of where the math runs.

    Rank r of G owns global candidates [r*N/G, (r+1)*N/G). Per iteration: local proposal draw +
    rollout (proposals keyed by the GLOBAL candidate index) -> one all-gather of the [E, N/G] local
    costs -> every rank runs the same deterministic select + refit on the full [E, N] costs. The
    refit regenerates the elites' actions from the counter RNG, so no moment collective is needed
    and mu / sigma are bit-identical on every rank and for every G.

    ops: .device; .rollout(it, mu, sigma, n_offset, n_local, costs_out[E, n_local], events) (events: None
    or a (start, end) pair to record around the rollout kernel alone);
    .all_gather(out_flat[G*E*n_local], local[E, n_local]); .select(costs[E, N], K, returns_out) -> elites;
    .refit(it, mu, sigma, elites, mu_out, sigma_out); .trajectory(actions[H, a]) -> states[H, s]; optionally
    .update(it, mu, sigma, costs, K, returns_out, mu_out, sigma_out, draw_next, n_offset, n_local) -> elites
    or None: select + refit (+ this rank's next proposals) at once, None when it does not apply.
    The fused path binds them to the HIP extension + RCCL; tests bind them to the CPU oracle + gloo."""
    N, K, H, I, E, a = st["N"], st["K"], st["H"], st["I"], st["E"], st["a"]
    if N % world:
        raise ValueError(f"num_candidates {N} must divide evenly over {world} ranks")
    Nl = N // world
    dev = ops.device
    mu = torch.zeros((H, a), dtype=torch.float32, device=dev)
    sigma = torch.full((H, a), st["init_std"], dtype=torch.float32, device=dev)
    mu_n, sigma_n = torch.empty_like(mu), torch.empty_like(sigma)
    local = torch.empty((E, Nl), dtype=torch.float32, device=dev)
    gathered = torch.empty(world * E * Nl, dtype=torch.float32, device=dev)
    rec = st["record"]
    hist = dict(costs=[], returns=[], elites=[])
    events = st["events"]
    for it in range(I):
        ops.rollout(it, mu, sigma, rank * Nl, Nl, local, None if events is None else events[it])
        ops.all_gather(gathered, local)
        # candidate r*Nl + j lives at gathered[r, :, j]
        costs = gathered.view(world, E, Nl).permute(1, 0, 2).reshape(E, N) if world > 1 else gathered.view(E, N)
        rets = torch.empty(N, dtype=torch.float32, device=dev) if rec else None
        upd = getattr(ops, "update", None)
        elites = None if upd is None else upd(it, mu, sigma, costs, K, rets, mu_n, sigma_n, it + 1 < I, rank * Nl, Nl)
        if elites is None:
            elites = ops.select(costs, K, rets)
            ops.refit(it, mu, sigma, elites, mu_n, sigma_n)
        mu, mu_n = mu_n, mu
        sigma, sigma_n = sigma_n, sigma
        if rec:
            hist["costs"].append(costs.clone())
            hist["returns"].append(rets)
            hist["elites"].append(elites)
    actions = mu.clamp(st["lo"], st["hi"]).contiguous()
    states = ops.trajectory(actions)
    out = dict(states=states, actions=actions, mu=mu, sigma=sigma)
    if rec:
        out.update({k: torch.stack(v) for k, v in hist.items()})
    return out


class _FusedShardOps:
    """cem_sharded_protocol bound to the HIP extension (C ABI) and torch.distributed (RCCL)."""

    def __init__(self, prob, s0, st):
        self.prob, self.s0, self.st, self.device = prob, s0, st, prob.device
        H, a, N, K = st["H"], prob.mdesc["a"], st["N"], st["K"]
        lib = _lib.load()
        self._acts = None
        self._drawn = None      # (iteration, n_offset, n_local) whose proposals self._acts holds
        self._fused_update = True
        self._sel_ws = _workspace(("sel", str(self.device)), lib.mbrl_select_workspace_bytes(N), self.device)
        self._refit_ws = _workspace(("refit", str(self.device)), lib.mbrl_refit_workspace_bytes(H, a, K), self.device)
        self._traj_ws = _workspace(("traj", str(self.device)),
                                   lib.mbrl_trajectory_workspace_bytes(fused.ctypes_ref(prob.shape), H), self.device)

    def _sampler(self, it, mu, sigma):
        return fused.make_sampler(self.st["seed"], it, mu, sigma, self.st["lo"], self.st["hi"])

    def rollout(self, it, mu, sigma, n_offset, n_local, costs_out, events=None):
        H, a = self.st["H"], self.prob.mdesc["a"]
        if self._acts is None or self._acts.shape[1] != n_local:
            self._acts = torch.empty((H, n_local, a), dtype=torch.float32, device=self.device)
            self._drawn = None
        # proposal draw (unless the last update drew this shard already), then the rollout kernel
        # alone between the events (bench.py's roofline)
        if self._drawn != (it, n_offset, n_local):
            fused.sample_actions(self._sampler(it, mu, sigma), H, a, n_local, n_offset, self._acts)
        self._drawn = None
        if events is not None:
            events[0].record()
        fused.rollout(self.prob, self.s0, n_local, H, actions=self._acts, costs=costs_out)
        if events is not None:
            events[1].record()

    def all_gather(self, out_flat, local):
        import torch.distributed as dist
        if dist.get_backend() == "gloo":
            # host-staged for gloo (CPU rehearsals of the sharded path on a shared GPU); RCCL gathers
            # device memory directly
            host = torch.empty(out_flat.shape, dtype=out_flat.dtype)
            dist.all_gather_into_tensor(host, local.reshape(-1).cpu())
            out_flat.copy_(host)
        else:
            dist.all_gather_into_tensor(out_flat, local.reshape(-1))

    def update(self, it, mu, sigma, costs, K, returns_out, mu_out, sigma_out, draw_next, n_offset, n_local):
        """mbrl_cem_update: selection, refit and (draw_next) this rank's proposals of iteration it + 1 in
        one launch, bit-identical to select + refit + sample_actions; None where it does not apply."""
        if not self._fused_update:
            return None
        H, a = self.st["H"], self.prob.mdesc["a"]
        nxt = self._acts if (draw_next and self._acts is not None and self._acts.shape[1] == n_local) else None
        if costs.stride(-1) != 1 or not costs.is_contiguous():
            costs = costs.contiguous()
        el = fused.cem_update(costs, K, self._sampler(it, mu, sigma), H, a, self.st["alpha"], mu_out, sigma_out,
                              returns_out=returns_out, next_actions=nxt, draw_offset=n_offset)
        if el is None:
            self._fused_update = False
            return None
        self._drawn = (it + 1, n_offset, n_local) if nxt is not None else None
        return el

    def select(self, costs, K, returns_out):
        return fused.select(costs, K, returns_out=returns_out, workspace=self._sel_ws)

    def refit(self, it, mu, sigma, elites, mu_out, sigma_out):
        fused.refit(self._sampler(it, mu, sigma), self.st["H"], self.prob.mdesc["a"], elites, self.st["alpha"],
                    mu_out, sigma_out, workspace=self._refit_ws)

    def trajectory(self, actions):
        return fused.trajectory(self.prob, self.s0, actions, self.st["H"], workspace=self._traj_ws)


# RCCL process groups run the sharded plan as ONE C call per plan (mbrl_cem_plan_sharded: the
# all-gather is a step on the plan's stream); False, or a gloo group, runs cem_sharded_protocol's
# per-iteration Python loop (the same plan bit for bit)
SHARDED_NATIVE = True
_COMMS = {}


def _rccl_comm(dev, world, rank):
    """The library's RCCL communicator for this process group (created once, collectively: rank 0's
    unique id is broadcast through torch.distributed, then every rank joins)."""
    import ctypes
    import torch.distributed as dist
    key = (str(dev), world, rank, id(dist.distributed_c10d._get_default_group()))
    comm = _COMMS.get(key)
    if comm is None:
        lib = _lib.load()
        obj = [None]
        if rank == 0:
            buf = ctypes.create_string_buffer(_lib.MBRL_COMM_ID_BYTES)
            _lib.check(lib.mbrl_comm_unique_id(buf), "mbrl_comm_unique_id")
            obj[0] = buf.raw
        dist.broadcast_object_list(obj, src=0)
        comm = ctypes.c_void_p()
        rc = lib.mbrl_comm_init(ctypes.c_char_p(obj[0]), world, rank, ctypes.byref(comm))
        # every rank learns whether every rank joined: if one could not, all of them take the
        # per-iteration protocol over torch.distributed instead (the same plan, bit for bit)
        ok = torch.tensor([1 if rc == 0 else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            if rc == 0:
                lib.mbrl_comm_destroy(comm)
            msg = lib.mbrl_last_error() if rc else b"another rank"
            warnings.warn(f"mbrl_amd: RCCL communicator unavailable ({msg.decode(errors='replace')}); "
                          "sharded plans use the torch.distributed protocol")
            comm = False
        _COMMS[key] = comm
    return comm


_OWN_COMM = object()


def _cem_sharded_native(prob, s0, st, world, rank, comm=_OWN_COMM):
    """mbrl_cem_plan_sharded: this rank's shard of the plan, every iteration's all-gather included, in
    one C-ABI call on the current stream (the result is the single-GPU plan's, on every rank).
    comm: the library's RCCL communicator for the default group (default), or None under
    _lib.option("shard_emulate", 1 or 2), where the call fills every rank's slot itself (tests, timing).
    s0 on the host with neither records nor device outputs asked for: the plan reads s0 from and writes
    its outputs to mapped host staging (as _cem_plan_host); the call returns after the plan completed
    (it synchronises once for the peers' status words when world > 1), so no copy launch follows it.
    A failure on any rank raises RuntimeError on every rank (MBRL_EPEER on the healthy ones); the
    communicator stays usable."""
    lib = _lib.load()
    dev = prob.device
    md = prob.mdesc
    N, K, H, I = st["N"], st["K"], st["H"], st["I"]
    a, s, E = md["a"], md["s"], md["E"]
    pkey = ("sharded", world, N, H, K, I, st["alpha"], st["lo"], st["hi"], st["init_std"],
            int(st["seed"]) & 0xFFFFFFFFFFFFFFFF, lib.mbrl_get_option(_lib.OPTIONS["shard_emulate"]))
    hit = prob.plan_cache.get(pkey)
    if hit is None:
        params = _lib.CemParams(N, H, K, I, st["alpha"], st["lo"], st["hi"], 0.0, st["init_std"], 0, pkey[10])
        need = lib.mbrl_cem_plan_sharded_workspace_bytes(fused.ctypes_ref(prob.shape), fused.ctypes_ref(params), world)
        if need == 0:
            raise ValueError(f"num_candidates {N} must divide evenly over {world} ranks")
        if len(prob.plan_cache) > 64:
            prob.plan_cache.clear()
        hit = prob.plan_cache[pkey] = (params, fused.ctypes_ref(params), need)
    params, pref, need = hit
    ws = _workspace(("cem_sharded", str(dev)), need, dev)
    if comm is _OWN_COMM:
        comm = _rccl_comm(dev, world, rank)
    rec = st["record"]
    staged = HOST_STAGING and not st["keep"] and not rec and not s0.is_cuda
    if staged:
        stage = _staging(dev, H * (s + 3 * a) + s)
        arr = stage.array
        o_s0 = H * (s + 3 * a)
        x = s0.detach() if s0.requires_grad else s0
        arr[o_s0:o_s0 + s] = x.numpy().reshape(-1) if x.dtype == torch.float32 else x.reshape(-1).to(torch.float32).numpy()
        o_act, o_mu, o_sg = H * s, H * (s + a), H * (s + 2 * a)
        at = stage.cached_at((H, s, a), (o_s0, o_mu, o_sg, o_act, 0))
        p_s0, p_mu, p_sg, p_act, p_st = at
    else:
        s0 = s0.to(device=dev, dtype=torch.float32).contiguous()
        buf = torch.empty(H * (s + 3 * a), dtype=torch.float32, device=dev)
        both = buf[:H * (s + a)]
        states, actions = both[:H * s].view(H, s), both[H * s:].view(H, a)
        mu, sigma = buf[H * (s + a):H * (s + 2 * a)].view(H, a), buf[H * (s + 2 * a):].view(H, a)
        p_s0, p_mu, p_sg, p_act, p_st = _lib.ptr(s0), _lib.ptr(mu), _lib.ptr(sigma), _lib.ptr(actions), _lib.ptr(states)
    cost_hist = torch.empty((I, E, N), dtype=torch.float32, device=dev) if rec else None
    ret_hist = torch.empty((I, N), dtype=torch.float32, device=dev) if rec else None
    elite_hist = torch.empty((I, K), dtype=torch.int64, device=dev) if rec else None
    pev = st.get("plan_events")
    if pev is not None:
        pev[0].record()
    rc = lib.mbrl_cem_plan_sharded(*prob.refs, p_s0, pref, comm, world, rank, p_mu, p_sg, p_act, p_st,
                                   _lib.ptr(cost_hist), _lib.ptr(ret_hist), _lib.ptr(elite_hist), _events(st, I),
                                   _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev))
    if pev is not None and rc == _lib.MBRL_OK:
        pev[1].record()
    # a failure after the argument checks still joined every all-gather of the plan, and every rank
    # learns of it (include/mbrl_cem.h): the communicator stays in step with the other ranks and is kept
    _lib.check(rc, "mbrl_cem_plan_sharded")
    if staged:
        if world == 1:     # (with peers the call has synchronised already)
            torch.cuda.current_stream(dev).synchronize()
        x = arr[:o_s0].copy()
        return dict(states=torch.from_numpy(x[:o_act].reshape(H, s)), actions=torch.from_numpy(x[o_act:o_mu].reshape(H, a)),
                    mu=torch.from_numpy(x[o_mu:o_sg].reshape(H, a)), sigma=torch.from_numpy(x[o_sg:].reshape(H, a)),
                    _host=True)
    out = dict(states=states, actions=actions, mu=mu, sigma=sigma, _both=both)
    if rec:
        out.update(costs=cost_hist, returns=ret_hist, elites=elite_hist)
    return out


def _cem_fused_sharded(prob, s0, st, world):
    import torch.distributed as dist
    if SHARDED_NATIVE and dist.get_backend() == "nccl" and _rccl_comm(prob.device, world, dist.get_rank()):
        return _cem_sharded_native(prob, s0, st, world, dist.get_rank())
    st = dict(st, E=prob.mdesc["E"], a=prob.mdesc["a"])
    return cem_sharded_protocol(_FusedShardOps(prob, s0.to(device=prob.device, dtype=torch.float32).contiguous(), st),
                                st, world, dist.get_rank())


def _cem_generic(model, cost, s0, st, a, dev):
    """CEM with opaque callables: HIP proposal draw, the callables on device tensors, HIP select/refit."""
    N, K, H, I = st["N"], st["K"], st["H"], st["I"]
    mu = torch.zeros((H, a), dtype=torch.float32, device=dev)
    sigma = torch.full((H, a), st["init_std"], dtype=torch.float32, device=dev)
    mu_n, sigma_n = torch.empty_like(mu), torch.empty_like(sigma)
    acts = torch.empty((H, N, a), dtype=torch.float32, device=dev)
    hist = dict(costs=[], returns=[], elites=[])
    for it in range(I):
        sp = fused.make_sampler(st["seed"], it, mu, sigma, st["lo"], st["hi"])
        fused.sample_actions(sp, H, a, N, 0, acts)
        costs, _ = _generic_costs(model, cost, s0, acts, H, N)
        rets = torch.empty(N, dtype=torch.float32, device=dev)
        elites = fused.select(costs, K, returns_out=rets)
        fused.refit(sp, H, a, elites, st["alpha"], mu_n, sigma_n)
        mu, mu_n = mu_n, mu
        sigma, sigma_n = sigma_n, sigma
        if st["record"]:
            hist["costs"].append(costs.clone())
            hist["returns"].append(rets)
            hist["elites"].append(elites)
    actions = mu.clamp(st["lo"], st["hi"]).contiguous()
    _, states = _generic_costs(model, cost, s0, actions.view(H, 1, a), H, 1)
    out = dict(states=states[:, 0, :], actions=actions, mu=mu, sigma=sigma)
    if st["record"]:
        out.update({k: torch.stack(v) for k, v in hist.items()})
    return out
