"""Parallel environment rollouts feeding one GPU planner service.

Restates /root/reference/src/mbrl/parallel.py:14-52: `get_rollouts_parallel(env_name, task_name,
flat_obs, num_rollouts, get_rollouts_kwargs, num_workers)` collects `num_rollouts` rollouts from
worker processes, each loading its environment with `EnvWrapper.load` and running
`env.get_rollout(**get_rollouts_kwargs)` (or `record_rollout` with an indexed `mp4path`), and
returns them in request order.

The difference is where planning happens. The reference pickles the policy (and so the model and
the planner) into every worker, so each worker plans on its own: one GPU context and one small
plan per worker. Here, when `get_action` is an MPC policy's (an `agents.MPCPolicy` or anything with
its planner/model/cost/sample_action/horizon attributes), the workers only step their
environments. Each step's action request goes to the parent process, which serves every worker
from one GPU:
  * lockstep: it waits until every running worker has asked for an action;
  * it orders the requests by rollout index;
  * it answers them all with one `planner.plan_batch` call (CEMPlanner: mbrl_cem_plan_batch, one
    rollout launch over B·N candidates per CEM iteration);
  * planners without plan_batch get one `get_action` per request on a per-rollout copy of the
    policy, so each rollout keeps its own warm start (agents.py:37-56).
Rollouts are statically assigned (rollout i runs on worker i mod num_workers). So the batches, and
with a fixed `seed` the actions, are the same on every run. Workers never touch the GPU. Any
`get_action` that is not a policy is pickled into the workers and called there, as the reference
does.

Workers are started with the "spawn" method (fresh interpreters, no inherited GPU state).
Rollouts travel back as NumPy arrays and are rebuilt as tensors, which avoids torch's
shared-memory file-descriptor passing (the reason the reference switches to the file_system
sharing strategy, parallel.py:1-2).
"""
import copy
import os
import queue
import traceback
from collections import namedtuple

import numpy as np
import torch
import torch.multiprocessing as multiprocessing

from .data import Rollout

CollectionRequest = namedtuple("CollectionRequest",
                               ["env_name", "task_name", "flat_obs", "get_rollouts_kwargs", "index"])

DEFAULT_NUM_WORKERS = int(os.environ.get("NUM_WORKERS", 2))
_POLICY_ATTRS = ("planner", "model", "cost", "sample_action", "horizon")


def _policy_of(get_action):
    """The MPC policy behind a bound get_action, or None."""
    pol = getattr(get_action, "__self__", None)
    if pol is not None and all(hasattr(pol, k) for k in _POLICY_ATTRS):
        return pol
    return None


def get_rollouts_parallel(env_name, task_name, flat_obs, num_rollouts, get_rollouts_kwargs,
                          num_workers=DEFAULT_NUM_WORKERS, env_factory=None, on_batch=None, timeout=600.0):
    """parallel.py:20-38. `env_factory(env_name=, task_name=, flat_obs=, index=)` replaces
    EnvWrapper.load (e.g. for environments built outside dm_control.suite). `on_batch(indices,
    observations, actions)` is called after each served planning batch. `timeout` bounds the wait
    for any one worker message, in seconds."""
    num_rollouts = int(num_rollouts)
    if num_rollouts <= 0:
        return []
    num_workers = max(1, min(int(num_workers), num_rollouts))
    kwargs = dict(get_rollouts_kwargs)
    policy = _policy_of(kwargs.get("get_action"))
    if policy is not None:
        kwargs.pop("get_action")
    ctx = multiprocessing.get_context("spawn")
    req_q = ctx.Queue()
    pipes = [ctx.Pipe(duplex=False) for _ in range(num_workers)]
    procs = []
    try:
        for w in range(num_workers):
            p = ctx.Process(target=_worker, daemon=True,
                            args=(w, list(range(w, num_rollouts, num_workers)), env_name, task_name, flat_obs,
                                  kwargs, policy is not None, env_factory, req_q, pipes[w][0]))
            p.start()
            procs.append(p)
        return _serve(policy, procs, req_q, [s for _, s in pipes], num_rollouts, on_batch, timeout)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
            p.join(timeout=10)
        req_q.close()
        for r, s in pipes:
            r.close()
            s.close()


def collect_from_env(request, env_factory=None):
    """parallel.py:41-52: load the environment and run one rollout (recorded when mp4path is given)."""
    if env_factory is None:
        from .env_wrappers import EnvWrapper
        env = EnvWrapper.load(env_name=request.env_name, task_name=request.task_name, flat_obs=request.flat_obs)
    else:
        env = env_factory(env_name=request.env_name, task_name=request.task_name, flat_obs=request.flat_obs,
                          index=request.index)
    kwargs = dict(request.get_rollouts_kwargs)
    if "mp4path" in kwargs:
        kwargs["mp4path"] = "{}_{}".format(kwargs["mp4path"], request.index)
        return env.record_rollout(**kwargs)
    return env.get_rollout(**kwargs)


# ----------------------------------------------------------------------------------- worker side

class _ServedAction:
    """get_action inside a worker: send (timestep, state, observation) to the planner service and
    wait for its action."""

    def __init__(self, wid, index, req_q, conn):
        self.wid, self.index, self.req_q, self.conn = wid, index, req_q, conn

    def __call__(self, state_and_obs):
        self.req_q.put(("act", self.wid, self.index,
                        (int(state_and_obs["timestep"]), _to_numpy(state_and_obs["state"]),
                         _to_numpy(state_and_obs["observation"]))))
        return torch.from_numpy(self.conn.recv())


def _worker(wid, indices, env_name, task_name, flat_obs, kwargs, served, env_factory, req_q, conn):
    try:
        for i in indices:
            kw = dict(kwargs)
            if served:
                kw["get_action"] = _ServedAction(wid, i, req_q, conn)
            rollout = collect_from_env(CollectionRequest(env_name, task_name, flat_obs, kw, i), env_factory)
            req_q.put(("done", wid, i, _pack_rollout(rollout)))
        req_q.put(("exit", wid, None, None))
    except BaseException as exc:  # report, then end: the parent raises
        req_q.put(("error", wid, None, "{}: {}\n{}".format(type(exc).__name__, exc, traceback.format_exc())))


def _to_numpy(x):
    if isinstance(x, dict):
        return {k: _to_numpy(v) for k, v in x.items()}
    if torch.is_tensor(x):
        return x.detach().cpu().numpy()
    return None if x is None else np.asarray(x)


def _to_torch(x):
    if isinstance(x, dict):
        return {k: _to_torch(v) for k, v in x.items()}
    return None if x is None else torch.from_numpy(np.asarray(x))


def _pack_rollout(r):
    d = dict(states=[_to_numpy(x) for x in r.states], observations=[_to_numpy(x) for x in r.observations],
             actions=[_to_numpy(x) for x in r.actions[:-1]], rewards=[_to_numpy(x) for x in r.rewards[1:]])
    if hasattr(r, "frames"):
        d["frames"] = r.frames
    return d


def _unpack_rollout(d):
    r = Rollout(states=[_to_torch(x) for x in d["states"]], observations=[_to_torch(x) for x in d["observations"]],
                actions=[_to_torch(x) for x in d["actions"]], rewards=[_to_torch(x) for x in d["rewards"]])
    if "frames" in d:
        r.frames = d["frames"]
    return r


# ----------------------------------------------------------------------------------- service side

def _serve(policy, procs, req_q, conns, num_rollouts, on_batch, timeout):
    active = set(range(len(procs)))
    pending = {}                  # worker -> (rollout index, timestep, state, observation)
    results = [None] * num_rollouts
    copies = {}                   # rollout index -> its policy copy (planners without plan_batch)
    last = {}                     # rollout index -> its previous plan (warm-starting planners)
    waited = 0.0
    while active:
        if pending and len(pending) == len(active):
            _answer(policy, pending, conns, copies, on_batch, last)
            pending.clear()
            continue
        try:
            kind, wid, i, payload = req_q.get(timeout=1.0)
        except queue.Empty:
            dead = [w for w in active if not procs[w].is_alive()]
            if dead:
                raise RuntimeError("rollout worker {} died (exit code {})".format(dead[0], procs[dead[0]].exitcode))
            waited += 1.0
            if waited >= timeout:
                raise RuntimeError("rollout workers sent nothing for {:.0f} s".format(waited))
            continue
        waited = 0.0
        if kind == "act":
            if policy is None:
                raise RuntimeError("worker {} asked for an action but no policy is served".format(wid))
            pending[wid] = (i,) + tuple(payload)
        elif kind == "done":
            results[i] = _unpack_rollout(payload)
        elif kind == "exit":
            active.discard(wid)
        else:
            raise RuntimeError("rollout worker {} failed:\n{}".format(wid, payload))
    return results


def _answer(policy, pending, conns, copies, on_batch, last):
    """One planning round: every waiting worker's request, ordered by rollout index."""
    order = sorted(pending, key=lambda w: pending[w][0])
    indices = [pending[w][0] for w in order]
    obs = [torch.from_numpy(np.asarray(pending[w][3])) for w in order]
    plan_batch = getattr(policy.planner, "plan_batch", None)
    if plan_batch is not None:
        kw = dict(getattr(policy, "plan_kwargs", {}))
        warm = getattr(policy.planner, "warm_starts", False)
        if warm:
            # what each rollout's own MPCPolicy.get_action would pass (agents.py:40-55): nothing at
            # timestep 0, else (previous states[1:], previous actions[0:]) of the same rollout
            inits = []
            for w in order:
                i, t = pending[w][0], pending[w][1]
                prev = None if t == 0 else last.get(i)
                inits.append(None if prev is None else (prev[0][1:], prev[1][0:]))
            kw["initial_trajectories"] = inits
        states, actions = plan_batch(torch.stack(obs), policy.model, policy.cost, policy.sample_action,
                                     policy.horizon, **kw)
        if warm:
            for b, i in enumerate(indices):
                last[i] = (list(states[b].split(1, 0)), list(actions[b].split(1, 0)))
        acts = [actions[b][0].flatten().detach().cpu() for b in range(len(order))]
    else:
        acts = []
        for w, o in zip(order, obs):
            i, t, state = pending[w][:3]
            pol = copies.get(i)
            if pol is None:
                pol = copies[i] = copy.copy(policy)
            acts.append(pol.get_action(dict(timestep=t, state=_to_torch(state), observation=o)).detach().cpu())
    for w, a in zip(order, acts):
        conns[w].send(a.numpy())
    if on_batch is not None:
        on_batch(indices, torch.stack(obs), torch.stack(acts))
