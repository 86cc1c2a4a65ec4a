"""GradientDescentPlanner: /root/reference/src/mbrl/planners.py:28-137 on the GPU.

The reference optimises one action sequence [H, a] by Adam(lr=0.01) through the learned dynamics:
each iteration rolls the sequence out (H batch-1 model calls), sums the cost over (s_{t+1}, a_t),
back-propagates to the actions, steps, and stops once mean |Δa| < stop_condition. It returns the
H+1 states of the LAST rollout (computed before the last update) and the updated actions, as
lists of [1, s] / [1, a] tensors.

Recognised closures (the same introspection as the CEM path: GoalStateAgent's and RewardAgent's
wiring) run on the device:
  * a single model with the goal-state cost, or a reward-head model with RewardAgent's reward cost
    -> mbrl_gd_plan (csrc/gd.hip): one launch runs every iteration's rollout, backward pass, Adam
    step and stop test; the host waits once per plan. GradientDescentPlanner.plan_batch runs B
    such plans (parallel environments) in shared launches (mbrl_gd_plan_batch);
  * ensembles -> a device restatement as differentiable torch ops: the MLP,
    normalisers and cost rebuilt from the described nn.Linear weights and statistics; the
    forward + loss + backward of one iteration (a chain of H x (L + 1) batch-1 layers) is captured
    once in a HIP graph and replayed each iteration; the Adam step and the stop test stay eager,
    with one host read per iteration, like the reference's .numpy().
Unrecognised closures run the reference's loop on the callables as given.
"""
import torch

from . import _lib, fused


def _stats(norm, key, dev):
    t = norm[key]
    return None if t is None else t.detach().to(device=dev, dtype=torch.float32)


class _DeviceModel:
    """The described model as differentiable torch ops on `dev` (weights detached, no grad)."""

    def __init__(self, mdesc, cdesc, dev):
        self.s, self.a, self.L = mdesc["s"], mdesc["a"], mdesc["L"]
        self.reward = bool(mdesc.get("reward"))
        self.members = [[(lin.weight.detach().to(dev, torch.float32), lin.bias.detach().to(dev, torch.float32))
                         for lin in lins] for lins in mdesc["members"]]
        n = mdesc["norm"]
        self.ns, self.us, self.na = n["normalize_state"], n["unnormalize_state"], n["normalize_action"]
        self.ur = n["unnormalize_reward"]
        self.om, self.os = _stats(n, "obs_mean", dev), _stats(n, "obs_std", dev)
        self.am, self.as_ = _stats(n, "act_mean", dev), _stats(n, "act_std", dev)
        self.rm, self.rs = _stats(n, "rew_mean", dev), _stats(n, "rew_std", dev)
        self.cdesc = cdesc
        if not self.reward:
            self.cw = cdesc["weights"].to(dev)
            self.goal = cdesc["goal"].to(dev)

    def _heads(self, s, a):
        """models.py:13-29 / 143-163 up to the output layer (mean over ensemble members)."""
        if self.na:
            a = (a - self.am) / self.as_
        if self.ns:
            s = (s - self.om) / self.os
        x0 = torch.cat([s, a], dim=1)
        outs = []
        for layers in self.members:
            x = x0
            for w, b in layers[:self.L]:
                x = torch.relu(torch.nn.functional.linear(x, w, b))
            if self.reward:
                (ws, bs), (wr, br) = layers[self.L], layers[self.L + 1]
                outs.append((torch.nn.functional.linear(x, ws, bs), torch.nn.functional.linear(x, wr, br)))
            else:
                w, b = layers[self.L]
                outs.append((torch.nn.functional.linear(x, w, b), None))
        if len(outs) == 1:
            return outs[0]
        return torch.stack([o[0] for o in outs]).mean(0), None

    def step(self, s, a):
        out, _ = self._heads(s, a)
        return out * self.os + self.om if self.us else out

    def cost(self, S, A):
        """Per-step cost on (s_{t+1}, a_t): goal-state (agents.py:182-183) or the reward head."""
        if self.reward:
            _, r = self._heads(S, A)
            return r * self.rs + self.rm if self.ur else r
        c = self.cdesc
        x = S - self.goal
        sc = torch.sum(torch.sqrt((x * self.cw) ** 2 + c["alpha_state"] ** 2) - c["alpha_state"], dim=-1)
        ac = (c["alpha_action"] ** 2) * torch.mean(torch.cosh(A / c["alpha_action"]) - 1, dim=-1)
        return sc + ac


class _Iteration:
    """One GD iteration's rollout + loss + backward for a fixed action leaf, as a replayable graph."""

    def __init__(self, dm, s0, actions, H, use_graph):
        self.dm, self.s0, self.actions, self.H = dm, s0, actions, H
        self.states = torch.zeros((H + 1, s0.shape[-1]), dtype=torch.float32, device=s0.device)
        self.graph = None
        if use_graph:
            try:
                self._capture()
            except RuntimeError:
                self.graph = None
                actions.grad = None

    def _body(self):
        rows = [self.s0.view(1, -1)]
        for i in range(self.H):                           # planners.py:123-124
            rows.append(self.dm.step(rows[-1], self.actions[i:i + 1]))
        st = torch.cat(rows)
        loss = torch.sum(self.dm.cost(st[1:], self.actions))  # planners.py:126
        loss.backward()
        with torch.no_grad():
            self.states.copy_(st)

    def _capture(self):
        dev = self.s0.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.grad = self.actions.grad
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()
        self.grad = self.actions.grad

    def run(self):
        if self.graph is None:
            self.actions.grad = None
            self._body()
            return
        self.actions.grad = self.grad
        self.grad.zero_()
        self.graph.replay()


def fused_supported(mdesc, cdesc, dev):
    want = _lib.MBRL_COST_MODEL_REWARD if mdesc.get("reward") else _lib.MBRL_COST_GOAL_STATE
    return dev.type == "cuda" and mdesc["E"] == 1 and cdesc is not None and cdesc["kind"] == want


def plan_fused(initial_state, mdesc, cdesc, action_list, horizon, num_iterations, stop_condition, dev, lr=0.01):
    """mbrl_gd_plan: the whole optimisation in one launch (csrc/gd.hip). Returns (states [H+1, s],
    actions [H, a], iterations run) on `dev`."""
    lib = _lib.load()
    prob = fused.device_problem(mdesc, cdesc, dev)
    H = int(horizon)
    s0 = initial_state.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    actions = torch.cat([a.reshape(1, -1) for a in action_list], 0).to(device=dev, dtype=torch.float32).contiguous()
    states = torch.empty((H + 1, mdesc["s"]), dtype=torch.float32, device=dev)
    iters = torch.zeros(1, dtype=torch.int32, device=dev)
    need = lib.mbrl_gd_workspace_bytes(fused.ctypes_ref(prob.shape), H)
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.mbrl_gd_plan(fused.ctypes_ref(prob.shape), _lib.ptr(prob.packed), fused.ctypes_ref(prob.norm),
                                fused.ctypes_ref(prob.cost), _lib.ptr(s0), _lib.ptr(actions), H, int(num_iterations),
                                float(stop_condition), float(lr), _lib.ptr(states), _lib.ptr(iters), _lib.ptr(ws),
                                need, _lib.stream_handle(dev)), "mbrl_gd_plan")
    return states, actions, iters


def plan_fused_batch(initial_states, mdesc, cdesc, actions, horizon, num_iterations, stop_condition, dev, lr=0.01):
    """mbrl_gd_plan_batch: B plans (initial_states [B, s], initial actions [B, H, a]) in shared
    launches, each exactly plan_fused's. Returns (states [B, H+1, s], actions [B, H, a], iterations [B])."""
    lib = _lib.load()
    prob = fused.device_problem(mdesc, cdesc, dev)
    H, B = int(horizon), int(initial_states.shape[0])
    s0 = initial_states.to(device=dev, dtype=torch.float32).reshape(B, -1).contiguous()
    acts = actions.to(device=dev, dtype=torch.float32).reshape(B, H, -1).contiguous().clone()
    states = torch.empty((B, H + 1, mdesc["s"]), dtype=torch.float32, device=dev)
    iters = torch.zeros(B, dtype=torch.int32, device=dev)
    need = lib.mbrl_gd_batch_workspace_bytes(fused.ctypes_ref(prob.shape), H, B)
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.mbrl_gd_plan_batch(fused.ctypes_ref(prob.shape), _lib.ptr(prob.packed), fused.ctypes_ref(prob.norm),
                                      fused.ctypes_ref(prob.cost), _lib.ptr(s0), _lib.ptr(acts), B, H,
                                      int(num_iterations), float(stop_condition), float(lr), _lib.ptr(states),
                                      _lib.ptr(iters), _lib.ptr(ws), need, _lib.stream_handle(dev)),
               "mbrl_gd_plan_batch")
    return states, acts, iters


def plan_device(initial_state, mdesc, cdesc, action_list, horizon, num_iterations, stop_condition, dev,
                use_graph=True, use_fused=True):
    """The reference's _optimize_trajectory (planners.py:103-137) on `dev` for described closures."""
    if use_fused and fused_supported(mdesc, cdesc, dev):
        states, actions, _ = plan_fused(initial_state, mdesc, cdesc, action_list, horizon, num_iterations,
                                        stop_condition, dev)
        return states, actions
    dm = _DeviceModel(mdesc, cdesc, dev)
    H = int(horizon)
    s0 = initial_state.to(device=dev, dtype=torch.float32).reshape(-1)
    if int(num_iterations) <= 0:
        # planners.py:115-135 with no iteration: the zero states tensor with s0 in row 0, and the
        # initial actions
        states = torch.zeros((H + 1, s0.shape[-1]), dtype=torch.float32, device=dev)
        states[0] = s0
        actions = torch.cat([a.reshape(1, -1) for a in action_list], 0).to(device=dev, dtype=torch.float32)
        return states, actions
    actions = torch.cat([a.reshape(1, -1) for a in action_list], 0).to(device=dev, dtype=torch.float32)
    actions = actions.detach().clone().requires_grad_(True)
    opt = torch.optim.Adam([actions], lr=0.01)
    it = _Iteration(dm, s0, actions, H, use_graph and dev.type == "cuda")
    for _ in range(num_iterations):
        opt.zero_grad(set_to_none=False)
        it.run()
        old = actions.detach().clone()
        opt.step()
        change = torch.mean(torch.abs(old - actions)).item()
        if change < stop_condition:
            break
    return it.states.detach(), actions.detach()


def plan_generic(initial_state, model, cost, sample_action, horizon, initial_trajectory, num_iterations,
                 stop_condition):
    """planners.py:59-137 with the callables as given (their own device)."""
    if initial_trajectory is None:
        state_list = [initial_state.unsqueeze(dim=0)]
        action_list = list(sample_action(batch_size=horizon).split(1, dim=0))
        for i in range(horizon):
            state_list.append(model(state_list[-1], action_list[i]))
    else:
        action_list = initial_trajectory[1]
    states = torch.zeros((horizon + 1, initial_state.shape[-1]))
    states[0] = initial_state
    actions = torch.cat(action_list, dim=0)
    actions.requires_grad = True
    opt = torch.optim.Adam([actions], lr=0.01)
    for _ in range(num_iterations):
        opt.zero_grad()
        for i in range(horizon):
            states[i + 1] = model(states[i:i + 1], actions[i:i + 1])
        loss = torch.sum(cost(states[1:], actions))
        loss.backward(retain_graph=True)
        old = actions.clone().detach()
        opt.step()
        if torch.mean(torch.abs(old - actions)).detach().numpy() < stop_condition:
            break
    return states.detach(), actions.detach()


def describe(model, cost, dev):
    """Recognised and semantically checked closures (fused.describe), else (None, None)."""
    return fused.describe(model, cost, dev)
