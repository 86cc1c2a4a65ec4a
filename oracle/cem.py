"""Oracle (TEST INFRASTRUCTURE ONLY): CPU restatement of the reference planning hot path + CEM refit.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline / parity legs import this.
The shipped planner (`mujoco-mbrl_amd/mbrl_amd`) never calls it and fails loudly without its HIP
library; this module is the checker it is compared against.

Pinning: `tests/golden/make_golden.py` runs the reference's own `RandomShootingPlanner`
(`/root/reference/src/mbrl/planners.py:140-216`), `models.Model` / `DynamicsModel`
(`models.py:8-29,96-110`), `SmoothAbsLoss` / `CoshLoss` (`models.py:244-272`) and
`TransitionsDataset.normalize_field` (`data.py:255-260`) in this container and commits their outputs
under `tests/golden/`; `tests/test_oracle_golden.py` checks this restatement against them.

Reference semantics restated here (file:line in /root/reference/src/mbrl):
  * dynamics step  -- DynamicsModel.forward (models.py:13-29): normalize_action(a), normalize_state(s),
    x = cat([s, a], 1) (state first), Linear-ReLU-...-Linear (models.py:106-110, generalised to L hidden
    layers with the same pattern), unnormalize_state(out). Absolute next state, not a delta.
  * normalisation  -- data.py:255-260: (x - mean) / std and y * std + mean, applied as written.
  * goal-state cost -- agents.py:182-183 state_action_cost = SmoothAbsLoss(s) + CoshLoss(a) on the
    (s_{t+1}, a_t) pair (planners.py:210).
  * rollout        -- planners.py:199-210: time-major [H, N, .]; per-candidate return = sum over t.
    The sum over t is sequential in float32 (t = 0 first): SURVEY.md §8c fixes this order because
    torch's .sum(0) is not bitwise sequential.
  * random shooting -- planners.py:176-187: np.argmin over the returns (first index wins ties,
    and np.argmin returns the first NaN if any).
  * CEM (not in the reference): stable argsort elites, population variance,
    alpha-smoothed refit; the elite sums run in a canonical chunked order (below) that the device
    kernel follows exactly, so mu / sigma come out bit-identical given identical elite sets.
"""
import hashlib
import numpy as np

from .philox import cem_actions

F32 = np.float32

# ---------------------------------------------------------------------------------------------
# Synthetic inputs. Seed = 1000 + config id.
# ---------------------------------------------------------------------------------------------
CONFIGS = {
    # id: name, obs dim, action dim, hidden width, hidden layers, candidates, horizon, ensemble, planner
    1: dict(name="cartpole-swingup-rs", s=5, a=1, W=256, L=2, N=128, H=12, E=1, planner="rs"),
    2: dict(name="cartpole-swingup-cem", s=5, a=1, W=256, L=2, N=1024, H=20, E=1, planner="cem"),
    3: dict(name="cheetah-run-cem", s=17, a=6, W=512, L=3, N=4096, H=30, E=1, planner="cem"),
    4: dict(name="walker-walk-cem", s=24, a=6, W=512, L=3, N=16384, H=30, E=1, planner="cem"),
    5: dict(name="humanoid-stand-cem-ens5", s=67, a=21, W=512, L=3, N=32768, H=50, E=5, planner="cem"),
    # reward-head variant: ModelWithReward's 2-layer trunk, RewardAgent cost
    6: dict(name="cheetah-run-reward-cem", s=17, a=6, W=512, L=2, N=4096, H=30, E=1, planner="cem", reward=True),
}

CEM_DEFAULTS = dict(num_iterations=5, elite_frac=0.1, alpha=0.1, lo=-1.0, hi=1.0)
ELITE_CHUNK = 32          # canonical chunk length of the elite sums (csrc: MBRL_ELITE_CHUNK)
SMOOTH_ABS_ALPHA = 0.4    # models.py:249 default
COSH_ALPHA = 0.25         # models.py:267 default


def synth_model(seed, s, a, W, L, E=1):
    """E members of an L-hidden-layer MLP [(W [out,in], b [out]) per layer], nn.Linear init law."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dims = [s + a] + [W] * L + [s]
    members = []
    for _ in range(E):
        layers = []
        for fan_in, fan_out in zip(dims[:-1], dims[1:]):
            bound = 1.0 / np.sqrt(fan_in)
            w = rng.uniform(-bound, bound, size=(fan_out, fan_in)).astype(F32)
            b = rng.uniform(-bound, bound, size=(fan_out,)).astype(F32)
            layers.append((w, b))
        members.append(layers)
    return members


def synth_reward_model(seed, s, a, W, L, E=1):
    """E ModelWithReward members (models.py:125-141, trunk generalised to L layers): trunk layers,
    state head [s, W] and reward head [1, W] drawn in that order with the nn.Linear law. The head is
    stored combined: the last layer is [s + 1, W] (state rows, then the reward row)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    dims = [s + a] + [W] * L
    members = []
    for _ in range(E):
        layers = []
        for fan_in, fan_out in list(zip(dims[:-1], dims[1:])) + [(W, s), (W, 1)]:
            bound = 1.0 / np.sqrt(fan_in)
            w = rng.uniform(-bound, bound, size=(fan_out, fan_in)).astype(F32)
            b = rng.uniform(-bound, bound, size=(fan_out,)).astype(F32)
            layers.append((w, b))
        (ws, bs), (wr, br) = layers[-2], layers[-1]
        members.append(layers[:-2] + [(np.vstack([ws, wr]), np.concatenate([bs, br]))])
    return members


def synth_norm(seed, s, a):
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    return dict(
        obs_mean=rng.uniform(-0.5, 0.5, size=s).astype(F32),
        obs_std=rng.uniform(0.5, 2.0, size=s).astype(F32),
        act_mean=rng.uniform(-0.5, 0.5, size=a).astype(F32),
        act_std=rng.uniform(0.5, 2.0, size=a).astype(F32),
    )


def synth_state_goal(seed, s):
    rng = np.random.Generator(np.random.PCG64(seed + 2))
    s0 = rng.standard_normal(s).astype(F32)
    goal = rng.standard_normal(s).astype(F32)
    return s0, goal


def synth_problem(config_id, **overrides):
    """Everything a config needs: model members, normalisation, s0, goal-state cost, CEM seed."""
    cfg = dict(CONFIGS[config_id])
    cfg.update(overrides)
    seed = 1000 + config_id
    s, a = cfg["s"], cfg["a"]
    norm = synth_norm(seed, s, a)
    s0, goal = synth_state_goal(seed, s)
    if cfg.get("reward"):
        model = synth_reward_model(seed, s, a, cfg["W"], cfg["L"], cfg["E"])
        rr = np.random.Generator(np.random.PCG64(seed + 4))
        norm.update(rew_mean=rr.uniform(-0.5, 0.5, size=1).astype(F32), rew_std=rr.uniform(0.5, 2.0, size=1).astype(F32))
        cost = dict(kind="reward")
    else:
        model = synth_model(seed, s, a, cfg["W"], cfg["L"], cfg["E"])
        cost = dict(weights=np.ones(s, dtype=F32), goal=goal, alpha_state=SMOOTH_ABS_ALPHA,
                    alpha_action=COSH_ALPHA)
    return dict(cfg=cfg, seed=seed, rng_seed=seed + 3, model=model, norm=norm, s0=s0, cost=cost)


def weights_sha256(model):
    h = hashlib.sha256()
    for layers in model:
        for w, b in layers:
            h.update(np.ascontiguousarray(w, dtype=F32).tobytes())
            h.update(np.ascontiguousarray(b, dtype=F32).tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------------------------------------
# Model, cost, rollout
# ---------------------------------------------------------------------------------------------
def mlp_forward(layers, x):
    """Model._forward (models.py:106-110) with L hidden layers: nn.Linear is y = x W^T + b."""
    for w, b in layers[:-1]:
        x = np.maximum(x @ w.T + b, F32(0))
    w, b = layers[-1]
    return (x @ w.T + b).astype(F32)


def _model_out(layers, norm, s, a):
    """normalize_action, normalize_state, cat (state first), the MLP (models.py:13-29 / 143-163)."""
    if norm is not None:
        a = ((a - norm["act_mean"]) / norm["act_std"]).astype(F32)        # normalize_action first
        sn = ((s - norm["obs_mean"]) / norm["obs_std"]).astype(F32)       # then normalize_state
    else:
        sn = s
    x = np.concatenate([sn, a], axis=1).astype(F32)                        # state first
    return mlp_forward(layers, x)


def dynamics_step(layers, norm, s, a):
    """DynamicsModel.forward (models.py:13-29) with the GoalStateAgent normalisers (agents.py:219-230);
    for a reward-head model, the state head of ModelWithReward.forward (models.py:143-163)."""
    out = _model_out(layers, norm, s, a)[:, :s.shape[1]]
    if norm is not None:
        out = (out * norm["obs_std"] + norm["obs_mean"]).astype(F32)       # unnormalize_state
    return out


def reward_cost(layers, norm, s_next, a):
    """RewardAgent's cost (agents.py:353-362): compose(partial(model, ...), itemgetter(1)) evaluated on
    (s_{t+1}, a_t) (planners.py:210) = the reward head, unnormalised (models.py:157-158)."""
    r = _model_out(layers, norm, s_next, a)[:, s_next.shape[1]]
    if norm is not None and norm.get("rew_mean") is not None:
        r = (r * norm["rew_std"][0] + norm["rew_mean"][0]).astype(F32)      # unnormalize_reward
    return r.astype(F32)


def goal_state_cost(s, a, cost):
    """state_action_cost (agents.py:182-183) = SmoothAbsLoss(s) (models.py:255-259) + CoshLoss(a) (:271-272)."""
    al = F32(cost["alpha_state"])
    al2 = F32(cost["alpha_state"] ** 2)
    x = (s - cost["goal"]).astype(F32)
    sc = np.sum(np.sqrt(((x * cost["weights"]) ** 2 + al2).astype(F32)) - al, axis=-1, dtype=F32)
    aa = F32(cost["alpha_action"])
    aa2 = F32(cost["alpha_action"] ** 2)
    ac = aa2 * np.mean(np.cosh((a / aa).astype(F32)) - F32(1), axis=-1, dtype=F32)
    return (sc + ac).astype(F32)


def rollout(model, norm, cost, s0, actions, store_states=False):
    """planners.py:199-210 for every ensemble member.

    actions: float32 [H, N, a] (time-major, as the reference's action_list.view(H, N, a)).
    s0: [s] (broadcast, planners.py:204) or [N, s] (per-candidate start, used by forward tests).
    Returns costs [E, N] (sequential float32 sum over t) and, optionally, states [E, H, N, s].
    """
    H, N, _ = actions.shape
    E = len(model)
    costs = np.zeros((E, N), dtype=F32)
    states = [] if store_states else None
    for e, layers in enumerate(model):
        st = np.broadcast_to(np.asarray(s0, F32), (N, len(s0) if np.ndim(s0) == 1 else s0.shape[1])).copy()
        member_states = []
        total = np.zeros(N, dtype=F32)
        for t in range(H):
            st = dynamics_step(layers, norm, st, actions[t])
            c = reward_cost(layers, norm, st, actions[t]) if cost.get("kind") == "reward" \
                else goal_state_cost(st, actions[t], cost)
            total = (total + c).astype(F32)
            if store_states:
                member_states.append(st)
        costs[e] = total
        if store_states:
            states.append(np.stack(member_states))
    return (costs, np.stack(states)) if store_states else costs


def ensemble_returns(costs):
    """Deterministic expectation over members: (c_0 + c_1 + ... + c_{E-1}) / E, sequential in e."""
    acc = costs[0].copy()
    for e in range(1, costs.shape[0]):
        acc = (acc + costs[e]).astype(F32)
    if costs.shape[0] > 1:
        acc = (acc / F32(costs.shape[0])).astype(F32)
    return acc


# ---------------------------------------------------------------------------------------------
# Selection and refit
# ---------------------------------------------------------------------------------------------
def select_elites(returns, K):
    """elite = np.argsort(returns, kind="stable")[:K] (NaN last, -0.0 == +0.0), returned in ascending
    candidate-index order (the order the refit sums them in)."""
    order = np.argsort(np.asarray(returns, F32), kind="stable")[:K]
    return np.sort(order).astype(np.int64)


def rs_argmin(returns):
    """planners.py:184 np.argmin: first minimum; first NaN if any NaN is present."""
    return int(np.argmin(np.asarray(returns, F32)))


def chunked_sum(x, chunk=ELITE_CHUNK):
    """Canonical elite sum: sequential inside chunks of `chunk` rows, then sequential over chunks."""
    K = x.shape[0]
    tot = None
    for c0 in range(0, K, chunk):
        acc = x[c0].copy()
        for e in range(c0 + 1, min(c0 + chunk, K)):
            acc = (acc + x[e]).astype(F32)
        tot = acc if tot is None else (tot + acc).astype(F32)
    return tot


def refit(mu, sigma, elite_actions, alpha):
    """mu' = mean_elite(A), var' = mean_elite((A - mu')^2) (population);
    mu <- alpha*mu + (1-alpha)*mu';  sigma <- sqrt(alpha*sigma^2 + (1-alpha)*var').
    elite_actions: [K, H, a] in ascending candidate order."""
    K = F32(elite_actions.shape[0])
    a_ = F32(alpha)
    oma = F32(1) - a_
    mean = (chunked_sum(elite_actions) / K).astype(F32)
    d = (elite_actions - mean).astype(F32)
    var = (chunked_sum((d * d).astype(F32)) / K).astype(F32)
    mu_new = ((a_ * mu).astype(F32) + (oma * mean).astype(F32)).astype(F32)
    var_new = ((a_ * (sigma * sigma).astype(F32)).astype(F32) + (oma * var).astype(F32)).astype(F32)
    return mu_new, np.sqrt(var_new).astype(F32)


def cem_plan(problem, N=None, H=None, K=None, num_iterations=None, alpha=None, lo=None, hi=None,
             record=True):
    """Full CEM plan on the synthetic problem. Returns a dict of per-iteration
    records and the final (states [H, s], actions [H, a])."""
    cfg = problem["cfg"]
    N = N or cfg["N"]
    H = H or cfg["H"]
    I = num_iterations if num_iterations is not None else CEM_DEFAULTS["num_iterations"]
    K = K or max(1, int(N * CEM_DEFAULTS["elite_frac"]))
    alpha = CEM_DEFAULTS["alpha"] if alpha is None else alpha
    lo = CEM_DEFAULTS["lo"] if lo is None else lo
    hi = CEM_DEFAULTS["hi"] if hi is None else hi
    a = cfg["a"]
    mu = np.zeros((H, a), F32)
    sigma = np.full((H, a), F32((hi - lo) / 4.0), F32)
    out = dict(costs=[], returns=[], elites=[], mu=[], sigma=[])
    for it in range(I):
        A = cem_actions(mu, sigma, lo, hi, problem["rng_seed"], it, np.arange(N))
        costs = rollout(problem["model"], problem["norm"], problem["cost"], problem["s0"], A)
        ret = ensemble_returns(costs)
        elites = select_elites(ret, K)
        mu, sigma = refit(mu, sigma, np.ascontiguousarray(A[:, elites, :].transpose(1, 0, 2)), alpha)
        if record:
            out["costs"].append(costs)
            out["returns"].append(ret)
            out["elites"].append(elites)
            out["mu"].append(mu)
            out["sigma"].append(sigma)
    actions = np.clip(mu, F32(lo), F32(hi)).astype(F32)
    _, states = rollout(problem["model"], problem["norm"], problem["cost"], problem["s0"],
                        actions[:, None, :], store_states=True)
    out["final_actions"] = actions
    out["final_states"] = np.mean(states[:, :, 0, :], axis=0, dtype=F32) if len(problem["model"]) > 1 \
        else states[0, :, 0, :]
    return out


def rs_plan(problem, actions_flat, N, H):
    """RandomShootingPlanner._plan (planners.py:166-216) given the sampled time-major actions
    [N*H, a]. Returns (states [H, s], actions [H, a], costs [N], idx)."""
    a = actions_flat.shape[1]
    A = np.asarray(actions_flat, F32).reshape(H, N, a)
    costs, states = rollout(problem["model"], problem["norm"], problem["cost"], problem["s0"], A,
                            store_states=True)
    ret = ensemble_returns(costs)
    idx = rs_argmin(ret)
    return states[0, :, idx, :], A[:, idx, :], ret, idx
