"""Environment wrappers (mbrl_amd.env_wrappers, restating /root/reference/src/mbrl/env_wrappers.py)
driven by stand-in dm_env environments: dm_control/MuJoCo are not installable here,
so these check the wrapper logic (state features, goals, samplers' draw order, rollout assembly),
not physics."""
import contextlib
import functools

import numpy as np
import pytest
import torch

from mbrl_amd import env as menv
from mbrl_amd import env_wrappers as ew


class _Step:
    def __init__(self, obs, reward, last):
        self.observation = {"observations": obs}
        self.reward = reward
        self._last = last

    def last(self):
        return self._last


class _Named:
    def __init__(self, **tables):
        self.__dict__.update(tables)


class _Physics:
    """Stand-in physics: a state vector, the named tables and feature methods the wrappers read."""

    def __init__(self, nstate, ntouch=2):
        self._state = np.arange(nstate, dtype=np.float64) * 0.1
        self._ntouch = ntouch
        xpos = {"right_foot": np.array([0.1, 0.2, 0.0]), "left_foot": np.array([0.3, -0.2, 0.0]),
                "torso": np.array([0.2, 0.1, 1.2])}
        self.named = _Named(data=_Named(subtree_com={"torso": np.array([0.0, 0.0, 0.55])}, xpos=xpos,
                                        xmat={"head": np.array([0.5, -0.25, 0.0])},
                                        site_xpos={("grasp", "x"): 0.7, ("grasp", "z"): 0.9},
                                        geom_xpos={"target": np.array([0.4, -0.3, 0.0])}),
                            model=_Named(geom_pos={}))
        self.set_states = []

    def state(self):
        return self._state.copy()

    def set_state(self, s):
        self.set_states.append(np.asarray(s))

    @contextlib.contextmanager
    def reset_context(self):
        yield

    def speed(self):
        return 1.5

    def torso_upright(self):
        return 0.9

    def torso_height(self):
        return 1.1

    def horizontal_velocity(self):
        return 0.7

    def height(self):
        return 0.8

    def touch(self):
        return np.arange(self._ntouch, dtype=np.float64)

    def center_of_mass_position(self):
        return np.array([0.25, 0.05, 1.0])

    def center_of_mass_velocity(self):
        return np.array([0.1, -0.1, 0.0])

    def body_location(self, name):
        return np.array([0.3, 0.6, 0.0])

    def render(self, camera_id=0):
        return np.zeros((4, 4, 3), np.uint8)


class _Env:
    """dm_env-like: fixed observation width, reward = step index, episode ends after `length` steps."""

    def __init__(self, nstate, nobs, adim, length=1000):
        self.physics = _Physics(nstate, ntouch=5 if nobs == 37 else 2)   # manipulator: 5 touch sensors
        self._spec = menv.BoundedActionSpec(adim, -1.0, 1.0)
        self._nobs, self._length, self._t = nobs, length, 0
        self.actions = []

    def action_spec(self):
        return self._spec

    def observation_spec(self):
        return {"observations": (self._nobs,)}

    def reset(self):
        self._t = 0
        return _Step(np.zeros(self._nobs), None, False)

    def step(self, action):
        self.actions.append(np.asarray(action))
        self._t += 1
        return _Step(np.full(self._nobs, float(self._t)), float(self._t), self._t >= self._length)


# (class, physics state size, flat observation size, action dim)
DOMAINS = [(ew.Cheetah, 18, 17, 6), (ew.Walker, 18, 24, 6), (ew.Hopper, 14, 15, 4), (ew.Humanoid, 55, 67, 21),
           (ew.Cartpole, 4, 5, 1), (ew.Reacher, 4, 6, 2), (ew.PointMass, 4, 4, 2), (ew.Swimmer, 10, 10, 2),
           (ew.Manipulator, 22, 37, 5)]


def test_registry_mirrors_the_reference_lookup():
    assert ew.EnvWrapper.wrapper_class("point_mass") is ew.PointMass
    assert ew.EnvWrapper.wrapper_class("cheetah") is ew.Cheetah
    assert ew.EnvWrapper.wrapper_class("cartpole") is ew.Cartpole
    with pytest.raises(NameError, match="No wrapper for"):
        ew.EnvWrapper.wrapper_class("acrobot")
    try:
        import dm_control  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError, match="dm_control"):
            ew.EnvWrapper.load("cheetah", "run")


@pytest.mark.parametrize("cls,ns,no,ad", DOMAINS, ids=[d[0].__name__ for d in DOMAINS])
def test_state_features_and_goal_dims(cls, ns, no, ad):
    w = cls(_Env(ns, no, ad), env_name=cls.domain, task_name="t")
    state = w.get_state()
    assert state.shape == (cls.state_dim,) and state.dtype == torch.float32
    assert w.get_goal_weights().shape in ((cls.state_dim,), (cls.observation_dim,))
    if cls is not ew.Reacher:
        np.random.seed(0)
        assert w.set_goal().shape == (cls.state_dim,)
    try:
        g, wt = w.observation_goal()
    except NotImplementedError:
        return
    assert g.shape == wt.shape == (no,)


def test_state_features_values():
    ch = ew.Cheetah(_Env(18, 17, 6))
    s = ch.get_state().numpy()
    assert np.allclose(s[:17], np.arange(1, 18) * 0.1) and np.isclose(s[17], 1.5) and np.isclose(s[18], 0.55)
    wk = ew.Walker(_Env(18, 24, 6))
    assert np.allclose(wk.get_state().numpy()[-3:], [0.9, 1.1, 0.7])
    assert torch.equal(wk.set_goal()[-3:], torch.tensor([1.0, 1.3, 3.0]))
    hu = ew.Humanoid(_Env(55, 67, 21)).get_state().numpy()
    feet = np.array([0.2, 0.0, 0.0])
    assert np.isclose(hu[55], np.linalg.norm([0.25 - feet[0], 0.05 - feet[1]]))
    assert np.isclose(hu[56], np.linalg.norm([0.25 - 0.2, 0.05 - 0.1]))
    assert np.isclose(hu[57], np.linalg.norm(np.array([0.1, 1.2]) - np.array([0.0, 1.3])))
    assert np.allclose(hu[58:], [0.1, -0.1])


def test_samplers_keep_the_reference_draw_order():
    """The same global NumPy stream yields the same states as the reference's samplers."""
    np.random.seed(3)
    s = ew.Walker(_Env(18, 24, 6)).sample_state().numpy()
    np.random.seed(3)
    body = np.random.uniform(-0.1, 0.1)
    hip = np.random.uniform(-0.15, 0.15)
    rk, ra = np.random.uniform(-0.3, 0), np.random.uniform(-0.1, 0.1)
    lk, la = np.random.uniform(-0.3, 0), np.random.uniform(-0.1, 0.1)
    assert np.allclose(s[2:9], np.float32([body, hip, rk, ra, -hip, lk, la]))
    np.random.seed(7)
    c = ew.Cheetah(_Env(18, 17, 6)).sample_state().numpy()
    np.random.seed(7)
    z = np.random.uniform(-0.2, 0.2)
    ang = np.random.uniform(-3.14, 3.14) if z > 0.05 else (
        np.random.uniform(-3.14, -1.5) if np.random.uniform() < 0.72 else np.random.uniform(2.5, 3.14))
    joints = [np.random.uniform(lo, hi) for _, lo, hi in ew.Cheetah._JOINTS]
    vel = np.random.uniform(-3, 3, 9)
    assert np.allclose(c, np.float32([0, z, ang] + joints + list(vel)))


def test_sample_action_semantics():
    w = ew.Cartpole(_Env(4, 5, 1))
    np.random.seed(0)
    a = w.sample_action(batch_size=7)
    assert a.shape == (7, 1) and a.dtype == torch.float32 and float(a.abs().max()) <= 1.0
    hu = ew.Humanoid(_Env(55, 67, 21))
    b = hu.sample_action(batch_size=3).numpy()
    assert b.shape == (3, 21) and np.all(b[:, 3:-6] == 0)
    # the planner's sampler is the bound static method (agents.py:233)
    fn = functools.partial(w._sample_action, action_spec=w.action_spec())
    np.random.seed(1)
    x = fn(batch_size=4)
    np.random.seed(1)
    assert torch.equal(x, torch.tensor(np.random.uniform(-1, 1, 4).reshape(4, 1), dtype=torch.float32))


def test_get_rollout_drives_the_policy_until_done():
    env = _Env(4, 5, 1, length=3)
    w = ew.Cartpole(env)
    seen = []

    def policy(d):
        seen.append((d["timestep"], d["observation"].clone()))
        return torch.tensor([0.5 * d["timestep"]])

    r = w.get_rollout(num_steps=10, get_action=policy)
    assert len(r) == 3 and len(r.observations) == 4 and len(r.states) == 4
    assert [t for t, _ in seen] == [0, 1, 2]
    assert torch.equal(seen[1][1], torch.full((5,), 1.0))
    assert [float(x) for x in r.rewards[1:]] == [1.0, 2.0, 3.0]
    assert np.allclose([a[0] for a in env.actions], [0.0, 0.5, 1.0])


def test_get_rollout_with_goal_target_sets_state_inside_reset_context():
    env = _Env(4, 6, 2)
    w = ew.Reacher(env)
    goal = torch.tensor([0.3, -0.4, 0.0, 0.0])
    np.random.seed(0)
    r = w.get_rollout(num_steps=2, set_state=True, goal_state=goal, initial_state=goal)
    assert len(r) == 2
    assert np.allclose(env.physics.set_states[0], goal.numpy())
    x, y = ew.Reacher.get_xy(goal.numpy())
    assert env.physics.named.model.geom_pos[("target", "x")] == x
    assert env.physics.named.model.geom_pos[("target", "y")] == y


def test_record_rollout_collects_frames():
    w = ew.Cartpole(_Env(4, 5, 1, length=4))
    r = w.record_rollout(num_steps=10)
    assert len(r.frames) == 4


def test_observation_goals_feed_the_goal_state_cost():
    """observation_goal() fits SmoothAbsLoss on the model's (observation-space) outputs."""
    from mbrl_amd import models
    for cls, ns, no, ad in DOMAINS:
        w = cls(_Env(ns, no, ad))
        try:
            g, wt = w.observation_goal()
        except NotImplementedError:
            continue
        loss = models.SmoothAbsLoss(wt, g)
        out = loss(torch.zeros(3, no))
        assert out.shape[0] == 3 and torch.all(out >= 0)


@pytest.mark.gpu
def test_cartpole_wrapper_rollout_driven_by_the_gpu_planner():
    """The reference's loop end to end on the device planner: Cartpole wrapper -> MPCPolicy ->
    CEMPlanner (fused path: GoalStateAgent closures, the wrapper's bound _sample_action and its
    observation-space goal) -> env.step, as agents.py:224-233 and env_wrappers.py:97-150 wire it."""
    from mbrl_amd import CEMPlanner, MPCPolicy, data, fused, models
    torch.manual_seed(0)
    w = ew.Cartpole(_Env(4, 5, 1, length=1000))
    m = models.Model(5, 1, hidden_units=256, n_hidden=2)
    ds = data.TransitionsDataset.from_statistics({"observations": {"mean": torch.zeros(5), "std": torch.ones(5)},
                                                  "actions": {"mean": torch.zeros(1), "std": torch.ones(1)}})
    g, wt = w.observation_goal()
    cost = models.goal_state_cost(models.SmoothAbsLoss(wt, g), models.CoshLoss())
    sample_action = functools.partial(w._sample_action, action_spec=w.action_spec())
    model_fn = functools.partial(m, **ds.normalizers())
    assert fused.describe_sampler(sample_action) == (-1.0, 1.0, 1)
    assert fused.describe_model(model_fn) is not None and fused.describe_cost(cost, 5) is not None
    pol = MPCPolicy(model_fn, cost, CEMPlanner, sample_action, 10, num_candidates=256, seed=11)
    r = w.get_rollout(num_steps=5, get_action=pol.get_action)
    assert len(r) == 5
    acts = torch.stack([a.reshape(-1) for a in r.actions[:-1]])
    assert acts.shape == (5, 1) and float(acts.abs().max()) <= 1.0
    # the first action is the planner's first planned action from the reset observation
    states, actions = CEMPlanner.plan(r.observations[0], model_fn, cost, sample_action, 10, num_candidates=256,
                                      seed=11)
    assert torch.equal(actions[0].flatten(), acts[0])
