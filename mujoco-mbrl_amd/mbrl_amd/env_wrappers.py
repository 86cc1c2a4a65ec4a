"""dm_control environment wrappers with the reference's interface.

Restates /root/reference/src/mbrl/env_wrappers.py so that the planner drops into the reference's
training loop unchanged: `EnvWrapper.load(env_name, task_name)` builds a dm_control suite task and
wraps it; `reset`/`step` return (state, observation, reward, done); `get_rollout` drives a policy
(`get_action(dict(timestep, state, observation))`, the MPCPolicy signature) and returns a
`data.Rollout`; per-domain subclasses give the state features, goal weights, goal states and
state samplers the reference's agents use.

Host plumbing only: nothing here touches the GPU. dm_control and MuJoCo are not installable in
this image, so `load` raises ImportError when the suite is absent; any object with
dm_env's `reset/step/action_spec/observation_spec` and a `.physics` works as the wrapped env
(tests/test_env_wrappers.py drives the wrappers with stand-in physics).

Differences from the reference, each a fix of a reference bug SURVEY.md §8f lists:
  * the wrapper class is looked up in a registry, not with eval();
  * `Cartpole` exists (config 1/2's domain; the reference has no cartpole wrapper, :20-34);
  * Humanoid, Swimmer and Walker read `self._env` (the reference's `self.env`, :441-456,531-535,
    raises AttributeError);
  * `observation_goal()` gives (goal, weights) in the FLAT OBSERVATION space the model is trained
    on (GoalStateAgent uses obs_only data, agents.py:217), for the four BASELINE domains. The
    reference's set_goal()/get_goal_weights() are state-space vectors (Cheetah: 19 entries against
    a 17-entry observation, :64-66,296-306) and stay available unchanged.
"""
from typing import Callable, Dict, Optional

import numpy as np
import torch

from . import env as _env
from .data import Rollout

_REGISTRY = {}


def _register(cls):
    _REGISTRY["".join(part.capitalize() for part in cls.domain.split("_"))] = cls
    return cls


class EnvWrapper:
    """env_wrappers.py:9-181."""
    domain = None
    state_dim = 0
    observation_dim = 0

    def __init__(self, env, flat_obs=True, env_name=None, task_name=None):
        self._env = env
        self._state_penalty = 1.0
        self._action_spec = env.action_spec()
        self.action_dim = self._action_spec.shape[0]
        self._flat_obs = flat_obs
        self._env_name = env_name
        self._task_name = task_name

    # ---------------------------------------------------------------- construction (:19-33)
    @staticmethod
    def wrapper_class(env_name):
        key = "".join(part.capitalize() for part in env_name.split("_"))
        try:
            return _REGISTRY[key]
        except KeyError:
            raise NameError(f"No wrapper for {env_name}") from None

    @staticmethod
    def load(env_name, task_name, flat_obs=True, **kwargs):
        cls = EnvWrapper.wrapper_class(env_name)
        try:
            from dm_control import suite
        except ImportError as exc:
            raise ImportError("EnvWrapper.load needs dm_control and MuJoCo (requirements.txt:3); wrap an "
                              "existing dm_env environment with the wrapper class instead") from exc
        env_kwargs = kwargs.setdefault("environment_kwargs", {})
        env_kwargs["flat_observation"] = flat_obs
        if getattr(cls, "override_control_timestep", None) is not None:
            env_kwargs["control_timestep"] = cls.override_control_timestep
        return cls(suite.load(env_name, task_name, **kwargs), flat_obs=flat_obs, env_name=env_name,
                   task_name=task_name)

    # ---------------------------------------------------------------- state, goal, actions
    def get_state(self) -> torch.Tensor:
        return torch.tensor(self._env.physics.state(), dtype=torch.float32)

    def sample_state(self) -> torch.Tensor:
        raise NotImplementedError

    def set_goal(self) -> torch.Tensor:
        raise NotImplementedError

    def get_goal_weights(self) -> torch.Tensor:
        return torch.zeros(self.state_dim)

    def observation_goal(self):
        """(goal, weights) over the flat observation, for SmoothAbsLoss on the model's outputs."""
        raise NotImplementedError(f"no observation-space goal for {type(self).__name__}")

    def sample_action(self, batch_size=None) -> torch.Tensor:
        return self._sample_action(self.action_spec(), batch_size)

    @staticmethod
    def _sample_action(action_spec, batch_size=None) -> torch.Tensor:
        return _env._sample_action(action_spec, batch_size)

    def action_spec(self):
        return self._action_spec

    def observation_spec(self):
        return self._env.observation_spec()

    # ---------------------------------------------------------------- stepping (:70-94)
    def reset(self):
        return self._parse_timestep(self._env.reset())

    def step(self, action):
        a = action.detach().cpu().numpy() if torch.is_tensor(action) else np.array(action)
        return self._parse_timestep(self._env.step(a))

    def _parse_timestep(self, t):
        if self._flat_obs:
            obs = torch.tensor(np.asarray(t.observation["observations"]), dtype=torch.float32)
        else:
            obs = {str(k): torch.tensor(np.asarray(v), dtype=torch.float32) for k, v in t.observation.items()}
        reward = torch.tensor(t.reward, dtype=torch.float32) if t.reward is not None else None
        return self.get_state(), obs, reward, t.last()

    # ---------------------------------------------------------------- rollouts (:97-150)
    def get_rollout(self, num_steps: int, get_action: Optional[Callable[[Dict], torch.Tensor]] = None,
                    step_callback: Optional[Callable] = None, set_state: bool = False,
                    goal_state: Optional[torch.Tensor] = None,
                    initial_state: Optional[torch.Tensor] = None) -> Rollout:
        if get_action is None:
            get_action = lambda _: self.sample_action()   # noqa: E731
        state, observation, _, _ = self.reset()
        if set_state:
            initial_state = self.sample_state() if initial_state is None else initial_state
        else:
            initial_state = self._env.physics.state()
        if goal_state is not None and hasattr(self, "set_target"):
            # a new target needs the initial state set again inside the reset context
            with self._env.physics.reset_context():
                self._env.physics.set_state(initial_state)
                self.set_target(goal_state)
            state, observation, _, _ = self.step(self.sample_action())
        states, observations, actions, rewards = [state], [observation], [], []
        for timestep in range(num_steps):
            action = get_action(dict(timestep=timestep, state=state, observation=observation))
            actions.append(action)
            state, observation, reward, done = self.step(action)
            states.append(state)
            observations.append(observation)
            rewards.append(reward)
            if step_callback is not None:
                step_callback(timestep)
            if done:
                break
        return Rollout(states=states, observations=observations, actions=actions, rewards=rewards)

    def record_rollout(self, *args, **kwargs):
        """get_rollout with a rendered frame per step in rollout.frames (:152-162; the reference's
        ffmpeg movie writer is left to the caller)."""
        kwargs.pop("mp4path", None)
        frames = []
        kwargs["step_callback"] = lambda t: frames.append(self._env.physics.render(camera_id=0))
        rollout = self.get_rollout(*args, **kwargs)
        rollout.frames = frames
        return rollout


def _uniform_into(state, ranges):
    """state[i] = U(lo, hi) for (i, lo, hi) in order: one np.random.uniform call per entry, the
    draw order of the reference's samplers."""
    for i, lo, hi in ranges:
        state[i] = np.random.uniform(lo, hi)
    return state


@_register
class PointMass(EnvWrapper):
    """:165-183."""
    domain = "point_mass"
    state_dim = 4
    observation_dim = 4

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[0:2] = 10 * self._state_penalty
        w[2:] = self._state_penalty / 4.0       # velocity penalties damp the approach
        return w

    def set_goal(self):
        target = np.random.uniform(-0.25, 0.25, 3)
        target[-1] = 0.01
        self._env.physics.named.model.geom_pos["target"] = target
        goal = torch.zeros(self.state_dim, dtype=torch.float32)
        goal[0], goal[1] = float(target[0]), float(target[1])
        return goal


@_register
class Reacher(EnvWrapper):
    """:186-259."""
    domain = "reacher"
    state_dim = 4
    observation_dim = 6
    override_control_timestep = 0.04

    def sample_state(self):
        s = _uniform_into(np.zeros(self.state_dim), [(0, -np.pi, np.pi), (1, -2.8, 2.8), (2, -3, 3), (3, -3, 3)])
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = torch.zeros(self.observation_dim)
        w[0:4] = self._state_penalty             # arm angles and the vector to the target
        w[4:] = self._state_penalty / 20         # velocities: damping
        return w

    def set_goal_state(self):
        g = torch.zeros(self.state_dim, dtype=torch.float32)
        g[0] = float(np.random.uniform(low=-np.pi, high=np.pi))
        g[1] = float(np.random.uniform(low=-2.8, high=2.8))   # reachable targets only
        return g

    def set_goal_observation(self):
        g = torch.zeros(self.observation_dim, dtype=torch.float32)
        g[0] = float(np.random.uniform(low=-np.pi, high=np.pi))
        g[1] = float(np.random.uniform(low=-2.8, high=2.8))
        return g

    def set_goal(self):
        return self.set_goal_observation()

    def set_target(self, state):
        x, y = self.get_xy(state)
        self._env.physics.named.model.geom_pos["target", "x"] = x
        self._env.physics.named.model.geom_pos["target", "y"] = y

    @staticmethod
    def get_xy(goal_state):
        """Fingertip position of the two-link arm (link lengths 0.12) at joint angles goal_state[:2]."""
        a = 0.12 * np.cos(goal_state[1])
        b = 0.12 * np.sin(goal_state[1])
        theta = goal_state[0] + np.arctan(b / (0.12 + a))
        mag = np.sqrt((0.12 + a) ** 2 + b ** 2)
        return mag * np.cos(theta), mag * np.sin(theta)

    def sample_rollouts_biased_rewards(self, num_rollouts=20, num_steps=100):
        out = []
        for _ in range(num_rollouts):
            s = self.set_goal_state()
            out.append(self.get_rollout(num_steps=num_steps, set_state=True, goal_state=s, initial_state=s))
        return out


@_register
class Cheetah(EnvWrapper):
    """:261-306. State: physics.state()[1:] (17), horizontal speed, torso height."""
    domain = "cheetah"
    state_dim = 18 - 1 + 2
    observation_dim = 17
    _JOINTS = [(3, -0.5236, 1.0472), (4, -0.8727, 0.8727), (5, -4.0143, 0.8727), (6, -0.9948, 0.0070),
               (7, -1.2217, 0.8727), (8, -0.4887, 0.4887)]   # bthigh .. ffoot limits (rad)

    def sample_state(self):
        s = np.zeros(18)
        s[1] = np.random.uniform(-0.2, 0.2)             # vertical position
        if s[1] > 0.05:
            s[2] = np.random.uniform(-3.14, 3.14)        # torso angle
        elif np.random.uniform() < 0.72:
            s[2] = np.random.uniform(-3.14, -1.5)
        else:
            s[2] = np.random.uniform(2.5, 3.14)
        _uniform_into(s, self._JOINTS)
        s[9:] = np.random.uniform(-3, 3, 9)             # velocities
        return torch.tensor(s, dtype=torch.float32)

    def get_state(self):
        s = super().get_state()[1:].numpy()
        s = np.append(s, self._env.physics.speed())
        s = np.append(s, self._env.physics.named.data.subtree_com["torso"][2])
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[17] = self._state_penalty
        w[18] = self._state_penalty / 2.0
        return w

    def set_goal(self):
        g = torch.zeros(self.state_dim, dtype=torch.float32)
        g[-2] = 2.0                                      # speed
        g[-1] = 0.4                                      # torso height
        return g

    def observation_goal(self):
        """Flat observation = qpos[1:] (8) | qvel (9) (dm_control cheetah.py:83-89): run at speed 2
        (qvel rootx, obs[8]) and hold the spawn height (qpos rootz, obs[0])."""
        g = torch.zeros(self.observation_dim)
        w = torch.zeros(self.observation_dim)
        g[8], w[8] = 2.0, self._state_penalty
        w[0] = self._state_penalty / 2.0
        return g, w


@_register
class Manipulator(EnvWrapper):
    """:309-341."""
    domain = "manipulator"
    state_dim = 22 + 7
    observation_dim = 37

    def get_state(self):
        p = self._env.physics
        s = super().get_state().numpy()
        s = np.append(s, p.named.data.site_xpos["grasp", "x"])
        s = np.append(s, p.named.data.site_xpos["grasp", "z"])
        s = np.append(s, p.touch())                      # 5 contact sensors
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[8:10] = 10 * self._state_penalty
        w[10:21] = self._state_penalty / 4
        w[-7:-5] = 10 * self._state_penalty
        w[-5:] = self._state_penalty / 20
        return w

    def set_goal(self):
        g = torch.zeros(self.state_dim, dtype=torch.float32)
        ball = self._env.physics.body_location("target_ball")[:2]
        g[8], g[9] = float(ball[0]), float(ball[1])      # ball over the target
        g[-7], g[-6] = float(ball[0]), float(ball[1])    # gripper at the target
        g[-5:] = 0.5                                      # contact sensors
        return g


@_register
class Humanoid(EnvWrapper):
    """:344-457 (reads self._env; the reference's self.env raises)."""
    domain = "humanoid"
    state_dim = 55 + 5
    observation_dim = 67
    _JOINTS = [(7, -0.7854, 0.7854), (8, -1.3089, 0.5236), (9, -0.6109, 0.6109),                  # abdomen z, y, x
               (10, -0.4363, 0.0873), (11, -1.0472, 0.6109), (12, -1.9199, 0.3491),              # right hip x, z, y
               (13, -2.7925, 0.0349), (14, -0.8727, 0.8727), (15, -0.8727, 0.8727),              # right knee, ankle y, x
               (16, -0.4363, 0.0873), (17, -1.0472, 0.6109), (18, -1.9199, 0.3491),              # left hip x, z, y
               (19, -2.7925, 0.0349), (20, -0.8727, 0.8727), (21, -0.8727, 0.8727),              # left knee, ankle y, x
               (22, -1.4835, 1.0472), (23, -1.4835, 1.0472), (24, -1.5708, 0.8727),              # right shoulder 1, 2, elbow
               (25, -1.0472, 1.4835), (26, -1.0472, 1.4835), (27, -1.5708, 0.8727)]              # left shoulder 1, 2, elbow

    def sample_state(self):
        s = np.zeros(55)
        s[2] = 1.3                                       # vertical position
        _uniform_into(s, self._JOINTS)
        return torch.tensor(s, dtype=torch.float32)

    def sample_action(self, batch_size=None):
        """Gaussian exploration with the abdomen/hip block zeroed (:426-435); the planner does not
        use it (agents.py:233 binds _sample_action)."""
        if batch_size is None:
            a = np.random.normal(0, 0.4, self.action_dim)
            a[3:-6] = 0.0
        else:
            a = np.random.normal(0, 0.4, self.action_dim * batch_size).reshape((batch_size, -1))
            a[:, 3:-6] = 0.0
        return torch.tensor(a, dtype=torch.float32)

    def get_state(self):
        p = self._env.physics
        s = super().get_state().numpy()                  # 55: the pure state
        com = p.center_of_mass_position()
        feet = (p.named.data.xpos["right_foot"] + p.named.data.xpos["left_foot"]) / 2.0
        above_feet = feet + np.array([0.0, 0.0, 1.3])
        torso = p.named.data.xpos["torso"]
        s = np.append(s, np.linalg.norm(com[:2] - feet[:2]))        # balance terms (Tassa et al.)
        s = np.append(s, np.linalg.norm(com[:2] - torso[:2]))
        s = np.append(s, np.linalg.norm(torso[1:] - above_feet[1:]))
        s = np.append(s, p.center_of_mass_velocity()[:2])
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[-5:] = 10 * self._state_penalty
        return w

    def set_goal(self):
        return torch.zeros(self.state_dim, dtype=torch.float32)

    def observation_goal(self):
        """Flat observation (dm_control humanoid.py:172-185): joint angles (21) | head height [21] |
        extremities (12) | torso vertical zx, zy, zz [34:37] | com velocity [37:40] | velocity (27).
        Stand: head at 1.6, torso upright, no horizontal com velocity."""
        g = torch.zeros(self.observation_dim)
        w = torch.zeros(self.observation_dim)
        g[21], w[21] = 1.6, 10 * self._state_penalty
        g[36], w[36] = 1.0, 10 * self._state_penalty
        w[37:39] = 10 * self._state_penalty
        return g, w


@_register
class Swimmer(EnvWrapper):
    """:460-487 (reads self._env; the reference's self.env raises)."""
    domain = "swimmer"
    state_dim = 10 + 2

    def sample_state(self):
        s = np.zeros(10)                                 # swimmer3
        s[2] = np.random.uniform(low=-3, high=3)
        return torch.tensor(s, dtype=torch.float32)

    def get_state(self):
        s = super().get_state().numpy()
        s = np.append(s, self._env.physics.named.data.xmat["head"][:2])   # head orientation
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[0:1] = 10 * self._state_penalty
        w[5:-2] = self._state_penalty
        return w

    def set_goal(self):
        t = self._env.physics.named.data.geom_xpos["target"][:2]
        g = torch.zeros(self.state_dim, dtype=torch.float32)
        g[0], g[1] = float(t[0]), float(t[1])
        return g


@_register
class Walker(EnvWrapper):
    """:490-544 (reads self._env; the reference's self.env raises)."""
    domain = "walker"
    state_dim = 18 - 1 + 3
    observation_dim = 24

    def sample_state(self):
        s = np.zeros(18)
        s[2] = np.random.uniform(-0.1, 0.1)              # main body rotation
        hip = np.random.uniform(-0.15, 0.15)
        s[3] = hip
        s[4] = np.random.uniform(-0.3, 0)                # right knee
        s[5] = np.random.uniform(-0.1, 0.1)              # right ankle
        s[6] = -hip
        s[7] = np.random.uniform(-0.3, 0)                # left knee
        s[8] = np.random.uniform(-0.1, 0.1)              # left ankle
        return torch.tensor(s, dtype=torch.float32)

    def get_state(self):
        p = self._env.physics
        s = super().get_state()[1:].numpy()
        s = np.append(s, p.torso_upright())
        s = np.append(s, p.torso_height())
        s = np.append(s, p.horizontal_velocity())
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[-3:] = self._state_penalty
        return w

    def set_goal(self):
        g = torch.zeros(self.state_dim, dtype=torch.float)
        g[-3], g[-2], g[-1] = 1.0, 1.3, 3.0               # upright, torso height, speed
        return g

    def observation_goal(self):
        """Flat observation (dm_control walker.py:135-141): orientations xx, xz of 7 bodies (14, torso
        first: obs[0] = torso xx = upright for a planar body) | torso height [14] | qvel (9, rootx
        first: [15]). The reference's walker goal on those entries: upright 1, height 1.3, speed 3."""
        g = torch.zeros(self.observation_dim)
        w = torch.zeros(self.observation_dim)
        for i, v in ((0, 1.0), (14, 1.3), (15, 3.0)):
            g[i], w[i] = v, self._state_penalty
        return g, w


@_register
class Hopper(EnvWrapper):
    """:547-592."""
    domain = "hopper"
    state_dim = 14 - 1 + 4
    observation_dim = 15

    def sample_state(self):
        s = np.zeros(14)
        s[1] = -0.078789                                 # vertical position
        _uniform_into(s, [(2, -0.01, 0.01), (3, -0.01, 0.01), (4, -0.01, 0.01), (5, 0.1, 0.12), (6, -0.01, 0.01)])
        s[7:] = np.random.uniform(-0.01, 0.01, 7)        # velocities
        return torch.tensor(s, dtype=torch.float32)

    def get_state(self):
        p = self._env.physics
        s = super().get_state()[1:].numpy()
        s = np.append(s, p.touch())                      # foot touch sensors
        s = np.append(s, p.height())
        s = np.append(s, p.speed())
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[-2] = self._state_penalty / 2.0
        w[-1] = self._state_penalty
        return w

    def set_goal(self):
        g = torch.zeros(self.state_dim, dtype=torch.float)
        g[-2], g[-1] = 0.9, 1.0                          # torso height, speed
        return g


@_register
class Cartpole(EnvWrapper):
    """Not in the reference (configs 1 and 2 are cartpole-swingup). State =
    physics.state() = (cart, hinge, their velocities); flat observation (dm_control
    cartpole.py:150-153,202-207) = cart position | pole cos, sin | cart, pole velocities."""
    domain = "cartpole"
    state_dim = 4
    observation_dim = 5

    def sample_state(self):
        s = np.zeros(self.state_dim)
        s[0] = np.random.uniform(-0.5, 0.5)              # cart position
        s[1] = np.random.uniform(-np.pi, np.pi)          # pole angle
        return torch.tensor(s, dtype=torch.float32)

    def get_goal_weights(self):
        w = super().get_goal_weights()
        w[0:2] = self._state_penalty
        w[2:] = self._state_penalty / 10
        return w

    def set_goal(self):
        return torch.zeros(self.state_dim, dtype=torch.float32)   # centred cart, upright pole, at rest

    def observation_goal(self):
        """Swing-up: pole upright (cos 1, sin 0), cart centred, velocities damped."""
        g = torch.tensor([0.0, 1.0, 0.0, 0.0, 0.0])
        p = self._state_penalty
        w = torch.tensor([p, p, p, p / 10, p / 10])
        return g, w


WRAPPERS = dict(_REGISTRY)
