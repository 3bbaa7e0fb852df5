"""Reference-shaped single-environment API.

Drop-in for the reference's task-env classes: ``Env(config)`` with
``reset(obs_as_dict=False)`` / ``step(action, obs_as_dict=False)`` returning
``[obs, reward, done, {'all_rewards': [...]}]``, gym-style ``action_space`` /
``observation_space`` / ``spec.timestep_limit`` and a no-op ``render``
(opensim_environment.py:33-113, muscle_walking_imitation_env2D.py:18-403,
torque_walking_imitation_env2D.py:18-366).  Every instance is one env of a
:class:`~bioimitation.vector_env.VectorEnv` on the GPU: the physics runs in
the HIP kernel, never on the host.  For throughput, step many envs at once
with ``VectorEnv`` directly.

Reset-index semantics follow the reference exactly: ``random.randint(0, hi)``
from Python's ``random`` module in train mode (so ``random.seed`` reproduces
the reference's choice) with ``hi = N/2`` (2D envs, Running3D) or ``cycle``
(Walking3D, LockedKnee3D, Palsy3D), index 0 in test mode
(muscle_walking_imitation_env2D.py:133-156, muscle_walking_imitation_env3D.py:133-144).
"""
from __future__ import annotations

import random

import numpy as np

from .registry import NOT_BUILT, RECIPES, load_pack

DEFAULT_CONFIG = {  # configs/env_default.py keys the envs read
    'mode': 'train', 'visualize': False, 'max_actuation': 200.0, 'log': False,
    'r_weights': [0.8, 0.2, 0.1], 'horizon': 5, 'use_target_obs': True, 'use_GRF': True,
    'apply_perturbations': False,
}


class Box:
    """Minimal gym.spaces.Box stand-in (used when gym is not installed)."""

    def __init__(self, low, high, dtype=np.float64):
        self.low = np.asarray(low, dtype=dtype)
        self.high = np.asarray(high, dtype=dtype)
        self.shape = self.low.shape
        self.dtype = np.dtype(dtype)

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(lo, hi).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f'Box({self.shape})'


def _box(low, high):
    try:
        from gym import spaces
        return spaces.Box(np.array(low), np.array(high))
    except Exception:
        return Box(low, high)


class Specification:
    """opensim_environment.py:9-13"""

    def __init__(self, timestep_limit):
        self.id = 0
        self.timestep_limit = timestep_limit


class ImitationEnv:
    """One environment of a registered ID on one GPU (see module docstring)."""
    env_id = None

    def __init__(self, config=None, device=0, precision=64, seed=0):
        cfg = dict(DEFAULT_CONFIG)
        cfg.update(config or {})
        from .vector_env import VectorEnv
        self.config = cfg
        self.test = cfg.get('mode') == 'test'
        self._env = VectorEnv(self.env_id, 1, config=dict(cfg, apply_perturbations=False), device=device,
                              precision=precision, seed=seed, auto_reset=False)
        if cfg.get('apply_perturbations'):
            # one schedule per construction from NumPy's global RNG, like the
            # reference (muscle_walking_imitation_env2D.py:83-100)
            from .perturb import reference_points
            x, y = reference_points(self.env_id)
            self._env.set_perturbation(x, y[None, :])
        pk = self._env.pack
        self.N = pk.n_episode
        self.cycle = pk.cycle
        if pk.nmuscle:
            lo, hi = [0.0] * pk.nact, [1.0] * pk.nact
        else:
            lo = [pk.coordact[a].min_control for a in range(pk.nact)]
            hi = [pk.coordact[a].max_control for a in range(pk.nact)]
        self.action_space = _box(lo, hi)
        n = self._env.obs_dim
        self.observation_space = _box([-np.inf] * n, [np.inf] * n)
        self.timestep_limit = 1e10
        self.spec = Specification(self.timestep_limit)
        self.spec.action_space = self.action_space
        self.spec.observation_space = self.observation_space
        self._names = None
        # the OsimModel facade callers reach through env.osim_model (save_simulation, istep, ...)
        from .obslayout import load_names
        from .simulation_io import OsimModelFacade
        self.osim_model = OsimModelFacade(self._env, load_names(self.env_id), lo, hi)
        self._last = None            # (reward, all_rewards, done) of the last step
        self.state_dict = None
        self._record = bool(cfg.get('record_trajectory', True))
        self._state_buf = None
        self._packed = None
        import torch
        if self._env.dtype == torch.float64:
            self._bind_packed()
        elif self._record:
            self._env.enable_force_report()
        if self._record and self._env.integrator == 'rk-merson':
            self._env.enable_state_storage(512)    # the Manager's rows: every accepted step
        ntrans = sum(1 for c in (pk.coord_tx, pk.coord_ty, pk.coord_tz) if c >= 0)
        self._qdd = slice(1 + (pk.ncoord - ntrans) + pk.ncoord, 1 + (pk.ncoord - ntrans) + 2 * pk.ncoord)

    def _bind_packed(self):
        """fp64: the step kernel writes the env's observation, reward, info and
        done byte — and, recording, its force-report row — into one device
        buffer, and the recorder's state row is gathered behind them
        (bioim_copy_state), so one asynchronous copy into pinned host memory
        brings a step's outputs back: no concatenating or converting kernels
        after the step.  The action goes up through a pinned buffer too, so
        the launch does not wait for a synchronous pageable copy
        (tools/facade_parts.py: 19.6 us of a 191 us C1 step)."""
        import torch
        e = self._env
        nobs, ninf = e.obs_dim, e.info_dim
        nfr = e.force_report_dim if self._record else 0
        nst = e.state_dim if self._record else 0
        self._lay = (nobs, ninf, nfr)
        n = nobs + 1 + ninf + 1 + nfr + nst
        dev = torch.zeros(n, dtype=torch.float64, device=e.device)
        e.obs = dev[:nobs].view(1, nobs)
        e.reward = dev[nobs:nobs + 1]
        e.info = dev[nobs + 1:nobs + 1 + ninf].view(1, ninf)
        # done: the kernel stores one byte, the first of this zeroed double slot
        e.done = dev[nobs + 1 + ninf:nobs + 2 + ninf].view(torch.uint8)[:1]
        if self._record:
            f0 = nobs + 2 + ninf
            e.enable_force_report(out=dev[f0:f0 + nfr].view(1, nfr))
            self._state_buf = dev[f0 + nfr:].view(1, nst)
        self._packed = (dev, torch.zeros(n, dtype=torch.float64).pin_memory())
        self._act = (torch.zeros((1, e.action_dim), dtype=torch.float64, device=e.device),
                     torch.zeros((1, e.action_dim), dtype=torch.float64).pin_memory())

    def _step_packed(self, action):
        import torch
        e = self._env
        a_dev, a_pin = self._act
        a = np.asarray(action, dtype=np.float64).reshape(-1)
        if a.shape != (e.action_dim,):
            raise ValueError(f'action must have {e.action_dim} entries, got shape {np.shape(action)}')
        # the last step's copies finished at its synchronize: the pinned buffers are free
        a_pin.numpy()[0] = a
        a_dev.copy_(a_pin, non_blocking=True)
        e.step(a_dev)
        self.osim_model._dirty()
        if self._record:
            e.state_rows(self._state_buf)
        dev, pin = self._packed
        pin.copy_(dev, non_blocking=True)
        torch.cuda.current_stream(e.device).synchronize()
        out = pin.numpy().copy()
        nobs, ninf, nfr = self._lay
        o = out[:nobs]
        done = bool(out[nobs + 1 + ninf:nobs + 2 + ninf].view(np.uint8)[0])
        if self._record:
            f0 = nobs + 2 + ninf
            self._record_row(o, fr=out[f0:f0 + nfr], state=out[f0 + nfr:])
        inf = [float(v) for v in out[nobs + 1:nobs + 1 + ninf]]
        return o, float(out[nobs]), inf, done

    # -- reference API -------------------------------------------------------
    def _out(self, obs, as_dict):
        o = obs[0] if isinstance(obs, np.ndarray) else obs[0].double().cpu().numpy()
        if not as_dict:
            return o
        from .obslayout import load_names, obs_to_dict   # the reference's nested dict, rebuilt host-side
        if self._names is None:
            self._names = load_names(self.env_id)
        return obs_to_dict(o, self._env.pack, self._names)

    def _record_row(self, o, stepped=True, fr=None, state=None):
        """o: the env's observation row on the host; fr, state: its
        force-report and state rows when the caller has already copied them"""
        if self._record:
            if fr is None:
                fr = self._env.force_report[0].double().cpu().numpy()
            if state is None:
                state = self._env.get_state()[0]
            self.osim_model.record_row(state, o[self._qdd], fr, stepped)

    def reset(self, obs_as_dict=False):
        index = 0 if self.test else random.randint(0, self._env.pack.reset_hi)
        obs = self._env.reset(env_ids=[0], ref_index=[index])
        self.osim_model._dirty()
        self.osim_model.recorder.clear()     # reset_manager re-initializes the analyses
        self._last = None
        o = obs[0].double().cpu().numpy()
        self._record_row(o, stepped=False)
        return self._out(o[None, :], obs_as_dict)

    def step(self, action, obs_as_dict=False):
        if self._packed is not None:
            o, rew, inf, done = self._step_packed(action)
            self._last = (rew, inf, done)
            return [self._out(o[None, :], obs_as_dict), rew, done, {'all_rewards': inf}]
        import torch
        a = torch.as_tensor(np.asarray(action, dtype=np.float64).reshape(1, -1), dtype=self._env.dtype,
                            device=self._env.device)
        obs, rew, done, info = self._env.step(a)
        self.osim_model._dirty()
        # one device-to-host copy for the step's outputs (each .cpu() waits on the stream),
        # the force-report row included when recording
        parts = [obs[0], rew[:1], info[0], done[:1].to(obs.dtype)]
        if self._record:
            # the force-report row and the state row (gathered on the device,
            # bioim_copy_state) ride in the same transfer: no separate
            # synchronizing bioim_get_state per step
            parts.append(self._env.force_report[0])
            if obs.dtype == torch.float64:   # fp32 envs keep get_state (t and q stay doubles)
                parts.append(self._env.state_rows(self._state_buf)[0])
        out = torch.cat(parts).double().cpu().numpy()
        nobs, ninf = obs.shape[1], info.shape[1]
        o = out[:nobs]
        if self._record:
            nfr = self._env.force_report.shape[1]
            f0 = nobs + 1 + ninf + 1
            self._record_row(o, fr=out[f0:f0 + nfr], state=out[f0 + nfr:] if len(out) > f0 + nfr else None)
        else:
            self._record_row(o)
        inf = [float(v) for v in out[nobs + 1:nobs + 1 + ninf]]
        self._last = (float(out[nobs]), inf, bool(out[nobs + 1 + ninf]))
        return [self._out(o[None, :], obs_as_dict), self._last[0], self._last[2], {'all_rewards': inf}]

    # -- the task envs' public methods (muscle_walking_imitation_env2D.py:102-403,
    #    opensim_environment.py:52-98); realizations run on the GPU (bioim_osim) --
    def get_state_dict(self):
        """The observation dict at the current state (obs_as_dict layout); also
        sets ``self.state_dict`` to the merged calc_* realizations, as the
        reference does (:158-230)."""
        om = self.osim_model
        self.state_dict = {}
        for part in (om.calc_joint_kinematics(), om.calc_body_kinematics(), om.calc_muscles_info(),
                     om.calc_forces_info()):
            self.state_dict.update(part)
        return self._out(om.observation()[None, :], True)

    def get_observation_dict(self):
        return self.get_state_dict()

    def get_observation(self):
        """the flattened observation (opensim_environment.py:52-64), a list"""
        return [float(v) for v in self.osim_model.observation()]

    def get_reward(self):
        """(reward, all_rewards) of the last step.  The reference recomputes it
        and advances its cross-step terms (last action, old pelvis x) as a side
        effect; here those advance inside the step kernel, so this returns the
        step's values and changes nothing."""
        if self._last is None:
            raise RuntimeError('get_reward: no step since the last reset')
        return self._last[0], list(self._last[1])

    def is_done(self):
        """the termination flag of the last step (False before any step)"""
        return bool(self._last[2]) if self._last is not None else False

    def get_limit_forces(self):
        """muscle_walking_imitation_env2D.py:232-235"""
        return list(self.osim_model.calc_forces_info()['coordinate_limit_forces'].values())

    def calc_cost_of_transport(self):
        """Umberger-style metabolic rate of the realized state
        (muscle_walking_imitation_env2D.py:360-403), computed on the GPU; muscle
        models only, like the reference."""
        if not self.osim_model.is_muscle_model:
            raise AttributeError(f'{type(self).__name__} has no calc_cost_of_transport (torque model)')
        return self.osim_model.report()['cot']

    def get_mass(self):
        self.mass = self.osim_model.model.getTotalMass(self.osim_model.state)
        return self.mass

    def get_height(self):
        self.height = 1.80   # hard-coded in every reference env (:106-109)
        return self.height

    def get_gravity(self):
        self.gravity = self.osim_model.model.getGravity()
        return self.gravity

    def render(self, mode='human', close=False):
        return

    def get_observation_space_size(self):
        return self._env.obs_dim

    def get_action_space_size(self):
        return self._env.action_dim

    def seed(self, s=None):
        random.seed(s)
        return [s]

    def close(self):
        self.osim_model.close()
        self._env.close()


def _env_class(env_id):
    """The reference's class name for an env ID (e.g. MuscleWalkingImitation2D-v0 ->
    MuscleWalkingImitationEnv2D, bioimitation/__init__.py:10-17,89-97)."""
    stem = env_id[:-len('-v0')]
    name = stem[:-2] + 'Env' + stem[-2:]
    return type(name, (ImitationEnv,), {'env_id': env_id, '__doc__': f'{env_id} on the HIP step.'})


ENV_CLASSES = {e: _env_class(e) for e in RECIPES}
globals().update({c.__name__: c for c in ENV_CLASSES.values()})


def make(env_id, config=None, **kw):
    """Construct the env class registered under ``env_id``."""
    if env_id not in ENV_CLASSES:
        if env_id in NOT_BUILT:
            raise NotImplementedError(f'{env_id}: {NOT_BUILT[env_id]}')
        raise KeyError(env_id)
    return ENV_CLASSES[env_id](config, **kw)


# rllib_creator: the env offset of worker w's vector slot v is
# (w << RLLIB_WORKER_SHIFT) + v * num_envs, distinct for up to 2**20 envs per worker
RLLIB_WORKER_SHIFT = 20


def _ray_vector_env_class():
    """RLlibVectorEnv with ``ray.rllib.env.vector_env.VectorEnv`` as a base
    class when ray is importable (RLlib's env conversion dispatches on
    isinstance, so the duck-typed protocol alone would be taken for a
    gym.Env), else None."""
    try:
        from ray.rllib.env.vector_env import VectorEnv as RayVectorEnv
    except Exception:
        return None
    from .adapters import RLlibVectorEnv

    class RayRLlibVectorEnv(RLlibVectorEnv, RayVectorEnv):
        def __init__(self, *args, **kw):
            RLlibVectorEnv.__init__(self, *args, **kw)
            RayVectorEnv.__init__(self, self.observation_space, self.action_space, self.num_envs)
    return RayRLlibVectorEnv


def rllib_creator(env_id):
    """The env creator registered with Ray for ``env_id``
    (bioimitation/__init__.py:135-143 registers ``lambda config: Env(config)``).
    With ``config['num_envs'] > 1`` it returns one batched
    :class:`~bioimitation.adapters.RLlibVectorEnv` of that many envs on the
    worker's GPU, instead of one single-env instance per call: the reference's
    one-env-per-worker layout costs a kernel launch and a host round trip per
    env step (180 us per step against 45-56 us for one CPU thread
    running the same algorithm), the batched env amortizes both over the batch.
    When ray is importable the returned object is also an instance of RLlib's
    ``VectorEnv`` (:func:`_ray_vector_env_class`), which is what RLlib's env
    conversion checks for.
    Optional keys: ``device`` (GPU ordinal, default 0), ``precision`` (64).
    RLlib's EnvContext ``worker_index`` and ``vector_index`` (several creator
    calls per worker when ``num_envs_per_worker > 1``) set the envs' global
    indices (``env_offset`` = (worker_index << 20) + vector_index * num_envs),
    so every worker and vector slot draws its own reset rows.
    Ray is not importable here: the CPU tests cover the creator's dispatch
    and offsets (tests/test_envs.py), not RLlib's own conversion."""
    if env_id not in ENV_CLASSES:
        if env_id in NOT_BUILT:
            raise NotImplementedError(f'{env_id}: {NOT_BUILT[env_id]}')
        raise KeyError(env_id)
    cls = ENV_CLASSES[env_id]

    def create(config=None):
        cfg = dict(config or {})
        n = int(cfg.pop('num_envs', 1))
        if n <= 1:
            return cls(config)
        from .adapters import RLlibVectorEnv
        device, precision = int(cfg.pop('device', 0)), int(cfg.pop('precision', 64))
        offset = rllib_env_offset(config, n)
        vcls = _ray_vector_env_class() or RLlibVectorEnv
        return vcls(env_id, n, config=cfg, device=device, precision=precision, env_offset=offset)
    return create


def rllib_env_offset(config, num_envs):
    """Global index of the first env of the batch an RLlib creator call makes
    (its EnvContext's worker_index and vector_index; 0 for a plain dict)."""
    w = int(getattr(config, 'worker_index', 0) or 0)
    v = int(getattr(config, 'vector_index', 0) or 0)
    if v * num_envs >= (1 << RLLIB_WORKER_SHIFT):
        raise ValueError(f'rllib_creator: vector_index {v} x num_envs {num_envs} exceeds 2**{RLLIB_WORKER_SHIFT} envs per worker')
    off = (w << RLLIB_WORKER_SHIFT) + v * num_envs
    # bioim_set_env_offset takes a C int and the kernel forms env_offset + env in 32 bits
    if w < 0 or v < 0 or off + num_envs > (1 << 31) - 1:
        raise ValueError(f'rllib_creator: worker_index {w} / vector_index {v} put the global env index '
                         f'{off} + {num_envs} past 2**31 - 1 (at most {(1 << (31 - RLLIB_WORKER_SHIFT)) - 1} workers)')
    return off


def register_with_gym():
    """gym.register / ray register_env for the built IDs when those packages
    are importable (bioimitation/__init__.py:23-143); returns the IDs
    registered with gym.  The Ray creators are :func:`rllib_creator`'s."""
    done = []
    try:
        from gym.envs.registration import register
        for env_id, cls in ENV_CLASSES.items():
            register(id=env_id, entry_point=f'bioimitation.envs:{cls.__name__}')
            done.append(env_id)
    except Exception:
        pass
    try:
        from ray.tune.registry import register_env
        for env_id in ENV_CLASSES:
            register_env(env_id, rllib_creator(env_id))
    except Exception:
        pass
    return done
