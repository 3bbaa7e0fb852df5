"""Consumer adapters around :class:`~bioimitation.vector_env.VectorEnv`
(SURVEY.md 8f rank 3): the step on either side of the HIP path.

The reference trains with RLlib PPO (``configs/train_default.py``:
``observation_filter = "MeanStdFilter"``, one env per rollout worker,
``register_env(ID, lambda config: Env(config))`` in ``bioimitation/__init__.py``)
or with a jaxrl SAC loop (``tests/sample_baselines_training.py:69-91``).
Neither ray nor gym is importable here, so the adapters are duck-typed:

- :class:`RLlibVectorEnv` — RLlib's ``VectorEnv`` protocol (``vector_reset``,
  ``reset_at``, ``vector_step``, ``get_sub_environments``): N envs of one ID
  stepped by one kernel launch; RLlib itself calls ``reset_at`` on done, so
  in-kernel auto-reset is off.
- :class:`GymVectorEnv` — gym's vector-env convention (batched ``reset`` /
  ``step``, finished envs reset automatically and report their reset
  observation, the terminal one in ``infos['final_observation']``): in-kernel
  auto-reset on.  Outputs are fresh tensors (the env's own buffers are
  overwritten by the next launch), so a replay loop may keep them.
- :class:`RLlibBaseEnv` — RLlib's asynchronous ``BaseEnv`` protocol (ray
  1.8, the reference's pin: ``poll`` / ``send_actions`` / ``try_reset``):
  only the envs that received actions step, and with the reference's
  RK-Merson integrator in budgeted launches an env whose step is not
  finished keeps integrating in later launches while the others are polled
  and sent new actions (``VectorEnv.set_rk_budget``).
- :class:`MeanStdFilter` — RLlib's ``MeanStdFilter`` (demean, destd,
  clip 10) as a running mean/variance kept on the GPU and updated from whole
  batches, so normalised observations never leave the device.
"""
from __future__ import annotations

import numpy as np

from .vector_env import VectorEnv


class MeanStdFilter:
    """Running observation normaliser on the device.

    Statistics follow RLlib's ``RunningStat`` (Welford: mean, sum of squared
    deviations ``S``, count ``n``; ``var = S / (n - 1)`` for n > 1, ``mean**2``
    for n == 1) and the filter's output is ``clip((x - mean) / (std + 1e-8),
    -clip, clip)``.  A batch is pushed with Chan's parallel update, which
    equals pushing its rows one by one up to rounding; unlike RLlib, every
    row of a batch is normalised with the statistics after the whole batch."""

    def __init__(self, shape, demean: bool = True, destd: bool = True, clip: float = 10.0, device=None,
                 dtype=None):
        import torch
        self.shape = tuple(shape) if not isinstance(shape, int) else (shape,)
        self.demean, self.destd, self.clip = demean, destd, clip
        self.n = 0
        self.mean = torch.zeros(self.shape, dtype=dtype or torch.float64, device=device)
        self.S = torch.zeros_like(self.mean)

    @property
    def var(self):
        import torch
        if self.n > 1:
            return self.S / (self.n - 1)
        return torch.square(self.mean)

    @property
    def std(self):
        import torch
        return torch.sqrt(self.var)

    def push(self, batch):
        """Add a batch of observations (B, *shape)."""
        import torch
        x = batch.reshape((-1,) + self.shape).to(self.mean.dtype)
        b = x.shape[0]
        if b == 0:
            return
        bm = x.mean(0)
        bS = torch.square(x - bm).sum(0)
        n = self.n + b
        delta = bm - self.mean
        self.mean = self.mean + delta * (b / n)
        self.S = self.S + bS + torch.square(delta) * (self.n * b / n)
        self.n = n

    def __call__(self, batch, update: bool = True):
        import torch
        if update:
            self.push(batch)
        x = batch.to(self.mean.dtype)
        if self.demean:
            x = x - self.mean
        if self.destd:
            x = x / (self.std + 1e-8)
        if self.clip:
            x = torch.clamp(x, -self.clip, self.clip)
        return x.to(batch.dtype)

    def state_dict(self):
        return {'n': self.n, 'mean': self.mean.clone(), 'S': self.S.clone()}

    def load_state_dict(self, d):
        self.n, self.mean, self.S = int(d['n']), d['mean'].clone(), d['S'].clone()


def _spaces(env: VectorEnv):
    from .envs import _box
    pk = env.pack
    if pk.nmuscle:
        lo, hi = [0.0] * pk.nact, [1.0] * pk.nact
    else:
        lo = [pk.coordact[a].min_control for a in range(pk.nact)]
        hi = [pk.coordact[a].max_control for a in range(pk.nact)]
    return _box([-np.inf] * env.obs_dim, [np.inf] * env.obs_dim), _box(lo, hi)


class RLlibVectorEnv:
    """RLlib ``VectorEnv`` protocol over one batched HIP env (numpy I/O, as
    RLlib's sampler expects).  ``reset_at`` resets one env on the device
    (``random.randint``-equivalent row drawn by the kernel's counter RNG)."""

    def __init__(self, env_id: str, num_envs: int, config: dict = None, device: int = 0, precision: int = 64,
                 seed: int = 0, env_offset: int = 0):
        self.env = VectorEnv(env_id, num_envs, config=config, device=device, precision=precision, seed=seed,
                             auto_reset=False, env_offset=env_offset)
        self.num_envs = num_envs
        self.observation_space, self.action_space = _spaces(self.env)
        # pinned host mirrors: the actions go up, and reward, done and info
        # come back, in asynchronous copies on the env's stream; the
        # observation's blocking copy then waits for all of them (one wait
        # per step instead of four)
        import torch
        e, dt = self.env, self.env.dtype
        pin = dict(dtype=dt, pin_memory=True)
        self._act = (torch.zeros((num_envs, e.action_dim), dtype=dt, device=e.device),
                     torch.zeros((num_envs, e.action_dim), **pin))
        self._host = (torch.zeros(num_envs, **pin), torch.zeros(num_envs, dtype=torch.uint8, pin_memory=True),
                      torch.zeros((num_envs, e.info_dim), **pin))

    def vector_reset(self):
        return list(self.env.reset().double().cpu().numpy())

    def reset_at(self, index: int):
        obs = self.env.reset(env_ids=[int(index)])
        return obs[int(index)].double().cpu().numpy()

    def vector_step(self, actions):
        import torch
        e = self.env
        a = np.asarray(actions, dtype=np.float64)
        if a.shape != (self.num_envs, e.action_dim):
            raise ValueError(f'actions must be ({self.num_envs}, {e.action_dim}), got {a.shape}')
        a_dev, a_pin = self._act
        # the last step's copies finished at its synchronize: the pinned buffers are free
        a_pin.numpy()[:] = a
        a_dev.copy_(a_pin, non_blocking=True)
        obs, rew, done, info = e.step(a_dev)
        for h, d in zip(self._host, (rew, done, info)):
            h.copy_(d, non_blocking=True)
        obs = obs.double().cpu().numpy()     # blocking, on the same stream: behind the copies above
        # fresh arrays: RLlib may keep the rows past the next step
        rew, done, info = (h.numpy().astype(np.float64) if h.dtype != torch.uint8 else h.numpy().copy()
                           for h in self._host)
        infos = [{'all_rewards': list(map(float, r))} for r in info]
        return list(obs), list(map(float, rew)), list(map(bool, done)), infos

    def get_sub_environments(self):
        return []

    get_unwrapped = get_sub_environments

    def try_render_at(self, index=None):
        return None

    def close(self):
        self.env.close()


class GymVectorEnv:
    """gym vector-env convention on the device: ``reset() -> obs (N, O)``,
    ``step(actions) -> (obs, rewards, dones, infos)`` with finished envs reset
    in the same kernel launch (their obs row is the post-reset observation;
    ``infos['final_observation']`` holds every env's observation from before
    the reset, i.e. the terminal observation of the done rows, and
    ``infos['_final_observation']`` marks those rows).  Returned tensors are
    copies, safe to store in a replay buffer across steps.
    ``normalize=True`` applies a device :class:`MeanStdFilter` to the
    observations (RLlib's ``observation_filter``); the final observations are
    normalised with the same statistics, without updating them."""

    def __init__(self, env_id: str, num_envs: int, config: dict = None, device: int = 0, precision: int = 64,
                 seed: int = 0, env_offset: int = 0, normalize: bool = False):
        self.env = VectorEnv(env_id, num_envs, config=config, device=device, precision=precision, seed=seed,
                             auto_reset=True, env_offset=env_offset)
        self.env.enable_final_obs()
        self.num_envs = num_envs
        self.single_observation_space, self.single_action_space = _spaces(self.env)
        self.filter = MeanStdFilter(self.env.obs_dim, device=self.env.device) if normalize else None

    def _obs(self, obs, update=True):
        return self.filter(obs, update=update) if self.filter is not None else obs.clone()

    def reset(self):
        return self._obs(self.env.reset())

    def step(self, actions):
        obs, rew, done, info = self.env.step(actions)
        d = done.bool()
        infos = {'all_rewards': info.clone(), 'final_observation': self._obs(self.env.final_obs, update=False),
                 '_final_observation': d.clone()}
        return self._obs(obs), rew.clone(), d, infos

    def close(self):
        self.env.close()


class RLlibBaseEnv:
    """RLlib 1.8 ``BaseEnv`` over one batched HIP env, asynchronous: ``poll()``
    returns the envs whose step (or reset) finished since the last poll,
    ``send_actions()`` steps exactly the envs it names (``bioim_set_active_mask``;
    the others are untouched), ``try_reset()`` resets one env on the device and
    returns its observation.  With ``config['integrator'] = 'rk-merson'`` the
    launches are budgeted (``rk_budget`` attempts per env): an
    env still mid-step after a launch is not polled, ignores new actions and
    resumes in the next launch, bit-identically, so one stiff env never holds
    the others.  Dicts are keyed env index -> {``AGENT``: value}; ``dones``
    carries ``'__all__'`` as RLlib's single-agent wrappers do."""

    AGENT = 'agent0'   # ray.rllib.env.base_env._DUMMY_AGENT_ID (ray 1.8)

    def __init__(self, env_id: str, num_envs: int, config: dict = None, device: int = 0, precision: int = 64,
                 seed: int = 0, env_offset: int = 0, rk_budget: int = 6):
        import torch
        self.env = VectorEnv(env_id, num_envs, config=config, device=device, precision=precision, seed=seed,
                             auto_reset=False, env_offset=env_offset)
        self.num_envs = num_envs
        self.observation_space, self.action_space = _spaces(self.env)
        self.budgeted = self.env.integrator == 'rk-merson' and rk_budget > 0
        if self.budgeted:
            self.env.set_rk_budget(rk_budget)
        dev = self.env.device
        self._active = torch.zeros(num_envs, dtype=torch.uint8, device=dev)
        self.env.set_active_mask(self._active)
        self._actions = torch.zeros((num_envs, self.env.action_dim), dtype=self.env.dtype, device=dev)
        self._fresh = np.zeros(num_envs, dtype=bool)      # results not yet polled
        self._from_reset = np.zeros(num_envs, dtype=bool)
        self._started = False
        # poll(): reward, done and info come back in asynchronous copies into
        # pinned buffers, the observation's blocking copy waits for them
        pin = dict(dtype=self.env.dtype, pin_memory=True)
        self._host = (torch.zeros(num_envs, **pin), torch.zeros(num_envs, dtype=torch.uint8, pin_memory=True),
                      torch.zeros((num_envs, self.env.info_dim), **pin))

    def _outputs(self, ids):
        """host rows ``ids`` of obs, reward, done and info (fresh arrays)"""
        e = self.env
        for h, d in zip(self._host, (e.reward, e.done, e.info)):
            h.copy_(d, non_blocking=True)
        o = e.obs.double().cpu().numpy()     # blocking, on the same stream: behind the copies above
        r, d, f = (h.numpy()[ids].astype(np.float64) for h in self._host)
        return o[ids], r, d, f

    def poll(self):
        if not self._started:
            self.env.reset()
            self._started = True
            self._fresh[:] = True
            self._from_reset[:] = True
        ids = np.nonzero(self._fresh)[0]
        A = self.AGENT
        obs, rew, done, info = {}, {}, {}, {}
        if len(ids):
            o, r, d, f = self._outputs(ids)
            for k, i in enumerate(ids):
                i = int(i)
                obs[i] = {A: o[k]}
                rew[i] = {A: None if self._from_reset[i] else float(r[k])}
                dn = False if self._from_reset[i] else bool(d[k])
                done[i] = {A: dn, '__all__': dn}
                info[i] = {A: {} if self._from_reset[i] else {'all_rewards': list(map(float, f[k]))}}
        self._fresh[:] = False
        self._from_reset[:] = False
        return obs, rew, done, info, {}

    def send_actions(self, action_dict):
        import torch
        ids = [int(i) for i in action_dict]
        if ids:
            a = np.stack([np.asarray(action_dict[i][self.AGENT], dtype=np.float64) for i in ids])
            idx = torch.as_tensor(ids, device=self.env.device)
            self._actions[idx] = torch.as_tensor(a, dtype=self.env.dtype, device=self.env.device)
            self._active[idx] = 1
        for _ in range(1 << 16):    # bounded: a suspended step finishes within its attempt cap
            if self.budgeted:
                self.env.ready.zero_()
            self.env.step(self._actions)
            ready = (self.env.ready if self.budgeted else self._active).bool().cpu().numpy()
            self._active.zero_()
            self._fresh |= ready
            if ready.any() or not self.budgeted or self.env.pending_count() == 0:
                break

    def try_reset(self, env_id):
        i = int(env_id)
        obs = self.env.reset(env_ids=[i])
        self._fresh[i] = False
        return {self.AGENT: obs[i].double().cpu().numpy()}

    def get_sub_environments(self):
        return []

    get_unwrapped = get_sub_environments

    def try_render(self, env_id=None):
        return None

    def stop(self):
        self.env.close()

    close = stop
