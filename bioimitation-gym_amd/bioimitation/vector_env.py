"""Batched env over the HIP C-ABI: N environments of one registered ID on
one GPU, stepped by one kernel launch.

This is the throughput surface (RLlib ``VectorEnv`` / gym vector-env shaped);
:class:`bioimitation.envs.ImitationEnv` is the single-instance, reference-
shaped surface built on top of it.  Buffers are torch tensors on the GPU;
each launch runs on torch's *current* stream of that device at the time of
the call (the handle is re-bound when the caller switches streams), so it
orders with the caller's torch work.

Aliasing: ``reset()`` and ``step()`` return the env's persistent output
tensors (``self.obs``, ``self.reward``, ``self.done``, ``self.info``), which
the next launch overwrites in place — zero-copy for callers that consume a
step before issuing the next.  Keep a result across steps with ``.clone()``
(the adapters in :mod:`bioimitation.adapters` do).  With auto-reset on, a
done env's row holds its post-reset observation; ``enable_final_obs()``
keeps the terminal one in ``self.final_obs``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .registry import load_pack

INTEGRATORS = {'semi-implicit': 0, 'rk-merson': 1}
OSIM_OPS = {'realize': 0, 'equilibrate': 1, 'integrate': 2}   # include/bioim.h BIOIM_OSIM_*


def check_env_mask(mask, num_envs, device):
    """A per-env mask the step kernel may read: a contiguous (num_envs,)
    uint8/bool tensor on the env's device (or None).  Anything else would
    make the kernel read host memory or past the end of the buffer."""
    import torch
    if mask is None:
        return
    if not isinstance(mask, torch.Tensor):
        raise ValueError('env mask must be a torch tensor (or None)')
    if mask.dtype not in (torch.uint8, torch.bool):
        raise ValueError(f'env mask dtype must be uint8 or bool, got {mask.dtype}')
    if mask.device != torch.device(device):
        raise ValueError(f'env mask must be on {device}, got {mask.device}')
    if mask.dim() != 1 or mask.numel() != num_envs:
        raise ValueError(f'env mask must have shape ({num_envs},), got {tuple(mask.shape)}')
    if not mask.is_contiguous():
        raise ValueError('env mask must be contiguous')


class VectorEnv:
    def __init__(self, env_id: str, num_envs: int, config: dict = None, device: int = 0, precision: int = 64,
                 seed: int = 0, auto_reset: bool = False, env_offset: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise _lib.BioimError('VectorEnv needs a HIP GPU (no CPU fallback)')
        L = _lib.load()
        self.env_id = env_id
        self.config = dict(config or {})
        self.pack = load_pack(env_id, config)
        self.num_envs = int(num_envs)
        self.device = torch.device('cuda', device)
        self.precision = precision
        self.dtype = torch.float32 if precision == 32 else torch.float64
        h = C.c_void_p()
        _lib.check(L.bioim_create(C.byref(self.pack), self.num_envs, device, precision, seed, C.byref(h)))
        self._h = h
        self._L = L
        self._stream = None
        self._bind_stream()
        q = (C.c_int32 * 8)()
        _lib.check(L.bioim_query(h, q))
        self.obs_dim, self.action_dim, self.info_dim, self.lanes_per_env, self.nsub, self.state_dim = \
            q[1], q[2], q[3], q[5], q[6], q[7]
        ql = (C.c_int32 * 5)()
        _lib.check(L.bioim_query_launch(h, ql))
        self.launch = dict(lanes_per_env=ql[0], threads_per_workgroup=ql[1], envs_per_workgroup=ql[2],
                           lds_bytes_per_workgroup=ql[3], workgroups=ql[4])
        _lib.check(L.bioim_set_auto_reset(h, 1 if auto_reset else 0))
        # config 'integrator': 'semi-implicit' (fixed substeps, the default) or 'rk-merson' (the
        # reference's adaptive integrator at 'integrator_accuracy', default the env's 1e-3)
        self.integrator = (config or {}).get('integrator', 'semi-implicit')
        if self.integrator not in INTEGRATORS:
            raise ValueError(f"integrator must be one of {sorted(INTEGRATORS)}, got {self.integrator!r}")
        self.integrator_accuracy = float((config or {}).get('integrator_accuracy', 1e-3))
        _lib.check(L.bioim_set_integrator(h, INTEGRATORS[self.integrator], self.integrator_accuracy))
        _lib.check(L.bioim_set_env_offset(h, int(env_offset)))
        self.env_offset = int(env_offset)
        n = self.num_envs
        self.obs = torch.zeros((n, self.obs_dim), dtype=self.dtype, device=self.device)
        self.reward = torch.zeros(n, dtype=self.dtype, device=self.device)
        self.done = torch.zeros(n, dtype=torch.uint8, device=self.device)
        self.info = torch.zeros((n, self.info_dim), dtype=self.dtype, device=self.device)
        self.final_obs = None
        self.perturbation = None
        if (config or {}).get('apply_perturbations'):
            from .perturb import batch_points
            self.set_perturbation(*batch_points(env_id, n, seed=(config or {}).get('perturbation_seed', seed),
                                                env_offset=env_offset))

    def set_perturbation(self, x, y, body='torso'):
        """apply_perturbations (muscle_walking_imitation_env2D.py:83-100): the
        reference's PiecewiseConstantFunction points ``x`` [n] (shared) and
        ``y`` [num_envs][n] (N) of the ground-x force on ``body``'s origin;
        ``x=None`` removes it.  Converted to the device's zero-order-hold
        table by :func:`bioimitation.perturb.zoh_table`."""
        from .obslayout import load_names
        from .perturb import os_body_index, zoh_table
        if x is None:
            _lib.check(self._L.bioim_set_perturbation(self._h, -1, 0, None, None))
            self.perturbation = None
            return
        xt, yt = zoh_table(x, y)
        yt = np.ascontiguousarray(np.broadcast_to(yt, (self.num_envs, len(xt))), dtype=np.float64)
        ob = os_body_index(load_names(self.env_id), body)
        dp = C.POINTER(C.c_double)
        xt = np.ascontiguousarray(xt)
        _lib.check(self._L.bioim_set_perturbation(self._h, ob, len(xt), xt.ctypes.data_as(dp), yt.ctypes.data_as(dp)))
        self.perturbation = (np.asarray(x, dtype=np.float64), yt)

    def set_reset_table(self, on: bool = True):
        """In-kernel auto-resets from the per-handle reset table (default on;
        bioim_set_reset_table): muscle models with the default step kernels
        read the drawn row's reset state and observation instead of running
        the reset realize in the step launch."""
        _lib.check(self._L.bioim_set_reset_table(self._h, 1 if on else 0))

    @property
    def reset_table_rows(self) -> int:
        """rows of the built reset table (0: not built / not used)"""
        return _lib.check(self._L.bioim_reset_table_rows(self._h))

    def _bind_stream(self):
        """Launch on torch's current stream of the env's device (re-bound
        whenever the caller has switched streams since the last launch)."""
        import torch
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream:
            _lib.check(self._L.bioim_set_stream(self._h, C.c_void_p(s)))
            self._stream = s

    def enable_final_obs(self, on: bool = True):
        """Keep each step's observation from before an in-kernel auto-reset in
        ``self.final_obs`` (N, O): a done env's terminal observation (gym's
        ``final_observation``); equal to ``obs`` for envs that did not reset."""
        import torch
        if on and self.final_obs is None:
            self.final_obs = torch.zeros_like(self.obs)
        elif not on:
            self.final_obs = None
        _lib.check(self._L.bioim_set_final_obs(self._h, self._ptr(self.final_obs)))

    @property
    def force_report_dim(self) -> int:
        """F of the force-report rows (bioim_force_report_dim)"""
        return _lib.check(self._L.bioim_force_report_dim(self._h))

    def enable_force_report(self, on: bool = True, out=None):
        """Per-force-element values of every realized state in
        ``self.force_report`` (N, F), F = bioim_force_report_dim (include/bioim.h);
        ``out``: a contiguous (N, F) tensor of the env's dtype and device to
        write them to instead (e.g. a view of a larger buffer)."""
        import torch
        if on and out is not None:
            f = self.force_report_dim
            if out.shape != (self.num_envs, f) or out.dtype != self.dtype or out.device != self.device \
                    or not out.is_contiguous():
                raise ValueError(f'force report buffer must be a contiguous ({self.num_envs}, {f}) {self.dtype} '
                                 f'tensor on {self.device}')
            self.force_report = out
        elif on and getattr(self, 'force_report', None) is None:
            f = _lib.check(self._L.bioim_force_report_dim(self._h))
            self.force_report = torch.zeros((self.num_envs, f), dtype=self.dtype, device=self.device)
        elif not on:
            self.force_report = None
        _lib.check(self._L.bioim_set_force_report(self._h, self._ptr(self.force_report)))

    def enable_state_storage(self, capacity: int = 64):
        """RK integrator: the state at every accepted integration step of each
        env step in ``self.storage_rows`` (N, capacity, 1 + 2 ndof + 2 nm: t,
        q, u, activation, fiber length) and their number in
        ``self.storage_count`` (bioim_set_state_storage).  ``capacity=0`` turns
        it off."""
        import torch
        if capacity:
            d = 1 + 2 * self.pack.ndof + 2 * self.pack.nmuscle
            self.storage_rows = torch.zeros((self.num_envs, capacity, d), dtype=self.dtype, device=self.device)
            self.storage_count = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        else:
            self.storage_rows = self.storage_count = None
        _lib.check(self._L.bioim_set_state_storage(self._h, self._ptr(self.storage_rows), int(capacity),
                                                   self._ptr(self.storage_count)))
        self._storage_grow = 0

    def grow_state_storage(self, capacity: int):
        """Ask for at least ``capacity`` storage rows from the NEXT ``step()``
        on: the reallocation (which zeroes ``storage_rows`` / ``storage_count``
        for every env of the batch) is deferred to just before that step's
        launch, so every reader of the current step's rows still sees them."""
        self._storage_grow = max(getattr(self, '_storage_grow', 0), int(capacity))

    def _apply_storage_growth(self):
        k = getattr(self, '_storage_grow', 0)
        if k and getattr(self, 'storage_rows', None) is not None and k > self.storage_rows.shape[1]:
            self.enable_state_storage(k)
        self._storage_grow = 0

    def set_rk_budget(self, attempts: int):
        """Budgeted steps for the 'rk-merson' integrator (``bioim_set_rk_budget``):
        each ``step()`` gives every env at most ``attempts`` Kutta-Merson step
        attempts; an env not finished by then resumes in the next ``step()``
        (its action row is ignored until then) and is 0 in ``self.ready``.
        Only ready rows of obs / reward / done / info are fresh.  The
        trajectories equal the unbudgeted run's bit for bit; a launch is no
        longer as long as its stiffest env.  ``attempts=0`` turns it off."""
        import torch
        if self.integrator != 'rk-merson' and attempts:
            raise ValueError("set_rk_budget needs config integrator='rk-merson'")
        self.rk_budget = int(attempts)
        if attempts and getattr(self, 'ready', None) is None:
            self.ready = torch.ones(self.num_envs, dtype=torch.uint8, device=self.device)
        elif not attempts:
            self.ready = None
        _lib.check(self._L.bioim_set_rk_budget(self._h, self.rk_budget, self._ptr(self.ready)))

    def set_active_mask(self, mask):
        """Per-env step mask (``bioim_set_active_mask``): a (N,) uint8 device
        tensor read by every later ``step()``; envs with 0 are left untouched
        unless they are finishing a suspended RK step.  ``None`` steps all.
        The tensor must stay alive while it is set."""
        check_env_mask(mask, self.num_envs, self.device)
        self._active = mask
        _lib.check(self._L.bioim_set_active_mask(self._h, self._ptr(mask)))

    def osim(self, op, env_ids, controls=None, want_obs=True):
        """OsimModel calls on the listed envs (``bioim_osim``): optional
        ``controls`` (n, nact) actuated first (NaN -> 0, clip, held), then op
        'realize' (nothing else), 'equilibrate' (reset_manager: a new integrator
        and the muscles' static fiber equilibrium at the held state) or
        'integrate' (istep += 1, integrate to step_size * istep), then the
        realize.  Returns the report rows (N, bioim_osim_report_dim) — rows of
        the listed envs are fresh — and writes their obs rows into
        ``self.obs`` when ``want_obs``."""
        import torch
        if getattr(self, 'osim_report', None) is None:
            d = _lib.check(self._L.bioim_osim_report_dim(self._h))
            self.osim_report = torch.zeros((self.num_envs, d), dtype=self.dtype, device=self.device)
        ids = self._env_ids(env_ids)
        ctl = None
        if controls is not None:
            ctl = torch.as_tensor(controls, dtype=self.dtype, device=self.device).reshape(ids.numel(), self.action_dim)
            ctl = ctl.contiguous()
        if getattr(self, '_storage_grow', 0):
            self._apply_storage_growth()
        self._bind_stream()
        _lib.check(self._L.bioim_osim(self._h, OSIM_OPS[op], self._ptr(ids), ids.numel(), self._ptr(ctl),
                                      self._ptr(self.obs) if want_obs else None, self._ptr(self.osim_report)))
        return self.osim_report

    def _env_ids(self, env_ids):
        """validated int32 device tensor of env ids: in range (a stray id is an
        out-of-bounds store in the kernel) and distinct (two lane groups would
        race on one env's state)"""
        import torch
        ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).reshape(-1).contiguous()
        if ids.numel():
            h = ids.cpu()
            if int(h.min()) < 0 or int(h.max()) >= self.num_envs:
                raise ValueError(f'env ids must lie in [0, {self.num_envs})')
            if h.unique().numel() != h.numel():
                raise ValueError('env ids must be distinct')
        return ids

    @property
    def build_id(self) -> str:
        """bioim_build_id() of the loaded library (sources + flags hash)"""
        return self._L.bioim_build_id().decode()

    def pending_count(self) -> int:
        """Envs suspended mid-step by the RK budget."""
        return _lib.check(self._L.bioim_pending_count(self._h))

    @staticmethod
    def _ptr(t):
        return C.c_void_p(t.data_ptr()) if t is not None else None

    def set_auto_reset(self, on: bool):
        _lib.check(self._L.bioim_set_auto_reset(self._h, 1 if on else 0))

    def reset(self, env_ids=None, ref_index=None):
        """Reset the listed envs (default all).  ref_index: reference rows
        (default: randint(0, reset_hi) drawn on the device)."""
        import torch
        ids = rows = None
        n = self.num_envs
        if env_ids is not None:
            ids = self._env_ids(env_ids)
            n = ids.numel()
            if n == 0:          # nothing listed: nothing to reset (a null id list would mean every env)
                return self.obs
        if ref_index is not None:
            rows = torch.as_tensor(ref_index, dtype=torch.int32, device=self.device).contiguous()
            if ids is None:
                ids = torch.arange(self.num_envs, dtype=torch.int32, device=self.device)
            assert rows.numel() == n
        self._bind_stream()
        _lib.check(self._L.bioim_reset(self._h, self._ptr(ids), self._ptr(rows), n, self._ptr(self.obs)))
        return self.obs

    def step(self, actions):
        """actions: (N, nact) tensor on the env's device (dtype = precision)."""
        a = actions
        if a.dtype != self.dtype or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=self.dtype).contiguous()
        assert a.shape == (self.num_envs, self.action_dim), a.shape
        if getattr(self, '_storage_grow', 0):
            self._apply_storage_growth()
        self._bind_stream()
        _lib.check(self._L.bioim_step(self._h, self._ptr(a), self._ptr(self.obs), self._ptr(self.reward),
                                      self._ptr(self.done), self._ptr(self.info)))
        return self.obs, self.reward, self.done, self.info

    def get_state(self) -> np.ndarray:
        s = np.zeros((self.num_envs, self.state_dim))
        _lib.check(self._L.bioim_get_state(self._h, s.ctypes.data_as(C.POINTER(C.c_double))))
        return s

    def state_rows(self, out=None):
        """The flat state rows of get_state as a (N, state_dim) float64 device
        tensor, gathered on the env's stream without synchronizing
        (bioim_copy_state): one transfer can carry them with a step's
        outputs."""
        import torch
        if out is None:
            out = torch.empty((self.num_envs, self.state_dim), dtype=torch.float64, device=self.device)
        self._bind_stream()
        _lib.check(self._L.bioim_copy_state(self._h, self._ptr(out)))
        return out

    def set_state(self, s: np.ndarray):
        s = np.ascontiguousarray(s, dtype=np.float64)
        assert s.shape == (self.num_envs, self.state_dim)
        _lib.check(self._L.bioim_set_state(self._h, s.ctypes.data_as(C.POINTER(C.c_double))))

    def reset_count(self) -> int:
        """Resets so far over all envs (explicit + in-kernel auto-resets)."""
        n = C.c_uint64()
        _lib.check(self._L.bioim_reset_count(self._h, C.byref(n)))
        return int(n.value)

    def eval_count(self) -> int:
        """Dynamics evaluations of the adaptive integrator so far over all envs
        (bioim_eval_count)."""
        n = C.c_uint64()
        _lib.check(self._L.bioim_eval_count(self._h, C.byref(n)))
        return int(n.value)

    def finished_count(self) -> int:
        """Env steps the adaptive integrator finished so far over all envs
        (bioim_finished_count: the rows whose ``ready`` was 1)."""
        n = C.c_uint64()
        _lib.check(self._L.bioim_finished_count(self._h, C.byref(n)))
        return int(n.value)

    def set_rk_counters(self, evals: int = 0, finished: int = 0):
        """Set every env's evaluation / finished-step counters
        (bioim_set_rk_counters; 32 bits each per env, wrapping independently)."""
        _lib.check(self._L.bioim_set_rk_counters(self._h, int(evals) & 0xffffffff, int(finished) & 0xffffffff))

    def sync(self):
        _lib.check(self._L.bioim_sync(self._h))

    def close(self):
        if getattr(self, '_h', None):
            self._L.bioim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MixedVectorEnv:
    """A batch of several env IDs on one GPU (BASELINE.json config C5:
    MuscleLockedKneeImitation3D-v0 + MusclePalsyImitation3D-v0), stepped by
    ``bioim_step_group``: segment i owns rows [off_i, off_i + n_i) of padded
    buffers — actions (N, max A), obs (N, max O), info (N, max I) — with
    ``action_mask`` / ``obs_mask`` marking each row's valid columns; one
    launch per segment, in order, on the first segment's stream.
    Device-drawn reset rows are keyed by the global env index (``env_offset``
    + row), as in :class:`VectorEnv`, so the batch reproduces each segment
    stepped alone bit for bit."""

    def __init__(self, segments, config=None, device: int = 0, precision: int = 64, seed: int = 0,
                 auto_reset: bool = False, env_offset: int = 0):
        import torch
        self.envs, off = [], 0
        for env_id, n in segments:
            self.envs.append(VectorEnv(env_id, n, config=config, device=device, precision=precision, seed=seed,
                                       auto_reset=auto_reset, env_offset=env_offset + off))
            off += int(n)
        self.num_envs = off
        self.device, self.dtype, self.precision = self.envs[0].device, self.envs[0].dtype, precision
        self.action_dim = max(e.action_dim for e in self.envs)
        self.obs_dim = max(e.obs_dim for e in self.envs)
        self.info_dim = max(e.info_dim for e in self.envs)
        n, dev = self.num_envs, self.device
        self.obs = torch.zeros((n, self.obs_dim), dtype=self.dtype, device=dev)
        self.reward = torch.zeros(n, dtype=self.dtype, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.info = torch.zeros((n, self.info_dim), dtype=self.dtype, device=dev)
        self.action_mask = torch.zeros((n, self.action_dim), dtype=torch.bool, device=dev)
        self.obs_mask = torch.zeros((n, self.obs_dim), dtype=torch.bool, device=dev)
        self.offsets = []
        off = 0
        for e in self.envs:
            _lib.check(e._L.bioim_set_io_strides(e._h, self.action_dim, self.obs_dim, self.info_dim))
            sl = slice(off, off + e.num_envs)
            e.obs, e.reward, e.done, e.info = self.obs[sl], self.reward[sl], self.done[sl], self.info[sl]
            self.action_mask[sl, :e.action_dim] = True
            self.obs_mask[sl, :e.obs_dim] = True
            self.offsets.append(off)
            off += e.num_envs
        self._hs = (C.c_void_p * len(self.envs))(*[e._h.value for e in self.envs])
        self._L = self.envs[0]._L

    @property
    def build_id(self) -> str:
        return self._L.bioim_build_id().decode()

    @property
    def last_step_fused(self) -> bool:
        """whether the last ``step`` ran as ONE fused two-topology launch
        (bioim_group_fused) rather than one launch per segment"""
        return _lib.check(self._L.bioim_group_fused(self.envs[0]._h)) == 1

    def reset(self):
        for e in self.envs:
            e.reset()
        return self.obs

    def step(self, actions):
        """actions: (N, max A) tensor; columns beyond a row's own action dim are ignored."""
        a = actions
        if a.dtype != self.dtype or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=self.dtype).contiguous()
        assert a.shape == (self.num_envs, self.action_dim), a.shape
        p = VectorEnv._ptr
        self.envs[0]._bind_stream()      # segment 0 launches on it; the others fork from and join into it
        _lib.check(self._L.bioim_step_group(self._hs, len(self.envs), p(a), p(self.obs), p(self.reward),
                                            p(self.done), p(self.info)))
        return self.obs, self.reward, self.done, self.info

    def close(self):
        for e in self.envs:
            e.close()
