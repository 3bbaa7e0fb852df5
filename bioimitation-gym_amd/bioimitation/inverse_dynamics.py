"""Inverse-dynamics primitives on the GPU.

Drop-in for the reference's Boost.Python ``InverseDynamics`` helper
(``bioimitation/imitation_envs/inverse_dynamics/inverse_dynamics.cpp:45-215``).
It has the same method names and the same argument meaning.  The helper loads
a model with its muscles disabled and no controller.  It evaluates, at a
state (t, q, q̇):
- ``calculateGravity``: g;
- ``calculateCoriolis``: c;
- ``multiplyByM``: M·a;
- ``multiplyByMInv``: M⁻¹·τ;
- ``calculateResidualForces``: M q̈ + c − f_applied;
- ``calculateTotalForces``: c − f_applied.

The convention is ``M q̈ + c = g + τ``.  ``f_applied`` is gravity,
Hunt-Crossley contact and coordinate limit forces.  Every call runs
``bioim_id_eval``, a batched HIP kernel over the env's model image.  There is
no CPU path.

The reference takes Simbody Q-order lists.  Here the single-state methods
take lists over all coordinates in CoordinateSet order
(``OsimModel.coordinate_names``).  Locked coordinates are not degrees of
freedom: their input entries are ignored and their outputs are 0.
``eval`` is the batched form on device tensors ``[n][ndof]``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

GRAVITY, CORIOLIS, MULT_M, MULT_MINV, RESIDUAL, TOTAL = range(6)


class InverseDynamics:
    def __init__(self, env_id: str, device: int = 0, precision: int = 64):
        from .vector_env import VectorEnv
        self._env = VectorEnv(env_id, 1, device=device, precision=precision)
        pk = self._env.pack
        self.ndof, self.ncoord = pk.ndof, pk.ncoord
        self.dof = np.array([pk.coord[c].dof for c in range(pk.ncoord)])
        self.device, self.dtype = self._env.device, self._env.dtype
        self._state = None

    # ------------------------------------------------------------ batched
    def eval(self, op, q, u=None, v=None):
        """op in (GRAVITY, CORIOLIS, MULT_M, MULT_MINV, RESIDUAL, TOTAL);
        q, u, v: [n][ndof] tensors (any device/dtype; moved to the env's).
        Returns a [n][ndof] tensor on the env's device."""
        import torch

        def dev(x):
            if x is None:
                return None
            return torch.as_tensor(x).to(device=self.device, dtype=self.dtype).contiguous()
        q, u, v = dev(q), dev(u), dev(v)
        n = q.shape[0]
        assert q.shape == (n, self.ndof)
        out = torch.empty((n, self.ndof), device=self.device, dtype=self.dtype)
        p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        _lib.check(self._env._L.bioim_id_eval(self._env._h, int(op), n, p(q), p(u), p(v), p(out)))
        return out

    # ------------------------------------------------------- reference API
    def _dofs(self, x):
        x = np.asarray(x, dtype=np.float64)
        if x.shape != (self.ncoord,):
            raise ValueError(f'expected {self.ncoord} coordinate values, got {x.shape}')
        out = np.zeros(self.ndof)
        free = self.dof >= 0
        out[self.dof[free]] = x[free]
        return out[None, :]

    def _coords(self, y):
        y = y[0].double().cpu().numpy()
        out = np.zeros(self.ncoord)
        free = self.dof >= 0
        out[free] = y[self.dof[free]]
        return [float(v) for v in out]

    def setStateAndRealizeDynamics(self, t, q, qDot):
        self._state = (float(t), list(q), list(qDot))

    def calculateResidualForces(self, t, q, qDot, qDDot):
        return self._coords(self.eval(RESIDUAL, self._dofs(q), self._dofs(qDot), self._dofs(qDDot)))

    def calculateTotalForces(self, t, q, qDot):
        return self._coords(self.eval(TOTAL, self._dofs(q), self._dofs(qDot)))

    def calculateGravity(self, t, q):
        return self._coords(self.eval(GRAVITY, self._dofs(q)))

    def calculateCoriolis(self, t, q, qDot):
        return self._coords(self.eval(CORIOLIS, self._dofs(q), self._dofs(qDot)))

    def multiplyByM(self, t, q, a):
        return self._coords(self.eval(MULT_M, self._dofs(q), v=self._dofs(a)))

    def multiplyByMInv(self, t, q, tau):
        return self._coords(self.eval(MULT_MINV, self._dofs(q), v=self._dofs(tau)))

    def close(self):
        self._env.close()
