"""``apply_perturbations``: the torso push of every task env.

Reference (``muscle_walking_imitation_env2D.py:83-100``; the same block in
every env class): when ``config['apply_perturbations']`` is set, the env adds
an OpenSim ``PrescribedForce`` on ``/bodyset/torso``.  Its application point
is the body origin (point functions ``Constant(0)``, body frame) and its
force is ``(fx(t), 0, 0)`` in ground, where ``fx`` is a
``PiecewiseConstantFunction`` of simulation time with 100 points on
``linspace(0, 10, 100)``: ``np.random.choice(choices)`` N at the points
where ``fmod(t, 2) > threshold``, 0 elsewhere.  The draw happens once per env
construction from NumPy's global RNG.  ``threshold`` is 1.8 in the planar
muscle envs and 1.5 in every other env; Palsy3D draws from ``[-50, -50]``
(:data:`RULES`).

The HIP step takes a zero-order-hold table per env
(``bioim_set_perturbation``).  :func:`zoh_table` converts the reference's
points into it.

PiecewiseConstantFunction evaluation [upstream, unverifiable offline]: the
value at ``x`` is the y of the first point with ``x_i >= x``, clamped to the
end points.  This is OpenSim's ``findIndex`` convention as we restate it.
The previous-point reading would shift every push 0.101 s earlier; only
:func:`zoh_table` would change.
"""
from __future__ import annotations

import numpy as np

N_POINTS, T_END = 100, 10.0
BODY = 'torso'
_PLANAR_MUSCLE = (1.8, (-50, 50))   # muscle_{walking,running,locked_knee}_imitation_env2D.py:90-93
_OTHER = (1.5, (-50, 50))           # torque_*_imitation_env{2D,3D}.py:91-95, muscle_*_imitation_env3D.py:90-93
# env ID -> (fmod threshold, np.random.choice population)
RULES = {
    'MuscleWalkingImitation2D-v0': _PLANAR_MUSCLE, 'MuscleRunningImitation2D-v0': _PLANAR_MUSCLE,
    'MuscleLockedKneeImitation2D-v0': _PLANAR_MUSCLE, 'MuscleJumpingImitation2D-v0': _PLANAR_MUSCLE,
    'MusclePalsyImitation3D-v0': (1.5, (-50, -50)),   # muscle_palsy_imitation_env3D.py:92-93
}


def rule(env_id):
    return RULES.get(env_id, _OTHER)


def reference_points(env_id, rng=None):
    """The reference's (t, fx) points for ``env_id``, drawing from ``rng``
    exactly as the reference draws from ``np.random``: one
    ``choice(population)`` per pushed point, in time order.  ``rng=None``
    uses NumPy's global RNG, as the reference does, so ``np.random.seed(s)``
    reproduces its schedule."""
    rng = np.random if rng is None else rng
    threshold, population = rule(env_id)
    x = np.linspace(0.0, T_END, N_POINTS, endpoint=True)
    y = np.zeros(N_POINTS)
    for i, t in enumerate(x):
        if np.fmod(t, 2.0) > threshold:
            y[i] = float(rng.choice(list(population)))
    return x, y


def pushed_mask(env_id):
    """Which of the 100 points carry a push (the same for every env of an ID)."""
    x = np.linspace(0.0, T_END, N_POINTS, endpoint=True)
    return np.fmod(x, 2.0) > rule(env_id)[0]


def batch_points(env_id, n_envs, seed=0, env_offset=0):
    """Reference-shaped schedules for a batch: env ``e`` (global index
    ``env_offset + e``) draws from ``RandomState(seed + global index)``, so a
    sharded batch reproduces an unsharded one.  Returns (x [100],
    y [n_envs][100])."""
    x = np.linspace(0.0, T_END, N_POINTS, endpoint=True)
    mask = pushed_mask(env_id)
    population = list(rule(env_id)[1])
    y = np.zeros((n_envs, N_POINTS))
    for e in range(n_envs):
        rs = np.random.RandomState((int(seed) + int(env_offset) + e) % (2 ** 32))
        y[e, mask] = rs.choice(population, size=int(mask.sum()))
    return x, y


def zoh_table(x, y):
    """Reference points -> the device's zero-order-hold table.

    The device holds ``y_tab[k]`` on ``[x_tab[k], x_tab[k+1])`` and ``y_tab[0]``
    before ``x_tab[0]``.  For the next-point convention the value on
    ``(x_{i-1}, x_i]`` is ``y_i``.  So the table is ``(x_0, y_0)`` followed by
    ``(nextafter(x_{i-1}), y_i)``.  ``y`` may be ``[n]`` or ``[n_envs][n]``."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xt = np.concatenate([x[:1], np.nextafter(x[:-1], np.inf)])
    return xt, y


def os_body_index(names: dict, body: str = BODY) -> int:
    """ModelPack OpenSim-body index of ``body`` (the pack's ``names`` record)."""
    bodies = list(names['bodies'])
    if body not in bodies:
        raise ValueError(f'apply_perturbations: the model has no body {body!r}')
    return bodies.index(body)


def force_at(x_tab, y_tab, t):
    """Evaluate a zero-order-hold table at time ``t`` (host-side check)."""
    k = int(np.searchsorted(x_tab, t, side='right')) - 1
    return y_tab[..., max(k, 0)]
