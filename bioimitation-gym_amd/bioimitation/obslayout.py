"""Names and layout of the flat observation vector.

The reference builds a nested observation dict in ``get_state_dict``
(``muscle_walking_imitation_env2D.py:158-230``, ``muscle_running_imitation_env3D.py:158-233``)
and ``OsimEnv.get_observation`` flattens it in insertion order
(``opensim_environment.py:52-64``).  The HIP kernel writes the flat vector
directly; this module recovers the dict (``obs_as_dict=True``) and labels
columns (tests, diagnostics).  Names come from the compiled pack's ``names``
record (``tools/build_packs.py``).
"""
from __future__ import annotations

import json
import os

import numpy as np

from .modelpack import OBS_BPOS, OBS_BVEL
from . import packdef as P

TRANS = ('pelvis_tx', 'pelvis_ty', 'pelvis_tz')


def load_names(env_id: str) -> dict:
    """coords / bodies / muscles / cforces / limits names of a committed pack."""
    from .registry import _pack_path
    with np.load(_pack_path(env_id), allow_pickle=False) as z:
        if 'names' not in z.files:
            raise KeyError(f'{env_id}: pack has no names record (rebuild with tools/build_packs.py)')
        return json.loads(str(z['names']))


def obs_layout(pk, names: dict):
    """[(key path, length)] in flat order; the lengths sum to pk.obs_dim."""
    coords = names['coords']
    out = [(('phase',), 1)]
    out += [(('coordinate_pos', c), 1) for c in coords if c not in TRANS]
    out += [(('coordinate_vel', c), 1) for c in coords]
    out += [(('coordinate_acc', c), 1) for c in coords]
    if pk.env_flags & P.ENV_TARGET_OBS:
        out += [(('target_coordinate_pos', c), 1) for c in coords if c != 'pelvis_tx']
        out += [(('target_coordinate_vel', c), 1) for c in coords if c != 'pelvis_tx']
    out += [(('body_pos', b), 3) for b in OBS_BPOS]
    out += [(('body_vel', b), 3) for b in OBS_BVEL]
    for m in (names['muscles'] if pk.nmuscle else []):
        out += [(('muscles', m, k), 1) for k in ('activation', 'fiber_length', 'fiber_velocity')]
    if pk.env_flags & P.ENV_GRF_OBS:
        out += [(('contact_forces', f), 6) for f in names['cforces']]
    n = sum(l for _, l in out)
    if n != pk.obs_dim:
        raise ValueError(f'layout has {n} entries, pack obs_dim {pk.obs_dim}')
    return out


def column_names(pk, names: dict):
    """one dotted label per flat column"""
    cols = []
    for path, n in obs_layout(pk, names):
        base = '.'.join(path)
        cols += [base] if n == 1 else [f'{base}[{i}]' for i in range(n)]
    return cols


def obs_to_dict(obs, pk, names: dict) -> dict:
    """flat observation (obs_dim,) -> the reference's nested observation dict"""
    obs = np.asarray(obs, dtype=np.float64)
    d: dict = {}
    k = 0
    for path, n in obs_layout(pk, names):
        node = d
        for key in path[:-1]:
            node = node.setdefault(key, {})
        node[path[-1]] = float(obs[k]) if n == 1 else [float(x) for x in obs[k:k + n]]
        k += n
    return d
