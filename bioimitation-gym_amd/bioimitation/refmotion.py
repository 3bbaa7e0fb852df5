"""Reference-motion tables the imitation envs read.

Every env loads ``*_reference_data/task_Kinematics_{q,u}.sto`` and
``task_BodyKinematics_{pos,vel}_global.sto``
(``muscle_walking_imitation_env2D.py:46-53``), produced upstream by an
OpenSim AnalyzeTool run (``data/3D/walking_reference_data/setup_ka.xml``:
Kinematics + BodyKinematics over the IK ``.mot`` with a 6 Hz low-pass).
Those ``.sto`` files are git-ignored in the reference (``.gitignore:18``) and
absent, and the 2D recipe's input (``data/2D/walking_reference_data/setup_ka.xml:70``,
``healthy_gait.sto``) is absent too.

:func:`synthesize_2d_walking` therefore regenerates a 2D walking reference from
the sagittal columns of the shipped 3D IK (``data/3D/inverse_kinematics/task_InverseKinematics.mot``):
6 Hz zero-phase low-pass, degrees to radians (both models share the gait2392
sign conventions: knee flexion negative), pelvis height shifted so the lowest
contact sphere touches the ground at the gait's deepest point, speeds from
the spline derivative, and BodyKinematics (body mass-center positions) from
this package's own forward kinematics.  The result is committed under
``bioimitation/data/2D/walking_reference_data``.
"""
from __future__ import annotations

import math
import os

import numpy as np

from .modelpack import REF_BODIES, raw_forward_kinematics
from .storage import read_sto, resample_linear, write_sto

SAGITTAL_MAP_2D = [  # 2D coordinate <- (3D IK column, sign)
    ('pelvis_tilt', 'pelvis_tilt', 1.0), ('pelvis_tx', 'pelvis_tx', 1.0), ('pelvis_ty', 'pelvis_ty', 1.0),
    ('hip_flexion_r', 'hip_flexion_r', 1.0), ('knee_angle_r', 'knee_angle_r', 1.0),
    ('ankle_angle_r', 'ankle_angle_r', 1.0), ('hip_flexion_l', 'hip_flexion_l', 1.0),
    ('knee_angle_l', 'knee_angle_l', 1.0), ('ankle_angle_l', 'ankle_angle_l', 1.0),
]


def _lowpass(x, dt, fc=6.0):
    from scipy.signal import butter, filtfilt
    b, a = butter(4, fc / (0.5 / dt))
    return filtfilt(b, a, x, axis=0, padtype='odd', padlen=min(3 * max(len(a), len(b)), x.shape[0] - 1))


def _spline_derivative(t, x):
    from scipy.interpolate import CubicSpline
    return CubicSpline(t, x, axis=0)(t, 1)


def lowest_sphere_y(model, qval):
    poses, _ = raw_forward_kinematics(model, qval)
    low = math.inf
    for s in model.spheres:
        R, p = poses[s.body]
        low = min(low, (R @ s.loc + p)[1] - s.radius)
    return low


def body_com_table(model, coord_order, q):
    """Mass-center positions (rows, len(bodies)+1, 3) in REF-style order:
    every body of the model then center_of_mass."""
    bodies = list(model.body_order)
    out = np.zeros((q.shape[0], len(bodies) + 1, 3))
    rot = np.zeros((q.shape[0], len(bodies), 3))
    for r in range(q.shape[0]):
        qv = dict(zip(coord_order, q[r]))
        poses, com = raw_forward_kinematics(model, qv)
        for k, b in enumerate(bodies):
            R, p = poses[b]
            out[r, k] = R @ model.bodies[b].com + p
            # body-fixed XYZ angles (BodyKinematics _Ox/_Oy/_Oz)
            rot[r, k] = [math.atan2(-R[1, 2], R[2, 2]), math.asin(max(-1.0, min(1.0, R[0, 2]))),
                         math.atan2(-R[0, 1], R[0, 0])]
        out[r, -1] = com
    return bodies, out, rot


def synthesize_reference(model, ik_mot_path, out_dir, coord_map=None, penetration=0.01, dt=0.01):
    """The AnalyzeTool recipe of ``setup_ka.xml`` (Kinematics + BodyKinematics
    over the IK ``.mot``, 6 Hz low-pass, ``data/3D/walking_reference_data/setup_ka.xml:72-76``)
    restated on this package's FK, plus one calibration the recipe does not
    have: pelvis_ty is shifted so the deepest contact-sphere penetration over
    the trial is ``penetration`` (the shipped IK puts the feet 2-9 cm into the
    ground plane of the predictive model), and pelvis_tx starts at 0.

    ``coord_map``: [(model coordinate, IK column, sign)]; None = every model
    coordinate from the IK column of the same name.  Locked coordinates keep
    their default value (``Coordinate.setValue`` is a no-op when locked)."""
    header, labels, arr = read_sto(ik_mot_path)
    col = {l: i for i, l in enumerate(labels)}
    t_raw = arr[:, 0]
    coord_order = list(model.coord_order)
    if coord_map is None:
        coord_map = [(c, c, 1.0) for c in coord_order]
    q = np.zeros((arr.shape[0], len(coord_order)))
    for c in coord_order:
        q[:, coord_order.index(c)] = model.coords[c].default_value
    for cm, cik, sign in coord_map:
        if model.coords[cm].locked:
            continue
        v = arr[:, col[cik]]
        if cik not in ('pelvis_tx', 'pelvis_ty', 'pelvis_tz'):
            v = v * math.pi / 180.0
        q[:, coord_order.index(cm)] = sign * v
    t, q = resample_linear(t_raw, q, dt)
    q = _lowpass(q, dt)
    for c in coord_order:
        if model.coords[c].locked:
            q[:, coord_order.index(c)] = model.coords[c].default_value
    ity = coord_order.index('pelvis_ty')
    lows = np.array([lowest_sphere_y(model, dict(zip(coord_order, row))) for row in q])
    q[:, ity] += -penetration - lows.min()
    itx = coord_order.index('pelvis_tx')
    q[:, itx] -= q[0, itx]
    u = _spline_derivative(t, q)
    for c in coord_order:
        if model.coords[c].locked:
            u[:, coord_order.index(c)] = 0.0
    bodies, com, rot = body_com_table(model, coord_order, q)
    vel = _spline_derivative(t, com)
    os.makedirs(out_dir, exist_ok=True)
    write_sto(os.path.join(out_dir, 'task_Kinematics_q.sto'), ['time'] + coord_order,
              np.column_stack([t, q]), name='Coordinates')
    write_sto(os.path.join(out_dir, 'task_Kinematics_u.sto'), ['time'] + coord_order,
              np.column_stack([t, u]), name='Speeds')
    for fname, tab in (('task_BodyKinematics_pos_global.sto', com), ('task_BodyKinematics_vel_global.sto', vel)):
        labs, cols = ['time'], [t]
        for k, b in enumerate(bodies):
            for a, ax in enumerate('XYZ'):
                labs.append(f'{b}_{ax}')
                cols.append(tab[:, k, a])
            for a, ax in enumerate(('Ox', 'Oy', 'Oz')):
                labs.append(f'{b}_{ax}')
                cols.append(rot[:, k, a] if fname.endswith('pos_global.sto') else _spline_derivative(t, rot[:, k, a]))
        for a, ax in enumerate('XYZ'):
            labs.append(f'center_of_mass_{ax}')
            cols.append(tab[:, -1, a])
        write_sto(os.path.join(out_dir, fname), labs, np.column_stack(cols), name='BodyKinematics')
    return t, q, u


def synthesize_2d_walking(model, ik_mot_path, out_dir, penetration=0.01, dt=0.01):
    """2D walking from the sagittal columns of the 3D IK (the 2D recipe's input
    ``healthy_gait.sto`` is absent)."""
    return synthesize_reference(model, ik_mot_path, out_dir, SAGITTAL_MAP_2D, penetration, dt)


def load_reference_tables(ref_dir, coord_order, dt=0.01):
    """Read the four tables the env reads (read_from_storage semantics) and
    return arrays in pack order: time, q/u (CoordinateSet order), x (REF_BODIES order)."""
    from .storage import read_from_storage
    qd = read_from_storage(os.path.join(ref_dir, 'task_Kinematics_q.sto'), dt)
    ud = read_from_storage(os.path.join(ref_dir, 'task_Kinematics_u.sto'), dt)
    xd = read_from_storage(os.path.join(ref_dir, 'task_BodyKinematics_pos_global.sto'), dt)
    n = min(len(qd), len(ud), len(xd))
    q = np.stack([qd[c].to_numpy()[:n] for c in coord_order], axis=1)
    u = np.stack([ud[c].to_numpy()[:n] for c in coord_order], axis=1)
    x = np.zeros((n, len(REF_BODIES), 3))
    for k, b in enumerate(REF_BODIES):
        for a, ax in enumerate('XYZ'):
            x[:, k, a] = xd[f'{b}_{ax}'].to_numpy()[:n]
    return dict(time=qd['time'].to_numpy()[:n], q=q, u=u, x=x)
