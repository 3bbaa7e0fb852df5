"""Trajectory recording and ``save_simulation`` (opensim_wrapper.py:334-338).

The reference's ``OsimModel.save_simulation(base_dir)`` writes two things.
The first is the Manager's state storage, ``simulation_States.sto``.  The
second is its analyses' results via ``analysis_set.printResults('simulation',
base_dir)``: the ``Kinematics`` analysis gives ``simulation_Kinematics_q.sto``,
``_u.sto`` and ``_dudt.sto``, and ``ForceReporter`` gives
``simulation_ForceReporter_forces.sto`` (analyses added at
opensim_wrapper.py:10-15).  The Manager and its analyses are re-initialized
at every reset (``reset_manager``, :287-291).  So the files hold the
trajectory since the last reset.

Here the single-env API records the realized state after the reset and after
every step, with the kernel's per-force-element report
(``bioim_set_force_report``).  Differences from the reference:
- One row per env step (0.01 s), not per internal RK-Merson step.
- ForceReporter columns: each muscle / coordinate actuator (its actuation),
  each Hunt-Crossley force's record values on the ground platform
  (``<force>.ground.force.X..Z``, ``.torque.X..Z``: the six values the
  reference itself reads and negates, opensim_wrapper.py:211-219), each
  CoordinateLimitForce (its generalized force).  The contact record's
  foot-side entries are not written (their layout is not pinned here).

Column names follow OpenSim 4.1:
- states: ``/jointset/<joint>/<coord>/value``, ``/speed``,
  ``/forceset/<muscle>/activation``, ``/forceset/<muscle>/fiber_length``;
- Kinematics: coordinate names, with rotational coordinates in degrees
  (``inDegrees=yes``).
"""
from __future__ import annotations

import math
import os

import numpy as np

from .storage import write_sto


class TrajectoryRecorder:
    """Rows of (time, q, u, q'', activation, fiber length) for one env.
    ``q``/``u``/``q''`` are over all coordinates in CoordinateSet order.
    Locked coordinates keep their default value with zero speed."""

    def __init__(self, pack, names: dict):
        self.pack = pack
        self.names = names
        self.nc = pack.ncoord
        self.dof = np.array([pack.coord[c].dof for c in range(self.nc)])
        self.default = np.array([pack.coord[c].default_value for c in range(self.nc)])
        self.clear()

    def clear(self):
        self.rows = []
        self.force_rows = []

    def record(self, state_row: np.ndarray, qdd: np.ndarray, forces: np.ndarray = None):
        """state_row: one env's flat state (include/bioim.h layout);
        qdd: its observation's coordinate_acc block (all coordinates);
        forces: its bioim_set_force_report row."""
        if forces is not None:
            self.force_rows.append(np.concatenate([[float(state_row[0])], np.asarray(forces, dtype=np.float64)]))
        pk = self.pack
        nd, nm = pk.ndof, pk.nmuscle
        t = float(state_row[0])
        qd = state_row[5:5 + nd]
        ud = state_row[5 + nd:5 + 2 * nd]
        act = state_row[5 + 2 * nd:5 + 2 * nd + nm]
        lce = state_row[5 + 2 * nd + nm:5 + 2 * nd + 2 * nm]
        free = self.dof >= 0
        q = self.default.copy()
        u = np.zeros(self.nc)
        q[free] = qd[self.dof[free]]
        u[free] = ud[self.dof[free]]
        self.rows.append(np.concatenate([[t], q, u, np.asarray(qdd, dtype=np.float64), act, lce]))

    # ------------------------------------------------------------------ output
    def _split(self):
        a = np.array(self.rows) if self.rows else np.zeros((0, 1 + 3 * self.nc + 2 * self.pack.nmuscle))
        nc, nm = self.nc, self.pack.nmuscle
        t = a[:, :1]
        q, u, qdd = a[:, 1:1 + nc], a[:, 1 + nc:1 + 2 * nc], a[:, 1 + 2 * nc:1 + 3 * nc]
        act, lce = a[:, 1 + 3 * nc:1 + 3 * nc + nm], a[:, 1 + 3 * nc + nm:]
        return t, q, u, qdd, act, lce

    def write(self, base_dir: str, prefix: str = 'simulation'):
        os.makedirs(base_dir, exist_ok=True)
        t, q, u, qdd, act, lce = self._split()
        coords = list(self.names['coords'])
        joints = list(self.names.get('coord_joints') or [''] * len(coords))
        rot = np.array(self.names.get('coord_rotational') or [True] * len(coords), dtype=bool)
        muscles = list(self.names['muscles']) if self.pack.nmuscle else []
        # Manager state storage (opensim_wrapper.py:336-337), interleaved per coordinate as OpenSim 4 orders them
        labels, cols = ['time'], [t]
        for i, (c, j) in enumerate(zip(coords, joints)):
            labels += [f'/jointset/{j}/{c}/value', f'/jointset/{j}/{c}/speed']
            cols += [q[:, i:i + 1], u[:, i:i + 1]]
        for i, m in enumerate(muscles):
            labels += [f'/forceset/{m}/activation', f'/forceset/{m}/fiber_length']
            cols += [act[:, i:i + 1], lce[:, i:i + 1]]
        paths = {}
        paths['states'] = os.path.join(base_dir, f'{prefix}_States.sto')
        write_sto(paths['states'], labels, np.hstack(cols), name='states')
        # Kinematics analysis (printResults, :338): degrees for rotational coordinates
        scale = np.where(rot, 180.0 / math.pi, 1.0)
        for key, arr in (('q', q), ('u', u), ('dudt', qdd)):
            paths[key] = os.path.join(base_dir, f'{prefix}_Kinematics_{key}.sto')
            write_sto(paths[key], ['time'] + coords, np.hstack([t, arr * scale]), name=f'Kinematics_{key}',
                      in_degrees=True)
        # ForceReporter analysis (printResults, :338)
        if self.force_rows:
            pk = self.pack
            labels = ['time'] + (muscles if pk.nmuscle else list(self.names.get('actuators') or
                                                                  [f'{c}_actuator' for c in self._act_coords()]))
            fr = np.array(self.force_rows)
            cols = [fr[:, :1 + pk.nact]]
            for i, cf in enumerate(self.names['cforces']):
                labels += [f'{cf}.ground.{k}.{x}' for k in ('force', 'torque') for x in 'XYZ']
                cols.append(-fr[:, 1 + pk.nact + 6 * i:1 + pk.nact + 6 * i + 6])    # ground side = -(feet side)
            o = 1 + pk.nact + 6 * pk.ncforce
            labels += list(self.names['limits'])
            cols.append(fr[:, o:o + pk.nlimit])
            paths['forces'] = os.path.join(base_dir, f'{prefix}_ForceReporter_forces.sto')
            write_sto(paths['forces'], labels, np.hstack(cols), name='ForceReporter_forces')
        return paths

    def _act_coords(self):
        coords = list(self.names['coords'])
        return [coords[self.pack.coordact[a].coord] for a in range(self.pack.nact)]


class OsimModelFacade:
    """The slice of ``OsimModel`` (opensim_wrapper.py:6-338) that callers of
    the reference touch from outside the env: ``istep``, ``step_size``,
    ``action_min/max``, ``coordinate_names``, ``muscle_names``,
    ``is_muscle_model``, ``get_action_space_size()`` and
    ``save_simulation(base_dir)`` (tests/sample_rllib_testing.py:71,
    tests/example_position_control.py:312).  It is backed by one env of a
    :class:`~bioimitation.vector_env.VectorEnv`."""

    def __init__(self, env, names, action_min, action_max):
        self._env = env
        self.step_size = float(env.pack.step_size)
        self.coordinate_names = list(names['coords'])
        self.muscle_names = list(names['muscles']) if env.pack.nmuscle else []
        self.is_muscle_model = env.pack.nmuscle > 0
        self.action_min, self.action_max = list(action_min), list(action_max)
        self.recorder = TrajectoryRecorder(env.pack, names)

    @property
    def istep(self):
        return int(self._env.get_state()[0, 1])

    def get_action_space_size(self):
        return len(self.action_min)

    def save_simulation(self, base_dir):
        """Writes simulation_States.sto, simulation_Kinematics_{q,u,dudt}.sto and
        simulation_ForceReporter_forces.sto."""
        return self.recorder.write(base_dir)
