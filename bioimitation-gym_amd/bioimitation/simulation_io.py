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
(``bioim_set_force_report``).  With the reference's integrator
(config ``integrator='rk-merson'``) the States storage holds, like the
Manager's, the state after the reset and at every accepted Kutta-Merson step
(``bioim_set_state_storage``).  Differences from the reference:
- The Kinematics and ForceReporter analyses get one row per env step
  (0.01 s); OpenSim's analyses record every integration step (step_interval
  1), which would need a realize per accepted step.  With the fixed
  semi-implicit substeps the States storage too has one row per env step.
- ForceReporter columns: each muscle / coordinate actuator (its actuation),
  each Hunt-Crossley force's record entries per geometry — the ground
  platform's (``<force>.ground.force.X..Z``, ``.torque.X..Z``: the six values
  the reference itself reads and negates, opensim_wrapper.py:211-219) and each
  sphere's body (``<force>.<body>.force...``: the force's wrench on that body
  about its origin, in ground, as HuntCrossleyForce::getRecordValues reports a
  geometry's body force [upstream]) — and each CoordinateLimitForce (its
  generalized force).

Column names follow OpenSim 4.1:
- states: ``/jointset/<joint>/<coord>/value``, ``/speed``,
  ``/forceset/<muscle>/activation``, ``/forceset/<muscle>/fiber_length``;
- Kinematics: coordinate names, with rotational coordinates in degrees
  (``inDegrees=yes``).
"""
from __future__ import annotations

import math
import os

import warnings

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
        self._rows = []
        self._force_rows = []
        self._state_rows = []
        self._pending = []

    # rows are formed when read: record() keeps copies of its arguments, so an
    # env step pays for three small copies instead of the row assembly
    # (the single-env facade records every step)
    @property
    def rows(self):
        self._flush()
        return self._rows

    @property
    def force_rows(self):
        self._flush()
        return self._force_rows

    @property
    def state_rows(self):
        self._flush()
        return self._state_rows

    def _flush(self):
        if self._pending:
            pending, self._pending = self._pending, []
            for args in pending:
                self._record_now(*args)

    def _full(self, t, qd, ud, act, lce):
        free = self.dof >= 0
        q = self.default.copy()
        u = np.zeros(self.nc)
        q[free] = qd[self.dof[free]]
        u[free] = ud[self.dof[free]]
        return np.concatenate([[t], q, u, act, lce])

    def record(self, state_row: np.ndarray, qdd: np.ndarray, forces: np.ndarray = None, storage=None):
        """state_row: one env's flat state (include/bioim.h layout);
        qdd: its observation's coordinate_acc block (all coordinates);
        forces: its bioim_set_force_report row; storage: the step's accepted
        integration steps (bioim_set_state_storage rows: t, q, u, activation,
        fiber length in dof order) — the States storage rows of the step
        (default: the step's end state)."""
        if storage is None:
            self._pending.append((np.array(state_row, dtype=np.float64), np.array(qdd, dtype=np.float64),
                                  None if forces is None else np.array(forces, dtype=np.float64)))
            return
        self._flush()
        self._record_now(state_row, qdd, forces, storage)

    def _record_now(self, state_row, qdd, forces=None, storage=None):
        if forces is not None:
            self._force_rows.append(np.concatenate([[float(state_row[0])], np.asarray(forces, dtype=np.float64)]))
        pk = self.pack
        nd, nm = pk.ndof, pk.nmuscle
        t = float(state_row[0])
        qd = state_row[5:5 + nd]
        ud = state_row[5 + nd:5 + 2 * nd]
        act = state_row[5 + 2 * nd:5 + 2 * nd + nm]
        lce = state_row[5 + 2 * nd + nm:5 + 2 * nd + 2 * nm]
        full = self._full(t, qd, ud, act, lce)
        nc = self.nc
        self._rows.append(np.concatenate([full[:1 + 2 * nc], np.asarray(qdd, dtype=np.float64), full[1 + 2 * nc:]]))
        if storage is None:
            self._state_rows.append(full)
        else:
            for r in np.asarray(storage, dtype=np.float64):
                self._state_rows.append(self._full(r[0], r[1:1 + nd], r[1 + nd:1 + 2 * nd], r[1 + 2 * nd:1 + 2 * nd + nm],
                                                  r[1 + 2 * nd + nm:1 + 2 * nd + 2 * nm]))

    def record_steps(self, state_rows, qdd_rows, force_rows):
        """One analysis row and one Manager state row per accepted
        integration step (RK mode): OpenSim's Manager stores the state after
        every accepted step and its analyses (Kinematics, ForceReporter;
        step_interval 1) record at the same states (opensim_wrapper.py:10-15,
        :336).  state_rows: the flat states (include/bioim.h layout) of the
        accepted steps; qdd_rows / force_rows: their realizations."""
        for s, qdd, f in zip(state_rows, qdd_rows, force_rows):
            self.record(s, qdd, f)

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
        nc, nm = self.nc, self.pack.nmuscle
        st = np.array(self.state_rows) if self.state_rows else np.zeros((0, 1 + 2 * nc + 2 * nm))
        st_t, st_q, st_u = st[:, :1], st[:, 1:1 + nc], st[:, 1 + nc:1 + 2 * nc]
        st_a, st_l = st[:, 1 + 2 * nc:1 + 2 * nc + nm], st[:, 1 + 2 * nc + nm:]
        coords = list(self.names['coords'])
        joints = list(self.names.get('coord_joints') or [''] * len(coords))
        rot = np.array(self.names.get('coord_rotational') or [True] * len(coords), dtype=bool)
        muscles = list(self.names['muscles']) if self.pack.nmuscle else []
        # Manager state storage (opensim_wrapper.py:336-337), interleaved per coordinate as OpenSim 4 orders them
        labels, cols = ['time'], [st_t]
        for i, (c, j) in enumerate(zip(coords, joints)):
            labels += [f'/jointset/{j}/{c}/value', f'/jointset/{j}/{c}/speed']
            cols += [st_q[:, i:i + 1], st_u[:, i:i + 1]]
        for i, m in enumerate(muscles):
            labels += [f'/forceset/{m}/activation', f'/forceset/{m}/fiber_length']
            cols += [st_a[:, i:i + 1], st_l[:, i:i + 1]]
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
            # HuntCrossleyForce record (getRecordValues): per geometry in the
            # force's order (platform first, then its spheres, opensim_utils.py:
            # 14-81) the force and torque on that geometry's body, in ground:
            # the platform's body is ground (the negated feet wrench), a
            # sphere's entry is the whole force's wrench on the sphere's body
            # about its origin, i.e. the sum over the force's spheres on it
            bodies = list(self.names['bodies'])
            so = 1 + pk.nact + 6 * pk.ncforce + pk.nlimit   # per-sphere foot-side values
            sph = [(pk.sphere[s].force, pk.sphere[s].obody) for s in range(pk.nsphere)]
            for i, cf in enumerate(self.names['cforces']):
                labels += [f'{cf}.ground.{k}.{x}' for k in ('force', 'torque') for x in 'XYZ']
                cols.append(-fr[:, 1 + pk.nact + 6 * i:1 + pk.nact + 6 * i + 6])    # ground side = -(feet side)
                if fr.shape[1] >= so + 6 * pk.nsphere:
                    for s, (f, ob) in enumerate(sph):
                        if f != i:
                            continue
                        labels += [f'{cf}.{bodies[ob]}.{k}.{x}' for k in ('force', 'torque') for x in 'XYZ']
                        same = [s2 for s2, (f2, ob2) in enumerate(sph) if f2 == i and ob2 == ob]
                        cols.append(sum(fr[:, so + 6 * s2:so + 6 * s2 + 6] for s2 in same))
            o = 1 + pk.nact + 6 * pk.ncforce
            labels += list(self.names['limits'])
            cols.append(fr[:, o:o + pk.nlimit])
            paths['forces'] = os.path.join(base_dir, f'{prefix}_ForceReporter_forces.sto')
            write_sto(paths['forces'], labels, np.hstack(cols), name='ForceReporter_forces')
        return paths

    def _act_coords(self):
        coords = list(self.names['coords'])
        return [coords[self.pack.coordact[a].coord] for a in range(self.pack.nact)]


def split_osim_report(pk, row) -> dict:
    """One env's ``bioim_osim`` report row (include/bioim.h layout) as named
    arrays: time, istep, q/u/qdd (CoordinateSet order), bodies (NOS, 18: pos,
    vel, acc, body-fixed XYZ angles, angular vel, angular acc), com (9: pos,
    vel, acc), muscles (NM, 7: activation, fiber length, fiber velocity, fiber
    force, active fiber force, excitation, tendon force), actuation (NA),
    contact (NF, 6: force, moment on the feet), limits (NL), cot."""
    row = np.asarray(row, dtype=np.float64)
    nc, nb, nm, na, nf, nl = pk.ncoord, pk.nosbody, pk.nmuscle, pk.nact, pk.ncforce, pk.nlimit
    r, k = {'time': float(row[0]), 'istep': int(round(row[1]))}, 2
    for key, n in (('q', nc), ('u', nc), ('qdd', nc)):
        r[key], k = row[k:k + n], k + n
    r['bodies'], k = row[k:k + 18 * nb].reshape(nb, 18), k + 18 * nb
    r['com'], k = row[k:k + 9], k + 9
    r['muscles'], k = row[k:k + 7 * nm].reshape(nm, 7), k + 7 * nm
    r['actuation'], k = row[k:k + na], k + na
    r['contact'], k = row[k:k + 6 * nf].reshape(nf, 6), k + 6 * nf
    r['limits'], k = row[k:k + nl], k + nl
    r['cot'] = float(row[k])
    assert k + 1 == len(row), (k + 1, len(row))
    return r


class _Muscle:
    def __init__(self, name, mu):
        self._name, self._mu = name, mu

    def getName(self):
        return self._name

    def getMaxIsometricForce(self):
        return float(self._mu.fiso)

    def getOptimalFiberLength(self):
        return float(self._mu.lopt)


class _Set(list):
    def getSize(self):
        return len(self)

    def get(self, i):
        return self[i]


class ModelView:
    """The slice of ``opensim.Model`` the task envs read through
    ``osim_model.model`` (getTotalMass, getGravity, getMuscles:
    muscle_walking_imitation_env2D.py:102-113, 360-403), from the ModelPack."""

    def __init__(self, pack, names):
        self._pack, self._names = pack, names

    def getTotalMass(self, state=None):
        return float(self._pack.total_mass)

    def getGravity(self):
        return [float(self._pack.gravity[i]) for i in range(3)]

    def getMuscles(self):
        pk = self._pack
        return _Set(_Muscle(n, pk.muscle[i]) for i, n in enumerate(self._names['muscles'][:pk.nmuscle]))


class OsimModelFacade:
    """``OsimModel`` (opensim_wrapper.py:6-338) over one env of a
    :class:`~bioimitation.vector_env.VectorEnv`: the fields
    (``istep``, ``step_size``, ``action_min/max``, ``coordinate_names``,
    ``muscle_names``, ``is_muscle_model``, ``coordinate_limit_min/max``,
    ``integrator_accuracy``, ``model``), the state calls (``reset``,
    ``set_time``, ``set_coordinates``, ``set_velocities``, ``actuate``,
    ``integrate``), the realizations (``calc_joint_kinematics``,
    ``calc_body_kinematics``, ``calc_muscles_info``, ``calc_forces_info``;
    same dict keys) and ``save_simulation``.  Every call runs on the GPU
    (``bioim_osim``); a realization is cached until the state changes.
    Callers that drive the model directly (tests/example_position_control.py)
    and the env methods (``get_state_dict``, ``get_limit_forces``,
    ``calc_cost_of_transport``) use it."""

    def __init__(self, env, names, action_min, action_max, index=0):
        self._env = env
        self._i = int(index)
        pk = env.pack
        self._pack, self._names = pk, names
        self.step_size = float(pk.step_size)
        self.integrator_accuracy = float(env.integrator_accuracy)
        self.coordinate_names = list(names['coords'])
        self.muscle_names = list(names['muscles']) if pk.nmuscle else []
        self.body_names = list(names['bodies'])
        self.is_muscle_model = pk.nmuscle > 0
        self.action_min, self.action_max = list(action_min), list(action_max)
        self.action_space_size = len(self.action_min)
        # opensim_wrapper.py:30-36: ranges of every coordinate but the pelvis translations
        keep = [c for c, n in enumerate(self.coordinate_names) if n not in ('pelvis_tx', 'pelvis_ty', 'pelvis_tz')]
        self.coordinate_limit_min = [float(pk.coord[c].range_min) for c in keep]
        self.coordinate_limit_max = [float(pk.coord[c].range_max) for c in keep]
        self.coordinate_names_multibody_order = self._multibody_order()
        self.model = ModelView(pk, names)
        self.recorder = TrajectoryRecorder(pk, names)
        self.last_action = None
        self._rep = None
        self._obs = None

    def _multibody_order(self):
        """opensim_wrapper.py:74-90 restated: the key of a coordinate is its
        mobilized body's index (ground 0, then the bodies in BodySet order; a
        composite body's mobilized body is its first OpenSim body) plus an
        offset — the running count, or the coordinate's q index within its
        joint when that is not 0 (the count then advances)."""
        pk, names = self._pack, self._names
        first = {}
        for b in range(pk.nosbody):
            first.setdefault(int(pk.osbody[b].cbody), b)
        joints = names.get('coord_joints') or [None] * len(self.coordinate_names)
        keyed, cnt = {}, 0
        for c, name in enumerate(self.coordinate_names):
            mbix = first.get(int(pk.coord[c].cbody), -1) + 1
            mqix = sum(1 for k in range(c) if joints[k] == joints[c])
            offset = cnt
            if mqix != 0:
                offset = mqix
                cnt += 1
            keyed[mbix + offset] = name
        return [keyed[k] for k in sorted(keyed)]

    # ------------------------------------------------------------ state
    def _dirty(self):
        self._rep = None
        self._obs = None

    def _call(self, op, controls=None):
        import torch
        ctl = None if controls is None else torch.as_tensor(np.asarray(controls, dtype=np.float64).reshape(1, -1))
        rep = self._env.osim(op, [self._i], controls=ctl, want_obs=True)
        self._rep = split_osim_report(self._pack, rep[self._i].double().cpu().numpy())
        self._obs = self._env.obs[self._i].double().cpu().numpy()
        return self._rep

    def report(self):
        """the realized state (split_osim_report), realized on demand"""
        if self._rep is None:
            self._call('realize')
        return self._rep

    def observation(self):
        """the env's observation row at the current state"""
        if self._obs is None:
            self._call('realize')
        return self._obs

    def _state(self):
        return self._env.get_state()

    def _set_state(self, s):
        self._env.set_state(s)
        self._dirty()

    def _edit(self, fn):
        """read-modify-write of this env's flat state row (include/bioim.h), then
        reset_manager (a new integrator + equilibrateMuscles, :287-291)"""
        s = self._state()
        fn(s[self._i])
        self._set_state(s)
        self._call('equilibrate')
        self.recorder.clear()       # the new Manager's state storage starts here (:336) ...
        self._record(stepped=False)  # ... with the initialized state (Manager.initialize)

    @property
    def istep(self):
        return int(self._state()[self._i, 1])

    @property
    def state(self):
        """the flat state row (include/bioim.h layout) standing in for the SimTK::State"""
        return self._state()[self._i]

    def reset(self):
        """opensim_wrapper.py:293-297: initializeState (defaults; the held
        controls stay), time 0, istep 0, reset_manager"""
        pk = self._pack
        nd = pk.ndof

        def f(s):
            s[0] = 0.0
            s[1] = 0
            for c in range(pk.ncoord):
                d = pk.coord[c].dof
                if d >= 0:
                    s[5 + d] = pk.coord[c].default_value
                    s[5 + nd + d] = 0.0
            for m in range(pk.nmuscle):
                s[5 + 2 * nd + m] = pk.muscle[m].default_act
        self._edit(f)

    def set_time(self, t):
        """opensim_wrapper.py:303-307 (istep = int(t / step_size), the float truncation kept)"""
        def f(s):
            s[0] = float(t)
            s[1] = int(float(t) / self.step_size)
        self._edit(f)

    def _set_coords(self, values: dict, speeds: bool):
        pk, nd = self._pack, self._pack.ndof

        def f(s):
            for name, v in values.items():
                c = self.coordinate_names.index(name)
                d = pk.coord[c].dof
                if d >= 0:              # a locked coordinate ignores setValue
                    s[5 + (nd if speeds else 0) + d] = float(v)
        self._edit(f)

    def set_coordinates(self, q_dict):
        """opensim_wrapper.py:309-319"""
        self._set_coords(q_dict, False)

    def set_velocities(self, u_dict):
        """opensim_wrapper.py:321-332"""
        self._set_coords(u_dict, True)

    def actuate(self, action):
        """opensim_wrapper.py:92-107: NaN -> 0, clip, held as the controls"""
        self._call('realize', controls=action)
        pk, nd, nm, H, na = self._pack, self._pack.ndof, self._pack.nmuscle, self._pack.horizon, self._pack.nact
        self.last_action = self._state()[self._i, 5 + 2 * nd + 2 * nm + H * na + na + 1:][:na].copy()

    def get_last_action(self):
        return self.last_action

    def integrate(self):
        """opensim_wrapper.py:299-301 with the handle's integrator"""
        self._call('integrate')
        self._record()

    def storage(self):
        """the last env step's accepted integration steps (RK; None otherwise).
        A step with more accepted steps than the buffer holds keeps its first
        ``cap`` rows: the rows past them were not recorded on the device, so
        the step warns, counts them in ``storage_truncated_rows`` (reported
        again by save_simulation) and grows the buffer to at least twice its
        size for the later steps.  The step itself is complete (the reference
        just integrates)."""
        env = self._env
        if getattr(env, 'storage_rows', None) is None:
            return None
        k = int(env.storage_count[self._i])
        cap = env.storage_rows.shape[1]
        rows = env.storage_rows[self._i, :min(k, cap)].double().cpu().numpy()
        if k > cap:
            self.storage_truncated_rows = getattr(self, 'storage_truncated_rows', 0) + (k - cap)
            warnings.warn(f'state storage: {k} accepted integration steps in one env step, the buffer held '
                          f'{cap}; the rows after the first {cap} are not recorded (buffer grown to '
                          f'{max(2 * cap, k)} rows for the next steps)', RuntimeWarning)
            env.grow_state_storage(max(2 * cap, k))   # applied before the next step's launch
        return rows

    def _realizer(self, k):
        """a batch of the same model (one env per stored state) on which the
        accepted integration steps are realized; grown on demand.  It carries
        this env's torso push (the PrescribedForce the reference model holds):
        the env's own row of its perturbation table on every scratch row, set
        at each use (the env's table may have been replaced since), and never
        a schedule of its own (``apply_perturbations`` off in its config)."""
        e = self._env
        rz = getattr(self, '_rz', None)
        if rz is None or rz.num_envs < k:
            from .vector_env import VectorEnv
            if rz is not None:
                rz.close()
            cfg = dict(e.config or {}, apply_perturbations=False)
            rz = VectorEnv(e.env_id, max(k, 64), config=cfg, device=e.device.index, precision=e.precision)
            rz.enable_force_report()
            self._rz = rz
        if e.perturbation is not None:
            x, y = e.perturbation
            rz.set_perturbation(x, np.asarray(y)[self._i])
        elif rz.perturbation is not None:
            rz.set_perturbation(None, None)
        return rz

    def analysis_rows(self, storage):
        """(states, q'' rows, ForceReporter rows) at the accepted integration
        steps of the last env step: each stored state (t, q, u, activation,
        fiber length; bioim_set_state_storage) is put into this env's state
        row — so the step's held controls come with it — and realized on a
        scratch batch (bioim_osim realize, the REP kernels), one env per row."""
        pk = self._pack
        nd, nm = pk.ndof, pk.nmuscle
        k = len(storage)
        rz = self._realizer(k)
        S = np.tile(self._state()[self._i], (rz.num_envs, 1))
        st = np.asarray(storage, dtype=np.float64)
        S[:k, 0] = st[:, 0]
        S[:k, 5:5 + 2 * nd + 2 * nm] = st[:, 1:1 + 2 * nd + 2 * nm]   # q u act lce: the same order
        rz.set_state(S)
        rep = rz.osim('realize', list(range(k)), want_obs=False)[:k].double().cpu().numpy()
        qdd = [split_osim_report(pk, r)['qdd'] for r in rep]
        return S[:k], qdd, rz.force_report[:k].double().cpu().numpy()

    def close(self):
        rz = getattr(self, '_rz', None)
        if rz is not None:
            rz.close()
            self._rz = None

    def record_row(self, state_row, qdd, force_row, stepped=True):
        """the analyses' rows of one env step: with the reference's integrator,
        one per accepted integration step (analysis_rows); otherwise the end
        state (one per 0.01 s)"""
        storage = self.storage() if stepped else None
        if storage is not None:
            if len(storage):
                self.recorder.record_steps(*self.analysis_rows(storage))
            return
        self.recorder.record(state_row, qdd, force_row)

    def _record(self, stepped=True):
        """one analysis row: the state, q'' of the realize and the ForceReporter
        row (``bioim_set_force_report``, the same full row ImitationEnv records:
        actuations, feet wrenches, limits and the per-sphere body entries)"""
        env = self._env
        if getattr(env, 'force_report', None) is None:
            env.enable_force_report()
            self._call('realize')          # fills the force row of the current state
        r = self.report()
        self.record_row(self._state()[self._i], r['qdd'], env.force_report[self._i].double().cpu().numpy(), stepped)

    # ------------------------------------------------------------ realizations
    def calc_joint_kinematics(self):
        """opensim_wrapper.py:118-135"""
        r = self.report()
        obs = {'time': r['time'], 'coordinate_pos': {}, 'coordinate_vel': {}, 'coordinate_acc': {}}
        for i, n in enumerate(self.coordinate_names):
            obs['coordinate_pos'][n] = float(r['q'][i])
            obs['coordinate_vel'][n] = float(r['u'][i])
            obs['coordinate_acc'][n] = float(r['qdd'][i])
        return obs

    def calc_body_kinematics(self):
        """opensim_wrapper.py:137-190: origins, body-fixed XYZ angles, ground-frame
        velocities and accelerations per body; the system mass center"""
        r = self.report()
        obs = {'time': r['time']}
        keys = ('body_pos', 'body_vel', 'body_acc', 'body_pos_rot', 'body_vel_rot', 'body_acc_rot')
        for k in keys:
            obs[k] = {}
        for i, n in enumerate(self.body_names):
            b = r['bodies'][i]
            obs['body_pos'][n] = [float(x) for x in b[0:3]]
            obs['body_vel'][n] = [float(x) for x in b[3:6]]
            obs['body_acc'][n] = [float(x) for x in b[6:9]]
            obs['body_pos_rot'][n] = [float(x) for x in b[9:12]]
            obs['body_vel_rot'][n] = [float(x) for x in b[12:15]]
            obs['body_acc_rot'][n] = [float(x) for x in b[15:18]]
        c = r['com']
        obs['body_pos']['center_of_mass'] = [float(x) for x in c[0:3]]
        obs['body_vel']['center_of_mass'] = [float(x) for x in c[3:6]]
        obs['body_acc']['center_of_mass'] = [float(x) for x in c[6:9]]
        return obs

    def calc_forces_info(self):
        """opensim_wrapper.py:192-236: contact_forces = the negated ground-platform
        record (the wrench on the feet), coordinate_limit_forces, and each
        actuator's record value (its actuation) in scalar_actuator_forces"""
        r = self.report()
        obs = {'time': r['time'], 'forces': {}, 'contact_forces': {}, 'coordinate_limit_forces': {},
               'scalar_actuator_forces': {}}
        for i, n in enumerate(self._names['cforces']):
            obs['contact_forces'][n] = [float(x) for x in r['contact'][i]]
        for i, n in enumerate(self._names['limits']):
            obs['coordinate_limit_forces'][n] = float(r['limits'][i])
        anames = self.muscle_names if self.is_muscle_model else list(
            self._names.get('actuators') or [f'{self.coordinate_names[self._pack.coordact[a].coord]}_actuator'
                                              for a in range(self._pack.nact)])
        for a, n in enumerate(anames):
            obs['scalar_actuator_forces'][n] = float(r['actuation'][a])
        return obs

    def calc_muscles_info(self):
        """opensim_wrapper.py:238-259"""
        r = self.report()
        obs = {'time': r['time']}
        if self.is_muscle_model:
            obs['muscles'] = {}
            for i, n in enumerate(self.muscle_names):
                m = r['muscles'][i]
                obs['muscles'][n] = {'activation': float(m[0]), 'fiber_length': float(m[1]),
                                     'fiber_velocity': float(m[2]), 'fiber_force': float(m[3])}
        return obs

    # ------------------------------------------------------------ fields
    def get_action_space_size(self):
        return self.action_space_size

    def get_coordinate_names(self):
        return self.coordinate_names

    def get_coordinate_names_multibody_order(self):
        return self.coordinate_names_multibody_order

    def save_simulation(self, base_dir):
        """Writes simulation_States.sto, simulation_Kinematics_{q,u,dudt}.sto and
        simulation_ForceReporter_forces.sto.  If a state-storage overflow
        dropped accepted integration steps (``storage``), the files miss those
        rows against the reference's: warned again here, with the count."""
        lost = getattr(self, 'storage_truncated_rows', 0)
        if lost:
            warnings.warn(f'save_simulation: {lost} accepted integration steps were not recorded '
                          f'(state-storage overflow); the .sto files miss those rows', RuntimeWarning)
        return self.recorder.write(base_dir)
