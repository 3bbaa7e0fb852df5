"""The OsimModel facade (bioimitation.simulation_io.OsimModelFacade) and the
task envs' public methods, host logic on the CPU.

The facade's device calls (VectorEnv.osim / get_state / set_state) are
served here by an oracle-backed stand-in (test infrastructure: the fp64 C
oracle's OsimModel restatement, orc_osim_*), so the facade's own logic — the
state edits of reset / set_time / set_coordinates / set_velocities, actuate,
integrate, the report parsing and the reference's dict keys
(opensim_wrapper.py:118-259) — is checked without a GPU.  The same calls on
the HIP path are compared with the oracle in tests/test_gpu_osim.py.
"""
import numpy as np
import pytest


class OracleVectorEnv:
    """VectorEnv's osim / get_state / set_state surface over the oracle."""

    def __init__(self, env_id, n=1, integrator='euler'):
        import torch
        import oracle
        from bioimitation.registry import load_pack
        self.pack = load_pack(env_id)
        self.orc = oracle.Oracle(self.pack)
        self.bufs = self.orc.new_envs(n)
        for i in range(n):
            self.orc.set_integrator(self.bufs, i, integrator, 1e-3)
        self.num_envs = n
        self.integrator_accuracy = 1e-3
        self.obs = torch.zeros((n, self.pack.obs_dim), dtype=torch.float64)
        self.force_report = None
        self.calls = []

    def enable_force_report(self, on=True):
        import torch
        pk = self.pack
        self.force_report = torch.zeros((self.num_envs, pk.nact + 6 * pk.ncforce + pk.nlimit + 6 * pk.nsphere),
                                        dtype=torch.float64) if on else None

    def get_state(self):
        return np.stack([self.orc.get_state(self.bufs, i) for i in range(self.num_envs)])

    def set_state(self, s):
        for i in range(self.num_envs):
            self.orc.set_state(self.bufs, i, s[i])

    def osim(self, op, env_ids, controls=None, want_obs=True):
        import torch
        rep = np.zeros((self.num_envs, self.orc.lib.orc_osim_full_report_dim(self.orc.pk)))
        for k, i in enumerate(env_ids):
            if controls is not None:
                self.orc.osim_actuate(self.bufs, i, np.asarray(controls)[k])
            if op == 'equilibrate':
                self.orc.osim_reset_manager(self.bufs, i)
            elif op == 'integrate':
                self.orc.osim_integrate(self.bufs, i)
            rep[i] = self.orc.osim_report(self.bufs, i)
            if self.force_report is not None:
                self.force_report[i] = torch.as_tensor(self.orc.force_report(self.bufs, i))
            if want_obs:
                self.obs[i] = torch.as_tensor(self.orc.observe(self.bufs, i))
        self.calls.append(op)
        return torch.as_tensor(rep)


def _facade(env_id, integrator='euler'):
    from bioimitation.obslayout import load_names
    from bioimitation.simulation_io import OsimModelFacade
    venv = OracleVectorEnv(env_id, 1, integrator)
    pk = venv.pack
    if pk.nmuscle:
        lo, hi = [0.0] * pk.nact, [1.0] * pk.nact
    else:
        lo = [pk.coordact[a].min_control for a in range(pk.nact)]
        hi = [pk.coordact[a].max_control for a in range(pk.nact)]
    return venv, OsimModelFacade(venv, load_names(env_id), lo, hi)


IDS = ['MuscleWalkingImitation2D-v0', 'TorqueWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0',
       'MuscleLockedKneeImitation3D-v0', 'TorqueWalkingImitation3D-v0']


@pytest.mark.parametrize('env_id', IDS)
def test_reference_reset_body_through_the_facade_equals_env_reset(env_id):
    """The reference's reset body (muscle_walking_imitation_env2D.py:133-156:
    osim_model.reset, set_time(q_d.time[index]), set_coordinates(q_d row),
    set_velocities(u_d row)) driven through the facade gives the state and
    observation of the env-level reset at that row (orc_env_reset, the
    restatement bioim_reset follows)."""
    venv, om = _facade(env_id)
    pk = venv.pack
    names = om.coordinate_names
    ref = venv.orc.new_envs(1)
    for index in (0, 17, pk.reset_hi):
        om.reset()
        assert om.istep == 0
        om.set_time(pk.ref_time[index])
        om.set_coordinates({n: pk.ref_q[index][c] for c, n in enumerate(names)})
        om.set_velocities({n: pk.ref_u[index][c] for c, n in enumerate(names)})
        obs = om.observation()
        want = venv.orc.reset(ref, 0, index)
        s, w = venv.get_state()[0], venv.orc.get_state(ref, 0)
        nd, nm = pk.ndof, pk.nmuscle
        sl = slice(0, 5 + 2 * nd + 2 * nm)
        keep = np.ones(sl.stop, bool)
        keep[2] = keep[4] = False        # has_last / done are env-level (the env's reset clears them)
        np.testing.assert_allclose(s[sl][keep], w[sl][keep], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(obs, want, rtol=1e-12, atol=1e-12)
        assert om.istep == pk.ref_istep[index]


def test_facade_dict_keys_follow_the_reference():
    """calc_* dicts carry opensim_wrapper.py's keys: joint kinematics per
    coordinate (:118-135), six body dicts over every body plus the mass center
    in pos/vel/acc (:137-190), forces by kind (:192-236), four values per
    muscle (:238-259)."""
    env_id = 'MuscleWalkingImitation2D-v0'
    venv, om = _facade(env_id)
    venv.orc.reset(venv.bufs, 0, 40)
    om._dirty()
    jk = om.calc_joint_kinematics()
    assert set(jk) == {'time', 'coordinate_pos', 'coordinate_vel', 'coordinate_acc'}
    assert list(jk['coordinate_pos']) == om.coordinate_names
    bk = om.calc_body_kinematics()
    assert set(bk) == {'time', 'body_pos', 'body_vel', 'body_acc', 'body_pos_rot', 'body_vel_rot', 'body_acc_rot'}
    for k in ('body_pos', 'body_vel', 'body_acc'):
        assert list(bk[k]) == om.body_names + ['center_of_mass']
    for k in ('body_pos_rot', 'body_vel_rot', 'body_acc_rot'):
        assert list(bk[k]) == om.body_names
    assert all(len(v) == 3 for d in bk.values() if isinstance(d, dict) for v in d.values())
    fi = om.calc_forces_info()
    assert set(fi) == {'time', 'forces', 'contact_forces', 'coordinate_limit_forces', 'scalar_actuator_forces'}
    assert list(fi['contact_forces']) == ['foot_r', 'foot_l'] and all(len(v) == 6 for v in fi['contact_forces'].values())
    assert len(fi['coordinate_limit_forces']) == venv.pack.nlimit
    assert list(fi['scalar_actuator_forces']) == om.muscle_names
    mi = om.calc_muscles_info()
    assert list(mi['muscles']) == om.muscle_names
    assert all(set(v) == {'activation', 'fiber_length', 'fiber_velocity', 'fiber_force'} for v in mi['muscles'].values())
    r = om.report()
    assert r['time'] == venv.pack.ref_time[40] and r['istep'] == venv.pack.ref_istep[40]
    assert om.observation()[0] == pytest.approx((r['istep'] % 132) / 132.0)


def test_observation_dict_keys_match_the_golden_fixture():
    """get_state_dict's nested dict flattens to the reference's own keys
    (tests/golden fixtures record flatten(get_observation_dict()) from the
    reference env classes)."""
    import os
    from bioimitation.obslayout import load_names, obs_to_dict
    env_id = 'MuscleWalkingImitation2D-v0'
    venv, om = _facade(env_id)
    venv.orc.reset(venv.bufs, 0, 12)
    om._dirty()
    d = obs_to_dict(om.observation(), venv.pack, load_names(env_id))
    keys = []

    def walk(prefix, v):
        if isinstance(v, dict):
            for k, x in v.items():
                walk(prefix + (k,), x)
        else:
            keys.append('.'.join(prefix) + ('' if np.ndim(v) == 0 else f'#{len(v)}'))
    walk((), d)
    z = np.load(os.path.join(os.path.dirname(__file__), 'golden', f'{env_id}.npz'), allow_pickle=False)
    assert keys == [str(k) for k in z['ep0_obs_keys']]


@pytest.mark.parametrize('env_id,integrator', [('TorqueWalkingImitation2D-v0', 'euler'),
                                               ('MuscleWalkingImitation2D-v0', 'rk-merson')])
def test_actuate_integrate_and_held_controls(env_id, integrator):
    """OsimModel.actuate clips and holds (get_last_action), integrate advances
    istep and time with the held controls; the recorder gets one row per
    integrate; a later reset keeps the held controls (they are controller
    properties, not state)."""
    venv, om = _facade(env_id, integrator)
    pk = venv.pack
    om.reset()
    om.set_time(pk.ref_time[30])
    om.set_coordinates({n: pk.ref_q[30][c] for c, n in enumerate(om.coordinate_names)})
    om.set_velocities({n: pk.ref_u[30][c] for c, n in enumerate(om.coordinate_names)})
    hi = np.array(om.action_max)
    a = np.linspace(-1.5, 1.5, pk.nact) * hi
    om.actuate(a)
    np.testing.assert_allclose(om.get_last_action(), np.clip(a, om.action_min, om.action_max))
    t0, i0 = om.report()['time'], om.istep
    om.integrate()
    om.integrate()
    assert om.istep == i0 + 2 and om.report()['time'] == pytest.approx(0.01 * (i0 + 2), abs=1e-12)
    assert len(om.recorder.rows) == 1 + 2      # the initialized state (reset_manager), then one per integrate
    held = om.get_last_action().copy()
    om.reset()
    s = venv.get_state()[0]
    np.testing.assert_array_equal(s[-pk.nact:], held)
    nan = a.copy()
    nan[0] = np.nan
    om.actuate(nan)
    np.testing.assert_array_equal(om.get_last_action(), np.zeros(pk.nact))


def test_multibody_order_restatement():
    """opensim_wrapper.py:74-90 restated: on the 2D model the tree order is
    the CoordinateSet order.  On the 3D model the reference's keys
    (mobilized body index + offset) collide — pelvis_rotation's key 3 is
    taken again by hip_adduction_r (femur_r's index 2 + q index 1) — and the
    later coordinate replaces the earlier in its dict, so the list is shorter
    than the CoordinateSet; the restatement keeps that behaviour of the
    reference (its own comment: "This solution might not work always")."""
    venv, om = _facade('MuscleWalkingImitation2D-v0')
    assert om.get_coordinate_names_multibody_order() == om.coordinate_names
    venv, om = _facade('MuscleRunningImitation3D-v0')
    order = om.get_coordinate_names_multibody_order()
    assert order[:6] == ['pelvis_tilt', 'pelvis_list', 'hip_adduction_r', 'hip_rotation_r', 'pelvis_ty', 'pelvis_tz']
    assert len(order) == 14 and set(order) < set(om.coordinate_names)


def test_facade_records_the_full_force_report_row(tmp_path):
    """The facade records the same ForceReporter row the env's step records
    (bioim_set_force_report: actuations, feet wrenches, limits and the
    per-sphere body entries), so a run that mixes facade calls and env steps
    (the reference's tests/example_position_control.py) writes one table with
    the per-body ``<force>.<body>.*`` columns."""
    from bioimitation.storage import read_sto
    venv, om = _facade('MuscleWalkingImitation2D-v0')
    pk = venv.pack
    om.reset()
    om.set_time(pk.ref_time[30])
    om.set_coordinates({n: pk.ref_q[30][c] for c, n in enumerate(om.coordinate_names)})
    om.actuate(np.full(pk.nact, 0.3))
    om.integrate()
    om.integrate()
    width = pk.nact + 6 * pk.ncforce + pk.nlimit + 6 * pk.nsphere
    assert {len(r) for r in om.recorder.force_rows} == {1 + width}
    np.testing.assert_array_equal(om.recorder.force_rows[-1][1:], venv.orc.force_report(venv.bufs, 0))
    paths = om.save_simulation(str(tmp_path))
    h, labels, data = read_sto(paths['forces'])
    assert data.shape[0] == len(om.recorder.force_rows) and np.isfinite(data).all()
    assert any('.calcn_r.force.X' in l for l in labels), labels
