"""Reference-shaped single-env API (bioimitation/envs.py)."""
import random

import numpy as np
import pytest

from conftest import gpu_available


def test_make_dispatch_without_gpu():
    from bioimitation import envs, _lib
    with pytest.raises(KeyError):
        envs.make('NoSuchEnv-v0')
    with pytest.raises(NotImplementedError):
        envs.make('MuscleJumpingImitation3D-v0')
    if not gpu_available():
        with pytest.raises(_lib.BioimError):
            envs.make('MuscleWalkingImitation2D-v0', {'mode': 'test'})


def test_box_stub():
    from bioimitation.envs import Box
    b = Box([0, 0], [1, 2])
    x = b.sample(np.random.default_rng(0))
    assert b.contains(x) and b.shape == (2,)
    assert not b.contains(np.array([2.0, 0.0]))


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
@pytest.mark.parametrize('env_id', ['MuscleWalkingImitation2D-v0', 'TorqueWalkingImitation2D-v0',
                                    'MuscleWalkingImitation3D-v0', 'MusclePalsyImitation3D-v0'])
def test_single_env_matches_oracle(env_id):
    import oracle
    from bioimitation import envs
    from bioimitation.registry import load_pack
    cfg = {'mode': 'train'}
    env = envs.make(env_id, cfg)
    pk = load_pack(env_id, cfg)
    orc = oracle.Oracle(pk)
    bufs = orc.new_envs(1)
    random.seed(3)
    obs = env.reset()
    random.seed(3)
    index = random.randint(0, pk.reset_hi)     # the reference's draw (N/2 or cycle)
    ref = orc.reset(bufs, 0, index)
    np.testing.assert_allclose(obs, ref, rtol=1e-9, atol=1e-9)
    assert env.observation_space.shape == (pk.obs_dim,) and env.action_space.shape == (pk.nact,)
    rng = np.random.default_rng(0)
    for t in range(5):
        a = env.action_space.sample(rng)
        if t == 2:
            a[0] = np.nan
        o, r, d, info = env.step(a)
        ro, rr, rd, rinfo = orc.step(bufs, 0, a)
        np.testing.assert_allclose(o, ro, rtol=1e-7, atol=1e-7)
        assert abs(r - rr) < 1e-7 and d == rd
        assert len(info['all_rewards']) == pk.info_dim
        np.testing.assert_allclose(info['all_rewards'], rinfo, rtol=1e-7, atol=1e-7)
    d = env.step(env.action_space.sample(rng), obs_as_dict=True)[0]      # the reference's nested dict
    assert set(d) >= {'phase', 'coordinate_pos', 'coordinate_vel', 'body_pos'} and len(d['body_pos']) == 10
    env.close()


def test_trajectory_recorder_writes_opensim_storage(tmp_path):
    """save_simulation's files (opensim_wrapper.py:334-338) from recorded
    rows: OpenSim 4 state paths, Kinematics in degrees for rotational
    coordinates, locked coordinates at their defaults.  Host logic only."""
    import math
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    from bioimitation.simulation_io import TrajectoryRecorder
    from bioimitation.storage import read_sto
    env_id = 'MuscleLockedKneeImitation3D-v0'
    pk, names = load_pack(env_id), load_names(env_id)
    rec = TrajectoryRecorder(pk, names)
    rng = np.random.default_rng(0)
    dim = 5 + 2 * pk.ndof + 2 * pk.nmuscle + pk.horizon * pk.nact + pk.nact + 1 + pk.nact
    rows = []
    for k in range(4):
        s = rng.normal(size=dim)
        s[0] = 0.3 + 0.01 * k
        rows.append(s)
        rec.record(s, rng.normal(size=pk.ncoord))
    paths = rec.write(str(tmp_path))
    h, labels, data = read_sto(paths['states'])
    assert data.shape == (4, 1 + 2 * pk.ncoord + 2 * pk.nmuscle)
    c = names['coords'].index('hip_flexion_r')
    j = names['coord_joints'][c]
    col = labels.index(f'/jointset/{j}/hip_flexion_r/value')
    d = pk.coord[c].dof
    np.testing.assert_allclose(data[:, col], [r[5 + d] for r in rows], atol=1e-9)
    locked = names['coords'].index('knee_angle_l')
    assert names['coord_locked'][locked]
    np.testing.assert_allclose(data[:, labels.index(f'/jointset/{names["coord_joints"][locked]}/knee_angle_l/speed')], 0)
    m0 = names['muscles'][0]
    np.testing.assert_allclose(data[:, labels.index(f'/forceset/{m0}/activation')], [r[5 + 2 * pk.ndof] for r in rows])
    hq, lq, dq = read_sto(paths['q'])
    assert hq['inDegrees'] == 'yes' and lq[1:] == names['coords']
    np.testing.assert_allclose(dq[:, 1 + c], data[:, col] * 180 / math.pi, atol=1e-6)
    tx = names['coords'].index('pelvis_tx')
    np.testing.assert_allclose(dq[:, 1 + tx], [r[5 + pk.coord[tx].dof] for r in rows], atol=1e-9)   # metres


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_single_env_save_simulation_and_perturbation(tmp_path):
    """env.osim_model.save_simulation after an episode (tests/sample_rllib_testing.py:71)
    holds the reset row plus one row per step, matching the oracle; and
    apply_perturbations draws its schedule from NumPy's global RNG like the
    reference (np.random.seed reproduces it)."""
    import oracle
    from bioimitation import envs
    from bioimitation.obslayout import load_names
    from bioimitation.perturb import os_body_index, reference_points, zoh_table
    from bioimitation.registry import load_pack
    from bioimitation.storage import read_sto
    env_id = 'TorqueWalkingImitation2D-v0'
    cfg = {'mode': 'train', 'apply_perturbations': True}
    np.random.seed(5)
    env = envs.make(env_id, cfg)
    np.random.seed(5)
    x, y = reference_points(env_id)
    np.testing.assert_array_equal(env._env.perturbation[1][0], y)
    pk = load_pack(env_id, cfg)
    orc = oracle.Oracle(pk)
    bufs = orc.new_envs(1)
    orc.set_perturbation(bufs, 0, os_body_index(load_names(env_id)), *zoh_table(x, y))
    random.seed(1)
    env.reset()
    random.seed(1)
    orc.reset(bufs, 0, random.randint(0, pk.reset_hi))
    states = [orc.get_state(bufs, 0)]
    forces = [orc.force_report(bufs, 0)]
    for t in range(6):
        a = np.array([pk.ref_q[min(env.osim_model.istep + 1, pk.nrows - 1)][pk.pd_coord[i]] for i in range(pk.nact)])
        o, r, d, _ = env.step(a)
        ro, rr, rd, _ = orc.step(bufs, 0, a)
        np.testing.assert_allclose(o, ro, rtol=1e-7, atol=1e-7)
        states.append(orc.get_state(bufs, 0))
        forces.append(orc.force_report(bufs, 0))
    paths = env.osim_model.save_simulation(str(tmp_path))
    # ForceReporter (opensim_wrapper.py:10-15, :338): actuators, per contact force its record entries
    # (the ground platform, then each sphere's body), limit forces
    hf, lf, df = read_sto(paths['forces'])
    fr = np.array(forces)
    na, nf, nl, ns = pk.nact, pk.ncforce, pk.nlimit, pk.nsphere
    assert df.shape == (7, 1 + na + 6 * nf + 6 * ns + nl) and lf[0] == 'time'
    names = load_names(env_id)
    assert lf[1 + na:1 + na + 6] == [f'{names["cforces"][0]}.ground.{k}.{x}' for k in ('force', 'torque')
                                     for x in 'XYZ']
    sph = [(pk.sphere[s].force, pk.sphere[s].obody) for s in range(ns)]
    assert lf[1 + na + 6:1 + na + 12] == [f'{names["cforces"][0]}.{names["bodies"][sph[0][1]]}.{k}.{x}'
                                          for k in ('force', 'torque') for x in 'XYZ']
    so = na + 6 * nf + nl
    want = []
    for f in range(nf):
        want.append(-fr[:, na + 6 * f:na + 6 * f + 6])
        for s, (ff, ob) in enumerate(sph):
            if ff == f:
                want.append(sum(fr[:, so + 6 * s2:so + 6 * s2 + 6] for s2, (f2, o2) in enumerate(sph)
                                if f2 == f and o2 == ob))
    np.testing.assert_allclose(df[:, 1:1 + na], fr[:, :na], rtol=1e-7, atol=1e-6)
    np.testing.assert_allclose(df[:, 1 + na:1 + na + 6 * nf + 6 * ns], np.hstack(want), rtol=1e-6, atol=1e-4)
    np.testing.assert_allclose(df[:, -nl:], fr[:, na + 6 * nf:na + 6 * nf + nl], rtol=1e-6, atol=1e-6)
    ground = np.hstack([want[k] for k in range(len(want)) if k % (1 + ns // nf) == 0])   # the platform entries
    assert np.abs(ground).max() > 1.0                        # feet on the ground
    h, labels, data = read_sto(paths['states'])
    assert data.shape[0] == 7
    np.testing.assert_allclose(data[:, 0], [s[0] for s in states], atol=1e-9)
    c = load_names(env_id)['coords'].index('knee_angle_r')
    col = labels.index('/jointset/knee_r/knee_angle_r/value')
    np.testing.assert_allclose(data[:, col], [s[5 + pk.coord[c].dof] for s in states], atol=1e-8)
    env.close()


def test_rllib_creator_dispatches_on_num_envs(monkeypatch):
    """the Ray creator registered for an ID
    (envs.rllib_creator; bioimitation/__init__.py:135-143 registers
    ``lambda config: Env(config)``) returns the single-env class for the
    reference's configs and one batched RLlibVectorEnv when the env config
    asks for num_envs > 1 (device / precision passed through, the worker
    and vector indices offsetting the global env indices).  Host logic
    only: both constructors are replaced by recorders; ray is not importable
    here, so the RLlib VectorEnv base class (envs._ray_vector_env_class) is
    checked with a stand-in module."""
    from bioimitation import adapters, envs
    calls = []

    class Single:
        def __init__(self, config=None):
            calls.append(('single', dict(config or {})))

    class Vec:
        def __init__(self, env_id, num_envs, config=None, device=0, precision=64, seed=0, env_offset=0):
            calls.append(('vec', env_id, num_envs, dict(config or {}), device, precision, env_offset))

    class EnvContext(dict):          # ray.rllib.env.EnvContext: a dict with worker_index / vector_index
        worker_index = 3
        vector_index = 0

    class EnvContextV(EnvContext):   # the second sub-env of worker 3 (num_envs_per_worker > 1)
        vector_index = 1

    env_id = 'MuscleWalkingImitation2D-v0'
    monkeypatch.setitem(envs.ENV_CLASSES, env_id, Single)
    monkeypatch.setattr(adapters, 'RLlibVectorEnv', Vec)
    create = envs.rllib_creator(env_id)
    create({'mode': 'test'})
    create(EnvContext(num_envs=1, horizon=3))
    create(EnvContext(num_envs=256, device=1, precision=32, horizon=3))
    create(EnvContextV(num_envs=256, horizon=3))
    assert calls[0] == ('single', {'mode': 'test'})
    assert calls[1] == ('single', {'num_envs': 1, 'horizon': 3})
    assert calls[2] == ('vec', env_id, 256, {'horizon': 3}, 1, 32, 3 << envs.RLLIB_WORKER_SHIFT)
    # a worker's vector slots get disjoint env ranges
    assert calls[3] == ('vec', env_id, 256, {'horizon': 3}, 0, 64, (3 << envs.RLLIB_WORKER_SHIFT) + 256)
    with pytest.raises(ValueError):
        envs.rllib_env_offset(EnvContextV(), 1 << envs.RLLIB_WORKER_SHIFT)

    # the global index must fit the C int env_offset
    class EnvContextBig(EnvContext):
        worker_index = 1 << (31 - envs.RLLIB_WORKER_SHIFT)
    last = (1 << (31 - envs.RLLIB_WORKER_SHIFT)) - 1
    class EnvContextLast(EnvContext):
        worker_index = last
    with pytest.raises(ValueError):
        envs.rllib_env_offset(EnvContextBig(), 16)
    assert envs.rllib_env_offset(EnvContextLast(), 16) == last << envs.RLLIB_WORKER_SHIFT
    with pytest.raises(NotImplementedError):
        envs.rllib_creator('MuscleJumpingImitation2D-v0')


def test_rllib_vector_env_class_derives_from_ray(monkeypatch):
    """with ray importable the batched creator's class is also an
    instance of ray.rllib.env.vector_env.VectorEnv (RLlib's env conversion
    dispatches on isinstance).  A stand-in ray module records the base
    class's constructor arguments; no GPU (RLlibVectorEnv's own constructor
    is replaced)."""
    import sys
    import types
    from bioimitation import adapters, envs
    seen = []

    class RayVectorEnv:
        def __init__(self, observation_space, action_space, num_envs):
            seen.append((observation_space, action_space, num_envs))

    mods = {}
    for name in ('ray', 'ray.rllib', 'ray.rllib.env', 'ray.rllib.env.vector_env'):
        mods[name] = types.ModuleType(name)
    mods['ray.rllib.env.vector_env'].VectorEnv = RayVectorEnv
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)

    def fake_init(self, env_id, num_envs, config=None, device=0, precision=64, seed=0, env_offset=0):
        self.num_envs, self.observation_space, self.action_space = num_envs, 'obs', 'act'
    monkeypatch.setattr(adapters.RLlibVectorEnv, '__init__', fake_init)
    cls = envs._ray_vector_env_class()
    assert cls is not None and issubclass(cls, RayVectorEnv) and issubclass(cls, adapters.RLlibVectorEnv)
    v = cls('MuscleWalkingImitation2D-v0', 8)
    assert isinstance(v, RayVectorEnv) and seen == [('obs', 'act', 8)]
    monkeypatch.delitem(sys.modules, 'ray.rllib.env.vector_env')
    monkeypatch.setitem(sys.modules, 'ray', None)
    assert envs._ray_vector_env_class() is None
