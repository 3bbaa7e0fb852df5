"""Oracle env semantics vs golden vectors produced by the reference's own env
classes (tests/golden/make_golden.py).  Pins: action smoothing deque, PD law,
NaN handling, actuation clip, obs layout/normalisation, reward and its
components, cost of transport, termination, reset index -> istep quirk,
cross-episode persistence of old_pos_pelvisx, config switches."""
import ast

import numpy as np
import pytest

from bioimitation.registry import load_pack

from bioimitation.registry import RECIPES

GOLDEN = {e: f'tests/golden/{e}.npz' for e in RECIPES}     # every built env ID has fixtures


def episodes(path):
    z = np.load(path, allow_pickle=False)
    n = int(z['n_episodes'])
    for i in range(n):
        yield {k[len(f'ep{i}_'):]: z[k] for k in z.files if k.startswith(f'ep{i}_')}


@pytest.mark.parametrize('env_id', list(GOLDEN))
def test_oracle_matches_reference_env_semantics(env_id, oracle_lib):
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), GOLDEN[env_id])
    envbuf = orc = None
    for ep in episodes(path):
        cfg = ast.literal_eval(str(ep['config']))
        if not ('chained' in ep and orc is not None):
            pk = load_pack(env_id, cfg)
            orc = oracle_lib.Oracle(pk)
            envbuf = orc.new_envs(1)
        obs0 = orc.reset(envbuf, 0, int(ep['index']))
        np.testing.assert_allclose(obs0, ep['obs0'], rtol=1e-12, atol=1e-12)
        for t in range(len(ep['reward'])):
            o, r, d, info = orc.step(envbuf, 0, ep['actions'][t])
            np.testing.assert_allclose(o, ep['obs'][t], rtol=1e-11, atol=1e-11, err_msg=f'obs step {t}')
            assert abs(r - ep['reward'][t]) < 1e-11, (t, r, ep['reward'][t])
            assert d == bool(ep['done'][t])
            np.testing.assert_allclose(info, ep['info'][t], rtol=1e-11, atol=1e-12)


@pytest.mark.parametrize('env_id', list(GOLDEN))
def test_obs_layout_matches_reference_keys(env_id):
    """bioimitation/obslayout.py labels every flat column exactly as the
    reference's flatten(get_observation_dict()) orders its keys, for every
    config the fixtures cover (target obs / GRF switches, horizon)."""
    import os
    from bioimitation.obslayout import column_names, load_names, obs_to_dict
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), GOLDEN[env_id])
    names = load_names(env_id)
    for ep in episodes(path):
        cfg = ast.literal_eval(str(ep['config']))
        pk = load_pack(env_id, cfg)
        ref_cols = []
        for k in ep['obs_keys']:
            k = str(k)
            if '#' in k:
                base, n = k.split('#')
                ref_cols += [f'{base}[{i}]' for i in range(int(n))]
            else:
                ref_cols.append(k)
        assert column_names(pk, names) == ref_cols
        d = obs_to_dict(ep['obs0'], pk, names)
        assert d['phase'] == ep['obs0'][0] and len(d['coordinate_vel']) == pk.ncoord


def test_oracle_matches_reference_config_switches(oracle_lib):
    """tests/golden/config_switches.npz: use_target_obs off, use_GRF off,
    horizons 1..8, r_weights overrides (configs/env_default.py:7-15), run by
    the reference's own env classes; the oracle must reproduce every step."""
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), 'tests/golden/config_switches.npz')
    z = np.load(path, allow_pickle=False)
    assert int(z['n_episodes']) >= 8
    for j in range(int(z['n_episodes'])):
        ep = {k[len(f'ep{j}_'):]: z[k] for k in z.files if k.startswith(f'ep{j}_')}
        env_id, cfg = str(ep['env_id']), ast.literal_eval(str(ep['config']))
        pk = load_pack(env_id, cfg)
        assert pk.obs_dim == ep['obs'].shape[1], (env_id, cfg)
        orc = oracle_lib.Oracle(pk)
        buf = orc.new_envs(1)
        np.testing.assert_allclose(orc.reset(buf, 0, int(ep['index'])), ep['obs0'], rtol=1e-12, atol=1e-12)
        for t in range(len(ep['reward'])):
            o, r, d, info = orc.step(buf, 0, ep['actions'][t])
            np.testing.assert_allclose(o, ep['obs'][t], rtol=1e-11, atol=1e-11, err_msg=f'{env_id} {cfg} step {t}')
            assert abs(r - ep['reward'][t]) < 1e-11 and d == bool(ep['done'][t])
            np.testing.assert_allclose(info, ep['info'][t], rtol=1e-11, atol=1e-12)


def test_perturbation_schedule_and_episodes(oracle_lib):
    """apply_perturbations (muscle_walking_imitation_env2D.py:83-100): the
    reference's own construction (np.random seeded) drew the push schedule
    recorded in tests/golden/perturbations.npz; bioimitation.perturb must draw
    the same points from the same seed, and the oracle with that table must
    replay the reference-driven episodes through the pushes."""
    import os
    from bioimitation.obslayout import load_names
    from bioimitation.perturb import os_body_index, reference_points, zoh_table
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), 'tests/golden/perturbations.npz')
    z = np.load(path, allow_pickle=False)
    for j in range(int(z['n_episodes'])):
        ep = {k[len(f'ep{j}_'):]: z[k] for k in z.files if k.startswith(f'ep{j}_')}
        env_id = str(ep['env_id'])
        np.random.seed(int(ep['np_seed']))
        x, y = reference_points(env_id)
        np.testing.assert_array_equal(x, ep['px'])
        np.testing.assert_array_equal(y, ep['py'])
        assert (y != 0).sum() == (9 if env_id == 'MuscleWalkingImitation2D-v0' else 24)
        ob = os_body_index(load_names(env_id), str(ep['body']))
        cfg = ast.literal_eval(str(ep['config']))
        pk = load_pack(env_id, cfg)
        orc = oracle_lib.Oracle(pk)
        buf = orc.new_envs(1)
        orc.set_perturbation(buf, 0, ob, *zoh_table(x, y))
        obs0 = orc.reset(buf, 0, int(ep['index']))
        np.testing.assert_allclose(obs0, ep['obs0'], rtol=1e-12, atol=1e-12)
        for t in range(len(ep['reward'])):
            o, r, d, info = orc.step(buf, 0, ep['actions'][t])
            np.testing.assert_allclose(o, ep['obs'][t], rtol=1e-11, atol=1e-11, err_msg=f'{env_id} obs step {t}')
            assert abs(r - ep['reward'][t]) < 1e-11 and d == bool(ep['done'][t])


def test_perturbation_changes_the_trajectory(oracle_lib):
    """The push is a real force: the same episode without it diverges once
    t passes the first pushed point (next-point convention, threshold 1.8:
    pushes on (1.717, 1.919])."""
    from bioimitation.perturb import reference_points, zoh_table, force_at
    from bioimitation.obslayout import load_names
    from bioimitation.perturb import os_body_index
    env_id = 'TorqueWalkingImitation2D-v0'
    pk = load_pack(env_id)
    orc = oracle_lib.Oracle(pk)
    x, y = reference_points('MuscleWalkingImitation2D-v0', np.random.RandomState(3))   # threshold 1.8
    xt, yt = zoh_table(x, y)
    assert force_at(xt, yt, 1.70) == 0 and force_at(xt, yt, 1.72) == y[18] and force_at(xt, yt, 1.919) == y[19]
    assert force_at(xt, yt, 1.92) == 0 and force_at(xt, yt, -1.0) == y[0] and force_at(xt, yt, 99.0) == y[-1]
    bufs = orc.new_envs(2)
    orc.set_perturbation(bufs, 1, os_body_index(load_names(env_id)), xt, yt)
    for i in range(2):
        orc.reset(bufs, i, 165)   # t = 1.65
    q = pk.ref_q
    diffs = []
    for t in range(12):
        a = np.array([q[min(166 + t, pk.nrows - 1)][pk.pd_coord[i]] for i in range(pk.nact)])
        o0 = orc.step(bufs, 0, a)[0]
        o1 = orc.step(bufs, 1, a)[0]
        diffs.append(np.abs(o0 - o1).max())
    diffs = np.array(diffs)
    # steps end at t = 1.66 .. 1.77: the realize at t = 1.72 (step 6) is the first to see the push
    assert (diffs[:6] == 0).all() and diffs[6:].min() > 1e-3, diffs
