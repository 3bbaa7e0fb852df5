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
