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
