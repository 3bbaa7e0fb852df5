"""HIP path (libbioim.so through the C-ABI) vs the fp64 C oracle.

Tolerances (north_star: obs/reward within 1e-4 rel of the fp64 reference):
  - precision 64: free-running, every step, rel 1e-6 (same fp64 math, only
    operation order and transcendental ulps differ);
  - precision 32: per-step re-synced (the oracle state is loaded into the GPU
    before every step) rel 1e-4 of max(|x|, 1) on obs, reward and info;
    free-running fp32 is reported (error curve) but not bounded, since
    contact transitions amplify fp32 rounding chaotically.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

ENV_IDS = ['MuscleWalkingImitation2D-v0', 'TorqueWalkingImitation2D-v0']
QUIRK_ROWS = [0, 29, 58, 59, 116, 117, 132]


def _actions(env_id, rng, n, a_dim, pk, rows=None):
    if 'Muscle' in env_id:
        return rng.uniform(0.0, 1.0, size=(n, a_dim))
    # torque: PD targets near the reference — q_d[istep+1] + N(0, 0.05)
    base = np.array([[pk.ref_q[min(r, pk.nrows - 1)][pk.pd_coord[i]] for i in range(a_dim)] for r in rows])
    return base + rng.normal(0.0, 0.05, size=(n, a_dim))


def _setup(env_id, n, precision, seed=0, config=None):
    import oracle
    from bioimitation.registry import load_pack
    from bioimitation.vector_env import VectorEnv
    pk = load_pack(env_id, config)
    env = VectorEnv(env_id, n, config=config, precision=precision, seed=seed)
    orc = oracle.Oracle(pk)
    bufs = orc.new_envs(n)
    return pk, env, orc, bufs


def _rel(a, b):
    return np.abs(a - b) / np.maximum(1.0, np.abs(b))


@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
@pytest.mark.parametrize('env_id', ENV_IDS)
def test_reset_parity(env_id):
    for precision, tol in ((64, 1e-9), (32, 1e-5)):
        rng = np.random.default_rng(1)
        n = 64
        rows = np.concatenate([QUIRK_ROWS, rng.integers(0, 133, size=n - len(QUIRK_ROWS))])
        pk, env, orc, bufs = _setup(env_id, n, precision)
        obs = env.reset(ref_index=rows).cpu().numpy().astype(np.float64)
        ref = np.stack([orc.reset(bufs, i, int(rows[i])) for i in range(n)])
        assert _rel(obs, ref).max() < tol, (precision, _rel(obs, ref).max(), np.unravel_index(_rel(obs, ref).argmax(), obs.shape))
        st = env.get_state()
        for i in range(n):
            np.testing.assert_allclose(st[i], orc.get_state(bufs, i), rtol=tol, atol=tol)
        env.close()


@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
@pytest.mark.parametrize('env_id', ENV_IDS)
def test_step_parity_fp64_free_running(env_id):
    import torch
    rng = np.random.default_rng(2)
    n, T = 48, 40
    rows = np.concatenate([QUIRK_ROWS, rng.integers(0, 133, size=n - len(QUIRK_ROWS))])
    pk, env, orc, bufs = _setup(env_id, n, 64)
    env.reset(ref_index=rows)
    for i in range(n):
        orc.reset(bufs, i, int(rows[i]))
    alive = np.ones(n, bool)
    worst = 0.0
    for t in range(T):
        st = np.array([orc.get_state(bufs, i)[1] for i in range(n)]).astype(int)
        acts = _actions(env_id, rng, n, env.action_dim, pk, st + 1)
        if t == 5:
            acts[3, 0] = np.nan       # NaN action -> zeros (muscle_walking_imitation_env2D.py:119-121)
        obs, rew, done, info = env.step(torch.as_tensor(acts, device=env.device))
        torch.cuda.synchronize()
        obs, rew, done, info = (x.cpu().numpy() for x in (obs, rew, done, info))
        for i in range(n):
            if not alive[i]:
                continue
            o, r, d, inf = orc.step(bufs, i, acts[i])
            e = max(_rel(obs[i], o).max(), abs(rew[i] - r), _rel(info[i], inf).max())
            assert e < 1e-6, (t, i, e)
            assert bool(done[i]) == d, (t, i)
            worst = max(worst, e)
            if d:
                alive[i] = False
    print(f'{env_id} fp64 free-running {T} steps: max rel err {worst:.2e}')
    env.close()


@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
@pytest.mark.parametrize('env_id', ENV_IDS)
def test_step_parity_fp32_resynced(env_id):
    import torch
    rng = np.random.default_rng(3)
    n, T = 64, 30
    rows = np.concatenate([QUIRK_ROWS, rng.integers(0, 133, size=n - len(QUIRK_ROWS))])
    pk, env, orc, bufs = _setup(env_id, n, 32)
    env.reset(ref_index=rows)
    for i in range(n):
        orc.reset(bufs, i, int(rows[i]))
    worst = {}
    for t in range(T):
        env.set_state(np.stack([orc.get_state(bufs, i) for i in range(n)]))
        st = np.array([orc.get_state(bufs, i)[1] for i in range(n)]).astype(int)
        acts = _actions(env_id, rng, n, env.action_dim, pk, st + 1)
        obs, rew, done, info = env.step(torch.as_tensor(acts, device=env.device, dtype=torch.float32))
        torch.cuda.synchronize()
        obs, rew, done, info = (x.cpu().numpy().astype(np.float64) for x in (obs, rew, done, info))
        for i in range(n):
            o, r, d, inf = orc.step(bufs, i, acts[i].astype(np.float32).astype(np.float64))
            worst['obs'] = max(worst.get('obs', 0), _rel(obs[i], o).max())
            worst['rew'] = max(worst.get('rew', 0), abs(rew[i] - r))
            worst['info'] = max(worst.get('info', 0), _rel(info[i], inf).max())
            if d:   # keep stepping a fresh episode from the oracle's reset
                orc.reset(bufs, i, int(rng.integers(0, 133)))
    print(f'{env_id} fp32 re-synced {T} steps: {worst}')
    assert worst['obs'] < 1e-4 and worst['rew'] < 1e-4 and worst['info'] < 1e-4, worst
    env.close()


@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_auto_reset_and_determinism():
    import torch
    from bioimitation.vector_env import VectorEnv
    env_id, n = 'MuscleWalkingImitation2D-v0', 256
    outs = []
    for rep in range(2):
        env = VectorEnv(env_id, n, precision=32, seed=7, auto_reset=True)
        env.reset()
        g = torch.Generator(device='cuda').manual_seed(0)
        dones = 0
        for t in range(60):
            a = torch.rand((n, env.action_dim), generator=g, device=env.device)
            obs, rew, done, info = env.step(a)
            dones += int(done.sum())
        torch.cuda.synchronize()
        assert torch.isfinite(obs).all()
        outs.append((obs.cpu().numpy().copy(), dones))
        env.close()
    assert outs[0][1] > 0, 'no episode terminated in 60 random-excitation steps'
    np.testing.assert_array_equal(outs[0][0], outs[1][0])   # bitwise reproducible
