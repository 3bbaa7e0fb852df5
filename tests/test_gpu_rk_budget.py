"""Budgeted steps of the reference integrator (bioim_set_rk_budget,
include/bioim.h): an env whose Kutta-Merson step does not finish within the
launch's attempt budget is suspended at an accepted integration point and
resumed by the next launch.  The consumer feeds each env its own next action
only when it is ready (RLlib BaseEnv.poll / send_actions).  Every env's
trajectory must equal the unbudgeted run's bit for bit."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def _run_sync(env_id, n, T, acts, rows, precision=64):
    import torch
    from bioimitation.vector_env import VectorEnv
    env = VectorEnv(env_id, n, config={'integrator': 'rk-merson'}, precision=precision)
    env.reset(ref_index=rows)
    out = []
    for k in range(T):
        o, r, d, _ = env.step(torch.as_tensor(acts[k], device=env.device, dtype=env.dtype))
        out.append((o.cpu().numpy().copy(), r.cpu().numpy().copy(), d.cpu().numpy().copy()))
    env.close()
    return out


def _run_budget(env_id, n, T, acts, rows, budget, precision=64):
    import torch
    from bioimitation.vector_env import VectorEnv
    env = VectorEnv(env_id, n, config={'integrator': 'rk-merson'}, precision=precision)
    env.set_rk_budget(budget)
    env.reset(ref_index=rows)
    k = np.zeros(n, dtype=int)
    res_o = np.zeros((T, n, env.obs_dim))
    res_r = np.zeros((T, n))
    res_d = np.zeros((T, n), dtype=np.uint8)
    launches = suspended = 0
    ready_total = 0
    fin0 = env.finished_count()
    while k.min() < T and launches < 40 * T:
        a = np.stack([acts[min(k[i], T - 1)][i] for i in range(n)])
        o, r, d, _ = env.step(torch.as_tensor(a, device=env.device, dtype=env.dtype))
        ready = env.ready.cpu().numpy().astype(bool)
        o, r, d = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy()
        for i in np.nonzero(ready & (k < T))[0]:
            res_o[k[i], i], res_r[k[i], i], res_d[k[i], i] = o[i], r[i], d[i]
        suspended += int((~ready).sum())
        ready_total += int(ready.sum())
        k += ready
        launches += 1
    # bioim_finished_count (bench.py's reference-integrator rate) counts exactly the ready rows
    assert env.finished_count() - fin0 == ready_total, (env.finished_count() - fin0, ready_total)
    pending = env.pending_count()
    env.close()
    return res_o, res_r, res_d, launches, suspended, pending, k


@pytest.mark.skipif(not gpu_available(), reason='needs a HIP GPU')
@pytest.mark.parametrize('env_id,budget,precision', [('MuscleRunningImitation3D-v0', 6, 64),
                                                     ('TorqueWalkingImitation2D-v0', 4, 64),
                                                     # fp32 RK kernels through the resume path (the
                                                     # fp32 Muscle2D RK kernel is the one the round-3 gate let
                                                     # carry flagged copies)
                                                     ('MuscleWalkingImitation2D-v0', 6, 32),
                                                     ('TorqueWalkingImitation2D-v0', 4, 32)])
def test_rk_budget_equals_unbudgeted(env_id, budget, precision):
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    n, T = 48, 12
    rng = np.random.default_rng(7)
    rows = rng.integers(0, 100, size=n)
    if pk.nmuscle:
        acts = rng.uniform(0, 0.5, size=(T, n, pk.nact))
    else:
        acts = np.stack([np.array([[pk.ref_q[min(int(r) + k + 1, pk.nrows - 1)][pk.pd_coord[a]] for a in range(pk.nact)]
                                   for r in rows]) for k in range(T)]) + rng.normal(0, 0.05, size=(T, n, pk.nact))
    ref = _run_sync(env_id, n, T, acts, rows, precision)
    o, r, d, launches, suspended, pending, k = _run_budget(env_id, n, T, acts, rows, budget, precision)
    print(f'{env_id} fp{precision}: budget {budget} attempts, {launches} launches for {T} steps, {suspended} suspensions, '
          f'{pending} pending at the end')
    assert (k >= T).all(), k
    assert suspended > 0, 'the budget never suspended an env: the test does not exercise the resume path'
    for t in range(T):
        np.testing.assert_array_equal(o[t], ref[t][0], err_msg=f'obs, step {t}')
        np.testing.assert_array_equal(r[t], ref[t][1], err_msg=f'reward, step {t}')
        np.testing.assert_array_equal(d[t], ref[t][2], err_msg=f'done, step {t}')


@pytest.mark.skipif(not gpu_available(), reason='needs a HIP GPU')
def test_rk_budget_state_roundtrip_clears_pending():
    """set_state starts every env at a step boundary; switching the integrator
    while envs are suspended is refused."""
    import torch
    from bioimitation import _lib
    from bioimitation.vector_env import VectorEnv
    env = VectorEnv('MuscleRunningImitation3D-v0', 32, config={'integrator': 'rk-merson'}, precision=64)
    env.set_rk_budget(1)
    env.reset()
    s = env.get_state()
    env.step(torch.full((32, env.action_dim), 0.3, dtype=torch.float64, device=env.device))
    assert env.pending_count() > 0
    with pytest.raises(_lib.BioimError):
        _lib.check(env._L.bioim_set_integrator(env._h, 0, 0.0))
    # a suspended env's state is not at a step boundary (t is the step's end
    # time, q/u/act/lce an accepted point inside it): get_state refuses it
    with pytest.raises(_lib.BioimError, match='suspended'):
        env.get_state()
    env.set_state(s)
    assert env.pending_count() == 0
    np.testing.assert_array_equal(env.get_state(), s)
    env.close()


def _sync_reference(env_id, n, T, acts, integrator, seed):
    import torch
    from bioimitation.vector_env import VectorEnv
    env = VectorEnv(env_id, n, config={'integrator': integrator}, precision=64, seed=seed)
    o0 = env.reset().cpu().numpy().copy()
    out = []
    for k in range(T):
        o, r, d, _ = env.step(torch.as_tensor(acts[k], device=env.device, dtype=env.dtype))
        out.append((o.cpu().numpy().copy(), r.cpu().numpy().copy(), d.cpu().numpy().copy()))
    env.close()
    return o0, out


@pytest.mark.skipif(not gpu_available(), reason='needs a HIP GPU')
@pytest.mark.parametrize('integrator,env_id', [('rk-merson', 'MuscleRunningImitation3D-v0'),
                                               ('semi-implicit', 'MuscleWalkingImitation2D-v0')])
def test_rllib_base_env_async_equals_sync(integrator, env_id):
    """RLlibBaseEnv driven like RLlib 1.8's sampler (poll, then actions for the
    polled envs only): each env follows its own action sequence and its
    results equal a synchronous run's bit for bit.  Semi-implicit: the runner
    withholds actions from every third env at every other round, so the
    active mask must leave those envs untouched."""
    from bioimitation.adapters import RLlibBaseEnv
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    n, T, seed = 48, 10, 3
    rng = np.random.default_rng(11)
    acts = rng.uniform(0, 0.5, size=(T, n, pk.nact))
    o0, ref = _sync_reference(env_id, n, T, acts, integrator, seed)
    benv = RLlibBaseEnv(env_id, n, config={'integrator': integrator}, seed=seed, rk_budget=5)
    obs, rew, done, info, _ = benv.poll()
    assert sorted(obs) == list(range(n)) and all(rew[i][benv.AGENT] is None for i in range(n))
    np.testing.assert_array_equal(np.stack([obs[i][benv.AGENT] for i in range(n)]), o0)
    k = np.zeros(n, dtype=int)
    waiting = set(range(n))          # polled, not yet sent an action
    rounds = 0
    while k.min() < T and rounds < 60 * T:
        rounds += 1
        send = {i: {benv.AGENT: acts[k[i]][i]} for i in sorted(waiting) if k[i] < T and
                not (integrator == 'semi-implicit' and i % 3 == 0 and rounds % 2 == 0)}
        waiting -= set(send)
        benv.send_actions(send)
        obs, rew, done, info, _ = benv.poll()
        for i, ob in obs.items():
            assert i in send or integrator == 'rk-merson', f'env {i} polled without having been sent an action'
            t = k[i]
            np.testing.assert_array_equal(ob[benv.AGENT], ref[t][0][i], err_msg=f'obs env {i} step {t}')
            assert rew[i][benv.AGENT] == ref[t][1][i] and done[i][benv.AGENT] == bool(ref[t][2][i]), (i, t)
            k[i] += 1
            waiting.add(i)
    print(f'{env_id} ({integrator}): {rounds} rounds for {T} steps per env')
    assert (k >= T).all(), k
    benv.stop()


@pytest.mark.skipif(not gpu_available(), reason='needs a HIP GPU')
def test_mixed_batch_rk_budget_matches_segments_alone():
    """BASELINE config C5 with the reference's integrator in budgeted launches
    (bench.py's reference_integrator leg for --mixed): each segment of a
    MixedVectorEnv carries its own budget and ready rows, and every launch's
    obs / reward / done / ready rows equal the segment stepped alone with the
    same budget, bit for bit, through auto-resets."""
    import torch
    from bioimitation.vector_env import MixedVectorEnv, VectorEnv
    segments = [('MuscleLockedKneeImitation3D-v0', 24), ('MusclePalsyImitation3D-v0', 40)]
    cfg = {'integrator': 'rk-merson'}
    mixed = MixedVectorEnv(segments, config=cfg, precision=64, seed=5, auto_reset=True)
    alone, off = [], 0
    for env_id, n in segments:
        alone.append(VectorEnv(env_id, n, config=cfg, precision=64, seed=5, auto_reset=True, env_offset=off))
        off += n
    for e in mixed.envs + alone:
        e.set_rk_budget(3)
    mixed.reset()
    for e in alone:
        e.reset()
    g = torch.Generator(device='cuda').manual_seed(7)
    suspended = 0
    for t in range(40):
        a = torch.rand((mixed.num_envs, mixed.action_dim), generator=g, device=mixed.device, dtype=mixed.dtype)
        obs, rew, done, _ = mixed.step(a)
        for seg, e, o in zip(mixed.envs, alone, mixed.offsets):
            sl = slice(o, o + e.num_envs)
            eo, er, ed, _ = e.step(a[sl, :e.action_dim].contiguous())
            assert torch.equal(seg.ready, e.ready), t
            ok = e.ready.bool()
            assert torch.equal(obs[sl, :e.obs_dim][ok], eo[ok]) and torch.equal(rew[sl][ok], er[ok]), t
            assert torch.equal(done[sl][ok], ed[ok]), t
            suspended += int((~ok).sum())
    assert suspended > 0          # the budget suspended some steps: the resume path ran
    assert sum(e.reset_count() for e in mixed.envs) == sum(e.reset_count() for e in alone)
    for e in alone + [mixed]:
        e.close()


@pytest.mark.skipif(not gpu_available(), reason='needs a HIP GPU')
def test_rk_counters_wrap_independently():
    """each env's RK evaluation count (low 32 bits of its counter)
    and finished-step count (high 32 bits) wrap on their own.  Seeded just
    below 2**32, the evaluation half wraps after a few steps while the
    finished half counts exactly the finished steps (no carry into it)."""
    import torch
    from bioimitation.vector_env import VectorEnv
    n, T = 64, 3
    runs = []
    for seed_ev in (0, 2**32 - 50):
        env = VectorEnv('MuscleWalkingImitation2D-v0', n, config={'integrator': 'rk-merson'}, precision=64, seed=2)
        env.reset(ref_index=np.arange(n) % 100)
        env.set_rk_counters(seed_ev, 7)
        assert env.finished_count() == 7 * n and env.eval_count() == n * seed_ev
        for t in range(T):
            env.step(torch.full((n, env.action_dim), 0.3, dtype=torch.float64, device=env.device))
        runs.append((env.eval_count(), env.finished_count()))
        env.close()
    (ev0, fin0), (ev1, fin1) = runs
    assert fin0 == fin1 == (7 + T) * n, runs
    assert ev0 > 50 * n                      # every env spent more than 50 evaluations: each low half wrapped once
    assert ev1 == n * (2**32 - 50) + ev0 - n * 2**32, runs
