"""Consumer adapters (bioimitation/adapters.py): the device MeanStdFilter
against RLlib's RunningStat algorithm restated in numpy (ray is absent:
parity unpinned against ray itself, pinned to its published Welford update
and filter formula), and the RLlib / gym vector-env protocols on the GPU."""
import numpy as np
import pytest

from conftest import gpu_available


class RunningStat:
    """RLlib 1.8 ray/rllib/utils/filter.py RunningStat, one sample at a time."""

    def __init__(self, shape):
        self.n, self.M, self.S = 0, np.zeros(shape), np.zeros(shape)

    def push(self, x):
        self.n += 1
        if self.n == 1:
            self.M[...] = x
        else:
            old = self.M.copy()
            self.M[...] = old + (x - old) / self.n
            self.S[...] = self.S + (x - old) * (x - self.M)

    @property
    def var(self):
        return self.S / (self.n - 1) if self.n > 1 else np.square(self.M)


def test_mean_std_filter_matches_running_stat():
    import torch
    from bioimitation.adapters import MeanStdFilter
    rng = np.random.default_rng(0)
    f = MeanStdFilter(5)
    rs = RunningStat((5,))
    for b in (1, 7, 64, 3):
        x = rng.normal(3.0, 2.0, size=(b, 5)) * np.array([1, 10, 0.1, 1, 5])
        out = f(torch.as_tensor(x)).numpy()
        for row in x:
            rs.push(row)
        np.testing.assert_allclose(f.mean.numpy(), rs.M, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(f.var.numpy(), rs.var, rtol=1e-10, atol=1e-12)
        ref = np.clip((x - rs.M) / (np.sqrt(rs.var) + 1e-8), -10, 10)
        np.testing.assert_allclose(out, ref, rtol=1e-10, atol=1e-10)
    st = f.state_dict()
    g = MeanStdFilter(5)
    g.load_state_dict(st)
    assert g.n == f.n and np.array_equal(g.mean.numpy(), f.mean.numpy())


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_rllib_vector_env_protocol():
    import torch
    from bioimitation.adapters import RLlibVectorEnv
    from bioimitation.vector_env import VectorEnv
    env_id, n = 'MuscleWalkingImitation2D-v0', 8
    venv = RLlibVectorEnv(env_id, n, seed=3)
    ref = VectorEnv(env_id, n, seed=3)
    obs = venv.vector_reset()
    assert len(obs) == n and obs[0].shape == (138,) and venv.action_space.shape == (14,)
    np.testing.assert_array_equal(np.stack(obs), ref.reset().cpu().numpy())
    rng = np.random.default_rng(0)
    kept = None
    for t in range(5):
        a = rng.uniform(0, 1, (n, 14))
        o, r, d, i = venv.vector_step(list(a))
        ro, rr, rd, ri = ref.step(torch.as_tensor(a, device=ref.device))
        np.testing.assert_array_equal(np.stack(o), ro.cpu().numpy())
        assert r == list(map(float, rr.cpu().numpy())) and len(i[0]['all_rewards']) == 5
        assert d == list(map(bool, rd.cpu().numpy()))
        # the rows a step returned are the caller's: the next step (through
        # the same pinned buffers) leaves them alone
        if kept is not None:
            np.testing.assert_array_equal(np.stack(kept[0]), kept[1])
        kept = (o, np.stack(o).copy())
    o3 = venv.reset_at(3)
    assert o3.shape == (138,) and np.isfinite(o3).all()
    venv.close()
    ref.close()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_gym_vector_env_autoreset_and_filter():
    import torch
    from bioimitation.adapters import GymVectorEnv
    venv = GymVectorEnv('TorqueWalkingImitation2D-v0', 64, seed=1, normalize=True)
    obs = venv.reset()
    assert obs.shape == (64, 96) and obs.device.type == 'cuda'
    for t in range(20):
        a = torch.zeros((64, 7), dtype=torch.float64, device=obs.device)
        obs, rew, done, info = venv.step(a)
        assert torch.isfinite(obs).all() and obs.abs().max() <= 10.0
    assert venv.filter.n == 64 * 21
    venv.close()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_gym_vector_env_final_observation_and_copies():
    """Terminal observations survive the in-kernel auto-reset
    (infos['final_observation'], bioim_set_final_obs), equal to what the same
    env produces without auto-reset; outputs are copies, so a replay loop that
    keeps (obs, next_obs) pairs sees distinct tensors."""
    import torch
    from bioimitation.adapters import GymVectorEnv
    from bioimitation.vector_env import VectorEnv
    env_id, n = 'MuscleWalkingImitation2D-v0', 48
    venv = GymVectorEnv(env_id, n, seed=4)
    ref = VectorEnv(env_id, n, seed=4, auto_reset=False)
    venv.reset()
    ref.reset()
    st = venv.env.get_state()
    st[:, 1] = venv.env.pack.n_episode - 1 - (np.arange(n) % 2)      # even envs end on step 1, odd envs on step 2
    st[:, 0] = 0.01 * st[:, 1]
    venv.env.set_state(st)
    ref.set_state(st)
    g = torch.Generator(device='cuda').manual_seed(1)
    kept, live, ndone = [], torch.ones(n, dtype=torch.bool, device=ref.device), 0
    for t in range(2):       # even envs end on step 1, odd envs on step 2
        a = torch.rand((n, venv.env.action_dim), generator=g, device=ref.device, dtype=torch.float64)
        obs, rew, done, info = venv.step(a)
        ro, rr, rd, _ = ref.step(a)
        kept.append(obs)
        lv = live                                  # rows not yet auto-reset in venv: same trajectory as ref
        assert torch.equal(done[lv], rd.bool()[lv]) and torch.equal(rew[lv], rr[lv])
        assert torch.equal(info['final_observation'][lv], ro[lv]), t     # pre-reset obs
        assert torch.equal(info['_final_observation'], done)
        nd = lv & done
        assert torch.equal(obs[lv & ~done], ro[lv & ~done])
        assert nd.any() and not torch.equal(obs[nd], ro[nd])              # done rows hold the reset observation
        assert torch.equal(done, torch.arange(n, device=ref.device) % 2 == t)
        ndone += int(nd.sum())
        live = live & ~done
    assert ndone == n and not torch.equal(kept[0], kept[1])
    venv.close()
    ref.close()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_launch_follows_the_callers_stream():
    """A step issued under `with torch.cuda.stream(s)` runs on s (the handle
    is re-bound), so work queued on s before it is ordered before it."""
    import torch
    from bioimitation.vector_env import VectorEnv
    env_id, n = 'TorqueWalkingImitation2D-v0', 32
    a_env, b_env = VectorEnv(env_id, n, seed=2), VectorEnv(env_id, n, seed=2)
    a_env.reset()
    b_env.reset()
    s = torch.cuda.Stream()
    acts = torch.zeros((n, 7), dtype=torch.float64, device=a_env.device)
    with torch.cuda.stream(s):
        big = torch.randn((4096, 4096), device=a_env.device)
        for _ in range(4):
            big = big @ big.T / 64.0                 # a slow producer on s
        acts_s = acts + 0.1 + 0 * big[0, 0].clamp(-1, 1)   # the action depends on it
        o_s = b_env.step(acts_s)[0].clone()
        assert b_env._stream == s.cuda_stream
    o = a_env.step(acts + 0.1)[0].clone()
    torch.cuda.synchronize()
    assert torch.equal(o, o_s)
    a_env.close()
    b_env.close()
