"""Free-running error curve of the GPU step against the fp64 C oracle
(SURVEY.md §8(d) parity run (ii): 200 identical-action steps, no auto-reset,
masked after done; the curve is reported, not bounded, for fp32).

Runs on the GPU box (the oracle here is the checker, never the measured path):
    python tools/error_curve.py --out gpurun_out/error_curve.json
Prints one summary line per env ID and precision; the JSON holds the per-step
curves (max / median relative error over the envs still alive in both runs).
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle')]


def _rel(a, b):
    return np.abs(a - b) / np.maximum(1.0, np.abs(b))


def oracle_run(env_id, n, T, seed):
    """fp64 oracle trajectory and the actions that drove it (mild actions, as
    tests/test_gpu_parity.py::test_parity_200_identical_action_steps)."""
    import oracle
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    bufs = orc.new_envs(n)
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, min(pk.reset_hi, pk.n_episode - T) + 1, size=n)
    for i in range(n):
        orc.reset(bufs, i, int(rows[i]))
    A = pk.nact
    acts = np.zeros((T, n, A))
    obs = np.zeros((T, n, pk.obs_dim))
    rew = np.zeros((T, n))
    done = np.zeros((T, n), bool)
    alive = np.ones(n, bool)
    for t in range(T):
        if 'Muscle' in env_id:
            acts[t] = rng.uniform(0.0, 0.4, size=(n, A))
        else:
            st = np.array([orc.get_state(bufs, i)[1] for i in range(n)]).astype(int) + 1
            acts[t] = np.array([[pk.ref_q[min(r, pk.nrows - 1)][pk.pd_coord[a]] for a in range(A)]
                                for r in st]) + rng.normal(0.0, 0.02, size=(n, A))
        for i in np.where(alive)[0]:
            o, r, d, _ = orc.step(bufs, i, acts[t, i])
            obs[t, i], rew[t, i], done[t, i] = o, r, d
            alive[i] = not d
        done[t, ~alive] = True
    return rows, acts, obs, rew, done


def gpu_curve(env_id, precision, rows, acts, obs_o, rew_o, done_o):
    import torch
    from bioimitation.vector_env import VectorEnv
    T, n, _ = acts.shape
    env = VectorEnv(env_id, n, precision=precision, seed=0)
    env.reset(ref_index=rows)
    alive = np.ones(n, bool)
    cur = {'max': [], 'median': [], 'reward_max': [], 'alive': [], 'done_mismatch': 0}
    for t in range(T):
        o, r, d, _ = env.step(torch.as_tensor(acts[t], device=env.device))
        torch.cuda.synchronize()
        o, r, d = (v.cpu().numpy().astype(np.float64) for v in (o, r, d))
        idx = np.where(alive)[0]
        if len(idx):
            e_env = _rel(o[idx], obs_o[t, idx]).max(axis=1)
            e_rew = _rel(r[idx], rew_o[t, idx])
            cur['max'].append(float(e_env.max()))
            cur['median'].append(float(np.median(e_env)))
            cur['reward_max'].append(float(e_rew.max()))
        else:
            cur['max'].append(None); cur['median'].append(None); cur['reward_max'].append(None)
        cur['done_mismatch'] += int((d[idx].astype(bool) != done_o[t, idx]).sum())
        alive &= ~(d.astype(bool) | done_o[t])
        cur['alive'].append(int(alive.sum()))
    env.close()
    return cur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ids', default='MuscleWalkingImitation2D-v0,TorqueWalkingImitation2D-v0,'
                                     'MuscleRunningImitation3D-v0')
    ap.add_argument('--envs', type=int, default=64)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--out', default=os.path.join(REPO, 'gpurun_out', 'error_curve.json'))
    a = ap.parse_args()
    res = {}
    marks = [1, 10, 50, 100, a.steps]
    for env_id in a.ids.split(','):
        rows, acts, obs, rew, done = oracle_run(env_id, a.envs, a.steps, seed=200)
        for precision in (64, 32):
            c = gpu_curve(env_id, precision, rows, acts, obs, rew, done)
            res[f'{env_id}/fp{precision}'] = c
            pts = ' '.join(f't{m}:{c["max"][m - 1]:.1e}/{c["median"][m - 1]:.1e}'
                           if c['max'][m - 1] is not None else f't{m}:-' for m in marks)
            print(f'{env_id} fp{precision}: max/median rel obs err {pts}; alive at end '
                  f'{c["alive"][-1]}/{a.envs}; done mismatches {c["done_mismatch"]}', flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({'envs': a.envs, 'steps': a.steps, 'curves': res}, open(a.out, 'w'))


if __name__ == '__main__':
    main()
