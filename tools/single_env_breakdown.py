"""where the single-env drop-in step's time goes (config
C1, TorqueWalkingImitation2D-v0, one env: the reference's RLlib layout of one
env per worker).  Per step, wall clock on the host, 300 steps after 30
warm-up steps, medians:
  facade        envs.make(ID).step(action) as a user calls it (trajectory
                recorder on, the default: one extra state copy per step)
  facade_norec  the same with config record_trajectory=False
  vector+sync   VectorEnv(ID, 1).step(actions on the device) + synchronize
  launch only   the same without the synchronize (host cost of one launch)
Run under `rocprofv3 --kernel-trace --stats` to get the kernel's own
duration per launch (the env_kernel row of the stats CSV).

    python tools/single_env_breakdown.py [env id]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import torch  # noqa: E402
from bioimitation import envs  # noqa: E402
from bioimitation.vector_env import VectorEnv  # noqa: E402

ENV = sys.argv[1] if len(sys.argv) > 1 else 'TorqueWalkingImitation2D-v0'
W, K = 30, 300


def med(ts):
    return 1e6 * float(np.median(ts))


def facade(record):
    e = envs.make(ENV, config={'record_trajectory': record, 'mode': 'test'})
    e.reset()
    rng = np.random.default_rng(0)
    lo, hi = np.asarray(e.action_space.low), np.asarray(e.action_space.high)
    ts = []
    for k in range(W + K):
        a = lo + (hi - lo) * rng.uniform(0.3, 0.7, size=lo.shape)
        t0 = time.perf_counter()
        e.step(a)
        ts.append(time.perf_counter() - t0)
        if k % 50 == 49:
            e.reset()
    return med(ts[W:])


def vector(sync):
    v = VectorEnv(ENV, 1, precision=64, auto_reset=True)
    v.reset()
    a = torch.full((1, v.action_dim), 0.5, dtype=torch.float64, device=v.device)
    if not v.pack.nmuscle:
        a.zero_()
    ts = []
    torch.cuda.synchronize()
    for k in range(W + K):
        t0 = time.perf_counter()
        v.step(a)
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    return med(ts[W:])


if __name__ == '__main__':
    r = {'facade': facade(True), 'facade_norec': facade(False), 'vector+sync': vector(True), 'launch only': vector(False)}
    print(f'{ENV} single env, host wall clock per step (median of {K}): ' +
          ', '.join(f'{k} {v:.1f} us' for k, v in r.items()))
