"""Host wall clock of RLlibVectorEnv.vector_step (the batch-per-worker path
of INTEGRATION.md section 3) against the same step with four blocking
pageable copies back (the round-5 form), C3's model at 64, 256 and 1024 envs,
median of 200 steps after 20.

    python tools/rllib_step_time.py
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import torch  # noqa: E402
from bioimitation.adapters import RLlibVectorEnv  # noqa: E402

ENV = 'MuscleWalkingImitation2D-v0'


def blocking_step(v, actions):
    a = torch.as_tensor(np.asarray(actions, dtype=np.float64), device=v.env.device)
    obs, rew, done, info = v.env.step(a)
    obs, rew, done, info = (t.double().cpu().numpy() for t in (obs, rew, done, info))
    infos = [{'all_rewards': list(map(float, r))} for r in info]
    return list(obs), list(map(float, rew)), list(map(bool, done)), infos


for n in (64, 256, 1024):
    v = RLlibVectorEnv(ENV, n, seed=0)
    v.vector_reset()
    rng = np.random.default_rng(0)
    res = {}
    for name, f in (('pinned async', v.vector_step), ('blocking pageable', lambda a: blocking_step(v, a))):
        ts = []
        for k in range(220):
            a = list(rng.uniform(0.2, 0.6, (n, v.env.action_dim)))
            t0 = time.perf_counter()
            _, _, d, _ = f(a)
            ts.append(time.perf_counter() - t0)
            if k % 40 == 39:
                v.vector_reset()
        res[name] = 1e6 * float(np.median(ts[20:]))
    print(f'{ENV} RLlibVectorEnv x{n}: vector_step ' + ', '.join(f'{k} {t:.1f} us' for k, t in res.items()))
    v.close()
