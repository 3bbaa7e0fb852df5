"""RK-Merson leg probe (GPU box; round 5): per budget B,
ms per budgeted launch and finished env steps/s at 4096 envs, timed the way
bench.py's reference_integrator_rate times it (host-side `fin += ready` after
every launch) and with the count taken from the per-env evaluation counter
instead (no extra kernel between the step launches).

    python tools/rk_probe.py ENV_ID [--budgets 3,4,5,6,7] [--steps 200] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'bioimitation-gym_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('env_id')
    ap.add_argument('--budgets', default='3,4,5,6,7')
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--envs', type=int, default=4096)
    a = ap.parse_args()
    import torch
    from bioimitation.vector_env import VectorEnv
    dev = torch.device('cuda', 0)
    n = a.envs
    for rnd in range(a.rounds):
        for b in [int(x) for x in a.budgets.split(',')]:
            env = VectorEnv(a.env_id, n, config={'integrator': 'rk-merson'}, device=0, seed=1000, auto_reset=True)
            env.set_rk_budget(b)
            pool = 64
            gen = np.random.Generator(np.random.PCG64(0))
            acts = torch.as_tensor(gen.uniform(0.0, 1.0, size=(pool, n, env.action_dim)), dtype=env.dtype, device=dev)
            env.reset()
            fin = torch.zeros(n, dtype=torch.int32, device=dev)
            k0 = 0
            while k0 < 50 * 155 and (k0 % 10 or int(fin.sum()) < n * 155):
                env.step(acts[k0 % pool])
                fin += env.ready
                k0 += 1
            out = {'env_id': a.env_id, 'budget': b, 'round': rnd}
            for mode in ('ready', 'counter'):
                fin.zero_()
                r0, e0 = env.reset_count(), env.eval_count()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for k in range(a.steps):
                    env.step(acts[(k0 + k) % pool])
                    if mode == 'ready':
                        fin += env.ready
                torch.cuda.synchronize(dev)
                wall = time.perf_counter() - t0
                k0 += a.steps
                dr, de = env.reset_count() - r0, env.eval_count() - e0
                if mode == 'ready':
                    done = int(fin.sum())
                    per = de / max(done, 1)
                    out['evals_per_step'] = per
                else:
                    # finished steps from the counters: each finished step adds one realize, each
                    # reset one more; attempts add 5 (the evals-per-finished-step of the ready pass)
                    done = de / per
                out[mode] = {'ms_per_launch': wall / a.steps * 1e3, 'finished_per_s': done / wall,
                             'finished': done}
            env.close()
            print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
