"""The premise of the scheduled tracking-drive parity tests, on the oracle
alone (CPU): replay tests/golden/drive_<ID>.npz and report survival and the
one-ulp twin ensemble's error curve (the quantity the GPU test bounds the
GPU-vs-oracle error by).

    python tools/drive_twins.py ENV_ID
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle'), os.path.join(REPO, 'tests')]


def run(env_id, T=200, ntwins=4):
    import oracle
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    from tracking import TrackingDrive, load_schedule, make_twin, twin_columns
    rows, sched, P, gains = load_schedule(env_id)
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    drive = TrackingDrive(orc, pk, load_names(env_id), gains)
    n = len(rows)
    bufs = orc.new_envs(n)
    cols = twin_columns(pk.ndof)[:ntwins]
    twins = [orc.new_envs(n) for _ in cols]
    for i in range(n):
        orc.reset(bufs, i, int(rows[i]))
        for tw, c in zip(twins, cols):
            orc.reset(tw, i, int(rows[i]))
            make_twin(orc, tw, i, c)
    live, alive = np.ones(n, bool), np.ones(n, bool)
    e_twin = np.zeros(T)
    e_env = np.zeros((T, n))
    for t in range(T):
        for i in range(n):
            a = drive(orc.get_state(bufs, i), sched[i, t // P])
            o, r, d, _ = orc.step(bufs, i, a)
            dt = False
            for tw in twins:
                o2, r2, d2, _ = orc.step(tw, i, a)
                if live[i]:
                    e = max((np.abs(o2 - o) / np.maximum(1.0, np.abs(o))).max(), abs(r2 - r) / max(1.0, abs(r)))
                    e_twin[t] = max(e_twin[t], e)
                    e_env[t, i] = max(e_env[t, i], e)
                dt = dt or d2
            alive[i] &= not d
            live[i] = live[i] and not (d or dt)
    return rows, alive, e_twin, e_env


if __name__ == '__main__':
    env_id = sys.argv[1]
    rows, alive, e, ee = run(env_id)
    print(f'{env_id}: rows {list(rows)}; alive at t=200 {alive.sum()}/{len(rows)}')
    print('twin envelope at t=1,25,50,75,100,125,150,175,200:',
          ' '.join(f'{e[k]:.1e}' for k in (0, 24, 49, 74, 99, 124, 149, 174, 199)))
    print(f'steps with twin <= 1e-5: {(e <= 1e-5).sum()}/200; first above: {int(np.argmax(e > 1e-5)) if (e > 1e-5).any() else None}')
    calm = ee <= 1e-5
    print('per env: worst twin', ' '.join(f'{x:.0e}' for x in ee.max(0)))
    print(f'env-steps with the env\'s twin <= 1e-5: {calm.sum()}/{calm.size}')
