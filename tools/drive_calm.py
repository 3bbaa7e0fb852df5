"""Re-search the drive schedule of the envs of a committed drive fixture
(tests/golden/drive_<ID>.npz) whose one-ulp twins leave 1e-5 within 200
steps (test infrastructure, round 5).

The scheduled tracking-drive test bounds GPU vs oracle by 1e-4 only on calm
env-steps (twin envelope <= 1e-5); an env whose twins diverge is held to
100 x its twin envelope instead.  For each such env this tool reruns
tools/drive_search.search_row with new seeds and keeps the first schedule
under which the env lives at least as long as before and the envelope of the
test's four one-ulp twins (tracking.twin_columns) stays <= 1e-5 on every
step the env is alive on all sides.  The rows are unchanged (the
reference's draw); the fixture records the seed used per env (``reseed``,
0 = the original search).

    python tools/drive_calm.py ENV_ID [--tries 24] [--write]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle'), os.path.join(REPO, 'tests'),
                os.path.join(REPO, 'tools')]

import drive_search as DS  # noqa: E402

T = 200


def envelope(row, sched, P):
    """(lived steps, per-step twin envelope) of one env under ``sched``, as
    the GPU test measures it (oracle vs its four one-ulp twins)"""
    from tracking import make_twin, twin_columns
    orc, drive, pk = DS._G['orc'], DS._G['drive'], DS._G['pk']
    cols = twin_columns(pk.ndof)
    b = orc.new_envs(1)
    tw = [orc.new_envs(1) for _ in cols]
    orc.reset(b, 0, row)
    for t_, c in zip(tw, cols):
        orc.reset(t_, 0, row)
        make_twin(orc, t_, 0, c)
    env = np.zeros(T)
    lived = T
    for t in range(T):
        a = drive(orc.get_state(b, 0), sched[t // P])
        o, r, d, _ = orc.step(b, 0, a)
        dt = False
        for t_ in tw:
            o2, r2, d2, _ = orc.step(t_, 0, a)
            env[t] = max(env[t], (np.abs(o2 - o) / np.maximum(1.0, np.abs(o))).max(), abs(r2 - r) / max(1.0, abs(r)))
            dt = dt or d2
        if d or dt:
            lived = t + 1
            break
    return lived, env[:lived]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('env_id')
    ap.add_argument('--tries', type=int, default=24)
    ap.add_argument('--write', action='store_true')
    a = ap.parse_args()
    from tracking import load_schedule
    path = os.path.join(REPO, 'tests', 'golden', f'drive_{a.env_id}.npz')
    z = dict(np.load(path, allow_pickle=False))
    rows, sched, P, gains = load_schedule(a.env_id)
    DS._init(a.env_id, gains)
    reseed = z.get('reseed', np.zeros(len(rows), dtype=np.int64)).copy()
    changed = False
    for i, row in enumerate(rows):
        lived0, env0 = envelope(int(row), sched[i], P)
        if env0.max() <= 1e-5:
            continue
        print(f'env {i} row {row}: lived {lived0}, twin envelope max {env0.max():.1e} (first > 1e-5 at t={int(np.argmax(env0 > 1e-5)) + 1})', flush=True)
        for s in range(1, a.tries + 1):
            sc, lived, _ = DS.search_row(int(row), int(z['seed']) + 1000 * s)
            full = np.zeros_like(sched[i])
            full[:len(sc)] = sc
            l2, env2 = envelope(int(row), full, P)
            print(f'  seed +{1000 * s}: lived {l2}, envelope max {env2.max():.1e}', flush=True)
            if l2 >= lived0 and env2.max() <= 1e-5:
                sched[i] = full
                reseed[i] = 1000 * s
                z['lived'][i] = l2
                changed = True
                print(f'  -> env {i} replaced (seed +{1000 * s})', flush=True)
                break
        else:
            print(f'  env {i}: no calm schedule in {a.tries} tries', flush=True)
    if changed and a.write:
        z['schedule'] = sched
        z['reseed'] = reseed
        np.savez_compressed(path, **z)
        print('written', path)


if __name__ == '__main__':
    main()
