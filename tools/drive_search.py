"""Offline lookahead search for the hip-target schedule of the tracking drive
(tests/tracking.py) on the fp64 oracle: test infrastructure for the 200-step
north_star parity tests on the spatial muscle configs (C4, C5).

The drive alone (a per-muscle stretch reflex toward the reference motion, the
pelvis balanced through the hips) does not keep the spatial models up.  Every
P env steps this search branches the oracle env, tries K offsets of the hip
flexion / adduction targets (the 4-vector ``offset`` of TrackingDrive) held
over a horizon of H steps with the drive's feedback running, and keeps the
offset under which the env lives longest (ties: the smallest pelvis
orientation error against the reference).  The chosen schedule, one 4-vector
per P steps, is committed as a fixture (tests/golden/drive_<ID>.npz) with the
reset rows; the GPU test replays it: the drive computes each step's
excitations from the oracle's state and that schedule, and the same actions go
to the GPU and to the oracle.

    python tools/drive_search.py ENV_ID [--seed 0] [--n 32] [--out tests/golden/drive_<ID>.npz]
"""
import argparse
import os
import random
import sys
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle'), os.path.join(REPO, 'tests')]

P, H, K, T, SIGMA, NOFF = 5, 60, 24, 200, 0.3, 8
_G = {}


def reference_rows(reset_hi, n, seed):
    """reset rows drawn by the reference's rule: ``random.randint(0, reset_hi)``
    after ``random.seed(seed)`` (muscle_running_imitation_env3D.py:144)"""
    random.seed(seed)
    return [random.randint(0, reset_hi) for _ in range(n)]


def _init(env_id, gains):
    import oracle
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    from tracking import TrackingDrive
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    _G.update(orc=orc, pk=pk, drive=TrackingDrive(orc, pk, load_names(env_id), gains))


def _rollout(state, offset, steps):
    """(lived steps, orientation cost) from ``state`` under the drive + offset"""
    orc, drive, nd = _G['orc'], _G['drive'], _G['pk'].ndof
    buf = orc.new_envs(1)
    orc.set_state(buf, 0, state)
    cost = 0.0
    for t in range(steps):
        s = orc.get_state(buf, 0)
        if orc.step(buf, 0, drive(s, offset))[2]:
            return t, cost
        s = orc.get_state(buf, 0)
        r = min(int(s[1]), _G['pk'].nrows - 1)
        cost += float(np.sum((s[5:8] - drive.qref[r, :3]) ** 2))
    return steps, cost


def _choose(s0, last, rng):
    cands = [np.zeros(NOFF), last] + list(rng.normal(0.0, SIGMA, (K, NOFF)))
    best = max(((_rollout(s0, c, H), i) for i, c in enumerate(cands)),
               key=lambda x: (x[0][0], -x[0][1], -x[1]))
    return cands[best[1]]


def search_row(row, seed, max_backtracks=40):
    """schedule (one offset per P steps) for reset row ``row``; when the env
    falls, the search backs up 2, 4, 8 ... decisions and draws new candidates
    there (a restart budget of ``max_backtracks``)"""
    orc, drive = _G['orc'], _G['drive']
    rng = np.random.default_rng(seed * 100003 + row)
    buf = orc.new_envs(1)
    orc.reset(buf, 0, row)
    states, sched = [], []
    backs, depth = 0, 1
    while len(sched) * P < T:
        s0 = orc.get_state(buf, 0)
        states.append(s0)
        last = sched[-1] if sched else np.zeros(NOFF)
        off = _choose(s0, last, rng)
        sched.append(off)
        done = False
        for _ in range(P):
            if orc.step(buf, 0, drive(orc.get_state(buf, 0), off))[2]:
                done = True
                break
        if done and _G['pk'].n_episode > int(orc.get_state(buf, 0)[1]) and backs < max_backtracks:
            backs += 1
            depth = min(depth * 2, len(sched))
            k = len(sched) - depth
            del sched[k:], states[k + 1:]
            orc.set_state(buf, 0, states.pop())
            continue
        if done:
            break
    # replay the schedule from the reset to count the lived steps
    orc.reset(buf, 0, row)
    lived = 0
    for t in range(T):
        lived = t + 1
        if orc.step(buf, 0, drive(orc.get_state(buf, 0), sched[t // P]))[2]:
            break
    return np.array(sched), lived, backs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('env_id')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--n', type=int, default=32)
    ap.add_argument('--gains', default='')
    ap.add_argument('--out', default=None)
    ap.add_argument('--procs', type=int, default=8)
    a = ap.parse_args()
    from bioimitation.registry import load_pack
    pk = load_pack(a.env_id)
    rows = reference_rows(pk.reset_hi, a.n, a.seed)
    gains = {k: float(v) for k, v in (kv.split('=') for kv in a.gains.split(',') if kv)}
    with Pool(a.procs, initializer=_init, initargs=(a.env_id, gains)) as p:
        res = p.starmap(search_row, [(r, a.seed) for r in rows])
    lived = [x[1] for x in res]
    print('rows:', rows)
    print('backtracks:', [x[2] for x in res])
    print('lived:', lived)
    print(f'alive at T={T}: {sum(x >= T for x in lived)}/{len(lived)}')
    if a.out:
        S = np.zeros((len(rows), T // P, NOFF))
        for i, (sc, _, _) in enumerate(res):
            S[i, :len(sc)] = sc
        from tracking import GAINS
        g = dict(GAINS, **gains)
        np.savez_compressed(a.out, env_id=np.array(a.env_id), seed=np.array(a.seed), rows=np.array(rows),
                            schedule=S, period=np.array(P), lived=np.array(lived),
                            gain_names=np.array(sorted(g)), gain_values=np.array([g[k] for k in sorted(g)]))


if __name__ == '__main__':
    main()
