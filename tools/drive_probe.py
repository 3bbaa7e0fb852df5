"""Survival of the muscle envs under the reference-tracking excitation drive
(tests/tracking.py) on the fp64 oracle, for a set of gains.

    python tools/drive_probe.py ENV_ID [--rows 0:64] [--gains a0=0.03,kl=20,...] [--T 200]
"""
import argparse
import os
import sys
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle'), os.path.join(REPO, 'tests')]

_G = {}


def _init(env_id, gains):
    import oracle
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    from tracking import TrackingDrive
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    _G.update(orc=orc, drive=TrackingDrive(orc, pk, load_names(env_id), gains), pk=pk)


def lived(row, T=200):
    orc, drive = _G['orc'], _G['drive']
    bufs = orc.new_envs(1)
    orc.reset(bufs, 0, row)
    for t in range(T):
        if orc.step(bufs, 0, drive(orc.get_state(bufs, 0)))[2]:
            return t + 1
    return T


def survival(env_id, rows, gains, T=200, procs=8):
    with Pool(procs, initializer=_init, initargs=(env_id, gains)) as p:
        return p.starmap(lived, [(r, T) for r in rows])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('env_id')
    ap.add_argument('--rows', default='0:32')
    ap.add_argument('--gains', default='')
    ap.add_argument('--T', type=int, default=200)
    a = ap.parse_args()
    lo, hi = (int(x) for x in a.rows.split(':'))
    gains = {k: float(v) for k, v in (kv.split('=') for kv in a.gains.split(',') if kv)}
    steps = survival(a.env_id, range(lo, hi), gains, a.T)
    print('lived:', steps)
    print(f'alive at T={a.T}: {sum(s == a.T for s in steps)}/{len(steps)}  mean lived {np.mean(steps):.1f}')


if __name__ == '__main__':
    main()
