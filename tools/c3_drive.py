"""Survival of MuscleWalkingImitation2D-v0 under the reference-tracking
excitation drive (tests/tracking.py) from every reset row 0..64, on the fp64
oracle (CPU): the rows tests/tracking.py lists as ROWS_UP (alive after 200
steps) and ROWS_FALL come from this run, and so does the non-chaotic twin
curve.

    python tools/c3_drive.py
"""
import os
import sys
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle'), os.path.join(REPO, 'tests')]

ENV_ID = 'MuscleWalkingImitation2D-v0'


def lived(row, T=200):
    import oracle
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    from tracking import TrackingDrive
    pk = load_pack(ENV_ID)
    orc = oracle.Oracle(pk)
    drive = TrackingDrive(orc, pk, load_names(ENV_ID))
    bufs = orc.new_envs(1)
    orc.reset(bufs, 0, row)
    for t in range(T):
        if orc.step(bufs, 0, drive(orc.get_state(bufs, 0)))[2]:
            return t + 1
    return T


def main():
    with Pool(min(8, os.cpu_count() or 1)) as p:
        steps = p.map(lived, range(65))
    print('lived steps per reset row 0..64:', steps)
    print('alive after 200 steps:', [r for r, s in enumerate(steps) if s == 200])


if __name__ == '__main__':
    main()
