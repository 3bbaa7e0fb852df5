"""Lived-step counts of the 200-step parity drive (tests/test_gpu_parity.py::
test_parity_200_identical_action_steps), computed with the fp64 oracle on the
CPU: same seeds, same actions, same masking.  The GPU test asserts these
counts (the HIP path agrees with the oracle on every `done`).  The open-loop
drives cannot keep the model up; test_parity_200_steps_3d_envs_kept_up uses a
stiff reference-tracking PD on the 3D torque IDs instead (22 / 24 of 32 envs
alive at t = 200 in the oracle).

    python tools/survival_probe.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle')]

import oracle  # noqa: E402
from bioimitation.registry import load_pack  # noqa: E402


def main():
    for env_id in ['MuscleWalkingImitation2D-v0', 'TorqueWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0']:
        rng = np.random.default_rng(200)
        n, T = 24, 200
        pk = load_pack(env_id)
        orc = oracle.Oracle(pk)
        bufs = orc.new_envs(n)
        rows = rng.integers(0, min(pk.reset_hi, pk.n_episode - T) + 1, size=n)
        for i in range(n):
            orc.reset(bufs, i, int(rows[i]))
        alive, lived = np.ones(n, bool), np.zeros(n, int)
        for t in range(T):
            if 'Muscle' in env_id:
                acts = rng.uniform(0.0, 0.4, size=(n, pk.nact))
            else:
                st = np.array([orc.get_state(bufs, i)[1] for i in range(n)]).astype(int) + 1
                acts = np.array([[pk.ref_q[min(r, pk.nrows - 1)][pk.pd_coord[a]] for a in range(pk.nact)]
                                 for r in st]) + rng.normal(0.0, 0.02, size=(n, pk.nact))
            for i in np.where(alive)[0]:
                d = orc.step(bufs, i, acts[i])[2]
                lived[i] += 1
                alive[i] = not d
        print(f'{env_id}: lived steps {sorted(lived.tolist())}, total {lived.sum()}, alive at t=200 {alive.sum()}/{n}')


if __name__ == '__main__':
    main()
