"""Long-run soak on the GPU box (round 6): the bench workloads for many
steps with auto-reset, each run twice — the outputs must be finite and the
two runs bitwise identical at every checkpoint (the realize cache, the reset
table and the counters over thousands of launches and resets).

    python tools/soak.py [steps]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bioimitation.vector_env import MixedVectorEnv, VectorEnv  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 2000


def run(make, steps):
    env = make()
    env.reset()
    g = torch.Generator(device='cuda').manual_seed(123)
    digests, resets = [], 0
    for t in range(steps):
        a = torch.rand((env.num_envs, env.action_dim), generator=g, device=env.device, dtype=env.dtype)
        obs, rew, done, info = env.step(a)
        resets += int(done.sum())
        if t % 100 == 99 or t == steps - 1:
            assert bool(torch.isfinite(obs).all()) and bool(torch.isfinite(rew).all()), t
            digests.append((obs.double().sum().item(), rew.double().sum().item(), obs.clone()))
    torch.cuda.synchronize()
    env.close()
    return digests, resets


def main():
    cases = [
        ('C3 MuscleWalkingImitation2D-v0 x4096', lambda: VectorEnv('MuscleWalkingImitation2D-v0', 4096, seed=1, auto_reset=True)),
        ('C2 TorqueWalkingImitation2D-v0 x4096', lambda: VectorEnv('TorqueWalkingImitation2D-v0', 4096, seed=1, auto_reset=True)),
        ('C4 MuscleRunningImitation3D-v0 x4096', lambda: VectorEnv('MuscleRunningImitation3D-v0', 4096, seed=1, auto_reset=True)),
        ('C5 LockedKnee3D + Palsy3D 2048 + 2048 (fused)',
         lambda: MixedVectorEnv([('MuscleLockedKneeImitation3D-v0', 2048), ('MusclePalsyImitation3D-v0', 2048)], seed=1,
                                auto_reset=True)),
    ]
    for name, make in cases:
        d1, r1 = run(make, STEPS)
        d2, r2 = run(make, STEPS)
        same = all(torch.equal(a[2], b[2]) for a, b in zip(d1, d2)) and r1 == r2
        print(f'{name}: {STEPS} steps x 2 runs, {r1} auto-resets, finite, runs bitwise identical: {same}; '
              f'final obs sum {d1[-1][0]:.6e}', flush=True)
        assert same, name


if __name__ == '__main__':
    main()
