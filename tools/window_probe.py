"""Kernel time and termination rate of the bench workload by step window
after the all-fresh start (bench.py's protocol: 4096 envs, U[0,1] actions
from a 64-batch pool, auto-reset), to see where the 150-step burn-in leaves
the timed window (round 5).

    python tools/window_probe.py [env_id] [steps]     (GPU box)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bioimitation.vector_env import VectorEnv  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else 'MuscleWalkingImitation2D-v0'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 600
n = 4096
env = VectorEnv(env_id, n, precision=64, seed=1000, auto_reset=True)
gen = np.random.Generator(np.random.PCG64(0))
acts = torch.as_tensor(gen.uniform(0.0, 1.0, size=(64, n, env.action_dim)), device=env.device)
env.reset()
s = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
dones = []
ev[0].record(s)
for k in range(steps):
    env.step(acts[k % 64])
    ev[k + 1].record(s)
    dones.append(env.done.sum())
torch.cuda.synchronize()
ms = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(steps)])
d = np.array([int(x) for x in dones]) / n
W = 25
print(f'{env_id}: per {W}-step window after the fresh start — kernel ms (mean) / termination rate')
for a in range(0, steps, W):
    print(f'  steps {a:4d}-{a + W - 1:4d}: {ms[a:a + W].mean():.4f} ms  {d[a:a + W].mean() * 100:.2f} %')
