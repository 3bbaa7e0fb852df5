"""Per-launch timing of the env kernel with HIP events (steady state vs warmup,
back-to-back vs synchronized launches)."""
import os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'bioimitation-gym_amd')]
import numpy as np, torch
from bioimitation.vector_env import VectorEnv
prec = int(sys.argv[1]) if len(sys.argv) > 1 else 64
env = VectorEnv('MuscleWalkingImitation2D-v0', 4096, precision=prec, seed=1, auto_reset=True)
env.reset()
dev = env.device
acts = torch.rand((400, 4096, env.action_dim), device=dev, dtype=env.dtype)
s = torch.cuda.current_stream(dev)
def run(k0, n, sync_each=False):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    evs[0].record(s)
    t0 = time.perf_counter()
    for i in range(n):
        env.step(acts[k0 + i])
        evs[i + 1].record(s)
        if sync_each: torch.cuda.synchronize()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    per = [evs[i].elapsed_time(evs[i + 1]) for i in range(n)]
    return wall, per
for name, k0, n, se in [('first', 0, 10, False), ('b2b', 10, 100, False), ('sync', 110, 30, True), ('b2b2', 140, 200, False)]:
    wall, per = run(k0, n, se)
    print(f'{name:6s} wall/launch {wall:.3f} ms  event/launch median {np.median(per):.3f} min {np.min(per):.3f} max {np.max(per):.3f}  first5 {np.round(per[:5],3)}')
