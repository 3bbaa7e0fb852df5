"""Host side of a timed window (GPU box; round 5): per env.step call, the
host time of the Python path (VectorEnv.step) and of the bare C-ABI call
(bioim_step through ctypes with cached pointers) while the GPU is busy, and
the wall time of one step from a synchronized, idle GPU against its kernel
time (events) — the start-up a 20-step window pays once.

    python tools/launch_latency.py [ENV_ID]
"""
import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'bioimitation-gym_amd'))


def main():
    import torch
    from bioimitation.vector_env import VectorEnv
    env_id = sys.argv[1] if len(sys.argv) > 1 else 'MuscleWalkingImitation2D-v0'
    n = 4096
    env = VectorEnv(env_id, n, seed=1000, auto_reset=True)
    dev = env.device
    gen = np.random.Generator(np.random.PCG64(0))
    acts = torch.as_tensor(gen.uniform(0, 1, size=(64, n, env.action_dim)), dtype=env.dtype, device=dev)
    env.reset()
    for k in range(160):
        env.step(acts[k % 64])
    torch.cuda.synchronize()
    P = lambda t: C.c_void_p(t.data_ptr())
    args = [(env._h, P(acts[k]), P(env.obs), P(env.reward), P(env.done), P(env.info)) for k in range(64)]
    L = env._L
    # host time per call with a busy GPU (the queue absorbs the launches)
    for label in ('VectorEnv.step', 'bioim_step (ctypes, cached args)'):
        ts = []
        torch.cuda.synchronize()
        for k in range(40):
            t0 = time.perf_counter()
            if label == 'VectorEnv.step':
                env.step(acts[k % 64])
            else:
                L.bioim_step(*args[k % 64])
            ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        ts = np.array(ts[1:]) * 1e6
        print(f'{label:34s} host us per call: median {np.median(ts):.1f}  p90 {np.percentile(ts, 90):.1f}', flush=True)
    # one step from an idle, synchronized GPU: wall vs kernel events
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for K in (1, 2, 5, 20):
        rows = []
        for rep in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev0.record()
            for k in range(K):
                env.step(acts[(rep + k) % 64])
            ev1.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e6
            rows.append((wall, ev0.elapsed_time(ev1) * 1e3))
        r = np.array(rows)
        print(f'K={K:3d}: wall {np.median(r[:, 0]):8.1f} us  events {np.median(r[:, 1]):8.1f} us  '
              f'wall/K {np.median(r[:, 0]) / K:7.1f}  events/K {np.median(r[:, 1]) / K:7.1f}', flush=True)
    # a 20-step window right after a host read of the state (bench.py reads the reset counter there):
    # does the full-state copy leave the first launches of the window cold?
    for pre in ('none', 'reset_count', 'small_d2h', 'none'):
        rows = []
        for rep in range(10):
            for k in range(5):
                env.step(acts[k % 64])
            if pre == 'reset_count':
                env.reset_count()
            elif pre == 'small_d2h':
                env.done[:16].cpu()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev0.record()
            for k in range(20):
                env.step(acts[(rep + k) % 64])
            ev1.record()
            torch.cuda.synchronize()
            rows.append(((time.perf_counter() - t0) * 1e6, ev0.elapsed_time(ev1) * 1e3))
        r = np.array(rows)
        print(f'K=20 after {pre:12s}: wall/K {np.median(r[:, 0]) / 20:7.1f}  events/K {np.median(r[:, 1]) / 20:7.1f} us', flush=True)
    # the steady launch from rocprof-free back-to-back runs
    torch.cuda.synchronize()
    ev0.record()
    for k in range(200):
        env.step(acts[k % 64])
    ev1.record()
    torch.cuda.synchronize()
    print(f'K=200 events/K {ev0.elapsed_time(ev1) * 1e3 / 200:.1f} us', flush=True)
    env.close()


if __name__ == '__main__':
    main()
