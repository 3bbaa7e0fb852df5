"""The first timed window of a process against the later ones (GPU box;
round 5): bench.py times ONE 20-step window per process, right after its
burn-in.  Prints wall and event time per step of six consecutive 20-step
windows, each after a synchronize, as bench.py's timed region does.

    python tools/first_window.py [--prime-events] [ENV_ID]

--prime-events: record and read a timing event pair once during the burn-in
(the first use of timing events in the process, outside the windows).
--counter-early: read the reset counter (a full state copy to the host) 5
steps before the end of the burn-in instead of after it.
--idle-ms X: leave the GPU idle X ms (synchronized, host sleep) before window 1.
--dry-window K: one untimed window of K steps, shaped like the timed ones
(events recorded and read, synchronize on both sides), before window 1.
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'bioimitation-gym_amd'))


def main():
    import torch
    from bioimitation.vector_env import VectorEnv
    argv = list(sys.argv[1:])
    idle = 0.0
    dry = 0
    if '--dry-window' in argv:
        i = argv.index('--dry-window')
        dry = int(argv[i + 1])
        del argv[i:i + 2]
    if '--idle-ms' in argv:
        i = argv.index('--idle-ms')
        idle = float(argv[i + 1])
        del argv[i:i + 2]
    args = [x for x in argv if not x.startswith('--')]
    env_id = args[0] if args else 'MuscleWalkingImitation2D-v0'
    prime = '--prime-events' in argv
    early = '--counter-early' in argv
    n = 4096
    env = VectorEnv(env_id, n, seed=1000, auto_reset=True)
    dev = env.device
    gen = np.random.Generator(np.random.PCG64(0))
    acts = torch.as_tensor(gen.uniform(0, 1, size=(64, n, env.action_dim)), dtype=env.dtype, device=dev)
    env.reset()
    stream = torch.cuda.current_stream(dev)
    for k in range(155):
        env.step(acts[k % 64])
        if prime and k == 100:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            e0.elapsed_time(e1)
        if early and k == 149:
            torch.cuda.synchronize(dev)
            env.reset_count()
    torch.cuda.synchronize(dev)
    if not early:
        env.reset_count()
    if idle:
        torch.cuda.synchronize(dev)
        time.sleep(idle / 1e3)
    k0 = 155
    if dry:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        ev0.record(stream)
        for k in range(dry):
            env.step(acts[(k0 + k) % 64])
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        ev0.elapsed_time(ev1)
        k0 += dry
    out = []
    for w in range(6):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(20):
            env.step(acts[(k0 + k) % 64])
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        k0 += 20
        out.append(f'{wall / 20 * 1e6:.1f}/{ev0.elapsed_time(ev1) / 20 * 1e3:.1f}')
    print(f'{env_id} prime_events={prime} counter_early={early} idle_ms={idle:g} dry={dry}: wall/events us per step, windows 1..6: ' + '  '.join(out), flush=True)
    env.close()


if __name__ == '__main__':
    main()
