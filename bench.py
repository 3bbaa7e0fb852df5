"""Throughput bench: batched env steps/sec of MuscleWalkingImitation2D-v0 at
4096 envs per GPU (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N --steps K --warmup W --envs 4096 --precision 64]
    (N > 1: launched by torch.distributed.run; RANK/LOCAL_RANK/WORLD_SIZE)

A "step" = one batched env step of every env on every rank (one kernel
launch per GPU): action pre-processing, nsub semi-implicit substeps of the
musculoskeletal dynamics, realize, obs/reward/done, in-kernel auto-reset.
Actions: PCG64(seed=rank) U[0,1] excitations generated on the host and
uploaded once before timing; inputs resident in HBM.
Environments shard by index across ranks (no data-path collective), so
scaling is weak: per-GPU work is fixed.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle')]

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes_per_env_step(pk, real_bytes):
    """Bytes one env step must move through HBM (state read + write, action
    read, obs/reward/done/info write); reference/model tables excluded."""
    nd, nm, na, H = pk.ndof, pk.nmuscle, pk.nact, pk.horizon
    state_reals = 2 * nd + 2 * nm + H * na + na + 1          # q u act lce hist last old_px
    state_bytes = state_reals * real_bytes + 8 + 4 * 4        # + t (f64) + istep/has_last/done/resets
    io = (na + pk.obs_dim + 1 + pk.info_dim) * real_bytes + 1
    return 2 * state_bytes + io


def cpu_baseline(env_id, seconds=12.0):
    """fp64 C oracle (oracle/, a port of the step) on host threads, bounded sample."""
    import numpy as np
    import oracle
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    threads = min(16, os.cpu_count() or 1)
    n = 64 * threads
    bufs = orc.new_envs(n)
    rng = np.random.Generator(np.random.PCG64(0))
    for i in range(n):
        orc.reset(bufs, i, int(rng.integers(0, pk.reset_hi + 1)))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        acts = rng.uniform(0, 1, size=(n, pk.nact))
        _, _, done, _ = orc.batch_step(bufs, n, acts, nthreads=threads, want_obs=True)
        for i in np.nonzero(done)[0]:
            orc.reset(bufs, int(i), int(rng.integers(0, pk.reset_hi + 1)))
        steps += 1
    dt = time.perf_counter() - t0
    return {'value': n * steps / dt, 'unit': 'env-steps/s', 'cores': threads, 'kind': 'port',
            'sample': f'{n} envs x {steps} steps ({dt:.1f} s), fp64 C oracle, {threads} threads, auto-reset on host'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--envs', type=int, default=4096, help='envs per GPU')
    ap.add_argument('--precision', type=int, default=int(os.environ.get('BIOIM_PRECISION', 64)))
    ap.add_argument('--env-id', default='MuscleWalkingImitation2D-v0')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--mixed', default=None,
                    help="mixed batch 'ID_A,ID_B' split 50/50 per GPU (BASELINE config C5), e.g. "
                         "MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0")
    a = ap.parse_args()

    import numpy as np
    import torch
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('gloo')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    from bioimitation.vector_env import MixedVectorEnv, VectorEnv
    if a.mixed:
        ids = a.mixed.split(',')
        sizes = [a.envs // len(ids)] * len(ids)
        sizes[-1] += a.envs - sum(sizes)
        env = MixedVectorEnv(list(zip(ids, sizes)), device=local, precision=a.precision, seed=1000, auto_reset=True,
                             env_offset=rank * a.envs)
        env.pack, env.nsub, env.lanes_per_env = env.envs[0].pack, env.envs[0].nsub, env.envs[0].lanes_per_env
        env.launch = {e.env_id: e.launch for e in env.envs}
        a.env_id = '+'.join(ids)
        a.no_cpu_baseline = True
    else:
        env = VectorEnv(a.env_id, a.envs, device=local, precision=a.precision, seed=1000, auto_reset=True,
                        env_offset=rank * a.envs)        # global env index block (bioimitation/parallel.py)
    n, A = a.envs, env.action_dim
    total = a.warmup + a.steps
    gen = np.random.Generator(np.random.PCG64(rank))
    acts = torch.as_tensor(gen.uniform(0.0, 1.0, size=(total, n, A)), dtype=env.dtype, device=dev)
    env.reset()
    stream = torch.cuda.current_stream(dev)
    for k in range(a.warmup):
        env.step(acts[k])
    torch.cuda.synchronize(dev)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(a.warmup, total):
        env.step(acts[k])
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    kernel_ms = ev0.elapsed_time(ev1) / a.steps      # per launch, events on the launch stream
    t_max = wall
    if dist:
        tt = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt[0])
    steps_total = world * n * a.steps
    value = steps_total / t_max
    # done rate: an untimed pass over the same actions after the
    # timed region, counting terminations on the device
    dones = torch.zeros((), dtype=torch.float64, device=dev)
    for k in range(a.warmup, total):
        done = env.step(acts[k])[2]
        dones += done.to(torch.float64).sum()
    done_rate = float(dones) / (n * a.steps)
    if rank == 0:
        real_bytes = 8 if a.precision == 64 else 4
        if a.mixed:   # env-weighted mean over the segments
            B = sum(algorithmic_bytes_per_env_step(e.pack, real_bytes) * e.num_envs for e in env.envs) / n
        else:
            B = algorithmic_bytes_per_env_step(env.pack, real_bytes)
        achieved = B * n / (kernel_ms * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(REPO, 'profiles', 'traffic.json')
        if os.path.exists(tf):
            try:
                rec = json.load(open(tf)).get(f'{a.env_id}/fp{a.precision}/{n}')
                traffic = rec['bytes'] if rec else None    # rocprofv3 FETCH_SIZE + WRITE_SIZE per launch
            except Exception:
                traffic = None
        line = {
            'metric': 'env steps/sec (whole node), MuscleWalkingImitation2D-v0 @ 4096 envs/GPU'
            if a.env_id == 'MuscleWalkingImitation2D-v0' and n == 4096 else f'env steps/sec, {a.env_id} @ {n} envs/GPU',
            'value': value, 'unit': 'env-steps/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': t_max / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': f'f{a.precision}', 'done_rate': done_rate,
            'data': 'synthetic: PCG64 U[0,1] muscle excitations; reference motion synthesized from the shipped 3D IK',
            'config': {'workload': f'{a.env_id} batched env.step, {n} envs/GPU, nsub={env.nsub}, auto-reset',
                       'envs_per_gpu': n, 'lanes_per_env': env.lanes_per_env, 'parallelism': f'env-shard x{world}',
                       'launch': env.launch},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'bytes_per_env_step': B, 'kernel_ms': kernel_ms},
        }
        if not a.no_cpu_baseline and world == 1:
            line['cpu_baseline'] = cpu_baseline(a.env_id)
        print(json.dumps(line), flush=True)
    env.close()
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
