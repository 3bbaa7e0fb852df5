"""Throughput bench: batched env steps/sec of MuscleWalkingImitation2D-v0 at
4096 envs per GPU (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N --steps K --warmup W --envs 4096 --precision 64]

N > 1: the driver launches N ranks with torch.distributed.run (RANK /
LOCAL_RANK / WORLD_SIZE set).  Run directly with --gpus N > 1, bench.py starts
that launcher itself as a child process, before anything touches a GPU, and
exits with its status; a WORLD_SIZE that disagrees with --gpus, or fewer
visible GPUs than ranks, is refused with a non-zero exit (never a silent
1-GPU number).

A "step" = one batched env step of every env on every rank (one kernel
launch per GPU): action pre-processing, nsub semi-implicit substeps of the
musculoskeletal dynamics, realize, obs/reward/done, in-kernel auto-reset.
Actions: PCG64(seed=rank) U[0,1] excitations generated on the host and
uploaded once before timing; inputs resident in HBM.  An
untimed burn-in (default 150 steps) first brings the batch to its
steady-state termination rate; the done rate reported is the one of the
timed steps themselves (device reset counters read before and after).
Environments shard by index across ranks (no data-path collective), so
scaling is weak: per-GPU work is fixed.
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle')]

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_VEC_PEAK_TF = 78.6    # 256 CU x 4 SIMD x 16 fp64 FMA lanes/clk x 2 flop x 2.4 GHz


def algorithmic_bytes_per_env_step(pk, real_bytes):
    """Bytes one env step must move through HBM (state read + write, action
    read, obs/reward/done/info write); reference/model tables excluded."""
    nd, nm, na, H = pk.ndof, pk.nmuscle, pk.nact, pk.horizon
    state_reals = 2 * nd + 2 * nm + H * na + na + 1          # q u act lce hist last old_px
    state_bytes = state_reals * real_bytes + 8 + 4 * 4        # + t (f64) + istep/has_last/done/resets
    io = (na + pk.obs_dim + 1 + pk.info_dim) * real_bytes + 1
    return 2 * state_bytes + io


def host_cores():
    """CPUs this process may run on: affinity mask, capped by a cgroup v2 CPU
    quota when one is set (the GPU box grants a share of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open('/sys/fs/cgroup/cpu.max').read().split()
        if quota != 'max':
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_rate(env_id, threads, seconds, n_per_thread=64, integrator='euler'):
    """fp64 C oracle (oracle/, a port of the step): env-steps/s of a batch of
    n_per_thread x threads envs, auto-reset on the host, bounded sample;
    integrator 'euler' (the kernel's default substeps) or 'rk-merson'."""
    import numpy as np
    import oracle
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    n = n_per_thread * threads
    bufs = orc.new_envs(n)
    rng = np.random.Generator(np.random.PCG64(0))
    for i in range(n):
        orc.set_integrator(bufs, i, integrator, 1e-3)
        orc.reset(bufs, i, int(rng.integers(0, pk.reset_hi + 1)))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        if pk.nmuscle:
            acts = rng.uniform(0, 1, size=(n, pk.nact))
        else:   # PD targets at the reference
            acts = np.tile([pk.ref_q[min(int(pk.reset_hi), pk.nrows - 1)][pk.pd_coord[a]] for a in range(pk.nact)],
                           (n, 1)) + rng.normal(0, 0.05, size=(n, pk.nact))
        _, _, done, _ = orc.batch_step(bufs, n, acts, nthreads=threads, want_obs=True)
        for i in np.nonzero(done)[0]:
            orc.reset(bufs, int(i), int(rng.integers(0, pk.reset_hi + 1)))
        steps += 1
    dt = time.perf_counter() - t0
    return n * steps / dt, f'{n} envs x {steps} steps ({dt:.1f} s)'


def cpu_baseline(env_id, seconds=12.0):
    """the fp64 CPU restatement on the GPU box's host cores,
    same run.  The headline config on every usable core, plus C1 (1 env, 1
    thread, us/step), C2 (Torque2D) and C4 (Running3D) batch rates."""
    cores = host_cores()
    value, sample = _cpu_rate(env_id, cores, seconds)
    extra = {}
    r1, s1 = _cpu_rate('TorqueWalkingImitation2D-v0', 1, 2.0, n_per_thread=1)
    extra['C1_TorqueWalkingImitation2D_1env_1thread'] = {'us_per_step': 1e6 / r1, 'sample': s1}
    for tag, eid in (('C2', 'TorqueWalkingImitation2D-v0'), ('C4', 'MuscleRunningImitation3D-v0')):
        if eid != env_id:
            r, s = _cpu_rate(eid, cores, 3.0)
            extra[f'{tag}_{eid[:-3]}'] = {'value': r, 'unit': 'env-steps/s', 'cores': cores, 'sample': s}
    # C5: the mixed LockedKnee3D + Palsy3D batch, half the threads on each ID
    half = max(1, cores // 2)
    rl, sl = _cpu_rate('MuscleLockedKneeImitation3D-v0', half, 3.0)
    rp, sp = _cpu_rate('MusclePalsyImitation3D-v0', half, 3.0)
    extra['C5_MuscleLockedKneeImitation3D+MusclePalsyImitation3D'] = {
        'value': rl + rp, 'unit': 'env-steps/s', 'cores': 2 * half,
        'sample': f'LockedKnee3D {sl} on {half} threads + Palsy3D {sp} on {half} threads, concurrently equivalent'}
    r, s = _cpu_rate(env_id, cores, 4.0, n_per_thread=16, integrator='rk-merson')
    extra[f'{env_id[:-3]}_rk_merson'] = {'value': r, 'unit': 'env-steps/s', 'cores': cores, 'sample': s,
                                         'integrator': 'RK-Merson 1e-3 (the reference integrator)'}
    return {'value': value, 'unit': 'env-steps/s', 'cores': cores, 'kind': 'port',
            'sample': f'{sample}, {env_id}, fp64 C oracle (CPU restatement, not OpenSim), {cores} threads = '
                      f'the CPUs this process may use (affinity, cgroup quota), auto-reset on host',
            'configs': extra}


def single_env_rate(env_id='TorqueWalkingImitation2D-v0', steps=300):
    """The drop-in single-env path (bioimitation.envs.make(...).step, one env
    per handle, one launch + host round trip per step; the reference's RLlib /
    jaxrl scripts drive gym.make per worker this way), with and without the
    save_simulation recorder (record_trajectory): env-steps/s on C1's config
    (TorqueWalkingImitation2D-v0, 1 env), next to C1's CPU time per step."""
    import numpy as np
    from bioimitation import envs
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    out = {}
    for rec in (True, False):
        env = envs.make(env_id, config={'record_trajectory': rec})
        rng = np.random.default_rng(0)
        if pk.nmuscle:
            acts = rng.uniform(0.0, 1.0, size=(steps + 20, pk.nact))
        else:   # PD targets near the reference
            base = np.array([pk.ref_q[60][pk.pd_coord[a]] for a in range(pk.nact)])
            acts = base + rng.normal(0.0, 0.05, size=(steps + 20, pk.nact))
        env.reset()
        for k in range(20):
            if env.step(acts[k])[2]:
                env.reset()
        t0 = time.perf_counter()
        for k in range(steps):
            if env.step(acts[20 + k])[2]:
                env.reset()
        dt = time.perf_counter() - t0
        env.close()
        out['record_trajectory' if rec else 'no_recorder'] = {'value': steps / dt, 'unit': 'env-steps/s',
                                                              'us_per_step': 1e6 * dt / steps}
    out['note'] = (f'{env_id}, 1 env on cuda:0, {steps} timed steps (resets included); a step is a full '
                   f'kernel (nsub substeps) plus a host round trip: latency-bound by design (the batched '
                   f'VectorEnv is the throughput path)')
    return out


def _profile_record(name, key, build_id):
    """profiles/<name>[key] (rocprofv3 evidence, tools/ingest_evidence.py) with
    ``stale`` set when the record was taken on another build than the library
    this bench loaded (its ``build_id`` differs from bioim_build_id())"""
    path = os.path.join(REPO, 'profiles', name)
    if not os.path.exists(path):
        return None
    try:
        rec = json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None
    if rec is not None:
        rec = dict(rec)
        rec['stale'] = rec.get('build_id') != build_id
    return rec


def _spawn_ranks(a):
    """`bench.py --gpus N` run directly: start torch.distributed.run as a child
    (nothing in this process has touched a GPU) and return its exit status."""
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={a.gpus}',
           '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--burn-in', type=int, default=150,
                    help='untimed steps before the warmup, to reach the steady-state termination rate')
    ap.add_argument('--envs', type=int, default=4096, help='envs per GPU')
    ap.add_argument('--precision', type=int, default=int(os.environ.get('BIOIM_PRECISION', 64)))
    ap.add_argument('--env-id', default='MuscleWalkingImitation2D-v0')
    ap.add_argument('--integrator', default='semi-implicit', choices=['semi-implicit', 'rk-merson'],
                    help="'rk-merson': the reference's adaptive integrator at accuracy 1e-3 (DESIGN.md §3)")
    ap.add_argument('--rk-budget', type=int, default=0,
                    help='rk-merson only: attempts per env per launch (bioim_set_rk_budget); value counts the env '
                         'steps that finished')
    ap.add_argument('--no-reference-integrator', action='store_true',
                    help='skip the second measurement: the same workload with the reference integrator '
                         '(RK-Merson 1e-3, budgeted launches), reported as "reference_integrator"')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-single-env', action='store_true', help='skip the single-env (envs.make) rate')
    ap.add_argument('--mixed', default=None,
                    help="mixed batch 'ID_A,ID_B' split 50/50 per GPU (BASELINE config C5), e.g. "
                         "MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0")
    ap.add_argument('--no-reset-table', action='store_true',
                    help='run every in-kernel auto-reset as a reset realize in the step launch (bioim_set_reset_table 0)')
    ap.add_argument('--no-fuse', action='store_true',
                    help='mixed batch: concurrent per-segment launches instead of the fused two-topology kernel')
    ap.add_argument('--share-gpu', action='store_true',
                    help='REHEARSAL ONLY: let ranks share the visible GPU(s) (rank r on GPU r mod count) to run '
                         'the multi-rank path on a 1-GPU box; the line is marked "rehearsal" and is no scaling number')
    a = ap.parse_args()
    if a.rk_budget and (a.integrator != 'rk-merson' or a.mixed):
        ap.error('--rk-budget needs --integrator rk-merson and a single env id')

    if 'WORLD_SIZE' not in os.environ and a.gpus > 1:
        sys.exit(_spawn_ranks(a))
    world = int(os.environ.get('WORLD_SIZE', 1))
    if world != a.gpus:
        print(f'bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; refusing to report a mismatched n_gpus',
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get('RANK', 0))
    local = int(os.environ.get('LOCAL_RANK', 0))

    import numpy as np
    import torch
    if local >= torch.cuda.device_count():
        if not a.share_gpu:
            print(f'bench.py: rank {rank} needs GPU {local} but {torch.cuda.device_count()} are visible',
                  file=sys.stderr)
            sys.exit(2)
        local %= torch.cuda.device_count()
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('gloo')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    from bioimitation.vector_env import MixedVectorEnv, VectorEnv
    if a.mixed:
        from bioimitation import _lib
        _lib.load().bioim_set_group_fusion(0 if a.no_fuse else 1)
        ids = a.mixed.split(',')
        sizes = [a.envs // len(ids)] * len(ids)
        sizes[-1] += a.envs - sum(sizes)
        env = MixedVectorEnv(list(zip(ids, sizes)), config={'integrator': a.integrator}, device=local,
                             precision=a.precision, seed=1000, auto_reset=True, env_offset=rank * a.envs)
        env.pack, env.nsub, env.lanes_per_env = env.envs[0].pack, env.envs[0].nsub, env.envs[0].lanes_per_env
        env.launch = {e.env_id: e.launch for e in env.envs}
        a.env_id = '+'.join(ids)
        a.no_cpu_baseline = True
        handles = env.envs
    else:
        env = VectorEnv(a.env_id, a.envs, config={'integrator': a.integrator}, device=local, precision=a.precision,
                        seed=1000, auto_reset=True, env_offset=rank * a.envs)   # global env index block (parallel.py)
        handles = [env]
        if a.rk_budget:
            env.set_rk_budget(a.rk_budget)
    for h in handles:
        h.set_reset_table(not a.no_reset_table)
    n, A = a.envs, env.action_dim
    pool = 64      # action batches cycled through (uploaded once; inputs resident in HBM)
    gen = np.random.Generator(np.random.PCG64(rank))
    acts = torch.as_tensor(gen.uniform(0.0, 1.0, size=(pool, n, A)), dtype=env.dtype, device=dev)
    env.reset()
    stream = torch.cuda.current_stream(dev)
    k0 = a.burn_in
    if a.rk_budget:
        # budgeted launches finish fewer than n steps each: burn in by finished env steps, so the
        # timed region sees envs as far past their resets (and as often fallen) as the unbudgeted run
        fin = torch.zeros(n, dtype=torch.int32, device=dev)
        k0 = 0
        while k0 < 50 * a.burn_in and (k0 % 10 or int(fin.sum()) < n * a.burn_in):
            env.step(acts[k0 % pool])
            fin += env.ready
            k0 += 1
    else:
        for k in range(k0):
            env.step(acts[k % pool])
    torch.cuda.synchronize(dev)
    # the counters first, then the W warm-up steps: a counter read copies the state to the host and
    # leaves the GPU idle for milliseconds, and launches after an idle GPU run slower until its clocks
    # are back -- the untimed warm-up, not the timed steps, absorbs that.  done_rate and
    # evals_per_env_step therefore cover warm-up + timed steps; value covers the timed steps only
    resets0 = sum(h.reset_count() for h in handles)
    rk = a.integrator == 'rk-merson'
    rk = rk and all(hasattr(h._L, 'bioim_eval_count') for h in handles)   # older A/B builds lack the counter
    evals0 = sum(h.eval_count() for h in handles) if rk else 0
    # budgeted RK: envs whose step finished, from the launches' own counter (bioim_finished_count),
    # minus the warm-up's (summed from ready[] on the device during the warm-up)
    fin0 = env.finished_count() if a.rk_budget else 0
    wfin = torch.zeros(n, dtype=torch.int32, device=dev) if a.rk_budget else None
    for k in range(a.warmup):
        env.step(acts[(k0 + k) % pool])
        if wfin is not None:
            wfin += env.ready
    k0 += a.warmup

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(a.steps):
        env.step(acts[(k0 + k) % pool])
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
    fin1 = env.finished_count() if a.rk_budget else 0
    steps_local = fin1 - fin0 - int(wfin.sum()) if a.rk_budget else n * a.steps
    steps_counted = fin1 - fin0 if a.rk_budget else n * (a.warmup + a.steps)   # the counters' interval
    if dist:
        st_ = torch.tensor([steps_local], dtype=torch.float64)
        dist.all_reduce(st_)
        steps_total = float(st_[0])
    else:
        steps_total = steps_local
    value = steps_total / t_max
    done_rate = (sum(h.reset_count() for h in handles) - resets0) / max(steps_counted, 1)
    if rank == 0:
        real_bytes = 8 if a.precision == 64 else 4
        if a.mixed:   # env-weighted mean over the segments
            B = sum(algorithmic_bytes_per_env_step(e.pack, real_bytes) * e.num_envs for e in env.envs) / n
        else:
            B = algorithmic_bytes_per_env_step(env.pack, real_bytes)
        achieved = B * n / (kernel_ms * 1e-3) / 1e9
        key = f'{a.env_id}/fp{a.precision}/{n}'
        build_id = env.build_id
        tr = _profile_record('traffic.json', key, build_id)
        # rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per launch, only when measured on this very build
        traffic = tr['bytes'] if tr and not tr['stale'] else None
        roofline = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                    'traffic_over_algorithmic': traffic / (B * n) if traffic else None,
                    'bytes_per_env_step': B, 'kernel_ms': kernel_ms}
        if tr:
            roofline['traffic_source'] = tr.get('source')
            roofline['traffic_build_id'] = tr.get('build_id')
            roofline['traffic_stale'] = tr['stale']
        line = {
            'metric': 'env steps/sec (whole node), MuscleWalkingImitation2D-v0 @ 4096 envs/GPU'
            if a.env_id == 'MuscleWalkingImitation2D-v0' and n == 4096 else f'env steps/sec, {a.env_id} @ {n} envs/GPU',
            'value': value, 'unit': 'env-steps/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'burn_in': a.burn_in, 'ms_per_step': t_max / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': f'f{a.precision}', 'done_rate': done_rate, 'build_id': build_id,
            'data': 'synthetic: PCG64 U[0,1] muscle excitations; reference motion synthesized from the shipped 3D IK',
            **({'rehearsal': f'{world} ranks shared {torch.cuda.device_count()} GPU(s) (--share-gpu): the multi-rank '
                              'code path, not a scaling number'} if a.share_gpu else {}),
            'config': {'workload': f'{a.env_id} batched env.step, {n} envs/GPU, ' +
                       (f'nsub={env.nsub}' if a.integrator == 'semi-implicit' else 'RK-Merson 1e-3') + ', auto-reset',
                       'integrator': a.integrator, 'rk_budget': a.rk_budget or None,
                       'envs_per_gpu': n, 'lanes_per_env': env.lanes_per_env, 'parallelism': f'env-shard x{world}',
                       'launch': env.launch, 'reset_table': not a.no_reset_table,
                       **({'group_fusion': not a.no_fuse} if a.mixed else {})},
            'roofline': roofline,
        }
        valu = _profile_record('valu.json', key, build_id)
        if valu:   # the bound that is live for this kernel, from the rocprofv3 SQ passes
            line['valu'] = valu
        if a.rk_budget:
            line['finished_env_steps'] = steps_total
        if rk:
            line['evals_per_env_step'] = (sum(h.eval_count() for h in handles) - evals0) / max(steps_counted, 1)
        if not a.no_cpu_baseline and world == 1:
            line['cpu_baseline'] = cpu_baseline(a.env_id)
        if world == 1 and not a.mixed and not a.no_single_env:
            line['single_env'] = single_env_rate()
    env.close()
    if not (a.no_reference_integrator or a.integrator != 'semi-implicit'):
        ref = reference_integrator_rate(a, acts, pool, dev, stream, rank, world, dist)
        if rank == 0:
            line['reference_integrator'] = ref
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


RK_BUDGET = 6   # attempts per env per launch (DESIGN.md §3 sweep: best at 4096 envs for every ID measured)
RK_WARMUP = 10  # untimed launches between the counter reads and the timed launches (at least --warmup)


def reference_integrator_rate(a, acts, pool, dev, stream, rank, world, dist):
    """The same workload (env ID, envs per GPU, actions, auto-reset) with the
    reference's integrator: RK-Merson at accuracy 1e-3 in budgeted launches
    (bioim_set_rk_budget; trajectories identical to unbudgeted RK).  Burned in
    by finished env steps to the same horizon as the main measurement; value =
    env steps finished in a.steps timed launches over all ranks / max time.
    A mixed batch (C5) runs as a MixedVectorEnv whose segments each carry
    their own budget and ready rows (concurrent per-segment launches: the
    fused kernel is semi-implicit only)."""
    import torch
    from bioimitation.vector_env import MixedVectorEnv, VectorEnv
    n = a.envs
    if a.mixed:
        ids = a.mixed.split(',')
        sizes = [n // len(ids)] * len(ids)
        sizes[-1] += n - sum(sizes)
        env = MixedVectorEnv(list(zip(ids, sizes)), config={'integrator': 'rk-merson'}, device=dev.index,
                             precision=a.precision, seed=1000, auto_reset=True, env_offset=rank * n)
        segs = env.envs
    else:
        env = VectorEnv(a.env_id, n, config={'integrator': 'rk-merson'}, device=dev.index, precision=a.precision,
                        seed=1000, auto_reset=True, env_offset=rank * n)
        segs = [env]
    for e in segs:
        e.set_rk_budget(RK_BUDGET)
    env.reset()
    fin = torch.zeros(n, dtype=torch.int32, device=dev)
    fins, off = [], 0
    for e in segs:   # each segment's rows of fin
        fins.append(fin[off:off + e.num_envs])
        off += e.num_envs

    def count_ready():
        for f, e in zip(fins, segs):
            f += e.ready
    k0 = 0
    while k0 < 50 * a.burn_in and (k0 % 10 or int(fin.sum()) < n * a.burn_in):
        env.step(acts[k0 % pool])
        count_ready()
        k0 += 1
    # the counters, then the warm-up launches (as in main(): a counter read idles the GPU, and the
    # launches after it run slower until the clocks are back)
    resets0 = sum(e.reset_count() for e in segs)
    counted = hasattr(segs[0]._L, 'bioim_eval_count')    # older A/B builds lack the counter
    evals0 = sum(e.eval_count() for e in segs) if counted else 0
    # finished steps from the launches' own per-env counter (bioim_finished_count), so the timed
    # region holds the step launches only (summing ready[] after each launch cost 1 % on C3); the
    # warm-up's finished steps are summed from ready[] on the device and subtracted
    in_kernel = hasattr(segs[0]._L, 'bioim_finished_count')
    fin0 = sum(e.finished_count() for e in segs) if in_kernel else 0
    fin.zero_()
    warm = max(a.warmup, RK_WARMUP)
    for k in range(warm):
        env.step(acts[k0 % pool])
        count_ready()
        k0 += 1
    warm_fin = fin.clone()
    fin.zero_()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        env.step(acts[(k0 + k) % pool])
        if not in_kernel:
            count_ready()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    fin1 = sum(e.finished_count() for e in segs) if in_kernel else 0
    local = fin1 - fin0 - int(warm_fin.sum()) if in_kernel else int(fin.sum())
    # the counters' interval (warm-up + timed launches) for the per-step statistics
    counted_steps = fin1 - fin0 if in_kernel else local + int(warm_fin.sum())
    counted_launches = warm + a.steps
    tot, t_max = float(local), wall
    if dist:
        tt = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt[0])
        st_ = torch.tensor([float(local)], dtype=torch.float64)
        dist.all_reduce(st_)
        tot = float(st_[0])
    rate = {'value': tot / t_max, 'unit': 'finished env-steps/s', 'integrator': 'rk-merson', 'accuracy': 1e-3,
            'rk_budget': RK_BUDGET, 'launches': a.steps, 'ms_per_launch': t_max / a.steps * 1e3,
            'finished_env_steps': tot, 'done_rate': (sum(e.reset_count() for e in segs) - resets0) / max(counted_steps, 1),
            'evals_per_env_step': (sum(e.eval_count() for e in segs) - evals0) / max(counted_steps, 1) if counted else None,
            # share of the launches' attempt capacity (RK_BUDGET attempts x 5 evaluations per env) that
            # envs spent idle after finishing their step (attempt evaluations = all evaluations minus one
            # realize per finished step and one per reset)
            'launch_idle_share': (1.0 - (sum(e.eval_count() for e in segs) - evals0 - counted_steps -
                                         (sum(e.reset_count() for e in segs) - resets0)) / (counted_launches * n * 5 * RK_BUDGET))
            if counted else None,
            'note': "the reference's integrator (opensim_wrapper.py:287-301) on the same workload; "
                    'GPU parity vs the oracle in tests/test_gpu_parity.py (RK) and tests/test_gpu_rk_budget.py'}
    env.close()
    return rate


if __name__ == '__main__':
    main()
