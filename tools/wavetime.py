"""Per-wave durations of the step kernel (diagnostic single-TU build with
-DBIOIM_WAVETIME, built by this script into build/libbioim_wavetime.so):
the launch lasts as long as its slowest wave, so the gap between the mean
and the maximum wave duration is time lost to imbalance (resets, Newton
iteration counts, divergent branches).

    python tools/wavetime.py [env_id] [--no-reset-table] [--rk]   (GPU box; build first on the CPU: --build)

--rk: the reference integrator in 6-attempt budgeted launches (bench.py's
reference_integrator_rate), burned in by finished steps; the per-wave cycles
are then split by how many of the wave's envs finished their step in the launch.
"""
import ctypes as C
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, 'bioimitation-gym_amd', 'build', 'libbioim_wavetime.so')
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), REPO]

if '--build' in sys.argv:
    from bioimitation import _buildinfo
    src = os.path.join(REPO, 'bioimitation-gym_amd', 'csrc', 'bioim_step.hip')
    subprocess.check_call(['hipcc'] + _buildinfo.hipcc_flags(['-DBIOIM_WAVETIME']) +
                          ['-DBIOIM_BUILD_ID="wavetime"', '-shared', '-o', LIB, src])
    sys.exit(0)

os.environ['BIOIM_LIB'] = LIB
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bioimitation import _lib  # noqa: E402
from bioimitation.vector_env import VectorEnv  # noqa: E402

args = [x for x in sys.argv[1:] if not x.startswith('--')]
env_id = args[0] if args else 'MuscleWalkingImitation2D-v0'
L = _lib.load()
f = L.bioim_debug_wavetime
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
n = 4096
rk = '--rk' in sys.argv
env = VectorEnv(env_id, n, config={'integrator': 'rk-merson'} if rk else None, precision=64, seed=1000,
                auto_reset=True)
env.set_reset_table('--no-reset-table' not in sys.argv)
if rk:
    env.set_rk_budget(6)
gen = np.random.Generator(np.random.PCG64(0))
acts = torch.as_tensor(gen.uniform(0, 1, size=(64, n, env.action_dim)), device=env.device)
env.reset()
if rk:
    fin = torch.zeros(n, dtype=torch.int32, device=env.device)
    k0 = 0
    while k0 < 50 * 155 and (k0 % 10 or int(fin.sum()) < n * 155):
        env.step(acts[k0 % 64])
        fin += env.ready
        k0 += 1
else:
    for k in range(150):
        env.step(acts[k % 64])
epw = 64 // env.lanes_per_env if env.lanes_per_env <= 64 else 1
by_fin = {}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
kms = []
nw = env.launch['workgroups'] * env.launch['threads_per_workgroup'] // 64
buf = (C.c_ulonglong * nw)()
fvf = getattr(L, 'bioim_debug_fviter', None)
nt = nw * 64
fvb = (C.c_uint * (3 * nt))()
if fvf is not None:
    fvf.argtypes = [C.POINTER(C.c_uint), C.c_int]
fv_rows = []
rows = []
raw = []
for k in range(20):
    r0 = int(env.done.sum()) if k else 0
    torch.cuda.synchronize()
    ev0.record()
    env.step(acts[k % 64])
    ev1.record()
    torch.cuda.synchronize()
    kms.append(ev0.elapsed_time(ev1))
    f(buf, nw)
    d = np.array(buf[:], dtype=np.float64)
    raw.append([d])
    # RK: envs of the wave that finished their step in the launch; semi-implicit: envs that were done
    # (and reset in the launch)
    rd = (env.ready if rk else env.done).cpu().numpy().astype(np.int64)
    nf = rd[:nw * epw].reshape(nw, epw).sum(1)
    for c in range(epw + 1):
        by_fin.setdefault(c, []).extend(d[nf == c].tolist())
    if fvf is not None:
        fvf(fvb, nt)
        it = np.array(fvb[:nt], dtype=np.float64).reshape(nw, 64)
        mx = np.array(fvb[nt:2 * nt], dtype=np.float64).reshape(nw, 64)
        bi = np.array(fvb[2 * nt:], dtype=np.float64).reshape(nw, 64)
        fv_rows.append((d, it.max(1), mx.max(1), bi.sum(1)))
    rows.append((d.mean(), np.median(d), np.percentile(d, 90), np.percentile(d, 99), d.max(), int(env.done.sum())))
a = np.array(rows)
if fv_rows:
    d = np.concatenate([r[0] for r in fv_rows]); itm = np.concatenate([r[1] for r in fv_rows])
    mxm = np.concatenate([r[2] for r in fv_rows]); bis = np.concatenate([r[3] for r in fv_rows])
    slow = d > np.percentile(d, 90)
    print(f'  fiber-velocity Newton per wave (max over its lanes of the launch total / of one solve; bisections): '
          f'all waves {itm.mean():.1f} / {mxm.mean():.1f}; {bis.mean():.2f};  slowest 10 % {itm[slow].mean():.1f} / '
          f'{mxm[slow].mean():.1f}; {bis[slow].mean():.2f};  corr(cycles, lane-max total) {np.corrcoef(d, itm)[0, 1]:.2f}, '
          f'corr(cycles, bisections) {np.corrcoef(d, bis)[0, 1]:.2f}')
out = os.environ.get('WAVETIME_OUT')
if out:   # raw per-wave cycles of the 20 launches, for offline analysis
    np.save(out, np.array([r[0] for r in raw]))
for c in sorted(by_fin):
    v = np.array(by_fin[c])
    if len(v):
        what = 'finishing their step' if rk else 'done (reset in the launch)'
        print(f'  waves with {c} of {epw} envs {what}: {len(v) / 20:.1f} per launch, cycles mean '
              f'{v.mean():.0f} p99 {np.percentile(v, 99):.0f} max {v.max():.0f}')
allw = np.concatenate([r[0] for r in raw])
top = allw >= np.percentile(allw, 99.5)
print(f'  slowest 0.5 % of waves: {top.sum()} waves')
print(f'  launch (events) {np.mean(kms) * 1e3:.1f} us; max wave {a[:, 4].mean():.0f} memtime ticks '
      f'(= {a[:, 4].mean() / (np.mean(kms) * 1e3):.0f} ticks per us of launch)')
print(f'{env_id} rk={rk} reset_table={"--no-reset-table" not in sys.argv}: {nw} waves, 20 launches; wave cycles '
      f'mean {a[:, 0].mean():.0f}  p50 {a[:, 1].mean():.0f}  p90 {a[:, 2].mean():.0f}  p99 {a[:, 3].mean():.0f}  '
      f'max {a[:, 4].mean():.0f}; mean/max {np.mean(a[:, 0] / a[:, 4]):.3f}; dones per launch {a[:, 5].mean():.1f}')
