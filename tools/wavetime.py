"""Per-wave durations of the step kernel (diagnostic single-TU build with
-DBIOIM_WAVETIME, built by this script into build/libbioim_wavetime.so):
the launch lasts as long as its slowest wave, so the gap between the mean
and the maximum wave duration is time lost to imbalance (resets, Newton
iteration counts, divergent branches).

    python tools/wavetime.py [env_id] [--no-reset-table]   (GPU box; build first on the CPU: --build)
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
env = VectorEnv(env_id, n, precision=64, seed=1000, auto_reset=True)
env.set_reset_table('--no-reset-table' not in sys.argv)
gen = np.random.Generator(np.random.PCG64(0))
acts = torch.as_tensor(gen.uniform(0, 1, size=(64, n, env.action_dim)), device=env.device)
env.reset()
for k in range(150):
    env.step(acts[k % 64])
nw = env.launch['workgroups'] * env.launch['threads_per_workgroup'] // 64
buf = (C.c_ulonglong * nw)()
rows = []
raw = []
for k in range(20):
    r0 = int(env.done.sum()) if k else 0
    env.step(acts[k % 64])
    f(buf, nw)
    d = np.array(buf[:], dtype=np.float64)
    raw.append([d])
    rows.append((d.mean(), np.median(d), np.percentile(d, 90), np.percentile(d, 99), d.max(), int(env.done.sum())))
a = np.array(rows)
out = os.environ.get('WAVETIME_OUT')
if out:   # raw per-wave cycles of the 20 launches, for offline analysis
    np.save(out, np.array([r[0] for r in raw]))
print(f'{env_id} reset_table={"--no-reset-table" not in sys.argv}: {nw} waves, 20 launches; wave cycles '
      f'mean {a[:, 0].mean():.0f}  p50 {a[:, 1].mean():.0f}  p90 {a[:, 2].mean():.0f}  p99 {a[:, 3].mean():.0f}  '
      f'max {a[:, 4].mean():.0f}; mean/max {np.mean(a[:, 0] / a[:, 4]):.3f}; dones per launch {a[:, 5].mean():.1f}')
