"""Per-phase cycle shares of the dynamics substep (diagnostic build
libbioim_stamps.so, -DBIOIM_STAMPS).  Read the shares, not absolute times."""
import ctypes as C, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ['BIOIM_LIB'] = os.path.join(REPO, 'bioimitation-gym_amd', 'build', 'libbioim_stamps.so')
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import numpy as np, torch
from bioimitation import _lib
from bioimitation.vector_env import VectorEnv
args = [x for x in sys.argv[1:] if not x.startswith('--')]
prec = int(args[0]) if args else 64
env_id = args[1] if len(args) > 1 else 'MuscleWalkingImitation2D-v0'
L = _lib.load()
f = L.bioim_debug_stamps
f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
rk = '--rk' in sys.argv
env = VectorEnv(env_id, 4096, config={'integrator': 'rk-merson'} if rk else None, precision=prec, seed=1,
                auto_reset=True)
if rk:
    env.set_rk_budget(6)
env.reset()
buf = (C.c_ulonglong * 24)()
steps = 30
acts = torch.rand((steps + 5, 4096, env.action_dim), device=env.device, dtype=env.dtype)
for k in range(5):
    env.step(acts[k])
torch.cuda.synchronize()
f(buf, 1)
for k in range(steps):
    env.step(acts[5 + k])
torch.cuda.synchronize()
f(buf, 1)
names = ['kin local (after slots)', 'kin compose (levels)', 'columns + inertias', 'subtree sums', 'muscle path',
         'muscle eval / actuators', 'contacts', 'limits + sync', 'M entries + rhs', 'cholesky']
tot = sum(buf[i] for i in range(len(names))) + buf[15]
print(f'  publish + function slots (phase 0/0b) {buf[15] / (steps * (env.nsub + 1)):9.0f} cyc  {100.0 * buf[15] / tot:5.1f} %')
calls = steps * (env.nsub + 1)
print(f'{env_id} fp{prec}: cycles per dynamics call {tot / calls:.0f} (workgroup 0, env 0)')
for i, n in enumerate(names):
    print(f'  {n:32s} {buf[i] / calls:9.0f} cyc  {100.0 * buf[i] / tot:5.1f} %')
print(f'  per launch: loop {buf[10] / steps:.0f} cyc, of which dynamics {tot / steps:.0f}; '
      f'model-image staging {buf[11] / steps:.0f} cyc')
if buf[21]:
    print(f'  report (wg 0, env 0): {buf[21]} reports, per report: observation {buf[19] / buf[21]:.0f} cyc, '
          f'reward + done + writes {buf[20] / buf[21]:.0f} cyc')
if buf[13]:
    print(f'  solve_fv (wg 0, env 0 lanes): mean iterations {buf[12] / buf[13]:.2f} over {buf[13]} solves, '
          f'{buf[14]} hit it_max')
if buf[16] or buf[17]:
    print(f'  muscle eval of lane 0 (wg 0, env 0), per dynamics call: curves + pennation {buf[16] / calls:.0f} cyc, '
          f'fiber-velocity solve {buf[17] / calls:.0f} cyc, rest {buf[18] / calls:.0f} cyc')
