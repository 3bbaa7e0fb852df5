"""Per-muscle / per-dof error of one GPU step (from the oracle's state) vs
the oracle: which lanes of an env disagree.  python tools/diag_lanes.py ENV_ID PREC"""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p)
                for p in ('bioimitation-gym_amd', 'oracle')]
import numpy as np
import torch
import oracle
from bioimitation.obslayout import column_names, load_names
from bioimitation.registry import load_pack
from bioimitation.vector_env import VectorEnv
env_id = sys.argv[1] if len(sys.argv) > 1 else 'MuscleWalkingImitation3D-v0'
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 32
pk = load_pack(env_id)
names = column_names(pk, load_names(env_id))
orc = oracle.Oracle(pk)
n = 32
rows = np.arange(n) * 3
bufs = orc.new_envs(n)
for i in range(n):
    orc.reset(bufs, i, int(rows[i]))
st = np.stack([orc.get_state(bufs, i) for i in range(n)])
env = VectorEnv(env_id, n, precision=prec)
env.reset(ref_index=rows)
env.set_state(st)
rng = np.random.default_rng(0)
acts = rng.uniform(0, 1, (n, env.action_dim)).astype(np.float32).astype(np.float64)
o, r, d, inf = env.step(torch.as_tensor(acts, device='cuda:0'))
o = o.cpu().numpy().astype(np.float64)
st2 = env.get_state()
ro = np.stack([orc.step(bufs, i, acts[i])[0] for i in range(n)])
rs = np.stack([orc.get_state(bufs, i) for i in range(n)])
e = np.abs(o - ro) / np.maximum(1, np.abs(ro))
print(env_id, 'prec', prec, 'max obs rel err', np.nanmax(e), 'nan rows', np.isnan(o).any(1).sum())
blocks = {}
for c, nm in enumerate(names):
    key = nm.split('.')[0] + ('.' + nm.split('.')[-1] if nm.startswith('muscles') else '')
    blocks.setdefault(key, []).append(c)
for k, cols in blocks.items():
    print(f'  {k:40s} {np.nanmax(e[:, cols]):.2e}')
if pk.nmuscle:
    nd, nm = pk.ndof, pk.nmuscle
    a = 5 + 2 * nd
    ea = np.abs(st2[:, a:a + nm] - rs[:, a:a + nm]).max(0)
    el = np.abs(st2[:, a + nm:a + 2 * nm] - rs[:, a + nm:a + 2 * nm]).max(0)
    print('  per-muscle act err ', np.array2string(ea, precision=1))
    print('  per-muscle lce err ', np.array2string(el, precision=1))
eu = np.abs(st2[:, 5 + pk.ndof:5 + 2 * pk.ndof] - rs[:, 5 + pk.ndof:5 + 2 * pk.ndof]).max(0)
print('  per-dof u err      ', np.array2string(eu, precision=1))
