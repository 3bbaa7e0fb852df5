"""GPU vs oracle on reset + one step for one env ID: prints every mismatched
observation column (name, GPU value, oracle value) for the first envs.
    python tools/diag_parity.py <env_id> [precision] [n]"""
import sys
import numpy as np
import torch
sys.path[:0] = ['bioimitation-gym_amd', 'oracle']
import oracle
from bioimitation.obslayout import column_names, load_names
from bioimitation.registry import load_pack
from bioimitation.vector_env import VectorEnv

env_id = sys.argv[1]
prec = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = int(sys.argv[3]) if len(sys.argv) > 3 else 16
pk = load_pack(env_id)
names = column_names(pk, load_names(env_id))
env = VectorEnv(env_id, n, precision=prec)
orc = oracle.Oracle(pk)
bufs = orc.new_envs(n)
rows = np.arange(n) * 3
obs = env.reset(ref_index=rows).cpu().numpy()
ref = np.stack([orc.reset(bufs, i, int(rows[i])) for i in range(n)])
tol = 1e-7 if prec == 64 else 1e-3
for tag, o, r in [('reset', obs, ref)]:
    bad = np.abs(o - r) > tol * np.maximum(1, np.abs(r))
    print(tag, 'bad envs', np.nonzero(bad.any(1))[0].tolist())
    for c in np.nonzero(bad.any(0))[0]:
        print(f'  {names[c]:40s} gpu {o[:4, c]} oracle {r[:4, c]}')
acts = np.random.default_rng(0).uniform(0, 1, (n, env.action_dim))
o, rw, d, inf = env.step(torch.as_tensor(acts, device='cuda', dtype=env.dtype))
o = o.cpu().numpy()
ro = np.stack([orc.step(bufs, i, acts[i])[0] for i in range(n)])
bad = np.abs(o - ro) > tol * np.maximum(1, np.abs(ro))
print('step bad envs', np.nonzero(bad.any(1))[0].tolist())
for c in np.nonzero(bad.any(0))[0]:
    print(f'  {names[c]:40s} gpu {o[:4, c]} oracle {ro[:4, c]}')
