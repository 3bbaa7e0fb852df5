"""Diagnostics: fp32 vs fp64 GPU reset/step against the oracle, per obs block."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p) for p in ('bioimitation-gym_amd', 'oracle')]
import numpy as np, torch
import oracle
from bioimitation.registry import load_pack
from bioimitation.vector_env import VectorEnv
env_id = sys.argv[1] if len(sys.argv) > 1 else 'MuscleWalkingImitation2D-v0'
pk = load_pack(env_id)
orc = oracle.Oracle(pk)
n = 16
rows = np.array([0, 29, 58, 59, 116, 117, 132, 5, 10, 20, 40, 60, 80, 100, 120, 131])
bufs = orc.new_envs(n)
ref = np.stack([orc.reset(bufs, i, int(rows[i])) for i in range(n)])
rst = np.stack([orc.get_state(bufs, i) for i in range(n)])
np.set_printoptions(linewidth=200, precision=4)
for prec in (64, 32):
    env = VectorEnv(env_id, n, precision=prec)
    obs = env.reset(ref_index=rows).cpu().numpy().astype(np.float64)
    st = env.get_state()
    d = np.abs(obs - ref)
    print(f'--- prec {prec} reset: max abs obs err per column (top 10):')
    cols = np.argsort(-d.max(0))[:10]
    print('  cols', cols, '\n  err ', d.max(0)[cols], '\n  ref ', ref[np.argmax(d[:, cols], 0), cols])
    ds = np.abs(st - rst)
    print('  state err per column', np.argsort(-ds.max(0))[:8], np.sort(ds.max(0))[::-1][:8])
    # one step from identical state
    env.set_state(rst)
    rng = np.random.default_rng(0)
    acts = rng.uniform(0, 1, (n, env.action_dim))
    o, r, dn, inf = env.step(torch.as_tensor(acts, device='cuda:0'))
    o = o.cpu().numpy().astype(np.float64); r = r.cpu().numpy()
    b2 = orc.new_envs(n)
    for i in range(n): orc.set_state(b2, i, rst[i])
    ro = np.stack([orc.step(b2, i, acts[i].astype(np.float32).astype(np.float64) if prec == 32 else acts[i])[0] for i in range(n)])
    d = np.abs(o - ro) / np.maximum(1, np.abs(ro))
    cols = np.argsort(-d.max(0))[:10]
    print(f'  step rel err top cols', cols, d.max(0)[cols])
    env.close()
