import sys, os
REPO = os.environ.get('GRAFT_REPO_ROOT', '/root/repo')
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import numpy as np, torch
from bioimitation.vector_env import VectorEnv
env_id = sys.argv[1] if len(sys.argv) > 1 else 'TorqueWalkingImitation3D-v0'
n, T = 1024, 160
a = VectorEnv(env_id, n, precision=64, seed=5, auto_reset=True)
b = VectorEnv(env_id, n, precision=64, seed=5, auto_reset=True)
b.set_reset_table(False)
rows = np.random.default_rng(6).integers(0, a.pack.reset_hi + 1, size=n)
a.reset(ref_index=rows); b.reset(ref_index=rows)
g = torch.Generator(device='cuda').manual_seed(7)
pk = a.pack
prev_done = np.zeros(n, bool)
for t in range(T):
    st = a.get_state()[:, 1].astype(int) + 1
    base = np.array([[pk.ref_q[min(r, pk.nrows - 1)][pk.pd_coord[i]] for i in range(a.action_dim)] for r in st])
    act = torch.as_tensor(base, device=a.device) + 0.3 * torch.randn((n, a.action_dim), generator=g, device=a.device, dtype=torch.float64)
    oa, ra, da, ia = (x.clone() for x in a.step(act))
    ob, rb, db, ib = b.step(act)
    sa, sb = a.get_state(), b.get_state()
    d = da.cpu().numpy().astype(bool)
    bad = np.nonzero((sa != sb).any(1) | (ra != rb).cpu().numpy())[0]
    if len(bad):
        e = bad[0]
        cols = np.nonzero(sa[e] != sb[e])[0]
        print(f't={t} first bad env {e} (done now {d[e]}, done prev {prev_done[e]}); {len(bad)} envs; state cols {cols[:20]}; '
              f'values a {sa[e][cols[:6]]} b {sb[e][cols[:6]]}; reward {float(ra[e])} {float(rb[e])}')
        break
    prev_done = d
else:
    print('no mismatch in', T, 'steps')
