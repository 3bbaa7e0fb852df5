"""Noise floor of the golden replay: the oracle replaying each golden episode
from a state one ulp away (first coordinate), max relative error vs the
fixture per step.  python tools/golden_twin.py <env-id> ..."""
import ast, sys, numpy as np
sys.path[:0] = ['bioimitation-gym_amd', 'oracle', '.']
import oracle as O
from bioimitation.registry import load_pack
def rel(a, b): return np.abs(np.asarray(a) - b) / np.maximum(1.0, np.abs(b))
for env_id in sys.argv[1:]:
    z = np.load(f'tests/golden/{env_id}.npz', allow_pickle=False)
    worst_t = {}
    for i in range(int(z['n_episodes'])):
        ep = {k[len(f'ep{i}_'):]: z[k] for k in z.files if k.startswith(f'ep{i}_')}
        if 'chained' in ep: continue
        cfg = ast.literal_eval(str(ep['config']))
        orc = O.Oracle(load_pack(env_id, cfg)); e = orc.new_envs(1)
        orc.reset(e, 0, int(ep['index']))
        s = orc.get_state(e, 0); s[5] = np.nextafter(s[5], np.inf); orc.set_state(e, 0, s)
        for t in range(len(ep['reward'])):
            o, r, d, info = orc.step(e, 0, ep['actions'][t])
            err = max(rel(o, ep['obs'][t]).max(), rel(r, ep['reward'][t]), rel(info, ep['info'][t]).max())
            worst_t[t] = max(worst_t.get(t, 0), err)
    print(env_id, ' '.join(f'{t}:{v:.1e}' for t, v in sorted(worst_t.items()) if t % 5 == 0 or t > 20))
