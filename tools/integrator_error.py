"""Error of the step's integrators against the reference's integrator, on the
fp64 oracle (CPU): the kernel's fixed-substep semi-implicit scheme at several
nsub, extrapolated variants, and the RK-Merson mode, each against
Kutta-Merson at accuracy 1e-3 (OpenSim's Manager as the reference envs set it,
opensim_wrapper.py:287-301) and against a converged run (Kutta-Merson at
1e-9).  Same start rows, same open-loop actions on every integrator; episodes
masked at the first termination on either side.  Output: a markdown table
 and profiles/r02/integrator_error.json.

    python tools/integrator_error.py [T] [ids...]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd'), os.path.join(REPO, 'oracle')]

import oracle  # noqa: E402
from bioimitation.registry import load_pack  # noqa: E402

ROWS = [10, 40, 70, 100]
SCHEMES = [('semi-implicit nsub=20 (default)', 'euler', 0, 20), ('semi-implicit nsub=40', 'euler', 0, 40),
           ('semi-implicit nsub=80', 'euler', 0, 80), ('extrapolated order 2, 7 macro steps', 'extrap2', 7, None),
           ('extrapolated order 3, 7 macro steps', 'extrap3', 7, None),
           ('RK-Merson accuracy 1e-3 (reference)', 'rk-merson', 1e-3, None),
           ('RK-Merson accuracy 1e-4', 'rk-merson', 1e-4, None)]


def run(pk, orc, kind, acc, nsub, row, T, acts):
    b = orc.new_envs(1)
    if nsub:
        pk.nsub = nsub
    if kind != 'euler':
        orc.set_integrator(b, 0, kind, acc)
    orc.reset(b, 0, row)
    out = []
    for t in range(T):
        a = acts[t] if acts is not None else \
            np.array([pk.ref_q[min(row + t + 1, pk.nrows - 1)][pk.pd_coord[i]] for i in range(pk.nact)])
        o, r, d, _ = orc.step(b, 0, a)
        out.append((orc.get_state(b, 0)[5:5 + pk.ndof].copy(), r, o, d))
    pk.nsub = 20
    st = orc.rk_stats(b, 0)
    evals = (st[0] + st[1]) * (5 if kind == 'rk-merson' else 3) / T if kind != 'euler' else nsub
    if kind == 'extrap2':
        evals = 3 * acc
    if kind == 'extrap3':
        evals = 6 * acc
    return out, evals


def compare(o, ref, qdd):
    eq = er = eo = 0.0
    for t in range(len(o)):
        eq = max(eq, np.abs(o[t][0] - ref[t][0]).max())
        er = max(er, abs(o[t][1] - ref[t][1]))
        keep = np.ones(len(ref[t][2]), bool)
        keep[qdd] = False
        eo = max(eo, (np.abs(o[t][2] - ref[t][2]) / np.maximum(1, np.abs(ref[t][2])))[keep].max())
        if o[t][3] or ref[t][3]:
            break
    return eq, er, eo


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ids = sys.argv[2:] or ['MuscleWalkingImitation2D-v0', 'TorqueWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0']
    res = {}
    for env_id in ids:
        pk = load_pack(env_id)
        orc = oracle.Oracle(pk)
        ntr = sum(1 for c in (pk.coord_tx, pk.coord_ty, pk.coord_tz) if c >= 0)
        qdd = np.arange(1 + pk.ncoord - ntr + pk.ncoord, 1 + pk.ncoord - ntr + 2 * pk.ncoord)
        rng = np.random.default_rng(0)
        acts = rng.uniform(0, 0.4, (T, pk.nact)) if pk.nmuscle else None
        conv = {r: run(pk, orc, 'rk-merson', 1e-9, None, r, T, acts)[0] for r in ROWS}
        rkm = {r: run(pk, orc, 'rk-merson', 1e-3, None, r, T, acts)[0] for r in ROWS}
        print(f'\n{env_id}, {T} steps ({0.01 * T:.2f} s), rows {ROWS}, open-loop actions; max over rows\n')
        print('| integrator | evals / env step | vs RK-Merson 1e-3: max \\|q\\| err (rad or m) | reward err | obs rel err (q\'\' block excluded) | vs converged: max \\|q\\| err |')
        print('|---|---|---|---|---|---|')
        res[env_id] = {}
        for name, kind, acc, nsub in SCHEMES:
            e_ref, e_conv, ev = [], [], []
            for r in ROWS:
                o, evals = run(pk, orc, kind, acc, nsub, r, T, acts)
                e_ref.append(compare(o, rkm[r], qdd))
                e_conv.append(compare(o, conv[r], qdd))
                ev.append(evals)
            a, c = np.max(e_ref, 0), np.max(e_conv, 0)
            res[env_id][name] = dict(evals=float(np.mean(ev)), q_vs_rkm=a[0], reward_vs_rkm=a[1], obs_vs_rkm=a[2],
                                     q_vs_converged=c[0])
            print(f'| {name} | {np.mean(ev):.0f} | {a[0]:.1e} | {a[1]:.1e} | {a[2]:.1e} | {c[0]:.1e} |')
    out = os.path.join(REPO, 'profiles', 'r02', 'integrator_error.json')
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, 'w'), indent=1)


if __name__ == '__main__':
    main()
