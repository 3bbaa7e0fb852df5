"""the Palsy3D drive's worst GPU/twin ratio (step 2, env 28,
reset row 46, coordinate_acc.hip_adduction_r: GPU 1.5e-9 from the oracle while
four one-ulp twins stay within 5.4e-13; tests/test_gpu_parity.py
test_parity_200_steps_muscle_tracking_drive, profiles/r06/r06b) is not moved by
the reciprocal / inverse-square-root refinements nor by FMA contraction (the
BIOIM_EXACT_RCP and -ffp-contract=off builds give the same ratio).  This CPU
script (test infrastructure: the oracle) rebuilds that env's state at the
realize of step 2 and asks how much of q'' the factorization itself decides:
M (the oracle's mass matrix, column by column through orc_id_eval) and the
realize's right-hand side b = M q'' are solved by the oracle's Cholesky order
and by the reverse-order (tree LTL, Featherstone 6.3, the kernel's
factorization) on the same inputs.  One-ulp twins of the *state* do not see
that channel: they run the same factorization.

    python tools/palsy_qdd_solver.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'oracle'), os.path.join(REPO, 'tests'), os.path.join(REPO, 'bioimitation-gym_amd')]
import oracle  # noqa: E402
from tracking import TrackingDrive, load_schedule  # noqa: E402
from bioimitation.obslayout import column_names, load_names  # noqa: E402
from bioimitation.registry import load_pack  # noqa: E402

ENV, ENV_I, STEPS = 'MusclePalsyImitation3D-v0', 28, 2


def ltl_solve(A, b):
    """A = L^T L with L lower triangular, factorized from the last dof up (the
    tree LTL order; dense here), then L^T y = b, L x = y"""
    n = len(b)
    L = np.tril(A).astype(np.float64).copy()
    for k in range(n - 1, -1, -1):
        L[k, k] = np.sqrt(L[k, k])
        for i in range(k):
            L[k, i] /= L[k, k]
        for i in range(k - 1, -1, -1):
            for j in range(i + 1):
                L[i, j] -= L[k, i] * L[k, j]
    y = b.astype(np.float64).copy()
    for k in range(n - 1, -1, -1):          # L^T y = b
        y[k] /= L[k, k]
        for i in range(k):
            y[i] -= L[k, i] * y[k]
    x = y.copy()
    for k in range(n):                      # L x = y
        for i in range(k):
            x[k] -= L[k, i] * x[i]
        x[k] /= L[k, k]
    return x


def chol_solve(A, b):
    Lc = np.linalg.cholesky(A)
    y = np.linalg.solve(Lc, b)
    return np.linalg.solve(Lc.T, y)


def main():
    pk = load_pack(ENV)
    names = column_names(pk, load_names(ENV))
    rows, sched, P, gains = load_schedule(ENV)
    orc = oracle.Oracle(pk)
    bufs = orc.new_envs(1)
    drive = TrackingDrive(orc, pk, load_names(ENV), gains)
    orc.reset(bufs, 0, int(rows[ENV_I]))
    for t in range(STEPS):
        a = drive(orc.get_state(bufs, 0), sched[ENV_I, t // P])
        obs, _, _, _ = orc.step(bufs, 0, a)
    s = orc.get_state(bufs, 0)
    nd, nm = pk.ndof, pk.nmuscle
    q, u = s[5:5 + nd], s[5 + nd:5 + 2 * nd]
    M = np.stack([orc.id_eval(2, q, u, np.eye(nd)[k]) for k in range(nd)], 1)
    M = 0.5 * (M + M.T)
    qa = [i for i, nme in enumerate(names) if nme.startswith('coordinate_acc.')]
    dof_of = {c: pk.coord[c].dof for c in range(pk.ncoord)}
    qdd_obs = obs[qa]
    qdd = np.zeros(nd)
    for c in range(pk.ncoord):
        if dof_of[c] >= 0:
            qdd[dof_of[c]] = qdd_obs[c]
    b = M @ qdd
    x_c, x_l = chol_solve(M, b), ltl_solve(M, b)
    rel = np.abs(x_c - x_l) / np.maximum(1.0, np.abs(x_c))
    cname = {dof_of[c]: names[qa[c]] for c in range(pk.ncoord) if dof_of[c] >= 0}
    ev = np.linalg.eigvalsh(M)
    print(f'{ENV} env {ENV_I} (reset row {rows[ENV_I]}), realize of step {STEPS}: cond(M) = {ev[-1] / ev[0]:.2e} '
          f'(eigenvalues {ev[0]:.2e} .. {ev[-1]:.2e})')
    print('q\'\' by the Cholesky order vs the LTL order on the same M and b, relative to max(|q\'\'|, 1):')
    for d in np.argsort(rel)[::-1][:6]:
        print(f'  {cname[d]:40s} {x_c[d]: .6e}  {rel[d]:.2e}')


if __name__ == '__main__':
    main()


def lce_sensitivity(rel=1e-13):
    """the same env's q'' at the realize of step 2 when one muscle's reset
    fiber length is moved by `rel` (relative): the size of the fiber-length
    channel against the twins' one-ulp coordinate perturbations"""
    pk = load_pack(ENV)
    names = column_names(pk, load_names(ENV))
    rows, sched, P, gains = load_schedule(ENV)
    orc = oracle.Oracle(pk)
    drive = TrackingDrive(orc, pk, load_names(ENV), gains)
    qa = [i for i, nme in enumerate(names) if nme.startswith('coordinate_acc.')]
    nd, nm = pk.ndof, pk.nmuscle

    def run(m=None, scale=0.0):
        b = orc.new_envs(1)
        orc.reset(b, 0, int(rows[ENV_I]))
        if m is not None:
            s = orc.get_state(b, 0)
            s[5 + 2 * nd + nm + m] *= 1.0 + scale
            orc.set_state(b, 0, s)
        for t in range(STEPS):
            a = drive(orc.get_state(b, 0), sched[ENV_I, t // P])
            obs, _, _, _ = orc.step(b, 0, a)
        return obs

    base = run()
    worst = []
    for m in range(nm):
        o = run(m, rel)
        d = np.abs(o - base) / np.maximum(1.0, np.abs(base))
        j = int(np.argmax(d[qa]))
        worst.append((float(d[qa].max()), m, names[qa[j]], float(d.max())))
    worst.sort(reverse=True)
    print(f'reset fiber length of one muscle moved by {rel:.0e} (relative): largest q\'\' change at the realize of step {STEPS}:')
    for w, m, c, dall in worst[:5]:
        print(f'  muscle {m:2d} ({load_names(ENV)["muscles"][m]}): {w:.2e} in {c} (any column {dall:.2e})')


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'lce':
    lce_sensitivity(float(sys.argv[2]) if len(sys.argv) > 2 else 1e-13)
