"""A reference-tracking excitation drive for the muscle models (test
infrastructure: it reads the fp64 oracle's muscle paths; used by
tests/test_gpu_parity.py's 200-step C3 parity test and tools/c3_drive.py).

Per muscle a stretch reflex toward the reference motion: the excitation is
a0 + kl (L - L*) / l_opt + kv (dL/dt - dL*/dt) / l_opt, clipped to [0, 1],
where L* / dL*/dt are the muscle's path length and lengthening speed at the
reference row istep + 1 (SURVEY 8d's targets, the row the observation's
target block shows).  The floating base is not actuated by muscles, so the
trunk is balanced through the hips: the targets' hip angles move by
kb (tilt - tilt*) + kbd (tilt' - tilt'*) (pelvis tilt error), entered through
the linearization L* + dL/dq . dq.  Gains from a search on the oracle
(tools/c3_drive.py): this keeps MuscleWalkingImitation2D-v0 up for 200 steps
(2 s) from 18 of the reset rows 0..64, and the trajectories are not chaotic
under it (an oracle twin started one ulp away stays within ~1e-9).
"""
import numpy as np

GAINS = dict(a0=0.03, kl=20.0, kv=0.5, kb=-1.0, kbd=-0.05, kl_b=0.0, kld_b=0.0)
# reset rows of MuscleWalkingImitation2D-v0 from which the drive keeps the
# model up for 200 steps (oracle run, tools/c3_drive.py), and rows from
# which it falls between steps 70 and 200
ROWS_UP = [1, 2, 3, 4, 5, 6, 7, 17, 18, 21, 23, 24, 46, 47, 50, 51]
ROWS_FALL = [0, 8, 9, 10, 11, 12, 13, 14, 15, 16, 19, 20, 22, 25, 26, 27]


class TrackingDrive:
    def __init__(self, orc, pack, names, gains=None):
        self.orc, self.pk = orc, pack
        self.g = dict(GAINS, **(gains or {}))
        nd, nm = pack.ndof, pack.nmuscle
        self.nd, self.nm = nd, nm
        dof = {n: pack.coord[c].dof for c, n in enumerate(names['coords'])}
        self.hips = [dof['hip_flexion_r'], dof['hip_flexion_l']]
        self.tilt = dof['pelvis_tilt']
        # spatial models: the pelvis list is balanced through the hip adductions
        self.adds = [dof[n] for n in ('hip_adduction_r', 'hip_adduction_l') if dof.get(n, -1) >= 0]
        self.list = dof.get('pelvis_list', -1)
        # joints an ``offset`` moves (absent or locked ones are skipped)
        self.odofs = [dof.get(n, -1) for n in ('hip_flexion_r', 'hip_flexion_l', 'hip_adduction_r', 'hip_adduction_l',
                                               'knee_angle_r', 'knee_angle_l', 'ankle_angle_r', 'ankle_angle_l')]

        def dofs(tab, r):
            v = np.zeros(nd)
            for c in range(pack.ncoord):
                if pack.coord[c].dof >= 0:
                    v[pack.coord[c].dof] = tab[r][c]
            return v
        self.qref = np.array([dofs(pack.ref_q, r) for r in range(pack.nrows)])
        self.uref = np.array([dofs(pack.ref_u, r) for r in range(pack.nrows)])
        self.Lref = np.zeros((pack.nrows, nm))
        self.Ldref = np.zeros((pack.nrows, nm))
        for r in range(pack.nrows):
            self.Lref[r], self.Ldref[r], _ = orc.muscle_paths(self.qref[r], self.uref[r])
        self.lopt = np.array([pack.muscle[m].lopt for m in range(nm)])

    def __call__(self, state, offset=None):
        """excitations for one env's flat state (include/bioim.h layout);
        ``offset`` (hip flexion r/l, hip adduction r/l, knee r/l, ankle r/l,
        radians) moves those joint targets on top of the balance terms
        (tools/drive_search.py)"""
        g, nd = self.g, self.nd
        q, u = state[5:5 + nd], state[5 + nd:5 + 2 * nd]
        r = min(int(state[1]) + 1, self.pk.nrows - 1)
        bal = g['kb'] * (q[self.tilt] - self.qref[r, self.tilt]) + g['kbd'] * (u[self.tilt] - self.uref[r, self.tilt])
        dq = np.zeros(nd)
        dq[self.hips] = bal
        if self.adds:
            lb = g['kl_b'] * (q[self.list] - self.qref[r, self.list]) + g['kld_b'] * (u[self.list] - self.uref[r, self.list])
            dq[self.adds] = lb
        if offset is not None:
            for k, d in enumerate(self.odofs[:len(offset)]):
                if d >= 0:
                    dq[d] += offset[k]
        L, Ld, dL = self.orc.muscle_paths(q, u)
        e = g['a0'] + g['kl'] * (L - self.Lref[r] - dL @ dq) / self.lopt + g['kv'] * (Ld - self.Ldref[r]) / self.lopt
        return np.clip(e, 0.0, 1.0)


def load_schedule(env_id):
    """(rows, schedule [n][T/P][8], period P, gains) of the committed drive
    fixture tests/golden/drive_<env_id>.npz (made by tools/drive_search.py:
    reset rows by the reference's rule, random.seed + random.randint, and the
    hip/knee/ankle target offsets its lookahead search chose per P steps)"""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', f'drive_{env_id}.npz')
    with np.load(path, allow_pickle=False) as z:
        gains = {str(k): float(v) for k, v in zip(z['gain_names'], z['gain_values'])}
        return z['rows'].astype(int), z['schedule'].copy(), int(z['period']), gains


def twin_columns(nd):
    """state columns a one-ulp twin ensemble nudges: the first coordinate, the
    first speed, a joint angle, the last speed (include/bioim.h state layout)"""
    return [5, 5 + nd, 5 + nd // 2, 5 + 2 * nd - 1]


def make_twin(orc, bufs, i, col):
    s = orc.get_state(bufs, i)
    s[col] = np.nextafter(s[col], np.inf)
    orc.set_state(bufs, i, s)
