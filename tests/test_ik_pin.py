"""Kinematics pinned to OpenSim's own output: the reference ships
InverseKinematicsTool solutions (task_InverseKinematics.mot) with their
inputs (task.trc markers, setup_ik.xml task weights, the model's MarkerSet);
tests/golden/make_ik_fixtures.py packs them into tests/golden/ik_*.npz.

OpenSim's IK minimises  f(q) = sum_i w_i |x_i(q) - x_i^exp|^2  over the free
coordinates (setup_ik.xml: 28 / 24 marker tasks, no coordinate tasks,
accuracy 1e-5).  If our model compiler reproduces OpenSim's forward
kinematics (CustomJoint axis order, SimmSpline knee translations, frame
offsets, scaling, welds and locked coordinates folded into composite
bodies), every IK frame is a stationary point of f built on OUR kinematics:
the Gauss-Newton step  dq = -(J^T W J)^-1 J^T W r  that would improve it is
~0.  Measured on the committed ModelPacks (fp64 oracle FK, central-difference
Jacobian): median over frames of max_coord |dq| = 2.0e-3 rad (3D trial),
1.4e-3 rad (02905 trial); largest 1.2e-2 rad, in the ankle angles (two
foot markers per foot).  A mutation of the pack shows what an error would
look like: a knee axis flipped gives 0.29 / 0.82 rad, the knee translation
splines swapped 1.2 / 1.6 rad, a 2 % longer right shank 0.029 / 0.025 rad,
i.e. >= 10x the unmutated step, while the marker RMS barely moves for the
last one (11.0 -> 11.8 mm): stationarity, not the residual, is the sharp
check.

The marker RMS itself is a weaker check (measurement noise, marker
placement): 11 mm median on the 3D trial; 60 mm on the 02905 trial, whose
MarkerSet sits centimetres off the measured markers (RKNE/LKNE ~9 cm, C7/T10
~10 cm) — the IK solution is nevertheless a stationary point there too.

The oracle consumes the same ModelPack as the HIP kernel, and
tests/test_gpu_golden.py::test_ik_frames_body_positions_on_hip_path checks
the kernel's reported body positions at these IK frames against the
oracle's FK, so the chain OpenSim IK -> oracle FK -> HIP path is closed.
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TRIALS = ['3D', '02905']
BOUNDS = {  # (median max-step rad, max max-step rad, median marker RMS m)
    '3D': (5e-3, 2e-2, 0.015),
    '02905': (5e-3, 2e-2, 0.075),
}


def load_trial(tag):
    return dict(np.load(os.path.join(HERE, 'golden', f'ik_{tag}.npz'), allow_pickle=False))


class MarkerModel:
    """Marker positions on the oracle's FK of a ModelPack (fp64)."""

    def __init__(self, oracle_lib, z, pk=None, mutate=None):
        from bioimitation.obslayout import load_names
        from bioimitation.registry import load_pack
        env_id = str(z['env_id'])
        self.pk = pk or load_pack(env_id)
        names = load_names(env_id)
        if mutate:
            mutate(self.pk, names)
        assert list(z['coords']) == names['coords']
        self.orc = oracle_lib.Oracle(self.pk)
        self.bidx = np.array([names['bodies'].index(str(b)) for b in z['bodies']])
        self.dof = np.array([self.pk.coord[c].dof for c in range(self.pk.ncoord)])
        self.free = [c for c in range(self.pk.ncoord) if self.dof[c] >= 0]
        self.L = z['locations']
        self.names = names

    def qdof(self, qc):
        qd = np.zeros(self.pk.ndof)
        for c in self.free:
            qd[self.dof[c]] = qc[c]
        return qd

    def markers(self, qc):
        R, p, _ = self.orc.fk(self.qdof(qc))
        return p[self.bidx] + np.einsum('mij,mj->mi', R[self.bidx], self.L)

    def gauss_newton_step(self, qc, x_exp, w, h=1e-6):
        r = self.markers(qc) - x_exp
        J = np.zeros((r.size, len(self.free)))
        for j, c in enumerate(self.free):
            qp, qm = qc.copy(), qc.copy()
            qp[c] += h
            qm[c] -= h
            J[:, j] = ((self.markers(qp) - self.markers(qm)) / (2 * h)).ravel()
        sw = np.repeat(np.sqrt(w), 3)
        dq = np.linalg.lstsq(J * sw[:, None], -(sw * r.ravel()), rcond=None)[0]
        return dq, np.sqrt((r ** 2).sum(1).mean())


def stationarity(oracle_lib, z, stride=1, mutate=None):
    mm = MarkerModel(oracle_lib, z, mutate=mutate)
    steps, rms = [], []
    for f in range(0, len(z['q']), stride):
        dq, e = mm.gauss_newton_step(z['q'][f], z['x_exp'][f], z['weights'])
        steps.append(np.abs(dq).max())
        rms.append(e)
    return np.array(steps), np.array(rms)


@pytest.mark.parametrize('tag', TRIALS)
def test_ik_solution_is_stationary_on_our_kinematics(tag, oracle_lib):
    z = load_trial(tag)
    assert float(z['accuracy']) == 1e-5 and len(z['q']) > 150
    # no IK solution sits on a clamped coordinate bound (the stationarity is unconstrained)
    lo, hi = z['ranges'][:, 0], z['ranges'][:, 1]
    at_bound = z['clamped'] & ((np.abs(z['q'] - lo) < 1e-9) | (np.abs(z['q'] - hi) < 1e-9))
    assert not at_bound.any()
    steps, rms = stationarity(oracle_lib, z)
    med_b, max_b, rms_b = BOUNDS[tag]
    print(f'{tag}: {len(steps)} IK frames, Gauss-Newton max step median {np.median(steps):.2e} rad, '
          f'max {steps.max():.2e} rad; marker RMS median {np.median(rms) * 1e3:.1f} mm')
    assert np.median(steps) < med_b and steps.max() < max_b
    assert np.median(rms) < rms_b


def _knee_fns(pk, names, coord='knee_angle_r'):
    ci = names['coords'].index(coord)
    return [(b, k, pk.cbody[b].fn[k]) for b in range(pk.ncbody) for k in range(6)
            if pk.cbody[b].fn[k] >= 0 and pk.fn[pk.cbody[b].fn[k]].coord == ci]


def flip_knee_axis(pk, names):
    b, k, _ = [x for x in _knee_fns(pk, names) if x[1] < 3][0]
    for i in range(3):
        pk.cbody[b].axis[k][i] *= -1


def swap_knee_splines(pk, names):
    (_, _, f0), (_, _, f1) = [x for x in _knee_fns(pk, names) if x[1] >= 3][:2]
    pk.fn[f0].knot_off, pk.fn[f1].knot_off = pk.fn[f1].knot_off, pk.fn[f0].knot_off


def longer_right_shank(pk, names):
    cb = pk.osbody[names['bodies'].index('talus_r')].cbody
    for i in range(3):
        pk.cbody[cb].p_pf[i] *= 1.02


@pytest.mark.parametrize('tag', TRIALS)
@pytest.mark.parametrize('mutation', [flip_knee_axis, swap_knee_splines, longer_right_shank])
def test_ik_stationarity_catches_kinematic_errors(tag, mutation, oracle_lib):
    """The check has teeth: each pack mutation moves the IK frames off
    stationarity by >= 5x the unmutated Gauss-Newton step."""
    z = load_trial(tag)
    base, _ = stationarity(oracle_lib, z, stride=6)
    mut, _ = stationarity(oracle_lib, z, stride=6, mutate=mutation)
    print(f'{tag} {mutation.__name__}: median max step {np.median(base):.2e} -> {np.median(mut):.2e} rad')
    assert np.median(mut) > 5 * np.median(base)
