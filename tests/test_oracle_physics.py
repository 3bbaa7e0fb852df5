"""Physics invariants of the fp64 oracle (parity with OpenSim itself is
unpinned — OpenSim is not available — so the restatement is checked against
mechanics identities instead).  Every invariant runs on
the planar model and on the spatial models (3D rotations, locked coordinates,
the prosthetic topology, the shipped palsy model)."""
import os

import numpy as np
import pytest

from bioimitation.registry import load_pack

ENVS = ['MuscleWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0', 'MuscleLockedKneeImitation3D-v0',
        'MusclePalsyImitation3D-v0']
REF_DATA = '/root/reference/bioimitation/imitation_envs/data'


@pytest.fixture(scope='module', params=ENVS)
def orc(request, oracle_lib):
    return oracle_lib.Oracle(load_pack(request.param))


def dof_of(pk, name_index):
    return pk.coord[name_index].dof


def ref_dofs(pk, row):
    """reference row r as a dof vector (locked coordinates dropped)"""
    q = np.zeros(pk.ndof)
    u = np.zeros(pk.ndof)
    for c in range(pk.ncoord):
        d = pk.coord[c].dof
        if d >= 0:
            q[d], u[d] = pk.ref_q[row][c], pk.ref_u[row][c]
    return q, u


def random_q(pk, rng, scale=0.5):
    """random pose around reference row 40"""
    q, _ = ref_dofs(pk, 40)
    return q + rng.normal(0, scale, pk.ndof)


def test_forward_kinematics_matches_raw_joint_chain(orc):
    """Composite-body FK (compiled pack) == FK straight from the parsed joints."""
    from bioimitation import modelpack, registry
    if not os.path.isdir(REF_DATA):
        pytest.skip('reference data not present')
    pk = orc.pack
    m = registry.build_model(pk.env_id.decode(), REF_DATA)
    rng = np.random.default_rng(0)
    for _ in range(5):
        q = random_q(pk, rng)
        R, p, com = orc.fk(q)
        qv = {c: q[pk.coord[i].dof] for i, c in enumerate(m.coord_order) if pk.coord[i].dof >= 0}
        poses, com2 = modelpack.raw_forward_kinematics(m, qv)
        for i, b in enumerate(m.body_order):
            np.testing.assert_allclose(p[i], poses[b][1], atol=1e-13)
            np.testing.assert_allclose(R[i], poses[b][0], atol=1e-13)
        np.testing.assert_allclose(com, com2, atol=1e-13)


def test_mass_matrix_spd_and_translational_mass(orc):
    pk = orc.pack
    rng = np.random.default_rng(1)
    trans = [pk.coord[c].dof for c in (pk.coord_tx, pk.coord_ty, pk.coord_tz) if c >= 0]
    for _ in range(5):
        M, _ = orc.mass_bias(random_q(pk, rng), rng.normal(0, 1, pk.ndof))
        assert np.abs(M - M.T).max() == 0.0
        assert np.linalg.eigvalsh(M).min() > 0
        for d in trans:      # pelvis translations are along ground axes: the whole mass
            assert abs(M[d, d] - pk.total_mass) < 1e-9


@pytest.mark.parametrize('env_id', ENVS)
def test_bias_equals_lagrangian_coriolis(oracle_lib, env_id):
    """bias(q,u) with g=0 equals Mdot u - 1/2 d(u'Mu)/dq (finite differences)."""
    pk = load_pack(env_id)
    pk.gravity[1] = 0.0
    o = oracle_lib.Oracle(pk)
    rng = np.random.default_rng(2)
    h = 1e-6
    nd = pk.ndof
    for _ in range(3):
        q, u = random_q(pk, rng), rng.normal(0, 2, nd)
        M, b = o.mass_bias(q, u)
        Md = np.zeros_like(M)
        grad = np.zeros(nd)
        for k in range(nd):
            e = np.zeros(nd); e[k] = h
            Mp, _ = o.mass_bias(q + e, u)
            Mm, _ = o.mass_bias(q - e, u)
            Md += (Mp - Mm) / (2 * h) * u[k]
            grad[k] = (u @ Mp @ u - u @ Mm @ u) / (2 * h)
        np.testing.assert_allclose(b, Md @ u - 0.5 * grad, atol=1e-6 * max(1, np.abs(b).max()))


def test_gravity_bias_is_potential_gradient(orc):
    pk = orc.pack
    nd = pk.ndof
    q = random_q(pk, np.random.default_rng(3))
    _, b = orc.mass_bias(q, np.zeros(nd))
    g = np.array(pk.gravity[:])

    def V(qq):
        return -pk.total_mass * g @ orc.fk(qq)[2]
    h = 1e-6
    grad = np.array([(V(q + h * np.eye(nd)[k]) - V(q - h * np.eye(nd)[k])) / (2 * h) for k in range(nd)])
    np.testing.assert_allclose(b, grad, atol=1e-6)


def test_moment_arms_are_path_length_gradients(orc):
    pk = orc.pack
    nd = pk.ndof
    q, u = ref_dofs(pk, 50)
    h = 1e-7
    for m in range(pk.nmuscle):
        L, Ld, d = orc.muscle_path(q, u, m)
        fd = np.array([(orc.muscle_path(q + h * np.eye(nd)[k], u, m)[0] -
                        orc.muscle_path(q - h * np.eye(nd)[k], u, m)[0]) / (2 * h) for k in range(nd)])
        np.testing.assert_allclose(d, fd, atol=1e-8)
        assert abs(Ld - d @ u) < 1e-12


def test_millard_curve_landmarks(orc):
    # ActiveForceLength peak, ForceVelocity isometric/vmax, passive and tendon toe
    # (4.1 default curve parameters; the palsy model sets fal minimum_value=0, 02905_PRE
    # model_predictive.osim:1855, so its plateau landmark differs)
    palsy = orc.pack.env_id.decode() == 'MusclePalsyImitation3D-v0'
    if palsy:
        pytest.skip('explicit curve parameters (checked by the curve tests)')
    assert abs(orc.curve(0, 0, 1.0)[0] - 1.0) < 1e-12
    assert abs(orc.curve(0, 0, 0.3)[0] - 0.1) < 1e-12          # minimum_value plateau
    y, d = orc.curve(0, 1, 0.0)
    assert abs(y - 1.0) < 1e-12 and abs(d - 5.0) < 1e-9          # isometric slope
    assert abs(orc.curve(0, 1, -1.0)[0]) < 1e-12 and abs(orc.curve(0, 1, 1.0)[0] - 1.4) < 1e-12
    assert orc.curve(0, 2, 1.0)[0] == 0.0 and abs(orc.curve(0, 2, 1.7)[0] - 1.0) < 1e-12
    y, d = orc.curve(0, 3, 1.049)
    assert abs(y - 1.0) < 1e-12 and abs(d - 1.375 / 0.049) < 1e-9


def test_static_equilibrium_balances_fiber_and_tendon(orc):
    pk = orc.pack
    for m in range(pk.nmuscle):
        mu = pk.muscle[m]
        for L in (mu.lts + 0.9 * mu.lopt, mu.lts + 1.1 * mu.lopt):
            lce = orc.muscle_equilibrium(m, 0.05, L)
            w = mu.width
            cphi = np.sqrt(lce ** 2 - w ** 2) / lce
            fal = orc.curve(m, 0, lce / mu.lopt)[0]
            fpe = orc.curve(m, 2, lce / mu.lopt)[0]
            fse = orc.curve(m, 3, (L - lce * cphi) / mu.lts)[0]
            assert abs((0.05 * fal + fpe) * cphi - fse) < 1e-10


def test_contact_pushes_up_and_opposes_slip(orc):
    pk = orc.pack
    q, _ = ref_dofs(pk, 0)
    dx, dy = pk.coord[pk.coord_tx].dof, pk.coord[pk.coord_ty].dof
    q[dy] -= 0.02                  # sink 2 cm into the ground
    u = np.zeros(pk.ndof)
    u[dx] = 0.5                    # pelvis sliding forward
    tau, w = orc.contact(q, u)
    Fy = w[1] + w[7]
    Fx = w[0] + w[6]
    assert Fy > 0 and Fx < 0
    # translational dofs see the net force
    assert abs(tau[dy] - Fy) < 1e-9 * Fy and abs(tau[dx] - Fx) < 1e-9 * Fy
    if pk.coord_tz >= 0:
        assert abs(tau[pk.coord[pk.coord_tz].dof] - (w[2] + w[8])) < 1e-9 * Fy


@pytest.mark.parametrize('env_id', ['TorqueWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0'])
def test_energy_conserved_without_dissipation(oracle_lib, env_id):
    """Zero controls (muscles removed), gravity only (no contact: model
    lifted), small substeps: total energy drifts only at O(dt)."""
    pk = load_pack(env_id, {'nsub': 200})
    pk.nlimit = 0
    pk.nmuscle = 0
    o = oracle_lib.Oracle(pk)
    envs = o.new_envs(1)
    o.reset(envs, 0, 10)
    s = o.get_state(envs, 0)
    nd = pk.ndof
    s[5 + pk.coord[pk.coord_ty].dof] += 1.0   # lift the pelvis 1 m: no contact during the test
    s[5 + nd:5 + 2 * nd] = np.random.default_rng(4).normal(0, 0.5, nd)
    o.set_state(envs, 0, s)

    def energy():
        st = o.get_state(envs, 0)
        q, u = st[5:5 + nd], st[5 + nd:5 + 2 * nd]
        M, _ = o.mass_bias(q, u)
        return 0.5 * u @ M @ u - pk.total_mass * np.dot(pk.gravity[:], o.fk(q)[2])
    e0 = energy()
    for _ in range(5):
        o.step(envs, 0, np.full(pk.nact, np.nan))   # NaN -> zero torques
    assert abs(energy() - e0) < 2e-3 * (abs(e0) + 1)


@pytest.mark.parametrize('env_id', ['MuscleWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0'])
def test_contact_record_foot_side_entries(oracle_lib, env_id):
    """The ForceReporter's Hunt-Crossley entries per sphere body (the force's
    wrench on the sphere's OpenSim body about its origin, force report tail):
    per contact force they sum, with each body origin's moment arm, to the
    force's wrench on the feet about the ground origin (the negated platform
    entry) — the third law the record's two sides must satisfy."""
    from bioimitation.simulation_io import split_osim_report
    pk = load_pack(env_id)
    orc = oracle_lib.Oracle(pk)
    bufs = orc.new_envs(1)
    orc.reset(bufs, 0, 0)
    st = orc.get_state(bufs, 0)
    dy = pk.coord[pk.coord_ty].dof
    st[5 + dy] -= 0.02                                   # 2 cm into the ground
    orc.set_state(bufs, 0, st)
    fr = orc.force_report(bufs, 0)
    rep = split_osim_report(pk, orc.osim_report(bufs, 0))
    na, nf, nl = pk.nact, pk.ncforce, pk.nlimit
    so = na + 6 * nf + nl
    assert len(fr) == so + 6 * pk.nsphere
    loaded = 0
    for f in range(nf):
        F = np.zeros(3)
        M = np.zeros(3)
        for s in range(pk.nsphere):
            if pk.sphere[s].force != f:
                continue
            Fs, Ts = fr[so + 6 * s:so + 6 * s + 3], fr[so + 6 * s + 3:so + 6 * s + 6]
            O = rep['bodies'][pk.sphere[s].obody][:3]
            F += Fs
            M += Ts + np.cross(O, Fs)
        np.testing.assert_allclose(F, fr[na + 6 * f:na + 6 * f + 3], rtol=1e-12, atol=1e-9)
        loaded += np.linalg.norm(F) > 10.0
        np.testing.assert_allclose(M, fr[na + 6 * f + 3:na + 6 * f + 6], rtol=1e-10, atol=1e-8)
    assert loaded >= 1                                   # a foot on the ground
