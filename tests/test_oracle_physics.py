"""Physics invariants of the fp64 oracle (parity with OpenSim itself is
unpinned — OpenSim is not available — so the restatement is checked against
mechanics identities instead)."""
import numpy as np
import pytest

from bioimitation.registry import load_pack

ENV = 'MuscleWalkingImitation2D-v0'


@pytest.fixture(scope='module')
def orc(oracle_lib):
    return oracle_lib.Oracle(load_pack(ENV))


def test_forward_kinematics_matches_raw_joint_chain(orc):
    """Composite-body FK (compiled pack) == FK straight from the parsed joints."""
    import os
    from bioimitation import modelpack, transforms
    from bioimitation.osim import load_osim
    path = '/root/reference/bioimitation/imitation_envs/data/2D/scale/model_scaled.osim'
    if not os.path.exists(path):
        pytest.skip('reference data not present')
    m = transforms.construct_predictive_model(load_osim(path))
    rng = np.random.default_rng(0)
    for _ in range(5):
        q = rng.normal(0, 0.5, 9)
        R, p, com = orc.fk(q)
        poses, com2 = modelpack.raw_forward_kinematics(m, dict(zip(m.coord_order, q)))
        for i, b in enumerate(m.body_order):
            np.testing.assert_allclose(p[i], poses[b][1], atol=1e-14)
            np.testing.assert_allclose(R[i], poses[b][0], atol=1e-14)
        np.testing.assert_allclose(com, com2, atol=1e-14)


def test_mass_matrix_spd_and_translational_mass(orc):
    rng = np.random.default_rng(1)
    for _ in range(5):
        M, _ = orc.mass_bias(rng.normal(0, 0.5, 9), rng.normal(0, 1, 9))
        assert np.abs(M - M.T).max() == 0.0
        assert np.linalg.eigvalsh(M).min() > 0
        assert abs(M[1, 1] - 75.1646) < 1e-9 and abs(M[2, 2] - 75.1646) < 1e-9


def test_bias_equals_lagrangian_coriolis(oracle_lib):
    """bias(q,u) with g=0 equals Mdot u - 1/2 d(u'Mu)/dq (finite differences)."""
    pk = load_pack(ENV)
    pk.gravity[1] = 0.0
    o = oracle_lib.Oracle(pk)
    rng = np.random.default_rng(2)
    h = 1e-6
    for _ in range(3):
        q, u = rng.normal(0, 0.5, 9), rng.normal(0, 2, 9)
        M, b = o.mass_bias(q, u)
        Md = np.zeros_like(M)
        grad = np.zeros(9)
        for k in range(9):
            e = np.zeros(9); e[k] = h
            Mp, _ = o.mass_bias(q + e, u)
            Mm, _ = o.mass_bias(q - e, u)
            Md += (Mp - Mm) / (2 * h) * u[k]
            grad[k] = (u @ Mp @ u - u @ Mm @ u) / (2 * h)
        np.testing.assert_allclose(b, Md @ u - 0.5 * grad, atol=1e-6 * max(1, np.abs(b).max()))


def test_gravity_bias_is_potential_gradient(orc):
    pk = orc.pack
    q = np.random.default_rng(3).normal(0, 0.5, 9)
    _, b = orc.mass_bias(q, np.zeros(9))
    g = np.array(pk.gravity[:])

    def V(qq):
        return -pk.total_mass * g @ orc.fk(qq)[2]
    h = 1e-6
    grad = np.array([(V(q + h * np.eye(9)[k]) - V(q - h * np.eye(9)[k])) / (2 * h) for k in range(9)])
    np.testing.assert_allclose(b, grad, atol=1e-6)


def test_moment_arms_are_path_length_gradients(orc):
    pk = orc.pack
    q, u = np.array(pk.ref_q[50][:9]), np.array(pk.ref_u[50][:9])
    h = 1e-7
    for m in range(pk.nmuscle):
        L, Ld, d = orc.muscle_path(q, u, m)
        fd = np.array([(orc.muscle_path(q + h * np.eye(9)[k], u, m)[0] -
                        orc.muscle_path(q - h * np.eye(9)[k], u, m)[0]) / (2 * h) for k in range(9)])
        np.testing.assert_allclose(d, fd, atol=1e-8)
        assert abs(Ld - d @ u) < 1e-12


def test_millard_curve_landmarks(orc):
    # ActiveForceLength peak, ForceVelocity isometric/vmax, passive and tendon toe
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
    q = np.array(pk.ref_q[0][:9])
    q[2] -= 0.02                   # sink 2 cm into the ground
    u = np.zeros(9)
    u[1] = 0.5                     # pelvis sliding forward
    tau, w = orc.contact(q, u)
    Fy = w[1] + w[7]
    Fx = w[0] + w[6]
    assert Fy > 0 and Fx < 0
    assert abs(tau[2] - Fy) < 1e-9 and abs(tau[1] - Fx) < 1e-9   # translational dofs see the net force


def test_energy_conserved_without_dissipation(oracle_lib):
    """Torque model, zero controls, gravity only (no contact: model lifted),
    small substeps: total energy drifts only at O(dt)."""
    pk = load_pack('TorqueWalkingImitation2D-v0', {'nsub': 200})
    pk.nlimit = 0
    o = oracle_lib.Oracle(pk)
    envs = o.new_envs(1)
    o.reset(envs, 0, 10)
    s = o.get_state(envs, 0)
    nd = pk.ndof
    s[5 + 2] += 1.0                # lift the pelvis 1 m: no contact during the test
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
