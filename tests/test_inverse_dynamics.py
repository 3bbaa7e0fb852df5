"""Inverse-dynamics primitives (inverse_dynamics.cpp:45-215): the oracle's
restatement checked by identities, and the HIP kernel (bioim_id_eval) against
the oracle."""
import numpy as np
import pytest

from conftest import gpu_available

IDS = ['TorqueWalkingImitation2D-v0', 'MuscleWalkingImitation2D-v0', 'MuscleRunningImitation3D-v0',
       'MuscleLockedKneeImitation3D-v0']
GRAVITY, CORIOLIS, MULT_M, MULT_MINV, RESIDUAL, TOTAL = range(6)


def _states(pk, rng, n):
    """reference rows (feet near the ground: contact active for some) plus noise"""
    rows = rng.integers(0, pk.nrows, size=n)
    q = np.zeros((n, pk.ndof))
    u = np.zeros((n, pk.ndof))
    for i, r in enumerate(rows):
        for c in range(pk.ncoord):
            d = pk.coord[c].dof
            if d >= 0:
                q[i, d] = pk.ref_q[r][c] + rng.normal(0, 0.02)
                u[i, d] = pk.ref_u[r][c] + rng.normal(0, 0.2)
    return q, u


@pytest.mark.parametrize('env_id', IDS)
def test_oracle_id_identities(env_id, oracle_lib):
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    orc = oracle_lib.Oracle(pk)
    rng = np.random.default_rng(0)
    q, u = _states(pk, rng, 12)
    for i in range(len(q)):
        v = rng.normal(size=pk.ndof)
        Mv = orc.id_eval(MULT_M, q[i], v=v)
        np.testing.assert_allclose(orc.id_eval(MULT_MINV, q[i], v=Mv), v, rtol=1e-9, atol=1e-9)
        M, bias = orc.mass_bias(q[i], u[i])
        np.testing.assert_allclose(Mv, M @ v, rtol=1e-12, atol=1e-12)
        g = orc.id_eval(GRAVITY, q[i])
        c = orc.id_eval(CORIOLIS, q[i], u[i])
        np.testing.assert_allclose(c - g, bias, rtol=1e-9, atol=1e-9)     # bias = c - g
        np.testing.assert_allclose(orc.id_eval(CORIOLIS, q[i], 2 * u[i]), 4 * c, rtol=1e-8, atol=1e-8)  # quadratic in u
        tot = orc.id_eval(TOTAL, q[i], u[i])
        np.testing.assert_allclose(orc.id_eval(RESIDUAL, q[i], u[i], v), Mv + tot, rtol=1e-10, atol=1e-9)
        # ID inverts FD: forward dynamics with muscles off and zero controls, then the residual vanishes
        if pk.nmuscle == 0:
            qdd, _, rc = orc.forward_dynamics(q[i], u[i], np.zeros(1), np.zeros(1), np.zeros(pk.nact))
            assert rc == 0
            res = orc.id_eval(RESIDUAL, q[i], u[i], qdd)
            assert np.abs(res).max() < 1e-8 * max(1.0, np.abs(tot).max()), res


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
@pytest.mark.parametrize('env_id', IDS)
def test_id_kernel_matches_oracle(env_id):
    import oracle
    import torch
    from bioimitation.inverse_dynamics import InverseDynamics
    from bioimitation.registry import load_pack
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    rng = np.random.default_rng(1)
    n = 200                      # 13 workgroups, a partial last one
    q, u = _states(pk, rng, n)
    v = rng.normal(size=(n, pk.ndof))
    for precision, tol in ((64, 1e-9), (32, 2e-3)):
        idd = InverseDynamics(env_id, precision=precision)
        for op in range(6):
            out = idd.eval(op, q, u, v).double().cpu().numpy()
            ref = np.stack([orc.id_eval(op, q[i], u[i], v[i]) for i in range(n)])
            scale = np.maximum(1.0, np.abs(ref).max(1, keepdims=True))
            err = (np.abs(out - ref) / scale).max()
            print(env_id, precision, 'op', op, 'max rel err', err)
            assert err < tol, (op, precision, err)
        idd.close()
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason='needs GPU')
def test_id_reference_api_single_state():
    """Method names and list-in/list-out shape of the reference helper
    (coordinate order, locked coordinates 0)."""
    import oracle
    from bioimitation.inverse_dynamics import InverseDynamics
    from bioimitation.registry import load_pack
    env_id = 'MuscleLockedKneeImitation3D-v0'
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    rng = np.random.default_rng(2)
    q, u = _states(pk, rng, 1)
    dof = np.array([pk.coord[c].dof for c in range(pk.ncoord)])
    full = lambda x: np.array([x[d] if d >= 0 else 0.0 for d in dof])  # noqa: E731
    qf, uf = full(q[0]), full(u[0])
    idd = InverseDynamics(env_id)
    idd.setStateAndRealizeDynamics(0.0, list(qf), list(uf))
    g = idd.calculateGravity(0.0, list(qf))
    assert isinstance(g, list) and len(g) == pk.ncoord
    np.testing.assert_allclose(g, full(orc.id_eval(GRAVITY, q[0])), rtol=1e-9, atol=1e-9)
    assert all(g[c] == 0.0 for c in range(pk.ncoord) if dof[c] < 0)
    a = rng.normal(size=pk.ncoord)
    Ma = idd.multiplyByM(0.0, list(qf), list(a))
    np.testing.assert_allclose(idd.multiplyByMInv(0.0, list(qf), Ma), np.where(dof >= 0, a, 0.0), rtol=1e-8, atol=1e-8)
    res = idd.calculateResidualForces(0.0, list(qf), list(uf), list(a))
    tot = idd.calculateTotalForces(0.0, list(qf), list(uf))
    np.testing.assert_allclose(np.array(res), np.array(Ma) + np.array(tot), rtol=1e-9, atol=1e-8)
    c = idd.calculateCoriolis(0.0, list(qf), list(uf))
    np.testing.assert_allclose(c, full(orc.id_eval(CORIOLIS, q[0], u[0])), rtol=1e-9, atol=1e-9)
    idd.close()
