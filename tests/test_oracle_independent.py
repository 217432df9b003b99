"""The C oracle against two independent references: numpy kinetics and scipy's Radau."""
import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y, h2_air_Y
from oracle.numpy_ref import NumpyKinetics


def test_c_oracle_rop_matches_numpy_restatement(oracle, tables, mech):
    nk = NumpyKinetics(tables)
    rng = np.random.default_rng(1)
    for _ in range(25):
        T = rng.uniform(300, 3000)
        P = P_ATM * 10 ** rng.uniform(-1, 2)
        Y = rng.dirichlet(0.5 * np.ones(mech.KK))
        qf, qr, w = oracle.rates(T, P, Y)
        qf2, qr2, w2 = nk.rates(T, P, Y)
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))


def test_c_oracle_thermo_matches_numpy(oracle, tables):
    nk = NumpyKinetics(tables)
    for T in (300.0, 999.0, 1000.0, 1001.0, 2500.0):
        a = oracle.thermo(T)
        b = nk.thermo(T)
        for x, y in zip(a, b):
            assert np.allclose(x, y, rtol=1e-14, atol=1e-14)


def test_jacobian_matches_finite_differences(oracle, mech):
    # state inside a CH4 induction (oracle run to 20 ms at 1200 K)
    Y0 = ch4_air_Y(mech, 1.0)[0]
    res, Yend = oracle.reactor(1200.0, P_ATM, 1.0, Y0, problem=1, energy=1, t_end=0.02, atol=1e-12, rtol=1e-9)
    y = np.concatenate([[res.T], Yend])
    rho0 = P_ATM / (1.3806504e-16 * 6.02214179e23 * 1200.0) / np.sum(Y0 / mech.wt)
    for problem in (1, 2):
        f, J = oracle.rhs_jac(y, problem=problem, rho0=rho0, P0=P_ATM)
        n = y.size
        Jfd = np.zeros((n, n))
        for j in range(n):
            d = max(abs(y[j]) * 1e-6, 1e-14)
            yp, ym = y.copy(), y.copy()
            yp[j] += d
            ym[j] -= d
            Jfd[:, j] = (oracle.rhs_jac(yp, problem=problem, rho0=rho0, P0=P_ATM)[0] -
                         oracle.rhs_jac(ym, problem=problem, rho0=rho0, P0=P_ATM)[0]) / (2 * d)
        scale = np.abs(Jfd).max(axis=1, keepdims=True) + 1e-300
        # approximate analytic Jacobian (third-body and falloff-F derivatives omitted by design)
        assert np.max(np.abs(J - Jfd) / scale) < 2e-2


def test_bdf_matches_scipy_radau_h2(oracle, mech):
    scipy_integrate = pytest.importorskip("scipy.integrate")
    Y0 = h2_air_Y(mech)
    y0 = np.concatenate([[1000.0], Y0])
    rho0 = P_ATM / (1.3806504e-16 * 6.02214179e23 * 1000.0) / np.sum(Y0 / mech.wt)
    ts = np.array([1e-4, 2e-4, 3e-4, 4e-4, 5e-4])
    f = lambda t, y: oracle.rhs_jac(y, rho0=rho0, P0=P_ATM)[0]
    jac = lambda t, y: oracle.rhs_jac(y, rho0=rho0, P0=P_ATM)[1]
    sol = scipy_integrate.solve_ivp(f, (0, 5e-4), y0, method="Radau", jac=jac, rtol=1e-11, atol=1e-20, t_eval=ts)
    res, Yend, (_, ys, _, _) = oracle.reactor(1000.0, P_ATM, 1.0, Y0, t_save=ts, problem=1, energy=1, t_end=5e-4,
                                              atol=1e-20, rtol=1e-11)
    assert np.max(np.abs(ys[:, 0] / sol.y[0] - 1)) < 1e-6
    assert abs(Yend[mech.species.index("H2O")] / sol.y[1 + mech.species.index("H2O"), -1] - 1) < 1e-6


def test_oracle_ignition_converges_in_tolerance(oracle, mech):
    Y0 = ch4_air_Y(mech, 1.0)[0]
    taus = []
    for rtol in (1e-8, 1e-10):
        res, _ = oracle.reactor(1400.0, 10 * P_ATM, 1.0, Y0, problem=1, energy=1, t_end=0.01, atol=1e-12, rtol=rtol,
                                ign_mode="TIFP")
        taus.append(res.tau)
    assert abs(taus[0] / taus[1] - 1) < 1e-4
