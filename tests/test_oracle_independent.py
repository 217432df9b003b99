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


def test_heat_loss_energy_balance_inert(oracle, mech):
    """QLOS on a non-reacting N2 charge at constant pressure: h(T(t)) = h(T0) - Q t / m exactly."""
    from scipy.optimize import brentq

    R = 1.3806504e-16 * 6.02214179e23
    k = mech.species.index("N2")
    Y = np.zeros(mech.KK)
    Y[k] = 1.0
    T0, V0, Q, tend = 1200.0, 10.0, 2.0, 0.05  # Q [cal/s]
    r, _ = oracle.reactor(T0, P_ATM, V0, Y, energy=1, t_end=tend, atol=1e-12, rtol=1e-10, qloss=Q)
    assert r.status == 0

    def h_mass(T):
        return oracle.thermo(T)[1][k] * R * T / mech.wt[k]

    mass = P_ATM * mech.wt[k] / (R * T0) * V0
    T_exact = brentq(lambda T: h_mass(T) - (h_mass(T0) - Q * 4.184e7 * tend / mass), 300.0, T0)
    assert abs(r.T / T_exact - 1) < 1e-7
    # wall heat transfer towards a hotter ambient heats the charge
    r2, _ = oracle.reactor(T0, P_ATM, V0, Y, energy=1, t_end=tend, atol=1e-12, rtol=1e-10, htc=1e-3, areaq=20.0,
                           tamb=1500.0)
    assert 1200.0 < r2.T < 1500.0
    # QPRO ramp 0 -> 2Q over t_end removes the same heat as a constant Q
    r3, _ = oracle.reactor(T0, P_ATM, V0, Y, energy=1, t_end=tend, atol=1e-12, rtol=1e-10,
                           profile2=([0.0, tend], [0.0, 2 * Q]), prof2_kind=1)
    assert abs(r3.T / T_exact - 1) < 1e-7
    # QPRO together with AEXT (batchreactor.py:2005-2067): heat loss QPRO(t) + HTC AEXT(t) (T - TAMB).
    # A constant AEXT profile equals AREAQ; wall transfer from TAMB = T0 gives back part of the loss
    kw = dict(energy=1, t_end=tend, atol=1e-12, rtol=1e-10, htc=1e-3, profile2=([0.0, tend], [0.0, 2 * Q]),
              prof2_kind=1)
    r4, _ = oracle.reactor(T0, P_ATM, V0, Y, tamb=T0, profile3=([0.0, tend], [20.0, 20.0]), **kw)
    r5, _ = oracle.reactor(T0, P_ATM, V0, Y, tamb=T0, areaq=20.0, **kw)
    assert r4.status == 0 and abs(r4.T / r5.T - 1) < 1e-12
    assert T_exact + 1.0 < r4.T < T0
    r6, _ = oracle.reactor(T0, P_ATM, V0, Y, tamb=T0, profile3=([0.0, tend], [0.0, 40.0]), **kw)
    # the ramp's area (mean 20) weighs the late times, when the charge is furthest below TAMB
    assert r4.T + 1.0 < r6.T < T0


def test_temperature_profile_given_T(oracle, mech):
    """TPRO on a fixed-temperature reactor: T follows the piecewise-linear profile exactly."""
    Y = ch4_air_Y(mech, 1.0)[0]
    prof = ([0.0, 1e-3, 2e-3], [1000.0, 1600.0, 1600.0])
    ts = np.linspace(0.0, 2e-3, 21)
    r, _, (_, ys, _, _) = oracle.reactor(1234.0, P_ATM, 1.0, Y, t_save=ts, energy=2, t_end=2e-3, atol=1e-12,
                                         rtol=1e-8, profile=prof, prof_kind=1)
    assert r.status == 0
    assert np.max(np.abs(ys[:, 0] - np.interp(ts, prof[0], prof[1]))) < 1e-6
    assert abs(r.T - 1600.0) < 1e-6


def test_gfac_scales_all_rates(oracle, mech):
    Y = ch4_air_Y(mech, 1.0)[0]
    y = np.concatenate([[1500.0], Y])
    f1, _ = oracle.rhs_jac(y)
    f2, _ = oracle.rhs_jac(y, gfac=2.0)
    assert np.allclose(f2, 2.0 * f1, rtol=1e-13, atol=0)


def test_c_oracle_matches_numpy_on_161_species_mechanism(big_mech):
    """The synthetic configs[4]-sized mechanism (GRI-3.0 + 108 tracer species, conftest.
    write_big_mechanism): the C oracle and the dense-matrix numpy restatement agree, so the oracle
    can check the > 63-species kernels."""
    from oracle.oracle import Oracle

    tables = big_mech.to_tables()
    orc = Oracle(big_mech)
    nk = NumpyKinetics(tables)
    rng = np.random.default_rng(5)
    for _ in range(10):
        T = rng.uniform(300, 3000)
        P = P_ATM * 10 ** rng.uniform(-1, 2)
        Y = rng.dirichlet(0.5 * np.ones(big_mech.KK))
        qf, qr, w = orc.rates(T, P, Y)
        qf2, qr2, w2 = nk.rates(T, P, Y)
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))
    assert big_mech.KK == 161 and np.any(tables["rsp"] > 63) and np.any(tables["eff_sp"] > 63)


def test_oracle_integrates_161_species_mechanism(big_mech):
    """The oracle's BDF on the configs[4]-sized stand-in (n = 162): CH4/air with 20 % of the N2
    replaced by tracer AX1 ignites, conserves mass, and spreads the tracer over AX1..AX108 by
    the exchange reactions -- the reference solution a > 63-species device integrator will be
    checked against."""
    from oracle.oracle import Oracle

    m = big_mech
    orc = Oracle(m)
    X = np.zeros(m.KK)
    X[m.species.index("CH4")] = 1.0
    X[m.species.index("O2")] = 2.0
    X[m.species.index("N2")] = 7.52 * 0.8
    X[m.species.index("AX1")] = 7.52 * 0.2
    Y = X * m.wt
    Y /= Y.sum()
    r, Ye = orc.reactor(1400.0, 10 * P_ATM, 1.0, Y, problem=1, energy=1, t_end=0.05, atol=1e-10, rtol=1e-8,
                        ign_mode="TIFP")
    assert r.status == 0 and 1e-4 < r.tau < 1e-3 and r.T > 2500.0
    assert abs(Ye.sum() - 1.0) < 1e-8
    tr = Ye[m.species.index("AX1"):]
    assert tr.size == 108 and np.all(tr > 0) and abs(tr.sum() / Y[m.species.index("AX1")] - 1) < 1e-6
