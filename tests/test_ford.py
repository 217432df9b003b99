"""FORD / RORD reaction orders and non-integral stoichiometric coefficients on the oracle and the
device path.

Mechanism: data/gri30_ford_chem.inp (data/make_ford_mechanism.py), GRI-3.0 with FORD on three
elementary reactions, RORD on two reversible ones and two global reactions with fractional
coefficients (CH4+1.5O2=>CO+2H2O with FORD /CH4 0.7/ /O2 0.8/, CO+0.5O2<=>CO2 with K_c over
Delta nu = -1/2).  Reference semantics: Chemistry.preprocess accepts any Chemkin mechanism
(chemistry.py:595-753); the closed library evaluates q_f = k_f prod C_k^ford_k.  No golden of the
reference uses these keywords, so parity with Chemkin is unpinned: the C oracle is checked against
the numpy restatement and the definition, its Jacobian against finite differences, and the GPU
kernels against the oracle with the GRI-3.0 bars.
"""
import math
import os

import numpy as np
import pytest

from conftest import P_ATM, ROOT, THERM, ch4_air_Y

FORD_CHEM = os.path.join(ROOT, "data", "gri30_ford_chem.inp")


@pytest.fixture(scope="module")
def fmech():
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism.from_files(FORD_CHEM, THERM)


@pytest.fixture(scope="module")
def forc(fmech):
    from oracle.oracle import Oracle

    return Oracle(fmech)


def _states(KK, n, seed):
    rng = np.random.default_rng(seed)
    T = rng.uniform(300.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, n)
    Y = rng.dirichlet(0.5 * np.ones(KK), n).T.copy()
    return T, P, Y


def _idx(m, eq):
    return next(j for j, rx in enumerate(m.reactions) if rx.equation == eq)


def test_ford_tables(fmech):
    t = fmech.to_tables()
    assert fmech.II == 327
    i = _idx(fmech, "CH4+1.5O2=>CO+2H2O")
    assert list(t["rnu"][i, :2]) == [1.0, 1.5] and list(t["ford"][i, :2]) == [0.7, 0.8]
    assert list(t["pnu"][i, :2]) == [1.0, 2.0] and list(t["rord"][i, :2]) == [1.0, 2.0]
    i = _idx(fmech, "OH+CH2O<=>HCO+H2O")
    assert list(t["ford"][i, :2]) == [0.8, 1.0] and list(t["rord"][i, :2]) == [1.0, 1.1]
    # without FORD / RORD the orders are the coefficients
    j = _idx(fmech, "O+H2<=>H+OH")
    assert np.array_equal(t["ford"][j], t["rnu"][j]) and np.array_equal(t["rord"][j], t["pnu"][j])


def test_ford_parser_rejects_non_participants():
    from pychemkin_amd.mechanism import MechanismError

    base = open(os.path.join(ROOT, "data", "grimech30_chem.inp")).read()
    bad = base.replace("O+H2<=>H+OH                              3.870E+04    2.700    6260.00",
                       "O+H2<=>H+OH                              3.870E+04    2.700    6260.00\n FORD / CH4 1.0 /", 1)
    assert bad != base
    with pytest.raises(MechanismError, match="FORD species CH4 is not a reactant"):
        _parse(bad)


def _parse(text):
    import tempfile

    from pychemkin_amd.mechanism import Mechanism

    with tempfile.NamedTemporaryFile("w", suffix=".inp", delete=False) as f:
        f.write(text)
    try:
        return Mechanism.from_files(f.name, THERM)
    finally:
        os.unlink(f.name)


def test_ford_rate_definition(fmech, forc):
    """q_f of the global CH4 reaction = k C_CH4^0.7 C_O2^0.8; q_r of CO+0.5O2<=>CO2 = k_f / K_c C_CO2
    with K_c = exp(-dG/RT) (P_atm / RT)^(-1/2)."""
    T, P = 1500.0, 2.0 * P_ATM
    Y = np.random.default_rng(4).dirichlet(np.ones(fmech.KK))
    qf, qr, _ = forc.rates(T, P, Y)
    RU = 1.3806504e-16 * 6.02214179e23  # the oracle's R (reference constants.py)
    C = P / (RU * T) * Y / fmech.wt / np.sum(Y / fmech.wt)
    sp = fmech.species.index
    i = _idx(fmech, "CH4+1.5O2=>CO+2H2O")
    rx = fmech.reactions[i]
    k = rx.A * T ** rx.b * math.exp(-rx.E * rx.E_scale / T)
    assert abs(qf[i] / (k * C[sp("CH4")] ** 0.7 * C[sp("O2")] ** 0.8) - 1) < 1e-6
    assert qr[i] == 0.0
    i = _idx(fmech, "CO+0.5O2<=>CO2")
    rx = fmech.reactions[i]
    k = rx.A * T ** rx.b * math.exp(-rx.E * rx.E_scale / T)
    assert abs(qf[i] / (k * C[sp("CO")] * C[sp("O2")] ** 0.25) - 1) < 1e-6
    cp, h, s = forc.thermo(T)
    g = h - s
    dG = g[sp("CO2")] - g[sp("CO")] - 0.5 * g[sp("O2")]
    Kc = math.exp(-dG) * (P_ATM / (RU * T)) ** (-0.5)
    assert abs(qr[i] / (k / Kc * C[sp("CO2")]) - 1) < 1e-6


def test_ford_oracle_matches_numpy(fmech, forc):
    from oracle.numpy_ref import NumpyKinetics

    nk = NumpyKinetics(fmech.to_tables())
    T, P, Y = _states(fmech.KK, 30, seed=7)
    Y[3, :] = 0.0  # exact zeros (CH2): a non-integral order of a zero concentration
    for j in range(T.size):
        qf, qr, w = forc.rates(T[j], P[j], Y[:, j])
        qf2, qr2, w2 = nk.rates(T[j], P[j], Y[:, j])
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))


FD_REACTIONS = {  # reaction -> {species: order of its concentration in q_f or q_r}
    "O+CH4<=>OH+CH3": {"CH4": 1.2}, "OH+CH2O<=>HCO+H2O": {"OH": 0.8, "H2O": 1.1},
    "2OH<=>O+H2O": {"OH": 1.5}, "HO2+CH3<=>OH+CH3O": {"OH": 0.9}, "CH4+1.5O2=>CO+2H2O": {"CH4": 0.7, "O2": 0.8},
    "CO+0.5O2<=>CO2": {"O2": 0.25, "CO2": 1.0},
}


@pytest.mark.parametrize("eq", list(FD_REACTIONS))
def test_ford_oracle_jacobian_matches_finite_differences(eq):
    """The analytic Jacobian terms of FORD / RORD / fractional-coefficient reactions (the device
    kernels use the same terms) against central differences of the RHS, one reaction at a time (the
    GRI-3.0 species with only that reaction of gri30_ford, none of them third-body), on a CONV state:
    there C_k = rho Y_k / W_k at fixed rho, so the approximate Chemkin Jacobian is exact in the species
    rows (the states here are far above the 1e-14 mol/cm3 chord floor, so the tangent applies)."""
    from oracle.oracle import Oracle

    import re

    text = open(FORD_CHEM).read()
    r0 = re.search(r"^REACTIONS", text, re.M | re.I).start()
    lines = text[r0:].splitlines()
    body = [lines[0]]
    for j, ln in enumerate(lines[1:], 1):
        tok = ln.split()
        if tok and tok[0] == eq:
            body.append(ln)
            if j + 1 < len(lines) and ("FORD" in lines[j + 1] or "RORD" in lines[j + 1]):
                body.append(lines[j + 1])
    body.append("END")
    m = _parse(text[:r0] + "\n".join(body) + "\n")
    assert m.II == 1
    orc = Oracle(m)
    Y0 = np.random.default_rng(11).dirichlet(np.ones(m.KK)) * 0.2 + ch4_air_Y(m, 1.0)[0] * 0.8
    Y0 /= Y0.sum()
    y = np.concatenate([[1700.0], Y0])
    rho0 = P_ATM * (1.0 / np.sum(Y0 / m.wt)) / (1.3806504e-16 * 6.02214179e23 * 1700.0)
    kw = dict(problem=2, energy=1, rho0=rho0, V0=1.0, P0=P_ATM)
    f, J = orc.rhs_jac(y, **kw)
    for sp, order in FD_REACTIONS[eq].items():
        col = 1 + m.species.index(sp)
        h = 1e-4 * y[col]  # central differences: O(h^2) truncation, roundoff grows below ~1e-5
        yp, ym = y.copy(), y.copy()
        yp[col] += h
        ym[col] -= h
        fd = (orc.rhs_jac(yp, **kw)[0] - orc.rhs_jac(ym, **kw)[0]) / (2 * h)
        sc = np.max(np.abs(fd[1:]))
        assert sc > 0
        assert np.max(np.abs(J[1:, col] - fd[1:])) < 1e-5 * sc, sp


def test_fractional_order_rule_near_zero(fmech, forc):
    """The fractional-order rule at C -> 0 (this implementation's choice; no reference golden): for
    0 < o < 1 the rate follows the chord CFLOOR^(o-1) C below CFLOOR = 1e-14 mol/cm3, so it is
    continuous, Lipschitz and sign-preserving through C = 0; the oracle and numpy agree on it."""
    from oracle.numpy_ref import CFLOOR, NumpyKinetics, _cpow

    C = np.array([-1e-12, -1e-14, 0.0, 1e-16, 1e-14, 1e-10])
    for o in (0.25, 0.7, 0.8):
        v = _cpow(C, o)
        assert np.all(np.sign(v) == np.sign(C))
        assert abs(v[4] - CFLOOR ** o) < 1e-12 * CFLOOR ** o
        assert np.allclose(v[:4], CFLOOR ** (o - 1.0) * C[:4], rtol=1e-14, atol=0)
    # orders >= 1 outside {1, 2, 3}: 0 at C <= 0, the power above (integral 4 included)
    assert np.array_equal(_cpow(np.array([-1e-3, 0.0]), np.array([1.5, 4.0])), np.zeros(2))
    assert _cpow(np.array([2.0]), np.array([4.0]))[0] == 16.0
    nk = NumpyKinetics(fmech.to_tables())
    T, P, Y = _states(fmech.KK, 4, seed=17)
    sp = fmech.species.index
    Y[sp("CH4"), 0], Y[sp("O2"), 1], Y[sp("OH"), 2], Y[sp("CH4"), 3] = -1e-12, -1e-9, 1e-18, 1e-30
    for j in range(T.size):
        qf, qr, w = forc.rates(T[j], P[j], Y[:, j])
        qf2, qr2, w2 = nk.rates(T[j], P[j], Y[:, j])
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)


def test_ford_reactor_robust_to_tolerance_perturbation(fmech, forc):
    """Round 2's stall: under rounding-level changes the integrator locked its step at a species
    running out with an order < 1 (period-2 corrector cycle at C ~ 0) and hit max steps (5 of 35 runs
    here).  With the Lipschitz chord rule every case at every tolerance finishes in under 2,000 steps."""
    cases = [(1200, 1, 1.0, 1), (1400, 10, 1.0, 2), (1100, 0.5, 0.7, 1), (1600, 50, 1.5, 1), (1300, 30, 0.5, 2)]
    for rt in (1e-8, 1.01e-8, 0.99e-8, 1.03e-8, 0.97e-8, 1e-7, 1e-9):
        for T0, p, phi, prob in cases:
            r, _ = forc.reactor(float(T0), p * P_ATM, 1.0, ch4_air_Y(fmech, phi)[0], problem=prob, energy=1,
                                t_end=1.0, atol=1e-10, rtol=rt, ign_mode="TIFP")
            assert r.status == 0 and r.nst < 2500 and r.ncf < 10, (T0, p, phi, prob, rt, r.nst, r.ncf)


def test_ford_changes_ignition(fmech, forc, oracle, mech):
    Y0 = ch4_air_Y(fmech, 1.0)[0]
    r1, _ = forc.reactor(1400.0, 10 * P_ATM, 1.0, Y0, problem=1, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8,
                         ign_mode="TIFP")
    r0, _ = oracle.reactor(1400.0, 10 * P_ATM, 1.0, Y0, problem=1, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8,
                           ign_mode="TIFP")
    assert r1.status == 0 and r0.status == 0 and r1.tau > 0
    assert abs(r1.tau / r0.tau - 1) > 1e-4


def test_ford_specialised_rop_kernel_emits_orders(fmech):
    """Round 3: the hipRTC state-per-lane kernel covers FORD / RORD orders and non-integral
    coefficients (round 2 declined them): the fractional orders take the conc_pow rule of the oracle
    (jcpow_lt1: the chord below 1e-14), K_c the real coefficients (host-only call, no GPU; the GPU
    parity is tests/test_gpu_rop_jit.py)."""
    from pychemkin_amd import _native

    src = _native.rop_jit_source(fmech.to_tables())
    assert "jcpow_lt1(" in src and "lnPRT" in src


# ------------------------------------------------------------------ GPU


@pytest.fixture(scope="module")
def fdm(fmech):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(fmech.to_tables())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 17, 1000, 20000])  # 20,000: the automatic path falls back from the
def test_ford_gpu_rop(fmech, forc, fdm, n):          # specialised kernel (which declines FORD) to the generic one
    T, P, Y = _states(fmech.KK, n, seed=n)
    Y[3, :] = 0.0  # CH2 absent: a non-integral order of a zero concentration
    w, cp, h = (x.cpu().numpy() for x in fdm.rop_thermo(T, P, Y))
    wo, cpo, ho = forc.rop_batch(T, P, Y)
    scale = np.max(np.abs(wo), axis=0, keepdims=True)
    assert np.max(np.abs(w - wo) / scale) < 1e-11
    assert np.max(np.abs(cp / cpo - 1)) < 1e-12


@pytest.mark.gpu
def test_ford_gpu_reaction_rates(fmech, forc, fdm):
    T, P, Y = _states(fmech.KK, 19, seed=3)
    qf, qr = (x.cpu().numpy() for x in fdm.reaction_rates(T, P, Y))
    for j in range(T.size):
        qfo, qro, _ = forc.rates(T[j], P[j], Y[:, j])
        sc = max(np.max(np.abs(qfo)), np.max(np.abs(qro)))
        assert np.max(np.abs(qf[:, j] - qfo)) < 1e-11 * sc
        assert np.max(np.abs(qr[:, j] - qro)) < 1e-11 * sc


@pytest.mark.gpu
@pytest.mark.parametrize("path", [0, 2])
def test_ford_gpu_reactor(fmech, forc, fdm, path):
    """CONP and CONV ignition on the FORD mechanism (automatic kernel choice -- the FP64 Newton
    inverse for mechanisms with fractional orders -- and forced FP64): the north_star bars (tau
    0.5 %, T 1e-4), held at 1e-4."""
    from pychemkin_amd import _native

    cases = [(1200, 1, 1.0, 1), (1400, 10, 1.0, 2), (1100, 0.5, 0.7, 1), (1600, 50, 1.5, 1), (1300, 30, 0.5, 2)]
    cfg = dict(energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    T0 = np.array([c[0] for c in cases], float)
    P0 = np.array([c[1] for c in cases], float) * P_ATM
    Y0 = np.stack([ch4_air_Y(fmech, c[2])[0] for c in cases])
    prob = np.array([c[3] for c in cases], np.int32)
    _native.set_reactor_path(path)
    try:
        res = {k: v.cpu().numpy() for k, v in fdm.reactor_run(_native.make_cfg(**cfg), prob, T0, P0,
                                                                 np.ones(len(cases)), Y0).items()}
    finally:
        _native.set_reactor_path(0)
    for i in range(len(cases)):
        r, Ye = forc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **cfg)
        assert res["stats"][i, 6] == r.status == 0
        assert r.tau > 0 and abs(res["tau"][i] / r.tau - 1) < 1e-4
        assert abs(res["T"][i] / r.T - 1) < 1e-4
        for sp in ("CH4", "O2", "H2O", "CO2", "CO"):
            k = fmech.species.index(sp)
            assert abs(res["Y"][i, k] - Ye[k]) <= 1e-4 * max(abs(Ye[k]), 1e-3)


@pytest.mark.gpu
def test_drop_in_api_on_ford_mechanism(fmech, forc):
    """Chemistry.preprocess / Mixture.ROP (mixture.py:1693-1808) on the FORD mechanism through the
    extended GPU kernel variant."""
    import pychemkin_amd as ck

    chem = ck.Chemistry(label="gri30-ford")
    chem.chemfile = FORD_CHEM
    chem.thermfile = THERM
    chem.preprocess()
    assert chem.KK == 53 and chem.IIGas == 327
    m = ck.Mixture(chem)
    m.temperature = 1650.0
    m.pressure = 3.0 * P_ATM
    m.X = [("CH4", 0.05), ("O2", 0.15), ("N2", 0.7), ("OH", 0.01), ("H", 0.01), ("O", 0.01), ("CO", 0.05),
           ("HO2", 0.01), ("CH2O", 0.01)]
    qfo, qro, wo = forc.rates(1650.0, 3.0 * P_ATM, m.Y)
    assert np.max(np.abs(m.ROP() - wo)) < 1e-11 * np.max(np.abs(wo))
