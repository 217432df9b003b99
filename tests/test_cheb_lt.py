"""Chebyshev (TCHEB / PCHEB / CHEB) and Landau-Teller (LT / RLT) reactions: parser, oracle, numpy
restatement and GPU kernels.

No mechanism with these forms ships with the reference or exists offline, so the stand-in is
data/gri30_cheb_chem.inp (data/make_cheb_mechanism.py): GRI-3.0 with four Troe falloff reactions
rewritten as 7 x 4 Chebyshev fits of their own rate, LT terms on two elementary reactions and REV +
RLT on a third.  Parity with Chemkin is unpinned (no golden); the rate definitions are checked
against direct formulas (numpy.polynomial.chebyshev for the series), the oracle against the numpy
restatement, the oracle's Jacobian against finite differences, and the GPU against the oracle."""
import math
import os

import numpy as np
import pytest

from conftest import P_ATM, ROOT, THERM, ch4_air_Y

CHEB_CHEM = os.path.join(ROOT, "data", "gri30_cheb_chem.inp")
RUC = 8.314510e7 / 4.184e7


@pytest.fixture(scope="module")
def cmech():
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism.from_files(CHEB_CHEM, THERM)


@pytest.fixture(scope="module")
def corc(cmech):
    from oracle.oracle import Oracle

    return Oracle(cmech)


def _idx(m, eq):
    return [rx.equation for rx in m.reactions].index(eq)


def _conc(m, T, P, Y):
    RU = 1.3806504e-16 * 6.02214179e23
    return P / (RU * T) * (Y / m.wt) / np.sum(Y / m.wt)


def test_tables(cmech):
    t = cmech.to_tables()
    assert (t["rtype"] == 5).sum() == 4 and (t["rtype"] == 6).sum() == 3
    i = _idx(cmech, "H+CH3(+M)<=>CH4(+M)")
    r = t["plog_par"][t["plog_ptr"][i]:t["plog_ptr"][i + 1]]
    assert r[0, :2].tolist() == [7.0, 4.0] and r[1].tolist() == [300.0, 3000.0, 0.01, 100.0]
    assert t["eff_ptr"][i + 1] == t["eff_ptr"][i]  # a Chebyshev rate has no [M]


def test_rate_definitions(cmech, corc):
    """q_f of a Chebyshev reaction = 10^(Chebyshev series) C_H C_CH3 (no [M]); of an LT reaction
    A T^b exp(-E/RT + B T^-1/3 + C T^-2/3) C_O C_H2; the RLT reverse rate from REV + RLT."""
    from numpy.polynomial import chebyshev as ch

    rng = np.random.default_rng(2)
    for T, Patm in ((900.0, 0.3), (1600.0, 7.0), (2400.0, 60.0)):
        P = Patm * P_ATM
        Y = rng.dirichlet(np.ones(cmech.KK))
        C = _conc(cmech, T, P, Y)
        qf, qr, _ = corc.rates(T, P, Y)
        sp = cmech.species.index
        i = _idx(cmech, "H+CH3(+M)<=>CH4(+M)")
        a = np.asarray(cmech.reactions[i].cheb[2:]).reshape(7, 4)
        Tr = (2 / T - 1 / 300.0 - 1 / 3000.0) / (1 / 3000.0 - 1 / 300.0)
        Pr = (2 * math.log10(Patm) - math.log10(0.01) - math.log10(100.0)) / (math.log10(100.0) - math.log10(0.01))
        k = 10.0 ** ch.chebval2d(Tr, Pr, a)
        assert abs(qf[i] / (k * C[sp("H")] * C[sp("CH3")]) - 1) < 1e-12
        i = _idx(cmech, "O+H2<=>H+OH")
        rx = cmech.reactions[i]
        k = rx.A * T ** rx.b * math.exp(-rx.E / (RUC * T) + 2.0 * T ** (-1 / 3) - 5.0 * T ** (-2 / 3))
        assert abs(qf[i] / (k * C[sp("O")] * C[sp("H2")]) - 1) < 1e-12
        i = _idx(cmech, "N+NO<=>N2+O")
        kr = 1.0e14 * math.exp(-75000.0 / (RUC * T) + 0.5 * T ** (-1 / 3) + 1.0 * T ** (-2 / 3))
        assert abs(qr[i] / (kr * C[sp("N2")] * C[sp("O")]) - 1) < 1e-12


def test_chebyshev_fit_tracks_the_troe_rate_it_replaces(cmech, corc, oracle, mech):
    """The generator's fit: each Chebyshev rate within 6 % of the GRI-3.0 Troe rate it replaces, at
    [M] = P/RT, over 500-2800 K and 0.03-80 atm (checks the series orientation and units)."""
    # a nitrogen bath with a little H and CH3: same concentrations on both sides, so q ratios are k ratios
    Y2 = np.zeros(mech.KK)
    for s, w in (("N2", 0.98), ("H", 0.01), ("CH3", 0.01)):
        Y2[mech.species.index(s)] = w
    for T in (500.0, 1200.0, 2800.0):
        for Patm in (0.03, 1.0, 80.0):
            q1 = corc.rates(T, Patm * P_ATM, Y2)[0]
            q0 = oracle.rates(T, Patm * P_ATM, Y2)[0]
            for eq in ("H+CH3(+M)<=>CH4(+M)", "2CH3(+M)<=>C2H6(+M)"):
                i0, i1 = _idx(mech, eq), _idx(cmech, eq)
                assert abs(q1[i1] / q0[i0] - 1) < 0.06, (eq, T, Patm, q1[i1] / q0[i0])


def test_oracle_matches_numpy(cmech, corc):
    from oracle.numpy_ref import NumpyKinetics

    nk = NumpyKinetics(cmech.to_tables())
    rng = np.random.default_rng(8)
    for _ in range(20):
        T, P = rng.uniform(400.0, 3200.0), P_ATM * 10.0 ** rng.uniform(-2.5, 2.5)  # also outside the fit range
        Y = rng.dirichlet(np.ones(cmech.KK))
        qf, qr, w = corc.rates(T, P, Y)
        qf2, qr2, w2 = nk.rates(T, P, Y)
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))


def _single(eq):
    """The CHEB mechanism's species and thermo with only reaction `eq` (and its auxiliary lines)."""
    import re

    from pychemkin_amd.mechanism import Mechanism

    text = open(CHEB_CHEM).read()
    r0 = re.search(r"^REACTIONS", text, re.M | re.I).start()
    lines = text[r0:].splitlines()
    body = [lines[0]]
    for j, ln in enumerate(lines[1:], 1):
        if ln.split()[:1] == [eq]:
            body.append(ln)
            k = j + 1
            while k < len(lines) and "=" not in lines[k] and lines[k].split()[:1] != ["END"]:
                body.append(lines[k])
                k += 1
    body.append("END")
    return Mechanism(text[:r0] + "\n".join(body) + "\n", open(THERM).read())


@pytest.mark.parametrize("eq,problem", [("H+CH3(+M)<=>CH4(+M)", 1), ("O+H2<=>H+OH", 1), ("O+H2<=>H+OH", 2),
                                        ("N+NO<=>N2+O", 1), ("N+NO<=>N2+O", 2)])
def test_oracle_temperature_jacobian_column(eq, problem):
    """d f / d T through the Chebyshev / Landau-Teller / RLT rate derivatives (dlkf, dlkr), one
    reaction at a time, against central differences.  (CONP: a Chebyshev rate's P is fixed; at
    constant volume its dependence on P(T) is left out of the approximate Chemkin Jacobian, as for
    PLOG, so that case is not checked.)"""
    from oracle.oracle import Oracle

    m = _single(eq)
    assert m.II == 1
    orc = Oracle(m)
    Y0 = ch4_air_Y(m, 1.0)[0] * 0.8 + np.random.default_rng(4).dirichlet(np.ones(m.KK)) * 0.2
    Y0 /= Y0.sum()
    T = 1750.0
    y = np.concatenate([[T], Y0])
    RU = 1.3806504e-16 * 6.02214179e23
    rho0 = 3 * P_ATM / (RU * T) / np.sum(Y0 / m.wt)
    kw = dict(problem=problem, energy=1, rho0=rho0, V0=1.0, P0=3 * P_ATM)
    f, J = orc.rhs_jac(y, **kw)
    h = 1e-3
    yp, ym = y.copy(), y.copy()
    yp[0] += h
    ym[0] -= h
    fd = (orc.rhs_jac(yp, **kw)[0] - orc.rhs_jac(ym, **kw)[0]) / (2 * h)
    sc = np.max(np.abs(fd[1:]))
    assert sc > 0 and np.max(np.abs(J[1:, 0] - fd[1:])) < 1e-6 * sc


def test_oracle_ignition_close_to_gri(cmech, corc, oracle, mech):
    for T0, Patm in ((1300.0, 1.0), (1500.0, 20.0)):
        Y0 = ch4_air_Y(mech, 1.0)[0]
        run = dict(problem=1, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
        r1, _ = corc.reactor(T0, Patm * P_ATM, 1.0, Y0, **run)
        r0, _ = oracle.reactor(T0, Patm * P_ATM, 1.0, Y0, **run)
        assert r1.status == 0 and r1.tau > 0
        assert abs(r1.tau / r0.tau - 1) < 0.1


# ------------------------------------------------------------------ GPU


@pytest.fixture(scope="module")
def cdm(cmech):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(cmech.to_tables())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 64, 20000])  # 20,000: the automatic path declines the specialised kernel
def test_gpu_rop(cmech, corc, cdm, n):
    rng = np.random.default_rng(n)
    T = rng.uniform(400.0, 3200.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-2.5, 2.5, n)
    Y = rng.dirichlet(np.ones(cmech.KK), n).T.copy()
    w = cdm.rop_thermo(T, P, Y)[0].cpu().numpy()
    m = min(n, 256)
    wo = corc.rop_batch(T[:m], P[:m], np.ascontiguousarray(Y[:, :m]))[0]
    assert np.max(np.abs(w[:, :m] - wo) / np.max(np.abs(wo), axis=0, keepdims=True)) < 1e-11


@pytest.mark.gpu
def test_gpu_reaction_rates(cmech, corc, cdm):
    rng = np.random.default_rng(1)
    n = 16
    T = rng.uniform(500.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-2.0, 2.0, n)
    Y = rng.dirichlet(np.ones(cmech.KK), n).T.copy()
    qf, qr = (x.cpu().numpy() for x in cdm.reaction_rates(T, P, Y))
    for j in range(n):
        qfo, qro, _ = corc.rates(T[j], P[j], Y[:, j])
        sc = max(np.max(np.abs(qfo)), np.max(np.abs(qro)))
        assert np.max(np.abs(qf[:, j] - qfo)) < 1e-11 * sc
        assert np.max(np.abs(qr[:, j] - qro)) < 1e-11 * sc


@pytest.mark.gpu
@pytest.mark.parametrize("path", [0, 1])  # 0: wave kernel (extended variant); 1: workgroup kernel forced
def test_gpu_reactors(cmech, corc, cdm, path):
    from pychemkin_amd import _native

    cases = [(1200, 1, 1.0, 1), (1400, 10, 0.7, 2), (1600, 50, 1.5, 1), (1300, 0.2, 1.0, 2)]
    run = dict(energy=1, t_end=0.2, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    T0 = np.array([c[0] for c in cases], float)
    P0 = np.array([c[1] for c in cases], float) * P_ATM
    Y0 = np.stack([ch4_air_Y(cmech, c[2])[0] for c in cases])
    prob = np.array([c[3] for c in cases], np.int32)
    _native.set_reactor_path(path)
    try:
        res = {k: v.cpu().numpy() for k, v in cdm.reactor_run(_native.make_cfg(**run), prob, T0, P0,
                                                                np.ones(len(cases)), Y0).items()}
    finally:
        _native.set_reactor_path(0)
    for i in range(len(cases)):
        r, Ye = corc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **run)
        assert r.status == 0 and res["stats"][i, 6] == 0
        assert abs(res["tau"][i] / r.tau - 1) < 1e-4 and abs(res["T"][i] / r.T - 1) < 1e-4
        for sp in ("CH4", "O2", "H2O", "CO2", "CO"):
            k = cmech.species.index(sp)
            assert abs(res["Y"][i, k] - Ye[k]) <= 1e-4 * max(abs(Ye[k]), 1e-3)
