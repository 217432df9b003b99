"""PLOG (pressure-dependent Arrhenius tables) and chemically activated (HIGH/) reactions on the
oracle and the device path.

Mechanism: data/gri30_plog_chem.inp (data/make_plog_mechanism.py), GRI-3.0 with PLOG tables of
1 to 5 points on seven elementary reactions and three falloff reactions rewritten as chemically
activated ones (one Lindemann, two Troe).  No such mechanism or golden exists in the reference, so parity with Chemkin is unpinned here: the C oracle is checked against the numpy
restatement and against the PLOG definition directly (ln k linear in ln P, end values outside
the table), and the GPU kernels against the oracle with the GRI-3.0 bars of
test_gpu_kernels.py / test_gpu_reactor.py.
"""
import math
import os

import numpy as np
from pychemkin_amd.constants import R_GAS
import pytest

from conftest import P_ATM, ROOT, THERM, ch4_air_Y

PLOG_CHEM = os.path.join(ROOT, "data", "gri30_plog_chem.inp")


@pytest.fixture(scope="module")
def pmech():
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism.from_files(PLOG_CHEM, THERM)


@pytest.fixture(scope="module")
def porc(pmech):
    from oracle.oracle import Oracle

    return Oracle(pmech)


def _states(KK, n, seed):
    rng = np.random.default_rng(seed)
    T = rng.uniform(300.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-2.5, 2.5, n)  # below, inside and above every table
    Y = rng.dirichlet(0.5 * np.ones(KK), n).T.copy()
    return T, P, Y


def test_plog_tables(pmech):
    t = pmech.to_tables()
    plog = np.nonzero(t["rtype"] == 3)[0]
    assert len(plog) == 7
    counts = sorted(int(t["plog_ptr"][i + 1] - t["plog_ptr"][i]) for i in plog)
    assert counts == [1, 2, 2, 3, 3, 4, 5]
    for i in plog:
        lnp = t["plog_par"][t["plog_ptr"][i]:t["plog_ptr"][i + 1], 0]
        assert np.all(np.diff(lnp) > 0)


def test_chemact_tables_and_rate_definition(pmech, porc):
    """O+CO(+M)<=>CO2(+M) as chemically activated Lindemann: kf = k0 / (1 + k0 [M] / k_inf)."""
    t = pmech.to_tables()
    assert int(np.sum(t["rtype"] == 4)) == 3
    i = next(j for j, rx in enumerate(pmech.reactions) if rx.equation == "O+CO(+M)<=>CO2(+M)")
    rx = pmech.reactions[i]
    assert t["rtype"][i] == 4 and t["ftype"][i] == 1
    T = 1300.0
    Y = np.random.default_rng(2).dirichlet(np.ones(pmech.KK))
    for p in (0.1, 1.0, 30.0):
        P = p * P_ATM
        qf, _, _ = porc.rates(T, P, Y)
        C = P / (R_GAS * T) * Y / pmech.wt / np.sum(Y / pmech.wt)
        M = C.sum() + sum((e - 1.0) * C[pmech.species.index(sp)] for sp, e in rx.efficiencies.items())
        k0 = rx.A * T ** rx.b * math.exp(-rx.E * rx.E_scale / T)
        kinf = rx.high[0] * T ** rx.high[1] * math.exp(-rx.high[2] * rx.E_scale / T)
        expect = k0 / (1.0 + k0 * M / kinf)
        kO, kCO = pmech.species.index("O"), pmech.species.index("CO")
        assert abs(qf[i] / (C[kO] * C[kCO]) / expect - 1) < 1e-9


def test_plog_rate_definition(pmech, porc):
    """kf of O+H2<=>H+OH at, between, below and above its table pressures (0.1, 1, 10, 100 atm)."""
    i = next(j for j, rx in enumerate(pmech.reactions) if rx.equation == "O+H2<=>H+OH")
    rx = pmech.reactions[i]
    T = 1500.0
    Y = np.random.default_rng(0).dirichlet(np.ones(pmech.KK))

    def k_entry(e):
        return e[1] * T ** e[2] * math.exp(-e[3] * rx.E_scale / T)

    ks = [k_entry(e) for e in rx.plog]
    for p, expect in [(0.1, ks[0]), (10.0, ks[2]), (0.01, ks[0]), (1000.0, ks[3]),
                      (3.0, math.exp(math.log(ks[1]) + (math.log(ks[2]) - math.log(ks[1])) * math.log(3.0) / math.log(10.0)))]:
        qf, _, _ = porc.rates(T, p * P_ATM, Y)
        C = (p * P_ATM) / (R_GAS * T) * np.asarray(Y) / pmech.wt / np.sum(np.asarray(Y) / pmech.wt)
        kO, kH2 = pmech.species.index("O"), pmech.species.index("H2")
        assert abs(qf[i] / (C[kO] * C[kH2]) / expect - 1) < 1e-6


def test_plog_oracle_matches_numpy(pmech, porc):
    from oracle.numpy_ref import NumpyKinetics

    nk = NumpyKinetics(pmech.to_tables())
    T, P, Y = _states(pmech.KK, 30, seed=5)
    for j in range(T.size):
        qf, qr, w = porc.rates(T[j], P[j], Y[:, j])
        qf2, qr2, w2 = nk.rates(T[j], P[j], Y[:, j])
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))


def test_plog_changes_ignition(pmech, porc, oracle, mech):
    """The PLOG tables matter: the oracle's ignition delay moves against plain GRI-3.0."""
    Y0 = ch4_air_Y(pmech, 1.0)[0]
    r1, _ = porc.reactor(1400.0, 10 * P_ATM, 1.0, Y0, problem=1, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8,
                         ign_mode="TIFP")
    r0, _ = oracle.reactor(1400.0, 10 * P_ATM, 1.0, Y0, problem=1, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8,
                           ign_mode="TIFP")
    assert r1.status == 0 and r0.status == 0 and r1.tau > 0
    assert abs(r1.tau / r0.tau - 1) > 1e-3


@pytest.fixture(scope="module")
def pdm(pmech):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(pmech.to_tables())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 17, 1000])
def test_plog_gpu_rop(pmech, porc, pdm, n):
    T, P, Y = _states(pmech.KK, n, seed=n)
    w, cp, h = (x.cpu().numpy() for x in pdm.rop_thermo(T, P, Y))
    wo, cpo, ho = porc.rop_batch(T, P, Y)
    scale = np.max(np.abs(wo), axis=0, keepdims=True)
    assert np.max(np.abs(w - wo) / scale) < 1e-11


@pytest.mark.gpu
def test_plog_gpu_reaction_rates(pmech, porc, pdm):
    T, P, Y = _states(pmech.KK, 19, seed=3)
    qf, qr = (x.cpu().numpy() for x in pdm.reaction_rates(T, P, Y))
    for j in range(T.size):
        qfo, qro, _ = porc.rates(T[j], P[j], Y[:, j])
        sc = max(np.max(np.abs(qfo)), np.max(np.abs(qro)))
        assert np.max(np.abs(qf[:, j] - qfo)) < 1e-11 * sc
        assert np.max(np.abs(qr[:, j] - qro)) < 1e-11 * sc


@pytest.mark.gpu
def test_plog_gpu_reactor(pmech, porc, pdm):
    """CONP and CONV ignition on the PLOG mechanism: the north_star bars (tau 0.5 %, T 1e-4)."""
    from pychemkin_amd import _native

    cases = [(1200, 1, 1.0, 1), (1400, 10, 1.0, 2), (1100, 0.05, 0.7, 1), (1600, 200, 1.5, 1), (1300, 30, 0.5, 2)]
    cfg = dict(energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    T0 = np.array([c[0] for c in cases], float)
    P0 = np.array([c[1] for c in cases], float) * P_ATM
    Y0 = np.stack([ch4_air_Y(pmech, c[2])[0] for c in cases])
    prob = np.array([c[3] for c in cases], np.int32)
    res = {k: v.cpu().numpy() for k, v in pdm.reactor_run(_native.make_cfg(**cfg), prob, T0, P0, np.ones(len(cases)),
                                                             Y0).items()}
    for i in range(len(cases)):
        r, Ye = porc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **cfg)
        assert res["stats"][i, 6] == r.status == 0
        assert r.tau > 0 and abs(res["tau"][i] / r.tau - 1) < 1e-4
        assert abs(res["T"][i] / r.T - 1) < 1e-4
        for sp in ("CH4", "O2", "H2O", "CO2", "CO"):
            k = pmech.species.index(sp)
            assert abs(res["Y"][i, k] - Ye[k]) <= 1e-4 * max(abs(Ye[k]), 1e-3)


@pytest.mark.gpu
def test_plog_afactor_set_rejected(pmech, pdm):
    from pychemkin_amd import _native

    i = int(np.nonzero(pmech.to_tables()["rtype"] == 3)[0][0])
    with pytest.raises(_native.NativeError):
        pdm.set_afactor(i, 1.0e10)


@pytest.mark.gpu
def test_drop_in_api_on_plog_mechanism(pmech, porc):
    """Chemistry.preprocess / Mixture.ROP / RxnRates (mixture.py:1693-1808) on the PLOG + HIGH
    mechanism, through the extended GPU kernel variant, at pressures inside and outside the tables."""
    import pychemkin_amd as ck

    chem = ck.Chemistry(label="gri30-plog")
    chem.chemfile = PLOG_CHEM
    chem.thermfile = THERM
    chem.preprocess()
    assert chem.KK == 53 and chem.IIGas == 325
    for p in (0.005, 0.7, 40.0, 500.0):
        m = ck.Mixture(chem)
        m.temperature = 1650.0
        m.pressure = p * P_ATM
        m.X = [("CH4", 0.05), ("O2", 0.15), ("N2", 0.7), ("OH", 0.01), ("H", 0.01), ("O", 0.01), ("CO", 0.05),
               ("HO2", 0.01), ("CH2O", 0.01)]
        qfo, qro, wo = porc.rates(1650.0, p * P_ATM, m.Y)
        assert np.max(np.abs(m.ROP() - wo)) < 1e-11 * np.max(np.abs(wo))
        qf, qr = m.RxnRates(reference_compat=False)
        assert np.max(np.abs(qf - qfo)) < 1e-11 * np.max(np.abs(qfo))
        assert np.max(np.abs(qr - qro)) < 1e-11 * np.max(np.abs(qro))
