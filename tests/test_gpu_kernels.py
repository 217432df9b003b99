"""GPU kernels vs the CPU oracle: species thermo, ROP / reaction rates (through the C ABI).

Tolerances: the oracle and the kernels evaluate the same FP64 expressions in a different
order (LDS atomics for the species sums), so results agree to rounding: 1e-11 relative to
the largest |wdot| of a state, 1e-12 relative for thermo.
"""
import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y, golden, within

pytestmark = pytest.mark.gpu

R = 1.3806504e-16 * 6.02214179e23


@pytest.fixture(scope="module")
def dm(tables):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(tables)


def _random_states(KK, n, seed=0):
    rng = np.random.default_rng(seed)
    T = rng.uniform(300.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, n)
    Y = rng.dirichlet(0.5 * np.ones(KK), n).T.copy()
    return T, P, Y


def test_species_thermo_matches_oracle(dm, oracle, mech):
    T = np.concatenate([np.linspace(250.0, 3500.0, 257), [1000.0, 999.999, 1000.001]])
    cp, h, s = (x.cpu().numpy() for x in dm.species_thermo(T))
    for j in range(0, T.size, 13):
        cpo, ho, so = oracle.thermo(T[j])
        assert np.allclose(cp[:, j], cpo, rtol=1e-13, atol=0)
        assert np.allclose(h[:, j], ho, rtol=1e-12, atol=1e-12)
        assert np.allclose(s[:, j], so, rtol=1e-12, atol=1e-12)


def test_species_cv_matches_speciesproperties_golden(chem):
    g = golden("speciesproperties")
    k = chem.get_specindex("N2")
    cv = np.array([chem.SpeciesCv(T)[k] * 1e-7 for T in g["state-temperature"]])
    assert np.max(np.abs(cv / np.asarray(g["state-Cv"]) - 1)) < 1e-12


@pytest.mark.parametrize("n", [1, 5, 8, 23, 63, 64, 4097])
def test_rop_thermo_matches_oracle(dm, oracle, mech, n):
    T, P, Y = _random_states(mech.KK, n, seed=n)
    w, cp, h = (x.cpu().numpy() for x in dm.rop_thermo(T, P, Y))
    wo, cpo, ho = oracle.rop_batch(T, P, Y)
    scale = np.max(np.abs(wo), axis=0, keepdims=True)
    assert np.max(np.abs(w - wo) / scale) < 1e-11
    assert np.max(np.abs(cp / cpo - 1)) < 1e-12
    assert np.max(np.abs(h - ho) / np.max(np.abs(ho))) < 1e-12


def test_reaction_rates_match_oracle(dm, oracle, mech):
    T, P, Y = _random_states(mech.KK, 33, seed=7)
    qf, qr = (x.cpu().numpy() for x in dm.reaction_rates(T, P, Y))
    for j in range(T.size):
        qfo, qro, _ = oracle.rates(T[j], P[j], Y[:, j])
        sc = max(np.max(np.abs(qfo)), np.max(np.abs(qro)))
        assert np.max(np.abs(qf[:, j] - qfo)) < 1e-11 * sc
        assert np.max(np.abs(qr[:, j] - qro)) < 1e-11 * sc


def test_reaction_rates_1800K_ordering_on_gpu(chem, mech):
    import pychemkin_amd as ck

    g = golden("reactionrates")
    m = ck.Mixture(chem)
    m.temperature = 1800.0
    m.pressure = 5 * P_ATM
    m.Y = ch4_air_Y(mech, 1.0)[0]
    order, net = m.list_reaction_rates()
    assert order.tolist() == g["state-order_1800"]
    # the reference reads the composition as mole fractions here (see test_oracle_golden)
    assert np.all(within(net, g["rate-net_reaction_rate_1800"], *g["tolerance-ROP"]))
    assert np.max(np.abs(net / np.asarray(g["rate-net_reaction_rate_1800"]) - 1)) < 2e-5


def test_afactor_update_is_seen_by_kernels(tables, oracle, mech):
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    T, P, Y = _random_states(mech.KK, 4, seed=3)
    qf0, _ = (x.cpu().numpy() for x in dm.reaction_rates(T, P, Y))
    A, _, _ = dm.arrhenius()
    dm.set_afactor(37, A[37] * 2.0)
    qf1, _ = (x.cpu().numpy() for x in dm.reaction_rates(T, P, Y))
    assert np.allclose(qf1[37], 2.0 * qf0[37], rtol=1e-13)
    mask = np.arange(mech.II) != 37
    assert np.array_equal(qf1[mask], qf0[mask])
    dm.close()


def test_mixture_rop_and_hrr(chem, oracle, mech):
    import pychemkin_amd as ck

    m = ck.Mixture(chem)
    m.temperature = 1500.0
    m.pressure = 2 * P_ATM
    m.X = [("CH4", 0.05), ("O2", 0.2), ("N2", 0.7), ("OH", 0.01), ("H", 0.01), ("CO", 0.03)]
    _, _, wo = oracle.rates(1500.0, 2 * P_ATM, m.Y)
    assert np.max(np.abs(m.ROP() - wo)) < 1e-11 * np.max(np.abs(wo))
    cpo, ho, _ = oracle.thermo(1500.0)
    # reference mixture.py:2172-2202 returns np.dot(H, ROP) without negation
    assert abs(m.volHRR() / np.sum(wo * ho * R * 1500.0) - 1) < 1e-10


def test_adiabatic_mixing_golden_on_gpu(chem):
    """mixturemixing.py:40-70 through the drop-in API: the mixture temperature comes from the device
    species thermo (ckmi_species_thermo) and the reference's Newton iteration."""
    import pychemkin_amd as ck

    g = golden("mixturemixing")
    fuel = ck.Mixture(chem)
    fuel.X = [("CH4", 1.0)]
    fuel.temperature = 300.0
    air = ck.Mixture(chem)
    air.X = [("O2", 0.21), ("N2", 0.79)]
    air.temperature = 300.0
    premixed = ck.isothermal_mixing(recipe=[(fuel, 1.0), (air, 17.19)], mode="mass", finaltemperature=300.0)
    ar = ck.Mixture(chem)
    ar.X = [("AR", 1.0)]
    ar.temperature = 600.0
    diluted = ck.adiabatic_mixing(recipe=[(premixed, 0.7), (ar, 0.3)], mode="mole")
    T = np.array([premixed.temperature, ar.temperature, diluted.temperature])
    assert np.all(within(T, g["state-temperature"], *g["tolerance-var"]))
    assert np.all(within(diluted.X, g["species-diluted_mole_fraction"], *g["tolerance-frac"]))


def test_static_rate_calls_match_mixture_methods(chem, mech):
    """Mixture.rate_of_production / reaction_rates (mixture.py:1353-1567) with the reference's signature give
    the numbers of the instance methods ROP() / RxnRates() on the same state (same kernels; the static forms
    renormalise the given fractions, so they agree to that rounding), for mole and mass input; the
    reactionrates golden through the static call."""
    import pychemkin_amd as ck

    M = ck.Mixture
    m = M(chem)
    m.temperature, m.pressure = 1500.0, 2 * P_ATM
    m.X = [("CH4", 0.05), ("O2", 0.2), ("N2", 0.7), ("OH", 0.01), ("H", 0.01), ("CO", 0.03)]
    w = m.ROP()
    for frac, mode in ((m.X, "mole"), (m.Y, "mass")):
        ws = M.rate_of_production(chem.chemID, m.pressure, m.temperature, frac, chem.WT, mode)
        assert np.allclose(ws, w, rtol=1e-13, atol=1e-13 * np.max(np.abs(w)))
    qf, qr = m.RxnRates()
    qfs, qrs = M.reaction_rates(chem.chemID, chem.IIGas, m.pressure, m.temperature, m.Y, chem.WT, "mass")
    assert np.allclose(qfs, qf, rtol=1e-13, atol=1e-13 * np.max(np.abs(qf)))
    assert np.allclose(qrs, qr, rtol=1e-13, atol=1e-13 * np.max(np.abs(qr)))
    # a state whose fractions are already normalised in floating point: bitwise the instance results
    y = np.asarray(m.Y)
    if y.sum() == 1.0:
        assert np.array_equal(M.rate_of_production(chem.chemID, m.pressure, m.temperature, y, chem.WT, "mass"),
                              m.ROP())
    # the reactionrates golden (1800 K, 5 atm, CH4/air phi = 1 as mass fractions): net rates of the top 5
    g = golden("reactionrates")
    y0 = ch4_air_Y(mech, 1.0)[0]
    qf, qr = M.reaction_rates(chem.chemID, chem.IIGas, 5 * P_ATM, 1800.0, y0, chem.WT, "mass")
    order, net = M._sorted_nonzero(qf - qr, 0.0)
    assert order.tolist() == g["state-order_1800"]
    assert np.all(within(net, g["rate-net_reaction_rate_1800"], *g["tolerance-ROP"]))
