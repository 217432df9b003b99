"""CPU oracle pinned against the reference's Chemkin goldens (tests/golden/*.json)."""
import numpy as np
import pytest

from conftest import (P_ATM, SENS_FACTOR, SENS_RUN, ch4_air_Y, check_h2_golden, golden, h2_air_Y,
                      sensitivity_mixture, top5, within)

R = 1.3806504e-16 * 6.02214179e23


def test_air_density_simple_baseline(mech):
    g = golden("simple")
    X = np.asarray(g["species-mole_fraction"])
    rho = g["state-pressure"][0] * np.sum(X * mech.wt) / (R * g["state-temperature"][0])
    assert abs(rho / g["state-density"][0] - 1) < 1e-15


def test_density_createmixture_baseline(mech):
    # createmixture.py:60-68,112-123: CH4 0.08, N2 0.6, O2 0.2, H2O 0.12 at 10 atm (last loop)
    g = golden("createmixture")
    X = np.zeros(mech.KK)
    for sp, x in (("CH4", 0.08), ("N2", 0.6), ("O2", 0.2), ("H2O", 0.12)):
        X[mech.species.index(sp)] = x
    T = np.asarray(g["state-temperature"])
    rho = 10 * P_ATM * np.sum(X * mech.wt) / (R * T)
    assert np.max(np.abs(rho / np.asarray(g["state-density"]) - 1)) < 1e-14


def test_n2_cv_speciesproperties_baseline(oracle, mech):
    g = golden("speciesproperties")
    k = mech.species.index("N2")
    cv = np.array([(oracle.thermo(T)[0][k] - 1.0) * R * 1e-7 for T in g["state-temperature"]])
    assert np.all(within(cv, g["state-Cv"], *g["tolerance-var"]))
    assert np.max(np.abs(cv / np.asarray(g["state-Cv"]) - 1)) < 1e-12


def test_h2_air_conp_trajectory(oracle, mech):
    """closed_homogeneous__transient.py:61-131: CONP, 1000 K, 1 atm, t_end 0.5 ms, 1e-20/1e-8, NNEG, DTIGN 400.

    All five golden columns on all 101 points, the ignition front included.  Round 2 held X_H2O on
    53/101 and wdot_H2O on 82/101: the radical pool grew 1e-4 slower than Chemkin's because E [cal/mol]
    was converted with R_GAS_CAL instead of Chemkin's RUC = 8.314510e7 / 4.184e7 (mechanism.RU_ACT)."""
    g = golden("closed_homogeneous__transient")
    ts = np.asarray(g["state-time"])
    Y0 = h2_air_Y(mech)
    res, Yend, (ts, ys, ps, vs) = oracle.reactor(1000.0, P_ATM, 1.0, Y0, t_save=ts, problem=1, energy=1, t_end=5e-4,
                                                 atol=1e-20, rtol=1e-8, nneg=True, ign_mode="T_rise", ign_val=400.0)
    assert res.status == 0
    k = mech.species.index("H2O")
    rop = np.array([oracle.rates(ys[i, 0], ps[i], ys[i, 1:])[2][k] for i in range(len(ts))])
    check_h2_golden(g, mech, ts, ys[:, 0], ys[:, 1:], rop, min_ok=101)
    Tg = np.asarray(g["state-temperature"])
    assert np.max(np.abs(ys[:, 0] / Tg - 1)) < 1e-6  # measured 3.6e-7, at the ignition front
    assert abs(ys[-1, 0] / Tg[-1] - 1) < 1e-7
    # ignition time (T0 + 400 K) from the golden trajectory by interpolation
    assert abs(res.tau / np.interp(1400.0, Tg, ts) - 1) < 2e-5


def test_ch4_air_rcm_conv_with_volume_profile(oracle, mech):
    """CONV.py:62-140: CONV, CH4/air phi 0.7, 800 K, 3 atm, VPRO 10->4 cm3 in 10 ms, 1e-10/1e-8, NNEG, TIFP."""
    g = golden("CONV")
    ts = np.asarray(g["state-time"])
    Y0 = ch4_air_Y(mech, 0.7)[0]
    X0 = (Y0 / mech.wt) / np.sum(Y0 / mech.wt)
    assert abs(X0[mech.species.index("CH4")] / g["species-CH4_mole_fraction"][0] - 1) < 1e-14
    res, Yend, (ts, ys, ps, vs) = oracle.reactor(800.0, 3 * P_ATM, 10.0, Y0, t_save=ts, problem=2, energy=1, t_end=0.1,
                                                 atol=1e-10, rtol=1e-8, nneg=True, ign_mode="TIFP",
                                                 profile=([0.0, 0.01, 2.0], [10.0, 4.0, 4.0]))
    assert res.status == 0
    assert np.all(within(ys[:, 0], g["state-temperature"], *g["tolerance-var"]))
    k = mech.species.index("CH4")
    x = ys[:, 1 + k] / mech.wt[k] / np.sum(ys[:, 1:] / mech.wt, axis=1)
    assert np.all(within(x, g["species-CH4_mole_fraction"], *g["tolerance-frac"]))
    rop = np.array([oracle.rates(ys[i, 0], ps[i], ys[i, 1:])[2][k] for i in range(len(ts))])
    assert np.all(within(rop, g["rate-CH4_production_rate"], *g["tolerance-ROP"]))
    assert abs(rop[0] / g["rate-CH4_production_rate"][0] - 1) < 1e-8
    # ignition (max dT/dt) between the 30 and 40 ms saved points of the golden
    assert 0.03 < res.tau < 0.04


def test_reaction_rates_1800K_ordering(oracle, mech):
    """reactionrates.py:72-116: CH4/air phi=1, 5 atm, 1800 K, nonzero net rates in descending order.

    The reference's Mixture.RxnRates hands the MASS fractions to KINGetGasReactionRates
    (mixture.py:1540), and the closed library reads that argument as MOLE fractions (Chemkin's
    CKKFKR(P, T, X) convention).  The golden rates are those of the state whose mole fractions
    equal the mixture's mass fractions: reproduced to <= 1.4e-5 that way (3 of 5 to 1e-14), while
    reading the array as mass fractions misses by 0.85-1.82x (the round-1 "parity partial").
    With Chemkin's activation-energy gas constant (mechanism.RU_ACT) all 5 agree to ~1e-14.
    """
    g = golden("reactionrates")
    Y0 = ch4_air_Y(mech, 1.0)[0]
    gold = np.asarray(g["rate-net_reaction_rate_1800"])

    def net_order(Y):
        qf, qr, _ = oracle.rates(1800.0, 5 * P_ATM, Y)
        net = qf - qr
        nz = np.nonzero(net)[0]
        order = nz[np.argsort(-net[nz], kind="stable")]
        return order, net[order]

    y_as_x = Y0 * mech.wt / np.sum(Y0 * mech.wt)  # mass fractions of the state with X = Y0
    order, net = net_order(y_as_x)
    assert order.tolist() == g["state-order_1800"]
    assert np.all(within(net, gold, *g["tolerance-ROP"]))
    assert np.max(np.abs(net / gold - 1)) < 1e-12
    # the same rates read as mass fractions: same ordering, magnitudes off by up to 1.8x
    order_m, net_m = net_order(Y0)
    assert order_m.tolist() == g["state-order_1800"]
    assert np.max(np.abs(net_m / gold - 1)) > 0.5


def test_afactor_sensitivity_golden(oracle, mech, chem):
    """sensitivity.baseline: 325 brute-force A-factor perturbations of a C3H8/CH4/H2 ignition
    (sensitivity.py:141-160).  The oracle reproduces Chemkin's top-5 positive and negative
    reactions exactly and the coefficients (d tau [ms] / 0.001) within 3 % (most within 1 %);
    this pins the kinetics, the integrator and the TIFP definition together."""
    g = golden("sensitivity")
    mix = sensitivity_mixture(chem)
    II = mech.II
    r0, _ = oracle.reactor(900.0, P_ATM, 10.0, mix.Y, **SENS_RUN)
    nf, res, _ = oracle.reactor_batch_pert(np.full(II, 900.0), np.full(II, P_ATM), np.tile(mix.Y, (II, 1)),
                                           np.arange(II, dtype=np.int32), np.full(II, SENS_FACTOR),
                                           V0=np.full(II, 10.0), **SENS_RUN)
    assert nf == 0 and r0.status == 0
    sens = (np.array([r.tau for r in res]) - r0.tau) * 1e3 / (SENS_FACTOR - 1.0)
    pos, neg = top5(sens)
    assert pos == set(g["state-index_positive"]) and neg == set(g["state-index_negative"])
    idx = g["state-index_positive"] + g["state-index_negative"]
    ref = np.array(g["rate-sensitivity_positive"] + g["rate-sensitivity_negative"])
    assert np.all(np.abs(sens[idx] / ref - 1) < 0.03)
    assert np.median(np.abs(sens[idx] / ref - 1)) < 0.01


def test_hp_equilibrium_adiabatic_flame_temperature(oracle, mech, tables):
    """adiabaticflametemperature.baseline (Chemkin HP equilibrium of CH4/O2 at 295.15 K, 1 atm,
    phi = 0.5..1.6): an adiabatic CONP reactor holding the reactants' H and P relaxes to the same
    state.  Reproduced to ~1e-8: pins NASA-7 (h, s), K_c of every reversible reaction and the
    CONP energy equation at 2900-3100 K together."""
    from conftest import hp_equilibrium_start

    g = golden("adiabaticflametemperature")
    for phi, Tg in zip(g["state-equivalence_ratio"], g["state-temperature"]):
        Ts, Yp = hp_equilibrium_start(mech, tables, phi)
        res, _ = oracle.reactor(Ts, P_ATM, 1.0, Yp, problem=1, energy=1, t_end=1.0, atol=1e-14, rtol=1e-9)
        assert res.status == 0
        assert within(np.array([res.T]), np.array([Tg]), *g["tolerance-var"]).all()
        assert abs(res.T / Tg - 1) < 1e-7, (phi, res.T, Tg)


def _equilibrium_premixed(mech):
    """equilibriumcomposition.py:50-62: fuel X CH4/H2 = 0.8/0.2, air Y O2/N2 = 0.23/0.77, mixed
    1 : 17.19 by mass (isothermal_mixing, mode="mass") -> mass fractions."""
    Xf = np.zeros(mech.KK)
    Xf[mech.species.index("CH4")], Xf[mech.species.index("H2")] = 0.8, 0.2
    Yf = Xf * mech.wt / np.sum(Xf * mech.wt)
    Ya = np.zeros(mech.KK)
    Ya[mech.species.index("O2")], Ya[mech.species.index("N2")] = 0.23, 0.77
    return (Yf + 17.19 * Ya) / 18.19


def test_tp_equilibrium_no_golden(oracle, mech):
    """equilibriumcomposition.baseline: TP-equilibrium NO [ppm] at 1 atm, T = 500..2480 K (100
    points), by element-potential Gibbs minimisation over the oracle's NASA-7 thermo
    (oracle/equilibrium.py).  Pins h and s of every species that matters for NO against the
    vendor's equilibrium solver: all 100 points inside the golden tolerance."""
    from oracle.equilibrium import TPEquilibrium

    g = golden("equilibriumcomposition")
    Y = _equilibrium_premixed(mech)
    eq = TPEquilibrium(mech, oracle.thermo)
    iNO = mech.species.index("NO")
    Ts = np.asarray(g["state-temperature"])
    no = np.zeros(Ts.size)
    for i in range(Ts.size - 1, -1, -1):  # hot to cold: continuation from the previous solution
        no[i] = eq.solve(Ts[i], 1.0, Y)[iNO] * 1e6
    gold = np.asarray(g["species-NO_mole_fraction"])
    assert np.all(within(no, gold, *g["tolerance-frac"]))
    big = gold > 1.0  # >= 1 ppm: relative agreement
    assert np.max(np.abs(no[big] / gold[big] - 1)) < 1e-7


def test_mixing_golden_composition(chem, mech):
    """mixturemixing.baseline, composition half (mixturemixing.py:40-60): CH4 + air 1 : 17.19 by
    mass at 300 K, then 0.7 : 0.3 by moles with Ar at 600 K.  Host-side mixing, no GPU."""
    import pychemkin_amd as ck

    g = golden("mixturemixing")
    fuel = ck.Mixture(chem)
    fuel.X = [("CH4", 1.0)]
    fuel.temperature = 300.0
    air = ck.Mixture(chem)
    air.X = [("O2", 0.21), ("N2", 0.79)]
    air.temperature = 300.0
    premixed = ck.isothermal_mixing(recipe=[(fuel, 1.0), (air, 17.19)], mode="mass", finaltemperature=300.0)
    assert np.all(within(premixed.X, g["species-premixed_mole_fraction"], *g["tolerance-frac"]))
    assert premixed.temperature == g["state-temperature"][0]
    ar = ck.Mixture(chem)
    ar.X = [("AR", 1.0)]
    ar.temperature = 600.0
    x, _ = ck.mixture._combine([(premixed, 0.7), (ar, 0.3)], "mole")
    assert np.all(within(x, g["species-diluted_mole_fraction"], *g["tolerance-frac"]))


def test_adiabatic_mixing_temperature_host_logic(chem, mech, oracle, monkeypatch):
    """mixturemixing.baseline, temperature half, with the oracle's thermo standing in for the device
    species thermo (the GPU run of the same call is in test_gpu_kernels): the reference's Newton
    iteration (mixture.py:3179-3266) lands within the golden tolerance of 368.674 K."""
    import pychemkin_amd as ck
    from pychemkin_amd.constants import R_GAS

    monkeypatch.setattr(type(chem), "SpeciesH", lambda self, T, pres=None: oracle.thermo(T)[1] * R_GAS * T)
    monkeypatch.setattr(type(chem), "SpeciesCp", lambda self, T, pres=None: oracle.thermo(T)[0] * R_GAS)
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
    assert within(np.array([diluted.temperature]), np.array([g["state-temperature"][2]]), *g["tolerance-var"]).all()
    assert ar.temperature == g["state-temperature"][1]
