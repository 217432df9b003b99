"""Host-side logic of the drop-in API (no GPU calls): composition, keywords, output grid."""
import numpy as np
import pytest

import pychemkin_amd as ck
from conftest import P_ATM, golden
from pychemkin_amd import _native
from pychemkin_amd.batchreactor import save_times
from pychemkin_amd.reactormodel import ReactorError


def test_preprocess_sizes(chem):
    assert chem.KK == 53 and chem.IIGas == 325 and chem.MM == 5
    assert chem.get_specindex("H2") == 0  # the reference rejects index 0 (chemistry.py:911-916)
    assert chem.get_specindex("n2") == 47
    assert chem.SpeciesComposition().shape == (5, 53)
    assert chem.SpeciesComposition(elemindex=1, specindex=chem.get_specindex("CH4")) == 4


def test_air_density_and_conversions(chem):
    air = ck.Mixture(chem)
    air.pressure = P_ATM
    air.temperature = 300.0
    air.X = ck.Air.X()
    g = golden("simple")
    assert abs(air.RHO / g["state-density"][0] - 1) < 1e-15
    y = air.Y
    x = ck.Mixture.mass_fraction_to_mole_fraction(y, chem.WT)
    assert np.allclose(x, air.X, rtol=1e-14)
    assert abs(air.WTM - (0.21 * chem.WT[3] + 0.79 * chem.WT[47])) < 1e-12


def test_fraction_to_concentration(chem):
    """mixture.py:821-935: c_k = rho Y_k / W_k = X_k P / (R T); negative entries removed, then normalised."""
    from pychemkin_amd.constants import R_GAS

    air = ck.Mixture(chem)
    air.pressure, air.temperature = 2 * P_ATM, 900.0
    air.X = ck.Air.X()
    cx = ck.Mixture.mole_fraction_to_concentration(chem.chemID, 2 * P_ATM, 900.0, air.X, chem.WT)
    cy = ck.Mixture.mass_fraction_to_concentration(chem.chemID, 2 * P_ATM, 900.0, air.Y, chem.WT)
    assert np.allclose(cx, air.X * 2 * P_ATM / (R_GAS * 900.0), rtol=1e-14, atol=0)
    assert np.allclose(cy, cx, rtol=1e-14, atol=0)
    assert np.allclose(air.concentration, cx, rtol=1e-14, atol=0)
    y = air.Y.copy()
    y[0] = -1e-3  # clipped, as Mixture.normalize does (mixture.py:506-511)
    assert np.allclose(ck.Mixture.mass_fraction_to_concentration(chem.chemID, 2 * P_ATM, 900.0, y, chem.WT), cy,
                       rtol=1e-14, atol=0)
    assert ck.Mixture.normalize([-1.0, 1.0, 3.0])[1].tolist() == [0.0, 0.25, 0.75]
    from pychemkin_amd.mixture import MixtureError

    with pytest.raises(MixtureError):
        ck.Mixture.mole_fraction_to_concentration(chem.chemID, P_ATM, 300.0, air.X[:5], chem.WT)


def test_equivalence_ratio_matches_conv_baseline(chem):
    fuel = ck.Mixture(chem)
    fuel.X = [("CH4", 1.0)]
    air = ck.Mixture(chem)
    air.X = [("O2", 0.21), ("N2", 0.79)]
    pre = ck.Mixture(chem)
    assert pre.X_by_Equivalence_Ratio(chem, fuel.X, air.X, np.zeros(chem.KK), ["CO2", "H2O", "N2"], 0.7) == 0
    assert abs(pre.X[chem.get_specindex("CH4")] / golden("CONV")["species-CH4_mole_fraction"][0] - 1) < 1e-14
    pre2 = ck.Mixture(chem)
    pre2.X_by_Equivalence_Ratio(chem, fuel.X, air.X, np.zeros(chem.KK), ["CO2", "H2O", "N2"], 1.0)
    assert abs(pre2.X[chem.get_specindex("CH4")] - 0.0950226) < 1e-7


def test_output_grid_matches_golden_times():
    g = golden("closed_homogeneous__transient")
    ts = save_times(5e-4, 5e-4 / 100)
    assert ts.tolist() == g["state-time"]
    g2 = golden("CONV")
    assert save_times(0.1, 0.01).tolist() == g2["state-time"]


def _reactor(chem):
    m = ck.Mixture(chem)
    m.X = [("H2", 2.0), ("N2", 3.76), ("O2", 1.0)]
    m.pressure = P_ATM
    m.temperature = 1000.0
    return ck.GivenPressureBatchReactor_EnergyConservation(m, label="tran")


def test_keywords_to_cfg(chem):
    r = _reactor(chem)
    with pytest.raises(ReactorError):
        r.reactor_cfg()  # TIME required
    r.time = 5e-4
    r.volume = 1.0
    r.tolerances = (1e-30, 1e-14)
    assert r.tolerances == (1e-20, 1e-12)  # clamps of batchreactor.py:193-214
    r.force_nonnegative = True
    r.set_ignition_delay(method="T_rise", val=400)
    r.stop_after_ignition()
    r.set_solver_max_timestep_size(1e-5)
    cfg = r.reactor_cfg()
    assert (cfg.energy, cfg.t_end, cfg.atol, cfg.rtol, cfg.nneg, cfg.ign_mode, cfg.ign_val, cfg.ign_stop, cfg.hmax) == \
        (1, 5e-4, 1e-20, 1e-12, 1, 2, 400.0, 1, 1e-5)
    r.set_ignition_delay(method="Species_peak", target="OH")
    cfg = r.reactor_cfg()
    assert cfg.ign_mode == 4 and cfg.ign_species == chem.get_specindex("OH")
    with pytest.raises(ReactorError):
        r.setkeyword("TIME", 1.0)  # protected (reactormodel.py:60-93)
    with pytest.raises(ReactorError):
        r.set_ignition_delay(method="bogus")


def test_one_keyword_policy_with_the_kin_abi(chem):
    """The drop-in's run() and the KIN ABI's KINAll0D_Calculate reject the same keywords
    (ckmi_kin_keyword_class): a typo'd ATLO is an error, not a silent default tolerance."""
    from pychemkin_amd import kin

    r = _reactor(chem)
    r.time = 5e-4
    r.setkeyword("ATLO", 1e-8)
    with pytest.raises(ReactorError, match="ATLO"):
        r.reactor_cfg()
    r.removekeyword("ATLO")
    r.setkeyword("MAXIT", 5000)
    r.setkeyword("NO_SDOUTPUT_WRITE", True)
    assert r.reactor_cfg().max_steps == 5000
    for k, c in (("ATOL", 1), ("rtol", 1), ("DTSV", 1), ("DELT", 2), ("NADAP", 2), ("ATLO", 0), ("ASEN", 0)):
        assert kin.keyword_class(k) == c, k
    # device keywords set as raw keywords are read, not dropped (round-3 advice)
    r.setkeyword("GFAC", 2.0)
    r.setkeyword("DXMX", 1e-5)
    cfg = r.reactor_cfg()
    assert cfg.gfac == 2.0 and cfg.hmax == 1e-5
    r.removekeyword("GFAC")
    r.removekeyword("DXMX")
    r.setkeyword("POLEN", 0.5)  # an engine keyword on a batch reactor: rejected, not silently unread
    with pytest.raises(ReactorError, match="POLEN"):
        r.reactor_cfg()
    r.removekeyword("POLEN")
    r.setprofile(ck.reactormodel.Profile("HTCPRO", [0.0, 1.0], [1.0, 2.0]))
    with pytest.raises(ReactorError, match="HTCPRO"):
        r.reactor_cfg()


def test_volume_profile_cfg(chem):
    m = ck.Mixture(chem)
    m.X = [("CH4", 0.1), ("O2", 0.2), ("N2", 0.7)]
    m.pressure = 3 * P_ATM
    m.temperature = 800.0
    r = ck.GivenVolumeBatchReactor_EnergyConservation(m, label="RCM")
    r.volume = 10.0
    r.time = 0.1
    r.set_volume_profile([0.0, 0.01, 2.0], [10.0, 4.0, 4.0])
    cfg = r.reactor_cfg()
    assert cfg.nprof == 3 and list(cfg.prof_v[:3]) == [10.0, 4.0, 4.0]
    r.heat_loss_rate = 5.0
    r.heat_transfer_coefficient = 1e-3
    r.heat_transfer_area = 20.0
    r.ambient_temperature = 350.0
    r.gasratemultiplier = 2.0
    r.adaptive_solution_saving(True, steps=20)
    cfg = r.reactor_cfg()
    assert (cfg.qloss, cfg.htc, cfg.areaq, cfg.tamb, cfg.gfac, cfg.asteps) == (5.0, 1e-3, 20.0, 350.0, 2.0, 20)
    r.set_heat_loss_profile([0.0, 0.05], [0.0, 10.0])
    cfg = r.reactor_cfg()
    assert cfg.prof2_kind == 1 and cfg.nprof2 == 2 and cfg.nprof == 3
    r.set_heat_transfer_area_profile([0.0, 0.05], [1.0, 2.0])
    cfg = r.reactor_cfg()  # QPRO with AEXT: QPRO in the second slot, AEXT in the third
    assert cfg.prof2_kind == 1 and cfg.nprof2 == 2 and cfg.nprof3 == 2 and list(cfg.prof3_v[:2]) == [1.0, 2.0]


def test_temperature_profile_cfg(chem):
    m = ck.Mixture(chem)
    m.X = [("CH4", 0.1), ("O2", 0.2), ("N2", 0.7)]
    m.pressure = P_ATM
    m.temperature = 1000.0
    r = ck.GivenPressureBatchReactor_FixedTemperature(m, label="TPRO")
    r.time = 1e-3
    r.set_temperature_profile([0.0, 5e-4, 1e-3], [1000.0, 1500.0, 1500.0])
    r.adaptive_solution_saving(True, value_change=10.0, target="temperature")
    cfg = r.reactor_cfg()
    assert cfg.energy == 2 and cfg.prof_kind == 1 and cfg.nprof == 3 and cfg.avar == 0 and cfg.avalue == 10.0


def test_afactor_get_set(chem):
    A0 = chem.get_reaction_AFactor(1)
    assert A0 == 1.2e17
    chem.set_reaction_AFactor(1, 2.4e17)
    assert chem.get_reaction_parameters()[0][0] == 2.4e17
    chem.set_reaction_AFactor(1, A0)
    assert chem.get_gas_reaction_string(52) == "H+CH3(+M)<=>CH4(+M)"
    with pytest.raises(Exception):
        chem.set_reaction_AFactor(0, 1.0)


def test_make_cfg_rejects_long_profiles():
    with pytest.raises(ValueError):
        _native.make_cfg(profile=(np.arange(70.0), np.ones(70)))


def test_static_rate_calls_check_arguments(chem):
    """Mixture.rate_of_production / reaction_rates (mixture.py:1353-1567) take the reference's signature and
    its argument checks (raised here instead of exit()); use_idealgas_law is the ideal-gas state."""
    import inspect

    M = ck.Mixture
    assert list(inspect.signature(M.rate_of_production).parameters) == ["chemID", "p", "t", "frac", "wt", "mode"]
    assert list(inspect.signature(M.reaction_rates).parameters) == ["chemID", "numbreaction", "p", "t", "frac",
                                                                    "wt", "mode"]
    x = np.full(chem.KK, 1.0 / chem.KK)
    with pytest.raises(ck.mixture.MixtureError, match="invalid chemistry"):
        M.rate_of_production(-1, P_ATM, 1000.0, x, chem.WT, "mole")
    with pytest.raises(ck.mixture.MixtureError, match="pressure"):
        M.rate_of_production(chem.chemID, 0.0, 1000.0, x, chem.WT, "mole")
    with pytest.raises(ck.mixture.MixtureError, match="same size"):
        M.rate_of_production(chem.chemID, P_ATM, 1000.0, x[:-1], chem.WT, "mole")
    with pytest.raises(ck.mixture.MixtureError, match='"mole" or "mass"'):
        M.reaction_rates(chem.chemID, chem.IIGas, P_ATM, 1000.0, x, chem.WT, "volume")
    with pytest.raises(ck.mixture.MixtureError, match="numbreaction"):
        M.reaction_rates(chem.chemID, chem.IIGas - 1, P_ATM, 1000.0, x, chem.WT, "mole")
    air = ck.Mixture(chem)
    air.use_idealgas_law()
    assert air.userealgas is False


def test_dropin_gap_methods_with_reference_signatures(chem):
    """setsolutionspeciesfracmode (reactormodel.py:1816), usefullkeywords (:814), validate_inputs
    (batchreactor.py:794) and create_solution_mixtures (:1487) with the reference's signatures (host only)."""
    from pychemkin_amd.reactormodel import Keyword

    r = _reactor(chem)
    assert r.validate_inputs() == 1  # TIME (batchreactor.py:1814-1815)
    r.time = 5e-4
    assert r.validate_inputs() == 0
    r.setsolutionspeciesfracmode(mode="mole")
    assert r._speciesmode == "mole"
    r.setsolutionspeciesfracmode()
    assert r._speciesmode == "mass"
    with pytest.raises(ReactorError):
        r.setsolutionspeciesfracmode("volume")
    assert r.create_solution_mixtures(np.zeros((chem.KK, 1))) == 1  # nothing processed yet
    with pytest.raises(ReactorError):
        r.setkeyword("CONP", True)  # protected in API mode
    try:
        r.usefullkeywords(True)
        assert Keyword.noFullKeyword is False
        r.setkeyword("CONP", True)  # full-keyword mode: protected keywords may be set
        r.removekeyword("CONP")
        r.tolerances = (1e-20, 1e-8)
        r.force_nonnegative = True
        r.set_ignition_delay(method="T_rise", val=400)
        lines = r.full_keyword_lines()
    finally:
        r.usefullkeywords(False)
    assert Keyword.noFullKeyword is True
    # the block of batchreactor.py:822-925: keywords, TRAN, CONP, ENRG, PRES [atm], TEMP, TIME, REAC, QRGEQ, END
    assert lines[-2:] == ["QRGEQ", "END"]
    for must in ("ATOL    1e-20", "RTOL    1e-08", "NNEG", "DTIGN    400.0", "TRAN", "CONP", "ENRG", "PRES    1.0",
                 "TEMP    1000.0", "TIME    0.0005"):
        assert must in lines, must
    reac = [x for x in lines if x.startswith("REAC")]
    assert sorted(x.split()[1] for x in reac) == ["H2", "N2", "O2"]
    X = dict((x.split()[1], float(x.split()[2])) for x in reac)
    assert abs(X["O2"] - 1.0 / 6.76) < 1e-15 and abs(sum(X.values()) - 1.0) < 1e-15
