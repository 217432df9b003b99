"""Batch-reactor kernel (ckmi_reactor_run) vs the CPU oracle and the reference goldens.

Parity bar (BASELINE.json north_star): ignition delay within 0.5 % relative, final T and major
species within rtol 1e-4.  The kernel runs the oracle's integrator step for step, so in
practice tau agrees to ~1e-5 or better (max 9.4e-6 over an 8,192-reactor bench sample); the
tests assert the north_star bar plus a tighter "same algorithm" bar on tau (1e-4).
"""
import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y, check_h2_golden, golden, h2_air_Y, within

pytestmark = pytest.mark.gpu

MAJOR = ("CH4", "O2", "N2", "H2O", "CO2", "CO", "H2")


@pytest.fixture(scope="module")
def dm(tables):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(tables)


def _run_both(dm, oracle, mech, cases, **cfg):
    from pychemkin_amd import _native

    T0 = np.array([c[0] for c in cases], float)
    P0 = np.array([c[1] for c in cases], float) * P_ATM
    Y0 = np.stack([ch4_air_Y(mech, c[2])[0] for c in cases])
    prob = np.array([c[3] for c in cases], np.int32)
    V0 = np.ones(len(cases))
    res = dm.reactor_run(_native.make_cfg(**cfg), prob, T0, P0, V0, Y0)
    res = {k: v.cpu().numpy() for k, v in res.items()}
    ref = [oracle.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **cfg) for i in range(len(cases))]
    return res, ref


def _check(res, ref, mech, tau_rtol=1e-4, stopped=False):
    for i, (r, Ye) in enumerate(ref):
        assert res["stats"][i, 6] == r.status == 0
        if r.tau > 0:
            assert abs(res["tau"][i] / r.tau - 1) < min(tau_rtol, 5e-3)
        else:
            assert res["tau"][i] == r.tau
        if stopped:
            # IGN_STOP ends the run at the end of the first step past the ignition point: that
            # time is a property of the step sequence, so the states are compared only there
            continue
        assert abs(res["T"][i] / r.T - 1) < 1e-4
        for sp in MAJOR:
            k = mech.species.index(sp)
            assert abs(res["Y"][i, k] - Ye[k]) <= 1e-4 * max(abs(Ye[k]), 1e-3)


CASES = [(1200, 1, 1.0, 1), (1200, 1, 1.0, 2), (1100, 1, 0.5, 1), (1700, 100, 2.0, 1), (1000, 3, 0.7, 2),
         (1400, 10, 1.0, 1), (1550, 30, 1.5, 2), (1300, 100, 0.5, 2)]


def test_conp_conv_energy_tifp(dm, oracle, mech):
    res, ref = _run_both(dm, oracle, mech, CASES, energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    _check(res, ref, mech)
    # same integrator: rounding-level differences (summation order of the rates, DPP reductions,
    # f32 step-size roots on both sides but different libm) flip individual accept/reject decisions
    # of the adaptive step control, so step counts drift by up to ~15 %; the trajectories do not
    nst = np.array([r.nst for r, _ in ref])
    ratio = res["stats"][:, 0] / nst
    assert np.all(np.abs(ratio - 1) < 0.25) and abs(np.mean(ratio) - 1) < 0.1


@pytest.mark.parametrize("path", [2, 3])
def test_newton_inverse_forms_match_oracle(dm, oracle, mech, path):
    """Both forms of the wave kernel's Newton inverse -- FP64 (path 2, 8 waves per workgroup) and
    FP32-stored (path 3, 12 waves; the automatic choice for rtol >= 1e-9) -- against the oracle
    (FP64 LU) at the north_star bars."""
    from pychemkin_amd import _native

    _native.set_reactor_path(path)
    try:
        res, ref = _run_both(dm, oracle, mech, CASES, energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    finally:
        _native.set_reactor_path(0)
    _check(res, ref, mech)


def test_given_temperature(dm, oracle, mech):
    res, ref = _run_both(dm, oracle, mech, CASES[:4], energy=2, t_end=2e-3, atol=1e-12, rtol=1e-7)
    _check(res, ref, mech)
    assert np.allclose(res["T"], [c[0] for c in CASES[:4]], rtol=0, atol=0)


@pytest.mark.parametrize("mode,val,target,stop", [("T_rise", 400.0, None, True), ("T_ignition", 1800.0, None, False),
                                                  ("Species_peak", 0.0, "OH", False)])
def test_ignition_definitions(dm, oracle, mech, mode, val, target, stop):
    sp = mech.species.index(target) if target else 0
    res, ref = _run_both(dm, oracle, mech, CASES[:6], energy=1, t_end=0.5, atol=1e-10, rtol=1e-8, ign_mode=mode,
                         ign_val=val, ign_species=sp, ign_stop=stop, nneg=True)
    _check(res, ref, mech, stopped=stop)
    assert np.all(res["tau"] > 0)
    if stop:
        T0 = np.array([c[0] for c in CASES[:6]], float)
        assert np.all(res["T"] >= T0 + val) and np.all([r.T >= T0[i] + val for i, (r, _) in enumerate(ref)])
        # stopped runs end shortly after ignition, long before t_end
        assert np.all(res["stats"][:, 0] < np.array([r.nst for r, _ in ref]) * 1.5 + 50)


def test_h2_air_golden_through_drop_in_api(chem, mech):
    """closed_homogeneous__transient.py:61-131 through the PyChemkin-style API on the GPU."""
    import pychemkin_amd as ck

    g = golden("closed_homogeneous__transient")
    m = ck.Mixture(chem)
    m.X = [("H2", 2.0), ("O2", 1.0), ("N2", 3.76)]
    m.temperature = 1000.0
    m.pressure = P_ATM
    r = ck.GivenPressureBatchReactor_EnergyConservation(m, label="tran")
    r.time = 5e-4
    r.tolerances = (1e-20, 1e-8)
    r.force_nonnegative = True
    r.timestep_for_saving_solution = 5e-4 / 100
    r.set_ignition_delay(method="T_rise", val=400)
    assert r.run() == 0
    r.process_solution()
    t = r.get_solution_variable_profile("time")
    T = r.get_solution_variable_profile("temperature")
    Tg = np.asarray(g["state-temperature"])
    mixes = [r.get_solution_mixture_at_index(i) for i in range(len(t))]
    k = chem.get_specindex("H2O")
    Y = np.stack([mx.Y for mx in mixes])
    wdot = np.array([mx.ROP()[k] for mx in mixes])  # closed_homogeneous__transient.py:176-181
    rho = np.array([mx.RHO for mx in mixes])
    check_h2_golden(g, mech, t, T, Y, wdot, min_ok=101)
    assert np.all(within(rho, g["state-density"], *g["tolerance-var"]))
    assert abs(T[-1] / Tg[-1] - 1) < 1e-6
    tg = np.interp(1400.0, Tg, t)
    assert abs(r.get_ignition_delay() * 1e-3 / tg - 1) < 1e-4


def test_rcm_conv_volume_profile_golden(chem, oracle, mech):
    """CONV.py:62-140 on the GPU: VPRO 10 -> 4 cm3 in 10 ms, then hold; CONV + ENERGY, TIFP."""
    import pychemkin_amd as ck

    g = golden("CONV")
    fuel = ck.Mixture(chem)
    fuel.X = [("CH4", 1.0)]
    air = ck.Mixture(chem)
    air.X = [("O2", 0.21), ("N2", 0.79)]
    m = ck.Mixture(chem)
    m.X_by_Equivalence_Ratio(chem, fuel.X, air.X, np.zeros(chem.KK), ["CO2", "H2O", "N2"], 0.7)
    m.temperature = 800.0
    m.pressure = 3 * P_ATM
    r = ck.GivenVolumeBatchReactor_EnergyConservation(m, label="RCM")
    r.volume = 10.0
    r.time = 0.1
    r.tolerances = (1e-10, 1e-8)
    r.force_nonnegative = True
    r.timestep_for_saving_solution = 0.01
    r.set_volume_profile([0.0, 0.01, 2.0], [10.0, 4.0, 4.0])
    r.set_ignition_delay(method="T_inflection")
    assert r.run() == 0
    r.process_solution()
    T = r.get_solution_variable_profile("temperature")
    assert np.all(within(T, g["state-temperature"], *g["tolerance-var"]))
    k = chem.get_specindex("CH4")
    x = np.array([r.get_solution_mixture_at_index(i).X[k] for i in range(len(T))])
    assert np.all(within(x, g["species-CH4_mole_fraction"], *g["tolerance-frac"]))
    assert 30.0 < r.get_ignition_delay() < 40.0
    res, _ = oracle.reactor(800.0, 3 * P_ATM, 10.0, m.Y, problem=2, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8,
                            nneg=True, ign_mode="TIFP", profile=([0.0, 0.01, 2.0], [10.0, 4.0, 4.0]))
    assert abs(r.get_ignition_delay() * 1e-3 / res.tau - 1) < 1e-6


def test_pressure_profile_conp(dm, oracle, mech):
    from pychemkin_amd import _native

    prof = ([0.0, 1e-3, 1.0], [P_ATM, 5 * P_ATM, 5 * P_ATM])
    cfg = dict(energy=1, t_end=0.05, atol=1e-10, rtol=1e-8, ign_mode="TIFP", profile=prof)
    Y0 = ch4_air_Y(mech, 1.0)
    res = dm.reactor_run(_native.make_cfg(**cfg), np.array([1], np.int32), [1300.0], [P_ATM], [1.0], Y0)
    r, Ye = oracle.reactor(1300.0, P_ATM, 1.0, Y0[0], problem=1, **cfg)
    assert r.status == 0 and int(res["stats"][0, 6]) == 0
    assert abs(res["tau"][0].item() / r.tau - 1) < 1e-6
    assert abs(res["P"][0].item() / (5 * P_ATM) - 1) < 1e-12


def test_save_points_match_oracle_dense_output(dm, oracle, mech):
    from pychemkin_amd import _native

    ts = np.linspace(0.0, 2e-3, 41)
    cfg = dict(energy=1, t_end=2e-3, atol=1e-12, rtol=1e-8, ign_mode="TIFP")
    Y0 = ch4_air_Y(mech, 1.0)
    res = dm.reactor_run(_native.make_cfg(**cfg), np.array([1], np.int32), [1500.0], [10 * P_ATM], [1.0], Y0, t_save=ts)
    _, _, (_, ys, _, _) = oracle.reactor(1500.0, 10 * P_ATM, 1.0, Y0[0], t_save=ts, problem=1, **cfg)
    got = res["y_save"][0].cpu().numpy()
    assert np.max(np.abs(got[:, 0] / ys[:, 0] - 1)) < 1e-6
    assert np.max(np.abs(got[:, 1:] - ys[:, 1:])) < 1e-6


def test_determinism_and_batch_order_invariance(dm, mech):
    from pychemkin_amd import _native

    import bench

    T0, P0, Y0, _ = bench.sweep(mech, 1, 0, nT=8, nphi=4, nP=4)
    n = T0.size
    cfg = _native.make_cfg(**bench.RUN)
    prob = np.ones(n, np.int32)
    a = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0).items()}
    b = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0).items()}
    perm = np.random.default_rng(1).permutation(n)
    c = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, prob, T0[perm], P0[perm], np.ones(n), Y0[perm]).items()}
    for k in ("tau", "T", "Y", "stats"):
        assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(a[k][perm], c[k]), k


def test_sweep_properties_at_scale(dm, mech):
    """Size-independent properties on 4096 reactors (a 1/16 slice of the bench sweep)."""
    from pychemkin_amd import _native

    import bench

    T0, P0, Y0, _ = bench.sweep(mech, 1, 0, nT=16, nphi=16, nP=16)
    n = T0.size
    res = {k: v.cpu().numpy() for k, v in dm.reactor_run(_native.make_cfg(**bench.RUN), np.ones(n, np.int32), T0, P0,
                                                          np.ones(n), Y0).items()}
    assert np.all(res["stats"][:, 6] == 0)
    assert np.all(res["tau"] > 0) and np.all(res["tau"] < 1.0)
    assert np.all(res["T"] > T0 + 300.0)
    assert np.allclose(res["Y"].sum(axis=1), 1.0, atol=1e-7)
    ncf = mech.ncf.astype(float)
    e0 = (Y0 / mech.wt) @ ncf.T
    e1 = (res["Y"] / mech.wt) @ ncf.T
    assert np.max(np.abs(e1 - e0) / np.max(e0, axis=1, keepdims=True)) < 1e-7
    tau = res["tau"].reshape(16, 16, 16)  # (T0, phi, P)
    assert np.all(np.diff(np.log(tau), axis=0) < 0)  # hotter ignites sooner (no NTC at 1100-1700 K)
    assert np.all(np.diff(np.log(tau), axis=2) < 0.02)  # higher pressure does not delay (within 2 %)


def test_batch_sweep_api_and_sharding(chem, mech):
    import pychemkin_amd as ck

    T0 = np.linspace(1100, 1600, 12)
    Y0 = ch4_air_Y(mech, 1.0)
    sw = ck.BatchSweep(chem, problem="CONP", energy="ENERGY", t_end=1.0, atol=1e-10, rtol=1e-8)
    r = sw.run(T0, 10 * P_ATM, Y0=Y0)
    assert np.all(r.status == 0) and np.all(np.diff(r.tau) < 0)
    r2 = ck.BatchSweep(chem, problem="CONP", energy="ENERGY", t_end=1.0, atol=1e-10, rtol=1e-8, devices=[0, 0]).run(
        T0, 10 * P_ATM, Y0=Y0)
    assert np.array_equal(r.tau, r2.tau)


def test_invalid_config_fails_loudly(dm, mech):
    from pychemkin_amd import _native

    Y0 = ch4_air_Y(mech, 1.0)
    with pytest.raises(_native.NativeError):
        dm.reactor_run(_native.make_cfg(t_end=-1.0), np.array([1], np.int32), [1200.0], [P_ATM], [1.0], Y0)
    with pytest.raises(_native.NativeError):
        dm.reactor_run(_native.make_cfg(t_end=1.0), np.array([5], np.int32), [1200.0], [P_ATM], [1.0], Y0)


def test_hp_equilibrium_golden_on_gpu(dm, mech, tables):
    """adiabaticflametemperature.baseline through the kernel: 12 adiabatic CONP reactors (one per
    phi = 0.5..1.6) started at the reactants' H and P relax to Chemkin's HP-equilibrium
    temperature (the oracle reproduces it to ~1e-8, test_oracle_golden.py)."""
    from conftest import hp_equilibrium_start
    from pychemkin_amd import _native

    g = golden("adiabaticflametemperature")
    starts = [hp_equilibrium_start(mech, tables, phi) for phi in g["state-equivalence_ratio"]]
    n = len(starts)
    T0 = np.array([s[0] for s in starts])
    Y0 = np.stack([s[1] for s in starts])
    cfg = _native.make_cfg(energy=1, t_end=1.0, atol=1e-14, rtol=1e-9)
    res = dm.reactor_run(cfg, np.ones(n, np.int32), T0, np.full(n, P_ATM), np.ones(n), Y0)
    Tend = res["T"].cpu().numpy()
    assert np.all(res["stats"].cpu().numpy()[:, 6] == 0)
    Tg = np.asarray(g["state-temperature"])
    assert np.all(within(Tend, Tg, *g["tolerance-var"]))
    assert np.max(np.abs(Tend / Tg - 1)) < 1e-7


def test_tp_equilibrium_golden_by_long_given_temperature_runs(dm, mech):
    """equilibriumcomposition.baseline on the GPU: a fixed-T, fixed-P reactor run long enough relaxes
    to the TP equilibrium, so 55 given-temperature CONP reactors (1400..2480 K, 1 atm) end on the
    golden NO mole fractions.  Two launches: 1e4 s from 1700 K up, 1e8 s below (thermal NO is slow
    there; once at equilibrium the step size grows to STPT = t_end / 100 and very long runs pick up
    ~1e-7 of drift, so the hot half stops early -- the oracle's runs land within 4e-9 both ways).
    Below 1400 K the chemistry is too slow even for 1e8 s (NO < 1 ppm there; the Gibbs oracle
    covers the whole range, test_oracle_golden)."""
    from pychemkin_amd import _native

    g = golden("equilibriumcomposition")
    Tg = np.asarray(g["state-temperature"])
    gold_all = np.asarray(g["species-NO_mole_fraction"])
    Xf = np.zeros(mech.KK)
    Xf[mech.species.index("CH4")], Xf[mech.species.index("H2")] = 0.8, 0.2
    Yf = Xf * mech.wt / np.sum(Xf * mech.wt)
    Ya = np.zeros(mech.KK)
    Ya[mech.species.index("O2")], Ya[mech.species.index("N2")] = 0.23, 0.77
    Ymix = (Yf + 17.19 * Ya) / 18.19
    iNO = mech.species.index("NO")
    for sel, t_end in (((Tg >= 1400.0) & (Tg < 1700.0), 1.0e8), (Tg >= 1700.0, 1.0e4)):
        T0 = Tg[sel]
        n = T0.size
        cfg = _native.make_cfg(energy=2, t_end=t_end, atol=1e-20, rtol=1e-10)
        res = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, np.ones(n, np.int32), T0, np.full(n, P_ATM),
                                                              np.ones(n), np.tile(Ymix, (n, 1))).items()}
        assert np.all(res["stats"][:, 6] == 0)
        X = res["Y"] / mech.wt
        X /= X.sum(axis=1, keepdims=True)
        no = X[:, iNO] * 1e6
        gold = gold_all[sel]
        assert np.all(within(no, gold, *g["tolerance-frac"])), (T0, no / gold - 1)
        assert np.max(np.abs(no / gold - 1)) < 1e-6


@pytest.mark.parametrize("path", [0, 1])  # 0: wave kernel; 1: workgroup kernel forced
def test_hot_run_above_the_fit_range_is_not_a_runaway(mech, path):
    """Round-4 advice: with every NASA-7 fit capped at 3,000 K, stoichiometric H2/O2 at constant volume ends
    near 3,900 K with status 0 in both kernels (guard at 2 max_k T_high), at the oracle's end state."""
    from oracle.oracle import Oracle
    from pychemkin_amd import _native
    from test_engine import _CappedFits, hot_h2_o2

    m = _CappedFits(mech, 3000.0)
    dm = _native.DeviceMechanism(m.to_tables())
    T0, P0, Y0 = hot_h2_o2(mech)
    run = dict(energy=1, t_end=1e-3, atol=1e-12, rtol=1e-8)
    _native.set_reactor_path(path)
    try:
        res = {k: v.cpu().numpy() for k, v in dm.reactor_run(_native.make_cfg(**run), np.array([2], np.int32),
                                                             np.array([T0]), np.array([P0]), np.array([1.0]),
                                                             Y0[None]).items()}
    finally:
        _native.set_reactor_path(0)
    r, _ = Oracle(m).reactor(T0, P0, 1.0, Y0, problem=2, **run)
    assert res["stats"][0, 6] == 0 and r.status == 0
    assert res["T"][0] > 3000.0 and abs(res["T"][0] / r.T - 1) < 1e-6


def test_dropin_mole_fraction_mode_and_full_keyword_mode(chem, mech):
    """setsolutionspeciesfracmode("mole") (reactormodel.py:1816): the species profiles and solution mixtures
    are X_k = Y_k Wbar / W_k of the mass-mode run (1e-15); usefullkeywords(True) (reactormodel.py:814): the
    same run through the full-keyword input path (KINAll0D_CalculateInput) gives the same trajectory."""
    import pychemkin_amd as ck

    def h2(mode=None, full=False):
        m = ck.Mixture(chem)
        m.X = [("H2", 2.0), ("O2", 1.0), ("N2", 3.76)]
        m.temperature = 1000.0
        m.pressure = P_ATM
        r = ck.GivenPressureBatchReactor_EnergyConservation(m, label="tran")
        r.time = 5e-4
        r.tolerances = (1e-20, 1e-8)
        r.force_nonnegative = True
        r.timestep_for_saving_solution = 5e-4 / 100
        r.set_ignition_delay(method="T_rise", val=400)
        if mode:
            r.setsolutionspeciesfracmode(mode)
        if full:
            r.usefullkeywords(True)
        try:
            assert r.run() == 0
        finally:
            r.usefullkeywords(False)
        r.process_solution()
        return r

    rm, rx = h2(), h2("mole")
    Y = np.stack([rm.get_solution_variable_profile(s) for s in chem.species_symbols], axis=1)
    X = np.stack([rx.get_solution_variable_profile(s) for s in chem.species_symbols], axis=1)
    Wbar = 1.0 / np.sum(Y / mech.wt, axis=1, keepdims=True)
    assert np.max(np.abs(X - Y * Wbar / mech.wt)) < 1e-15
    for i in (0, 40, 100):
        assert np.max(np.abs(rx.get_solution_mixture_at_index(i).X - rm.get_solution_mixture_at_index(i).X)) < 1e-15
    rf = h2(full=True)
    T = rm.get_solution_variable_profile("temperature")
    Tf = rf.get_solution_variable_profile("temperature")
    assert rf.get_solution_variable_profile("time").tolist() == rm.get_solution_variable_profile("time").tolist()
    assert np.allclose(Tf, T, rtol=1e-9, atol=0)  # REAC mole fractions -> Y: last-bit differences only
    assert abs(rf.get_ignition_delay() / rm.get_ignition_delay() - 1) < 1e-9
