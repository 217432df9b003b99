"""Single-zone IC engine (problem 4; SURVEY.md §8(f) rank 4: HCCI reuse of the batch-reactor ODE
kernel), CPU side: kinematics, the oracle against the reference's hcciengine golden, the conductivity
fits behind the wall heat transfer, and the drop-in HCCIengine's host logic.

Golden case (hcciengine.py:48-176): GRI-3.0, fuel CH4 / C3H8 / C2H6 = 0.9 / 0.05 / 0.05, air, phi 0.8
with 30 % EGR (the equilibrium products of the fresh charge at 447 K, 1.065 atm, threshold 1e-8),
447 K and 1.065 atm at IVC = -142 CA, EVO 116 CA, 1000 RPM, bore 12.065, stroke 14.005, rod 26.0093,
CR 16.5, pin offset -0.5 cm, ICHX 0.035 / 0.71 / 0 with a 400 K wall, Woschni 2.28 / 0.308 / 3.24 / 0,
head areas 123.5 (cylinder) and 124.75 (piston) cm2, saved every 0.5 CA, ATOL 1e-12, RTOL 1e-10, NNEG.
"""
import numpy as np
import pytest

from conftest import P_ATM, TRAN, golden, within

T_IVC, P_IVC = 447.0, 1.065 * P_ATM
ENG = dict(ca0=-142.0, ca1=116.0, rpm=1000.0, cr=16.5, bore=12.065, stroke=14.005, rod=26.0093, polen=-0.5,
           ht=(0.035, 0.71, 0.0), twall=400.0, gvel=(2.28, 0.308, 3.24, 0.0), cyl=123.5, pis=124.75)


def engine_block(ht=True):
    ab = np.pi * ENG["bore"] ** 2 / 4
    e = np.zeros(20)
    e[:7] = [ENG["ca0"], ENG["rpm"], ENG["cr"], ENG["bore"], ENG["stroke"], ENG["rod"] / (ENG["stroke"] / 2),
             ENG["polen"]]
    if ht:
        e[7] = 1.0
        e[8:11] = ENG["ht"]
        e[11] = ENG["twall"]
        e[12:16] = ENG["gvel"]
        e[16], e[17] = ENG["cyl"] / ab, ENG["pis"] / ab
    return e


def golden_times():
    ca = np.asarray(golden("hcciengine")["state-crank_angle"])
    return ca, (ca - ENG["ca0"]) / (6.0 * ENG["rpm"])


def charge_Y(mech):
    """The golden's fresh charge with EGR (hcciengine.py:63-110), mass fractions."""
    from oracle.equilibrium import TPEquilibrium
    from oracle.oracle import Oracle

    sp = mech.species
    KK = mech.KK

    def vec(pairs):
        x = np.zeros(KK)
        for s, v in pairs:
            x[sp.index(s)] = v
        return x

    fuel = vec([("CH4", 0.9), ("C3H8", 0.05), ("C2H6", 0.05)])
    oxid = vec([("O2", 0.21), ("N2", 0.79)])
    A = mech.ncf.astype(float)
    el = mech.elements
    o2 = A[el.index("C")] @ fuel + A[el.index("H")] @ fuel / 4 - A[el.index("O")] @ fuel / 2
    alpha = o2 / oxid[sp.index("O2")]

    def x_by_phi(add, thr):  # mixture.py X_by_Equivalence_Ratio (products CO2, H2O, N2)
        add = np.where(add < thr, 0.0, add)
        x = 0.8 * fuel + alpha * oxid
        x /= x.sum()
        return x * (1 - add.sum()) + add if add.sum() > 0 else x

    x0 = x_by_phi(np.zeros(KK), 1e-10)
    Y0 = x0 * mech.wt
    Y0 /= Y0.sum()
    eq = TPEquilibrium(mech, Oracle(mech).thermo)
    for Tq in (2500.0, 2000.0, 1500.0, 1200.0, 1000.0, 800.0, 650.0, 550.0, 480.0, T_IVC):  # continuation
        xe = eq.solve(Tq, P_IVC / P_ATM, Y0)
    egr = np.where(xe > 1e-8, 0.3 * xe, 0.0)  # get_EGR_mole_fraction(0.3, threshold=1e-8)
    x1 = x_by_phi(egr, 1e-8)
    Y1 = x1 * mech.wt
    return Y1 / Y1.sum()


def tran_fits(mech):
    from oracle import transport_ref as tr
    P = tr.parse_transport(open(TRAN).read())
    params = [P[s] for s in mech.species]
    th = mech.to_tables()["thermo"]
    return np.hstack([tr.viscosity_fits(mech.wt, params, 3500.0), tr.conductivity_fits(mech.wt, params, th, 3500.0)])


@pytest.fixture(scope="module")
def hcci_oracle_run(oracle, mech):
    ca, ts = golden_times()
    Y0 = charge_Y(mech)
    res, _, (t, ys, ps, vs) = oracle.reactor(T_IVC, P_IVC, 1.0, Y0, t_save=ts, problem=4, energy=1, t_end=ts[-1],
                                             atol=1e-12, rtol=1e-10, nneg=True, ign_mode="TIFP",
                                             engine=engine_block(), tran=tran_fits(mech))
    return res, ys, ps, vs, Y0


def test_engine_volume_matches_golden():
    from pychemkin_amd.engines.HCCI import engine_volume

    ca, ts = golden_times()
    V = engine_volume(engine_block(), ts)
    assert np.max(np.abs(V / np.asarray(golden("hcciengine")["state-volume"]) - 1)) < 1e-13
    # zero offset: the textbook slider-crank
    e = engine_block()
    e[6] = 0.0
    R = ENG["rod"] / (ENG["stroke"] / 2)
    th = np.radians(ca)
    Vd = np.pi * ENG["bore"] ** 2 / 4 * ENG["stroke"]
    Vtb = Vd / (ENG["cr"] - 1) * (1 + (ENG["cr"] - 1) / 2 * (R + 1 - np.cos(th) - np.sqrt(R * R - np.sin(th) ** 2)))
    assert np.allclose(engine_volume(e, ts), Vtb, rtol=1e-13)


def test_oracle_engine_against_golden(hcci_oracle_run, mech):
    res, ys, ps, vs, Y0 = hcci_oracle_run
    g = golden("hcciengine")
    assert res.status == 0
    assert np.max(np.abs(vs / np.asarray(g["state-volume"]) - 1)) < 1e-13
    rho = ps / (8.31447247e7 * ys[:, 0]) / np.sum(ys[:, 1:] / mech.wt, axis=1)
    # mass / V: the charge (fuel, air, 30 % EGR at equilibrium) and its density are the golden's
    assert np.max(np.abs(rho / np.asarray(g["state-density"]) - 1)) < 1e-7
    Pg = np.asarray(g["state-pressure"])
    p = ps * 1e-6
    ok = within(p, Pg, *g["tolerance-var"])
    # pressure (measured, film-temperature properties): within the golden's tolerance on exactly the first
    # 58 points and one more (-142 ... -113.5 CA), then the residual of the heat-transfer coefficient shows
    # (the golden's h is 0.888 x this form, uniformly: test_golden_heat_loss_is_a_uniform_multiple); the
    # pressure peak comes 2 CA late (11.5 vs 9.5 CA)
    assert ok[:58].all() and ok.sum() == 59
    assert abs(np.argmax(p) - np.argmax(Pg)) * 0.5 == 2.0
    assert abs(p.max() / Pg.max() - 1) < 0.15
    # the golden's Cp column (CPBL [kJ/mol-K]) on all 517 points: the first 181 (to -52 CA) and 186 in all
    cp_R = np.array([np.sum(ys[i, 1:] / mech.wt * _cpR(mech, ys[i, 0])) for i in range(len(ys))])
    cp = cp_R * 8.31447247 / np.sum(ys[:, 1:] / mech.wt, axis=1) * 1e-3
    okc = within(cp, np.asarray(g["state-Cp"]), *g["tolerance-var"])
    assert okc[:181].all() and okc.sum() == 186


def test_golden_heat_loss_is_a_uniform_multiple(mech):
    """The hcciengine golden's own wall heat loss, backed out of its P / rho / V / Cp columns before the
    low-temperature chemistry (-134 ... -90 CA; frozen charge, so T = P Wbar / (rho R) and the golden's Cp
    column reproduces to 1e-15 at that T), is a constant multiple of the ICHX / Woschni h A (T - Twall)
    with mu and lambda at the film temperature (T + Twall) / 2: the same factor on the head and the liner
    area, relative spread < 1e-3; with bulk-temperature properties the ratio drifts with T (spread 7e-3).
    The factor itself, 0.888, is the unexplained residual; scripts/hcci_golden_heat.py."""
    from oracle import transport_ref as trf
    from oracle.oracle import Oracle
    from pychemkin_amd.constants import R_GAS

    orc = Oracle(mech)
    Y = charge_Y(mech)
    Wbar = 1.0 / np.sum(Y / mech.wt)
    X = Y / mech.wt * Wbar
    g = golden("hcciengine")
    ca = np.asarray(g["state-crank_angle"])
    P, rho, V = (np.asarray(g[k]) for k in ("state-pressure", "state-density", "state-volume"))
    P = P * 1e6
    T = P * Wbar / (rho * R_GAS)
    cp_mol = R_GAS * np.array([orc.thermo(t)[0] for t in T]) @ X
    sel = (ca >= -134) & (ca <= -90)
    assert np.max(np.abs(cp_mol[sel] * 1e-10 / np.asarray(g["state-Cp"])[sel] - 1)) < 1e-13
    e = engine_block()
    t = (ca - ca[0]) / (6 * ENG["rpm"])
    Q = -(rho[0] * V[0] * (cp_mol - R_GAS) / Wbar * np.gradient(T, t) + P * np.gradient(V, t))
    params = trf.parse_transport(open(TRAN).read())
    pl = [params[s] for s in mech.species]
    vf, cf = trf.viscosity_fits(mech.wt, pl, 3500.0), trf.conductivity_fits(mech.wt, pl, mech.to_tables()["thermo"], 3500.0)
    B, Tw = ENG["bore"], ENG["twall"]
    Ab = np.pi * B * B / 4
    a, L, ee = ENG["stroke"] / 2, ENG["rod"], -ENG["polen"]
    Vc = Ab * (np.sqrt((L + a) ** 2 - ee ** 2) - np.sqrt((L - a) ** 2 - ee ** 2)) / (ENG["cr"] - 1)
    w = ENG["gvel"][0] * 2 * ENG["stroke"] * ENG["rpm"] / 60  # P = P_motored before ignition
    head, liner = np.full_like(T, (e[16] + e[17]) * Ab), np.pi * B * (V - Vc) / Ab

    def h_of(Tp):
        mu = trf.mixture_viscosity(Tp, np.tile(X, (len(Tp), 1)), mech.wt, vf)
        lam = trf.mixture_conductivity(Tp, np.tile(X, (len(Tp), 1)), cf)
        return ENG["ht"][0] * (rho * w * B / mu) ** ENG["ht"][1] * lam / B

    for Tp, spread in ((0.5 * (T + Tw), 1e-3), (T, 5e-3)):
        Aeff = (Q / (h_of(Tp) * (T - Tw)))[sel]
        r = Aeff / (head + liner)[sel]
        if spread < 2e-3:
            assert r.std() / r.mean() < spread and abs(r.mean() - 0.888) < 2e-3
            coef = np.linalg.lstsq(np.stack([head[sel], liner[sel]], 1), Aeff, rcond=None)[0]
            assert np.all(np.abs(coef - 0.888) < 5e-3)  # head and liner alike: not an area form
        else:
            assert r.std() / r.mean() > spread


def _cpR(mech, T):
    th = mech.to_tables()["thermo"]
    a = np.where(T > th[:, 1:2], th[:, 10:15], th[:, 3:8])
    return a[:, 0] + T * (a[:, 1] + T * (a[:, 2] + T * (a[:, 3] + T * a[:, 4])))


def test_oracle_engine_heat_loss_bracket(oracle, mech):
    """The golden lies between the adiabatic cylinder and the one with wall heat transfer (compression)."""
    ca, ts = golden_times()
    Y0 = charge_Y(mech)
    tq = ts[:100]
    kw = dict(problem=4, energy=1, t_end=tq[-1], atol=1e-12, rtol=1e-10, nneg=True)
    _, _, (_, _, pa, _) = oracle.reactor(T_IVC, P_IVC, 1.0, Y0, t_save=tq, engine=engine_block(ht=False), **kw)
    _, _, (_, _, ph, _) = oracle.reactor(T_IVC, P_IVC, 1.0, Y0, t_save=tq, engine=engine_block(),
                                         tran=tran_fits(mech), **kw)
    Pg = np.asarray(golden("hcciengine")["state-pressure"])[:100] * 1e6
    assert np.all(ph[1:] < Pg[1:]) and np.all(Pg[1:] < pa[1:])


def test_oracle_engine_adiabatic_compression_is_isentropic(oracle, mech):
    """Frozen chemistry (GFAC 1e-30), no wall heat: the mixture entropy stays constant along the stroke."""
    Y0 = charge_Y(mech)
    ts = np.linspace(0.0, 0.02, 41)  # -142 .. -22 CA
    _, _, (_, ys, ps, _) = oracle.reactor(T_IVC, P_IVC, 1.0, Y0, t_save=ts, problem=4, energy=1, t_end=ts[-1],
                                          atol=1e-14, rtol=1e-12, gfac=1e-30, engine=engine_block(ht=False))
    X = Y0 / mech.wt
    X /= X.sum()
    nz = X > 0
    s = []
    for i in range(len(ts)):
        _, _, sR = oracle.thermo(ys[i, 0])
        s.append(np.sum(X[nz] * (sR[nz] - np.log(X[nz] * ps[i] / P_ATM))))
    s = np.asarray(s)
    assert np.max(np.abs(s / s[0] - 1)) < 1e-9
    assert ys[-1, 0] > T_IVC + 300.0


def test_conductivity_fits_native_vs_numpy_and_golden(chem_tran, mech):
    from oracle import transport_ref as tr
    P = tr.parse_transport(open(TRAN).read())
    ref = tr.conductivity_fits(mech.wt, [P[s] for s in mech.species], mech.to_tables()["thermo"], 3500.0)
    assert np.max(np.abs(chem_tran.conductivity_fits - ref)) < 1e-9
    g = golden("speciesproperties")  # species conductivity of N2 (speciesproperties.py:106-121)
    k = chem_tran.get_specindex("N2")
    c = chem_tran.conductivity_fits[k]  # the fit evaluated here; the device evaluation is test_gpu_transport's
    x = np.log(np.asarray(g["state-temperature"]))
    lam = np.exp(c[0] + x * (c[1] + x * (c[2] + x * c[3]))) * 1e-7  # J/(cm s K)
    gl = np.asarray(g["state-conductivity"])
    # Warnatz form + Neufeld Omega(1,1)*: 2.2e-3 at most (Chemkin's tabulated collision integrals are
    # not restated); within the golden's tolerance (1e-6 J/(cm s K) + 1e-4) on 79 of 100 points
    assert np.max(np.abs(lam / gl - 1)) < 2.5e-3
    assert within(lam, gl, *g["tolerance-var"]).sum() >= 79


def test_hcci_host_setup(chem_tran):
    import pychemkin_amd as ck
    from pychemkin_amd.engines import HCCIengine
    from pychemkin_amd.reactormodel import ReactorError

    m = ck.Mixture(chem_tran)
    m.temperature, m.pressure = T_IVC, P_IVC
    m.X = [("CH4", 1.0), ("O2", 2.0), ("N2", 7.52)]
    with pytest.raises(ReactorError, match="multi-zone"):
        HCCIengine(m, nzones=2)
    e = HCCIengine(reactor_condition=m, nzones=1)
    with pytest.raises(ReactorError, match="missing"):
        e.validate_inputs()
    e.bore, e.stroke, e.connecting_rod_length = ENG["bore"], ENG["stroke"], ENG["rod"]
    e.compression_ratio, e.RPM = ENG["cr"], ENG["rpm"]
    e.set_piston_pin_offset(offset=ENG["polen"])
    e.starting_CA, e.ending_CA = ENG["ca0"], ENG["ca1"]
    assert e.validate_inputs() == 0
    with pytest.raises(ReactorError, match="not on the device path"):
        e.set_wall_heat_transfer("hohenburg", [1, 2, 3, 4, 5], 400.0)
    e.set_wall_heat_transfer("dimensionless", list(ENG["ht"]), ENG["twall"])
    e.set_gas_velocity_correlation(list(ENG["gvel"]))
    e.set_piston_head_area(area=ENG["pis"])
    e.set_cylinder_head_area(area=ENG["cyl"])
    assert np.allclose(e.engine_block(), engine_block(), rtol=1e-15)
    e.CAstep_for_saving_solution = 0.5
    ca, ts = golden_times()
    from pychemkin_amd.batchreactor import save_times

    tg = save_times(e.rundurationCA / e.degpersec, 0.5 / e.degpersec)
    assert len(tg) == len(ca) and np.allclose(e.get_CA(tg), ca, rtol=0, atol=1e-9)
    assert abs(e.get_displacement_volume() - np.pi * ENG["bore"] ** 2 / 4 * ENG["stroke"]) < 1e-12
    assert e.get_number_of_zones() == 1


def test_engine_keywords_in_the_one_keyword_policy():
    """The KIN path's engine keywords (HCCI.py / engine.py write them) are device keywords; DEGPRINT has no
    effect; the multi-zone / other correlations stay rejected."""
    from pychemkin_amd import kin

    for k in ("POLEN", "ICHX", "GVEL", "CYBAR", "PSBAR", "DEGSAVE"):
        assert kin.keyword_class(k) == 1, k
    assert kin.keyword_class("DEGPRINT") == 2
    for k in ("ICHW", "ICHH", "HIMP", "MLMT"):
        assert kin.keyword_class(k) == 0, k


def test_oracle_runaway_guard(mech, oracle):
    """CKMI_RUN_RUNAWAY in the oracle: without NNEG, one of 200 rtol-perturbed runs of the bench's five
    cold-lean cylinders (389 at rtol 9.13e-9 with the Jacobian refreshed every 15 steps; with every 50: 378 at
    1.02e-8; round 3: 389 at 1.062e-8, 8,277 K after 200,000 steps) runs away through negative trace
    concentrations; the guard ends it within ~600 steps at a mass fraction of -1e-3, while the same cylinder
    at rtol 1e-8 completes with status 0."""
    import bench

    T0, P0, Y0 = bench.model_sweep(mech, 1, 0, 16 ** 3 * 4, 420.0, 520.0, P_ATM, 2 * P_ATM, 0.3, 1.0)
    tf = tran_fits(mech)
    run = dict(bench.RUN, t_end=258.0 / 6000.0, problem=4, engine=bench.hcci_block(), tran=tf)
    r, Y = oracle.reactor(T0[389], P0[389], 1.0, Y0[389], **dict(run, rtol=9.13e-9))
    assert r.status == 4 and r.nst < 1000 and -0.01 < Y.min() < -1e-3 and r.T < 1000.0
    r, Y = oracle.reactor(T0[389], P0[389], 1.0, Y0[389], **run)
    assert r.status == 0 and Y.min() > -1e-3


class _CappedFits:
    """A mechanism whose NASA-7 fits all end at `thi` (the upper fit extrapolated beyond it)."""

    def __init__(self, mech, thi):
        self._m, self._thi = mech, thi

    def __getattr__(self, k):
        return getattr(self._m, k)

    def to_tables(self):
        t = dict(self._m.to_tables())
        th = t["thermo"].copy()
        th[:, 2] = np.minimum(th[:, 2], self._thi)
        t["thermo"] = th
        return t


def hot_h2_o2(mech):
    """Stoichiometric H2/O2 at constant volume from 1500 K and 10 atm: its end state is ~3,900 K."""
    Y0 = np.zeros(mech.KK)
    Y0[mech.species.index("H2")] = 2 * 2.016
    Y0[mech.species.index("O2")] = 31.998
    return 1500.0, 10 * P_ATM, Y0 / Y0.sum()


def test_oracle_hot_run_above_the_fit_range_is_not_a_runaway(mech):
    """Round-4 advice: the runaway guard's upper bound is 2 max_k T_high (ckoracle.c, ckmi.hip), so a run that
    legitimately ends above every fit's upper limit (here all fits capped at 3,000 K, the end state ~3,900 K)
    keeps status 0; only a real runaway (8-10k K) trips it."""
    from oracle.oracle import Oracle

    orc = Oracle(_CappedFits(mech, 3000.0))
    T0, P0, Y0 = hot_h2_o2(mech)
    r, Y = orc.reactor(T0, P0, 1.0, Y0, problem=2, energy=1, t_end=1e-3, atol=1e-12, rtol=1e-8)
    assert r.status == 0 and 3000.0 < r.T < 6000.0
