"""Single-zone IC engines on the GPU (problem 4 of ckmi_reactor_run, the wave-per-reactor kernel):
batches of cylinders against the oracle, the drop-in HCCIengine through hcciengine.py line for line
against the golden, and the workgroup kernel's refusal."""
import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y, golden, within
from test_engine import ENG, P_IVC, T_IVC, charge_Y, engine_block, golden_times, tran_fits

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ht", [False, True])
def test_engine_batch_matches_oracle(tables, oracle, mech, ht):
    import torch

    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    cases = [(447.0, 1.065, 0.8), (500.0, 1.5, 0.5), (420.0, 2.0, 1.0), (470.0, 1.0, 0.35)]
    T0 = np.array([c[0] for c in cases])
    P0 = np.array([c[1] for c in cases]) * P_ATM
    Y0 = np.stack([ch4_air_Y(mech, c[2])[0] for c in cases])
    eng = engine_block(ht=ht)
    tf = tran_fits(mech)
    ca, ts = golden_times()
    ts = ts[::8]
    run = dict(energy=1, t_end=ts[-1], atol=1e-12, rtol=1e-9, nneg=True, ign_mode="TIFP")
    tran = torch.tensor(tf, dtype=torch.float64, device=dm.device) if ht else None
    res = {k: v.cpu().numpy() for k, v in
           dm.reactor_run(_native.make_cfg(engine=eng, tran=tran, **run), np.full(len(cases), 4, np.int32),
                          T0, P0, np.ones(len(cases)), Y0, t_save=ts).items()}
    for i in range(len(cases)):
        r, Ye, (_, ys, ps, vs) = oracle.reactor(T0[i], P0[i], 1.0, Y0[i], t_save=ts, problem=4, engine=eng,
                                                tran=tf if ht else None, **run)
        assert r.status == 0 and res["stats"][i, 6] == 0
        assert abs(res["V"][i] / r.V - 1) < 1e-13
        assert abs(res["T"][i] / r.T - 1) < 1e-5 and abs(res["P"][i] / r.P - 1) < 1e-5
        if r.tau > 0:
            assert abs(res["tau"][i] / r.tau - 1) < 1e-4
        assert np.max(np.abs(res["y_save"][i][:, 0] / ys[:, 0] - 1)) < 1e-4


def test_hcci_golden_through_drop_in(chem_tran, mech, oracle):
    """hcciengine.py:63-236 through the drop-in HCCIengine (the charge composed as in test_engine)."""
    import pychemkin_amd as ck
    from pychemkin_amd.engines.HCCI import HCCIengine

    fresh = ck.Mixture(chem_tran)
    fresh.temperature, fresh.pressure = T_IVC, P_IVC
    fresh.Y = charge_Y(mech)
    e = HCCIengine(reactor_condition=fresh, nzones=1)
    e.bore, e.stroke, e.connecting_rod_length = ENG["bore"], ENG["stroke"], ENG["rod"]
    e.compression_ratio, e.RPM = ENG["cr"], ENG["rpm"]
    e.set_piston_pin_offset(offset=ENG["polen"])
    e.starting_CA, e.ending_CA = ENG["ca0"], ENG["ca1"]
    e.set_wall_heat_transfer("dimensionless", list(ENG["ht"]), ENG["twall"])
    e.set_gas_velocity_correlation(list(ENG["gvel"]))
    e.set_piston_head_area(area=ENG["pis"])
    e.set_cylinder_head_area(area=ENG["cyl"])
    e.CAstep_for_saving_solution = 0.5
    e.CAstep_for_printing_solution = 10.0
    e.adaptive_solution_saving(mode=False, steps=20)
    e.tolerances = (1.0e-12, 1.0e-10)
    e.force_nonnegative = True
    e.set_ignition_delay(method="T_inflection")
    assert e.run() == 0
    delayCA = e.get_ignition_delay()
    HR10, HR50, HR90 = e.get_engine_heat_release_CAs()
    assert e.starting_CA < HR10 < HR50 < HR90 < e.ending_CA
    e.process_engine_solution()
    n = e.getnumbersolutionpoints()
    t = e.get_solution_variable_profile("time")
    CA = np.array([e.get_CA(x) for x in t])
    pres = e.get_solution_variable_profile("pressure") * 1e-6
    vol = e.get_solution_variable_profile("volume")
    den = np.array([e.get_solution_mixture_at_index(solution_index=i).RHO for i in range(n)])
    g = golden("hcciengine")
    assert n == 517 and np.allclose(CA, g["state-crank_angle"], rtol=0, atol=1e-9)
    assert np.max(np.abs(vol / np.asarray(g["state-volume"]) - 1)) < 1e-13
    assert np.max(np.abs(den / np.asarray(g["state-density"]) - 1)) < 1e-7
    Pg = np.asarray(g["state-pressure"])
    ok = within(pres, Pg, *g["tolerance-var"])
    # measured, as the oracle (test_engine.py): the first 58 points and 59 in all; the peak 2 CA late
    assert ok[:58].all() and ok.sum() == 59
    assert abs(np.argmax(pres) - np.argmax(Pg)) * 0.5 == 2.0
    assert abs(delayCA - CA[np.argmax(Pg)]) < 3.0
    # heat-release rates (round-4 verdict: no silent zeros): the apparent heat release of the integrator's
    # RHS peaks within 2 CA of the golden's pressure peak, the constant-gamma P-V form agrees on where,
    # the wall loses heat to the 400 K liner over the hot part of the cycle
    hr = e.get_engine_heat_release_rates()
    assert np.allclose(hr["CA"], CA, rtol=0, atol=1e-9)
    ca_pk = CA[np.argmax(hr["AHRR"])]
    assert abs(ca_pk - CA[np.argmax(Pg)]) <= 2.0
    assert abs(CA[np.argmax(hr["AHRRP"])] - ca_pk) <= 1.0
    assert HR10 - 1.0 <= ca_pk <= HR90 + 1.0
    assert hr["AHRR"].max() > 0 and hr["QLossRateCA"].max() > 0
    q = hr["QLossRateCA"]
    assert q[np.argmax(pres)] > 0.0 and np.all(np.isfinite(q))
    # first law of the closed cylinder on the saved points (trapezoids on the 0.5 CA grid):
    #   m [u(T, Y)_end - u(T, Y)_0] + int P dV + int Qloss = 0
    T = e.get_solution_variable_profile("temperature")
    Ys = np.stack([e.get_solution_mixture_at_index(solution_index=i).Y for i in range(n)])
    P = pres * 1e6
    m = den[0] * vol[0]
    uk = np.stack([chem_tran.SpeciesU(x) for x in T]) / chem_tran.WT  # erg/g
    U = m * np.sum(Ys * uk, axis=1)
    scale = np.trapezoid(np.abs(P * np.gradient(vol, CA)), CA)
    first_law = (U[-1] - U[0] + np.trapezoid(P, vol) + np.trapezoid(q, CA)) / scale
    # and pointwise: the apparent heat release m c_v dT/dCA + P dV/dCA of the device RHS plus the wall loss is the
    # chemical heat release rate -m sum_k u_k dY_k/dCA, dY_k/dt = wdot_k W_k / rho from the oracle's rates at the
    # saved state (the cycle integral of AHRR is not a usable check: the ignition spike is narrower than the
    # 0.5 CA grid the profile is sampled on)
    pts = sorted(set(range(0, n, 16)) | {int(np.argmax(hr["AHRR"]))})
    chem = np.array([-m * np.sum(uk[i] * oracle.rates(T[i], P[i], Ys[i])[2] * chem_tran.WT) / den[i] / e.degpersec
                     for i in pts])
    dev = (hr["AHRR"] + q)[pts]
    err = np.max(np.abs(dev - chem)) / np.max(np.abs(chem))
    print("first law: cycle balance %.3e of int|P dV|; AHRR + Qloss vs chemical heat release: %.3e of its peak"
          % (first_law, err))
    assert abs(first_law) < 1e-2
    assert err < 1e-6
    # the golden's Cp column (CPBL kJ/(mol K)) on all 517 points: the first 181 and 186 in all (oracle alike)
    cp = np.array([e.get_solution_mixture_at_index(solution_index=i).CPBL() for i in range(n)]) * 1e-10
    okc = within(cp, np.asarray(g["state-Cp"]), *g["tolerance-var"])
    assert okc[:181].all() and okc.sum() == 186


def test_engine_refused_above_63_species(big_mech):
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(big_mech.to_tables())
    Y0 = np.zeros((1, big_mech.KK))
    Y0[0, big_mech.species.index("N2")] = 1.0
    with pytest.raises(_native.NativeError, match="problem 4"):
        dm.reactor_run(_native.make_cfg(energy=1, t_end=1e-3, engine=engine_block(ht=False)), np.array([4], np.int32),
                       np.array([450.0]), np.array([P_ATM]), np.ones(1), Y0)


def test_hcci_golden_through_kin_calls(mech, oracle):
    """HCCI.py:1058-1239 through the KIN ABI alone: KINPreProcess (itran = 1) -> KINAll0D_Setup (type 4,
    ICEN) -> KINAll0D_SetupHCCIInputs -> the engine keywords (POLEN, ICHX, GVEL, CYBAR, PSBAR, DEGSAVE)
    -> KINAll0D_Calculate -> KINAll0D_GetGasSolnResponse / KINAll0D_GetEngineHeatRelease."""
    import ctypes as ct

    from conftest import CHEM, THERM, TRAN
    from pychemkin_amd import kin

    L = kin.bind()
    cs = ct.c_int(0)
    z, one = ct.c_int(0), ct.c_int(1)
    names = [CHEM, "", THERM, TRAN, "chem.asc", "surf.asc", "tran.asc", ""]
    assert L.KINPreProcess(ct.byref(z), ct.byref(one), *[ct.c_char_p(x.encode()) for x in names], ct.byref(cs)) == 0, \
        kin.last_error()
    try:
        i = lambda v: ct.byref(ct.c_int(v))  # noqa: E731
        d = lambda v: ct.byref(ct.c_double(v))  # noqa: E731
        assert L.KINAll0D_Setup(ct.byref(cs), i(4), i(3), i(1), i(1), i(1), np.zeros(1, np.int32), i(1)) == 0, \
            kin.last_error()
        Y0 = charge_Y(mech)
        a = ENG["stroke"] / 2
        assert L.KINAll0D_SetupHCCIInputs(ct.byref(cs), d(ENG["ca0"]), d(ENG["ca1"]), d(ENG["rpm"]), d(ENG["cr"]),
                                          d(ENG["bore"]), d(ENG["stroke"]), d(ENG["rod"] / a), d(T_IVC), d(P_IVC),
                                          d(0.0), Y0) == 0, kin.last_error()
        ab = np.pi * ENG["bore"] ** 2 / 4
        lines = [f"POLEN    {ENG['polen']}", "ICHX    0.035    0.71    0.0    400.0", "GVEL    2.28    0.308    3.24    0.0",
                 f"CYBAR    {ENG['cyl'] / ab}", f"PSBAR    {ENG['pis'] / ab}", "DEGSAVE    0.5", "DEGPRINT    10.0",
                 "ATOL    1e-12", "RTOL    1e-10", "NNEG", "TIFP"]
        for line in lines:
            assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
        assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, kin.last_error()
        nr, npts = ct.c_int(0), ct.c_int(0)
        assert L.KINAll0D_GetSolnResponseSize(ct.byref(nr), ct.byref(npts)) == 0
        n = npts.value
        t, T, P, V = (np.zeros(n) for _ in range(4))
        Y = np.zeros((mech.KK, n), order="F")
        assert L.KINAll0D_GetGasSolnResponse(ct.byref(nr), ct.byref(npts), i(mech.KK), t, T, P, V, Y) == 0
        g = golden("hcciengine")
        assert n == 517 and np.allclose(ENG["ca0"] + t * 6.0 * ENG["rpm"], g["state-crank_angle"], rtol=0, atol=1e-9)
        assert np.max(np.abs(V / np.asarray(g["state-volume"]) - 1)) < 1e-13
        rho = P / (8.31447247e7 * T) / np.sum(Y.T / mech.wt, axis=1)
        assert np.max(np.abs(rho / np.asarray(g["state-density"]) - 1)) < 1e-7
        ok = within(P * 1e-6, np.asarray(g["state-pressure"]), *g["tolerance-var"])
        assert ok[:58].all() and ok.sum() == 59  # as the drop-in and the oracle
        hr = [ct.c_double(0.0) for _ in range(6)]
        q = np.zeros(1)
        assert L.KINAll0D_GetEngineHeatRelease(q, *[ct.byref(x) for x in hr[1:]]) == 0
        assert ENG["ca0"] < hr[3].value < hr[4].value < hr[5].value < ENG["ca1"]
        # peak rates per CA (erg/degree), not silent zeros: AHRRP restated here from the returned P and V
        # (numpy central differences, gamma of the charge); the instantaneous AHRR of the device RHS peaks
        # above the grid-resolved AHRRP (the ignition front is narrower than the 0.5 CA save step); the
        # wall loss is positive and far below the heat-release peak
        ahrr, ahrrp = hr[1].value, hr[2].value
        CAg = ENG["ca0"] + t * 6.0 * ENG["rpm"]
        cpR = oracle.thermo(T[0])[0]
        Y0 = Y[:, 0]
        cpm = np.sum(Y0 * cpR / mech.wt)
        gam = cpm / (cpm - np.sum(Y0 / mech.wt))
        ap = gam / (gam - 1) * P * np.gradient(V, CAg) + V * np.gradient(P, CAg) / (gam - 1)
        assert abs(ahrrp / ap.max() - 1) < 1e-6
        assert ahrr > 0.5 * ahrrp > 0.0
        assert 0.0 < q[0] < 1e-2 * ahrr
        print("KIN engine heat release: AHRR %.4e AHRRP %.4e QLOSS %.4e erg/deg" % (ahrr, ahrrp, q[0]))
    finally:
        kin.release(cs.value)


def test_cold_lean_cylinders_with_nneg(tables, oracle, mech):
    """Non-igniting cold / lean cylinders of the bench sweep (T_IVC 420-437 K), ICHX heat transfer, with NNEG
    as the reference's HCCI example sets it: every one completes and ends at the oracle's state.  (Without
    NNEG, at the bench's rtol 1e-8 / atol 1e-10, 3-4 of 15,625 such cylinders run away through negative
    trace concentrations in the expansion stroke -- the oracle too at slightly different rtol)"""
    import torch

    import bench
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    T0, P0, Y0 = bench.model_sweep(mech, 1, 0, 16 ** 3 * 4, 420.0, 520.0, P_ATM, 2 * P_ATM, 0.3, 1.0)
    idx = [378, 389, 1738, 1815, 2903]
    tf = tran_fits(mech)
    run = dict(bench.RUN, t_end=258.0 / 6000.0, nneg=True)
    res = {k: v.cpu().numpy() for k, v in dm.reactor_run(
        _native.make_cfg(engine=bench.hcci_block(), tran=torch.tensor(tf, dtype=torch.float64, device=dm.device), **run),
        np.full(len(idx), 4, np.int32), T0[idx], P0[idx], np.ones(len(idx)), Y0[idx]).items()}
    for j, i in enumerate(idx):
        r, _ = oracle.reactor(T0[i], P0[i], 1.0, Y0[i], problem=4, engine=bench.hcci_block(), tran=tf, **run)
        assert r.status == 0 and res["stats"][j, 6] == 0
        assert abs(res["T"][j] / r.T - 1) < 1e-5 and abs(res["P"][j] / r.P - 1) < 1e-5


def test_cold_lean_cylinders_without_nneg_fail_fast(tables, oracle, mech):
    """The same five cylinders without NNEG (round-3 verdict): those that run away end at once with
    CKMI_RUN_RUNAWAY (status 4) instead of burning up to 200,000 steps, on the GPU and in the oracle; the
    rest complete.  Every cylinder stops within 2,000 steps (the oracle finishes the healthy ones in ~530)."""
    import torch

    import bench
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    T0, P0, Y0 = bench.model_sweep(mech, 1, 0, 16 ** 3 * 4, 420.0, 520.0, P_ATM, 2 * P_ATM, 0.3, 1.0)
    idx = [378, 389, 1738, 1815, 2903]
    tf = tran_fits(mech)
    run = dict(bench.RUN, t_end=258.0 / 6000.0)
    res = {k: v.cpu().numpy() for k, v in dm.reactor_run(
        _native.make_cfg(engine=bench.hcci_block(), tran=torch.tensor(tf, dtype=torch.float64, device=dm.device), **run),
        np.full(len(idx), 4, np.int32), T0[idx], P0[idx], np.ones(len(idx)), Y0[idx]).items()}
    st = res["stats"]
    assert set(st[:, 6].tolist()) <= {0, 4}, st[:, 6]
    assert st[:, 0].max() < 2000, st[:, 0]
    for j, i in enumerate(idx):
        if st[j, 6] == 4:  # ended in the physical domain's neighbourhood, not at 10,000 K
            assert res["T"][j] < 1000.0 and res["Y"][j].min() > -0.01
        else:
            r, _ = oracle.reactor(T0[i], P0[i], 1.0, Y0[i], problem=4, engine=bench.hcci_block(), tran=tf, **run)
            if r.status == 0:
                assert abs(res["T"][j] / r.T - 1) < 1e-4
    # the oracle's own runaway (cylinder 389 at rtol 9.13e-9) ends with the same status
    r, Y = oracle.reactor(T0[389], P0[389], 1.0, Y0[389], problem=4, engine=bench.hcci_block(), tran=tf,
                          **dict(run, rtol=9.13e-9))
    assert r.status == 4 and r.nst < 1000 and Y.min() > -0.01
