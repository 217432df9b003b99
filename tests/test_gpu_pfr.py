"""Plug-flow reactors on the GPU (problem 3 of ckmi_reactor_run): the reference's plugflow golden through
the drop-in PlugFlowReactor_FixedTemperature and through KIN calls alone, and batches of tubes
(fixed-T and adiabatic, wave kernel and workgroup kernel) against the oracle."""
import ctypes as ct

import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y, golden
from test_pfr import DIAM, FEED, LENGTH, P_IN, T_IN, U_IN, check_plugflow_golden, feed_Y

pytestmark = pytest.mark.gpu


def test_plugflow_golden_through_drop_in(chem, mech):
    """plugflow.py:38-110 line for line."""
    import pychemkin_amd as ck
    from pychemkin_amd.flowreactors.PFR import PlugFlowReactor_FixedTemperature

    feed = ck.Stream(chem)
    feed.temperature = T_IN
    feed.pressure = P_IN
    feed.X = FEED
    feed.velocity = U_IN
    tube = PlugFlowReactor_FixedTemperature(feed)
    tube.diameter = DIAM
    tube.length = LENGTH
    assert abs(tube.velocity - U_IN) < 1e-12
    tube.timestep_for_saving_solution = 0.0005
    tube.adaptive_solution_saving(mode=False, steps=100)
    assert tube.run() == 0
    tube.process_solution()
    n = tube.getnumbersolutionpoints()
    x = tube.get_solution_variable_profile("time")
    T = tube.get_solution_variable_profile("temperature")
    ratio = tube.mass_flowrate / tube.flowarea
    mixes = [tube.get_solution_mixture_at_index(solution_index=i) for i in range(n)]
    u = np.array([ratio / m.RHO for m in mixes])
    Y = np.array([m.Y for m in mixes])
    check_plugflow_golden(mech, x, T, Y, u)


def test_plugflow_golden_through_kin_calls(mech):
    """PFR.py:440-624 through the KIN ABI: KINAll0D_Setup (type 3) -> KINAll0D_SetupPFRInputs -> keywords
    -> KINAll0D_Calculate -> KINAll0D_GetGasSolnResponse."""
    from pychemkin_amd import kin

    L = kin.bind()
    cs = ct.c_int(kin.register(mech))
    try:
        i = lambda v: ct.byref(ct.c_int(v))  # noqa: E731
        d = lambda v: ct.byref(ct.c_double(v))  # noqa: E731
        assert L.KINAll0D_Setup(ct.byref(cs), i(3), i(1), i(2), i(1), i(1), np.zeros(1, np.int32), i(0)) == 0
        Y0 = feed_Y(mech)
        from pychemkin_amd.constants import R_GAS

        rho = P_IN / (R_GAS * T_IN) / np.sum(Y0 / mech.wt)  # the engine's gas constant
        mdot = rho * np.pi * DIAM ** 2 / 4 * U_IN
        assert L.KINAll0D_SetupPFRInputs(ct.byref(cs), d(0.0), d(LENGTH), d(T_IN), d(P_IN), d(0.0), d(DIAM),
                                         np.zeros(1), np.zeros(1), d(mdot), Y0) == 0, kin.last_error()
        for line in ("RTIME    ON", "MOMEN    ON", "DTSV    0.0005", "ATOL    1e-12", "RTOL    1e-06"):
            assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
        assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, kin.last_error()
        nr, npts = ct.c_int(0), ct.c_int(0)
        assert L.KINAll0D_GetSolnResponseSize(ct.byref(nr), ct.byref(npts)) == 0
        n = npts.value
        x, T, P, V = (np.zeros(n) for _ in range(4))
        Y = np.zeros((mech.KK, n), order="F")
        assert L.KINAll0D_GetGasSolnResponse(ct.byref(nr), ct.byref(npts), i(mech.KK), x, T, P, V, Y) == 0
        check_plugflow_golden(mech, x, T, Y.T, V)
    finally:
        kin.release(cs.value)


def test_kin_tube_from_x0_with_pressure_profile(mech):
    """Round-4 advice: the KIN path's P and V columns of a tube that starts at x0 > 0 under a PPRO profile
    are the profile at the absolute positions and the inlet mass flux over the local density (what the kernel
    integrated, ckmi_kin.cpp Reactor0D post-processing)."""
    from pychemkin_amd import kin
    from pychemkin_amd.constants import R_GAS

    x0, xend = 1.0, 4.0
    px = np.array([0.0, 1.0, 2.0, 4.0])
    pv = P_IN * np.array([1.0, 0.9, 0.8, 0.7])
    L = kin.bind()
    cs = ct.c_int(kin.register(mech))
    try:
        i = lambda v: ct.byref(ct.c_int(v))  # noqa: E731
        d = lambda v: ct.byref(ct.c_double(v))  # noqa: E731
        assert L.KINAll0D_Setup(ct.byref(cs), i(3), i(1), i(2), i(1), i(1), np.zeros(1, np.int32), i(0)) == 0
        Y0 = feed_Y(mech)
        rho_in = P_IN / (R_GAS * T_IN) / np.sum(Y0 / mech.wt)
        mdot = rho_in * np.pi * DIAM ** 2 / 4 * U_IN
        assert L.KINAll0D_SetupPFRInputs(ct.byref(cs), d(x0), d(xend), d(T_IN), d(P_IN), d(0.0), d(DIAM),
                                         np.zeros(1), np.zeros(1), d(mdot), Y0) == 0, kin.last_error()
        assert L.KINAll0D_SetProfileParameter(b"PPRO", i(len(px)), px, pv) == 0, kin.last_error()
        for line in ("DTSV    0.01", "ATOL    1e-12", "RTOL    1e-08"):
            assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
        assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, kin.last_error()
        nr, npts = ct.c_int(0), ct.c_int(0)
        assert L.KINAll0D_GetSolnResponseSize(ct.byref(nr), ct.byref(npts)) == 0
        n = npts.value
        x, T, P, V = (np.zeros(n) for _ in range(4))
        Y = np.zeros((mech.KK, n), order="F")
        assert L.KINAll0D_GetGasSolnResponse(ct.byref(nr), ct.byref(npts), i(mech.KK), x, T, P, V, Y) == 0
    finally:
        kin.release(cs.value)
    # output positions are absolute (x0 + the integration variable), increasing, up to about the tube's end
    assert abs(x[0] - x0) < 1e-12 and np.all(np.diff(x) > 0) and xend - 0.1 < x[-1] < xend + 0.1
    np.testing.assert_allclose(P, np.interp(x, px, pv), rtol=1e-12)  # the profile at absolute positions
    rho = P / (R_GAS * T) / np.sum(Y / mech.wt[:, None], axis=0)
    np.testing.assert_allclose(V, rho_in * U_IN / rho, rtol=1e-10)  # inlet mass flux / local density
    assert abs(T[-1] / T_IN - 1) < 1e-12  # fixed-temperature tube
    assert np.all(np.isfinite(Y)) and abs(np.sum(Y[:, -1]) - 1) < 1e-8


@pytest.mark.parametrize("path", [0, 1])  # 0: wave kernel; 1: workgroup kernel forced
def test_tube_batches_match_oracle(dm_gri, oracle, mech, path):
    """CH4/air tubes, fixed T and adiabatic, different inlet velocities and pressures in one launch."""
    from pychemkin_amd import _native

    cases = [(1300.0, 1.0, 1.0, 50.0), (1500.0, 5.0, 0.7, 200.0), (1250.0, 20.0, 1.2, 10.0), (1700.0, 0.5, 1.0, 900.0)]
    T0 = np.array([c[0] for c in cases])
    P0 = np.array([c[1] for c in cases]) * P_ATM
    Y0 = np.stack([ch4_air_Y(mech, c[2])[0] for c in cases])
    u0 = np.array([c[3] for c in cases])
    prob = np.full(len(cases), 3, np.int32)
    xs = np.linspace(0.0, 30.0, 31)
    for energy in (1, 2):
        run = dict(energy=energy, t_end=30.0, atol=1e-12, rtol=1e-8, ign_mode="TIFP" if energy == 1 else None)
        _native.set_reactor_path(path)
        try:
            res = {k: v.cpu().numpy() for k, v in
                   dm_gri.reactor_run(_native.make_cfg(**run), prob, T0, P0, u0, Y0, t_save=xs).items()}
        finally:
            _native.set_reactor_path(0)
        for i in range(len(cases)):
            r, Ye, (_, ys, ps, vs) = oracle.reactor(T0[i], P0[i], u0[i], Y0[i], t_save=xs, problem=3, **run)
            assert r.status == 0 and res["stats"][i, 6] == 0
            assert abs(res["T"][i] / r.T - 1) < 1e-6
            assert abs(res["V"][i] / r.V - 1) < 1e-6 and abs(res["P"][i] / r.P - 1) < 1e-9
            if energy == 1 and r.tau > 0:
                assert abs(res["tau"][i] / r.tau - 1) < 1e-4
            ysg = res["y_save"][i]
            assert np.max(np.abs(ysg[:, 0] / ys[:, 0] - 1)) < 1e-5
            for sp in ("CH4", "O2", "H2O", "CO2", "CO"):
                k = mech.species.index(sp)
                assert np.max(np.abs(ysg[:, 1 + k] - ys[:, 1 + k])) <= 1e-4 * max(np.max(np.abs(ys[:, 1 + k])), 1e-3)


@pytest.fixture(scope="module")
def dm_gri(tables):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(tables)


def test_big_mechanism_tube(big_mech):
    """A 161-species tube on the workgroup-per-reactor kernel against the oracle."""
    from oracle.oracle import Oracle
    from pychemkin_amd import _native

    orc = Oracle(big_mech)
    dm = _native.DeviceMechanism(big_mech.to_tables())
    X = np.zeros(big_mech.KK)
    X[big_mech.species.index("CH4")] = 1.0
    X[big_mech.species.index("O2")] = 2.0
    X[big_mech.species.index("N2")] = 7.52
    Y0 = X * big_mech.wt
    Y0 /= Y0.sum()
    run = dict(energy=1, t_end=20.0, atol=1e-12, rtol=1e-8, ign_mode="TIFP")
    res = {k: v.cpu().numpy() for k, v in dm.reactor_run(_native.make_cfg(**run), np.array([3], np.int32),
                                                          np.array([1400.0]), np.array([2 * P_ATM]),
                                                          np.array([100.0]), Y0[None]).items()}
    r, Ye = orc.reactor(1400.0, 2 * P_ATM, 100.0, Y0, problem=3, **run)
    assert r.status == 0 and res["stats"][0, 6] == 0
    assert abs(res["tau"][0] / r.tau - 1) < 1e-4 and abs(res["T"][0] / r.T - 1) < 1e-5
    assert abs(res["V"][0] / r.V - 1) < 1e-5


def test_start_position_with_pressure_profile(chem):
    """Round-3 advice: a tube that starts at x0 > 0 reads its PPRO profile at absolute positions, and its mass
    flux is the inlet's (mdot / A) whatever PPRO(x0) is.  A tube from x0 = 1 cm with P(x) equals a tube from 0
    with the profile shifted by -x0; both end at the pressure the profile gives at the absolute end."""
    import pychemkin_amd as ck
    from pychemkin_amd.flowreactors.PFR import PlugFlowReactor_FixedTemperature

    def tube(x0, px, pv):
        feed = ck.Stream(chem)
        feed.temperature = T_IN
        feed.pressure = P_IN
        feed.X = FEED
        feed.velocity = U_IN
        t = PlugFlowReactor_FixedTemperature(feed)
        t.diameter = DIAM
        t.length = 3.0 + x0
        if x0 > 0.0:
            t.set_start_position(x0)
        t.set_pressure_profile(px, pv)
        t.timestep_for_saving_solution = 0.01
        assert t.run() == 0
        return t

    px = np.array([0.0, 1.0, 2.0, 4.0])
    pv = P_IN * np.array([1.0, 0.9, 0.8, 0.7])
    a = tube(1.0, px, pv)
    b = tube(0.0, px - 1.0, pv)
    assert abs(a._final["P"] / (P_IN * 0.7) - 1) < 1e-12  # P(4 cm) of the absolute profile
    assert abs(a._final["P"] / b._final["P"] - 1) < 1e-12
    assert abs(a._final["T"] / b._final["T"] - 1) < 1e-12
    assert np.max(np.abs(a._final["Y"] - b._final["Y"])) < 1e-12
    # the outlet velocity is mdot / (rho A): the inlet's mass flux at the outlet density
    rho_out = a._final["P"] / (ck.constants.R_GAS * a._final["T"]) / np.sum(a._final["Y"] / chem.WT)
    rho_in = P_IN / (ck.constants.R_GAS * T_IN) / np.sum(a.reactormixture.Y / chem.WT)
    assert abs(a._final["V"] / (rho_in * U_IN / rho_out) - 1) < 1e-10


@pytest.mark.parametrize("path", [0, 1])  # 0: wave kernel; 1: workgroup kernel forced
def test_choked_tube_ends_with_status_5(dm_gri, oracle, mech, path):
    """A tube driven past the choke point of the momentum equation ends with CKMI_RUN_CHOKED (5) in both
    kernels, at the oracle's stop position and state; a slower tube in the same launch runs to the end."""
    from pychemkin_amd import _native
    from test_pfr import choked_tube

    T0, P0, u0, Y0, W0 = choked_tube(mech)
    run = dict(energy=1, t_end=300.0, atol=1e-12, rtol=1e-8)
    _native.set_reactor_path(path)
    try:
        res = {k: v.cpu().numpy() for k, v in dm_gri.reactor_run(
            _native.make_cfg(**run), np.array([3, 3], np.int32), np.array([T0, T0]), np.array([P0, P0]),
            np.array([u0, 0.5 * u0]), np.stack([Y0, Y0])).items()}
    finally:
        _native.set_reactor_path(0)
    assert list(res["stats"][:, 6]) == [5, 0]
    r, Ye = oracle.reactor(T0, P0, u0, Y0, problem=3, **run)
    assert r.status == 5
    assert abs(res["t_stop"][0] / r.t_end - 1) < 1e-3
    assert abs(res["T"][0] / r.T - 1) < 1e-3
    assert np.all(np.isfinite(res["P"])) and np.all(np.isfinite(res["V"]))
