"""The reference's KIN call sequences on libckmi.so, through the KIN-compatible C ABI only.

Every call here goes through ctypes with the reference's prototypes (pychemkin_amd.kin, restated
from chemkin_wrapper.py) the way mixture.py / chemistry.py / batchreactor.py make them: scalars by
pointer, host numpy arrays, int return.  The goldens are the reference's own example outputs."""
import ctypes as ct

import numpy as np
import pytest

from conftest import P_ATM, check_h2_golden, golden, h2_air_Y, within

pytestmark = pytest.mark.gpu

RU = 1.3806504e-16 * 6.02214179e23


@pytest.fixture(scope="module")
def K(mech):
    from pychemkin_amd import kin

    L = kin.bind()
    cs = kin.register(mech)
    yield L, ct.c_int(cs)
    kin.release(cs)


def _nasa(tables, T):
    th = np.asarray(tables["thermo"])
    a = np.where((T > th[:, 1])[:, None], th[:, 10:17], th[:, 3:10])
    cpR = a[:, 0] + T * (a[:, 1] + T * (a[:, 2] + T * (a[:, 3] + T * a[:, 4])))
    hRT = a[:, 0] + T * (a[:, 1] / 2 + T * (a[:, 2] / 3 + T * (a[:, 3] / 4 + T * a[:, 4] / 5))) + a[:, 5] / T
    return cpR, hRT


def test_sizes_and_tables(K, mech):
    L, cs = K
    s = [ct.c_int(-1) for _ in range(8)]
    assert L.KINGetChemistrySizes(ct.byref(cs), *[ct.byref(x) for x in s]) == 0
    assert [s[0].value, s[1].value, s[2].value] == [mech.MM, mech.KK, mech.II]
    buf = (ct.POINTER(ct.c_char) * mech.KK)()
    for i in range(mech.KK):
        buf[i] = ct.create_string_buffer(17)  # MAX_SPECIES_LENGTH (chemistry.py:42)
    assert L.KINGetGasSpeciesNames(ct.byref(cs), ct.cast(buf, ct.POINTER(ct.POINTER(ct.c_char)))) == 0
    names = [ct.cast(buf[i], ct.c_char_p).value.decode() for i in range(mech.KK)]
    assert names == mech.species
    wt = np.zeros(mech.KK)
    assert L.KINGetGasMolecularWeights(ct.byref(cs), wt) == 0
    assert np.array_equal(wt, mech.wt)
    awt = np.zeros(mech.MM)
    assert L.KINGetAtomicWeights(ct.byref(cs), awt) == 0
    assert np.array_equal(awt, np.asarray(mech.awt))
    ncf = np.zeros((mech.MM, mech.KK), dtype=np.int32, order="F")
    assert L.KINGetGasSpeciesComposition(ct.byref(cs), ncf) == 0
    assert np.array_equal(ncf, mech.ncf)


@pytest.mark.parametrize("T", [300.0, 999.0, 1000.0, 2500.0])
def test_species_thermo_per_mass(K, mech, tables, T):
    L, cs = K
    cp, h, u = (np.zeros(mech.KK) for _ in range(3))
    t = ct.c_double(T)
    assert L.KINGetGasSpecificHeat(ct.byref(cs), ct.byref(t), cp) == 0
    assert L.KINGetGasSpeciesEnthalpy(ct.byref(cs), ct.byref(t), h) == 0
    assert L.KINGetGasSpeciesInternalEnergy(ct.byref(cs), ct.byref(t), u) == 0
    cpR, hRT = _nasa(tables, T)
    r = RU / mech.wt
    assert np.allclose(cp, cpR * r, rtol=1e-12, atol=0)
    assert np.allclose(h, hRT * r * T, rtol=1e-11, atol=1e-3)
    assert np.allclose(u, h - r * T, rtol=1e-11, atol=1e-3)


def test_density_and_mixture_thermo(K, mech, tables):
    L, cs = K
    Y = np.ascontiguousarray(h2_air_Y(mech))
    T, P = ct.c_double(1234.5), ct.c_double(3.0 * P_ATM)
    rho, cp, h = ct.c_double(0), ct.c_double(0), ct.c_double(0)
    assert L.KINGetMassDensity(ct.byref(cs), ct.byref(T), ct.byref(P), Y, ct.byref(rho)) == 0
    assert abs(rho.value / (3.0 * P_ATM / (RU * 1234.5 * np.sum(Y / mech.wt))) - 1) < 1e-14
    assert L.KINGetGasMixtureSpecificHeat(ct.byref(cs), ct.byref(T), Y, ct.byref(cp)) == 0
    assert L.KINGetGasMixtureEnthalpy(ct.byref(cs), ct.byref(T), Y, ct.byref(h)) == 0
    cpR, hRT = _nasa(tables, 1234.5)
    assert abs(cp.value / np.sum(Y * cpR * RU / mech.wt) - 1) < 1e-12
    assert abs(h.value / np.sum(Y * hRT * RU * 1234.5 / mech.wt) - 1) < 1e-11


def test_rop_and_rates_match_batched_kernels(K, mech, tables, oracle):
    from pychemkin_amd import _native

    L, cs = K
    dm = _native.DeviceMechanism(tables)
    rng = np.random.default_rng(3)
    for T_, P_ in ((1500.0, P_ATM), (900.0, 20 * P_ATM)):
        Y = rng.random(mech.KK)
        Y /= Y.sum()
        T, P = ct.c_double(T_), ct.c_double(P_)
        wdot = np.zeros(mech.KK)
        qf, qr = np.zeros(mech.II), np.zeros(mech.II)
        assert L.KINGetGasROP(ct.byref(cs), ct.byref(T), ct.byref(P), Y, wdot) == 0
        assert L.KINGetGasReactionRates(ct.byref(cs), ct.byref(T), ct.byref(P), Y, qf, qr) == 0
        w_b, _, _ = dm.rop_thermo([T_], [P_], Y[:, None])
        y_x = Y * mech.wt / np.sum(Y * mech.wt)  # KINGetGasReactionRates reads mole fractions
        qf_b, qr_b = dm.reaction_rates([T_], [P_], y_x[:, None])
        assert np.array_equal(wdot, w_b.cpu().numpy()[:, 0])  # same kernel, batch of one
        # (host X -> Y conversions may round differently in the last bit)
        assert np.allclose(qf, qf_b.cpu().numpy()[:, 0], rtol=1e-13, atol=0)
        assert np.allclose(qr, qr_b.cpu().numpy()[:, 0], rtol=1e-13, atol=0)
        w_o = oracle.rates(T_, P_, Y)[2]
        scale = np.max(np.abs(w_o))
        assert np.max(np.abs(wdot - w_o)) <= 1e-9 * scale


def test_afactor_get_put_and_rate_parameters(K, mech):
    L, cs = K
    A, b, E = (np.zeros(mech.II) for _ in range(3))
    assert L.KINGetReactionRateParameters(ct.byref(cs), A, b, E) == 0
    i = 37
    a = ct.c_double(0.0)
    assert L.KINSetAFactorForAReaction(ct.byref(cs), ct.byref(ct.c_int(i + 1)), ct.byref(a)) == 0
    assert a.value == A[i]
    a2 = ct.c_double(2.5 * A[i])
    assert L.KINSetAFactorForAReaction(ct.byref(cs), ct.byref(ct.c_int(-(i + 1))), ct.byref(a2)) == 0
    chk = ct.c_double(0.0)
    assert L.KINSetAFactorForAReaction(ct.byref(cs), ct.byref(ct.c_int(i + 1)), ct.byref(chk)) == 0
    assert abs(chk.value / (2.5 * A[i]) - 1) < 1e-14
    a0 = ct.c_double(A[i])
    assert L.KINSetAFactorForAReaction(ct.byref(cs), ct.byref(ct.c_int(-(i + 1))), ct.byref(a0)) == 0
    assert L.KINSetAFactorForAReaction(ct.byref(cs), ct.byref(ct.c_int(mech.II + 1)), ct.byref(chk)) != 0


def _setup(L, cs, problem, energy, t_end, T, P, V, Y):
    assert L.KINAll0D_Setup(ct.byref(cs), ct.byref(ct.c_int(1)), ct.byref(ct.c_int(problem)),
                            ct.byref(ct.c_int(energy)), ct.byref(ct.c_int(1)), ct.byref(ct.c_int(1)),
                            np.zeros(1, np.int32), ct.byref(ct.c_int(0))) == 0
    assert L.KINAll0D_SetupWorkArrays(ct.byref(ct.c_int(6)), ct.byref(cs)) == 0
    z = np.zeros(1)
    assert L.KINAll0D_SetupBatchInputs(ct.byref(cs), ct.byref(ct.c_double(t_end)), ct.byref(ct.c_double(T)),
                                       ct.byref(ct.c_double(P)), ct.byref(ct.c_double(V)), ct.byref(ct.c_double(0)),
                                       ct.byref(ct.c_double(0)), np.ascontiguousarray(Y), z, z) == 0
    if energy == 1:
        assert L.KINAll0D_IntegrateHeatRelease() == 0


def _solution(L, KK):
    nr, npt = ct.c_int(0), ct.c_int(0)
    assert L.KINAll0D_GetSolnResponseSize(ct.byref(nr), ct.byref(npt)) == 0
    n = npt.value
    t, T, P, V = (np.zeros(n) for _ in range(4))
    Y = np.zeros((KK, n), order="F")
    assert L.KINAll0D_GetGasSolnResponse(ct.byref(nr), ct.byref(npt), ct.byref(ct.c_int(KK)), t, T, P, V, Y) == 0
    return t, T, P, V, Y


def test_h2_golden_through_kin_calls(K, mech):
    """closed_homogeneous__transient.py:61-131 as the reference's batchreactor.py drives the native
    library (__process_keywords :980-1147, __run_model :1149-1159, solution :1297-1410)."""
    L, cs = K
    g = golden("closed_homogeneous__transient")
    _setup(L, cs, 1, 1, 5e-4, 1000.0, P_ATM, 1.0, h2_air_Y(mech))
    for line in ("ATOL    1e-20", "RTOL    1e-08", "NNEG", "DTSV    5e-06", "DTIGN    400", "!ADAP", "NADAP"):
        assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
    assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, L.ckmi_kin_last_error()
    tau = ct.c_double(0.0)
    assert L.KINAll0D_GetIgnitionDelay(ct.byref(tau)) == 0
    t, T, P, V, Y = _solution(L, mech.KK)
    Tg = np.asarray(g["state-temperature"])
    assert np.allclose(P, P_ATM, rtol=1e-14)
    assert np.allclose(Y.sum(axis=0), 1.0, atol=1e-10)
    # closed_homogeneous__transient.py:176-181: ROP()[H2O] of each solution mixture, via KINGetGasROP
    k = mech.species.index("H2O")
    wdot = np.zeros(mech.KK)
    rop = np.zeros(len(t))
    for i in range(len(t)):
        assert L.KINGetGasROP(ct.byref(cs), ct.byref(ct.c_double(T[i])), ct.byref(ct.c_double(P[i])),
                              np.ascontiguousarray(Y[:, i]), wdot) == 0
        rop[i] = wdot[k]
    check_h2_golden(g, mech, t, T, Y.T, rop, min_ok=101)
    assert abs(T[-1] / Tg[-1] - 1) < 1e-6
    assert abs(tau.value / np.interp(1400.0, Tg, t) - 1) < 1e-4


def test_conv_volume_profile_golden_through_kin_calls(K, mech, chem, oracle):
    """CONV.py:62-140: CONV + ENERGY with a VPRO profile, TIFP ignition."""
    import pychemkin_amd as ck

    L, cs = K
    g = golden("CONV")
    fuel = ck.Mixture(chem)
    fuel.X = [("CH4", 1.0)]
    air = ck.Mixture(chem)
    air.X = [("O2", 0.21), ("N2", 0.79)]
    m = ck.Mixture(chem)
    m.X_by_Equivalence_Ratio(chem, fuel.X, air.X, np.zeros(chem.KK), ["CO2", "H2O", "N2"], 0.7)
    _setup(L, cs, 2, 1, 0.1, 800.0, 3 * P_ATM, 10.0, m.Y)
    x, v = np.array([0.0, 0.01, 2.0]), np.array([10.0, 4.0, 4.0])
    assert L.KINAll0D_SetProfileParameter(b"VPRO", ct.byref(ct.c_int(3)), x, v) == 0
    for line in ("ATOL    1e-10", "RTOL    1e-08", "NNEG", "DTSV    0.01", "TIFP"):
        assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
    assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, L.ckmi_kin_last_error()
    t, T, P, V, Y = _solution(L, mech.KK)
    assert np.all(within(T, g["state-temperature"], *g["tolerance-var"]))
    assert np.allclose(V, np.interp(t, x, v), rtol=1e-14)
    tau = ct.c_double(0.0)
    assert L.KINAll0D_GetIgnitionDelay(ct.byref(tau)) == 0
    res, _ = oracle.reactor(800.0, 3 * P_ATM, 10.0, m.Y, problem=2, energy=1, t_end=0.1, atol=1e-10, rtol=1e-8,
                            nneg=True, ign_mode="TIFP", profile=(x, v))
    assert abs(tau.value / res.tau - 1) < 1e-6


def test_unknown_and_unsupported_keywords_fail(K, mech):
    L, cs = K
    _setup(L, cs, 1, 1, 1e-3, 1200.0, P_ATM, 1.0, h2_air_Y(mech))
    assert L.KINAll0D_SetUserKeyword(b"BOGUS    3") == 0  # stored; rejected by Calculate
    assert L.KINAll0D_Calculate(ct.byref(cs)) != 0
    assert b"BOGUS" in L.ckmi_kin_last_error()
    _setup(L, cs, 1, 1, 1e-3, 1200.0, P_ATM, 1.0, h2_air_Y(mech))
    assert L.KINAll0D_SetUserKeyword(b"ATOL    abc") == 0
    assert L.KINAll0D_Calculate(ct.byref(cs)) != 0
    _setup(L, cs, 1, 1, 1e-3, 1200.0, P_ATM, 1.0, h2_air_Y(mech))
    x = np.array([0.0, 1.0])
    assert L.KINAll0D_SetProfileParameter(b"VPRO", ct.byref(ct.c_int(2)), x, x + 1) == 0
    assert L.KINAll0D_Calculate(ct.byref(cs)) != 0  # VPRO on a CONP reactor
    assert b"VPRO" in L.ckmi_kin_last_error()


def test_reaction_rates_golden_through_kin_call(K, mech):
    """reactionrates.baseline exactly as the reference produces it: mixture.py:1540 passes the mass
    fractions to KINGetGasReactionRates, which reads them as mole fractions."""
    from conftest import ch4_air_Y

    L, cs = K
    g = golden("reactionrates")
    Y = np.ascontiguousarray(ch4_air_Y(mech, 1.0)[0])
    qf, qr = np.zeros(mech.II), np.zeros(mech.II)
    assert L.KINGetGasReactionRates(ct.byref(cs), ct.byref(ct.c_double(1800.0)), ct.byref(ct.c_double(5 * P_ATM)), Y,
                                    qf, qr) == 0
    net = qf - qr
    nz = np.nonzero(net)[0]
    order = nz[np.argsort(-net[nz], kind="stable")]
    assert order.tolist() == g["state-order_1800"]
    assert np.all(within(net[order], g["rate-net_reaction_rate_1800"], *g["tolerance-ROP"]))


def test_qpro_with_aext_through_kin_calls(K, mech, oracle):
    """set_heat_loss_profile + set_heat_transfer_area_profile together (batchreactor.py:2005-2067,
    QPRO and AEXT through KINAll0D_SetProfileParameter, either order) with HTC / TAMB keywords:
    the heat loss is QPRO(t) + HTC AEXT(t) (T - TAMB); against the oracle."""
    from conftest import ch4_air_Y

    L, cs = K
    Y0 = ch4_air_Y(mech, 1.0)[0]
    xq, vq = np.array([0.0, 0.02]), np.array([0.0, 1.0])
    xa, va = np.array([0.0, 0.01, 0.03]), np.array([2.0, 8.0, 6.0])
    ref, _ = oracle.reactor(1250.0, 2 * P_ATM, 3.0, Y0, problem=1, energy=1, t_end=0.05, atol=1e-10, rtol=1e-8,
                            ign_mode="TIFP", htc=2e-3, tamb=400.0, profile2=(xq, vq), prof2_kind=1,
                            profile3=(xa, va))
    assert ref.status == 0  # the heat loss holds this charge below ignition (tau = -1 on both sides)
    for order in (("QPRO", "AEXT"), ("AEXT", "QPRO")):
        _setup(L, cs, 1, 1, 0.05, 1250.0, 2 * P_ATM, 3.0, Y0)
        for key in order:
            x, v = (xq, vq) if key == "QPRO" else (xa, va)
            assert L.KINAll0D_SetProfileParameter(key.encode(), ct.byref(ct.c_int(len(x))), x, v) == 0
        for line in ("ATOL    1e-10", "RTOL    1e-08", "TIFP", "HTC    2e-3", "TAMB    400"):
            assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
        assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, L.ckmi_kin_last_error()
        tau = ct.c_double(0.0)
        assert L.KINAll0D_GetIgnitionDelay(ct.byref(tau)) == 0
        assert (abs(tau.value / ref.tau - 1) < 1e-4) if ref.tau > 0 else tau.value == ref.tau, order
        t, T, P, V, Y = _solution(L, mech.KK)
        assert abs(T[-1] / ref.T - 1) < 1e-5, order


def _preprocess(L, chem, therm, summary=""):
    """chemistry.py:675-687: KINPreProcess with the reference's argument list (isurf, itran, 8 file
    names, chemset)."""
    cs = ct.c_int(0)
    z = ct.c_int(0)
    names = [chem, "", therm, "", "chem.asc", "surf.asc", "tran.asc", summary]
    rc = L.KINPreProcess(ct.byref(z), ct.byref(z), *[ct.c_char_p(x.encode()) for x in names], ct.byref(cs))
    return rc, cs


def test_preprocess_then_h2_golden_through_kin_calls_only(mech, tmp_path):
    """File paths -> KINPreProcess (native interpreter) -> KINGetChemistrySizes / names / weights
    (chemistry.py:693-1064) -> the closed_homogeneous__transient golden on all five columns, through
    KIN calls alone -- no Python parser, no ckmi_kin_register."""
    from conftest import CHEM, THERM
    from pychemkin_amd import kin

    L = kin.bind()
    summary = str(tmp_path / "Summary.out")
    rc, cs = _preprocess(L, CHEM, THERM, summary)
    assert rc == 0, kin.last_error()
    s = [ct.c_int(-1) for _ in range(8)]
    assert L.KINGetChemistrySizes(ct.byref(cs), *[ct.byref(x) for x in s]) == 0
    assert [s[0].value, s[1].value, s[2].value] == [5, 53, 325]
    buf = (ct.POINTER(ct.c_char) * 53)()
    for i in range(53):
        buf[i] = ct.create_string_buffer(17)
    assert L.KINGetGasSpeciesNames(ct.byref(cs), ct.cast(buf, ct.POINTER(ct.POINTER(ct.c_char)))) == 0
    names = [ct.cast(buf[i], ct.c_char_p).value.decode() for i in range(53)]
    assert names == mech.species
    wt = np.zeros(53)
    assert L.KINGetGasMolecularWeights(ct.byref(cs), wt) == 0 and np.array_equal(wt, mech.wt)
    mode, eos = ct.c_int(-1), ct.create_string_buffer(17)
    assert L.KINRealGas_GetEOSMode(ct.byref(cs), ct.byref(mode), eos) == 0 and mode.value == 0
    assert L.KINRealGas_CheckRealGasStatus(ct.byref(cs), ct.byref(mode)) == 0 and mode.value == 0
    n = ct.c_int(0)
    rs = ct.create_string_buffer(b" " * 1024)
    assert L.KINGetGasReactionString(ct.byref(cs), ct.byref(ct.c_int(38)), ct.byref(n), rs) == 0
    assert rs.raw[:n.value].decode() == "H+O2<=>O+OH"
    assert "H+O2<=>O+OH" in open(summary).read()
    g = golden("closed_homogeneous__transient")
    _setup(L, cs, 1, 1, 5e-4, 1000.0, P_ATM, 1.0, h2_air_Y(mech))
    for line in ("ATOL    1e-20", "RTOL    1e-08", "NNEG", "DTSV    5e-06", "DTIGN    400", "NADAP"):
        assert L.KINAll0D_SetUserKeyword(line.encode()) == 0, line
    assert L.KINAll0D_Calculate(ct.byref(cs)) == 0, kin.last_error()
    t, T, P, V, Y = _solution(L, mech.KK)
    k = mech.species.index("H2O")
    wdot = np.zeros(mech.KK)
    rop = np.zeros(len(t))
    for i in range(len(t)):
        assert L.KINGetGasROP(ct.byref(cs), ct.byref(ct.c_double(T[i])), ct.byref(ct.c_double(P[i])),
                              np.ascontiguousarray(Y[:, i]), wdot) == 0
        rop[i] = wdot[k]
    check_h2_golden(g, mech, t, T, Y.T, rop, min_ok=101)
    kin.release(cs.value)


def test_full_keyword_mode_calculate_input(K, mech):
    """KINAll0D_CalculateInput (chemkin_wrapper.py:690-697): the keyword block the reference builds
    in full-keyword mode (batchreactor.py:822-978: TRAN, CONP, ENRG, PRES [atm], TEMP, TIME, REAC
    lines, solver keywords, QRGEQ, END) gives the same run as API mode -- the H2 golden case."""
    L, cs = K
    g = golden("closed_homogeneous__transient")
    Y0 = h2_air_Y(mech)
    _setup(L, cs, 1, 1, 5e-4, 1000.0, P_ATM, 1.0, Y0)
    X0 = (Y0 / mech.wt) / np.sum(Y0 / mech.wt)
    lines = ["TRAN", "CONP", "ENRG", "PRES    1.0", "TEMP    1000.0", "TIME    0.0005"]
    lines += [f"REAC    {mech.species[k]}    {float(X0[k])!r}" for k in range(mech.KK) if X0[k] > 1e-12]
    lines += ["ATOL    1e-20", "RTOL    1e-08", "NNEG", "DTSV    5e-06", "DTIGN    400", "NADAP", "QRGEQ", "END"]
    blob = "".join(lines).encode()
    lens = np.array([len(x) for x in lines], np.int32)
    assert L.KINAll0D_CalculateInput(ct.byref(ct.c_int(154)), ct.byref(cs), blob, ct.byref(ct.c_int(len(lines))),
                                     lens) == 0, L.ckmi_kin_last_error()
    t, T, P, V, Y = _solution(L, mech.KK)
    tau_full = ct.c_double(0.0)
    assert L.KINAll0D_GetIgnitionDelay(ct.byref(tau_full)) == 0
    Tg = np.asarray(g["state-temperature"])
    assert t.tolist() == g["state-time"]
    assert within(T, Tg, *g["tolerance-var"]).sum() >= 99
    # API mode on the same inputs: the same numbers
    _setup(L, cs, 1, 1, 5e-4, 1000.0, P_ATM, 1.0, Y0)
    for line in ("ATOL    1e-20", "RTOL    1e-08", "NNEG", "DTSV    5e-06", "DTIGN    400", "NADAP"):
        assert L.KINAll0D_SetUserKeyword(line.encode()) == 0
    assert L.KINAll0D_Calculate(ct.byref(cs)) == 0
    t2, T2, P2, V2, Y2 = _solution(L, mech.KK)
    assert np.allclose(T2, T, rtol=1e-9, atol=0)  # REAC mole fractions -> Y: last-bit differences only
    tau = ct.c_double(0.0)
    assert L.KINAll0D_GetIgnitionDelay(ct.byref(tau)) == 0 and abs(tau.value / tau_full.value - 1) < 1e-9
    # an unknown keyword in the block is rejected with a message
    _setup(L, cs, 1, 1, 5e-4, 1000.0, P_ATM, 1.0, Y0)
    bad = ["TRAN", "CONP", "ENRG", "FROB    3", "END"]
    assert L.KINAll0D_CalculateInput(ct.byref(ct.c_int(154)), ct.byref(cs), "".join(bad).encode(),
                                     ct.byref(ct.c_int(len(bad))), np.array([len(x) for x in bad], np.int32)) != 0
    assert b"FROB" in L.ckmi_kin_last_error()
