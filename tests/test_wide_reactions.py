"""Reactions with more than four distinct species on a side (up to CKMI_SLOTS = 8).

Round 2 stored four species per side and rejected wider reactions.  The slot width is now 8; a
reaction with more than four distinct species on a side is a general reaction (RX_GEN: its
stoichiometry and orders come from the per-reaction slot record, ckmi_image.hpp eval_gen_img) in
every kernel -- the wave-per-reactor kernel, the workgroup kernel, the ROP kernels and the
mechanism-specialised ROP kernel.  No mechanism in the reference uses such reactions, so the stand-in
is GRI-3.0 plus two balanced lumped steps (5 reactants; one reversible with 3 products).  Parity
with Chemkin is unpinned (no golden); the oracle is checked against its numpy restatement and
finite differences, the GPU against the oracle.  The 161-species case (6 species per side) is in
tests/test_gpu_bigmech_ext.py."""
import os

import numpy as np
import pytest

from conftest import P_ATM, ROOT, THERM, ch4_air_Y

GRI = os.path.join(ROOT, "data", "grimech30_chem.inp")
WIDE = ["CH4+O2+H+O+OH=>CO+2H2O+OH+H                1.000E+33    0.000    2000.00",
        "CH3+HCO+OH+H+O<=>C2H6+O2+O                 1.000E+33    0.000       0.00"]


def _text(lines):
    text = open(GRI).read()
    end = text.rstrip().rfind("END")
    return text[:end] + "\n".join(lines) + "\nEND\n"


@pytest.fixture(scope="module")
def wmech():
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism(_text(WIDE), open(THERM).read())


@pytest.fixture(scope="module")
def worc(wmech):
    from oracle.oracle import Oracle

    return Oracle(wmech)


def test_wide_tables(wmech):
    t = wmech.to_tables()
    assert t["rsp"].shape[1] == 8
    assert t["nr"][-2:].tolist() == [5, 5] and t["np"][-2:].tolist() == [4, 3]
    assert t["rev"][-2:].tolist() == [0, 1]


def test_wide_rate_is_the_mass_action_product(wmech, worc):
    rng = np.random.default_rng(3)
    T, P = 1500.0, 2 * P_ATM
    Y = rng.dirichlet(np.ones(wmech.KK))
    RU = 1.3806504e-16 * 6.02214179e23
    C = P / (RU * T) * (Y / wmech.wt) / np.sum(Y / wmech.wt)
    qf, qr, _ = worc.rates(T, P, Y)
    sp = wmech.species.index
    k = 1e33 * np.exp(-2000.0 / (8.314510e7 / 4.184e7 * T))
    prod = C[sp("CH4")] * C[sp("O2")] * C[sp("H")] * C[sp("O")] * C[sp("OH")]
    assert abs(qf[-2] / (k * prod) - 1) < 1e-12 and qr[-2] == 0.0
    assert qr[-1] > 0


def test_wide_oracle_matches_numpy(wmech, worc):
    from oracle.numpy_ref import NumpyKinetics

    nk = NumpyKinetics(wmech.to_tables())
    rng = np.random.default_rng(9)
    for _ in range(10):
        T, P = rng.uniform(500.0, 3000.0), P_ATM * 10.0 ** rng.uniform(-1.5, 1.5)
        Y = rng.dirichlet(np.ones(wmech.KK))
        qf, qr, w = worc.rates(T, P, Y)
        qf2, qr2, w2 = nk.rates(T, P, Y)
        assert np.allclose(qf, qf2, rtol=1e-11, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))


@pytest.mark.parametrize("which", [0, 1])
def test_wide_oracle_jacobian(which):
    """The analytic Jacobian of a single wide reaction against central differences (all columns)."""
    from oracle.oracle import Oracle
    from pychemkin_amd.mechanism import Mechanism

    import re

    text = open(GRI).read()
    r0 = re.search(r"^REACTIONS", text, re.M | re.I).start()
    m = Mechanism(text[:r0] + "REACTIONS\n" + WIDE[which] + "\nEND\n", open(THERM).read())
    assert m.II == 1
    orc = Oracle(m)
    Y0 = np.random.default_rng(which).dirichlet(np.ones(m.KK))
    T = 1600.0
    y = np.concatenate([[T], Y0])
    RU = 1.3806504e-16 * 6.02214179e23
    rho0 = 5 * P_ATM / (RU * T) / np.sum(Y0 / m.wt)
    kw = dict(problem=2, energy=1, rho0=rho0, V0=1.0, P0=5 * P_ATM)
    f, J = orc.rhs_jac(y, **kw)
    for j in [m.species.index(s) + 1 for s in ("CH4", "O2", "H", "O", "OH", "CH3", "HCO", "C2H6")]:
        h = 1e-7 * max(abs(y[j]), 1e-3)
        yp, ym = y.copy(), y.copy()
        yp[j] += h
        ym[j] -= h
        fd = (orc.rhs_jac(yp, **kw)[0] - orc.rhs_jac(ym, **kw)[0]) / (2 * h)
        sc = max(np.max(np.abs(fd[1:])), 1e-300)
        assert np.max(np.abs(J[1:, j] - fd[1:])) < 1e-5 * sc, j


# ------------------------------------------------------------------ GPU


@pytest.fixture(scope="module")
def wdm(wmech):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(wmech.to_tables())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 64, 20000])  # small n: the mechanism-specialised kernel; 20,000: generic
def test_gpu_wide_rop(wmech, worc, wdm, n):
    rng = np.random.default_rng(n)
    T = rng.uniform(500.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-1.5, 1.5, n)
    Y = rng.dirichlet(np.ones(wmech.KK), n).T.copy()
    w = wdm.rop_thermo(T, P, Y)[0].cpu().numpy()
    m = min(n, 256)
    wo = worc.rop_batch(T[:m], P[:m], np.ascontiguousarray(Y[:, :m]))[0]
    assert np.max(np.abs(w[:, :m] - wo) / np.max(np.abs(wo), axis=0, keepdims=True)) < 1e-11


@pytest.mark.gpu
def test_gpu_wide_reaction_rates(wmech, worc, wdm):
    rng = np.random.default_rng(1)
    n = 16
    T = rng.uniform(500.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-1.5, 1.5, n)
    Y = rng.dirichlet(np.ones(wmech.KK), n).T.copy()
    qf, qr = (x.cpu().numpy() for x in wdm.reaction_rates(T, P, Y))
    for j in range(n):
        qfo, qro, _ = worc.rates(T[j], P[j], Y[:, j])
        sc = max(np.max(np.abs(qfo)), np.max(np.abs(qro)))
        assert np.max(np.abs(qf[:, j] - qfo)) < 1e-11 * sc
        assert np.max(np.abs(qr[:, j] - qro)) < 1e-11 * sc


@pytest.mark.gpu
@pytest.mark.parametrize("path", [0, 1])  # 0: wave kernel (extended variant); 1: workgroup kernel forced
def test_gpu_wide_reactors(wmech, worc, wdm, path):
    from pychemkin_amd import _native

    cases = [(1200, 1, 1.0, 1), (1400, 10, 0.7, 2), (1600, 40, 1.5, 1), (1300, 0.3, 1.0, 2)]
    run = dict(energy=1, t_end=0.2, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    T0 = np.array([c[0] for c in cases], float)
    P0 = np.array([c[1] for c in cases], float) * P_ATM
    Y0 = np.stack([ch4_air_Y(wmech, c[2])[0] for c in cases])
    prob = np.array([c[3] for c in cases], np.int32)
    _native.set_reactor_path(path)
    try:
        res = {k: v.cpu().numpy() for k, v in wdm.reactor_run(_native.make_cfg(**run), prob, T0, P0,
                                                                np.ones(len(cases)), Y0).items()}
    finally:
        _native.set_reactor_path(0)
    for i in range(len(cases)):
        r, Ye = worc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **run)
        assert r.status == 0 and res["stats"][i, 6] == 0
        # tau within 1e-4 of the oracle's own envelope under a +-1 % perturbation of rtol (11 runs): the
        # step sequence of an adaptive BDF is chaotic at rounding level, so the device (another summation
        # order of wdot) lands anywhere the oracle itself lands.  Measured envelopes (rel. to rtol = 1e-8):
        # 1e-6 wide for three cases; -1.7e-4 / +3.8e-4 for the 5.3 us ignition at 1600 K, 40 atm, phi 1.5,
        # whose device tau is 1.5e-4 off the unperturbed oracle run
        env = [worc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **dict(run, rtol=run["rtol"] * f))[0].tau
               for f in np.linspace(0.99, 1.01, 11)]
        assert min(env) * (1 - 1e-4) <= res["tau"][i] <= max(env) * (1 + 1e-4)
        assert abs(res["T"][i] / r.T - 1) < 1e-4
        for sp in ("CH4", "O2", "H2O", "CO2", "CO", "C2H6"):
            k = wmech.species.index(sp)
            assert abs(res["Y"][i, k] - Ye[k]) <= 1e-4 * max(abs(Ye[k]), 1e-3)
