"""The mechanism-specialised ROP kernel (ckmi_jit.cpp: one state per lane, generated from the
mechanism, compiled with hipRTC) against the oracle and the generic kernel.

Same bar as the generic kernel (test_gpu_kernels): wdot within 1e-11 of the largest |wdot| of the
state, cp / h within 1e-12.  The reverse rates use products of exp(+-g_k) instead of exp(dG) per
reaction, so the two GPU kernels agree to rounding, not bitwise."""
import numpy as np
import pytest

from conftest import P_ATM

pytestmark = pytest.mark.gpu


@pytest.fixture
def jit_path():
    from pychemkin_amd import _native

    _native.set_rop_path(2)
    yield
    _native.set_rop_path(0)


def _states(KK, n, seed):
    rng = np.random.default_rng(seed)
    T = rng.uniform(300.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, n)
    Y = rng.dirichlet(0.5 * np.ones(KK), n).T.copy()
    return T, P, Y


def _jit_state(dm):
    import ctypes as ct

    from pychemkin_amd import _native

    st = ct.c_int32(0)
    _native._check(_native.lib().ckmi_rop_jit_state(dm.handle, ct.byref(st)), "ckmi_rop_jit_state")
    return st.value


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097])
def test_jit_rop_matches_oracle(tables, oracle, mech, jit_path, n):
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    T, P, Y = _states(mech.KK, n, seed=100 + n)
    w, cp, h = (x.cpu().numpy() for x in dm.rop_thermo(T, P, Y))
    assert _jit_state(dm) == 1
    wo, cpo, ho = oracle.rop_batch(T, P, Y)
    scale = np.max(np.abs(wo), axis=0, keepdims=True)
    assert np.max(np.abs(w - wo) / scale) < 1e-11
    assert np.max(np.abs(cp / cpo - 1)) < 1e-12
    assert np.max(np.abs(h - ho) / np.max(np.abs(ho))) < 1e-12


def test_jit_matches_generic_kernel_and_sees_afactor(tables, mech):
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    T, P, Y = _states(mech.KK, 20000, seed=7)
    _native.set_rop_path(1)
    wg = dm.rop_thermo(T, P, Y)[0].cpu().numpy()
    _native.set_rop_path(2)
    try:
        wj = dm.rop_thermo(T, P, Y)[0].cpu().numpy()
        scale = np.max(np.abs(wg), axis=0, keepdims=True)
        assert np.max(np.abs(wj - wg) / scale) < 1e-11
        # the A-factor lives in the parameter block: a change is seen without recompiling
        A, b, E = dm.arrhenius()
        dm.set_afactor(37, A[37] * 3.0)
        i0 = int(np.nonzero((b == 0.0) & (E == 0.0))[0][0])  # a k = A reaction (its A is read directly)
        dm.set_afactor(i0, A[i0] * 0.5)
        wj3 = dm.rop_thermo(T, P, Y)[0].cpu().numpy()
        _native.set_rop_path(1)
        wg3 = dm.rop_thermo(T, P, Y)[0].cpu().numpy()
        assert np.max(np.abs(wj3 - wg3) / np.max(np.abs(wg3), axis=0, keepdims=True)) < 1e-11
        assert np.max(np.abs(wj3 - wj)) > 0.0
    finally:
        _native.set_rop_path(0)


def test_jit_zero_and_trace_compositions(tables, oracle, mech, jit_path):
    """Pure species and exact zeros (C_k = 0 in every product) -- the equilibrium factors
    exp(+-g_k) stay finite from 300 to 3500 K."""
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    KK = mech.KK
    T = np.array([300.0, 300.0, 1000.0, 3500.0, 2000.0, 600.0])
    P = np.array([1.0, 100.0, 1.0, 1.0, 0.1, 30.0]) * P_ATM
    Y = np.zeros((KK, T.size))
    Y[mech.species.index("N2"), 0] = 1.0
    Y[mech.species.index("H2"), 1] = 1.0
    Y[:, 2] = 1.0 / KK
    Y[mech.species.index("H"), 3] = 0.5
    Y[mech.species.index("O2"), 3] = 0.5
    Y[mech.species.index("CH4"), 4] = 0.05
    Y[mech.species.index("O2"), 4] = 0.2
    Y[mech.species.index("N2"), 4] = 0.75
    Y[:, 5] = np.linspace(0.0, 1.0, KK)
    Y[:, 5] /= Y[:, 5].sum()
    w = dm.rop_thermo(T, P, Y)[0].cpu().numpy()
    wo, _, _ = oracle.rop_batch(T, P, Y)
    assert np.all(np.isfinite(w))
    scale = np.maximum(np.max(np.abs(wo), axis=0, keepdims=True), 1e-300)
    assert np.max(np.abs(w - wo) / scale) < 1e-11


EXT = {
    "plog": ("gri30_plog_chem.inp", "grimech30_thermo.dat"),
    "cheb": ("gri30_cheb_chem.inp", "grimech30_thermo.dat"),
    "ford": ("gri30_ford_chem.inp", "grimech30_thermo.dat"),
    "ext161": ("gri30_tracer161_ext_chem.inp", "gri30_tracer161_thermo.dat"),
}


@pytest.mark.parametrize("name", sorted(EXT))
def test_jit_every_reaction_form_matches_oracle(jit_path, name):
    """PLOG (bracketing row per lane), Chebyshev, Landau-Teller (+ RLT), chemically activated, FORD /
    RORD / fractional orders (the conc_pow rule) and wide reactions on the specialised kernel: same
    bar as GRI-3.0 (1e-11 of the state's largest |wdot|), including states below the order floor."""
    import os

    from conftest import ROOT
    from oracle.oracle import Oracle

    from pychemkin_amd import _native
    from pychemkin_amd.mechanism import Mechanism

    chem, therm = EXT[name]
    m = Mechanism.from_files(os.path.join(ROOT, "data", chem), os.path.join(ROOT, "data", therm))
    dm = _native.DeviceMechanism(m.to_tables())
    orc = Oracle(m)
    n = 1500
    rng = np.random.default_rng(11)
    T = rng.uniform(300.0, 3000.0, n)
    P = P_ATM * 10.0 ** rng.uniform(-2.5, 2.5, n)  # PLOG / Chebyshev clamps and extrapolation
    Y = rng.dirichlet(0.5 * np.ones(m.KK), n).T.copy()
    Y[:, :200] *= rng.uniform(0.0, 1.0, (m.KK, 200)) < 0.3  # exact zeros: C^o at and below the floor
    Y[:, :200] /= np.maximum(Y[:, :200].sum(axis=0, keepdims=True), 1e-300)
    Y[:, 0] = 0.0
    Y[m.species.index("N2"), 0] = 1.0
    w, cp, h = (x.cpu().numpy() for x in dm.rop_thermo(T, P, Y))
    assert _jit_state(dm) == 1
    wo, cpo, ho = orc.rop_batch(T, P, Y)
    assert np.all(np.isfinite(w))
    scale = np.maximum(np.max(np.abs(wo), axis=0, keepdims=True), 1e-300)
    assert np.max(np.abs(w - wo) / scale) < 1e-11
    assert np.max(np.abs(cp / cpo - 1)) < 1e-12


def test_jit_disabled_fails_loudly_on_forced_path(jit_path, tables, monkeypatch):
    """CKMI_ROP_JIT=0 at mechanism creation: path 2 raises, the automatic path runs the generic kernel."""
    from pychemkin_amd import _native

    monkeypatch.setenv("CKMI_ROP_JIT", "0")
    dm = _native.DeviceMechanism(tables)
    assert _jit_state(dm) == -1
    T, P, Y = _states(int(tables["KK"]), 70000, seed=3)
    with pytest.raises(_native.NativeError, match="CKMI_ROP_JIT"):
        dm.rop_thermo(T, P, Y)
    _native.set_rop_path(0)
    w = dm.rop_thermo(T, P, Y)[0].cpu().numpy()
    assert np.all(np.isfinite(w))


@pytest.mark.skipif(not (__import__("torch").cuda.is_available() and __import__("torch").cuda.device_count() >= 2),
                    reason="needs two GPUs")
def test_jit_module_loads_on_the_mechanism_device(tables, oracle, mech):
    """A mechanism on GPU 1 driven while GPU 0 is current, with a batch large enough for the
    specialised kernel: jit_ready loads the hipRTC module on the mechanism's device (ckmi.hip
    DeviceScope) and the launch runs there, and the caller's current device is left as it was."""
    import torch

    from pychemkin_amd import _native

    torch.cuda.set_device(0)
    dm = _native.DeviceMechanism(tables, device=1)
    n = 20000
    T, P, Y = _states(mech.KK, n, seed=5)
    w = dm.rop_thermo(T, P, Y)[0]
    assert w.device.index == 1 and torch.cuda.current_device() == 0
    assert _jit_state(dm) == 1
    wo = oracle.rop_batch(T[:64], P[:64], Y[:, :64].copy())[0]
    err = np.max(np.abs(w.cpu().numpy()[:, :64] - wo) / np.max(np.abs(wo), axis=0, keepdims=True))
    assert err < 1e-11
    dm.close()
