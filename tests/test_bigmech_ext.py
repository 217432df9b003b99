"""The extended 161-species stand-in (data/gri30_tracer161_ext_chem.inp: PLOG, chemically activated,
FORD / RORD and fractional-coefficient reactions, several with species indices > 63) on the CPU:
the C oracle against its numpy restatement, and the oracle's BDF on the reactor cases of
tests/test_gpu_bigmech_ext.py (every case finishes; a fractional order on a fast exchange is
integrated without the step-size lock the round-3 chord-slope Jacobian showed)."""
import os

import numpy as np

from conftest import P_ATM, ROOT

CHEM = os.path.join(ROOT, "data", "gri30_tracer161_ext_chem.inp")
THERM = os.path.join(ROOT, "data", "gri30_tracer161_thermo.dat")


def _mech():
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism.from_files(CHEM, THERM)


def test_ext_oracle_matches_numpy():
    from oracle.numpy_ref import NumpyKinetics
    from oracle.oracle import Oracle

    m = _mech()
    orc, nk = Oracle(m), NumpyKinetics(m.to_tables())
    rng = np.random.default_rng(9)
    for _ in range(6):
        T, P = rng.uniform(700.0, 2600.0), P_ATM * 10.0 ** rng.uniform(-1.5, 2.0)
        Y = rng.dirichlet(np.ones(m.KK))
        qf, qr, w = orc.rates(T, P, Y)
        qf2, qr2, w2 = nk.rates(T, P, Y)
        assert np.allclose(qf, qf2, rtol=1e-10, atol=1e-300)
        assert np.allclose(qr, qr2, rtol=1e-10, atol=1e-300)
        assert np.max(np.abs(w - w2)) <= 1e-10 * np.max(np.abs(w2))


def test_ext_oracle_reactors_finish():
    from oracle.oracle import Oracle
    from test_gpu_bigmech_ext import _Y

    m = _mech()
    orc = Oracle(m)
    rng = np.random.default_rng(6)
    n = 4
    T0 = rng.uniform(1250.0, 1650.0, n)
    P0 = P_ATM * rng.uniform(0.5, 60.0, n)
    Y0 = _Y(m, rng.uniform(0.5, 1.5, n))
    nf, res, _ = orc.reactor_batch(T0, P0, Y0, problem=np.array([1, 2, 1, 2], np.int32), V0=np.ones(n), nthreads=4,
                                   energy=1, t_end=0.02, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    assert nf == 0
    assert all(r.status == 0 and r.tau > 0 and r.nst < 4000 for r in res), [(r.status, r.nst) for r in res]
