import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

CHEM = os.path.join(ROOT, "data", "grimech30_chem.inp")
THERM = os.path.join(ROOT, "data", "grimech30_thermo.dat")
TRAN = os.path.join(ROOT, "data", "grimech30_transport.dat")
P_ATM = 1.01325e6


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def golden(name):
    with open(os.path.join(ROOT, "tests", "golden", name + ".json")) as f:
        return json.load(f)


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def mech():
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism.from_files(CHEM, THERM)


@pytest.fixture(scope="session")
def tables(mech):
    return mech.to_tables()


@pytest.fixture(scope="session")
def oracle(mech):
    from oracle.oracle import Oracle

    return Oracle(mech)


@pytest.fixture(scope="session")
def chem():
    import pychemkin_amd as ck

    c = ck.Chemistry(label="GRI 3.0")
    c.chemfile = CHEM
    c.thermfile = THERM
    c.preprocess()
    return c


@pytest.fixture(scope="session")
def chem_tran():
    """GRI-3.0 with its transport data (viscosity / conductivity fits)."""
    import pychemkin_amd as ck

    c = ck.Chemistry(chem=CHEM, therm=THERM, tran=TRAN, label="GRI 3.0")
    c.preprocess()
    return c


def ch4_air_Y(mech, phi):
    phi = np.atleast_1d(np.asarray(phi, dtype=np.float64))
    X = np.zeros((phi.size, mech.KK))
    alpha = 2.0 / 0.21
    X[:, mech.species.index("CH4")] = phi
    X[:, mech.species.index("O2")] = 0.21 * alpha
    X[:, mech.species.index("N2")] = 0.79 * alpha
    X /= X.sum(axis=1, keepdims=True)
    Y = X * mech.wt
    return Y / Y.sum(axis=1, keepdims=True)


def h2_air_Y(mech):
    """H2:O2:N2 = 2:1:3.76 (closed_homogeneous__transient.py:62)."""
    X = np.zeros(mech.KK)
    X[mech.species.index("H2")] = 2.0
    X[mech.species.index("O2")] = 1.0
    X[mech.species.index("N2")] = 3.76
    X /= X.sum()
    Y = X * mech.wt
    return Y / Y.sum()


def check_h2_golden(g, mech, t, T, Y, wdot_h2o, min_ok=101):
    """All five columns of closed_homogeneous__transient.baseline, each point within the golden's
    own per-column tolerance (closed_homogeneous__transient.py:195-207).  ``Y`` is the saved
    mass-fraction trajectory [npts, KK]; X_H2O and the density follow from it as the reference's
    solution mixtures compute them; ``wdot_h2o`` is the caller's ROP()[H2O] at each point."""
    R = 1.3806504e-16 * 6.02214179e23
    P = P_ATM
    Y = np.asarray(Y, dtype=np.float64)
    k = mech.species.index("H2O")
    X = Y[:, k] / mech.wt[k] / np.sum(Y / mech.wt, axis=1)
    rho = P / (R * np.asarray(T)) / np.sum(Y / mech.wt, axis=1)
    assert np.asarray(t).tolist() == g["state-time"]
    cols = {"state-temperature": (T, "tolerance-var"), "species-H2O_mole_fraction": (X, "tolerance-frac"),
            "rate-H2O_production_rate": (wdot_h2o, "tolerance-ROP"), "state-density": (rho, "tolerance-var")}
    counts = {}
    for key, (v, tol) in cols.items():
        counts[key] = int(within(v, g[key], *g[tol]).sum())
    assert all(c >= min_ok for c in counts.values()), counts
    return counts


def sensitivity_mixture(chem):
    """sensitivity.py:66-86: C3H8:CH4:H2 = 0.1:0.8:0.1 fuel, O2:N2 = 1:3.76, phi = 1.1, 900 K, 1 atm."""
    import pychemkin_amd as ck

    oxid = ck.Mixture(chem)
    oxid.X = [("O2", 1.0), ("N2", 3.76)]
    fuel = ck.Mixture(chem)
    fuel.X = [("C3H8", 0.1), ("CH4", 0.8), ("H2", 0.1)]
    mix = ck.Mixture(chem)
    mix.pressure = P_ATM
    mix.temperature = 900.0
    assert mix.X_by_Equivalence_Ratio(chem, fuel.X, oxid.X, np.zeros(chem.KK), ["CO2", "H2O", "N2"],
                                      equivalenceratio=1.1) == 0
    return mix


# sensitivity.py:95-122: CONP + ENERGY, V = 10 cm3, t_end = 2 s, 1e-10/1e-8, TIFP; perturbation 0.1 %
SENS_RUN = dict(energy=1, t_end=2.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
SENS_FACTOR = 1.001


def top5(sens):
    """Indices of the 5 largest positive and 5 most negative coefficients (sensitivity.py:166-174)."""
    pos = np.argpartition(sens, -5)[-5:]
    neg = np.argpartition(-sens, -5)[-5:]
    return set(pos.tolist()), set(neg.tolist())


def within(a, b, atol, rtol):
    """Symmetric golden tolerance |a - b| <= atol + rtol |b| (SURVEY.md section 4 comparator fix)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b) <= atol + rtol * np.abs(b)


def _h_mass(tables, Y, T):
    """Mixture enthalpy per mass [erg/g] from the NASA-7 tables (numpy; [KK][17] layout of ckmi_mech_desc)."""
    th = np.asarray(tables["thermo"])
    a = np.where((T > th[:, 1])[:, None], th[:, 10:17], th[:, 3:10])
    hRT = a[:, 0] + T * (a[:, 1] / 2 + T * (a[:, 2] / 3 + T * (a[:, 3] / 4 + T * a[:, 4] / 5))) + a[:, 5] / T
    return float(np.sum(Y * hRT * 8.314462618e7 * T / np.asarray(tables["wt"])))


def hp_equilibrium_start(mech, tables, phi, T_reac=295.15):
    """Start state for the HP-equilibrium golden (adiabaticflametemperature.py:54-91: CH4/O2,
    products CO2/H2O, 295.15 K, 1 atm): the same elements burned to {CO, CO2, H2O, H2, O2} and
    heated to the temperature with the reactants' enthalpy per mass.  An adiabatic constant-pressure
    reactor started there keeps H and P, so its long-time state is the HP equilibrium of the
    reactant mixture (no ignition wait at 295 K).  Returns (T*, Y*)."""
    def Y_of(moles):
        X = np.zeros(mech.KK)
        for k, v in moles.items():
            X[mech.species.index(k)] = v
        Y = X * mech.wt
        return Y / Y.sum()

    h_r = _h_mass(tables, Y_of({"CH4": phi, "O2": 2.0}), T_reac)   # X = phi X_fuel + 2 X_oxid
    n_co, o_left = phi, 4.0 - phi
    n_h2o = min(2.0 * phi, o_left)
    o_left -= n_h2o
    n_h2 = (4.0 * phi - 2.0 * n_h2o) / 2.0
    conv = min(n_co, o_left)
    n_co -= conv
    o_left -= conv
    Yp = Y_of({"CO": n_co, "CO2": conv, "H2O": n_h2o, "H2": n_h2, "O2": o_left / 2.0})
    lo, hi = 300.0, 8000.0
    for _ in range(100):
        mid = 0.5 * (lo + hi)
        if _h_mass(tables, Yp, mid) > h_r:
            hi = mid
        else:
            lo = mid
    return 0.5 * (lo + hi), Yp


BIG_CHEM = os.path.join(ROOT, "data", "gri30_tracer161_chem.inp")
BIG_THERM = os.path.join(ROOT, "data", "gri30_tracer161_thermo.dat")


@pytest.fixture(scope="session")
def big_mech():
    """Synthetic 161-species mechanism (data/make_tracer_mechanism.py)."""
    from pychemkin_amd.mechanism import Mechanism

    return Mechanism.from_files(BIG_CHEM, BIG_THERM)
