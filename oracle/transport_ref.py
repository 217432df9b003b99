"""Numpy restatement of the Chemkin pure-species and mixture viscosity (test infrastructure only).

The reference computes viscosity inside the closed libKINetics.so (KINGetViscosity /
KINGetMixtureViscosity, chemkin_wrapper.py:407-412,442-448; called by mixture.py:1860-1977) from
the transport data file read at preprocess (chemistry.py:636-687).  The published Chemkin TRANFIT /
TRANLIB method restated here:

* pure species (Chapman-Enskog):  eta_k(T) = 5/16 sqrt(pi m_k kB T) / (pi sigma_k^2 Omega22*(T*, delta*))
  with T* = kB T / eps_k and the reduced dipole moment delta* = mu_k^2 / (2 eps_k sigma_k^3);
* the collision integral Omega(2,2)* of the Lennard-Jones 12-6 potential by the Neufeld-Janzen-Aziz
  (1972) correlation of the Hirschfelder table, plus the polar correction 0.2 delta*^2 / T* (Brokaw
  1969) of the Stockmayer potential (Monchick-Mason) for the polar species;
* ln eta_k fitted as a cubic polynomial in ln T by least squares on 50 temperatures equally spaced
  between 300 K and the mechanism's highest thermo temperature (the TRANFIT form: the library
  evaluates the fit, not the kinetic-theory expression);
* mixture (Wilke):  eta = sum_k X_k eta_k / sum_j X_j Phi_kj,
  Phi_kj = (1 + W_k / W_j)^(-1/2) (1 + (eta_k / eta_j)^(1/2) (W_j / W_k)^(1/4))^2 / sqrt(8).

Parity with Chemkin is pinned by the reference's viscosity goldens (simple, CONV, createmixture
state-viscosity); see tests/test_transport.py.  This file shares no code with the product's C++
fit (pychemkin_amd/csrc/ckmi_transport.hip).
"""
from __future__ import annotations

import numpy as np

BOLTZMANN = 1.380649e-16   # erg / K
AVOGADRO = 6.02214076e23
DEBYE = 1e-18              # esu cm
ANGSTROM = 1e-8            # cm
FIT_TLOW = 300.0
FIT_NPTS = 50
FIT_ORDER = 4              # coefficients of the ln T polynomial


def parse_transport(text: str) -> dict:
    """name -> (geometry, eps/k [K], sigma [A], dipole [D], polarizability [A^3], Zrot)."""
    out = {}
    for raw in text.splitlines():
        line = raw.split("!", 1)[0].strip()
        if not line:
            continue
        tok = line.split()
        if len(tok) < 7:
            continue
        out[tok[0].upper()] = (int(tok[1]), float(tok[2]), float(tok[3]), float(tok[4]), float(tok[5]),
                               float(tok[6]))
    return out


def omega22(tstar, dstar):
    """Omega(2,2)*: Neufeld et al. (1972) Lennard-Jones correlation + 0.2 delta*^2 / T*."""
    tstar = np.asarray(tstar, dtype=np.float64)
    lj = 1.16145 * tstar ** -0.14874 + 0.52487 * np.exp(-0.77320 * tstar) + 2.16178 * np.exp(-2.43787 * tstar)
    return lj + 0.2 * dstar * dstar / tstar


def species_viscosity_exact(T, wt, params):
    """eta_k(T) [g/(cm s)] from kinetic theory; T [n] -> [n, KK]."""
    T = np.atleast_1d(np.asarray(T, dtype=np.float64))
    eps = np.array([p[1] for p in params])
    sig = np.array([p[2] for p in params]) * ANGSTROM
    mu = np.array([p[3] for p in params]) * DEBYE
    dstar = 0.5 * mu * mu / (eps * BOLTZMANN * sig ** 3)
    m = np.asarray(wt, dtype=np.float64) / AVOGADRO
    tstar = T[:, None] / eps[None, :]
    return (5.0 / 16.0) * np.sqrt(np.pi * m[None, :] * BOLTZMANN * T[:, None]) / (
        np.pi * sig[None, :] ** 2 * omega22(tstar, dstar[None, :]))


def viscosity_fits(wt, params, thigh):
    """Cubic fits of ln eta_k in ln T: [KK, 4], coefficient of (ln T)^n in column n."""
    Tf = np.linspace(FIT_TLOW, thigh, FIT_NPTS)
    lnT = np.log(Tf)
    V = np.vander(lnT, FIT_ORDER, increasing=True)
    y = np.log(species_viscosity_exact(Tf, wt, params))
    coef, *_ = np.linalg.lstsq(V, y, rcond=None)
    return coef.T.copy()


def species_viscosity(T, fits):
    """eta_k(T) from the fits; T [n] -> [n, KK]."""
    lnT = np.log(np.atleast_1d(np.asarray(T, dtype=np.float64)))
    V = np.vander(lnT, FIT_ORDER, increasing=True)
    return np.exp(V @ fits.T)


def mixture_viscosity(T, X, wt, fits):
    """Wilke mixture viscosity; T [n], X [n, KK] mole fractions -> [n]."""
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    eta = species_viscosity(T, fits)                  # [n, KK]
    W = np.asarray(wt, dtype=np.float64)
    A = (1.0 + W[:, None] / W[None, :]) ** -0.5 / np.sqrt(8.0)   # [k, j]
    B = (W[None, :] / W[:, None]) ** 0.25
    s = np.sqrt(eta)
    phi = A[None] * (1.0 + (s[:, :, None] / s[:, None, :]) * B[None]) ** 2   # [n, k, j]
    den = np.einsum("nkj,nj->nk", phi, X)
    return np.sum(X * eta / den, axis=1)


def mole_fractions(Y, wt):
    Y = np.atleast_2d(np.asarray(Y, dtype=np.float64))
    x = Y / np.asarray(wt)[None, :]
    return x / x.sum(axis=1, keepdims=True)
