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


def omega11(tstar, dstar):
    """Omega(1,1)*: Neufeld et al. (1972) Lennard-Jones correlation + 0.19 delta*^2 / T* (Brokaw)."""
    tstar = np.asarray(tstar, dtype=np.float64)
    lj = (1.06036 * tstar ** -0.15610 + 0.19300 * np.exp(-0.47635 * tstar) + 1.03587 * np.exp(-1.52996 * tstar)
          + 1.76474 * np.exp(-3.89411 * tstar))
    return lj + 0.19 * dstar * dstar / tstar


def _parker(tstar):
    """Parker's temperature dependence of the rotational collision number, F(T*) (Zrot(T) = Zrot(298) F(298/eps) / F(T*))."""
    r = 1.0 / np.asarray(tstar, dtype=np.float64)
    return 1.0 + 0.5 * np.pi ** 1.5 * r ** 0.5 + (0.25 * np.pi ** 2 + 2.0) * r + np.pi ** 1.5 * r ** 1.5


def species_conductivity_exact(T, wt, params, cv_R):
    """lambda_k(T) [erg/(cm s K)], the Warnatz form of the Chemkin TRANFIT species conductivity:
    lambda = eta / W (f_tr Cv_tr + f_rot Cv_rot + f_vib Cv_vib), rho D_kk / eta from the self-diffusion
    coefficient (Omega(1,1)*), Zrot with Parker's correction; atoms: 15/4 R eta / W.
    T [n], cv_R [n, KK] (cv / R of each species at T) -> [n, KK]."""
    T = np.atleast_1d(np.asarray(T, dtype=np.float64))
    geo = np.array([p[0] for p in params])
    eps = np.array([p[1] for p in params])
    sig = np.array([p[2] for p in params]) * ANGSTROM
    mu = np.array([p[3] for p in params]) * DEBYE
    zrot = np.array([p[5] for p in params])
    dstar = 0.5 * mu * mu / (eps * BOLTZMANN * sig ** 3)
    W = np.asarray(wt, dtype=np.float64)
    m = W / AVOGADRO
    R = BOLTZMANN * AVOGADRO
    eta = species_viscosity_exact(T, wt, params)
    tstar = T[:, None] / eps[None, :]
    kT = BOLTZMANN * T[:, None]
    # rho D_kk = (3/16) sqrt(2 pi (kT)^3 / (m / 2)) / (pi sigma^2 Omega11*) * m / kT
    rhoD = 3.0 / 16.0 * np.sqrt(2.0 * np.pi * kT ** 3 / (0.5 * m[None, :])) / (
        np.pi * sig[None, :] ** 2 * omega11(tstar, dstar[None, :])) * m[None, :] / kT
    x = rhoD / eta
    cvt = 1.5
    cvr = np.where(geo == 1, 1.0, np.where(geo == 2, 1.5, 0.0))[None, :]
    cvv = np.asarray(cv_R) - cvt - cvr
    Z = zrot[None, :] * _parker(298.0 / eps)[None, :] / _parker(tstar)
    A = 2.5 - x
    Bc = Z + 2.0 / np.pi * (5.0 / 3.0 * cvr + x)
    ftr = 2.5 * (1.0 - 2.0 / np.pi * cvr / cvt * A / Bc)
    frot = x * (1.0 + 2.0 / np.pi * A / Bc)
    lam = eta / W[None, :] * R * (ftr * cvt + frot * cvr + x * cvv)
    atom = (geo == 0)[None, :]
    return np.where(atom, 3.75 * R * eta / W[None, :], lam)


def cv_R_nasa(thermo, T):
    """cv / R of every species from the [KK][17] NASA-7 table at T [n] -> [n, KK]."""
    th = np.asarray(thermo, dtype=np.float64)
    T = np.atleast_1d(np.asarray(T, dtype=np.float64))
    hi = T[:, None] > th[None, :, 1]
    a = np.where(hi[:, :, None], th[None, :, 10:17], th[None, :, 3:10])
    Tn = T[:, None]
    cp = a[..., 0] + Tn * (a[..., 1] + Tn * (a[..., 2] + Tn * (a[..., 3] + Tn * a[..., 4])))
    return cp - 1.0


def conductivity_fits(wt, params, thermo, thigh):
    """Cubic fits of ln lambda_k in ln T: [KK, 4] (same grid as viscosity_fits)."""
    Tf = np.linspace(FIT_TLOW, thigh, FIT_NPTS)
    V = np.vander(np.log(Tf), FIT_ORDER, increasing=True)
    y = np.log(species_conductivity_exact(Tf, wt, params, cv_R_nasa(thermo, Tf)))
    coef, *_ = np.linalg.lstsq(V, y, rcond=None)
    return coef.T.copy()


def mixture_conductivity(T, X, fits):
    """0.5 (sum X_k lambda_k + 1 / sum X_k / lambda_k); T [n], X [n, KK] -> [n]."""
    X = np.atleast_2d(np.asarray(X, dtype=np.float64))
    lam = species_viscosity(T, fits)  # same ln-T cubic evaluation
    return 0.5 * (np.sum(X * lam, axis=1) + 1.0 / np.sum(X / lam, axis=1))


def mole_fractions(Y, wt):
    Y = np.atleast_2d(np.asarray(Y, dtype=np.float64))
    x = Y / np.asarray(wt)[None, :]
    return x / x.sum(axis=1, keepdims=True)
