"""TP gas-phase equilibrium by element-potential Gibbs minimisation -- TEST INFRASTRUCTURE ONLY.

Part of the oracle: imported only by tests/ (never by the product path).  It pins the NASA-7
species thermo that the reactor kernels use against the reference's equilibrium golden
(equilibriumcomposition.baseline, examples/mixture/equilibriumcomposition.py:50-80, which calls
ck.equilibrium(opt=1) -> KINCalculateEquil, mixture.py:3800-3895, inside the closed library).

Restated algorithm (the standard element-potential method; not the reference's code, which is
closed): for an ideal gas at (T, P) the minimiser of G = sum_k n_k (mu0_k/RT + ln(n_k P / N))
subject to A n = b has n_k = N exp(-mu0_k/RT - ln P + sum_m A_mk lambda_m).  Newton on
(lambda, ln N) with the element balances and sum n = N as equations, damped to steps of at most
2 in log space.  Only species made of the elements present take part."""
from __future__ import annotations

import numpy as np


class TPEquilibrium:
    """Equilibrium compositions of one element inventory over a sequence of temperatures (solved
    from the previous solution, so sweep from hot to cold for a robust continuation)."""

    def __init__(self, mech, thermo, guess=(("CO2", 0.08), ("CO", 0.01), ("H2O", 0.18), ("H2", 0.01),
                                            ("N2", 0.72))):
        """mech: pychemkin_amd.mechanism.Mechanism; thermo(T) -> (cp/R, h/RT, s/R) arrays [KK]."""
        self.mech = mech
        self.thermo = thermo
        self.A = mech.ncf.astype(np.float64)  # [MM, KK]
        self.guess = [(s, v) for s, v in guess if s in mech.species]
        self._lam = None
        self._lnN = None

    def solve(self, T: float, P_atm: float, Y: np.ndarray, tol: float = 1e-13, maxit: int = 500) -> np.ndarray:
        """Equilibrium mole fractions [KK] at T [K], P [atm] of the elements in mass fractions Y."""
        m, A = self.mech, self.A
        n0 = np.asarray(Y, np.float64) / m.wt  # mol/g
        b = A @ n0
        act = b > 1e-30
        Ae, be = A[act], b[act]
        sp = np.all(A[~act] == 0, axis=0)
        _, hRT, sR = self.thermo(T)
        mu0 = ((hRT - sR) + np.log(P_atm))[sp]
        As = Ae[:, sp]
        if self._lam is None or self._lam.size != be.size:
            lnN = np.log(n0.sum())
            names = [m.species[k] for k in np.nonzero(sp)[0]]
            idx = [names.index(s) for s, _ in self.guess if s in names]
            x = np.array([v for s, v in self.guess if s in names])
            rhs = mu0[idx] + np.log(x * np.exp(lnN)) - lnN
            lam = np.linalg.lstsq(As[:, idx].T, rhs, rcond=None)[0]
        else:
            lam, lnN = self._lam.copy(), self._lnN
        ne = be.size
        for _ in range(maxit):
            n = np.exp(np.clip(lnN - mu0 + As.T @ lam, -700.0, 700.0))
            N = np.exp(lnN)
            F = np.concatenate([As @ n - be, [n.sum() - N]])
            J = np.zeros((ne + 1, ne + 1))
            J[:ne, :ne] = (As * n) @ As.T
            J[:ne, -1] = As @ n
            J[-1, :ne] = As @ n
            J[-1, -1] = n.sum() - N
            dy = np.linalg.solve(J, -F)
            step = min(1.0, 2.0 / max(np.max(np.abs(dy)), 1e-300))
            lam += step * dy[:-1]
            lnN += step * dy[-1]
            if np.max(np.abs(dy)) < tol:
                break
        else:
            raise RuntimeError(f"TP equilibrium did not converge at T = {T}")
        self._lam, self._lnN = lam, lnN
        x = np.zeros(m.KK)
        x[sp] = n / n.sum()
        return x
