"""Second, independent CPU restatement of thermo + ROP in numpy (test infrastructure only).

Written in matrix form (dense stoichiometric matrices nu' and nu'' [II, KK], Kc from the
stoichiometric change of g/RT) rather than the slot loops of ckoracle.c, so the two CPU
restatements share no code path.  Used by tests to pin the C oracle's kinetics, and with
scipy's Radau to pin the C oracle's integrator.  Standard Chemkin-II gas kinetics (the closed
library's call sites: chemkin_wrapper.py:375-498, mixture.py:1442,1551).
"""
from __future__ import annotations

import numpy as np

BOLTZMANN = 1.3806504e-16
AVOGADRO = 6.02214179e23
RU = BOLTZMANN * AVOGADRO
PATM = 1.01325e6


CFLOOR = 1e-14  # oracle/ckoracle.c CFLOOR


def _cpow(C, o):
    """C ** o elementwise under the rule of oracle/ckoracle.c conc_pow and the device kernels:
    exact for o in {0, 1, 2, 3}; for 0 < o < 1 the chord CFLOOR^(o-1) C below CFLOOR (negative C
    included); otherwise 0 for C <= 0."""
    C, o = np.broadcast_arrays(np.asarray(C, dtype=np.float64), np.asarray(o, dtype=np.float64))
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        r = np.power(C, o)
        chord = np.power(CFLOOR, o - 1.0) * C
    exact = (o == 0.0) | (o == 1.0) | (o == 2.0) | (o == 3.0)
    r = np.where(~exact & (C <= 0.0), 0.0, r)
    return np.where(~exact & (o < 1.0) & (C < CFLOOR), chord, r)


class NumpyKinetics:
    def __init__(self, tables):
        t = tables
        self.KK = KK = int(t["KK"])
        self.II = II = int(t["II"])
        self.wt = t["wt"]
        self.th = t["thermo"]
        self.nuf = np.zeros((II, KK))
        self.nur = np.zeros((II, KK))
        # concentration exponents: FORD / RORD where given, else the stoichiometric coefficients
        self.ordf = np.zeros((II, KK))
        self.ordr = np.zeros((II, KK))
        ford = t.get("ford", t["rnu"])
        rord = t.get("rord", t["pnu"])
        for i in range(II):
            for s in range(int(t["nr"][i])):
                self.nuf[i, t["rsp"][i, s]] += t["rnu"][i, s]
                self.ordf[i, t["rsp"][i, s]] += ford[i, s]
            for s in range(int(t["np"][i])):
                self.nur[i, t["psp"][i, s]] += t["pnu"][i, s]
                self.ordr[i, t["psp"][i, s]] += rord[i, s]
        self.dnu_mat = self.nur - self.nuf
        self.arr = t["arr"]
        self.low = t["low"]
        self.revp = t["revp"]
        self.has_rev = t["has_rev"].astype(bool)
        self.rev = t["rev"].astype(bool)
        self.rtype = t["rtype"]
        self.ftype = t["ftype"]
        self.fpar = t["fpar"]
        self.tbsp = t["tbsp"]
        self.plog_ptr = t["plog_ptr"]
        self.plog_par = t["plog_par"]
        self.eff = np.ones((II, KK))
        for i in range(II):
            for p in range(t["eff_ptr"][i], t["eff_ptr"][i + 1]):
                self.eff[i, t["eff_sp"][p]] = t["eff_val"][p]

    def thermo(self, T):
        th = self.th
        hi = T > th[:, 1]
        a = np.where(hi[:, None], th[:, 10:17], th[:, 3:10])
        cp = a[:, 0] + T * (a[:, 1] + T * (a[:, 2] + T * (a[:, 3] + T * a[:, 4])))
        h = a[:, 0] + T * (a[:, 1] / 2 + T * (a[:, 2] / 3 + T * (a[:, 3] / 4 + T * a[:, 4] / 5))) + a[:, 5] / T
        s = a[:, 0] * np.log(T) + T * (a[:, 1] + T * (a[:, 2] / 2 + T * (a[:, 3] / 3 + T * a[:, 4] / 4))) + a[:, 6]
        return cp, h, s

    def _plog_k(self, i, P, T):
        # PLOG: ln k linear in ln P between the bracketing table pressures, end values outside
        tab = self.plog_par[self.plog_ptr[i]:self.plog_ptr[i + 1]]
        lnk = tab[:, 1] + tab[:, 2] * np.log(T) - tab[:, 3] / T
        return float(np.exp(np.interp(np.log(P), tab[:, 0], lnk)))

    def _cheb_k(self, i, P, T):
        # Chebyshev: log10 k = sum_t sum_p a[t][p] T_t(Tr) T_p(Pr) (numpy.polynomial.chebyshev)
        from numpy.polynomial import chebyshev as ch

        r = self.plog_par[self.plog_ptr[i]:self.plog_ptr[i + 1]].ravel()
        nt, npr = int(r[0]), int(r[1])
        tmin, tmax, pmin, pmax = r[4:8]
        a = r[8:8 + nt * npr].reshape(nt, npr)
        Tr = (2.0 / T - 1.0 / tmin - 1.0 / tmax) / (1.0 / tmax - 1.0 / tmin)
        lp = np.log10([pmin * PATM, pmax * PATM])
        Pr = (2.0 * np.log10(P) - lp[0] - lp[1]) / (lp[1] - lp[0])
        return float(10.0 ** ch.chebval2d(Tr, Pr, a))

    def rates(self, T, P, Y):
        Y = np.asarray(Y, dtype=np.float64)
        rho = P / (RU * T) / np.sum(Y / self.wt)
        C = rho * Y / self.wt
        cp, h, s = self.thermo(T)
        g = h - s
        kf = np.exp(self.arr[:, 0] + self.arr[:, 1] * np.log(T) - self.arr[:, 2] / T)
        for i in np.nonzero(self.rtype == 3)[0]:
            kf[i] = self._plog_k(i, P, T)
        for i in np.nonzero(self.rtype == 5)[0]:
            kf[i] = self._cheb_k(i, P, T)
        lt = self.rtype == 6  # Landau-Teller: + B T^-1/3 + C T^-2/3 (low[:, :2]; RLT in fpar[:, :2])
        t13 = T ** (-1.0 / 3.0)
        kf = np.where(lt, kf * np.exp(self.low[:, 0] * t13 + self.low[:, 1] * t13 * t13), kf)
        M = self.eff @ C
        tbc = self.tbsp >= 0
        M = np.where(tbc, C[np.maximum(self.tbsp, 0)], M)
        mfac = np.where(self.rtype == 1, M, 1.0)
        ca = self.rtype == 4  # chemically activated: arr = k0, low = HIGH (k_inf)
        fo = (self.rtype == 2) | ca
        k0 = np.exp(self.low[:, 0] + self.low[:, 1] * np.log(T) - self.low[:, 2] / T)
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            Pr = np.where(ca, kf * M / k0, np.where(fo, k0 * M / kf, 0.0))
            a, T3, T1, T2 = self.fpar[:, 0], self.fpar[:, 1], self.fpar[:, 2], self.fpar[:, 3]
            Fc = (1 - a) * np.exp(-T / np.where(T3 != 0, T3, 1.0)) + a * np.exp(-T / np.where(T1 != 0, T1, 1.0))
            Fc = Fc + np.where(self.ftype == 3, np.exp(-T2 / T), 0.0)
            lFc = np.log10(np.maximum(Fc, 1e-300))
            lPr = np.log10(np.maximum(Pr, 1e-300))
            c = -0.4 - 0.67 * lFc
            nn = 0.75 - 1.27 * lFc
            f1 = (lPr + c) / (nn - 0.14 * (lPr + c))
            Ftroe = 10.0 ** (lFc / (1 + f1 ** 2))
            X = 1.0 / (1.0 + lPr ** 2)
            Fsri = self.fpar[:, 3] * (self.fpar[:, 0] * np.exp(-self.fpar[:, 1] / T) + np.exp(-T / np.where(self.fpar[:, 2] != 0, self.fpar[:, 2], 1.0))) ** X * T ** self.fpar[:, 4]
        F = np.where((self.ftype == 2) | (self.ftype == 3), Ftroe, np.where(self.ftype == 4, Fsri, 1.0))
        kinf = kf.copy()
        kf = np.where(ca, kf / (1 + Pr) * F, np.where(fo, kf * Pr / (1 + Pr) * F, kf))
        dG = self.dnu_mat @ g
        dn = self.dnu_mat.sum(axis=1)
        Kc = np.exp(-dG) * (PATM / (RU * T)) ** dn
        kr_rev = np.exp(self.revp[:, 0] + self.revp[:, 1] * np.log(T) - self.revp[:, 2] / T)
        kr_rev = np.where(fo, kr_rev * kf / kinf, kr_rev)
        kr_rev = np.where(lt, kr_rev * np.exp(self.fpar[:, 0] * t13 + self.fpar[:, 1] * t13 * t13), kr_rev)
        kr = np.where(self.rev, np.where(self.has_rev, kr_rev, kf / Kc), 0.0)
        pf = np.prod(_cpow(C[None, :], self.ordf), axis=1)
        pr = np.prod(_cpow(C[None, :], self.ordr), axis=1)
        qf = mfac * kf * pf
        qr = mfac * kr * pr
        wdot = self.dnu_mat.T @ (qf - qr)
        return qf, qr, wdot
