"""Algorithmic work model of the hot path ("count_ops").

FLOPs are counted per operation of the algorithm, not per instruction the kernel issues:
one add/multiply/divide/compare-free arithmetic op = 1 FLOP, and every transcendental
(exp, log, log10, exp10, pow) = TRANS_COST FLOPs (the FP64 library routines on gfx950 are
~20 FMA-class operations each).  These counts feed roofline.achieved in bench.py:

  reactor  = sum over reactors of  nfe*F_rhs + nje*F_jac_extra + nlu*(F_build + F_lu) + nni*F_solve
  rop      = F_rhs_rop per state,  bytes = 8*(2 + KK) in + 8*(KK + 2) out per state
  rop_jit  = the same for the specialised kernel (ckmi_jit.cpp): reactions with b = E = 0 take
             k = A without the Arrhenius exp
"""
from __future__ import annotations

from typing import Dict

import numpy as np

TRANS_COST = 20


def count_ops(tables: Dict[str, np.ndarray]) -> Dict[str, float]:
    KK = int(tables["KK"])
    II = int(tables["II"])
    n = KK + 1
    rtype, rev, has_rev = tables["rtype"], tables["rev"], tables["has_rev"]
    nr, np_, ftype = tables["nr"], tables["np"], tables["ftype"]
    rnu, pnu = tables["rnu"], tables["pnu"]
    eff = int(tables["eff_ptr"][-1])
    T = TRANS_COST
    # mixture + thermo
    f = 2 * KK + 10                  # mean molecular weight, density
    f += T + 33 * KK                 # log T, NASA-7 cp/h/s and g per species
    f += 3 * KK                      # concentrations and total
    f += 2 * eff                     # third-body sums
    jac = 0.0
    fj = f
    for i in range(II):
        slots = int(nr[i] + np_[i])
        powf = float(np.sum(rnu[i][: nr[i]]) + np.sum(pnu[i][: np_[i]]))
        r = 4 + T                    # forward Arrhenius
        if rtype[i] == 3:            # PLOG: log P, two Arrhenius exponents, interpolation
            r += T + 8 + 6
        if rtype[i] in (2, 4):       # falloff / chemically activated
            r += 4 + T + 2           # k0, Pr
            if ftype[i] in (2, 3):
                r += 6 + 2 * T + (T + 1 if ftype[i] == 3 else 0)  # Fcent
                r += 2 * T + 9 + T + 3                            # log10 x2, f1, exp10
            elif ftype[i] == 4:
                r += 8 + 2 * T + 3 * T
            r += 3
        if rev[i]:
            if has_rev[i]:
                r += 4 + T
            else:
                r += 2 * slots + 3 + T + 2 + T   # dG, (Patm/RT)^dnu, exp
        r += powf + 4                # concentration products and q
        r += 2 * slots               # production scatter
        f += r
        arr = tables["arr"][i]
        fj += r - ((4 + T) if (arr[1] == 0.0 and arr[2] == 0.0 and rtype[i] != 3) else 0)
        # Jacobian extra work for this reaction
        j = 2 * slots + 6 + 10 + 2 * slots
        for nsl in (int(nr[i]), int(np_[i])):
            j += nsl * (nsl + 2 + 4 * slots)
        jac += j
    f += 2 * KK + 10 * KK + 10       # species derivatives, energy equation
    jac += 4 * KK + 2 * KK * KK + 4 * KK + 4 * KK   # T column, T row, J00
    return dict(
        F_rhs=float(f),
        F_jac_extra=float(jac),
        F_build=2.0 * n * n,
        F_lu=(2.0 / 3.0) * n ** 3,
        F_solve=2.0 * n * n,
        F_rop=float(f),
        F_rop_jit=float(fj + 2 * KK + 10 * KK + 10),
        bytes_rop=8.0 * (2 + KK) + 8.0 * (KK + 2),
        n=n,
    )


def reactor_flops(ops: Dict[str, float], stats: np.ndarray) -> float:
    """Total algorithmic FLOPs of a reactor batch from its ckmi statistics [n][8]."""
    st = np.asarray(stats, dtype=np.float64)
    nfe, nje, nlu, nni = st[:, 1].sum(), st[:, 2].sum(), st[:, 3].sum(), st[:, 7].sum()
    return (nfe * ops["F_rhs"] + nje * ops["F_jac_extra"] + nlu * (ops["F_build"] + ops["F_lu"])
            + nni * ops["F_solve"])
