"""Host utilities of the batch path (reference utilities.py).

calculate_stoichiometrics   element balance for the complete-combustion mixture
                            (utilities.py:295-489, used by X_by_Equivalence_Ratio)
find_interpolate_parameters bisection in a monotone array (utilities.py:114-166)
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np


def calculate_stoichiometrics(chem, fuel_molefrac: np.ndarray, oxid_molefrac: np.ndarray,
                              prod_index: Sequence[int]) -> Tuple[float, np.ndarray]:
    """Return (alpha, nu): moles of oxidizer per mole of fuel mixture and product moles.

    Solves  sum_k NCF[m,k] (fuel_k + alpha*oxid_k) = sum_p NCF[m,p] nu_p  for every element m
    that appears in the fuel or oxidizer, in the least-squares sense (exact when consistent),
    as the reference does with np.linalg.solve on the square element-balance system
    (utilities.py:485-488).
    """
    ncf = np.asarray(chem.SpeciesComposition(), dtype=np.float64)  # [MM, KK]
    fuel = np.asarray(fuel_molefrac, dtype=np.float64)
    oxid = np.asarray(oxid_molefrac, dtype=np.float64)
    ef = ncf @ fuel
    eo = ncf @ oxid
    used = np.nonzero((np.abs(ef) + np.abs(eo) + np.abs(ncf[:, list(prod_index)]).sum(axis=1)) > 0)[0]
    # unknowns: alpha, nu_1..nu_P ;  eo*alpha - NCF_p nu = -ef
    A = np.zeros((len(used), 1 + len(prod_index)))
    A[:, 0] = eo[used]
    A[:, 1:] = -ncf[np.ix_(used, list(prod_index))]
    b = -ef[used]
    sol, *_ = np.linalg.lstsq(A, b, rcond=None)
    return float(sol[0]), sol[1:]


def find_interpolate_parameters(x: float, xarray: np.ndarray) -> Tuple[int, float]:
    """Left index and linear ratio of x in the ascending array (utilities.py:114-166)."""
    xa = np.asarray(xarray, dtype=np.float64)
    if x <= xa[0]:
        return 0, 0.0
    if x >= xa[-1]:
        return len(xa) - 2, 1.0
    i = int(np.searchsorted(xa, x, side="right") - 1)
    i = min(max(i, 0), len(xa) - 2)
    return i, float((x - xa[i]) / (xa[i + 1] - xa[i]))
