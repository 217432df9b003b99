"""Transport data of a chemistry set: the TRANLIB file reader and the viscosity fits.

The reference hands the transport file to KINPreProcess (itran = 1, chemistry.py:636-687;
``tranfile`` chemistry.py:402-431; ``preprocess_transportdata`` chemistry.py:450-480 for a
``TRANSPORT ALL`` block inside the mechanism file), and its closed library fits the kinetic-theory
viscosities (TRANFIT) that KINGetViscosity / KINGetMixtureViscosity evaluate (mixture.py:1860-1977).
Here the file is read on the host (this module, and the same grammar in the native KINPreProcess),
the fits come from ``ckmi_transport_fit`` (host C++, pychemkin_amd/csrc/ckmi_transport.hip) and the
viscosities from the GPU kernels behind ``_native.DeviceTransport``.

Format (one species per line, ``!`` starts a comment): name, geometry (0 atom, 1 linear,
2 nonlinear), eps/kB [K], sigma [A], dipole [D], polarizability [A^3], Zrot.
"""
from __future__ import annotations

import re
from typing import Dict, List, Sequence, Tuple

import numpy as np

# TRANFIT fit interval [K]: 50 points equally spaced in [FIT_TLOW, FIT_THIGH] (our choice, pinned
# by the reference's viscosity goldens: simple 1.1e-3, CONV <= 4.8e-4 relative; tests/test_transport.py)
FIT_TLOW = 300.0
FIT_THIGH = 3500.0

Params = Tuple[int, float, float, float, float, float]


class TransportError(ValueError):
    pass


def parse_transport_text(text: str) -> Dict[str, Params]:
    """TRANLIB records -> {NAME (upper case): (geometry, eps/k, sigma, dipole, polarizability, Zrot)}."""
    out: Dict[str, Params] = {}
    for ln, raw in enumerate(text.splitlines(), 1):
        line = raw.split("!", 1)[0].strip()
        if not line or line.upper().startswith(("TRANSPORT", "END")):
            continue
        tok = line.split()
        if len(tok) < 7:
            raise TransportError(f"transport line {ln}: expected 7 fields, got {raw!r}")
        try:
            geo = int(tok[1])
            vals = [float(t) for t in tok[2:7]]
        except ValueError as exc:
            raise TransportError(f"transport line {ln}: bad number in {raw!r}") from exc
        if geo not in (0, 1, 2):
            raise TransportError(f"transport line {ln}: geometry must be 0, 1 or 2")
        out.setdefault(tok[0].upper(), (geo, *vals))  # the first record of a species wins
    return out


def inline_transport_block(chem_text: str) -> str:
    """The ``TRANSPORT [ALL] ... END`` block of a mechanism file ('' if none)."""
    m = re.search(r"^\s*TRAN\w*(?:\s+ALL)?\s*$(.*?)^\s*END\b", chem_text, re.S | re.M | re.I)
    return m.group(1) if m else ""


def species_params(data: Dict[str, Params], species: Sequence[str]) -> np.ndarray:
    """[KK][6] parameter table in mechanism order; every species needs a record (as TRANFIT)."""
    missing: List[str] = [s for s in species if s.upper() not in data]
    if missing:
        raise TransportError(f"no transport data for species {missing}")
    return np.array([data[s.upper()] for s in species], dtype=np.float64)


def viscosity_fits(wt: np.ndarray, params: np.ndarray) -> np.ndarray:
    """[KK][4] coefficients of ln eta_k [g/(cm s)] in powers of ln T (native TRANFIT restatement)."""
    from . import _native

    return _native.transport_fit(wt, params, FIT_TLOW, FIT_THIGH)


def conductivity_fits(wt: np.ndarray, params: np.ndarray, thermo: np.ndarray) -> np.ndarray:
    """[KK][4] ln-T cubic fits of the species thermal conductivities (host C++: ckmi_conductivity_fit)."""
    from . import _native

    return _native.conductivity_fit(wt, params, thermo, FIT_TLOW, FIT_THIGH)
