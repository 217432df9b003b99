"""ctypes binding of the KIN-compatible C ABI (include/ckmi_kin.h).

This is the binding a PyChemkin maintainer points ``chemkin_wrapper.chemkin`` at to run the
reference's own call sites (mixture.py, chemistry.py, batchreactor.py) on libckmi.so: the
prototypes below are the reference's (chemkin_wrapper.py:296-763, restated entry by entry) and
libckmi.so implements exactly those.  The one step that differs is the mechanism parse
(KINPreProcess, chemkin_wrapper.py:303-316): the Chemkin-format parser is this package's
mechanism.py and hands the tables over with :func:`register`, which returns the chemistry-set
index every KIN* call takes.  See INTEGRATION.md.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np

from . import _native

_I = ct.POINTER(ct.c_int)
_D = ct.POINTER(ct.c_double)
_C = ct.POINTER(ct.c_char)
_DC = np.ctypeslib.ndpointer(dtype=np.double, flags="C_CONTIGUOUS")
_DF = np.ctypeslib.ndpointer(dtype=np.double, flags="F_CONTIGUOUS")
_IC = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_IF = np.ctypeslib.ndpointer(dtype=np.int32, flags="F_CONTIGUOUS")

# name -> (restype, argtypes), as chemkin_wrapper.py declares them (line of each in ckmi_kin.h)
KIN_PROTOTYPES = {
    "KINSetUnitSystem": (ct.c_int, [_I]),
    "KINInitialize": (ct.c_int, [_I, _I]),
    "KINFinish": (None, []),
    "KINUpdateChemistrySet": (ct.c_int, [_I]),
    "KINSwitchChemistrySet": (ct.c_int, [_I]),
    "KINGetChemistrySizes": (ct.c_int, [_I] * 9),
    "KINGetGasSpeciesNames": (ct.c_int, [_I, ct.POINTER(_C)]),
    "KINGetElementNames": (ct.c_int, [_I, ct.POINTER(_C)]),
    "KINGetAtomicWeights": (ct.c_int, [_I, _DC]),
    "KINGetGasMolecularWeights": (ct.c_int, [_I, _DC]),
    "KINGetGasSpeciesComposition": (ct.c_int, [_I, _IF]),
    "KINGetGasSpecificHeat": (ct.c_int, [_I, _D, _DC]),
    "KINGetGasSpeciesEnthalpy": (ct.c_int, [_I, _D, _DC]),
    "KINGetGasSpeciesInternalEnergy": (ct.c_int, [_I, _D, _DC]),
    "KINGetMassDensity": (ct.c_int, [_I, _D, _D, _DC, _D]),
    "KINGetGasMixtureSpecificHeat": (ct.c_int, [_I, _D, _DC, _D]),
    "KINGetGasMixtureEnthalpy": (ct.c_int, [_I, _D, _DC, _D]),
    "KINGetGasROP": (ct.c_int, [_I, _D, _D, _DC, _DC]),
    "KINGetGasReactionRates": (ct.c_int, [_I, _D, _D, _DC, _DC, _DC]),
    "KINGetReactionRateParameters": (ct.c_int, [_I, _DC, _DC, _DC]),
    "KINSetAFactorForAReaction": (ct.c_int, [_I, _I, _D]),
    "KINAll0D_Setup": (ct.c_int, [_I, _I, _I, _I, _I, _I, _IC, _I]),
    "KINAll0D_SetupWorkArrays": (ct.c_int, [_I, _I]),
    "KINAll0D_SetupBatchInputs": (ct.c_int, [_I, _D, _D, _D, _D, _D, _D, _DC, _DC, _DC]),
    "KINAll0D_IntegrateHeatRelease": (ct.c_int, []),
    "KINAll0D_SetProfilePoints": (ct.c_int, [_I]),
    "KINAll0D_SetProfileParameter": (ct.c_int, [_C, _I, _DC, _DC]),
    "KINAll0D_SetUserKeyword": (ct.c_int, [_C]),
    "KINAll0D_Calculate": (ct.c_int, [_I]),
    "KINAll0D_GetIgnitionDelay": (ct.c_int, [_D]),
    "KINAll0D_GetSolnResponseSize": (ct.c_int, [_I, _I]),
    "KINAll0D_GetGasSolnResponse": (ct.c_int, [_I, _I, _I, _DC, _DC, _DC, _DC, _DF]),
}

_REG = {
    "ckmi_kin_register": (ct.c_int, [ct.POINTER(_native.MechDesc), ct.c_int32, ct.c_char_p, ct.c_char_p, ct.c_void_p,
                                     ct.c_void_p, ct.POINTER(ct.c_int32)]),
    "ckmi_kin_release": (ct.c_int, [ct.c_int32]),
    "ckmi_kin_last_error": (ct.c_char_p, []),
}

NAME_LEN = 16


def bind(L: ct.CDLL = None) -> ct.CDLL:
    """Set the reference's prototypes on libckmi.so (what chemkin_wrapper.py does to libKINetics.so)."""
    L = L or _native.lib()
    for name, (res, args) in list(KIN_PROTOTYPES.items()) + list(_REG.items()):
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def last_error() -> str:
    return bind().ckmi_kin_last_error().decode(errors="replace")


def _names(symbols) -> bytes:
    buf = bytearray(NAME_LEN * len(symbols))
    for i, s in enumerate(symbols):
        b = s.encode()[:NAME_LEN]
        buf[NAME_LEN * i:NAME_LEN * i + len(b)] = b
    return bytes(buf)


def register(mech) -> int:
    """Register a parsed Mechanism (pychemkin_amd.mechanism) as a KIN chemistry set on the current
    GPU; returns the chemistry-set index (the value KINPreProcess returns in the reference)."""
    L = bind()
    tables = {k: np.ascontiguousarray(v) for k, v in mech.to_tables().items() if isinstance(v, np.ndarray)}
    d = _native.MechDesc()
    d.KK, d.II = int(mech.KK), int(mech.II)
    for name, _ in _native.MechDesc._fields_[2:]:
        setattr(d, name, tables[name].ctypes.data)
    awt = np.ascontiguousarray(mech.awt, dtype=np.float64)
    ncf = np.ascontiguousarray(mech.ncf, dtype=np.int32)  # [MM][KK]
    cs = ct.c_int32(0)
    rc = L.ckmi_kin_register(ct.byref(d), len(mech.elements), _names(mech.species), _names(mech.elements),
                             awt.ctypes.data, ncf.ctypes.data, ct.byref(cs))
    if rc != 0:
        raise _native.NativeError(f"ckmi_kin_register failed (code {rc}): {last_error()}")
    return int(cs.value)


def release(chemset: int) -> None:
    rc = bind().ckmi_kin_release(int(chemset))
    if rc != 0:
        raise _native.NativeError(f"ckmi_kin_release failed (code {rc}): {last_error()}")
