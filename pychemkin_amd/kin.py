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
    "KINSetUnitSystem": (ct.c_int, [_I]),                                                           # :301
    "KINPreProcess": (ct.c_int, [_I, _I, _C, _C, _C, _C, _C, _C, _C, _C, _I]),                      # :304
    "KINInitialize": (ct.c_int, [_I, _I]),                                                          # :318
    "KINFinish": (None, []),                                                                        # :323
    "KINUpdateChemistrySet": (ct.c_int, [_I]),                                                      # :325
    "KINSwitchChemistrySet": (ct.c_int, [_I]),                                                      # :329
    "KINGetChemistrySizes": (ct.c_int, [_I, _I, _I, _I, _I, _I, _I, _I, _I]),                       # :334
    "KINGetGasSpeciesNames": (ct.c_int, [_I, ct.POINTER(_C)]),                                      # :346
    "KINGetElementNames": (ct.c_int, [_I, ct.POINTER(_C)]),                                         # :351
    "KINGetAtomicWeights": (ct.c_int, [_I, _DC]),                                                   # :356
    "KINGetGasMolecularWeights": (ct.c_int, [_I, _DC]),                                             # :361
    "KINGetGasReactionString": (ct.c_int, [_I, _I, _I, _C]),                                        # :366
    "KINGetReactionStringLength": (ct.c_int, [_I]),                                                 # :373
    "KINGetGasSpecificHeat": (ct.c_int, [_I, _D, _DC]),                                             # :376
    "KINGetGasSpeciesEnthalpy": (ct.c_int, [_I, _D, _DC]),                                          # :382
    "KINGetGasSpeciesInternalEnergy": (ct.c_int, [_I, _D, _DC]),                                    # :388
    "KINGetGasSpeciesComposition": (ct.c_int, [_I, _IF]),                                           # :394
    "KINGetMassDensity": (ct.c_int, [_I, _D, _D, _DC, _D]),                                         # :399
    "KINGetViscosity": (ct.c_int, [_I, _D, _DC]),                                                   # :408
    "KINGetConductivity": (ct.c_int, [_I, _D, _DC]),                                                # :414
    "KINGetDiffusionCoeffs": (ct.c_int, [_I, _D, _D, _DF]),                                         # :420
    "KINGetGasMixtureSpecificHeat": (ct.c_int, [_I, _D, _DC, _D]),                                  # :428
    "KINGetGasMixtureEnthalpy": (ct.c_int, [_I, _D, _DC, _D]),                                      # :435
    "KINGetMixtureViscosity": (ct.c_int, [_I, _D, _DC, _D]),                                        # :443
    "KINGetMixtureConductivity": (ct.c_int, [_I, _D, _DC, _D]),                                     # :450
    "KINGetMixtureDiffusionCoeffs": (ct.c_int, [_I, _D, _D, _DC, _DC]),                             # :457
    "KINGetOrdinaryDiffusionCoeffs": (ct.c_int, [_I, _D, _D, _DC, _DF]),                            # :465
    "KINGetThermalDiffusionCoeffs": (ct.c_int, [_I, _D, _D, _DC, _DC, _D]),                         # :473
    "KINGetGasROP": (ct.c_int, [_I, _D, _D, _DC, _DC]),                                             # :483
    "KINGetGasReactionRates": (ct.c_int, [_I, _D, _D, _DC, _DC, _DC]),                              # :491
    "KINGetReactionRateParameters": (ct.c_int, [_I, _DC, _DC, _DC]),                                # :500
    "KINSetAFactorForAReaction": (ct.c_int, [_I, _I, _D]),                                          # :507
    "KINCalculateEquil": (ct.c_int, [_I, _D, _D, _DC, _DC]),                                        # :514
    "KINCalculateEquilWithOption": (ct.c_int, [_I, _I, _D, _D, _DC, _DC]),                          # :522
    "KINCalculateEqGasWithOption": (ct.c_int, [_I, _I, _I, _D, _D, _DC, _D, _D, _D, _D, _DC]),      # :531
    "KINRealGas_SetParameter": (ct.c_int, [_C, _D]),                                                # :546
    "KINRealGas_GetEOSMode": (ct.c_int, [_I, _I, _C]),                                              # :551
    "KINRealGas_SetMixingRule": (ct.c_int, [_I, _I, _I]),                                           # :557
    "KINRealGas_UseIdealGasLaw": (ct.c_int, [_I, _I]),                                              # :563
    "KINRealGas_UseCubicEOS": (ct.c_int, [_I, _I]),                                                 # :568
    "KINRealGas_SetCurrentPressure": (ct.c_int, [_I, _D]),                                          # :573
    "KINRealGas_CheckRealGasStatus": (ct.c_int, [_I, _I]),                                          # :578
    "KINGetGamma": (ct.c_int, [_I, _D, _DC, _D]),                                                   # :583
    "KINAll0D_Setup": (ct.c_int, [_I, _I, _I, _I, _I, _I, _IC, _I]),                                # :591
    "KINAll0D_SetupWorkArrays": (ct.c_int, [_I, _I]),                                               # :602
    "KINAll0D_SetupBatchInputs": (ct.c_int, [_I, _D, _D, _D, _D, _D, _D, _DC, _DC, _DC]),           # :607
    "KINAll0D_SetupPSRReactorInputs": (ct.c_int, [_I, _I, _D, _D, _D, _D, _D, _D, _D, _DC, _DC, _DC]),# :620
    "KINAll0D_SetupPSRInletInputs": (ct.c_int, [_I, _I, _I, _D, _D, _DC]),                          # :635
    "KINAll0D_SetupPFRInputs": (ct.c_int, [_I, _D, _D, _D, _D, _D, _D, _DC, _DC, _D, _DC]),         # :644
    "KINAll0D_SetupHCCIInputs": (ct.c_int, [_I, _D, _D, _D, _D, _D, _D, _D, _D, _D, _D, _DC]),      # :658
    "KINAll0D_SetupHCCIZoneInputs": (ct.c_int, [_I, _I, _D, _D]),                                   # :673
    "KINAll0D_SetupSIInputs": (ct.c_int, [_I, _D, _D, _D, _D, _D]),                                 # :680
    "KINAll0D_Calculate": (ct.c_int, [_I]),                                                         # :689
    "KINAll0D_CalculateInput": (ct.c_int, [_I, _I, _C, _I, _IC]),                                   # :691
    "KINAll0D_SetUserKeyword": (ct.c_int, [_C]),                                                    # :699
    "KINAll0D_IntegrateHeatRelease": (ct.c_int, []),                                                # :701
    "KINAll0D_SetHeatTransfer": (ct.c_int, [_D, _D]),                                               # :703
    "KINAll0D_SetHeatTransferArea": (ct.c_int, [_D]),                                               # :708
    "KINAll0D_SetProfilePoints": (ct.c_int, [_I]),                                                  # :711
    "KINAll0D_SetProfileParameter": (ct.c_int, [_C, _I, _DC, _DC]),                                 # :713
    "KINAll0D_SetProfileKeyword": (ct.c_int, [_I, _I, _C, _I, _DC, _DC]),                           # :720
    "KINAll0D_SetSolverInitialStepTime": (ct.c_int, [_D]),                                          # :730
    "KINAll0D_SetSolverMaximumStepTime": (ct.c_int, [_D]),                                          # :732
    "KINAll0D_SetSolverMaximumIteration": (ct.c_int, [_I]),                                         # :734
    "KINAll0D_SetRelaxIteration": (ct.c_int, []),                                                   # :736
    "KINAll0D_SetMinimumSpeciesBound": (ct.c_int, [_D]),                                            # :738
    "KINAll0D_GetSolution": (ct.c_int, [_D, _D, _DC]),                                              # :741
    "KINAll0D_GetSolnResponseSize": (ct.c_int, [_I, _I]),                                           # :747
    "KINAll0D_GetGasSolnResponse": (ct.c_int, [_I, _I, _I, _DC, _DC, _DC, _DC, _DF]),               # :752
    "KINAll0D_GetIgnitionDelay": (ct.c_int, [_D]),                                                  # :763
    "KINAll0D_GetHeatRelease": (ct.c_int, [_D, _D]),                                                # :765
    "KINAll0D_GetEngineHeatRelease": (ct.c_int, [_DC, _D, _D, _D, _D, _D]),                         # :770
    "KINAll0D_GetExitMassFlowRate": (ct.c_int, [_D]),                                               # :779
    "KINPremix_SetParameter": (ct.c_int, [_C, _D]),                                                 # :782
    "KINPremix_CalculateFlame": (ct.c_int, [_I, _I, _D, _D, _DC, _D, _D]),                          # :787
    "KINPremix_GetSolution": (ct.c_int, [_I, _I, _DC, _DC, _DF]),                                   # :797
    "KINPremix_GetSolutionGridPoints": (ct.c_int, [_I]),                                            # :805
    "KINPremix_GetFlameMassFlux": (ct.c_int, [_D]),                                                 # :809
    "KINOppdif_SetInlet": (ct.c_int, [_C, _I, _D, _DC, _D, _I]),                                    # :818
    "KINOppdif_SetParameter": (ct.c_int, [_C, _D]),                                                 # :826
    "KINOppdif_CalculateFlame": (ct.c_int, [_I, _I, _D, _D]),                                       # :831
    "KINOppdif_GetSolutionGridPoints": (ct.c_int, [_I]),                                            # :837
    "KINOppdif_GetSolution": (ct.c_int, [_I, _I, _D, _D, ct.POINTER(_D)]),                          # :838
    "KINOppdif_GetSolnSpeciesIntegratedROP": (ct.c_int, [_I, _I, _I, _I, ct.POINTER(_D)]),          # :847
    "KINGetMassFractionFromMoleFraction": (ct.c_int, [_I, _DC, _DC]),                               # :856
    "KINGetMoleFractionFromMassFraction": (ct.c_int, [_I, _DC, _DC]),                               # :863
}

_REG = {
    "ckmi_kin_register": (ct.c_int, [ct.POINTER(_native.MechDesc), ct.c_int32, ct.c_char_p, ct.c_char_p, ct.c_void_p,
                                     ct.c_void_p, ct.POINTER(ct.c_int32)]),
    "ckmi_kin_release": (ct.c_int, [ct.c_int32]),
    "ckmi_kin_last_error": (ct.c_char_p, []),
    "ckmi_kin_keyword_class": (ct.c_int, [ct.c_char_p]),
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


def keyword_class(key: str) -> int:
    """The device path's keyword policy (ckmi_kin_keyword_class; host only): 1 sets a reactor
    configuration field, 2 accepted without effect, 0 rejected."""
    return int(bind().ckmi_kin_keyword_class(key.encode()))


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
    t = mech.to_tables()
    tables = {k: np.ascontiguousarray(v) for k, v in t.items() if isinstance(v, np.ndarray) and v.ndim > 0}
    d = _native.MechDesc()
    _native.fill_desc(d, t, tables)
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
