"""The KIN-compatible C ABI (include/ckmi_kin.h) against the reference's ctypes prototypes.

The argtypes below are restated independently from chemkin_wrapper.py (one entry per reference
declaration, line cited) -- they are what the reference's call sites pass.  On CPU: every symbol
is exported, binds with those prototypes, and the host-side argument checks answer with a non-zero
code and a message (no call here reaches the GPU)."""
import ctypes as ct
import os
import re
import subprocess

import numpy as np

from conftest import ROOT

I, D, C = ct.POINTER(ct.c_int), ct.POINTER(ct.c_double), ct.POINTER(ct.c_char)
DC = np.ctypeslib.ndpointer(dtype=np.double, flags="C_CONTIGUOUS")
DF = np.ctypeslib.ndpointer(dtype=np.double, flags="F_CONTIGUOUS")
IC = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
IF = np.ctypeslib.ndpointer(dtype=np.int32, flags="F_CONTIGUOUS")

REFERENCE_ARGTYPES = {
    "KINSetUnitSystem": [I],                                                  # chemkin_wrapper.py:301
    "KINPreProcess": [I, I, C, C, C, C, C, C, C, C, I],                       # chemkin_wrapper.py:304
    "KINInitialize": [I, I],                                                  # chemkin_wrapper.py:318
    "KINFinish": [],                                                          # chemkin_wrapper.py:323
    "KINUpdateChemistrySet": [I],                                             # chemkin_wrapper.py:325
    "KINSwitchChemistrySet": [I],                                             # chemkin_wrapper.py:329
    "KINGetChemistrySizes": [I, I, I, I, I, I, I, I, I],                      # chemkin_wrapper.py:334
    "KINGetGasSpeciesNames": [I, ct.POINTER(C)],                              # chemkin_wrapper.py:346
    "KINGetElementNames": [I, ct.POINTER(C)],                                 # chemkin_wrapper.py:351
    "KINGetAtomicWeights": [I, DC],                                           # chemkin_wrapper.py:356
    "KINGetGasMolecularWeights": [I, DC],                                     # chemkin_wrapper.py:361
    "KINGetGasReactionString": [I, I, I, C],                                  # chemkin_wrapper.py:366
    "KINGetReactionStringLength": [I],                                        # chemkin_wrapper.py:373
    "KINGetGasSpecificHeat": [I, D, DC],                                      # chemkin_wrapper.py:376
    "KINGetGasSpeciesEnthalpy": [I, D, DC],                                   # chemkin_wrapper.py:382
    "KINGetGasSpeciesInternalEnergy": [I, D, DC],                             # chemkin_wrapper.py:388
    "KINGetGasSpeciesComposition": [I, IF],                                   # chemkin_wrapper.py:394
    "KINGetMassDensity": [I, D, D, DC, D],                                    # chemkin_wrapper.py:399
    "KINGetViscosity": [I, D, DC],                                            # chemkin_wrapper.py:408
    "KINGetConductivity": [I, D, DC],                                         # chemkin_wrapper.py:414
    "KINGetDiffusionCoeffs": [I, D, D, DF],                                   # chemkin_wrapper.py:420
    "KINGetGasMixtureSpecificHeat": [I, D, DC, D],                            # chemkin_wrapper.py:428
    "KINGetGasMixtureEnthalpy": [I, D, DC, D],                                # chemkin_wrapper.py:435
    "KINGetMixtureViscosity": [I, D, DC, D],                                  # chemkin_wrapper.py:443
    "KINGetMixtureConductivity": [I, D, DC, D],                               # chemkin_wrapper.py:450
    "KINGetMixtureDiffusionCoeffs": [I, D, D, DC, DC],                        # chemkin_wrapper.py:457
    "KINGetOrdinaryDiffusionCoeffs": [I, D, D, DC, DF],                       # chemkin_wrapper.py:465
    "KINGetThermalDiffusionCoeffs": [I, D, D, DC, DC, D],                     # chemkin_wrapper.py:473
    "KINGetGasROP": [I, D, D, DC, DC],                                        # chemkin_wrapper.py:483
    "KINGetGasReactionRates": [I, D, D, DC, DC, DC],                          # chemkin_wrapper.py:491
    "KINGetReactionRateParameters": [I, DC, DC, DC],                          # chemkin_wrapper.py:500
    "KINSetAFactorForAReaction": [I, I, D],                                   # chemkin_wrapper.py:507
    "KINCalculateEquil": [I, D, D, DC, DC],                                   # chemkin_wrapper.py:514
    "KINCalculateEquilWithOption": [I, I, D, D, DC, DC],                      # chemkin_wrapper.py:522
    "KINCalculateEqGasWithOption": [I, I, I, D, D, DC, D, D, D, D, DC],       # chemkin_wrapper.py:531
    "KINRealGas_SetParameter": [C, D],                                        # chemkin_wrapper.py:546
    "KINRealGas_GetEOSMode": [I, I, C],                                       # chemkin_wrapper.py:551
    "KINRealGas_SetMixingRule": [I, I, I],                                    # chemkin_wrapper.py:557
    "KINRealGas_UseIdealGasLaw": [I, I],                                      # chemkin_wrapper.py:563
    "KINRealGas_UseCubicEOS": [I, I],                                         # chemkin_wrapper.py:568
    "KINRealGas_SetCurrentPressure": [I, D],                                  # chemkin_wrapper.py:573
    "KINRealGas_CheckRealGasStatus": [I, I],                                  # chemkin_wrapper.py:578
    "KINGetGamma": [I, D, DC, D],                                             # chemkin_wrapper.py:583
    "KINAll0D_Setup": [I, I, I, I, I, I, IC, I],                              # chemkin_wrapper.py:591
    "KINAll0D_SetupWorkArrays": [I, I],                                       # chemkin_wrapper.py:602
    "KINAll0D_SetupBatchInputs": [I, D, D, D, D, D, D, DC, DC, DC],           # chemkin_wrapper.py:607
    "KINAll0D_SetupPSRReactorInputs": [I, I, D, D, D, D, D, D, D, DC, DC, DC],# chemkin_wrapper.py:620
    "KINAll0D_SetupPSRInletInputs": [I, I, I, D, D, DC],                      # chemkin_wrapper.py:635
    "KINAll0D_SetupPFRInputs": [I, D, D, D, D, D, D, DC, DC, D, DC],          # chemkin_wrapper.py:644
    "KINAll0D_SetupHCCIInputs": [I, D, D, D, D, D, D, D, D, D, D, DC],        # chemkin_wrapper.py:658
    "KINAll0D_SetupHCCIZoneInputs": [I, I, D, D],                             # chemkin_wrapper.py:673
    "KINAll0D_SetupSIInputs": [I, D, D, D, D, D],                             # chemkin_wrapper.py:680
    "KINAll0D_Calculate": [I],                                                # chemkin_wrapper.py:689
    "KINAll0D_CalculateInput": [I, I, C, I, IC],                              # chemkin_wrapper.py:691
    "KINAll0D_SetUserKeyword": [C],                                           # chemkin_wrapper.py:699
    "KINAll0D_IntegrateHeatRelease": [],                                      # chemkin_wrapper.py:701
    "KINAll0D_SetHeatTransfer": [D, D],                                       # chemkin_wrapper.py:703
    "KINAll0D_SetHeatTransferArea": [D],                                      # chemkin_wrapper.py:708
    "KINAll0D_SetProfilePoints": [I],                                         # chemkin_wrapper.py:711
    "KINAll0D_SetProfileParameter": [C, I, DC, DC],                           # chemkin_wrapper.py:713
    "KINAll0D_SetProfileKeyword": [I, I, C, I, DC, DC],                       # chemkin_wrapper.py:720
    "KINAll0D_SetSolverInitialStepTime": [D],                                 # chemkin_wrapper.py:730
    "KINAll0D_SetSolverMaximumStepTime": [D],                                 # chemkin_wrapper.py:732
    "KINAll0D_SetSolverMaximumIteration": [I],                                # chemkin_wrapper.py:734
    "KINAll0D_SetRelaxIteration": [],                                         # chemkin_wrapper.py:736
    "KINAll0D_SetMinimumSpeciesBound": [D],                                   # chemkin_wrapper.py:738
    "KINAll0D_GetSolution": [D, D, DC],                                       # chemkin_wrapper.py:741
    "KINAll0D_GetSolnResponseSize": [I, I],                                   # chemkin_wrapper.py:747
    "KINAll0D_GetGasSolnResponse": [I, I, I, DC, DC, DC, DC, DF],             # chemkin_wrapper.py:752
    "KINAll0D_GetIgnitionDelay": [D],                                         # chemkin_wrapper.py:763
    "KINAll0D_GetHeatRelease": [D, D],                                        # chemkin_wrapper.py:765
    "KINAll0D_GetEngineHeatRelease": [DC, D, D, D, D, D],                     # chemkin_wrapper.py:770
    "KINAll0D_GetExitMassFlowRate": [D],                                      # chemkin_wrapper.py:779
    "KINPremix_SetParameter": [C, D],                                         # chemkin_wrapper.py:782
    "KINPremix_CalculateFlame": [I, I, D, D, DC, D, D],                       # chemkin_wrapper.py:787
    "KINPremix_GetSolution": [I, I, DC, DC, DF],                              # chemkin_wrapper.py:797
    "KINPremix_GetSolutionGridPoints": [I],                                   # chemkin_wrapper.py:805
    "KINPremix_GetFlameMassFlux": [D],                                        # chemkin_wrapper.py:809
    "KINOppdif_SetInlet": [C, I, D, DC, D, I],                                # chemkin_wrapper.py:818
    "KINOppdif_SetParameter": [C, D],                                         # chemkin_wrapper.py:826
    "KINOppdif_CalculateFlame": [I, I, D, D],                                 # chemkin_wrapper.py:831
    "KINOppdif_GetSolutionGridPoints": [I],                                   # chemkin_wrapper.py:837
    "KINOppdif_GetSolution": [I, I, D, D, ct.POINTER(D)],                     # chemkin_wrapper.py:838
    "KINOppdif_GetSolnSpeciesIntegratedROP": [I, I, I, I, ct.POINTER(D)],     # chemkin_wrapper.py:847
    "KINGetMassFractionFromMoleFraction": [I, DC, DC],                        # chemkin_wrapper.py:856
    "KINGetMoleFractionFromMassFraction": [I, DC, DC],                        # chemkin_wrapper.py:863
}


def header_kin_functions():
    src = open(os.path.join(ROOT, "include", "ckmi_kin.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:KIN|ckmi_kin_)\w+)\s*\(", src)))


def _lib():
    from pychemkin_amd import build

    L = ct.CDLL(build.build())
    for name, args in REFERENCE_ARGTYPES.items():
        fn = getattr(L, name)
        fn.restype = None if name == "KINFinish" else ct.c_int
        fn.argtypes = args
    L.ckmi_kin_last_error.restype = ct.c_char_p
    return L


def test_header_declares_every_reference_entry_point():
    declared = header_kin_functions()
    assert set(REFERENCE_ARGTYPES) <= set(declared)
    assert {"ckmi_kin_register", "ckmi_kin_release", "ckmi_kin_last_error"} <= set(declared)


def test_library_exports_kin_symbols():
    from pychemkin_amd import build

    out = subprocess.run(["nm", "-D", "--defined-only", build.build()], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (\w+)", out))
    missing = [f for f in header_kin_functions() if f not in exported]
    assert not missing, missing


def test_package_binding_matches_reference_prototypes():
    from pychemkin_amd import kin

    assert set(kin.KIN_PROTOTYPES) == set(REFERENCE_ARGTYPES)
    for name, args in REFERENCE_ARGTYPES.items():
        got = kin.KIN_PROTOTYPES[name][1]
        assert len(got) == len(args), name
        for a, b in zip(got, args):
            if hasattr(b, "_dtype_"):  # ndpointer: same dtype and flags
                assert a._dtype_ == b._dtype_ and a._flags_ == b._flags_, name
            else:
                assert a == b, name


def test_host_side_argument_checks():
    L = _lib()
    assert L.KINSetUnitSystem(ct.byref(ct.c_int(1))) == 0
    assert L.KINSetUnitSystem(ct.byref(ct.c_int(2))) != 0
    assert b"cgs" in L.ckmi_kin_last_error()
    bad = ct.c_int(77)
    assert L.KINInitialize(ct.byref(bad), ct.byref(ct.c_int(0))) != 0
    sizes = [ct.c_int(0) for _ in range(8)]
    assert L.KINGetChemistrySizes(ct.byref(bad), *[ct.byref(s) for s in sizes]) != 0
    assert L.KINAll0D_Setup(ct.byref(bad), *[ct.byref(ct.c_int(1)) for _ in range(5)], np.zeros(1, np.int32),
                            ct.byref(ct.c_int(0))) != 0
    assert b"chemistry set" in L.ckmi_kin_last_error()
    # the reactor state machine: no inputs, no keywords, no results
    assert L.KINAll0D_SetUserKeyword(b"ATOL    1e-20") != 0
    tau = ct.c_double(0.0)
    assert L.KINAll0D_GetIgnitionDelay(ct.byref(tau)) != 0
    n1, n2 = ct.c_int(0), ct.c_int(0)
    assert L.KINAll0D_GetSolnResponseSize(ct.byref(n1), ct.byref(n2)) != 0
    L.KINFinish()
