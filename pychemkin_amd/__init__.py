"""pychemkin_amd -- MI355X-native batched batch-reactor engine with a PyChemkin-compatible API.

Drop-in names for the reference's batch-reactor path (``ansys.chemkin``, __init__.py:37-81):
Chemistry, Mixture, the four closed-homogeneous batch reactors, constants, logger, the inlet Stream
and the plug-flow reactors (``pychemkin_amd.flowreactors.PFR``, on the same kernels); plus the
batched entry point BatchSweep.  Numerics run in hand-written gfx950 HIP kernels
(libckmi.so, include/ckmi.h).  Units are cgs as the reference sets with KINSetUnitSystem(1).
"""
from .batch import BatchResult, BatchSweep, afactor_sensitivity
from .batchreactor import (
    BatchReactors,
    GivenPressureBatchReactor_EnergyConservation,
    GivenPressureBatchReactor_FixedTemperature,
    GivenVolumeBatchReactor_EnergyConservation,
    GivenVolumeBatchReactor_FixedTemperature,
)
from .chemistry import Chemistry, chemkin_version, done, set_verbose, verbose
from .constants import (
    AVOGADRO,
    BOLTZMANN,
    ERGS_PER_CALORIE,
    ERGS_PER_JOULE,
    JOULES_PER_CALORIE,
    P_ATM,
    P_TORRS,
    R_GAS,
    R_GAS_CAL,
    Air,
    air,
)
from .inlet import Stream
from .logger import logger
from .mixture import (Mixture, adiabatic_mixing, calculate_mixture_temperature_from_enthalpy, interpolate_mixtures,
                      isothermal_mixing)
from .reactormodel import Keyword, Profile

__version__ = "0.1.0"

_IGNITION_DEFINITIONS = """ignition delay definitions (ChemkinKeywordTips.yaml:184-199):
  'T_inflection' : TIFP   time of the temperature inflection point (max dT/dt)
  'T_rise'       : DTIGN  time when T exceeds T0 + val
  'T_ignition'   : TLIM   time when T exceeds val
  'Species_peak' : KLIM   time of the peak of the target species"""


def show_ignition_definitions() -> None:
    print(_IGNITION_DEFINITIONS)
