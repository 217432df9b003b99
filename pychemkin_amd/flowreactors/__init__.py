"""Open flow reactors (reference flowreactors/): the plug-flow reactor on the batch-reactor kernels."""
from .PFR import PlugFlowReactor, PlugFlowReactor_EnergyConservation, PlugFlowReactor_FixedTemperature

__all__ = ["PlugFlowReactor", "PlugFlowReactor_EnergyConservation", "PlugFlowReactor_FixedTemperature"]
