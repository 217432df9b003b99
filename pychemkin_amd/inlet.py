"""Inlet stream: a Mixture with a flow rate (reference inlet.py:42-460).

Drop-in subset used by the plug-flow reactor (flowreactors/PFR.py): one of mass flow rate [g/s],
volumetric flow rate [cm3/s], velocity [cm/s] (with a flow area) or SCCM, converted to the others
at the stream's state as inlet.py:86-236 does (SCCM at 298.15 K and 1 atm).
"""
from __future__ import annotations

from .chemistry import Chemistry
from .constants import P_ATM, R_GAS
from .mixture import Mixture, MixtureError


class Stream(Mixture):
    """Inlet stream of an open reactor model."""

    def __init__(self, chem: Chemistry, label: str = None):
        super().__init__(chem)
        self._flowratemode = -1  # 0 mass flow rate, 1 volumetric flow rate, 2 velocity, 3 SCCM
        self._inletflowrate = [0.0] * 4
        self._haveflowarea = False
        self._flowarea = 1.0
        self._label = label or "inlet"

    @property
    def label(self) -> str:
        return self._label

    # ------------------------------------------------------------------ conversions
    def _standard_density(self) -> float:
        """Density at 298.15 K and 1 atm (the SCCM reference state, inlet.py:100-110)."""
        return P_ATM * self.WTM / (R_GAS * 298.15)

    def convert_to_mass_flowrate(self) -> float:
        m = self._flowratemode
        if m == 0:
            return self._inletflowrate[0]
        if m == 1:
            return self.RHO * self._inletflowrate[1]
        if m == 2:
            if not self._haveflowarea:
                raise MixtureError("flow area is not given for this inlet")
            return self.RHO * self._flowarea * self._inletflowrate[2]
        if m == 3:
            return self._standard_density() * self._inletflowrate[3] / 60.0
        raise MixtureError("the inlet flow rate is not set")

    def convert_to_vol_flowrate(self) -> float:
        return self.convert_to_mass_flowrate() / self.RHO

    def convert_to_SCCM(self) -> float:
        return self.convert_to_mass_flowrate() / self._standard_density() * 60.0

    # ------------------------------------------------------------------ properties
    @property
    def flowarea(self) -> float:
        if not self._haveflowarea:
            raise MixtureError("flow area is not given for this inlet")
        return self._flowarea

    @flowarea.setter
    def flowarea(self, farea: float):
        if farea <= 0.0:
            raise MixtureError("flow area must be > 0")
        self._flowarea = float(farea)
        self._haveflowarea = True

    @property
    def mass_flowrate(self) -> float:
        """Mass flow rate [g/s]."""
        return self.convert_to_mass_flowrate()

    @mass_flowrate.setter
    def mass_flowrate(self, mflowrate: float):
        if mflowrate <= 0.0:
            raise MixtureError("mass flow rate must be > 0")
        self._flowratemode = 0
        self._inletflowrate[0] = float(mflowrate)

    @property
    def vol_flowrate(self) -> float:
        """Volumetric flow rate [cm3/s]."""
        return self.convert_to_vol_flowrate()

    @vol_flowrate.setter
    def vol_flowrate(self, vflowrate: float):
        if vflowrate <= 0.0:
            raise MixtureError("volumetric flow rate must be > 0")
        self._flowratemode = 1
        self._inletflowrate[1] = float(vflowrate)

    @property
    def sccm(self) -> float:
        """Volumetric flow rate at 298.15 K and 1 atm [standard cm3/min]."""
        return self.convert_to_SCCM()

    @sccm.setter
    def sccm(self, vflowrate: float):
        if vflowrate <= 0.0:
            raise MixtureError("SCCM must be > 0")
        self._flowratemode = 3
        self._inletflowrate[3] = float(vflowrate)

    @property
    def velocity(self) -> float:
        """Gas velocity [cm/s] (needs the flow area unless given directly)."""
        if self._flowratemode == 2:
            return self._inletflowrate[2]
        return self.convert_to_mass_flowrate() / (self.RHO * self.flowarea)

    @velocity.setter
    def velocity(self, vel: float):
        if vel <= 0.0:
            raise MixtureError("velocity must be > 0")
        self._flowratemode = 2
        self._inletflowrate[2] = float(vel)
