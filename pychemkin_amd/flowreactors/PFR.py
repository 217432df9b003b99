"""Plug-flow reactor (reference flowreactors/PFR.py), integrated by the batch-reactor kernels.

The reference sets up Chemkin's PLUG model through KINAll0D_Setup (reactor type 3) and
KINAll0D_SetupPFRInputs (PFR.py:498-512, 766-780, 1017-1031) and runs KINAll0D_Calculate.  Without
surface chemistry and at constant flow area a plug-flow reactor is a constant-pressure batch
reactor in the distance x: dy/dx = (rho / G) dy/dt with G = rho u the constant mass flux, the
pressure from the inviscid momentum equation P + G u = P0 + G u0 (MOMEN ON, PFR.py:146-149) or from
a PPRO profile (MOMEN OFF, PFR.py:515-518).  ckmi_reactor_run runs it as problem 3 (include/ckmi.h)
on the same wave- / workgroup-per-reactor kernels, so many tubes integrate in one launch.

Output follows the reference: the solution variable "time" is the distance [cm] (plugflow.py:63),
the saved points are 0, dx, 2 dx, ... up to the length with dx = DTSV u_inlet (the plugflow golden's
grid), get_ignition_delay() returns a distance [cm] (batchreactor.py:624-639).
Not on this path (rejected at run()): diameter / area profiles (DPRO, AFLO), wall heat transfer,
friction (VISC), surface chemistry (PSV), the velocity profile.
"""
from __future__ import annotations

import numpy as np

from .. import _native
from ..batchreactor import BatchReactors
from ..constants import R_GAS
from ..inlet import Stream
from ..logger import logger
from ..mixture import Mixture
from ..reactormodel import ReactorError

PFR_PROBLEM = 3  # ckmi_reactor_run problem code of a plug-flow reactor


class PlugFlowReactor(BatchReactors):
    """Generic plug-flow reactor (PFR.py:46-727)."""

    def __init__(self, inlet: Stream, label: str = "PFR"):
        if not isinstance(inlet, Stream):
            raise ReactorError("the first argument must be an Inlet (Stream) object")
        if inlet._flowratemode < 0:
            raise ReactorError("inlet flow rate is not set; please specify the flow rate of the Stream")
        super().__init__(inlet, label)
        self._reactortype = self.ReactorTypes["PFR"]
        self._problemtype = self.ProblemTypes["CONP"]
        self._startposition = 0.0
        self._length = 0.0
        self._diameter = 0.0
        self._flowarea = 0.0
        if inlet._haveflowarea:
            self._flowarea = inlet._flowarea
            self._diameter = float(np.sqrt(4.0 * self._flowarea / np.pi))
        self._absolute_tolerance = 1.0e-12
        self._relative_tolerance = 1.0e-6
        self._requiredlist = ["XEND", "AREAF"]

    # ------------------------------------------------------------------ geometry
    @property
    def length(self) -> float:
        """Reactor length (XEND) [cm]."""
        return self._length

    @length.setter
    def length(self, length: float = 0.0):
        if length <= 0.0:
            raise ReactorError("reactor length must > 0.0")
        self._length = float(length)

    def set_start_position(self, x0: float) -> None:
        """Start of the simulated section [cm] (PFR.py:182-203; must lie inside the reactor)."""
        if x0 >= self._length:
            raise ReactorError("starting position must < reactor length")
        if x0 < 0.0:
            raise ReactorError("starting position must >= 0")
        self._startposition = float(x0)

    @property
    def diameter(self) -> float:
        return self._diameter

    @diameter.setter
    def diameter(self, diam: float):
        if diam <= 0.0:
            raise ReactorError("reactor diameter must > 0.0")
        self._diameter = float(diam)
        self._flowarea = np.pi * diam * diam / 4.0
        self.reactormixture._haveflowarea = True
        self.reactormixture._flowarea = self._flowarea

    @property
    def flowarea(self) -> float:
        return self._flowarea

    @flowarea.setter
    def flowarea(self, area: float):
        if area <= 0.0:
            raise ReactorError("cross-sectional flow area must > 0.0")
        self._flowarea = float(area)
        self._diameter = float(np.sqrt(4.0 * area / np.pi))
        self.reactormixture._haveflowarea = True
        self.reactormixture._flowarea = self._flowarea

    def set_diameter_profile(self, x, diam) -> int:
        raise ReactorError("diameter profiles (DPRO) are not on the device path: constant flow area only")

    def set_flowarea_profile(self, x, area) -> int:
        raise ReactorError("flow-area profiles (AFLO) are not on the device path: constant flow area only")

    def set_inlet_viscosity(self, visc: float) -> None:
        raise ReactorError("wall friction (VISC) is not on the device path: inviscid momentum equation only")

    def set_pseudo_surface_velocity(self, vel: float) -> None:
        raise ReactorError("surface chemistry is not on the device path")

    def set_solver_max_timestep_size(self, size: float) -> None:
        """Largest solver step [cm] (DXMX, PFR.py:356-370)."""
        if size <= 0.0:
            raise ReactorError("solver maximum step size must > 0")
        self.setkeyword("STPT", float(size))

    # ------------------------------------------------------------------ inlet flow
    @property
    def mass_flowrate(self) -> float:
        return self.reactormixture.mass_flowrate

    @property
    def velocity(self) -> float:
        return self.reactormixture.velocity

    @property
    def vol_flowrate(self) -> float:
        return self.reactormixture.vol_flowrate

    @property
    def sccm(self) -> float:
        return self.reactormixture.sccm

    # ------------------------------------------------------------------ run
    def _save_grid(self, span: float, u0: float) -> np.ndarray:
        dtsv = self.getkeyword("DTSV")
        dx = float(dtsv) * u0 if dtsv is not None else span / 100.0
        n = int(np.floor(span / dx * (1.0 + 1e-12))) + 1
        return np.minimum(np.arange(n) * dx, span)

    def run(self) -> int:
        """Integrate the tube on the GPU (problem 3 of ckmi_reactor_run); 0 on success (PFR.py:627-727)."""
        if self._length <= 0.0:
            raise ReactorError("required input XEND (reactor.length) is not set")
        if self._flowarea <= 0.0:
            raise ReactorError("required input AREAF (reactor.diameter or reactor.flowarea) is not set")
        for key in self._profiles_index:
            if key not in ("PPRO", "TPRO"):
                raise ReactorError(f"{key} profiles are not supported on a plug-flow reactor on the device path")
        if (self._heat_loss_rate != 0.0 or self.getkeyword("QLOS") is not None or self.getkeyword("HTC") is not None
                or self.getprofile("QPRO") is not None or self.getprofile("AEXT") is not None):
            raise ReactorError("wall heat transfer of a plug-flow reactor is not on the device path")
        span = self._length - self._startposition
        self._endtime = span
        mix = self.reactormixture
        u0 = float(mix.velocity)
        cfg = self.reactor_cfg()  # PPRO (in x: the momentum equation is then off) or TPRO(x) as for CONP
        for i in range(cfg.nprof):  # the kernel integrates in x - x0; profile abscissae are absolute positions
            cfg.prof_t[i] -= self._startposition
        dm = self._chem.device_mechanism()
        xs = self._save_grid(span, u0)
        res = dm.reactor_run(cfg, np.array([PFR_PROBLEM], np.int32), np.array([mix.temperature]),
                             np.array([mix.pressure]), np.array([u0]), mix.Y.reshape(1, -1), t_save=xs)
        stats = res["stats"].cpu().numpy()[0]
        self._stats = dict(zip(_native.STAT_NAMES, stats.tolist()))
        status = int(stats[6])
        self._tau = float(res["tau"][0].item())
        self._final = dict(T=float(res["T"][0].item()), P=float(res["P"][0].item()), V=float(res["V"][0].item()),
                           Y=res["Y"][0].cpu().numpy())
        ys = res["y_save"][0].cpu().numpy()
        keep = ~np.isnan(ys[:, 0])
        self._raw = (xs[keep], ys[keep])
        self._u0 = u0
        self._solution_rawarray = {}
        self._solution_mixturearray = []
        self._numbsolutionpoints = 0
        self.setrunstatus(status)
        if status != 0:
            logger.critical("reactor %s failed: %s", self.label, _native.RUN_STATUS.get(status, status))
        return status

    def get_ignition_delay(self) -> float:
        """Ignition distance [cm] from the inlet of the simulated section (batchreactor.py:624-639)."""
        if self.runstatus != 0 or self._tau is None:
            return 0.0
        if self._tau <= 0.0:
            logger.warning("potential bad ignition distance value")
            return self._tau
        return self._startposition + self._tau

    def _PV_of(self, x: np.ndarray, T: np.ndarray, Y: np.ndarray):
        """Pressure and velocity along the tube (the kernel's momentum equation, or the PPRO profile)."""
        mix0 = self.reactormixture
        Wbar = 1.0 / (Y / mix0.WT).sum(axis=1)
        pp = self.getprofile("PPRO")
        # mass flux mdot / A = the inlet density (at the inlet pressure) x u0, with or without PPRO
        G = mix0.pressure * mix0.WTM / (R_GAS * mix0.temperature) * self._u0
        if pp is not None:
            P = np.interp(x + self._startposition, pp.x, pp.y)  # x from the start position; pp.x absolute
        else:
            Pm = mix0.pressure + G * self._u0
            P = 0.5 * (Pm + np.sqrt(np.maximum(Pm * Pm - 4.0 * G * G * R_GAS * T / Wbar, 0.0)))  # choked: status 5
        u = G / (P * Wbar / (R_GAS * T))
        return P, u

    def process_solution(self) -> None:
        """Raw solution arrays and solution mixtures along the tube (batchreactor.py:1335-1435)."""
        if self.runstatus != 0:
            raise ReactorError("please run the reactor successfully first")
        xs, ys = self._raw
        T, Y = ys[:, 0], ys[:, 1:]
        P, u = self._PV_of(xs, T, Y)
        x = self._startposition + xs
        self._numbsolutionpoints = len(xs)
        self._solution_rawarray = {"time": x.copy(), "distance": x.copy(), "temperature": T.copy(), "pressure": P,
                                   "velocity": u, "volume": u}
        for k, sp in enumerate(self._specieslist):
            self._solution_rawarray[sp] = Y[:, k].copy()
        self._solution_mixturearray = []
        for i in range(len(xs)):
            m = Mixture(self._chem)
            m.temperature = T[i]
            m.pressure = P[i]
            m.Y = np.maximum(Y[i], 0.0)
            self._solution_mixturearray.append(m)


class PlugFlowReactor_EnergyConservation(PlugFlowReactor):
    """Adiabatic plug-flow reactor with the energy equation (PFR.py:730-980; no wall heat loss here)."""

    def __init__(self, inlet: Stream, label: str = "PFR"):
        super().__init__(inlet, label)
        self._energytype = self.EnergyTypes["ENERGY"]


class PlugFlowReactor_FixedTemperature(PlugFlowReactor):
    """Plug-flow reactor at the inlet temperature or a TPRO(x) profile (PFR.py:983-1067)."""

    def __init__(self, inlet: Stream, label: str = "PFR"):
        super().__init__(inlet, label)
        self._energytype = self.EnergyTypes["GivenT"]
