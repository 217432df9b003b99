"""Generic engine cylinder (reference engines/engine.py:41-1203) on the batch-reactor kernels.

The reference hands the engine geometry to Chemkin's closed library (KINAll0D_SetupHCCIInputs,
HCCI.py:1105-1125; the wall heat-transfer and gas-velocity keywords ICHX / GVEL / CYBAR / PSBAR /
POLEN, engine.py:490-924) and runs KINAll0D_Calculate.  Here the cylinder is problem 4 of
ckmi_reactor_run (include/ckmi.h): a closed reactor whose volume follows the slider-crank of the
CKMI_ENG_* parameter block, integrated by the wave-per-reactor kernel, many cylinders per launch.

Kinematics (pinned by the hcciengine golden's volume column to 1e-14): piston-pin offset e = -POLEN,
crank angle counted from the offset engine's top dead centre, clearance volume from the actual
stroke.  get_displacement_volume() / get_clearance_volume() return the reference's nominal values
(stroke x bore area, engine.py:570-602) as the reference does.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from ..batchreactor import BatchReactors
from ..constants import R_GAS
from ..logger import logger
from ..reactormodel import ReactorError

ENGINE_PROBLEM = 4  # ckmi_reactor_run problem code of an engine cylinder
HT_MODELS = {"dimensionless": 1}  # ICHX; "dimensional" (ICHW) and "hohenburg" (ICHH) are not on the device path


class Engine(BatchReactors):
    """Engine cylinder parameters and crank-angle bookkeeping (engine.py:41-1203)."""

    def __init__(self, reactor_condition, label: str):
        super().__init__(reactor_condition, label)
        self._numstroke = 4
        self.borediam = 0.0
        self.borearea = 0.0
        self.enginestroke = 0.0
        self.crankradius = 0.0
        self.connectrodlength = 0.0
        self.pistonoffset = 0.0
        self.cylinderheadarea = 0.0
        self.pistonheadarea = 0.0
        self.headareas = 0.0
        self.compressratio = 1.0
        self.enginespeed = 1.0
        self.degpersec = 0.0
        self.radpersec = 0.0
        self.IVCCA = -180.0
        self.EVOCA = 180.0
        self.rundurationCA = 360.0
        self.heattransfermodel: int = -1
        self.heattransferparameters: List[float] = []
        self.cylinderwalltemperature = 298.15
        self.gasvelocity: List[float] = []
        self.HuberIMEP: Optional[float] = None
        self._wallheattransfer = False
        self._inputcheck: List[str] = []
        self._degsave: Optional[float] = None
        self._degprint: Optional[float] = None

    # ------------------------------------------------------------------ crank angle <-> time
    @staticmethod
    def convert_CA_to_Time(CA: float, startCA: float, RPM: float) -> float:
        if RPM <= 0.0:
            raise ReactorError("engine speed RPM must > 0.")
        t = (CA - startCA) / RPM / 6.0
        if t < 0.0:
            raise ReactorError("given CA is less then the starting CA @ IVC.")
        return t

    @staticmethod
    def convert_Time_to_CA(time: float, startCA: float, RPM: float) -> float:
        if time < 0.0:
            raise ReactorError("simulation time must > 0.")
        return startCA + time * RPM * 6.0

    def get_Time(self, CA: float) -> float:
        return (CA - self.IVCCA) / self.degpersec

    def get_CA(self, time: float) -> float:
        return self.IVCCA + time * self.degpersec

    # ------------------------------------------------------------------ parameters
    @property
    def starting_CA(self) -> float:
        return self.IVCCA

    @starting_CA.setter
    def starting_CA(self, startCA: float):
        self.IVCCA = float(startCA)
        self.rundurationCA = self.EVOCA - self.IVCCA
        self._inputcheck.append("DEG0")

    @property
    def ending_CA(self) -> float:
        return self.EVOCA

    @ending_CA.setter
    def ending_CA(self, endCA: float):
        if endCA <= self.starting_CA:
            raise ReactorError(f"ending CA must > starting CA = {self.starting_CA}")
        self.EVOCA = float(endCA)
        self.rundurationCA = self.EVOCA - self.IVCCA
        self._inputcheck.append("DEGE")

    @property
    def duration_CA(self) -> float:
        return self.rundurationCA

    @duration_CA.setter
    def duration_CA(self, CA: float):
        if CA <= 0.0:
            raise ReactorError("duration CA must > 0.")
        self.rundurationCA = float(CA)
        self.EVOCA = self.IVCCA + CA
        self._inputcheck.append("DEGE")

    @property
    def bore(self) -> float:
        return self.borediam

    @bore.setter
    def bore(self, diameter: float):
        if diameter <= 0.0:
            raise ReactorError("engine bore diameter must > 0.")
        self.borediam = float(diameter)
        self.borearea = np.pi * diameter * diameter / 4.0
        self._inputcheck.append("BORE")

    @property
    def stroke(self) -> float:
        return self.enginestroke

    @stroke.setter
    def stroke(self, s: float):
        if s <= 0.0:
            raise ReactorError("piston stroke must > 0.")
        self.enginestroke = float(s)
        self.crankradius = s / 2.0
        self._inputcheck.append("STRK")

    @property
    def connecting_rod_length(self) -> float:
        return self.connectrodlength

    @connecting_rod_length.setter
    def connecting_rod_length(self, s: float):
        if s <= 0.0:
            raise ReactorError("piston connecting rod length must > 0.")
        self.connectrodlength = float(s)
        self._inputcheck.append("CRLEN")

    @property
    def compression_ratio(self) -> float:
        return self.compressratio

    @compression_ratio.setter
    def compression_ratio(self, cratio: float):
        if cratio <= 1.0:
            raise ReactorError("engine compression ratio must > 1.")
        self.compressratio = float(cratio)
        self._inputcheck.append("CMPR")

    @property
    def RPM(self) -> float:
        return self.enginespeed

    @RPM.setter
    def RPM(self, speed: float):
        if speed <= 0.0:
            raise ReactorError("engine speed RPM must > 0.")
        self.enginespeed = float(speed)
        self.degpersec = speed * 6.0
        self.radpersec = self.degpersec * np.pi / 180.0
        self._inputcheck.append("RPM")

    def set_cylinder_head_area(self, area: float):
        if area <= 0.0:
            raise ReactorError("cylinder head surface area must > 0.")
        if "BORE" not in self._inputcheck:
            raise ReactorError("please set cylinder BORE diameter first.")
        self.cylinderheadarea = float(area)
        self.headareas = area + self.pistonheadarea

    def set_piston_head_area(self, area: float):
        if area <= 0.0:
            raise ReactorError("piston head surface area must > 0.")
        if "BORE" not in self._inputcheck:
            raise ReactorError("please set cylinder BORE diameter first.")
        self.pistonheadarea = float(area)
        self.headareas = area + self.cylinderheadarea

    def set_piston_pin_offset(self, offset: float):
        if offset >= self.crankradius:
            raise ReactorError(f"piston pin offset distance must < crank radius {self.crankradius} [cm]")
        self.pistonoffset = float(offset)

    def get_clearance_volume(self) -> float:
        if "CMPR" not in self._inputcheck:
            raise ReactorError("please set engine compression ratio first.")
        return self.get_displacement_volume() / (self.compressratio - 1.0)

    def get_displacement_volume(self) -> float:
        return self.enginestroke * self.borearea

    def list_engine_parameters(self):
        """Print the cylinder geometry and operating point, one quantity per line."""
        rows = (("bore", self.borediam, "cm"), ("stroke", self.enginestroke, "cm"),
                ("rod length", self.connectrodlength, "cm"), ("head area", self.cylinderheadarea, "cm2"),
                ("piston area", self.pistonheadarea, "cm2"), ("pin offset", self.pistonoffset, "cm"),
                ("CMPR", self.compressratio, "-"), ("speed", self.enginespeed, "rpm"),
                ("IVC", self.IVCCA, "deg CA"), ("EVO", self.EVOCA, "deg CA"))
        print("engine:")
        for name, value, unit in rows:
            print(f"  {name:<12s} {value:>14.6g}  {unit}")

    @property
    def CAstep_for_saving_solution(self) -> float:
        return self._degsave if self._degsave is not None else self.rundurationCA / 100.0

    @CAstep_for_saving_solution.setter
    def CAstep_for_saving_solution(self, delta_CA: float):
        if delta_CA <= 0.0:
            raise ReactorError("solution saving CA interval must > 0.")
        self._degsave = float(delta_CA)

    @property
    def CAstep_for_printing_solution(self) -> float:
        return self._degprint if self._degprint is not None else self.rundurationCA / 100.0

    @CAstep_for_printing_solution.setter
    def CAstep_for_printing_solution(self, delta_CA: float):
        """Text-output interval: accepted, no text output on the device path."""
        if delta_CA <= 0.0:
            raise ReactorError("solution printing CA interval must > 0.")
        self._degprint = float(delta_CA)

    def set_wall_heat_transfer(self, model: str, HTparameters: List[float], walltemperature: float):
        """ICHX "dimensionless" Nu = a Re^b Pr^c (engine.py:766-839); ICHW / ICHH are rejected."""
        mymodel = model.lower().rstrip()
        if mymodel not in HT_MODELS:
            raise ReactorError(f"engine wall heat transfer model {model!r} is not on the device path "
                               "(only 'dimensionless', ICHX)")
        if len(HTparameters) != 3:
            raise ReactorError(f"{model} requires 3 parameters <a> <b> <c>")
        self.heattransfermodel = 0
        self.heattransferparameters = [float(x) for x in HTparameters]
        self.cylinderwalltemperature = float(walltemperature)
        self._wallheattransfer = True

    def set_gas_velocity_correlation(self, gasvelparameters: List[float], IMEP: Optional[float] = None):
        """Woschni GVEL <C11> <C12> <C2> <swirl ratio> (engine.py:841-896); the Huber IMEP form is rejected."""
        if self.heattransfermodel < 0:
            raise ReactorError("please specify the wall heat transfer model first.")
        if len(gasvelparameters) != 4:
            raise ReactorError("gas velocity correlation requires 4 parameters <C11> <C12> <C2> <swirl ratio>")
        if IMEP is not None:
            raise ReactorError("the Huber IMEP gas velocity correlation (HIMP) is not on the device path")
        self.gasvelocity = [float(x) for x in gasvelparameters]

    # ------------------------------------------------------------------ device configuration
    def validate_inputs(self) -> int:
        missing = [k for k in ("DEG0", "DEGE", "RPM", "CMPR", "BORE", "STRK", "CRLEN") if k not in self._inputcheck]
        if missing:
            raise ReactorError(f"missing required engine inputs: {missing}")
        return 0

    def engine_block(self) -> np.ndarray:
        """The CKMI_ENG_* parameter block (include/ckmi.h) of this cylinder."""
        e = np.zeros(20)
        e[0:7] = [self.IVCCA, self.enginespeed, self.compressratio, self.borediam, self.enginestroke,
                  self.connectrodlength / self.crankradius, self.pistonoffset]
        if self._wallheattransfer:
            gv = self.gasvelocity or [2.28, 0.308, 3.24, 0.0]  # Woschni's constants when GVEL is absent
            e[7] = 1.0
            e[8:11] = self.heattransferparameters
            e[11] = self.cylinderwalltemperature
            e[12:16] = gv
            # CYBAR / PSBAR default to 1 (the head areas equal the bore area, ChemkinKeywordTips.yaml:429-436)
            e[16] = self.cylinderheadarea / self.borearea if self.cylinderheadarea > 0.0 else 1.0
            e[17] = self.pistonheadarea / self.borearea if self.pistonheadarea > 0.0 else 1.0
        return e

    def save_times(self) -> np.ndarray:
        """Solution points every CAstep_for_saving_solution degrees from IVC to EVO (both included)."""
        dca = self.CAstep_for_saving_solution
        n = int(np.floor(self.rundurationCA / dca * (1.0 + 1e-12))) + 1
        ca = np.minimum(self.IVCCA + np.arange(n) * dca, self.EVOCA)
        if ca[-1] < self.EVOCA * (1.0 - 1e-15) - 1e-12:
            ca = np.append(ca, self.EVOCA)
        return (ca - self.IVCCA) / self.degpersec

    def get_engine_heat_release_rates(self) -> dict:
        """Heat rates per crank-angle degree on the saved solution points (extension: the profiles behind
        the scalars of KINAll0D_GetEngineHeatRelease, engine.py:953-988).

        Returns a dict of arrays over the solution points: ``CA`` [degree]; ``AHRR`` the apparent heat-
        release rate m c_v dT/dCA + P dV/dCA [erg/degree] from the integrator's own right-hand side on the
        device (chemical heat release net of the wall loss); ``AHRRP`` the same from the pressure trace
        with a constant gamma (that of the charge at IVC), gamma/(gamma-1) P dV/dCA + 1/(gamma-1) V dP/dCA
        (central differences on the saved points); ``QLossRateCA`` the wall heat-loss rate hA (T - T_wall)
        [erg/degree] (0 for an adiabatic cylinder)."""
        if self.runstatus != 0:
            raise ReactorError("no successful engine run")
        ts, ys = self._raw
        mix0 = self.reactormixture
        dm = self._chem.device_mechanism()
        ahrr, qloss = dm.engine_heat_rates(self.reactor_cfg(), mix0.temperature, mix0.pressure, mix0.Y, ts, ys)
        ca = self.IVCCA + ts * self.degpersec
        P, V = self._PV_of(ts, ys[:, 0], ys[:, 1:])
        gamma = mix0.CPBL() / (mix0.CPBL() - R_GAS)  # cp / cv of the charge (molar cp)
        dP, dV = np.gradient(P, ca), np.gradient(V, ca)
        ahrrp = gamma / (gamma - 1.0) * P * dV + 1.0 / (gamma - 1.0) * V * dP
        return {"CA": ca, "AHRR": ahrr.cpu().numpy() / self.degpersec, "AHRRP": ahrrp,
                "QLossRateCA": qloss.cpu().numpy() / self.degpersec}

    def get_engine_heat_release_CAs(self):
        """Crank angles of 10 / 50 / 90 % of the cumulative chemical heat release (engine.py:953-988).
        Heat release = -m sum_k h_k(298.15 K) (Y_k(t) - Y_k(0)), the standard-state heat of the reactions
        run so far, on the saved solution points (linear interpolation of the crossing)."""
        if self.runstatus != 0:
            return 0.0, 0.0, 0.0
        ts, ys = self._raw
        hk = self._chem.SpeciesH(298.15) / self._chem.WT  # erg/g
        q = -(ys[:, 1:] - ys[0, 1:]) @ hk
        if q[-1] <= 0.0:
            logger.warning("no net heat release in the engine solution")
            return self.IVCCA, self.IVCCA, self.IVCCA
        frac = q / q[-1]
        out = []
        for level in (0.1, 0.5, 0.9):
            i = int(np.argmax(frac >= level))
            if i == 0:
                out.append(self.get_CA(ts[0]))
                continue
            w = (level - frac[i - 1]) / (frac[i] - frac[i - 1])
            out.append(self.get_CA(ts[i - 1] + w * (ts[i] - ts[i - 1])))
        return tuple(out)
