"""Single-zone HCCI engine (reference engines/HCCI.py:44-1340) on the wave-per-reactor kernel.

The reference sets the cylinder up with KINAll0D_Setup (reactor type HCCI, problem ICEN) and
KINAll0D_SetupHCCIInputs (HCCI.py:1105-1125) and runs KINAll0D_Calculate.  Here run() sends the
cylinder to ckmi_reactor_run as problem 4 with the engine parameter block and the transport fits
(include/ckmi.h): volume from the slider-crank, energy equation with the ICHX / Woschni wall heat
transfer (engine.py:766-924).  Multi-zone engines (nzones > 1) are not on the device path.

Parity (tests/test_engine.py): the hcciengine golden's volume column to 1e-14 and density column to
1e-8; its pressure only in part: the published ICHX / Woschni form loses about 1.2x the golden's
wall heat during compression (the golden lies between the adiabatic cylinder and this one), so the
pressure stays within the golden's 1e-4 until about -110 CA and peaks 3 CA late.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..constants import R_GAS
from ..reactormodel import ReactorError
from .engine import ENGINE_PROBLEM, Engine


def engine_volume(eng: np.ndarray, t: np.ndarray) -> np.ndarray:
    """V(t) [cm3] of the CKMI_ENG_* block (the kernel's engine_volume, ckmi_reactor.hpp)."""
    B, a = eng[3], 0.5 * eng[4]
    L, e = eng[5] * a, -eng[6]
    Ab = 0.25 * np.pi * B * B
    st, sb = np.sqrt((L + a) ** 2 - e * e), np.sqrt((L - a) ** 2 - e * e)
    Vc = Ab * (st - sb) / (eng[2] - 1.0)
    th = np.radians(eng[0] + 6.0 * eng[1] * np.asarray(t, np.float64)) + np.arcsin(e / (L + a))
    return Vc + Ab * (st - (a * np.cos(th) + np.sqrt(L * L - (a * np.sin(th) - e) ** 2)))


class HCCIengine(Engine):
    """Homogeneous charge compression ignition engine, single zone (HCCI.py:44-1340)."""

    def __init__(self, reactor_condition, label: str = "", nzones: Optional[int] = None):
        nzones = 1 if nzones is None else int(nzones)
        if nzones != 1:
            raise ReactorError("multi-zone HCCI engines are not on the device path (nzones must be 1)")
        super().__init__(reactor_condition, label or "HCCI")
        self._reactortype = self.ReactorTypes["HCCI"]
        # ckmi_reactor_run's engine problem code (the reference's ICEN problem type)
        self._problemtype = ENGINE_PROBLEM
        self._energytype = self.EnergyTypes["ENERGY"]
        self._nzones = 1

    def get_number_of_zones(self) -> int:
        return self._nzones

    # ------------------------------------------------------------------ run
    def reactor_cfg(self):
        if (self._heat_loss_rate != 0.0 or self.getkeyword("QLOS") is not None or self.getkeyword("HTC") is not None
                or self._profiles_index):
            raise ReactorError("QLOS / HTC / profiles do not apply to an engine cylinder: use set_wall_heat_transfer")
        cfg = super().reactor_cfg()
        eng = self.engine_block()
        for i, v in enumerate(eng):
            cfg.eng[i] = float(v)
        if self._wallheattransfer:
            import torch

            dm = self._chem.device_mechanism()
            fits = np.hstack([self._chem.viscosity_fits, self._chem.conductivity_fits])
            tran = torch.tensor(fits, dtype=torch.float64, device=dm.device)
            cfg.tran = tran.data_ptr()
            cfg._tran_keep = tran
        return cfg

    def run(self) -> int:
        """Integrate the cylinder from IVC to EVO on the GPU (HCCI.py:1241-1340); 0 on success."""
        self.validate_inputs()
        if self._chem.KK + 1 > 64:
            raise ReactorError("engine cylinders need a mechanism of at most 63 species (wave-per-reactor kernel)")
        if self._wallheattransfer and not self._chem.verify_transport_data():
            raise ReactorError("wall heat transfer needs transport data: set chemistry.tranfile before preprocess")
        self._endtime = self.rundurationCA / self.degpersec
        self.timestep_for_saving_solution = self.CAstep_for_saving_solution / self.degpersec
        return super().run()

    def get_ignition_delay(self) -> float:
        """Ignition crank angle [degree] (TIFP etc. in CA, HCCI.py / batchreactor.py:545-642)."""
        if self.runstatus != 0 or self._tau is None:
            return 0.0
        if self._tau <= 0.0:
            return self._tau
        return self.get_CA(self._tau)

    def _PV_of(self, t: np.ndarray, T: np.ndarray, Y: np.ndarray):
        mix0 = self.reactormixture
        eng = self.engine_block()
        V = engine_volume(eng, t)
        V0 = float(engine_volume(eng, np.array([0.0]))[0])
        Wbar = 1.0 / (Y / mix0.WT).sum(axis=1)
        rho = mix0.RHO * V0 / V
        return rho * R_GAS * T / Wbar, V

    def process_engine_solution(self, zoneID: Optional[int] = None) -> None:
        """Solution arrays and mixtures of the (single) zone (engine.py:1067-1193)."""
        if zoneID not in (None, 0, 1):
            raise ReactorError("single-zone engine: zoneID must be 1 (or None)")
        self.process_solution()

    def process_average_engine_solution(self) -> None:
        self.process_solution()
