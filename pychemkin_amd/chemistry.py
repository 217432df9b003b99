"""Chemistry set: mechanism load and mechanism-level getters (reference chemistry.py).

Drop-in for the reference's ``Chemistry`` on the batch-reactor path:
  chemfile / thermfile / tranfile / surffile   file names (chemistry.py:353-501)
  preprocess()           KINPreProcess + size/name/weight getters (chemistry.py:595-753);
                         here the host parser builds the flat tables (mechanism.py) and the
                         device tables are created lazily on first GPU use
  KK, MM, IIGas, species_symbols, element_symbols, WT, AWT, get_specindex
  SpeciesCp/Cv/H/U       NASA-7 per species in erg/mol(-K), evaluated by the
                         ckmi_species_thermo kernel (chemistry.py:1069-1314)
  SpeciesComposition     NCF element counts (chemistry.py:1472-1522)
  get_reaction_parameters / set_reaction_AFactor / get_reaction_AFactor (1-based, as the
                         reference, chemistry.py:1604-1724), get_gas_reaction_string
  tranfile / preprocess_transportdata / verify_transport_data   transport data read at
                         preprocess (chemistry.py:402-480,636-687,794-808): viscosity fits for
                         Mixture.mixture_viscosity / species_Visc (transport.py)
Deviations: errors raise exceptions instead of exit(); get_specindex
accepts index 0 (H2 in GRI-3.0); real-gas EOS is not supported (ideal gas only).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np

from . import device as _device
from . import transport as _transport
from .constants import R_GAS
from .logger import logger
from .mechanism import Mechanism

_verbose = False
_chemistry_sets: Dict[int, "Chemistry"] = {}
_active_chemistry_set = -1


def verbose() -> bool:
    return _verbose


def set_verbose(OnOff: bool) -> None:
    global _verbose
    _verbose = bool(OnOff)


def chemkin_version() -> int:
    """Version of this engine (the reference reports the Ansys release, chemistry.py:84)."""
    return 252


def done() -> None:
    """Release all device mechanisms (reference: KINFinish, chemistry.py:126)."""
    for c in list(_chemistry_sets.values()):
        _device.drop(c)
    _chemistry_sets.clear()


def check_active_chemistryset(chem_index: int) -> bool:
    return chem_index == _active_chemistry_set


class ChemistryError(RuntimeError):
    pass


class Chemistry:
    """A Chemkin chemistry set (gas phase)."""

    realgas_CuEOS = ["ideal gas"]

    def __init__(self, chem: str = "", surf: str = "", therm: str = "", tran: str = "", label: str = ""):
        self._chemfile = chem
        self._thermfile = therm
        self._tranfile = tran
        self._surffile = surf
        self.label = label
        self._chemset_index = -1
        self._mech: Optional[Mechanism] = None
        self._version = 0
        self.userealgas = False
        self._inline_transport = False
        self._tran_params: Optional[np.ndarray] = None  # [KK][6] TRANLIB parameters
        self._vfits: Optional[np.ndarray] = None        # [KK][4] viscosity fits

    def __deepcopy__(self, memo):
        # chemistry sets are shared, global objects in the reference (chemistry.py:46-51)
        return self

    # ------------------------------------------------------------------ files
    @property
    def chemfile(self) -> str:
        return self._chemfile

    @chemfile.setter
    def chemfile(self, filename: str):
        self._chemfile = filename

    @property
    def thermfile(self) -> str:
        return self._thermfile

    @thermfile.setter
    def thermfile(self, filename: str):
        self._thermfile = filename

    @property
    def tranfile(self) -> str:
        return self._tranfile

    @tranfile.setter
    def tranfile(self, filename: str):
        self._tranfile = filename

    def preprocess_transportdata(self) -> None:
        """Process the transport data: the ``tranfile``, or without one the ``TRANSPORT ALL`` block of
        the mechanism file (chemistry.py:450-480)."""
        self._inline_transport = True

    def verify_transport_data(self) -> bool:
        """True once transport data have been processed (chemistry.py:794-808)."""
        return self._vfits is not None

    @property
    def transport_parameters(self) -> np.ndarray:
        """[KK][6] TRANLIB parameters (geometry, eps/k, sigma, dipole, polarizability, Zrot)."""
        if self._tran_params is None:
            raise ChemistryError("no transport data processed")
        return self._tran_params.copy()

    @property
    def viscosity_fits(self) -> np.ndarray:
        """[KK][4] coefficients of ln eta_k [g/(cm s)] in powers of ln T."""
        if self._vfits is None:
            raise ChemistryError("no transport data processed")
        return self._vfits.copy()

    @property
    def conductivity_fits(self) -> np.ndarray:
        """[KK][4] coefficients of ln lambda_k [erg/(cm s K)] in powers of ln T (ckmi_conductivity_fit)."""
        if self._tran_params is None:
            raise ChemistryError("no transport data processed")
        if getattr(self, "_cfits", None) is None or self._cfits_version != self._version:
            self._cfits = _transport.conductivity_fits(self._mech.wt, self._tran_params, self._mech.to_tables()["thermo"])
            self._cfits_version = self._version
        return self._cfits.copy()

    def SpeciesCond(self, temp: float = 0.0) -> np.ndarray:
        """Species thermal conductivities [erg/(cm s K)] at temp, on the GPU (chemistry.py:1361-1396,
        KINGetConductivity -> ckmi_species_conductivity)."""
        import torch

        if temp <= 0.0:
            raise ChemistryError("temperature must be > 0")
        dt = self.device_transport()
        T = torch.tensor([float(temp)], dtype=torch.float64, device=dt.dm.device)
        return dt.species_conductivity(T)[:, 0].cpu().numpy()

    def SpeciesVisc(self, temp: float = 0.0) -> np.ndarray:
        """Species viscosities [g/(cm s)] at temp, on the GPU (chemistry.py:1316-1359, KINGetViscosity)."""
        import torch

        if temp <= 0.0:
            raise ChemistryError("temperature must be > 0")
        dt = self.device_transport()
        T = torch.tensor([float(temp)], dtype=torch.float64, device=dt.dm.device)
        return dt.species_viscosity(T)[:, 0].cpu().numpy()

    def device_transport(self, device_index: int = None):
        """The viscosity tables of this chemistry set on a GPU (created on first use)."""
        if self._vfits is None:
            raise ChemistryError("no transport data processed")
        return _device.device_transport(self, device_index)

    @property
    def surffile(self) -> str:
        return self._surffile

    @surffile.setter
    def surffile(self, filename: str):
        if filename:
            raise ChemistryError("surface chemistry is outside the batch gas-phase path")
        self._surffile = filename

    def set_file_names(self, chemfile: str = "", thermfile: str = "", tranfile: str = "", surffile: str = "") -> None:
        if chemfile:
            self.chemfile = chemfile
        if thermfile:
            self.thermfile = thermfile
        if tranfile:
            self.tranfile = tranfile
        if surffile:
            self.surffile = surffile

    # ------------------------------------------------------------------ preprocess
    def preprocess(self) -> int:
        """Parse the mechanism; returns 0 on success (reference chemistry.py:595-753)."""
        global _active_chemistry_set
        if not self._chemfile or not os.path.isfile(self._chemfile):
            raise ChemistryError(f"gas mechanism file not found: {self._chemfile!r}")
        if self._thermfile and not os.path.isfile(self._thermfile):
            raise ChemistryError(f"thermodynamic data file not found: {self._thermfile!r}")
        if self._tranfile and not os.path.isfile(self._tranfile):
            raise ChemistryError(f"transport data file not found: {self._tranfile!r}")
        self._mech = Mechanism.from_files(self._chemfile, self._thermfile or None)
        self._tran_params = self._vfits = None
        tran_text = ""
        if self._tranfile:
            with open(self._tranfile) as f:
                tran_text = f.read()
        elif self._inline_transport:
            with open(self._chemfile) as f:
                tran_text = _transport.inline_transport_block(f.read())
            if not tran_text:
                raise ChemistryError("preprocess_transportdata(): the mechanism file has no TRANSPORT block")
        if tran_text:
            self._tran_params = _transport.species_params(_transport.parse_transport_text(tran_text),
                                                         self._mech.species)
            self._vfits = _transport.viscosity_fits(self._mech.wt, self._tran_params)
        self._version += 1
        if self._chemset_index < 0:
            self._chemset_index = len(_chemistry_sets)
        _chemistry_sets[self._chemset_index] = self
        _active_chemistry_set = self._chemset_index
        if verbose():
            logger.info("preprocessed %s: KK=%d II=%d", self._chemfile, self.KK, self.IIGas)
        return 0

    def _need(self) -> Mechanism:
        if self._mech is None:
            raise ChemistryError("please preprocess the chemistry set first")
        return self._mech

    def save(self) -> None:
        pass

    def activate(self) -> int:
        global _active_chemistry_set
        self._need()
        _active_chemistry_set = self._chemset_index
        return 0

    @property
    def mechanism(self) -> Mechanism:
        return self._need()

    def device_mechanism(self, device_index: int = None):
        """The ckmi device tables of this chemistry set on a GPU (created on first use)."""
        return _device.device_mechanism(self, device_index)

    # ------------------------------------------------------------------ sizes / names
    @property
    def chemID(self) -> int:
        return self._chemset_index

    @property
    def surfchem(self) -> int:
        return 0

    @property
    def KK(self) -> int:
        return self._need().KK

    @property
    def MM(self) -> int:
        return self._need().MM

    @property
    def IIGas(self) -> int:
        return self._need().II

    @property
    def species_symbols(self) -> List[str]:
        return list(self._need().species)

    @property
    def element_symbols(self) -> List[str]:
        return list(self._need().elements)

    def get_specindex(self, specname: str) -> int:
        """0-based species index (the reference rejects index 0, chemistry.py:911-916: fixed)."""
        sp = self._need().species
        if specname in sp:
            return sp.index(specname)
        up = [s.upper() for s in sp]
        if specname.upper() in up:
            return up.index(specname.upper())
        raise ChemistryError(f"species {specname!r} is not in the mechanism")

    @property
    def AWT(self) -> np.ndarray:
        return np.asarray(self._need().awt, dtype=np.float64)

    @property
    def WT(self) -> np.ndarray:
        return np.asarray(self._need().wt, dtype=np.float64)

    @property
    def EOS(self) -> int:
        return 0

    def use_idealgas_law(self) -> None:
        self.userealgas = False

    def use_realgas_cubicEOS(self) -> None:
        raise ChemistryError("real-gas cubic EOS is not supported (GRI-type gas mechanisms are ideal gas)")

    # ------------------------------------------------------------------ thermo
    def _species_thermo(self, temp: float):
        import torch

        if temp <= 1.0:
            raise ChemistryError("temperature value is too low")
        dm = self.device_mechanism()
        cp, h, s = dm.species_thermo(torch.tensor([float(temp)], dtype=torch.float64, device=dm.device))
        return cp[:, 0].cpu().numpy(), h[:, 0].cpu().numpy(), s[:, 0].cpu().numpy()

    def SpeciesCp(self, temp: float = 0.0, pres: Optional[float] = None) -> np.ndarray:
        """Species cp [erg/mol-K] (KINGetGasSpecificHeat x WT, chemistry.py:1069-1135)."""
        cp, _, _ = self._species_thermo(temp)
        return cp * R_GAS

    def SpeciesCv(self, temp: float = 0.0, pres: Optional[float] = None) -> np.ndarray:
        """Species cv [erg/mol-K] (chemistry.py:1137-1174)."""
        cp, _, _ = self._species_thermo(temp)
        return (cp - 1.0) * R_GAS

    def SpeciesH(self, temp: float = 0.0, pres: Optional[float] = None) -> np.ndarray:
        """Species enthalpy [erg/mol] (chemistry.py:1176-1241)."""
        _, h, _ = self._species_thermo(temp)
        return h * R_GAS * temp

    def SpeciesU(self, temp: float = 0.0, pres: Optional[float] = None) -> np.ndarray:
        """Species internal energy [erg/mol] (chemistry.py:1243-1314)."""
        _, h, _ = self._species_thermo(temp)
        return (h - 1.0) * R_GAS * temp

    def SpeciesComposition(self, elemindex: int = -1, specindex: int = -1):
        """Element counts: NCF[MM, KK], a row, a column or a single count (chemistry.py:1472-1522)."""
        ncf = self._need().ncf
        if elemindex >= 0 and specindex >= 0:
            return int(ncf[elemindex, specindex])
        if elemindex >= 0:
            return ncf[elemindex, :].copy()
        if specindex >= 0:
            return ncf[:, specindex].copy()
        return ncf.copy()

    # ------------------------------------------------------------------ kinetics parameters
    def get_reaction_parameters(self):
        """(A [cgs], beta, E/R [K]) for all reactions (KINGetReactionRateParameters)."""
        return self._need().arrhenius()

    def set_reaction_AFactor(self, reaction_index: int, AFactor: float) -> None:
        """Reset A of reaction `reaction_index` (1-based, chemistry.py:1636-1678)."""
        mech = self._need()
        if reaction_index < 1 or reaction_index > mech.II:
            raise ChemistryError(f"reaction index is out of bound, range = [1 ~ {mech.II}]")
        # validate everything before any state changes, so host and device tables stay consistent
        if not AFactor > 0.0:
            raise ChemistryError("A-factor must be > 0")
        if mech.reactions[reaction_index - 1].plog:
            raise ChemistryError("the A-factor of a PLOG reaction is set by its PLOG table")
        mech.set_A_cgs(reaction_index - 1, AFactor)
        for (cid, dev), dm in list(_device._cache.items()):
            if cid == id(self):
                dm.set_afactor(reaction_index - 1, AFactor)

    def get_reaction_AFactor(self, reaction_index: int) -> float:
        mech = self._need()
        if reaction_index < 1 or reaction_index > mech.II:
            raise ChemistryError(f"reaction index is out of bound, range = [1 ~ {mech.II}]")
        return mech.A_cgs(reaction_index - 1)

    def get_gas_reaction_string(self, reaction_index: int) -> str:
        mech = self._need()
        if reaction_index < 1 or reaction_index > mech.II:
            raise ChemistryError(f"reaction index is out of bound, range = [1 ~ {mech.II}]")
        return mech.reactions[reaction_index - 1].equation
