"""Gas mixture state, composition algebra and single-state kinetics (reference mixture.py).

Drop-in subset of ``Mixture`` used by the batch-reactor path:
state (temperature, pressure, volume, X, Y), composition conversion and normalisation,
WTM, RHO, concentration, HML/CPBL, ROP, RxnRates, massROP, volHRR, list_ROP,
list_reaction_rates, X/Y_by_Equivalence_Ratio, list_composition, validate,
mixture_viscosity and species_Visc (transport data preprocessed, mixture.py:1860-1977).

Kinetics and mixture thermo go through the GPU kernels (ckmi_rop_thermo,
ckmi_reaction_rates, ckmi_species_thermo) with a batch of one state, exactly as the
reference goes through KINGetGasROP / KINGetGasReactionRates (mixture.py:1442,1551).
Errors raise exceptions instead of calling exit().
"""
from __future__ import annotations

import copy
from typing import List, Tuple, Union

import numpy as np

from .chemistry import Chemistry
from .constants import R_GAS
from .utilities import calculate_stoichiometrics


class MixtureError(ValueError):
    pass


class Mixture:
    """A gas mixture defined on the species of a Chemistry set."""

    def __init__(self, chem: Chemistry):
        if not isinstance(chem, Chemistry):
            raise MixtureError("the argument must be a Chemistry object")
        if chem.chemID < 0:
            raise MixtureError("invalid chemistry, please preprocess the chemistry first")
        self._chem = chem
        self._temp = 0.0
        self._press = 0.0
        self._vol = 0.0
        self._Tset = self._Pset = self._Xset = self._Yset = 0
        self._KK = chem.KK
        self._IIgas = chem.IIGas
        self._specieslist = chem.species_symbols
        self._WT = chem.WT
        self._molefrac = np.zeros(self._KK)
        self._massfrac = np.zeros(self._KK)
        self._EOS = 0
        self.userealgas = False

    # ------------------------------------------------------------------ state
    @property
    def chemistry(self) -> Chemistry:
        return self._chem

    @property
    def chemID(self) -> int:
        return self._chem.chemID

    @property
    def KK(self) -> int:
        return self._KK

    @property
    def pressure(self) -> float:
        return self._press

    @pressure.setter
    def pressure(self, p: float):
        if p <= 0.0:
            raise MixtureError("pressure must be > 0")
        self._press = float(p)
        self._Pset = 1

    @property
    def temperature(self) -> float:
        return self._temp

    @temperature.setter
    def temperature(self, t: float):
        if t <= 10.0:
            raise MixtureError("temperature must be > 10 K")
        self._temp = float(t)
        self._Tset = 1

    @property
    def volume(self) -> float:
        return self._vol

    @volume.setter
    def volume(self, vol: float):
        if vol <= 0.0:
            raise MixtureError("volume must be > 0")
        self._vol = float(vol)

    def _recipe_to_array(self, recipe) -> np.ndarray:
        arr = np.zeros(self._KK)
        if isinstance(recipe, np.ndarray) or (len(recipe) and isinstance(recipe[0], (float, int, np.floating, np.integer))):
            a = np.asarray(recipe, dtype=np.float64)
            if a.shape != (self._KK,):
                raise MixtureError(f"fraction array must have {self._KK} entries")
            return np.maximum(a, 0.0)
        for sp, x in recipe:
            k = self._chem.get_specindex(sp)
            if x < 0.0:
                raise MixtureError(f"negative fraction for {sp}")
            arr[k] = x
        return arr

    @property
    def X(self) -> np.ndarray:
        if self._Xset:
            return Mixture.normalize(self._molefrac)[1]
        if self._Yset:
            return Mixture.mass_fraction_to_mole_fraction(self.Y, self._WT)
        raise MixtureError("mixture composition is not provided")

    @X.setter
    def X(self, recipe: Union[List[Tuple[str, float]], np.ndarray]):
        self._molefrac = self._recipe_to_array(recipe)
        self._massfrac[:] = 0.0
        self._Xset, self._Yset = 1, 0

    mole_fractions = X

    @property
    def Y(self) -> np.ndarray:
        if self._Yset:
            return Mixture.normalize(self._massfrac)[1]
        if self._Xset:
            return Mixture.mole_fraction_to_mass_fraction(self.X, self._WT)
        raise MixtureError("mixture composition is not provided")

    @Y.setter
    def Y(self, recipe: Union[List[Tuple[str, float]], np.ndarray]):
        self._massfrac = self._recipe_to_array(recipe)
        self._molefrac[:] = 0.0
        self._Xset, self._Yset = 0, 1

    mass_fractions = Y

    @property
    def EOS(self) -> int:
        return self._EOS

    # ------------------------------------------------------------------ algebra
    @staticmethod
    def normalize(frac) -> Tuple[int, np.ndarray]:
        """(0, frac / sum(frac)) with negative entries set to 0 first (reference mixture.py:486-523);
        (1, the clipped copy) when nothing positive is left (the reference exits there)."""
        f = np.maximum(np.asarray(frac, dtype=np.float64), 0.0)
        s = f.sum()
        if s <= 0.0:
            return 1, f
        return 0, f / s

    @property
    def WT(self) -> np.ndarray:
        return self._WT

    @property
    def WTM(self) -> float:
        """Mean molar mass [g/mol] (mixture.py:541-584)."""
        return float(1.0 / np.sum(self.Y / self._WT))

    @staticmethod
    def mean_molar_mass(frac, wt, mode: str = "mole") -> float:
        f = Mixture.normalize(frac)[1]
        if mode.lower() == "mole":
            return float(np.sum(f * wt))
        return float(1.0 / np.sum(f / wt))

    @staticmethod
    def mole_fraction_to_mass_fraction(molefrac, wt) -> np.ndarray:
        x = Mixture.normalize(molefrac)[1]
        y = x * np.asarray(wt)
        return y / y.sum()

    @staticmethod
    def mass_fraction_to_mole_fraction(massfrac, wt) -> np.ndarray:
        y = Mixture.normalize(massfrac)[1]
        x = y / np.asarray(wt)
        return x / x.sum()

    @staticmethod
    def density(chemID: int = -1, p: float = 0.0, t: float = 0.0, frac=None, wt=None, mode: str = "mole") -> float:
        """Ideal-gas density [g/cm3] (KINGetMassDensity, mixture.py:993-1089)."""
        if p <= 0.0 or t <= 0.0:
            raise MixtureError("invalid pressure and/or temperature")
        W = Mixture.mean_molar_mass(frac, wt, mode)
        return p * W / (R_GAS * t)

    @staticmethod
    def mass_fraction_to_concentration(chemID: int, p: float, t: float, massfrac, wt) -> np.ndarray:
        """Molar concentrations [mol/cm3] of a mass-fraction composition at (p, t) (mixture.py:821-877):
        c_k = rho Y_k / W_k of the normalised (negatives removed) fractions; the input back when the
        density is not positive."""
        massfrac = np.asarray(massfrac, dtype=np.float64)
        wt = np.asarray(wt, dtype=np.float64)
        if len(massfrac) != len(wt):
            raise MixtureError(f"mass fraction and molar mass arrays must have the same size = {len(massfrac)}")
        den = Mixture.density(chemID, p, t, frac=massfrac, wt=wt, mode="mass")
        if not den > 0.0:
            return massfrac
        err, c = Mixture.normalize(massfrac)
        return c * den / wt if err == 0 else c

    @staticmethod
    def mole_fraction_to_concentration(chemID: int, p: float, t: float, molefrac, wt) -> np.ndarray:
        """Molar concentrations [mol/cm3] of a mole-fraction composition at (p, t) (mixture.py:879-935):
        c_k = X_k rho / W-bar = X_k P / (R T)."""
        molefrac = np.asarray(molefrac, dtype=np.float64)
        wt = np.asarray(wt, dtype=np.float64)
        if len(molefrac) != len(wt):
            raise MixtureError(f"mole fraction and molar mass arrays must have the same size = {len(molefrac)}")
        mwt = Mixture.mean_molar_mass(molefrac, wt, "mole")
        den = Mixture.density(chemID, p, t, frac=molefrac, wt=wt, mode="mole")
        if not mwt * den > 0.0:
            return molefrac
        err, c = Mixture.normalize(molefrac)
        return c * (den / mwt) if err == 0 else c

    @property
    def RHO(self) -> float:
        self._need_TP()
        return float(self._press * self.WTM / (R_GAS * self._temp))

    @property
    def concentration(self) -> np.ndarray:
        """Molar concentrations [mol/cm3]."""
        return self.RHO * self.Y / self._WT

    def _need_TP(self):
        if not self._Tset:
            raise MixtureError("mixture temperature [K] is not provided")
        if not self._Pset:
            raise MixtureError("mixture pressure [dynes/cm2] is not provided")
        if not (self._Xset or self._Yset):
            raise MixtureError("mixture composition is not provided")

    def validate(self) -> int:
        """0 if temperature, pressure and composition are set (mixture.py:2637-2662)."""
        try:
            self._need_TP()
        except MixtureError:
            return 1
        return 0

    def list_composition(self, mode: str, option: str = " ", bound: float = 0.0) -> None:
        frac = self.X if mode.lower() == "mole" else self.Y
        print(f"{mode} fractions:")
        for k, v in enumerate(frac):
            if option.lower() == "all" or v > bound:
                print(f"  {self._specieslist[k]:>16s}  {v: .6e}")

    # ------------------------------------------------------------------ GPU kernels, one state
    def _state_tensors(self):
        import torch

        self._need_TP()
        dm = self._chem.device_mechanism()
        T = torch.tensor([self._temp], dtype=torch.float64, device=dm.device)
        P = torch.tensor([self._press], dtype=torch.float64, device=dm.device)
        Y = torch.as_tensor(self.Y.reshape(self._KK, 1).copy(), dtype=torch.float64, device=dm.device)
        return dm, T, P, Y

    def _rop_thermo(self):
        dm, T, P, Y = self._state_tensors()
        w, cp, h = dm.rop_thermo(T, P, Y)
        return w[:, 0].cpu().numpy(), float(cp[0].item()), float(h[0].item())

    def ROP(self) -> np.ndarray:
        """Species molar rates of production [mol/cm3-s] (KINGetGasROP, mixture.py:1693-1746)."""
        return self._rop_thermo()[0]

    def RxnRates(self, reference_compat: bool = True) -> Tuple[np.ndarray, np.ndarray]:
        """Forward and reverse rates of progress [mol/cm3-s] (KINGetGasReactionRates, mixture.py:1748-1810).

        reference_compat (default) returns what the reference returns: its Mixture.reaction_rates
        hands the mass fractions to KINGetGasReactionRates (mixture.py:1540), which reads its
        composition argument as mole fractions (Chemkin CKKFKR convention), so the rates belong to
        the state whose mole fractions equal this mixture's mass fractions.  The reactionrates
        golden is reproduced to 1e-14 that way (tests/test_oracle_golden.py).  False gives the rates
        of this mixture's own composition (consistent with ROP())."""
        dm, T, P, Y = self._state_tensors()
        if reference_compat:
            import torch

            y = self.Y * self._WT
            Y = torch.as_tensor((y / y.sum()).reshape(self._KK, 1), dtype=torch.float64, device=dm.device)
        qf, qr = dm.reaction_rates(T, P, Y)
        return qf[:, 0].cpu().numpy(), qr[:, 0].cpu().numpy()

    # ------------------------------------------------------------------ static forms (chemistry set id)
    @staticmethod
    def _static_state(chemID: int, p: float, t: float, frac, wt, mode: str):
        """Chemistry set and normalised mass fractions of the static rate calls (mixture.py:1386-1430):
        the same argument checks, raised instead of exit()."""
        from .chemistry import _chemistry_sets

        if chemID < 0 or chemID not in _chemistry_sets:
            raise MixtureError("invalid chemistry.")
        if p <= 0.0 or (p * t) <= 0.0:
            raise MixtureError("invalid pressure and/or temperature value(s).")
        frac = np.asarray(frac, dtype=np.float64)
        wt = np.asarray(wt, dtype=np.float64)
        if len(frac) != len(wt):
            raise MixtureError(f"{mode} fraction and molar mass arrays must have the same size = {len(frac)}")
        if mode.lower() == "mole":
            y = Mixture.mole_fraction_to_mass_fraction(molefrac=frac, wt=wt)
        elif mode.lower() == "mass":
            y = Mixture.normalize(frac=frac)[1]
        else:
            raise MixtureError('must specify "mole" or "mass" fractions given.')
        chem = _chemistry_sets[chemID]
        if len(y) != chem.KK:
            raise MixtureError(f"composition has {len(y)} entries, the chemistry set {chem.KK} species")
        return chem, y

    @staticmethod
    def rate_of_production(chemID: int, p: float, t: float, frac, wt, mode: str) -> np.ndarray:
        """Species molar rates of production [mol/cm3-s] of the state (p, t, frac) (mixture.py:1353-1454):
        KINGetGasROP with the normalised mass fractions, on the GPU (the same kernel as ROP())."""
        import torch

        chem, y = Mixture._static_state(chemID, p, t, frac, wt, mode)
        dm = chem.device_mechanism()
        T = torch.tensor([float(t)], dtype=torch.float64, device=dm.device)
        P = torch.tensor([float(p)], dtype=torch.float64, device=dm.device)
        Y = torch.as_tensor(y.reshape(-1, 1).copy(), dtype=torch.float64, device=dm.device)
        return dm.rop_thermo(T, P, Y)[0][:, 0].cpu().numpy()

    @staticmethod
    def reaction_rates(chemID: int, numbreaction: int, p: float, t: float, frac, wt,
                       mode: str) -> Tuple[np.ndarray, np.ndarray]:
        """Forward and reverse rates of the gas reactions [mol/cm3-s] (mixture.py:1456-1567).

        The reference hands the normalised mass fractions to KINGetGasReactionRates (mixture.py:1540),
        which reads its composition argument as mole fractions (Chemkin's CKKFKR convention; the
        reactionrates golden decides): the rates returned are those of the state whose mole
        fractions equal these mass fractions, exactly as RxnRates() (reference_compat=True) returns them."""
        import torch

        chem, y = Mixture._static_state(chemID, p, t, frac, wt, mode)
        if int(numbreaction) != chem.IIGas:
            raise MixtureError(f"numbreaction = {numbreaction}, the chemistry set has {chem.IIGas} reactions")
        dm = chem.device_mechanism()
        yy = y * chem.WT  # y read as mole fractions -> the mass fractions of that state, for the kernel
        T = torch.tensor([float(t)], dtype=torch.float64, device=dm.device)
        P = torch.tensor([float(p)], dtype=torch.float64, device=dm.device)
        Y = torch.as_tensor((yy / yy.sum()).reshape(-1, 1), dtype=torch.float64, device=dm.device)
        qf, qr = dm.reaction_rates(T, P, Y)
        return qf[:, 0].cpu().numpy(), qr[:, 0].cpu().numpy()

    def use_idealgas_law(self) -> None:
        """Ideal-gas law for the mixture properties (mixture.py:2706-2740).  The device path is ideal-gas
        only (real-gas cubic EOS is out of scope), so this is the state every mixture is already in."""
        self.userealgas = False

    def CPBL(self) -> float:
        """Mixture cp [erg/mol-K] (KINGetGasMixtureSpecificHeat x WTM, mixture.py:1646)."""
        return self._rop_thermo()[1] * self.WTM

    def HML(self) -> float:
        """Mixture enthalpy [erg/mol] (KINGetGasMixtureEnthalpy x WTM, mixture.py:1599)."""
        return self._rop_thermo()[2] * self.WTM

    def mixture_specific_heat(self) -> float:
        return self.CPBL()

    def mixture_enthalpy(self) -> float:
        return self.HML()

    def species_Cp(self) -> np.ndarray:
        self._need_TP()
        return self._chem.SpeciesCp(self._temp)

    def species_H(self) -> np.ndarray:
        self._need_TP()
        return self._chem.SpeciesH(self._temp)

    @property
    def transport_data(self) -> int:
        """1 if the chemistry set has processed transport data (mixture.py:108)."""
        return 1 if self._chem.verify_transport_data() else 0

    def _need_transport(self):
        if not self.transport_data:
            raise MixtureError("no transport data processed")
        if not self._Tset:
            raise MixtureError("mixture temperature [K] is not provided")

    def species_Visc(self) -> np.ndarray:
        """Species viscosities [g/(cm s)] at the mixture temperature (KINGetViscosity, mixture.py:1860-1883)."""
        import torch

        self._need_transport()
        dt = self._chem.device_transport()
        T = torch.tensor([self._temp], dtype=torch.float64, device=dt.dm.device)
        return dt.species_viscosity(T)[:, 0].cpu().numpy()

    def mixture_viscosity(self) -> float:
        """Mixture viscosity [g/(cm s)] (KINGetMixtureViscosity with the mass fractions,
        mixture.py:1943-1977; Wilke's rule on the GPU)."""
        import torch

        self._need_transport()
        if not (self._Xset or self._Yset):
            raise MixtureError("mixture composition is not provided")
        dt = self._chem.device_transport()
        T = torch.tensor([self._temp], dtype=torch.float64, device=dt.dm.device)
        Y = torch.as_tensor(self.Y.reshape(self._KK, 1).copy(), dtype=torch.float64, device=dt.dm.device)
        return float(dt.mixture_viscosity(T, Y)[0].item())

    def species_Cond(self) -> np.ndarray:
        """Species thermal conductivities [erg/(cm s K)] at the mixture temperature, on the GPU
        (KINGetConductivity, mixture.py:1885-1909)."""
        import torch

        self._need_transport()
        dt = self._chem.device_transport()
        T = torch.tensor([self._temp], dtype=torch.float64, device=dt.dm.device)
        return dt.species_conductivity(T)[:, 0].cpu().numpy()

    def mixture_conductivity(self) -> float:
        """Mixture-averaged thermal conductivity [erg/(cm s K)] (KINGetMixtureConductivity with the mass
        fractions, mixture.py:1979-2013): (sum X lambda + 1 / sum X / lambda) / 2 on the GPU."""
        import torch

        self._need_transport()
        if not (self._Xset or self._Yset):
            raise MixtureError("mixture composition is not provided")
        dt = self._chem.device_transport()
        T = torch.tensor([self._temp], dtype=torch.float64, device=dt.dm.device)
        Y = torch.as_tensor(self.Y.reshape(self._KK, 1).copy(), dtype=torch.float64, device=dt.dm.device)
        return float(dt.mixture_conductivity(T, Y)[0].item())

    def massROP(self) -> np.ndarray:
        """Species mass rates of production [g/cm3-s]."""
        return self.ROP() * self._WT

    def volHRR(self) -> float:
        """Volumetric "heat release rate" [erg/cm3-s] = sum_k H_k ROP_k, sign as the reference
        returns it (mixture.py:2172-2202: np.dot(H, ROP), no negation; negative when heat is
        released)."""
        return float(np.dot(self.species_H(), self.ROP()))

    @staticmethod
    def _sorted_nonzero(values: np.ndarray, threshold: float):
        idx = np.nonzero(np.abs(values) > threshold)[0]
        order = idx[np.argsort(-values[idx], kind="stable")]
        return order.astype(np.int32), values[order]

    def list_ROP(self, threshold: float = 0.0):
        """Nonzero species ROP in descending order: (species order, rates)."""
        return Mixture._sorted_nonzero(self.ROP(), threshold)

    def list_massROP(self, threshold: float = 0.0):
        return Mixture._sorted_nonzero(self.massROP(), threshold)

    def list_reaction_rates(self, threshold: float = 0.0):
        """Nonzero net reaction rates in descending order: (0-based reaction order, rates).

        Same selection and ordering as the reference (mixture.py:2325-2381).
        """
        qf, qr = self.RxnRates()
        return Mixture._sorted_nonzero(qf - qr, threshold)

    # ------------------------------------------------------------------ phi mixtures
    def X_by_Equivalence_Ratio(self, chemistryset: Chemistry, fuel_molefrac, oxid_molefrac, add_molefrac,
                               products: List[str], equivalenceratio: float, threshold: float = 1.0e-10) -> int:
        """X = normalise(phi*X_fuel + alpha*X_oxid) (+ additives), mixture.py:2383-2539."""
        KK = chemistryset.KK
        fuel = np.asarray(fuel_molefrac, dtype=np.float64)
        oxid = np.asarray(oxid_molefrac, dtype=np.float64)
        add = np.asarray(add_molefrac, dtype=np.float64).copy()
        if fuel.shape != (KK,) or oxid.shape != (KK,) or add.shape != (KK,):
            return 2
        if equivalenceratio <= 0.0:
            return 3
        if not products:
            return 4
        add[add < threshold] = 0.0
        suma = add.sum()
        prod_index = [chemistryset.get_specindex(s) for s in products]
        alpha, nu = calculate_stoichiometrics(chemistryset, fuel, oxid, prod_index)
        if alpha <= 0.0:
            return 5
        x = equivalenceratio * fuel + alpha * oxid
        x = x / x.sum()
        if suma > 0.0:
            x = x * (1.0 - suma) + add
        self.X = x
        return 0

    def Y_by_Equivalence_Ratio(self, chemistryset: Chemistry, fuel_massfrac, oxid_massfrac, add_massfrac,
                               products: List[str], equivalenceratio: float, threshold: float = 1.0e-10) -> int:
        wt = chemistryset.WT
        fx = Mixture.mass_fraction_to_mole_fraction(fuel_massfrac, wt)
        ox = Mixture.mass_fraction_to_mole_fraction(oxid_massfrac, wt)
        add = np.asarray(add_massfrac, dtype=np.float64)
        ax = np.zeros_like(add) if add.sum() <= 0 else Mixture.mass_fraction_to_mole_fraction(add, wt) * add.sum()
        err = self.X_by_Equivalence_Ratio(chemistryset, fx, ox, ax, products, equivalenceratio, threshold)
        if err == 0:
            self.Y = self.Y
        return err


def interpolate_mixtures(mixtureleft: Mixture, mixtureright: Mixture, ratio: float) -> Mixture:
    """Linear interpolation of T, P, V and mass fractions (reference mixture.py:3268-3384)."""
    m = copy.deepcopy(mixtureleft)
    m.temperature = (1.0 - ratio) * mixtureleft.temperature + ratio * mixtureright.temperature
    m.pressure = (1.0 - ratio) * mixtureleft.pressure + ratio * mixtureright.pressure
    if mixtureleft.volume > 0 and mixtureright.volume > 0:
        m.volume = (1.0 - ratio) * mixtureleft.volume + ratio * mixtureright.volume
    m.Y = (1.0 - ratio) * mixtureleft.Y + ratio * mixtureright.Y
    return m


def _combine(recipe, mode: str):
    """Mole fractions of a mixed recipe [(Mixture, ratio), ...] and the normalised mixing mole
    ratios (reference mixture.py:2920-2975 / 3108-3160): 'mole' ratios are used as given,
    'mass' ratios are converted to moles with each mixture's WTM."""
    if not recipe:
        raise MixtureError("empty mixing recipe")
    chem_id = recipe[0][0].chemID
    x = np.zeros(recipe[0][0].KK)
    ratios = np.zeros(len(recipe))
    for i, (m, v) in enumerate(recipe):
        if not isinstance(m, Mixture):
            raise MixtureError("the recipe must hold Mixture objects")
        if m.chemID != chem_id:
            raise MixtureError(f"mixture {i} of the recipe uses a different chemistry set")
        if v <= 0.0:
            raise MixtureError(f"mixing ratio {i} must be > 0")
        ratios[i] = v if mode.lower() == "mole" else v / m.WTM
        x += m.X * ratios[i]
    total = ratios.sum()
    return x / total, ratios / total


def isothermal_mixing(recipe: List[Tuple[Mixture, float]], mode: str, finaltemperature: float) -> Mixture:
    """Mix gas mixtures at a given final temperature (reference mixture.py:2802-2988)."""
    if finaltemperature <= 10.0:
        raise MixtureError("the final mixture temperature must be given (> 10 K)")
    x, _ = _combine(recipe, mode)
    final = copy.deepcopy(recipe[0][0])
    final.X = x
    final.temperature = finaltemperature
    return final


def calculate_mixture_temperature_from_enthalpy(mixture: Mixture, mixtureH: float,
                                                guesstemperature: float = 0.0) -> int:
    """Newton iteration for T with HML(T) = mixtureH [erg/mol], converged when the correction is
    below 0.1 K (reference mixture.py:3179-3266: the last, sub-0.1 K correction is not applied;
    this keeps that, and returns 2 instead of looping when 200 iterations do not converge).
    Mixture enthalpy and cp come from the device species thermo (only T is needed)."""
    X = mixture.X
    T = guesstemperature if guesstemperature > 0.0 else mixture.temperature
    if T <= 1.0:
        T = 300.0
    chem = mixture.chemistry
    for _ in range(200):
        f = float(np.dot(X, chem.SpeciesH(T))) - mixtureH
        df = float(np.dot(X, chem.SpeciesCp(T)))
        if df == 0.0:
            return 1
        dt = f / df
        if abs(dt) <= 0.1:
            mixture.temperature = T
            return 0
        T -= dt
    mixture.temperature = T
    return 2


def adiabatic_mixing(recipe: List[Tuple[Mixture, float]], mode: str) -> Mixture:
    """Mix gas mixtures at constant total enthalpy (reference mixture.py:2990-3177)."""
    x, ratios = _combine(recipe, mode)
    h = 0.0
    for (m, _), r in zip(recipe, ratios):
        h += float(np.dot(m.X, m.chemistry.SpeciesH(m.temperature))) * r  # erg/mol of the final mixture
    final = copy.deepcopy(recipe[0][0])
    final.X = x
    err = calculate_mixture_temperature_from_enthalpy(final, h)
    if err != 0:
        raise MixtureError(f"mixture temperature from enthalpy did not converge (error {err})")
    return final
