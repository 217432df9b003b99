"""Chemkin-format mechanism compiler: ``chem.inp`` + ``therm.dat`` -> flat SoA tables.

This is the host half of what the reference hands to the closed native library as
``KINPreProcess`` (``chemistry.py:675-687``, prototype ``chemkin_wrapper.py:303-316``)
followed by ``KINGetChemistrySizes`` / ``KINGetGasSpeciesNames`` / ``KINGetAtomicWeights`` /
``KINGetGasMolecularWeights`` / ``KINGetGasSpeciesComposition`` /
``KINGetReactionRateParameters`` (``chemistry.py:693-1634``).  The parsed mechanism is
flattened once into the fixed-slot, struct-of-arrays layout declared in
``include/ckmi.h`` (``ckmi_mech_desc``) and uploaded to HBM by ``ckmi_mech_create``.

Supported syntax (Chemkin-II gas phase): ELEMENTS (with optional /weight/), SPECIES,
optional THERMO block, REACTIONS with unit keywords, ``=``/``<=>``/``=>``, ``+M``,
``(+M)``/``(+species)`` falloff, LOW, TROE (3 or 4 parameters), SRI (3 or 5), REV,
DUPLICATE, third-body efficiencies, FORD/RORD and non-integral stoichiometric coefficients,
PLOG (elementary reactions; ln k interpolated in ln P, clamped outside the table), Chebyshev
(TCHEB / PCHEB / CHEB on a (+M) reaction; log10 k a double Chebyshev series in the reduced 1/T and
log P, not clamped outside the fit's range), Landau-Teller (LT, with RLT on REV), per-reaction UNITS.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .constants import AVOGADRO, P_ATM

# Chemkin default atomic weights [g/mol] (reproduces loadmechanism.baseline "state-AWT")
ATOMIC_WEIGHTS = {
    "H": 1.00797, "HE": 4.0026, "LI": 6.939, "BE": 9.01220, "B": 10.811, "C": 12.01115,
    "N": 14.0067, "O": 15.9994, "F": 18.9984, "NE": 20.183, "NA": 22.9898, "MG": 24.312,
    "AL": 26.9815, "SI": 28.086, "P": 30.9738, "S": 32.064, "CL": 35.453, "AR": 39.948,
    "K": 39.102, "CA": 40.08, "SC": 44.956, "TI": 47.90, "V": 50.942, "CR": 51.996,
    "MN": 54.938, "FE": 55.847, "CO": 58.9332, "NI": 58.71, "CU": 63.54, "ZN": 65.37,
    "GA": 69.72, "GE": 72.59, "AS": 74.9216, "SE": 78.96, "BR": 79.9009, "KR": 83.80,
    "RB": 85.47, "SR": 87.62, "Y": 88.905, "ZR": 91.22, "NB": 92.906, "MO": 95.94,
    "TC": 99.0, "RU": 101.07, "RH": 102.905, "PD": 106.4, "AG": 107.87, "CD": 112.40,
    "IN": 114.82, "SN": 118.69, "SB": 121.75, "TE": 127.60, "I": 126.904, "XE": 131.30,
    "CS": 132.905, "BA": 137.34, "D": 2.01410, "E": 5.45e-4,
}

# reaction type codes (must match include/ckmi.h)
RXN_ELEMENTARY = 0
RXN_THIRDBODY = 1
RXN_FALLOFF = 2
RXN_CHEMACT = 3  # chemically activated (HIGH/): main line = k0, HIGH = k_inf
TAB_PLOG = 3     # rtype of a PLOG reaction in to_tables() (CKMI_RXN_PLOG in include/ckmi.h)
TAB_CHEMACT = 4  # rtype of a chemically activated reaction (CKMI_RXN_CHEMACT)
TAB_CHEB = 5     # rtype of a Chebyshev (T, P) reaction (CKMI_RXN_CHEB)
TAB_LT = 6       # rtype of a Landau-Teller elementary reaction (CKMI_RXN_LT)
CHEB_MAX = 12    # Chebyshev orders per dimension the kernels accept

FALL_NONE = 0
FALL_LINDEMANN = 1
FALL_TROE3 = 2
FALL_TROE4 = 3
FALL_SRI = 4

MAX_SLOTS = 8  # distinct species per reaction side in the flat tables (CKMI_SLOTS in include/ckmi.h)

# Gas constant of the activation-energy conversion.  Chemkin's interpreter converts E of the
# REACTIONS block with its own RU = 8.314510e7 erg/mol-K (RUC = RU / 4.184e7 = 1.98721558
# cal/mol-K), not with the R_GAS = k_B N_A of constants.py that the closed library uses for
# the equation of state (simple.baseline density to 2e-16).  The two differ by 4.5e-6; at
# E/RT ~ 8.6 (H+O2<=>O+OH at 1000 K) that is 4e-5 in k and 1e-4 in the H2/air radical-pool
# growth rate: with R_GAS_CAL the closed_homogeneous__transient golden holds on 53/101 (X_H2O)
# and 82/101 (wdot_H2O) points, with RU_ACT on 101/101 for every column (tests/test_oracle_golden.py).
RU_ACT = 8.314510e7  # [erg/mol-K]
RUC_ACT = RU_ACT / 4.184e7  # [cal/mol-K]


class MechanismError(ValueError):
    pass


@dataclass
class Reaction:
    equation: str
    reactants: List[Tuple[str, float]]
    products: List[Tuple[str, float]]
    reversible: bool
    A: float
    b: float
    E: float  # activation energy in the file's units
    kind: int = RXN_ELEMENTARY
    third_body: Optional[str] = None  # "M" or a species name for (+SP)
    efficiencies: Dict[str, float] = field(default_factory=dict)
    low: Optional[Tuple[float, float, float]] = None
    high: Optional[Tuple[float, float, float]] = None
    troe: Optional[Tuple[float, ...]] = None
    sri: Optional[Tuple[float, ...]] = None
    rev: Optional[Tuple[float, float, float]] = None
    duplicate: bool = False
    ford: Dict[str, float] = field(default_factory=dict)
    rord: Dict[str, float] = field(default_factory=dict)
    plog: List[Tuple[float, float, float, float]] = field(default_factory=list)
    cheb: List[float] = field(default_factory=list)  # CHEB values: NT, NP, then NT x NP coefficients
    tcheb: Optional[Tuple[float, float]] = None      # TCHEB Tmin, Tmax [K] (Chemkin default 300, 2500)
    pcheb: Optional[Tuple[float, float]] = None      # PCHEB Pmin, Pmax [atm] (default 0.001, 100)
    lt: Optional[Tuple[float, float]] = None         # LT B, C: k = A T^b exp(-E/RT + B T^-1/3 + C T^-2/3)
    rlt: Optional[Tuple[float, float]] = None        # RLT B, C of the explicit reverse rate
    E_scale: float = 1.0  # multiply E by this to get E/R [K]
    A_scale_per_order: float = 1.0  # molecules->moles conversion factor base


@dataclass
class Thermo:
    tlow: float
    thigh: float
    tmid: float
    high: List[float]
    low: List[float]
    composition: Dict[str, int]


def _strip_comment(line: str) -> str:
    i = line.find("!")
    return line if i < 0 else line[:i]


_NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[EeDd][-+]?\d+)?"


def _to_float(s: str) -> float:
    return float(s.replace("D", "E").replace("d", "e"))


def parse_thermo_text(text: str, wanted: Optional[set] = None) -> Dict[str, Thermo]:
    """Parse Chemkin fixed-column NASA-7 thermo records."""
    lines = text.splitlines()
    out: Dict[str, Thermo] = {}
    i = 0
    # skip to THERMO keyword if present
    while i < len(lines):
        s = lines[i].strip().upper()
        if s.startswith("THERMO"):
            i += 1
            # the optional default-temperature line
            if i < len(lines) and re.match(r"^\s*" + _NUM + r"\s+" + _NUM + r"\s+" + _NUM + r"\s*$", _strip_comment(lines[i])):
                i += 1
            break
        if s and not s.startswith("!"):
            break
        i += 1
    while i < len(lines):
        raw = lines[i]
        if not raw.strip() or raw.lstrip().startswith("!"):
            i += 1
            continue
        if raw.strip().upper().startswith("END"):
            break
        if i + 3 >= len(lines):
            break
        l1 = raw.rstrip("\n").ljust(80)
        name = l1[0:18].split()[0] if l1[0:18].split() else ""
        comp: Dict[str, int] = {}
        for k in range(4):
            fld = l1[24 + 5 * k: 29 + 5 * k]
            el = fld[0:2].strip().upper()
            cnt = fld[2:5].strip()
            if el and el != "0" and cnt:
                try:
                    n = int(float(cnt))
                except ValueError:
                    n = 0
                if n != 0:
                    comp[el] = comp.get(el, 0) + n
        fld5 = l1[73:78]
        el5 = fld5[0:2].strip().upper()
        if el5 and fld5[2:5].strip():
            try:
                n5 = int(float(fld5[2:5]))
                if n5:
                    comp[el5] = comp.get(el5, 0) + n5
            except ValueError:
                pass
        try:
            tlow = float(l1[45:55])
            thigh = float(l1[55:65])
            tmid_s = l1[65:73].strip()
            tmid = float(tmid_s) if tmid_s else 1000.0
        except ValueError as exc:
            raise MechanismError(f"bad thermo header for {name!r}: {raw!r}") from exc
        coeffs: List[float] = []
        for k in range(1, 4):
            ln = lines[i + k].rstrip("\n").ljust(80)
            nfield = 5 if k < 3 else 4
            for m in range(nfield):
                s = ln[15 * m: 15 * m + 15].strip()
                coeffs.append(_to_float(s) if s else 0.0)
        i += 4
        if wanted is not None and name.upper() not in wanted:
            continue
        if name.upper() in out:  # first definition wins (Chemkin rule)
            continue
        out[name.upper()] = Thermo(tlow, thigh, tmid, coeffs[0:7], coeffs[7:14], comp)
    return out


class Mechanism:
    """A parsed gas-phase Chemkin mechanism and its flattened device tables."""

    def __init__(self, chem_text: str, therm_text: Optional[str] = None):
        self.elements: List[str] = []
        self.awt: List[float] = []
        self.species: List[str] = []
        self.reactions: List[Reaction] = []
        self.thermo: Dict[str, Thermo] = {}
        self._parse_chem(chem_text)
        inline = self._inline_thermo
        data: Dict[str, Thermo] = {}
        if therm_text:
            data.update(parse_thermo_text(therm_text, set(s.upper() for s in self.species)))
        if inline:
            # THERMO block inside chem.inp overrides the thermo file
            data.update(parse_thermo_text(inline, set(s.upper() for s in self.species)))
        missing = [s for s in self.species if s.upper() not in data]
        if missing:
            raise MechanismError(f"no thermo data for species {missing}")
        self.thermo = {s: data[s.upper()] for s in self.species}
        self._A_override: Dict[int, float] = {}
        self._finish()

    @classmethod
    def from_files(cls, chemfile: str, thermfile: Optional[str] = None) -> "Mechanism":
        with open(chemfile) as f:
            chem = f.read()
        therm = None
        if thermfile:
            with open(thermfile) as f:
                therm = f.read()
        return cls(chem, therm)

    # ------------------------------------------------------------------ parsing
    def _parse_chem(self, text: str) -> None:
        self._inline_thermo = ""
        lines = [_strip_comment(l).rstrip() for l in text.splitlines()]
        section = None
        e_units = "CAL/MOLE"
        a_units = "MOLES"
        thermo_lines: List[str] = []
        current: Optional[Reaction] = None
        raw_lines = text.splitlines()
        for ln_no, line in enumerate(lines):
            s = line.strip()
            if not s:
                if section == "THERMO":
                    thermo_lines.append(raw_lines[ln_no])
                continue
            up = s.upper()
            head = up.split()[0]
            if section != "THERMO" and head in ("ELEMENTS", "ELEM"):
                section = "ELEMENTS"
                s = s.split(None, 1)[1] if len(s.split(None, 1)) > 1 else ""
                up = s.upper()
                if not s:
                    continue
            elif section != "THERMO" and head in ("SPECIES", "SPEC"):
                section = "SPECIES"
                s = s.split(None, 1)[1] if len(s.split(None, 1)) > 1 else ""
                up = s.upper()
                if not s:
                    continue
            elif section != "THERMO" and head in ("THERMO", "THER"):
                section = "THERMO"
                thermo_lines.append(raw_lines[ln_no])
                continue
            elif section != "THERMO" and head in ("REACTIONS", "REAC"):
                section = "REACTIONS"
                for tok in up.split()[1:]:
                    e_units, a_units = _unit_token(tok, e_units, a_units)  # other options ignored
                continue
            if up == "END" or up.startswith("END "):
                if section == "THERMO":
                    thermo_lines.append(raw_lines[ln_no])
                section = None
                current = None
                continue
            end_here = False
            if section in ("ELEMENTS", "SPECIES"):
                toks = s.split()
                if any(t.upper() == "END" for t in toks):
                    cut = [t.upper() for t in toks].index("END")
                    s = " ".join(toks[:cut])
                    end_here = True
            if section == "ELEMENTS":
                for tok in re.findall(r"([A-Za-z][A-Za-z0-9]*)\s*(?:/\s*(" + _NUM + r")\s*/)?", s):
                    el = tok[0].upper()
                    if el in self.elements:
                        continue
                    self.elements.append(el)
                    if tok[1]:
                        self.awt.append(_to_float(tok[1]))
                    elif el in ATOMIC_WEIGHTS:
                        self.awt.append(ATOMIC_WEIGHTS[el])
                    else:
                        raise MechanismError(f"unknown element {el} without atomic weight")
            elif section == "SPECIES":
                for tok in s.split():
                    if tok.upper() not in (x.upper() for x in self.species):
                        self.species.append(tok)
            if end_here:
                section = None
                current = None
                continue
            elif section == "THERMO":
                thermo_lines.append(raw_lines[ln_no])
            elif section == "REACTIONS":
                current = self._reaction_line(s, current, e_units, a_units)
        if thermo_lines:
            self._inline_thermo = "\n".join(thermo_lines)

    def _species_index_upper(self) -> Dict[str, str]:
        return {s.upper(): s for s in self.species}

    def _parse_side(self, side: str, eq: str) -> Tuple[List[Tuple[str, float]], Optional[str], bool]:
        """Return (species list, third body token, is_falloff)."""
        names = self._species_index_upper()
        third = None
        falloff = False
        m = re.search(r"\(\+\s*([^)]+)\)", side)
        if m:
            third = m.group(1).strip()
            falloff = True
            side = side[: m.start()] + side[m.end():]
        terms = []
        # split on '+' that separates terms; species names may contain '+' only in
        # ionic species (not supported), so a plain split is adequate
        for tok in [t for t in side.split("+") if t.strip()]:
            tok = tok.strip()
            up = tok.upper()
            if up == "M":
                if third is not None and not falloff:
                    raise MechanismError(f"two third bodies in {eq}")
                third = "M"
                continue
            if up in names:
                terms.append((names[up], 1.0))
                continue
            mm = re.match(r"^(\d+\.?\d*|\.\d+)(.+)$", tok)
            if mm and mm.group(2).upper() in names:
                terms.append((names[mm.group(2).upper()], float(mm.group(1))))
                continue
            raise MechanismError(f"unknown species {tok!r} in reaction {eq}")
        merged: Dict[str, float] = {}
        order: List[str] = []
        for sp, nu in terms:
            if sp not in merged:
                order.append(sp)
                merged[sp] = 0.0
            merged[sp] += nu
        return [(sp, merged[sp]) for sp in order], third, falloff

    def _reaction_line(self, s: str, current: Optional[Reaction], e_units: str, a_units: str) -> Optional[Reaction]:
        up = s.upper()
        is_aux = "=" not in s or re.match(
            r"^\s*(LOW|TROE|SRI|REV|HIGH|FORD|RORD|PLOG|DUP|DUPLICATE|UNITS|CHEB|TCHEB|PCHEB|LT|RLT)\b", up)
        if not is_aux:
            toks = s.split()
            if len(toks) < 4:
                raise MechanismError(f"reaction line needs equation + A b E: {s!r}")
            A, b, E = _to_float(toks[-3]), _to_float(toks[-2]), _to_float(toks[-1])
            eq = "".join(toks[:-3])
            if "<=>" in eq:
                lhs, rhs = eq.split("<=>")
                rev = True
            elif "=>" in eq:
                lhs, rhs = eq.split("=>")
                rev = False
            elif "=" in eq:
                lhs, rhs = eq.split("=")
                rev = True
            else:
                raise MechanismError(f"no '=' in {eq}")
            r_sp, r_tb, r_fo = self._parse_side(lhs, eq)
            p_sp, p_tb, p_fo = self._parse_side(rhs, eq)
            if (r_tb is None) != (p_tb is None) or r_fo != p_fo:
                raise MechanismError(f"unbalanced third body in {eq}")
            rx = Reaction(eq, r_sp, p_sp, rev, A, b, E)
            if r_fo:
                rx.kind = RXN_FALLOFF
                rx.third_body = r_tb.upper() if r_tb.upper() == "M" else self._species_index_upper().get(r_tb.upper(), r_tb)
                if rx.third_body != "M" and rx.third_body not in self.species:
                    raise MechanismError(f"unknown falloff collider {r_tb} in {eq}")
            elif r_tb is not None:
                rx.kind = RXN_THIRDBODY
                rx.third_body = "M"
            rx.E_scale = _e_to_kelvin(e_units)
            rx.A_scale_per_order = 1.0 / AVOGADRO if a_units == "MOLECULES" else 1.0
            self.reactions.append(rx)
            return rx
        if current is None:
            raise MechanismError(f"auxiliary data before any reaction: {s!r}")
        # auxiliary line: keywords with /values/ and efficiency pairs
        for key, vals in re.findall(r"([A-Za-z0-9()\-,*#\[\]_]+)\s*(?:/([^/]*)/)?", s):
            k = key.upper()
            if not k:
                continue
            # FORD / RORD carry "species order"; every other keyword numbers only
            nums = [_to_float(v) for v in vals.split()] if vals and k not in ("FORD", "RORD", "UNITS") else []
            if k in ("DUP", "DUPLICATE"):
                current.duplicate = True
            elif k == "LOW":
                current.low = tuple(nums[:3])
                if current.kind != RXN_FALLOFF:
                    raise MechanismError(f"LOW on a non-falloff reaction {current.equation}")
            elif k == "HIGH":
                # chemically activated: only a (+M) pressure-dependent reaction can carry HIGH
                if current.kind not in (RXN_FALLOFF, RXN_CHEMACT) or current.third_body is None:
                    raise MechanismError(f"HIGH on a reaction without (+M): {current.equation}")
                current.high = tuple(nums[:3])
                current.kind = RXN_CHEMACT
            elif k == "TROE":
                current.troe = tuple(nums)
            elif k == "SRI":
                if len(nums) not in (3, 5):
                    raise MechanismError(f"SRI needs 3 or 5 parameters: {current.equation}")
                current.sri = tuple(nums)
            elif k == "REV":
                current.rev = tuple(nums[:3])
            elif k in ("FORD", "RORD"):
                parts = vals.split() if vals else []
                names = self._species_index_upper()
                if len(parts) != 2 or parts[0].upper() not in names:
                    raise MechanismError(f"{k} needs /species order/: {s!r}")
                (current.ford if k == "FORD" else current.rord)[names[parts[0].upper()]] = _to_float(parts[1])
            elif k == "PLOG":
                current.plog.append(tuple(nums[:4]))
            elif k == "CHEB":
                current.cheb.extend(nums)
            elif k in ("TCHEB", "PCHEB"):
                if len(nums) != 2:
                    raise MechanismError(f"{k} needs /min max/: {s!r}")
                if k == "TCHEB":
                    current.tcheb = (nums[0], nums[1])
                else:
                    current.pcheb = (nums[0], nums[1])
            elif k in ("LT", "RLT"):
                if len(nums) != 2:
                    raise MechanismError(f"{k} needs /B C/: {s!r}")
                if k == "LT":
                    current.lt = (nums[0], nums[1])
                else:
                    current.rlt = (nums[0], nums[1])
            elif k == "UNITS":
                # per-reaction units: this reaction's A and E (and its LOW / HIGH / REV / PLOG
                # parameters) are in them (Chemkin's UNITS auxiliary keyword, e.g. UNITS /KCAL/)
                toks = vals.split() if vals else []
                if not toks:
                    raise MechanismError(f"UNITS needs /unit .../: {s!r}")
                e_u = a_u = None
                for t in toks:
                    e2, a2 = _unit_token(t.upper(), None, None)
                    if e2 is None and a2 is None:
                        raise MechanismError(f"unknown UNITS {t!r} for {current.equation}")
                    e_u, a_u = e2 or e_u, a2 or a_u
                if e_u is not None:
                    current.E_scale = _e_to_kelvin(e_u)
                if a_u is not None:
                    current.A_scale_per_order = 1.0 / AVOGADRO if a_u == "MOLECULES" else 1.0
            else:
                names = self._species_index_upper()
                if k in names:
                    if current.kind == RXN_ELEMENTARY:
                        raise MechanismError(f"efficiency on a reaction without +M: {current.equation}")
                    current.efficiencies[names[k]] = nums[0] if nums else 1.0
                else:
                    raise MechanismError(f"unknown auxiliary keyword {key!r} for {current.equation}")
        return current

    # --------------------------------------------------------------- finishing
    def _finish(self) -> None:
        KK, MM = len(self.species), len(self.elements)
        self.ncf = np.zeros((MM, KK), dtype=np.int32)
        for k, sp in enumerate(self.species):
            for el, n in self.thermo[sp].composition.items():
                if el not in self.elements:
                    raise MechanismError(f"species {sp} uses undeclared element {el}")
                self.ncf[self.elements.index(el), k] = n
        self.wt = (np.asarray(self.awt, dtype=np.float64)[:, None] * self.ncf).sum(axis=0)
        for rx in self.reactions:
            # FORD / RORD change the order of a species already on that side (Chemkin: the
            # concentration exponent of that reactant / product in the forward / reverse rate)
            for sp in rx.ford:
                if sp not in [r for r, _ in rx.reactants]:
                    raise MechanismError(f"FORD species {sp} is not a reactant of {rx.equation}")
            for sp in rx.rord:
                if sp not in [p for p, _ in rx.products]:
                    raise MechanismError(f"RORD species {sp} is not a product of {rx.equation}")
            if rx.rord and not rx.reversible:
                raise MechanismError(f"RORD on an irreversible reaction {rx.equation}")
            # element balance check
            bal = np.zeros(MM)
            for sp, nu in rx.products:
                bal += nu * self.ncf[:, self.species.index(sp)]
            for sp, nu in rx.reactants:
                bal -= nu * self.ncf[:, self.species.index(sp)]
            if np.any(np.abs(bal) > 1e-6):
                raise MechanismError(f"reaction {rx.equation} is not element balanced")

    # ------------------------------------------------------------------ sizes
    @property
    def KK(self) -> int:
        return len(self.species)

    @property
    def II(self) -> int:
        return len(self.reactions)

    @property
    def MM(self) -> int:
        return len(self.elements)

    def set_A_cgs(self, i: int, A: float) -> None:
        """Override the forward pre-exponential factor of reaction i (0-based) in cgs units."""
        if not (0 <= i < self.II) or not (A > 0.0):
            raise MechanismError("bad reaction index or A-factor")
        self._A_override[i] = float(A)

    def A_cgs(self, i: int) -> float:
        rx = self.reactions[i]
        if i in self._A_override:
            return self._A_override[i]
        return self._A_cgs(rx, rx.A, rx.reactants, True, 1 if rx.kind in (RXN_THIRDBODY, RXN_CHEMACT) else 0)

    def arrhenius(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """A [cgs], b, E/R [K] as KINGetReactionRateParameters returns them."""
        A = np.array([self.A_cgs(i) for i in range(self.II)])
        b = np.array([rx.b for rx in self.reactions])
        E = np.array([rx.E * rx.E_scale for rx in self.reactions])
        return A, b, E

    def _cheb_rows(self, rx: Reaction):
        """plog_par rows of a Chebyshev reaction: (NT, NP, 0, 0), (Tmin, Tmax, Pmin, Pmax) [K, atm],
        then the NT x NP coefficients of log10 k (temperature-major, 4 per row, zero padded), k in
        cgs mole units (a MOLECULES-unit reaction shifts a_00 by (order - 1) log10 N_A)."""
        if rx.kind not in (RXN_FALLOFF,) or rx.third_body != "M":
            raise MechanismError(f"CHEB needs a (+M) reaction ({rx.equation})")
        if rx.low is not None or rx.high is not None or rx.troe is not None or rx.sri is not None or rx.plog or \
                rx.rev is not None:
            raise MechanismError(f"CHEB with LOW / HIGH / TROE / SRI / PLOG / REV ({rx.equation})")
        if len(rx.cheb) < 2:
            raise MechanismError(f"CHEB needs /NT NP/ then the coefficients ({rx.equation})")
        nt, npr = int(rx.cheb[0]), int(rx.cheb[1])
        coef = list(rx.cheb[2:])
        if nt != rx.cheb[0] or npr != rx.cheb[1] or not (1 <= nt <= CHEB_MAX and 1 <= npr <= CHEB_MAX) or \
                len(coef) != nt * npr:
            raise MechanismError(f"CHEB needs NT x NP coefficients with 1 <= NT, NP <= {CHEB_MAX} ({rx.equation})")
        tmin, tmax = rx.tcheb if rx.tcheb is not None else (300.0, 2500.0)
        pmin, pmax = rx.pcheb if rx.pcheb is not None else (0.001, 100.0)
        if not (0.0 < tmin < tmax and 0.0 < pmin < pmax):
            raise MechanismError(f"TCHEB / PCHEB ranges must be positive and increasing ({rx.equation})")
        if rx.A_scale_per_order != 1.0:
            coef[0] += (self._order(rx.reactants, 0) - 1.0) * math.log10(AVOGADRO)
        coef += [0.0] * (-len(coef) % 4)
        rows = [(float(nt), float(npr), 0.0, 0.0), (tmin, tmax, pmin, pmax)]
        rows += [tuple(coef[j:j + 4]) for j in range(0, len(coef), 4)]
        return rows

    @staticmethod
    def _order(terms, third_extra: int) -> float:
        return sum(nu for _, nu in terms) + third_extra

    def _A_cgs(self, rx: Reaction, A: float, side, forward: bool, extra: int = 0) -> float:
        if rx.A_scale_per_order == 1.0:
            return A
        order = self._order(side, extra)
        return A * (AVOGADRO ** (order - 1.0))

    # ------------------------------------------------------------- device tables
    def to_tables(self) -> Dict[str, np.ndarray]:
        """Flatten to the ckmi_mech_desc layout (include/ckmi.h).

        Fixed MAX_SLOTS species per side; third-body efficiency lists in CSR.
        """
        KK, II = self.KK, self.II
        S = MAX_SLOTS
        idx = {s: k for k, s in enumerate(self.species)}
        rtype = np.zeros(II, np.int32)
        rev = np.zeros(II, np.int32)
        nr = np.zeros(II, np.int32)
        np_ = np.zeros(II, np.int32)
        rsp = np.zeros((II, S), np.int32)
        psp = np.zeros((II, S), np.int32)
        rnu = np.zeros((II, S), np.float64)
        pnu = np.zeros((II, S), np.float64)
        ford = np.zeros((II, S), np.float64)     # forward order of each reactant slot (FORD, else nu)
        rord = np.zeros((II, S), np.float64)     # reverse order of each product slot (RORD, else nu)
        arr = np.zeros((II, 3), np.float64)      # ln A, b, E/R  (forward / high-pressure)
        low = np.zeros((II, 3), np.float64)      # ln A0, b0, E0/R
        revp = np.zeros((II, 3), np.float64)     # explicit REV: ln Ar, br, Er/R
        has_rev = np.zeros(II, np.int32)
        ftype = np.zeros(II, np.int32)
        fpar = np.zeros((II, 5), np.float64)     # TROE a,T3,T1,T2  or SRI a,b,c,d,e
        tbsp = np.full(II, -1, np.int32)         # -1 = mixture "M", else collider species
        eff_ptr = [0]
        eff_sp: List[int] = []
        eff_val: List[float] = []
        plog_ptr = np.zeros(II + 1, np.int32)     # CSR into plog_par (rtype TAB_PLOG; TAB_CHEB rows, _cheb_rows)
        plog_par: List[Tuple[float, float, float, float]] = []  # ln P [dyn/cm2], ln A [cgs], b, E/R
        for i, rx in enumerate(self.reactions):
            if rx.cheb:
                plog_par.extend(self._cheb_rows(rx))
            if rx.lt is not None or rx.rlt is not None:
                if rx.kind != RXN_ELEMENTARY or rx.plog or rx.cheb:
                    raise MechanismError(f"LT / RLT on a pressure-dependent or third-body reaction ({rx.equation})")
                if rx.rlt is not None and rx.rev is None:
                    raise MechanismError(f"RLT without REV ({rx.equation})")
            if rx.plog:
                if rx.kind != RXN_ELEMENTARY or rx.rev is not None:
                    raise MechanismError(f"PLOG on a third-body/falloff reaction or with REV ({rx.equation})")
                pts = sorted(rx.plog, key=lambda e: e[0])
                if any(pts[j][0] == pts[j + 1][0] for j in range(len(pts) - 1)) or pts[0][0] <= 0.0:
                    raise MechanismError(f"PLOG pressures must be positive and distinct ({rx.equation})")
                for p_atm, a, b, e in pts:
                    Ap = self._A_cgs(rx, a, rx.reactants, True, 0)
                    plog_par.append((math.log(p_atm * P_ATM), math.log(Ap), b, e * rx.E_scale))
            if len(rx.reactants) > S or len(rx.products) > S:
                raise MechanismError(f"more than {S} species on one side of {rx.equation}")
            if rx.cheb:
                rtype[i] = TAB_CHEB
            elif rx.lt is not None or rx.rlt is not None:
                rtype[i] = TAB_LT
            else:
                rtype[i] = TAB_PLOG if rx.plog else (TAB_CHEMACT if rx.kind == RXN_CHEMACT else rx.kind)
            plog_ptr[i + 1] = len(plog_par)
            rev[i] = 1 if rx.reversible else 0
            nr[i] = len(rx.reactants)
            np_[i] = len(rx.products)
            for j, (sp, nu) in enumerate(rx.reactants):
                rsp[i, j] = idx[sp]
                rnu[i, j] = nu
                ford[i, j] = rx.ford.get(sp, nu)
            for j, (sp, nu) in enumerate(rx.products):
                psp[i, j] = idx[sp]
                pnu[i, j] = nu
                rord[i, j] = rx.rord.get(sp, nu)
            extra = 1 if rx.kind == RXN_THIRDBODY else 0
            A = self.A_cgs(i)
            arr[i] = (math.log(A) if A > 0 else -1e300, rx.b, rx.E * rx.E_scale)
            if rx.cheb:  # the rate is the series alone: no [M], no falloff, no efficiencies
                eff_ptr.append(len(eff_sp))
                continue
            if rx.lt is not None or rx.rlt is not None:
                low[i, :2] = rx.lt if rx.lt is not None else (0.0, 0.0)
                fpar[i, :2] = rx.rlt if rx.rlt is not None else (0.0, 0.0)
            if rx.kind in (RXN_FALLOFF, RXN_CHEMACT):
                if rx.kind == RXN_FALLOFF and rx.low is None:
                    raise MechanismError(f"falloff reaction without LOW: {rx.equation}")
                if rx.kind == RXN_CHEMACT and (rx.high is None or rx.low is not None):
                    raise MechanismError(f"chemically activated reaction needs HIGH and no LOW: {rx.equation}")
                # falloff: low[] = LOW (k0, main line = k_inf); chemically activated: low[] = HIGH
                # (k_inf, main line = k0), Chemkin's k = k0 F / (1 + Pr) with Pr = k0 [M] / k_inf
                lim = rx.low if rx.kind == RXN_FALLOFF else rx.high
                A0 = self._A_cgs(rx, lim[0], rx.reactants, True, 1 if rx.kind == RXN_FALLOFF else 0)
                low[i] = (math.log(A0), lim[1], lim[2] * rx.E_scale)
                if rx.troe is not None:
                    t = list(rx.troe)
                    if len(t) == 3:
                        ftype[i] = FALL_TROE3
                        fpar[i, :3] = t
                    elif len(t) == 4:
                        ftype[i] = FALL_TROE4
                        fpar[i, :4] = t
                    else:
                        raise MechanismError(f"TROE needs 3 or 4 parameters: {rx.equation}")
                elif rx.sri is not None:
                    ftype[i] = FALL_SRI
                    sri = list(rx.sri) + ([1.0, 0.0] if len(rx.sri) == 3 else [])
                    fpar[i, :5] = sri[:5]
                else:
                    ftype[i] = FALL_LINDEMANN
                if rx.third_body != "M":
                    tbsp[i] = idx[rx.third_body]
            if rx.rev is not None:
                if not rx.reversible:
                    raise MechanismError(f"REV on an irreversible reaction {rx.equation}")
                has_rev[i] = 1
                Ar = self._A_cgs(rx, rx.rev[0], rx.products, False, extra)
                revp[i] = (math.log(Ar) if Ar > 0 else -1e300, rx.rev[1], rx.rev[2] * rx.E_scale)
            if rx.kind in (RXN_THIRDBODY, RXN_FALLOFF, RXN_CHEMACT) and tbsp[i] < 0:
                for sp, val in rx.efficiencies.items():
                    eff_sp.append(idx[sp])
                    eff_val.append(val)
            eff_ptr.append(len(eff_sp))
        thermo = np.zeros((KK, 17), np.float64)  # tlow, tmid, thigh, low[7], high[7]
        for k, sp in enumerate(self.species):
            th = self.thermo[sp]
            thermo[k, 0] = th.tlow
            thermo[k, 1] = th.tmid
            thermo[k, 2] = th.thigh
            thermo[k, 3:10] = th.low
            thermo[k, 10:17] = th.high
        return dict(
            KK=np.int32(KK), II=np.int32(II), wt=self.wt.astype(np.float64), thermo=thermo,
            rtype=rtype, rev=rev, nr=nr, np=np_, rsp=rsp, psp=psp, rnu=rnu, pnu=pnu, ford=ford, rord=rord,
            arr=arr, low=low, revp=revp, has_rev=has_rev, ftype=ftype, fpar=fpar, tbsp=tbsp,
            eff_ptr=np.asarray(eff_ptr, np.int32), eff_sp=np.asarray(eff_sp, np.int32),
            eff_val=np.asarray(eff_val, np.float64),
            plog_ptr=plog_ptr,
            plog_par=np.asarray(plog_par if plog_par else [(0.0, 0.0, 0.0, 0.0)], np.float64).reshape(-1, 4),
            # element counts (KINGetGasSpeciesComposition): the reactors' element projection
            MM=np.int32(self.ncf.shape[0]), ncf=np.ascontiguousarray(self.ncf, np.int32),
        )


def _unit_token(tok: str, e_units, a_units):
    """A REACTIONS-line unit keyword or a UNITS abbreviation (MOLE, MOLC, CAL, KCAL, JOUL, KJOU,
    KELV, EVOL) -> updated (e_units, a_units); anything else leaves both unchanged."""
    t = tok.upper()
    if t.startswith(("MOLEC", "MOLC")):
        return e_units, "MOLECULES"
    if t.startswith("MOLE"):
        return e_units, "MOLES"
    for pre, name in (("KCAL", "KCAL/MOLE"), ("CAL", "CAL/MOLE"), ("KJOU", "KJOULES/MOLE"), ("JOUL", "JOULES/MOLE"),
                      ("KELV", "KELVINS"), ("EVOL", "EVOLTS")):
        if t.startswith(pre):
            return name, a_units
    return e_units, a_units


def _e_to_kelvin(units: str) -> float:
    """Factor converting the file's activation-energy unit to E/R [K]."""
    if units == "CAL/MOLE":
        return 1.0 / RUC_ACT
    if units == "KCAL/MOLE":
        return 1.0e3 / RUC_ACT
    if units == "JOULES/MOLE":
        return 1.0 / (RU_ACT * 1.0e-7)
    if units == "KJOULES/MOLE":
        return 1.0e3 / (RU_ACT * 1.0e-7)
    if units == "KELVINS":
        return 1.0
    if units == "EVOLTS":
        return 1.602176487e-12 / 1.3806504e-16
    raise MechanismError(f"unknown energy units {units}")
