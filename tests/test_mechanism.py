"""Host mechanism compiler (pychemkin_amd/mechanism.py) against the reference's data pins."""
import numpy as np
import pytest

from conftest import golden
from pychemkin_amd.mechanism import Mechanism, MechanismError, parse_thermo_text


def test_sizes_and_order(mech):
    # GRI-3.0: 53 species, 325 reactions, 5 elements; O2 at index 3 and N2 at 47 (simple.baseline)
    assert (mech.KK, mech.II, mech.MM) == (53, 325, 5)
    x = np.asarray(golden("simple")["species-mole_fraction"])
    assert x[mech.species.index("O2")] == 0.21 and x[mech.species.index("N2")] == 0.79
    assert mech.elements == ["O", "H", "C", "N", "AR"]


def test_atomic_weights_are_chemkin_defaults(mech):
    awt = dict(zip(mech.elements, mech.awt))
    assert awt["H"] == 1.00797 and awt["C"] == 12.01115 and awt["O"] == 15.9994 and awt["N"] == 14.0067


def test_golden_reaction_indices(mech):
    # reactionrates.baseline lists reactions 180, 0, 210, 117, 51 (0-based) as the only nonzero ones
    eq = {i: mech.reactions[i].equation for i in golden("reactionrates")["state-order_1800"]}
    assert eq[0] == "2O+M<=>O2+M"
    assert eq[51] == "H+CH3(+M)<=>CH4(+M)"
    assert eq[117] == "HO2+CH3<=>O2+CH4"
    assert eq[180] == "N2O+O<=>N2+O2"
    assert eq[210] == "NNH+CH3<=>CH4+N2"


def test_reaction_details(mech):
    r = mech.reactions[51]
    assert r.low == (2.62e33, -4.76, 2440.0) and r.troe == (0.783, 74.0, 2941.0, 6964.0)
    assert r.efficiencies["CH4"] == 3.0
    assert sum(x.duplicate for x in mech.reactions) == 6
    assert sum(not x.reversible for x in mech.reactions) == 16
    kinds = [x.kind for x in mech.reactions]
    assert kinds.count(0) == 284 and kinds.count(1) == 12 and kinds.count(2) == 29


def test_nasa7_continuity_at_tmid(mech):
    for sp, th in mech.thermo.items():
        T = th.tmid
        for a, b in ((th.low, th.high),):
            cp = lambda c: c[0] + c[1] * T + c[2] * T**2 + c[3] * T**3 + c[4] * T**4
            h = lambda c: c[0] + c[1] * T / 2 + c[2] * T**2 / 3 + c[3] * T**3 / 4 + c[4] * T**4 / 5 + c[5] / T
            assert abs(cp(a) - cp(b)) < 2e-4, sp
            assert abs(h(a) - h(b)) < 1e-4, sp


def test_tables_layout(tables):
    assert tables["rsp"].shape == (325, 8) and tables["arr"].shape == (325, 3)  # CKMI_SLOTS = 8
    assert tables["thermo"].shape == (53, 17)
    assert tables["eff_ptr"].shape == (326,)
    # E/R of H+O2<=>O+OH: 17041 cal/mol / RUC, Chemkin's activation-energy gas constant
    # (8.314510e7 / 4.184e7 cal/mol-K, mechanism.RU_ACT), not constants.R_GAS_CAL
    assert abs(tables["arr"][37, 2] / (17041.0 / (8.314510e7 / 4.184e7)) - 1) < 1e-14


CHEM_MINI = """ELEMENTS H O N END
SPECIES H2 O2 H O OH H2O N2 HO2 END
REACTIONS KJOULES/MOLE
H+O2<=>O+OH   3.5E15 -0.406 69.45
H2+O=OH+H     5.0E4 2.67 26.3
  REV / 1.0E4 2.6 20.0 /
H+O2(+N2)<=>HO2(+N2)   4.65E12 0.44 0.0
  LOW/ 6.37E20 -1.72 2.1/
  SRI/ 0.5 100. 1000. /
2OH(+M)=H2O+O(+M)      1.0E12 0.0 0.0
  LOW/1.0E16 0.0 0.0/
H2O+M=H+OH+M    1.0E20 -1.0 400.
 H2O/12.0/ N2/1.5/
END
"""


def test_parser_variants(mech):
    therm = open(__import__("conftest").THERM).read()
    m = Mechanism(CHEM_MINI, therm)
    assert m.KK == 8 and m.II == 5
    r1 = m.reactions[1]
    assert r1.rev == (1.0e4, 2.6, 20.0)
    assert abs(r1.E * r1.E_scale - 26.3e3 / 8.31447247) < 1e-6 * 26.3e3
    assert m.reactions[2].third_body == "N2" and m.reactions[2].sri == (0.5, 100.0, 1000.0)
    t = m.to_tables()
    assert t["tbsp"][2] == m.species.index("N2") and t["ftype"][2] == 4 and t["has_rev"][1] == 1
    assert t["ftype"][3] == 1  # Lindemann
    assert m.reactions[4].efficiencies == {"H2O": 12.0, "N2": 1.5}


def test_parser_errors():
    therm = open(__import__("conftest").THERM).read()
    with pytest.raises(MechanismError):
        Mechanism("ELEMENTS H O END\nSPECIES H2 O2 END\nREACTIONS\nH2+O2=OH+OH 1 0 0\nEND\n", therm)
    with pytest.raises(MechanismError):  # element imbalance
        Mechanism("ELEMENTS H O END\nSPECIES H2 O2 H2O END\nREACTIONS\nH2+O2=H2O 1 0 0\nEND\n", therm)


def test_thermo_parser_roundtrip(mech):
    text = open(__import__("conftest").THERM).read()
    d = parse_thermo_text(text)
    assert len(d) == 53 and d["N2"].composition == {"N": 2}


def test_tracer_mechanism_files_match_generator(tmp_path):
    """data/gri30_tracer161_* (the configs[4]-sized stand-in) are exactly what
    data/make_tracer_mechanism.py writes, and parse to KK = 161, II = 505."""
    import importlib.util
    import os

    from conftest import BIG_CHEM, BIG_THERM, ROOT
    from pychemkin_amd.mechanism import Mechanism

    spec = importlib.util.spec_from_file_location("mtm", os.path.join(ROOT, "data", "make_tracer_mechanism.py"))
    mtm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mtm)
    cp, tp = mtm.write_big_mechanism(str(tmp_path))
    assert open(cp).read() == open(BIG_CHEM).read()
    assert open(tp).read() == open(BIG_THERM).read()
    m = Mechanism.from_files(BIG_CHEM, BIG_THERM)
    assert (m.KK, m.II) == (161, 505)
    assert m.species[53] == "AX1" and m.species[-1] == "AX108"
