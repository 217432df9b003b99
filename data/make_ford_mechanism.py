"""Write data/gri30_ford_chem.inp: GRI-Mech 3.0 with FORD / RORD orders and non-integral
stoichiometric coefficients.

No mechanism with FORD, RORD or fractional coefficients ships with the reference or exists
offline, so this stand-in exercises those paths (Chemkin ``FORD /species order/`` and
``RORD /species order/`` auxiliary lines, real coefficients such as ``1.5O2``) on a mechanism
whose thermo and other reactions are GRI-3.0's:
  * FORD on three elementary reactions (orders 1.2, 0.8 and 2 -> 1.5), RORD on two reversible
    ones (the reverse rate then uses the given product exponent; K_c is unchanged);
  * two global reactions with fractional coefficients appended: the irreversible
    ``CH4+1.5O2=>CO+2H2O`` with FORD /CH4 0.7/ /O2 0.8/ (Westbrook-Dryer form) and the reversible
    ``CO+0.5O2<=>CO2`` (Delta nu = -1/2 in K_c) with FORD /O2 0.25/ and RORD /CO2 1.0/.
Their A-factors are small enough that ignition behaves like GRI-3.0's.  Parity with Chemkin itself
is unpinned (no golden uses FORD / RORD); the C oracle, its numpy restatement and the GPU kernels
are checked against each other (tests/test_ford.py, tests/test_gpu_ford.py).

Run: python data/make_ford_mechanism.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "grimech30_chem.inp")
DST = os.path.join(HERE, "gri30_ford_chem.inp")

# equation -> auxiliary line appended after its main line
AUX = {
    "O+CH4<=>OH+CH3": "     FORD / CH4 1.2 /",
    "OH+CH2O<=>HCO+H2O": "     FORD / OH 0.8 / RORD / H2O 1.1 /",
    "2OH<=>O+H2O": "     FORD / OH 1.5 /",
    "HO2+CH3<=>OH+CH3O": "     RORD / OH 0.9 /",
}
GLOBAL = [
    "CH4+1.5O2=>CO+2H2O                       2.000E+09    0.000   30000.00",
    "     FORD / CH4 0.7 / FORD / O2 0.8 /",
    "CO+0.5O2<=>CO2                           1.000E+08    0.000   40000.00",
    "     FORD / O2 0.25 / RORD / CO2 1.0 /",
]


def main():
    out, seen = [], set()
    with open(SRC) as f:
        lines = f.read().splitlines()
    last_end = max(i for i, ln in enumerate(lines) if ln.split()[:1] == ["END"])  # end of REACTIONS
    for j, ln in enumerate(lines):
        tok = ln.split()
        if j == last_end:
            out.extend(GLOBAL)
        out.append(ln)
        if len(tok) == 4 and tok[0] in AUX and tok[0] not in seen:
            seen.add(tok[0])
            out.append(AUX[tok[0]])
    missing = set(AUX) - seen
    if missing:
        raise SystemExit(f"reactions not found: {sorted(missing)}")
    with open(DST, "w") as f:
        f.write("\n".join(out) + "\n")
    print(DST)


if __name__ == "__main__":
    main()
