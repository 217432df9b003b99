"""Write gri30_tracer161_chem.inp / gri30_tracer161_thermo.dat: a synthetic 161-species mechanism.

SURVEY.md 8(d) configs[4] asks for a ~160-species mechanism (reduced n-heptane); none exists
offline, so the large-mechanism kernels (ROP/thermo with more than 63 species, the batched MFMA
LU of n = 162 Newton matrices) are exercised on this one and checked against the oracle, not
against the reference (parity with Chemkin unpinned for this size).  Run
``python data/make_tracer_mechanism.py`` to regenerate the two files next to this script.
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CHEM = os.path.join(HERE, "grimech30_chem.inp")
THERM = os.path.join(HERE, "grimech30_thermo.dat")

N_TRACER = 108  # GRI-3.0 + 108 = 161 species: the configs[4] size (n = KK + 1 = 162)


def write_big_mechanism(dirpath=HERE, n_tracer=N_TRACER):
    """A synthetic > 63-species mechanism for the large-mechanism kernels (no ~160-species
    mechanism exists offline; SURVEY 8c: parity for configs[4] is unpinned against the reference).

    GRI-Mech 3.0 plus n_tracer argon pseudo-species AX1..AXn (composition AR, NASA-7 of AR with
    the enthalpy offset shifted by 10 K per index, so every exchange has K_c != 1), coupled by
    elementary (AXk + H <=> AXk+1 + H), coefficient-2 (2AXk <=> AXk+1 + AXk-1), third-body (with
    AX and H2O efficiencies) and Troe falloff reactions, so species indices > 63 occur in every
    reaction type, in efficiency lists and as duplicated slots.  Returns (chem_path, therm_path)."""
    chem = open(CHEM).read().splitlines()
    therm = open(THERM).read().splitlines()
    names = [f"AX{k}" for k in range(1, n_tracer + 1)]
    out, in_species = ["! SYNTHETIC test mechanism written by data/make_tracer_mechanism.py: GRI-Mech 3.0",
                       f"! + {n_tracer} argon tracer species AX1..AX{n_tracer} and their exchange reactions.",
                       "! Not a physical mechanism; the GRI-Mech 3.0 header below describes the base set."], False
    for line in chem:
        if line.strip().upper() == "SPECIES":
            in_species = True
        elif in_species and line.strip().upper() == "END":
            for i in range(0, len(names), 8):
                out.append("  ".join(names[i:i + 8]))
            in_species = False
        out.append(line)
    # drop the final END and append the tracer reactions
    while out and out[-1].strip().upper() != "END":
        out.pop()
    out.pop()
    for k in range(1, n_tracer):
        a, b = f"AX{k}", f"AX{k + 1}"
        out.append(f"{a}+H<=>{b}+H    1.000E+12   0.500   1000.00")
        if k % 3 == 2:
            out.append(f"2{a}<=>{b}+AX{k - 1}    1.000E+10   0.000   2000.00")
        if k % 5 == 1 and k + 2 <= n_tracer:
            out.append(f"{a}+M<=>{b}+M    1.000E+14   0.000   5000.00")
            out.append(f"AX{k + 2}/2.00/ H2O/5.00/")
        if k % 7 == 3:
            out.append(f"{a}(+M)<=>{b}(+M)    1.000E+10   0.000  10000.00")
            out.append("LOW/ 1.000E+16 0.000 8000.00/")
            out.append("TROE/ 0.5000 100.00 1000.00 1000.00/")
    out.append("END")
    tout = [t for t in therm if t.strip().upper() != "END"]
    i_ar = next(i for i, t in enumerate(therm) if t.startswith("AR "))
    ar = therm[i_ar:i_ar + 4]
    for k, nm in enumerate(names, start=1):
        l1 = nm.ljust(18) + ar[0][18:]
        h5 = -745.375 + 10.0 * k
        l3 = f"{h5:15.8E}" + ar[2][15:30] + f"{2.5:15.8E}" + ar[2][45:]
        l4 = ar[3][:30] + f"{h5:15.8E}" + ar[3][45:]
        tout += [l1, ar[1], l3, l4]
    tout.append("END")
    cp = os.path.join(dirpath, "gri30_tracer161_chem.inp")
    tp = os.path.join(dirpath, "gri30_tracer161_thermo.dat")
    with open(cp, "w") as f:
        f.write("\n".join(out) + "\n")
    with open(tp, "w") as f:
        f.write("\n".join(tout) + "\n")
    return cp, tp


if __name__ == "__main__":
    print(write_big_mechanism())
