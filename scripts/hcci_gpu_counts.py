"""GPU check: the hcciengine golden's pressure / Cp within-tolerance counts and peak CA, drop-in path."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pychemkin_amd as ck  # noqa: E402
from conftest import CHEM, THERM, TRAN, golden, within  # noqa: E402
from pychemkin_amd.engines.HCCI import HCCIengine  # noqa: E402
import test_engine as te  # noqa: E402

chem = ck.Chemistry(chem=CHEM, therm=THERM, tran=TRAN, label="GRI 3.0")
assert chem.preprocess() == 0
fresh = ck.Mixture(chem)
fresh.temperature, fresh.pressure = te.T_IVC, te.P_IVC
fresh.Y = te.charge_Y(chem._mech)
E = te.ENG
e = HCCIengine(reactor_condition=fresh, nzones=1)
e.bore, e.stroke, e.connecting_rod_length = E["bore"], E["stroke"], E["rod"]
e.compression_ratio, e.RPM = E["cr"], E["rpm"]
e.set_piston_pin_offset(offset=E["polen"])
e.starting_CA, e.ending_CA = E["ca0"], E["ca1"]
e.set_wall_heat_transfer("dimensionless", list(E["ht"]), E["twall"])
e.set_gas_velocity_correlation(list(E["gvel"]))
e.set_piston_head_area(area=E["pis"])
e.set_cylinder_head_area(area=E["cyl"])
e.CAstep_for_saving_solution = 0.5
e.tolerances = (1.0e-12, 1.0e-10)
e.force_nonnegative = True
e.set_ignition_delay(method="T_inflection")
assert e.run() == 0
e.process_engine_solution()
n = e.getnumbersolutionpoints()
pres = e.get_solution_variable_profile("pressure") * 1e-6
cp = np.array([e.get_solution_mixture_at_index(solution_index=i).CPBL() for i in range(n)]) * 1e-10
g = golden("hcciengine")
Pg = np.asarray(g["state-pressure"])
ok = within(pres, Pg, *g["tolerance-var"])
okc = within(cp, np.asarray(g["state-Cp"]), *g["tolerance-var"])
ca = np.asarray(g["state-crank_angle"])
print(json.dumps({"P_ok": int(ok.sum()), "P_first_bad": int(np.argmin(ok)), "Cp_ok": int(okc.sum()),
                  "Cp_first_bad": int(np.argmin(okc)), "peak_ca": float(ca[np.argmax(pres)]),
                  "golden_peak_ca": float(ca[np.argmax(Pg)]), "ign_ca": float(e.get_ignition_delay())}))
