"""Convert the reference's golden result files into JSON fixtures (run in the dev container).

Source: /root/reference/tests/baseline/<name>.baseline (Python dict literals produced by the
licensed Chemkin, compared by tests/test_pychemkin_comparisons.py in the reference).  Only
the data values are kept; the inputs that produced them are restated in the tests that use
the fixtures, with the reference script file:line they come from.
"""
import ast
import json
import os

SRC = "/root/reference/tests/baseline"
HERE = os.path.dirname(os.path.abspath(__file__))
KEEP = {
    "closed_homogeneous__transient": None,
    "CONV": None,
    "reactionrates": None,
    "simple": None,
    "speciesproperties": ["tolerance-var", "tolerance-frac", "tolerance-ROP", "state-temperature", "state-Cv",
                          "state-conductivity"],
    "createmixture": ["tolerance-var", "tolerance-frac", "tolerance-ROP", "state-temperature", "state-density"],
    "sensitivity": None,
    "adiabaticflametemperature": None,
    "equilibriumcomposition": None,
    "mixturemixing": None,
    "plugflow": None,
    "hcciengine": None,
}

if __name__ == "__main__":
    for name, keys in KEEP.items():
        with open(os.path.join(SRC, name + ".baseline")) as f:
            d = ast.literal_eval(f.read())
        if keys is not None:
            d = {k: d[k] for k in keys}
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(d, f, indent=0)
        print(name, sorted(d))
