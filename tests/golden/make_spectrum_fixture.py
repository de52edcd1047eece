"""Extract the Smits-style RGB reference spectra (data, not code) from the reference.

The reference keeps seven 32-sample reflection spectra (WHITE, CYAN, MAGENTA,
YELLOW, RED, GREEN, BLUE) over 380-720 nm in
``src/colour/spectrum.rs:178-421`` (module ``rgb_reference_spectrum``).  This
script reads that file as text, pulls out the numbers and writes them to
``rgb_reference_spectrum.json`` next to this script.  The JSON is the fixture
that pins both the product's and the oracle's copies of the tables
(``tests/test_tables.py``).  Run only where ``/root/reference`` exists.
"""
import json
import os
import re
import sys

SRC = "/root/reference/src/colour/spectrum.rs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rgb_reference_spectrum.json")


def main():
    text = open(SRC).read()
    start = text.index("mod rgb_reference_spectrum")
    body = text[start:]
    out = {}
    for m in re.finditer(r"pub const SHORTEST_WAVELENGTH: f64 = ([0-9.]+);", body):
        out["shortest_wavelength"] = float(m.group(1))
    for m in re.finditer(r"pub const LONGEST_WAVELENGTH: f64 = ([0-9.]+);", body):
        out["longest_wavelength"] = float(m.group(1))
    tables = {}
    for m in re.finditer(r"pub const ([A-Z]+): \[f64; 32\] = \[(.*?)\];", body, re.S):
        vals = [v.strip() for v in m.group(2).split(",") if v.strip()]
        assert len(vals) == 32, (m.group(1), len(vals))
        # keep the decimal strings too, so the fixture is exactly what the reference holds
        tables[m.group(1)] = vals
    assert sorted(tables) == sorted(["WHITE", "CYAN", "MAGENTA", "YELLOW", "RED", "GREEN", "BLUE"])
    out["reflection"] = tables
    out["source"] = "src/colour/spectrum.rs:178-421"
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
