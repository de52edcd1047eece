"""The ordered reduce's table-driven exp (vanrijn_amd/csrc/vr_exp_table.h) against libm exp.

accumulate_kernel evaluates the CIE lobes of ColourXyz::x/y/z (colour_xyz.rs:86-103) with
vr_exp_tab instead of the general exp; the header is plain C99, so gcc builds it unchanged here and
tests/exp_table_check.c measures the largest ulp distance from libm's exp over 10^7 arguments in
[-745, 0], 10^6 small ones and every lobe exponent at 0 nm and 380..740 nm in 1e-4 nm steps.
"""
import os
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
MAX_ULP = 2


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_exp_table_within_two_ulp():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "exp_check")
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-ffp-contract=off", os.path.join(HERE, "exp_table_check.c"),
                               "-o", exe, "-lm"])
        worst, points = subprocess.check_output([exe], timeout=120).split()
    assert int(points) > 36_000_000
    assert float(worst) <= MAX_ULP
