"""BestFit's and DotProduct's divisions by MaxSpecCpu / MaxSpecGpu (best_fit_score.go:66-97,
dot_product_score.go:64-107) are computed without a division (ksim_device.hpp div125 / div_spec_*): the
corrected product equals IEEE x / 125 for every integer below 2^31, which this test checks exhaustively
(the quotients the engine forms are of integers in that range; scaling by 2^-10 / 2^-6 is exact)."""
import os
import subprocess
import tempfile

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def test_div125_equals_division_for_every_int31():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "div125_check")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "div125_check.c"), "-lm"],
                       check=True)
        plain, corrected = (int(x) for x in subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split())
    assert corrected == 0
    assert plain > 0  # the plain product alone is not the division: the correction is needed
