"""the bit-level tricks (FAST's f16-subnormal ordering, rBRIEF's
magic-number cvRound) must fail the BUILD when a flag that breaks them is added, not
the parity tests.  The Makefile refuses each flag (checked here with `make -n`); the
device-side k_arith_guard (extract.hip) re-checks the arithmetic at the first call."""
import os
import subprocess

import pytest

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orb-ygz-slam_amd")


@pytest.mark.parametrize("var", ["HIPFLAGS", "EXTRA", "XDEFS"])
@pytest.mark.parametrize("flag", ["-ffast-math", "-fgpu-flush-denormals-to-zero", "-ffp-contract=fast",
                                  "-funsafe-math-optimizations", "-ffinite-math-only"])
def test_make_refuses_breaking_flags(var, flag):
    r = subprocess.run(["make", "-n", "-C", PKG, f"{var}={flag}"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "breaks ygzfe's bit-exact paths" in r.stderr


def test_make_accepts_default_flags():
    r = subprocess.run(["make", "-n", "-C", PKG], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
