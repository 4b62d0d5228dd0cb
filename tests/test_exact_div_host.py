"""The epilogue division identity (csrc/exact_div.h) checked on the host: scripts/check_exact_div.c
compiled with gcc (hardware fma) over 2 x 2e6 quotients — random binary64 over the fast path's
whole range, binary64 near the quotient grid's midpoints — must equal IEEE division bit for bit.
(The GPU suite checks the kernels themselves against the oracle.)"""

from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

SRC = Path(__file__).resolve().parent.parent / "scripts" / "check_exact_div.c"


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_reciprocal_correction_equals_ieee_division(tmp_path):
    exe = tmp_path / "check_exact_div"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", str(SRC), "-lm", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, check=False)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 differ" in out.stdout
