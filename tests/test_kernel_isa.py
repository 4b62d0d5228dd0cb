"""Build-time checks on the compiled gfx950 code object (no GPU needed).

* The QSGD fold's inline-asm client loads (fedavg_kernels.hip, qsgd_tile_kernel `issue`) are
  invisible to the compiler's wait insertion; every path from one of them must reach
  ``s_waitcnt vmcnt(0)`` before any instruction names its destination registers
  (scripts/isa_hazards.py walks the disassembly's control flow). Validated compiler: the
  ``.comment`` of the code object is recorded in the failure message; the kernels were written
  against ROCm 7.2 (AMD clang 22.0.0git roc-7.2.0).
* No kernel uses scratch memory or spills VGPRs (SGPR spills go to VGPR lanes and are listed in
  profiles/r04_kernel_resources.json).
"""

from __future__ import annotations

import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "scripts"))

import isa_hazards  # noqa: E402
import kernel_resources  # noqa: E402

pytestmark = pytest.mark.skipif(
    not kernel_resources.LIB.exists() or not (kernel_resources.LLVM / "llvm-objdump").exists(),
    reason="library not built or LLVM tools missing")


def _compiler() -> str:
    co = kernel_resources.code_objects()[0]
    m = re.search(rb"AMD clang version [^\0]*", co)
    return m.group(0).decode(errors="replace") if m else "unknown"


@pytest.fixture(scope="module")
def qsgd_isa() -> dict[str, str]:
    names = [k["name"] for k in kernel_resources.kernel_metadata() if "qsgd_tile_kernel" in k["name"]]
    assert len(names) == 12, names  # 3 output kinds x {float, double} inputs x {FULL, ragged}
    text = kernel_resources.disassemble("qsgd_tile_kernel")
    out, cur, buf = {}, None, []
    for line in text.splitlines():
        if line.endswith(">:"):
            if cur is not None:
                out[cur] = "\n".join(buf)
            cur, buf = line, []
        buf.append(line)
    if cur is not None:
        out[cur] = "\n".join(buf)
    assert len(out) == 12
    return out


def test_qsgd_asm_loads_are_drained_before_use(qsgd_isa):
    for name, isa in qsgd_isa.items():
        n = isa_hazards.marked_loads(isa)
        # issue() is inlined at the prologue and once per buffer of the loop: G slot + G sign
        # loads each (kQsgdGroup = 2, kQsgdBufs = 2)
        assert n >= 4 and n % 4 == 0, (name, n)
        bad = isa_hazards.hazards(isa)
        assert not bad, f"{name}: register of a pending asm load used before vmcnt(0) " \
                        f"(compiler {_compiler()}):\n" + "\n".join(bad[:10])


def test_hazard_checker_catches_a_missing_wait(qsgd_isa):
    """Negative control: with the vmcnt(0) waits deleted the fold reads pending registers."""
    isa = next(iter(qsgd_isa.values()))
    stripped = re.sub(r"s_waitcnt\s+vmcnt\(0\)", "s_nop 0", isa)
    assert isa_hazards.hazards(stripped)


def test_no_kernel_uses_scratch_or_spills_vgprs():
    ks = kernel_resources.kernel_metadata()
    assert len(ks) > 100
    bad = [(k["name"], k.get("private_segment_fixed_size"), k.get("vgpr_spill_count")) for k in ks
           if k.get("private_segment_fixed_size", 0) or k.get("vgpr_spill_count", 0)]
    assert not bad, bad


def test_llvm_objdump_is_available():
    assert shutil.which(str(kernel_resources.LLVM / "llvm-objdump"))
    subprocess.run([str(kernel_resources.LLVM / "llvm-objdump"), "--version"], check=True, capture_output=True)
