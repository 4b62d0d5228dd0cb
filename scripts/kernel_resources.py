"""Per-kernel resources of the built gfx950 code object, read from the library itself.

The .so embeds a clang offload bundle (section .hip_fatbin); the gfx950 entry is an AMDGPU ELF
whose NT_AMDGPU_METADATA note lists every kernel's VGPR / SGPR counts, spills, scratch (private
segment) and LDS (group segment) sizes. `python scripts/kernel_resources.py [--match NAME]
[--json OUT]` prints them (profiles/r04_kernel_resources.json is this output); `--isa NAME` writes
the kernel's disassembly (llvm-objdump) to stdout. tests/test_kernel_isa.py uses the same helpers.
"""

from __future__ import annotations

import argparse
import json
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
LIB = REPO / "distributed_learning_simulation_lib_amd" / "_lib" / "libfedavg_hip.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path: Path, name: str) -> bytes:
    """Raw bytes of an ELF64 section by name (no external tools)."""
    data = path.read_bytes()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    heads = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    strtab = heads[shstrndx]
    names = data[strtab[4]: strtab[4] + strtab[5]]
    for h in heads:
        n = names[h[0]: names.index(b"\0", h[0])].decode()
        if n == name:
            return data[h[4]: h[4] + h[5]]
    raise KeyError(name)


def code_objects(lib: Path = LIB, arch: str = "gfx950") -> list[bytes]:
    """The gfx950 code objects of the library's offload bundles (one per HIP translation unit)."""
    blob = _section(lib, ".hip_fatbin")
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", blob, pos + len(MAGIC))
        off = pos + len(MAGIC) + 8
        ends = []
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24: off + 24 + tlen].decode()
            off += 24 + tlen
            ends.append(pos + eoff + esize)
            if arch in triple:
                out.append(blob[pos + eoff: pos + eoff + esize])
        pos = blob.find(MAGIC, max(ends) if ends else pos + 1)
    if not out:
        raise KeyError(f"no {arch} code object in {lib}")
    return out


def _with_object(fn):
    """fn(path) over each code object, outputs concatenated."""
    texts = []
    for co in code_objects():
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            texts.append(fn(f.name))
    return "\n".join(texts)


def kernel_metadata() -> list[dict]:
    """Kernel records of the code object's metadata note (llvm-readelf --notes)."""
    text = _with_object(lambda p: subprocess.run([str(LLVM / "llvm-readelf"), "--notes", p], capture_output=True,
                                                 text=True, check=True).stdout)
    kernels, cur = [], None
    for line in text.splitlines():
        s = line.strip()
        m = re.match(r"^-?\s*\.(\w+):\s*(.*)$", s)
        if m is None:
            continue
        key, val = m.group(1), m.group(2).strip()
        if key == "agpr_count" and s.startswith("- "):
            cur = {}
            kernels.append(cur)
        if cur is None:
            continue
        if key in ("name", "symbol"):
            cur[key] = val.strip("'")
        elif key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "agpr_count",
                     "private_segment_fixed_size", "group_segment_fixed_size", "wavefront_size",
                     "max_flat_workgroup_size"):
            try:
                cur[key] = int(val)
            except ValueError:
                pass
    return [k for k in kernels if "name" in k]


def disassemble(symbol_substr: str) -> str:
    """llvm-objdump -d of the kernels whose symbol contains ``symbol_substr``."""
    text = _with_object(lambda p: subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", p],
                                                 capture_output=True, text=True, check=True).stdout)
    out, keep = [], False
    for line in text.splitlines():
        if line.endswith(">:"):
            keep = symbol_substr in line
        if keep:
            out.append(line)
    return "\n".join(out)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default=None)
    ap.add_argument("--isa", default=None)
    ap.add_argument("--lib", default=None, help="another build of the library (a tuning variant)")
    args = ap.parse_args()
    if args.lib:
        global LIB
        LIB = Path(args.lib).resolve()
        code_objects.__defaults__ = (LIB, "gfx950")
    if args.isa:
        print(disassemble(args.isa))
        return 0
    ks = [k for k in kernel_metadata() if args.match in k["name"]]
    for k in ks:
        print(f"{k['name'][:110]:110s} vgpr {k.get('vgpr_count')} sgpr {k.get('sgpr_count')} "
              f"spill v/s {k.get('vgpr_spill_count')}/{k.get('sgpr_spill_count')} "
              f"scratch {k.get('private_segment_fixed_size')} lds {k.get('group_segment_fixed_size')}")
    if args.json:
        Path(args.json).write_text(json.dumps({"library": str(LIB.relative_to(REPO)), "arch": "gfx950",
                                               "source": "NT_AMDGPU_METADATA of the built code object "
                                                         "(scripts/kernel_resources.py)",
                                               "kernels": ks}, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
