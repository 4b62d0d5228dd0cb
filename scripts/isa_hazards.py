"""Check the inline-asm vector loads of a kernel against the compiled code's control flow.

The QSGD fold issues its client loads with inline asm (fedavg_kernels.hip, qsgd_tile_kernel
`issue`), so the compiler does not track them: it inserts no wait before their registers are
read and could, in principle, allocate another value into a register whose load is still in
flight. The kernel's contract is that every path from such a load reaches an
``s_waitcnt vmcnt(0)`` before any instruction names one of the load's destination registers.
``hazards(isa_text, marker)`` walks every path of the disassembly (branch targets included) from
each load whose text contains ``marker`` and returns the instructions that break the contract
(tests/test_kernel_isa.py runs it on every built QSGD tile kernel).
"""

from __future__ import annotations

import re

_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<[^>+]*\+0x([0-9a-f]+)>")
_HEAD = re.compile(r"^([0-9a-f]+)\s+<([^>]+)>:$")
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _regs(operands: str) -> set[int]:
    out: set[int] = set()
    for m in _VREG.finditer(operands):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(isa_text: str) -> tuple[list[tuple[int, str, str]], dict[int, int], int]:
    """(instructions as (address, mnemonic, operands), address -> index, symbol base address)."""
    insts: list[tuple[int, str, str]] = []
    base = None
    for line in isa_text.splitlines():
        h = _HEAD.match(line.strip())
        if h:
            if base is not None:
                break  # first kernel only
            base = int(h.group(1), 16)
            continue
        m = _ADDR.search(line)
        if m is None or base is None:
            continue
        body = line[: m.start()].strip()
        if not body:
            continue
        mnem, _, ops = body.partition(" ")
        t = _TARGET.search(line[m.start():])
        if t is not None:  # a branch: its target (symbol offset) follows the encoding
            ops = f"{ops.strip()} <+0x{t.group(1)}>"
        insts.append((int(m.group(1), 16), mnem, ops.strip()))
    assert base is not None, "no kernel symbol in the disassembly"
    return insts, {a: i for i, (a, _, _) in enumerate(insts)}, base


def _successors(i: int, insts, index, base) -> list[int]:
    addr, mnem, ops = insts[i]
    if mnem == "s_endpgm":
        return []
    nxt = [i + 1] if i + 1 < len(insts) else []
    if mnem.startswith("s_branch") or mnem.startswith("s_cbranch"):
        t = _TARGET.search(ops)
        assert t is not None, f"branch without target: {mnem} {ops}"
        tgt = index[base + int(t.group(1), 16)]
        return [tgt] if mnem.startswith("s_branch") else nxt + [tgt]
    if mnem.startswith("s_setpc"):
        return []
    return nxt


def _drains(mnem: str, ops: str) -> bool:
    return mnem == "s_waitcnt" and re.search(r"\bvmcnt\(0\)", ops) is not None


def hazards(isa_text: str, marker: str = " nt") -> list[str]:
    """Instructions that name a destination register of a pending marked load."""
    insts, index, base = parse(isa_text)
    loads = _marked(insts, marker)
    found: list[str] = []
    for li in loads:
        dst = _regs(insts[li][2].split(",")[0])
        seen: set[int] = set()
        stack = _successors(li, insts, index, base)
        while stack:
            i = stack.pop()
            if i in seen:
                continue
            seen.add(i)
            addr, mn, ops = insts[i]
            if _drains(mn, ops):
                continue
            if _regs(ops) & dst:
                found.append(f"{insts[li][0]:x} {insts[li][1]} {insts[li][2]} -> {addr:x} {mn} {ops}")
            stack.extend(_successors(i, insts, index, base))
    return found


def _marked(insts, marker: str) -> list[int]:
    """The asm loads: every load carrying ``marker`` (the slot loads are the kernel's only `nt`
    loads) plus the sign-word load (global_load_ushort) the asm issues right after each."""
    out: list[int] = []
    for i, (_, mn, ops) in enumerate(insts):
        if mn.startswith("global_load") and marker in " " + ops:
            out.append(i)
            for j in range(i + 1, min(i + 6, len(insts))):
                if insts[j][1] == "global_load_ushort":
                    out.append(j)
                    break
    return out


def marked_loads(isa_text: str, marker: str = " nt") -> int:
    insts, _, _ = parse(isa_text)
    return len(_marked(insts, marker))
