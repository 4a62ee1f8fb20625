"""Tiny eBPF assembler (host-side tool).

The reference has no assembler of its own; its programs arrive as hex from bpf_conformance
(main.rs:33-38). This module turns the bpf_conformance / ubpf text syntax into the little-endian
program image that `ins.hexs_to_instructions` / `ebpf_prog_load` decode, so that test programs
and the synthetic XDP workloads can be written readably.

Label arithmetic follows the REFERENCE's jump semantics, not the kernel's: a jump offset counts
decoded instructions, and a wide `lddw` is ONE decoded instruction (ins.rs:107-116,
emu.rs:227; quirk Q9). Pass `slots="words"` to count lddw as two slots like a standard eBPF
toolchain does.

Syntax: `%r3` or `r3`; memory operands `[r1+2]` / `[r10-8]`; numbers in C syntax; comments
after `#`, `;` or `//`.
`call +N` encodes the reference's offset-based call (emu.rs:265-272: pc += off).
`lock [fetch] {add,or,and,xor,xchg,cmpxchg}[32] [rD+off], rS` encodes atomics
(xchg/cmpxchg always carry the fetch bit, as the kernel's encodings do).
"""
from __future__ import annotations

import re
import struct

ALU_OPS = {"add": 0x0, "sub": 0x1, "mul": 0x2, "div": 0x3, "or": 0x4, "and": 0x5, "lsh": 0x6,
           "rsh": 0x7, "neg": 0x8, "mod": 0x9, "xor": 0xA, "mov": 0xB, "arsh": 0xC}
JMP_OPS = {"ja": 0x0, "jeq": 0x1, "jgt": 0x2, "jge": 0x3, "jset": 0x4, "jne": 0x5, "jsgt": 0x6,
           "jsge": 0x7, "jlt": 0xA, "jle": 0xB, "jslt": 0xC, "jsle": 0xD}
SIZES = {"w": 0x00, "h": 0x08, "b": 0x10, "dw": 0x18}
ATOMIC_OPS = {"add": 0x00, "or": 0x40, "and": 0x50, "xor": 0xA0, "xchg": 0xE1, "cmpxchg": 0xF1}

CLASS_LD, CLASS_LDX, CLASS_ST, CLASS_STX = 0, 1, 2, 3
CLASS_ALU, CLASS_JMP, CLASS_JMP32, CLASS_ALU64 = 4, 5, 6, 7


class AsmError(ValueError):
    pass


def _s16(v: int) -> int:
    v &= 0xFFFF
    return v - 0x10000 if v & 0x8000 else v


def _s32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def encode(code: int, dst: int = 0, src: int = 0, off: int = 0, imm: int = 0) -> bytes:
    """One 8-byte instruction word, little-endian (the byte order the reference's hex uses)."""
    return struct.pack("<BBhi", code & 0xFF, (dst & 0xF) | ((src & 0xF) << 4),
                       _s16(off), _s32(imm))


def lddw(dst: int, value: int) -> bytes:
    value &= (1 << 64) - 1
    return encode(0x18, dst, 0, 0, value & 0xFFFFFFFF) + encode(0, 0, 0, 0, value >> 32)


_REG = re.compile(r"^%?r(\d+)$")
_MEM = re.compile(r"^\[\s*%?r(\d+)\s*(?:([+-])\s*(\w+))?\s*\]$")
_LABEL = re.compile(r"^([A-Za-z_.][\w.]*)\s*:(.*)$")


def _reg(tok: str) -> int:
    m = _REG.match(tok.strip())
    if not m:
        raise AsmError(f"expected register, got {tok!r}")
    return int(m.group(1))


def _num(tok: str) -> int:
    return int(tok.strip(), 0)


def _mem(tok: str):
    m = _MEM.match(tok.strip())
    if not m:
        raise AsmError(f"expected memory operand, got {tok!r}")
    off = 0
    if m.group(2):
        off = _num(m.group(3))
        if m.group(2) == "-":
            off = -off
    return int(m.group(1)), off


def _parse(text: str):
    """-> list of ("label", name) | (mnemonic, [operands])."""
    items = []
    for raw in text.splitlines():
        raw = re.split(r"#|;|//", raw)[0].strip()
        while True:
            m = _LABEL.match(raw)
            if not m:
                break
            items.append(("label", m.group(1)))
            raw = m.group(2).strip()
        if not raw:
            continue
        parts = raw.split(None, 1)
        mnem = parts[0].lower()
        rest = parts[1] if len(parts) > 1 else ""
        if mnem == "lock":  # lock [fetch] op[32] [mem], reg
            words = rest.split(None, 2 if rest.lower().startswith("fetch") else 1)
            fetch = words[0].lower() == "fetch"
            if fetch:
                words = words[1:]
            op = words[0].lower()
            ops = [o.strip() for o in re.split(r",(?![^\[]*\])", words[1])]
            items.append(("lock", [fetch, op] + ops))
            continue
        ops = [o.strip() for o in re.split(r",(?![^\[]*\])", rest)] if rest else []
        items.append((mnem, ops))
    return items


def assemble(text: str, slots: str = "decoded") -> bytes:
    """Assemble a program; returns the little-endian byte image."""
    items = _parse(text)
    labels, idx = {}, 0
    for mnem, ops in items:
        if mnem == "label":
            labels[ops] = idx
        else:
            idx += 2 if (mnem == "lddw" and slots == "words") else 1
    out, idx = bytearray(), 0
    for mnem, ops in items:
        if mnem == "label":
            continue
        out += _one(mnem, ops, idx, labels)
        idx += 2 if (mnem == "lddw" and slots == "words") else 1
    return bytes(out)


asm = assemble


def _target(tok: str, idx: int, labels) -> int:
    tok = tok.strip()
    if tok in labels:
        return labels[tok] - (idx + 1)
    return _num(tok)


def _one(mnem: str, ops, idx: int, labels) -> bytes:
    if mnem == "exit":
        return encode(0x95)
    if mnem == "call":
        return encode(0x85, 0, 0, _target(ops[0], idx, labels), 0)
    if mnem == "lddw":
        return lddw(_reg(ops[0]), _num(ops[1]))
    if mnem == "lock":
        fetch, op, mem, src = ops
        is32 = op.endswith("32")
        op = op[:-2] if is32 else op
        if op not in ATOMIC_OPS:
            raise AsmError(f"unknown atomic op {op!r}")
        d, off = _mem(mem)
        imm = ATOMIC_OPS[op] | (1 if fetch else 0)
        return encode(0xC0 | (0x00 if is32 else 0x18) | CLASS_STX, d, _reg(src), off, imm)
    if mnem in ("le16", "le32", "le64", "be16", "be32", "be64"):
        src_bit = 0x08 if mnem.startswith("be") else 0x00
        return encode(0xD4 | src_bit, _reg(ops[0]), 0, 0, int(mnem[2:]))
    m = re.match(r"^(ldx|stx|st)(dw|w|h|b)$", mnem)
    if m:
        kind, size = m.group(1), SIZES[m.group(2)]
        if kind == "ldx":
            s, off = _mem(ops[1])
            return encode(0x60 | size | CLASS_LDX, _reg(ops[0]), s, off, 0)
        d, off = _mem(ops[0])
        if kind == "stx":
            return encode(0x60 | size | CLASS_STX, d, _reg(ops[1]), off, 0)
        return encode(0x60 | size | CLASS_ST, d, 0, off, _num(ops[1]))
    is32 = mnem.endswith("32")
    base = mnem[:-2] if is32 else mnem
    if base in ALU_OPS:
        cls = CLASS_ALU if is32 else CLASS_ALU64
        op = ALU_OPS[base]
        dst = _reg(ops[0])
        if base == "neg":
            return encode((op << 4) | cls, dst)
        if _REG.match(ops[1]):
            return encode((op << 4) | 0x08 | cls, dst, _reg(ops[1]))
        return encode((op << 4) | cls, dst, 0, 0, _num(ops[1]))
    if base in JMP_OPS:
        cls = CLASS_JMP32 if is32 else CLASS_JMP
        op = JMP_OPS[base]
        if base == "ja":
            return encode((op << 4) | cls, 0, 0, _target(ops[0], idx, labels))
        dst = _reg(ops[0])
        off = _target(ops[2], idx, labels)
        if _REG.match(ops[1]):
            return encode((op << 4) | 0x08 | cls, dst, _reg(ops[1]), off)
        return encode((op << 4) | cls, dst, 0, off, _num(ops[1]))
    raise AsmError(f"unknown mnemonic {mnem!r}")


def to_hex(img: bytes) -> str:
    """Space-separated hex, the format the reference's plugin reads (main.rs:33-38)."""
    return " ".join(f"{b:02x}" for b in img)
