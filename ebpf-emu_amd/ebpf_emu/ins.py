"""ebpf_emu.ins — the reference's `ins` module surface (src/ins.rs), over libebpfemu.so.

Names, argument meaning and error behaviour follow ins.rs:
  hexs_to_u8s / hexs_to_u64s / hexs_to_u64s_le   ins.rs:46-89 (Err strings -> HexError)
  hexs_to_instructions / u64s_to_instructions     ins.rs:91-119 (decode panics -> DecodeError)
  Instruction, Code.AJ / Code.LS, Register, Mode, Source, OP, AOp, JOp, Class  ins.rs:13-279
Decoding itself happens in the library's loader (ebpf_prog_load), the same code that feeds the
GPU micro-op table, so what these functions return is exactly what the kernel executes.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass

from . import _lib


class HexError(ValueError):
    """Err(String) of the hex parsers (ins.rs:52,67,82)."""


class DecodeError(ValueError):
    """A decode-time panic of the reference (ins.rs:32,112,187,251,257)."""

    def __init__(self, code: int, word: int):
        super().__init__(f"{_lib.strerror(code)} (code {code}) at word {word}")
        self.code = code
        self.word = word


class Register(enum.IntEnum):  # ins.rs:13-28
    R0 = 0
    R1 = 1
    R2 = 2
    R3 = 3
    R4 = 4
    R5 = 5
    R6 = 6
    R7 = 7
    R8 = 8
    R9 = 9
    R10 = 10
    FP = 11


class Mode(enum.IntEnum):  # ins.rs:175-183
    IMM = 0x00
    ABS = 0x20
    IND = 0x40
    MEM = 0x60
    ATOMIC = 0xC0


class Source(enum.IntEnum):  # ins.rs:191-196
    IMM = 0
    SRC = 1


class AOp(enum.IntEnum):  # ins.rs:211-228
    ADD = 0
    SUB = 1
    MUL = 2
    DIV = 3
    OR = 4
    AND = 5
    LSH = 6
    RSH = 7
    NEG = 8
    MOD = 9
    XOR = 10
    MOV = 11
    ARSH = 12
    END = 13


class JOp(enum.IntEnum):  # ins.rs:230-247
    JA = 0
    JEQ = 1
    JGT = 2
    JGE = 3
    JSET = 4
    JNE = 5
    JSGT = 6
    JSGE = 7
    CALL = 8
    EXIT = 9
    JLT = 10
    JLE = 11
    JSLT = 12
    JSLE = 13


class Class(enum.IntEnum):  # ins.rs:261-272
    LD = 0
    LDX = 1
    ST = 2
    STX = 3
    ALU = 4
    JMP = 5
    JMP32 = 6
    ALU64 = 7


@dataclass(frozen=True)
class OP:  # ins.rs:204-209: OP::Alu(AOp) | OP::Jmp(JOp)
    kind: str
    op: int

    @staticmethod
    def Alu(op: AOp) -> "OP":
        return OP("Alu", AOp(op))

    @staticmethod
    def Jmp(op: JOp) -> "OP":
        return OP("Jmp", JOp(op))


@dataclass(frozen=True)
class AJ:  # Code::AJ {op, source, class}
    op: OP
    source: Source
    cls: Class


@dataclass(frozen=True)
class LS:  # Code::LS {mode, size, class}
    mode: Mode
    size: int
    cls: Class


class Code:  # ins.rs:134-173
    AJ = AJ
    LS = LS

    @staticmethod
    def from_u8(code: int):
        cls = Class(code & 0b111)
        if cls in (Class.ALU, Class.ALU64):
            return AJ(OP.Alu(AOp(code >> 4)), Source((code >> 3) & 1), cls)
        if cls in (Class.JMP, Class.JMP32):
            return AJ(OP.Jmp(JOp(code >> 4)), Source((code >> 3) & 1), cls)
        return LS(Mode(code & 0b1110_0000), code & 0b0001_1000, cls)


@dataclass(frozen=True)
class Instruction:  # ins.rs:37-45
    imm: int
    imm64: int
    off: int
    src: Register
    dst: Register
    code: object  # AJ | LS

    @property
    def opcode(self) -> int:
        c = self.code
        if isinstance(c, AJ):
            return (c.op.op << 4) | (c.source << 3) | c.cls
        return c.mode | c.size | c.cls


def _clean(hx: str) -> str:
    return hx.strip().replace(" ", "")


def _radix(chunk: str) -> int:
    # u8/u64::from_str_radix(…, 16): optional leading '+', then hex digits only
    body = chunk[1:] if chunk.startswith("+") else chunk
    if not body or any(c not in "0123456789abcdefABCDEF" for c in body):
        raise HexError("invalid digit found in string")
    return int(body, 16)


def hexs_to_u8s(hx: str) -> list[int]:
    """ins.rs:46-59."""
    hx = _clean(hx)
    out = []
    for i in range(0, len(hx), 2):
        chunk = hx[i:i + 2]
        if len(chunk) < 2:
            raise HexError("invalid hex format")
        out.append(_radix(chunk))
    return out


def hexs_to_u64s(hx: str) -> list[int]:
    """ins.rs:60-74: 16-digit big-endian chunks."""
    hx = _clean(hx)
    out = []
    for i in range(0, len(hx), 16):
        chunk = hx[i:i + 16]
        if len(chunk) < 16:
            raise HexError("invalid hex format for u64")
        out.append(_radix(chunk))
    return out


def hexs_to_u64s_le(hx: str) -> list[int]:
    """ins.rs:76-89: as hexs_to_u64s, then u64::from_be."""
    return [int.from_bytes(v.to_bytes(8, "big"), "little") for v in hexs_to_u64s(hx)]


def _image_from_u64s(u64s) -> bytes:
    # u64s_to_instructions applies from_be to BE-parsed words (ins.rs:97): the word's
    # big-endian bytes are the program's little-endian byte image.
    return b"".join((int(v) & ((1 << 64) - 1)).to_bytes(8, "big") for v in u64s)


def load_image(image: bytes):
    """ebpf_prog_load on a little-endian byte image -> raw ebpf_prog* (caller frees)."""
    L = _lib.lib()
    handle = ctypes.c_void_p()
    bad = ctypes.c_size_t(0)
    rc = L.ebpf_prog_load(bytes(image), len(image), ctypes.byref(handle), ctypes.byref(bad))
    if rc != 0:
        raise DecodeError(rc, bad.value)
    return handle


def _decoded(handle) -> list[Instruction]:
    L = _lib.lib()
    n = L.ebpf_prog_len(handle)
    imm, imm64, off = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int16()
    src, dst, code = ctypes.c_uint8(), ctypes.c_uint8(), ctypes.c_uint8()
    out = []
    for i in range(n):
        L.ebpf_prog_insn(handle, i, ctypes.byref(imm), ctypes.byref(imm64), ctypes.byref(off),
                         ctypes.byref(src), ctypes.byref(dst), ctypes.byref(code))
        out.append(Instruction(imm.value, imm64.value, off.value, Register(src.value),
                               Register(dst.value), Code.from_u8(code.value)))
    return out


def decode_image(image: bytes) -> list[Instruction]:
    handle = load_image(image)
    try:
        return _decoded(handle)
    finally:
        _lib.lib().ebpf_prog_free(handle)


def u64s_to_instructions(u64s) -> list[Instruction]:
    """ins.rs:96-119 (input: words as parsed big-endian from hex)."""
    return decode_image(_image_from_u64s(u64s))


def hexs_to_instructions(hx: str) -> list[Instruction]:
    """ins.rs:91-94."""
    return u64s_to_instructions(hexs_to_u64s(hx))
