"""pyref.py — TEST INFRASTRUCTURE ONLY.

An independently written, pure-Python restatement of b1tg/ebpf-emu (snapshot 2024-12-20),
structured like the Rust crate (Instruction / Code / Emu / Mmu), so that it can be
cross-checked against the C oracle (oracle/ebpf_oracle.c) by differential fuzzing. Two
restatements written separately are the substitute for running the Rust reference, which
cannot be built here (no Rust toolchain). Slow: small cases only.

Status numbering is shared with oracle/ebpf_oracle.h and include/ebpf_emu.h.
"""
from __future__ import annotations

from dataclasses import dataclass

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1

ST_OK, ST_MEM, ST_MEM_UB, ST_INSN, ST_ARITH, ST_STEPS, ST_CALLDEPTH, ST_BADPKT = range(8)
E_LEN, E_REG, E_OP, E_MODE, E_LDDW, E_LDDW_OVF = -2, -3, -4, -5, -6, -7
MAX_CALL_DEPTH = 64

LS_CLASSES = (0, 1, 2, 3)  # ins.rs:163 CLASS_LD, CLASS_LDX, CLASS_ST, CLASS_STX


def s64(v: int) -> int:
    v &= M64
    return v - (1 << 64) if v >> 63 else v


def s32(v: int) -> int:
    v &= M32
    return v - (1 << 32) if v >> 31 else v


class Panic(Exception):
    """A Rust panic of the reference; carries the status the build reports for it."""

    def __init__(self, status: int):
        super().__init__(status)
        self.status = status


class DecodeError(Exception):
    def __init__(self, code: int, word: int):
        super().__init__(code, word)
        self.code = code
        self.word = word


@dataclass
class Instruction:  # ins.rs:37-45
    imm: int
    imm64: int
    off: int
    src: int
    dst: int
    code: int  # raw opcode byte; Code is derived below

    @property
    def cls(self) -> int:
        return self.code & 0b111

    @property
    def is_ls(self) -> bool:
        return self.cls in LS_CLASSES


def _from_u64(w: int, idx: int) -> Instruction:  # ins.rs:121-132 (field order preserved)
    imm = s32(w >> 32)
    imm64 = (w >> 32) & M32
    off = (w >> 16) & 0xFFFF
    off = off - 0x10000 if off & 0x8000 else off
    src = (w >> 12) & 0xF
    if src >= 12:
        raise DecodeError(E_REG, idx)
    dst = (w >> 8) & 0xF
    if dst >= 12:
        raise DecodeError(E_REG, idx)
    code = w & 0xFF
    cls = code & 7
    if cls in (4, 7, 5, 6):  # Code::AJ, ins.rs:151-162
        if (code >> 4) > 0xD:
            raise DecodeError(E_OP, idx)
    else:  # Code::LS, ins.rs:163-168
        mode = code & 0xE0
        if mode > 0xC0 or mode in (0x80, 0xA0):
            raise DecodeError(E_MODE, idx)
    return Instruction(imm, imm64, off, src, dst, code)


def decode(prog: bytes) -> list[Instruction]:
    """u64s_to_instructions(hexs_to_u64s(hex(prog))) — ins.rs:60-74,96-119."""
    if len(prog) % 8:
        raise DecodeError(E_LEN, len(prog) // 8)
    words = [int.from_bytes(prog[i:i + 8], "little") for i in range(0, len(prog), 8)]
    out, i = [], 0
    while i < len(words):
        ins = _from_u64(words[i], i)
        if ins.is_ls and (ins.code & 0xE0) == 0:
            if i + 1 >= len(words):
                raise DecodeError(E_LDDW, i)
            i += 1
            v = (ins.imm & M32) + s64(words[i])
            if not (I64_MIN <= v <= I64_MAX):
                raise DecodeError(E_LDDW_OVF, i - 1)
            ins.imm64 = v
            ins.imm = 0
        out.append(ins)
        i += 1
    return out


class Mmu:  # mmu.rs
    def __init__(self, memory: bytearray):
        self.memory = memory

    def _first_byte(self, addr: int, width: int) -> int:
        # read_ptr_mut::<u8> bounds-checks one byte (mmu.rs:23-30); the caller copies `width`.
        if addr < 0 or addr >= len(self.memory):
            raise Panic(ST_MEM)
        if addr + width > len(self.memory):
            raise Panic(ST_MEM_UB)
        return addr

    def load(self, addr: int, width: int) -> int:
        a = self._first_byte(addr, width)
        return int.from_bytes(self.memory[a:a + width], "little")

    def store(self, addr: int, width: int, value: int) -> None:
        a = self._first_byte(addr, width)
        self.memory[a:a + width] = (value & ((1 << (8 * width)) - 1)).to_bytes(width, "little")

    def read_i64(self, addr: int) -> int:  # mmu.rs:13-22
        if addr < 0 or addr + 8 > len(self.memory):
            raise Panic(ST_MEM)
        return s64(int.from_bytes(self.memory[addr:addr + 8], "little"))

    def write(self, addr: int, val: bytes) -> None:  # mmu.rs:7-12 (growth never reached)
        self.memory[addr:addr + len(val)] = val


def _checked_add(a: int, b: int, status: int) -> int:
    v = a + b
    if not (I64_MIN <= v <= I64_MAX):
        raise Panic(status)
    return v


def _rotr(x: int, k: int, bits: int) -> int:
    mask = (1 << bits) - 1
    x &= mask
    k %= bits
    return ((x >> k) | (x << (bits - k))) & mask


class Emu:  # emu.rs:19-45
    def __init__(self, instructions, memory: bytearray, regs=None):
        self.regs = list(regs) if regs is not None else [0] * 11
        self.mmu = Mmu(memory)
        self.instructions = instructions
        self.pc = 0
        self.fp: list[int] = []
        self.ins_count = 0

    def _reg(self, r: int) -> int:
        if r >= 11:
            raise Panic(ST_INSN)  # regs: [i64; 11] indexed with 11
        return self.regs[r]

    def step(self) -> bool:
        if self.pc >= len(self.instructions):  # emu.rs:49
            return False
        ins = self.instructions[self.pc]
        self.pc = (self.pc + 1) & M32
        if not ins.is_ls:
            self._aj(ins)
        else:
            self._ls(ins)
        self.ins_count += 1
        return True

    def _aj(self, ins: Instruction) -> None:  # emu.rs:65-309
        op, source, cls = ins.code >> 4, (ins.code >> 3) & 1, ins.cls
        src = ins.imm if source == 0 else self._reg(ins.src)
        if cls in (4, 7):
            dst = self._reg(ins.dst)
            is32 = cls == 4
            if is32 and op != 13:
                dst &= M32
                src &= M32
            if op == 0:
                dst = s64(dst + src)
            elif op == 1:
                dst = s64(dst - src)
            elif op == 2:
                dst = s64(dst * src)
            elif op == 3:
                dst = s64((dst & M64) // (src & M64)) if src != 0 else 0
            elif op == 4:
                dst = s64(dst | src)
            elif op == 5:
                dst = s64(dst & src)
            elif op == 6:
                dst = ((dst & M32) << ((src & M32) % 32)) & M32 if is32 else s64((dst & M64) << ((src & M32) % 64))
            elif op == 7:
                dst = (dst & M32) >> ((src & M32) % 32) if is32 else s64((dst & M64) >> ((src & M32) % 64))
            elif op == 8:
                dst = s64(-dst)
            elif op == 9:
                if src != 0:
                    dst = s64((dst & M64) % (src & M64))
            elif op == 10:
                dst = s64(dst ^ src)
            elif op == 11:
                dst = src
            elif op == 12:
                if is32:
                    sign = -1 if s32(dst) < 0 else 1
                    dst = s32(_rotr(dst, src & M32, 32)) * sign
                else:
                    sign = -1 if dst < 0 else 1
                    dst = s64(_rotr(dst, src & M32, 64)) * sign
                    if not (I64_MIN <= dst <= I64_MAX):
                        raise Panic(ST_ARITH)
            else:  # 13: END
                width = {16: 2, 32: 4, 64: 8}.get(ins.imm)
                if width is None:
                    raise Panic(ST_INSN)
                v = (dst & M64) & ((1 << (8 * width)) - 1)
                if source == 1:
                    v = int.from_bytes(v.to_bytes(width, "little"), "big")
                dst = s64(v)
            if is32 and op != 13:
                dst &= M32
            self.regs[ins.dst] = dst
            return
        # JMP / JMP32
        dst = self._reg(ins.dst)
        if cls == 6:
            dst, src = s32(dst), s32(src)
        off = ins.off
        take = False
        if op == 0:
            take = True
        elif op == 1:
            take = dst == src
        elif op in (2, 6):
            take = dst > src
        elif op in (3, 7):
            take = dst >= src
        elif op == 4:
            take = (dst & src) != 0
        elif op == 5:
            take = dst != src
        elif op in (10, 12):
            take = dst < src
        elif op in (11, 13):
            take = dst <= src
        elif op == 8:  # CALL
            if source != 0:
                raise Panic(ST_INSN)
            self.pc = (self.pc + off) & M32
            if self.pc == M32:
                raise Panic(ST_ARITH)
            if len(self.fp) >= MAX_CALL_DEPTH:
                raise Panic(ST_CALLDEPTH)
            self.fp.append(self.pc + 1)
        elif op == 9:  # EXIT
            if self.fp:
                self.pc = self.fp.pop()
            else:
                raise StopIteration
        if take:
            self.pc = (self.pc + off) & M32

    def _ls(self, ins: Instruction) -> None:  # emu.rs:311-444
        mode, size, cls = ins.code & 0xE0, ins.code & 0x18, ins.cls
        width = {0x00: 4, 0x08: 2, 0x10: 1, 0x18: 8}[size]
        imm = ins.imm64
        src = self._reg(ins.src)
        r0 = self.regs[0]
        dst = self._reg(ins.dst)
        if cls in (0, 1):
            if mode == 0x00:
                dst = imm
            elif mode == 0x60 and cls == 1:
                addr = _checked_add(src, ins.off, ST_MEM)
                v = self.mmu.load(addr, width)
                keep = M64 ^ ((1 << (8 * width)) - 1)
                dst = s64((dst & keep) | v)
            else:
                raise Panic(ST_INSN)
        else:
            source = imm if cls == 2 else src
            if mode == 0x60:
                addr = _checked_add(dst, ins.off, ST_MEM)
                self.mmu.store(addr, width, source)
            elif mode == 0xC0:
                addr = _checked_add(dst, ins.off, ST_MEM)
                orig = self.mmu.read_i64(addr)
                fetch = imm & 1 == 1
                bak = orig if fetch else 0
                high = 0
                if size == 0:
                    src &= M32
                    high = (orig & M64) >> 32
                    orig &= M32
                    r0 &= M32
                    bak &= M32
                aop = imm & 0xFE
                if aop == 0x00:
                    orig = _checked_add(orig, src, ST_ARITH)
                elif aop == 0x40:
                    orig |= src
                elif aop == 0x50:
                    orig &= src
                elif aop == 0xA0:
                    orig ^= src
                elif aop == 0xE0:
                    orig, bak = src, orig
                elif aop == 0xF0:
                    if orig == r0:
                        orig = src
                    self.regs[0] = bak
                else:
                    raise Panic(ST_INSN)
                orig = _checked_add(orig, s64(high << 32), ST_ARITH)
                self.mmu.write(addr, (orig & M64).to_bytes(8, "little"))
                if fetch:
                    self.regs[ins.src] = bak
            else:
                raise Panic(ST_INSN)
        self.regs[ins.dst] = dst

    def run(self, max_steps: int = 0) -> int:
        """Emu::run (emu.rs:452-458) with an optional step budget. Returns a status."""
        try:
            while True:
                if self.pc >= len(self.instructions):
                    return ST_OK
                if max_steps and self.ins_count >= max_steps:
                    return ST_STEPS
                self.step()
        except StopIteration:
            self.ins_count += 1  # the final exit counts as retired
            return ST_OK
        except Panic as p:
            return p.status


def run_packet(prog: bytes | list, pkt: bytes, mem_size: int = 1024, r10: int = 512,
               max_steps: int = 0):
    """main.rs:14-43 layout. Returns (status, r0 as u64, steps)."""
    insns = decode(prog) if isinstance(prog, (bytes, bytearray)) else prog
    if len(pkt) > mem_size:
        return ST_BADPKT, 0, 0
    mem = bytearray(mem_size)
    mem[:len(pkt)] = pkt
    regs = [0] * 11
    regs[2] = len(pkt)
    regs[1] = 0
    regs[10] = r10
    emu = Emu(insns, mem, regs)
    st = emu.run(max_steps)
    return st, emu.regs[0] & M64, emu.ins_count


def run_full(prog: bytes | list, pkt: bytes, mem_size: int = 1024, r10: int = 512,
             max_steps: int = 0):
    """-> (status, regs u64[11], final memory bytes, steps)."""
    insns = decode(prog) if isinstance(prog, (bytes, bytearray)) else prog
    if len(pkt) > mem_size:
        return ST_BADPKT, [0] * 11, bytes(mem_size), 0
    mem = bytearray(mem_size)
    mem[:len(pkt)] = pkt
    regs = [0] * 11
    regs[2] = len(pkt)
    regs[10] = r10
    emu = Emu(insns, mem, regs)
    st = emu.run(max_steps)
    return st, [r & M64 for r in emu.regs], bytes(emu.mmu.memory), emu.ins_count
