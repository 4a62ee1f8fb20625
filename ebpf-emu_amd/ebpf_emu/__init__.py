"""ebpf_emu — MI355X-native batched eBPF/XDP interpreter (host side).

Mirrors the reference crate's module layout (`ebpf_emu::{ins, emu, mmu}`, src/lib.rs:1-3, plus
the uncompiled `xdp` types) over the C ABI of libebpfemu.so, whose gfx950 kernel does every
execution. Batched use: `Program(image).run(frames, ...)`.
"""
from . import asm, ins, mmu, xdp  # noqa: F401
from ._lib import (DEFAULT_MEM, DEFAULT_R10, DEFAULT_STEPS, STATUS_NAMES, ST_ARITH,  # noqa: F401
                   ST_BADPKT, ST_CALLDEPTH, ST_INSN, ST_JIT, ST_MEM, ST_MEM_UB, ST_OK, ST_STEPS,
                   EbpfError, lib)
from .ins import DecodeError, HexError, hexs_to_instructions, hexs_to_u8s  # noqa: F401


def __getattr__(name):  # lazy: these import torch
    if name in ("Program", "BatchResult"):
        from . import program

        return getattr(program, name)
    if name in ("Emu", "EmuPanic"):
        from . import emu

        return getattr(emu, name)
    raise AttributeError(name)
