"""ebpf_emu.emu — the reference's `Emu` surface (src/emu.rs:13-45,452-458) on the GPU.

    emu = Emu()                        # Emu::default()
    emu.state.mmu = Mmu(bytearray(1024))
    emu.state.regs[1] = 0; emu.state.regs[10] = 512
    emu.instructions = hexs_to_instructions(hx)
    emu.run()                          # executes as a one-packet batch of the gfx950 kernel
    r0 = emu.state.regs[0]

Error behaviour: where the reference panics (killing the process) `run()` raises EmuPanic with
the fault status; the reference's hang (no step limit) becomes EmuPanic(ST_STEPS) after
`max_steps` instructions.
"""
from __future__ import annotations

from . import _lib
from .ins import AJ, Class, Instruction, LS, Mode
from .mmu import Mmu

M64 = (1 << 64) - 1


class EmuPanic(RuntimeError):
    def __init__(self, status: int):
        super().__init__(f"emulator fault: {_lib.STATUS_NAMES[status]}")
        self.status = status


def _s64(v: int) -> int:
    v &= M64
    return v - (1 << 64) if v >> 63 else v


class State:  # emu.rs:13-17
    def __init__(self):
        self.regs = [0] * 11
        self.mmu = Mmu(bytearray())


def encode_instructions(insns) -> bytes:
    """Re-encode decoded Instructions as a program image that decodes back to the same list
    (a wide instruction's imm64 goes whole into the second word, first-word imm = 0)."""
    out = bytearray()
    for ins in insns:
        op = ins.opcode
        regs = (int(ins.dst) & 0xF) | ((int(ins.src) & 0xF) << 4)
        wide = isinstance(ins.code, LS) and ins.code.mode == Mode.IMM
        imm = 0 if wide else ins.imm
        out += bytes([op, regs]) + (ins.off & 0xFFFF).to_bytes(2, "little")
        out += (imm & 0xFFFFFFFF).to_bytes(4, "little")
        if wide:
            out += (ins.imm64 & M64).to_bytes(8, "little")
    return bytes(out)


class Emu:  # emu.rs:19-45
    def __init__(self, max_steps: int = _lib.DEFAULT_STEPS, device: int = 0):
        self.state = State()
        self.instructions: list[Instruction] = []
        self.fp: list[int] = []
        self.max_steps = max_steps
        self.device = device

    def run(self) -> None:
        """Emu::run (emu.rs:452-458): one execution on the GPU, on the caller's state -- the
        memory image of any length (Mmu.memory: Vec<u8>, mmu.rs:2-4), the registers and the frame
        stack `fp` (emu.rs:26); all three are written back."""
        import numpy as np
        import torch

        from .program import Program

        mem = bytes(self.state.mmu.memory)
        if len(self.fp) > _lib.MAX_CALL_DEPTH:
            raise ValueError(f"frame stack deeper than {_lib.MAX_CALL_DEPTH}")
        prog = Program(encode_instructions(self.instructions))
        dev = torch.device("cuda", self.device)
        # the image as one packet of its own length: [0, len) = the image, nothing past it
        frames = torch.tensor(list(mem) or [0], dtype=torch.uint8, device=dev)
        if mem:
            layout = dict(stride=len(mem))
        else:  # an empty image: one zero-length packet
            layout = dict(offsets=torch.zeros(1, dtype=torch.int32, device=dev),
                          lens=torch.zeros(1, dtype=torch.int16, device=dev))
        regs = torch.tensor([_s64(r) for r in self.state.regs], dtype=torch.int64, device=dev)
        init_fp = None
        if self.fp:
            init_fp = torch.from_numpy(np.array([int(x) & 0xFFFFFFFF for x in self.fp],
                                                dtype=np.uint32).view(np.int32)).to(dev)
        res = prog.run(frames, n=1, mem_size=len(mem), init_regs=regs, **layout,
                       max_steps=self.max_steps, verdict=False, status=True, mem=len(mem) > 0,
                       regs=True, init_fp=init_fp, fp=True)
        torch.cuda.synchronize(dev)
        st = int(res.status[0].item())
        self.state.regs = [_s64(v) for v in res.regs[0].tolist()]
        if len(mem):
            self.state.mmu.memory = bytearray(bytes(res.mem[0].cpu().numpy().tobytes()))
        depth = int(res.fp_len[0].item())
        self.fp = [int(v) & 0xFFFFFFFF for v in res.fp[0, :depth].tolist()]
        prog.close()
        if st != _lib.ST_OK:
            raise EmuPanic(st)
