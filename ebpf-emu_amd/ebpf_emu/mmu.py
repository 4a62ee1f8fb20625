"""ebpf_emu.mmu — the reference's `Mmu` data holder (src/mmu.rs:1-5).

On the device the bounds checks of mmu.rs:7-30 are inlined in the kernel (interp.hip); this
host object only carries the flat image in and out of `Emu.run()`. Its helpers restate the
reference's accessors for host-side inspection of images.
"""
from __future__ import annotations


class Mmu:
    def __init__(self, memory: bytearray | bytes | None = None):
        self.memory = bytearray(memory or b"")

    def write(self, addr: int, val: bytes) -> None:  # mmu.rs:7-12
        if len(self.memory) < addr + len(val):
            self.memory.extend(bytes(addr + len(val) + 0x1000 - len(self.memory)))
        self.memory[addr:addr + len(val)] = val

    def read(self, addr: int, size: int) -> int:  # mmu.rs:13-22 (read::<T>, LE)
        if addr < 0 or addr + size > len(self.memory):
            raise IndexError("range end index out of range for slice")
        return int.from_bytes(self.memory[addr:addr + size], "little")
