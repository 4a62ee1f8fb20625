"""ebpf_emu.xdp — verdict and context types of the reference (src/xdp.rs, not compiled there).

An XDP verdict is r0 after exit (xdp.rs:3-9). The device path writes a verdict byte per
packet: r0 for r0 < 5, VERDICT_OTHER (0xFE) for any other r0, VERDICT_FAULT (0xFF) when the
execution faulted; and counts packets per bucket (counters[0..4], [5] other, [6] faults,
[7] instructions retired).
"""
from __future__ import annotations

import ctypes
import enum

from ._lib import VERDICT_FAULT, VERDICT_OTHER  # noqa: F401


class xdp_action(enum.IntEnum):  # xdp.rs:1-9
    XDP_ABORTED = 0
    XDP_DROP = 1
    XDP_PASS = 2
    XDP_TX = 3
    XDP_REDIRECT = 4

    @classmethod
    def from_u8(cls, val: int) -> "xdp_action":  # xdp.rs:10-15 (assert val < 5)
        if not 0 <= val < 5:
            raise AssertionError("assertion failed: val < 5")
        return cls(val)


class xdp_md(ctypes.Structure):  # xdp.rs:16-26, #[repr(C)]
    _fields_ = [("data", ctypes.c_uint32), ("data_end", ctypes.c_uint32)]


def verdict_of(status: int, r0: int) -> int:
    """The verdict byte the kernel writes for (status, r0)."""
    if status != 0:
        return VERDICT_FAULT
    r0 &= (1 << 64) - 1
    return r0 if r0 < 5 else VERDICT_OTHER
