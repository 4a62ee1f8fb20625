"""ctypes binding of the C oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class OrInsn(ctypes.Structure):  # ebpf_oracle.h or_insn
    _fields_ = [("imm", ctypes.c_int32), ("imm64", ctypes.c_int64), ("off", ctypes.c_int16),
                ("src", ctypes.c_uint8), ("dst", ctypes.c_uint8), ("code", ctypes.c_uint8)]


def build(force: bool = False) -> str:
    path = os.path.join(_HERE, "liboracle.so")
    if force or not os.path.exists(path):
        subprocess.run(["make", "-C", _HERE, "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        L = _LIB
        L.or_decode.restype = ctypes.c_long
        L.or_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(OrInsn),
                                ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.or_run_packet.restype = ctypes.c_int
        L.or_run_packet.argtypes = [ctypes.POINTER(OrInsn), ctypes.c_size_t, ctypes.c_char_p,
                                    ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_uint64)]
        L.or_run.restype = ctypes.c_int
        L.or_run.argtypes = [ctypes.POINTER(OrInsn), ctypes.c_size_t, ctypes.c_void_p,
                             ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64), ctypes.c_uint64,
                             ctypes.POINTER(ctypes.c_uint64)]
        L.or_run_fp.restype = ctypes.c_int
        L.or_run_fp.argtypes = [ctypes.POINTER(OrInsn), ctypes.c_size_t, ctypes.c_void_p,
                                ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64),
                                ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_size_t),
                                ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.or_run_batch.restype = ctypes.c_int
        L.or_run_batch.argtypes = [ctypes.POINTER(OrInsn), ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                   ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint64,
                                   ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int]
        L.or_run_batch_xdp.restype = ctypes.c_int
        L.or_run_batch_xdp.argtypes = L.or_run_batch.argtypes + [ctypes.c_int]
    return _LIB


class OracleDecodeError(Exception):
    def __init__(self, code: int, word: int):
        super().__init__(code, word)
        self.code = code
        self.word = word


class Program:
    """A decoded program held by the C oracle."""

    def __init__(self, image: bytes):
        L = lib()
        bad = ctypes.c_size_t(0)
        cap = max(1, len(image) // 8)
        arr = (OrInsn * cap)()
        n = L.or_decode(bytes(image), len(image), arr, cap, ctypes.byref(bad))
        if n < 0:
            raise OracleDecodeError(int(n), bad.value)
        self.insns = arr
        self.n = int(n)

    def decoded(self):
        return [(i.imm, i.imm64, i.off, i.src, i.dst, i.code) for i in self.insns[: self.n]]

    def run_packet(self, pkt: bytes, mem_size: int = 1024, r10: int = 512, max_steps: int = 0):
        """-> (status, r0 u64, steps)"""
        r0 = ctypes.c_uint64(0)
        steps = ctypes.c_uint64(0)
        st = lib().or_run_packet(self.insns, self.n, bytes(pkt), len(pkt), mem_size, r10,
                                 max_steps, ctypes.byref(r0), ctypes.byref(steps))
        return st, r0.value, steps.value

    def run_full(self, pkt: bytes, mem_size: int = 1024, r10: int = 512, max_steps: int = 0,
                 init_regs=None):
        """-> (status, regs u64[11], final memory bytes, steps); main.rs layout unless
        init_regs (11 ints) is given, as the device path's init_regs does."""
        if len(pkt) > mem_size:
            return 7, [0] * 11, bytes(mem_size), 0
        mem = (ctypes.c_uint8 * mem_size)()
        ctypes.memmove(mem, bytes(pkt), len(pkt))
        regs = (ctypes.c_int64 * 11)()
        if init_regs is None:
            regs[2] = len(pkt)
            regs[10] = r10
        else:
            for i, v in enumerate(init_regs):
                v &= (1 << 64) - 1
                regs[i] = v - (1 << 64) if v >> 63 else v
        steps = ctypes.c_uint64(0)
        st = lib().or_run(self.insns, self.n, mem, mem_size, regs, max_steps, ctypes.byref(steps))
        return st, [r & ((1 << 64) - 1) for r in regs], bytes(mem), steps.value

    def run_image(self, image: bytes, regs, fp=(), max_steps: int = 0):
        """Emu::run on a caller-built state (emu.rs:14-26 pub fields): the memory image of any
        length, 11 registers, the frame stack fp (bottom first). -> (status, regs u64[11],
        final memory bytes, final fp list, steps)."""
        mem = (ctypes.c_uint8 * max(1, len(image)))()
        ctypes.memmove(mem, bytes(image), len(image))
        r = (ctypes.c_int64 * 11)()
        for i, v in enumerate(regs):
            v &= (1 << 64) - 1
            r[i] = v - (1 << 64) if v >> 63 else v
        f = (ctypes.c_uint32 * 64)(*[int(x) & 0xFFFFFFFF for x in fp])
        fl = ctypes.c_size_t(len(fp))
        steps = ctypes.c_uint64(0)
        st = lib().or_run_fp(self.insns, self.n, mem, len(image), r, f, ctypes.byref(fl),
                             max_steps, ctypes.byref(steps))
        return (st, [x & ((1 << 64) - 1) for x in r], bytes(mem)[:len(image)],
                [int(f[i]) for i in range(fl.value)], steps.value)

    def run_batch(self, frames: np.ndarray, n: int, stride: int = 0, offsets=None, lens=None,
                  mem_size: int = 1024, r10: int = 512, max_steps: int = 0, threads: int = 1,
                  xdp_md: bool = False):
        """-> (r0 u64[n], status u8[n], counters u64[8]). xdp_md: each packet runs as the
        image [u32 8][u32 8 + len][packet] (the xdp_md calling convention, xdp.rs:16-20)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        r0 = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.uint8)
        counters = np.zeros(8, dtype=np.uint64)
        off_p = None
        len_p = None
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
            off_p = offsets.ctypes.data
        if lens is not None:
            lens = np.ascontiguousarray(lens, dtype=np.uint16)
            len_p = lens.ctypes.data
        lib().or_run_batch_xdp(self.insns, self.n, frames.ctypes.data, off_p, len_p, stride, n,
                               mem_size, r10, max_steps, r0.ctypes.data, status.ctypes.data,
                               counters.ctypes.data, threads, 1 if xdp_md else 0)
        return r0, status, counters
