"""ctypes binding of libebpfemu.so (include/ebpf_emu.h).

The product path: every execution goes through the gfx950 kernel inside libebpfemu.so. There
is no Python or CPU fallback; if the library is missing this module raises at import time of
`lib()`.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# (EBPFEMU_LIB_PATH: another build of the same library, for A/B runs of two builds on one box)
LIB_PATH = os.environ.get("EBPFEMU_LIB_PATH") or os.path.join(_HERE, "libebpfemu.so")

# ---- constants mirrored from include/ebpf_emu.h ----
EBPF_OK = 0
EBPF_EINVAL, EBPF_ELEN, EBPF_EREG, EBPF_EOP, EBPF_EMODE = -1, -2, -3, -4, -5
EBPF_ELDDW, EBPF_ELDDW_OVF, EBPF_EHEX, EBPF_ENOMEM, EBPF_EHIP = -6, -7, -8, -9, -10
EBPF_ETOOBIG, EBPF_ERCCL, EBPF_EPCAP, EBPF_EJIT = -11, -12, -13, -14

ST_OK, ST_MEM, ST_MEM_UB, ST_INSN, ST_ARITH, ST_STEPS, ST_CALLDEPTH, ST_BADPKT, ST_JIT = range(9)
STATUS_NAMES = ["OK", "MEM", "MEM_UB", "INSN", "ARITH", "STEPS", "CALLDEPTH", "BADPKT", "JIT"]
VERDICT_OTHER, VERDICT_FAULT = 0xFE, 0xFF
NCOUNTERS = 8
DEFAULT_MEM, DEFAULT_R10, DEFAULT_STEPS = 1024, 512, 1 << 22
BATCH_GENERIC = 1  # ebpf_batch.flags: EBPF_BATCH_GENERIC
BATCH_XDP_MD = 2   # ebpf_batch.flags: EBPF_BATCH_XDP_MD (the xdp_md calling convention)
BATCH_NO_JIT = 4   # ebpf_batch.flags: EBPF_BATCH_NO_JIT (the tile interpreter, not the compiled program)
MAX_CALL_DEPTH = 64
# ebpf_batch_kernel ids (EBPF_KERNEL_*)
(EBPF_KERNEL_GENERAL_T0, EBPF_KERNEL_GENERAL_T1, EBPF_KERNEL_DAG, EBPF_KERNEL_TILE,
 EBPF_KERNEL_TILE_LOOP, EBPF_KERNEL_JIT_FIXED, EBPF_KERNEL_JIT_VAR, EBPF_KERNEL_JIT_LOOP,
 EBPF_KERNEL_JIT_STACK, EBPF_KERNEL_JIT_VAR_STACK, EBPF_KERNEL_JIT_LOOP_STACK,
 EBPF_KERNEL_JIT_VARL, EBPF_KERNEL_JIT_VARL_STACK, EBPF_KERNEL_JIT_FIXED_OCC) = range(14)
KERNEL_NAMES = ["ebpfemu::interp_kernel<0>", "ebpfemu::interp_kernel<1>", "ebpfemu::dag_kernel",
                "ebpfemu::tile_kernel<forward>", "ebpfemu::tile_kernel<loops>",
                "ebpf_tile_jit_fixed (compiled program)", "ebpf_tile_jit_var (compiled program)",
                "ebpf_tile_jit_loop (compiled loop program)",
                "ebpf_tile_jit_fixed (compiled stack-window program)",
                "ebpf_tile_jit_var_stack (compiled stack-window program)",
                "ebpf_tile_jit_loop_stack (compiled stack-window loop program)",
                "ebpf_tile_jit_varl (compiled program, var tile loop)",
                "ebpf_tile_jit_varl_stack (compiled stack-window program, var tile loop)",
                "ebpf_tile_jit_fixed_occ (compiled issue-bound program, fixed slots)"]

EXPORTS = ["ebpf_batch_init", "ebpf_prog_load", "ebpf_prog_load_hex", "ebpf_prog_free",
           "ebpf_prog_len", "ebpf_prog_insn", "ebpf_prog_tier", "ebpf_prog_forward_only",
           "ebpf_prog_stack_window", "ebpf_prog_store_mode",
           "ebpf_workspace_bytes", "ebpf_prog_compile", "ebpf_prog_jit_asm", "ebpf_prog_jit_error", "ebpf_debug_trace",
           "ebpf_prog_upload", "ebpf_run_batch", "ebpf_run_batch_multi", "ebpf_batch_kernel", "ebpf_batch_staged",
           "ebpf_pcap_index",
           "ebpf_strerror", "ebpf_version"]


class Batch(ctypes.Structure):  # ebpf_batch
    _fields_ = [("frames", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("lens", ctypes.c_void_p), ("stride", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("mem_size", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("r10", ctypes.c_uint64), ("max_steps", ctypes.c_uint64),
                ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_uint64),
                ("init_regs", ctypes.c_void_p), ("init_fp", ctypes.c_void_p),
                ("init_fp_len", ctypes.c_uint32)]


class BatchOut(ctypes.Structure):  # ebpf_batch_out
    _fields_ = [("verdict", ctypes.c_void_p), ("r0", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("counters", ctypes.c_void_p), ("mem", ctypes.c_void_p), ("regs", ctypes.c_void_p),
                ("fp", ctypes.c_void_p), ("fp_len", ctypes.c_void_p)]


class EbpfError(RuntimeError):
    def __init__(self, code: int, what: str = "", word: int | None = None):
        self.code = code
        self.word = word
        msg = f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})"
        if word is not None:
            msg += f" at word {word}"
        super().__init__(msg)


_LIB = None


def lib():
    """Load libebpfemu.so (built by __graft_entry__.build() / `make -C ebpf-emu_amd`)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C ebpf-emu_amd` "
                          "(there is no CPU fallback)")
    # PyTorch ships its own HIP runtime (torch/lib/libamdhip64.so). Load it first, so this
    # library's libamdhip64 dependency resolves to that same runtime by soname; loaded the other
    # way round, torch would bind to /opt/rocm's runtime and find no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
    L.ebpf_batch_init.argtypes = [ctypes.POINTER(Batch)]
    L.ebpf_batch_init.restype = None
    L.ebpf_prog_load.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    L.ebpf_prog_load_hex.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    L.ebpf_prog_free.argtypes = [vp]
    L.ebpf_prog_free.restype = None
    L.ebpf_prog_len.argtypes = [vp]
    L.ebpf_prog_len.restype = sz
    L.ebpf_prog_insn.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_int32),
                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int16),
                                 ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint8),
                                 ctypes.POINTER(ctypes.c_uint8)]
    L.ebpf_prog_tier.argtypes = [vp]
    L.ebpf_prog_forward_only.argtypes = [vp]
    L.ebpf_prog_stack_window.argtypes = [vp]
    L.ebpf_prog_store_mode.argtypes = [vp]
    L.ebpf_prog_compile.argtypes = [vp]
    L.ebpf_debug_trace.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    L.ebpf_prog_jit_asm.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.ebpf_prog_jit_error.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    L.ebpf_workspace_bytes.argtypes = [vp, ctypes.POINTER(Batch), ctypes.c_int]
    L.ebpf_workspace_bytes.restype = u64
    L.ebpf_prog_upload.argtypes = [vp, ctypes.c_int]
    L.ebpf_run_batch.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(BatchOut), vp]
    L.ebpf_batch_kernel.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(BatchOut), ctypes.c_int]
    L.ebpf_batch_staged.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(BatchOut), ctypes.c_int]
    L.ebpf_run_batch_multi.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(Batch), ctypes.POINTER(BatchOut),
                                       ctypes.POINTER(vp)]
    L.ebpf_pcap_index.argtypes = [vp, sz, vp, vp, sz, ctypes.POINTER(sz),
                                  ctypes.POINTER(ctypes.c_uint32)]
    L.ebpf_strerror.argtypes = [ctypes.c_int]
    L.ebpf_strerror.restype = ctypes.c_char_p
    L.ebpf_version.restype = ctypes.c_char_p
    _LIB = L
    return L


def strerror(code: int) -> str:
    try:
        return lib().ebpf_strerror(code).decode()
    except ImportError:
        return "error"
